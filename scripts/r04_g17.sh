#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; grep -v "^Extension\|amdgpu.ids" "gpurun_out/$name.log" | tail -n 1 | cut -c1-700; [ $rc -le 1 ] || { echo "!! $name rc=$rc"; exit $rc; }; }
run t17 600 python -u -m pytest tests/test_gpu_dropin.py tests/test_gpu_multirank.py tests/test_gpu_large.py -x -q -p no:cacheprovider --timeout 400 --timeout-method thread -k "grid4 or S4 or c4"
run c4_res 600 python tools/ab_env.py --config C4 --env g4_res --values 0,1 --rounds 3
run c4_dc0 600 python tools/ab_env.py --config C4 --env g4_dc0 --values 0,1 --rounds 3
