#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; grep -v "^Extension\|amdgpu.ids" "gpurun_out/$name.log" | tail -n 3 | cut -c1-1500; [ $rc -le 1 ] || { echo "!! $name rc=$rc"; exit $rc; }; }
run t11 400 python -u -m pytest tests/test_gpu_dropin.py tests/test_gpu_multirank.py -q -p no:cacheprovider --timeout 200 --timeout-method thread
run t11b 600 python -u -m pytest tests/test_gpu_large.py -q -p no:cacheprovider --timeout 400 --timeout-method thread -k c4
run c4_def 600 python tools/ab_env.py --config C4 --env g4_ring --values 0,2048 --rounds 3
