#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; grep -v "^Extension\|amdgpu.ids" "gpurun_out/$name.log" | tail -n 1 | cut -c1-700; [ $rc -le 1 ] || { echo "!! $name rc=$rc"; exit $rc; }; }
run t16 600 python -u -m pytest tests/test_gpu_band.py tests/test_gpu_line.py tests/test_gpu_x0.py tests/test_gpu_large.py -x -q -p no:cacheprovider --timeout 400 --timeout-method thread
run c3_cyc 600 python tools/ab_env.py --config C3 --env cyc_ring --values 0,512,1024 --rounds 4
run l_cyc 300 python tools/ab_env.py --prec line --config C3 --env cyc_ring --values 0,1024 --rounds 4
