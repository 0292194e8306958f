#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; grep -v "^Extension\|amdgpu.ids" "gpurun_out/$name.log" | tail -n 1 | cut -c1-700; [ $rc -le 1 ] || { echo "!! $name rc=$rc"; exit $rc; }; }
run t15 600 python -u -m pytest tests/test_gpu_band.py tests/test_gpu_line.py tests/test_gpu_x0.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread
run c4_xb 600 python tools/ab_env.py --config C4 --env upd_xb --values 0,8 --rounds 3
run c4_ug8 600 python tools/ab_env.py --config C4 --env upd_grid --values 0,2048,4096 --set upd_xb=8 --rounds 2
run c4_ug0 600 python tools/ab_env.py --config C4 --env upd_grid --values 2048,4096 --set upd_xb=0 --rounds 2
run l_xb 300 python tools/ab_env.py --prec line --config C3 --env upd_xb --values 0,8 --rounds 4
run l_ug 300 python tools/ab_env.py --prec line --config C3 --env upd_grid --values 0,2048,4096 --rounds 4
