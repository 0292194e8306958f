#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; grep -v "^Extension\|amdgpu.ids" "gpurun_out/$name.log" | tail -n 1 | cut -c1-700; [ $rc -le 1 ] || { echo "!! $name rc=$rc"; exit $rc; }; }
run t18 600 python -u -m pytest tests/test_gpu_line.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread
run l_nli 300 python tools/ab_env.py --prec line --config C3 --env lsv_nli --values 1,2,4 --rounds 4
run l_nli2 300 python tools/ab_env.py --prec line --config C3 --env lsv_ring --values 1024,2048,4096 --set lsv_nli=2 --rounds 3
