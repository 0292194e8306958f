#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; grep -v "^Extension\|amdgpu.ids" "gpurun_out/$name.log" | tail -n 2 | cut -c1-1200; [ $rc -le 1 ] || { echo "!! $name rc=$rc"; exit $rc; }; }
run t13 400 python -u -m pytest tests/test_gpu_line.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread
for rep in 1 2 3; do
  VTK_LIB=.abl/lib_prev.so run lab_prev_$rep 300 python tools/ab_env.py --prec line --config C3 --env lsv_ring --values 2048 --rounds 4
  run lab_new_$rep 300 python tools/ab_env.py --prec line --config C3 --env lsv_ring --values 2048 --rounds 4
done
run bline 300 python bench.py --prec line --steps 5 --warmup 1 --no-cpu-baseline
