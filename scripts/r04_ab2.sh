#!/bin/bash
# plain SpMV: grid sweep on the current build, the r01 / r03 builds side by side (bisection), and
# the line path's LDS-staged table SpMV
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; grep -v "^Extension\|amdgpu.ids" "gpurun_out/$name.log" | tail -n 2; [ $rc -eq 0 ] || { echo "!! $name rc=$rc"; exit $rc; }; }
run spmv_grid 300 python tools/spmv_ab.py --config C3 --settings "plain_grid=2048;plain_grid=3072;plain_grid=4096;plain_grid=6144;plain_grid=8192;plain_grid=16384;plain_grid=100000;sell_swz=1,plain_grid=8192"
for rep in 1 2; do
  for L in tools/bin/lib_r01/libvtkrylov.so tools/bin/lib_r03/libvtkrylov.so vt-precondition_amd/vtkrylov/lib/libvtkrylov.so; do
    run spmv_lib_$(basename $(dirname $L))_$rep 120 python tools/spmv_lib_time.py --lib $L
  done
done
run line_ring 300 python tools/ab_env.py --env lsv_ring --values 0,1024,2048,4096 --rounds 6 --prec line
run line_sweep 300 python tools/ab_env.py --env line_sweep --values 0,512,1024,2048 --rounds 6 --prec line --perj
run c4_g4 600 python tools/ab_env.py --config C4 --env grid4 --values 1,0 --rounds 3
run c4_fused 600 python tools/ab_env.py --config C4 --env c4_fused --values 0,1 --rounds 3
