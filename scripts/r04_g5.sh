#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; grep -v "^Extension\|amdgpu.ids" "gpurun_out/$name.log" | tail -n 3 | cut -c1-3000; [ $rc -le 1 ] || { echo "!! $name rc=$rc"; exit $rc; }; }
run t5 1000 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 400 --timeout-method thread
run spmv_var 300 python tools/spmv_ab.py --config C3 --settings "plain_var=0;plain_var=1;plain_var=1,plain_grid=4096"
run spmv_r01 120 python tools/spmv_lib_time.py --lib tools/bin/lib_r01/libvtkrylov.so
run line_combo 300 python tools/ab_env.py --env line_sweep --values 0,256,512,1024 --rounds 6 --prec line --perj --set lsv_ring=2048
run bench_c4 600 python bench.py --config C4 --steps 2 --warmup 1 --no-cpu-baseline --spmv-reps 10
run bench_c3 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline
