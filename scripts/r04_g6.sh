#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; grep -v "^Extension\|amdgpu.ids" "gpurun_out/$name.log" | tail -n 3 | cut -c1-600; [ $rc -le 1 ] || { echo "!! $name rc=$rc"; exit $rc; }; }
run t6 1000 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 400 --timeout-method thread
run bench_c3 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline
run bench_upload 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --operator upload
run bench_line 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline --prec line
run bench_c4 600 python bench.py --config C4 --steps 2 --warmup 1 --no-cpu-baseline --spmv-reps 10
run c4_fused 600 python tools/ab_env.py --config C4 --env c4_fused --values 0,1 --rounds 3
