#!/bin/bash
# Round-4 final measurements: GPU suite + smoke, C3 bench (with the CPU baseline) and its
# rocprofv3 kernel-trace / FETCH_SIZE / WRITE_SIZE passes, the same for C4 and the line path.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; grep -v "^Extension\|amdgpu.ids\|^W2026\|^E2026\|^I2026" "gpurun_out/$name.log" | tail -n 2 | cut -c1-600; [ $rc -le 1 ] || { echo "!! $name rc=$rc"; exit $rc; }; }
S=${STAGES:-tests smoke c3 c4 line}
for st in $S; do case $st in
tests) run tests 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 400 --timeout-method thread ;;
smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
c3) run bench_c3 600 python bench.py
    run prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline --spmv-reps 5
    run pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline --spmv-reps 5
    run pmc_write 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline --spmv-reps 5 ;;
c4) run bench_c4 600 python bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline
    run prof_c4 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c4 -o run --output-format csv -- python bench.py --config C4 --steps 1 --warmup 1 --no-cpu-baseline --spmv-reps 5
    run pmcf_c4 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcf_c4 -o run --output-format csv -- python bench.py --config C4 --steps 1 --warmup 1 --no-cpu-baseline --spmv-reps 5
    run pmcw_c4 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcw_c4 -o run --output-format csv -- python bench.py --config C4 --steps 1 --warmup 1 --no-cpu-baseline --spmv-reps 5 ;;
line) run bench_line 300 python bench.py --prec line --steps 5 --warmup 1 --no-cpu-baseline
      run prof_line 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_line -o run --output-format csv -- python bench.py --prec line --steps 3 --warmup 1 --no-cpu-baseline ;;
slabs) run slab_c3_8 300 python bench.py --config C3 --slab 8 --comm-solo --steps 5 --warmup 1 --no-cpu-baseline
       run slab_c3_4 300 python bench.py --config C3 --slab 4 --comm-solo --steps 5 --warmup 1 --no-cpu-baseline
       run slab_c3_2 300 python bench.py --config C3 --slab 2 --comm-solo --steps 5 --warmup 1 --no-cpu-baseline
       run slab_c3_1 300 python bench.py --config C3 --comm-solo --steps 5 --warmup 1 --no-cpu-baseline
       run slab_c4_8 300 python bench.py --config C4 --slab 8 --comm-solo --steps 3 --warmup 1 --no-cpu-baseline ;;
*) echo "unknown stage $st"; exit 2 ;;
esac; done
