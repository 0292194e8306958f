#!/bin/bash
# Run GPU steps on the gpurun box, each under its own time limit; stop at the first crash,
# abort, fault or timeout (test failures, exit 1, do not stop the chain).
#   scripts/gpu_steps.sh smoke tests bench prof ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
    local name=$1 to=$2; shift 2
    echo "== $name: $*"
    local t0=$(date +%s)
    timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc ($(( $(date +%s) - t0 ))s)"
    tail -n 15 "gpurun_out/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "!! fatal rc=$rc: stopping"; exit $rc; fi
    return 0
}
for s in "$@"; do
    case $s in
        smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
        tests) step tests 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider ;;
        testsall) step testsall 900 python -m pytest tests -m gpu -q -p no:cacheprovider ;;
        bench) step bench 600 python bench.py ;;
        benchq) step benchq 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline ;;
        benchc4) step benchc4 600 python bench.py --config C4 --steps 2 --warmup 1 --no-cpu-baseline --spmv-reps 10 ;;
        benchc2) step benchc2 300 python bench.py --config C2 --steps 3 --warmup 1 --no-cpu-baseline ;;
        line) step line 900 python -u -m pytest tests/test_gpu_line.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread ;;
        benchline) step benchline 300 python bench.py --prec line --steps 5 --warmup 1 --no-cpu-baseline ;;
        benchlinec4) step benchlinec4 600 python bench.py --config C4 --prec line --steps 3 --warmup 1 --no-cpu-baseline --spmv-reps 10 ;;
        benchc1) step benchc1 300 python bench.py --config C1 --steps 5 --warmup 1 --no-cpu-baseline ;;
        benchinv) step benchinv 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --bj-mode inverse ;;
        benchc4csr) step benchc4csr 600 python bench.py --config C4 --steps 2 --warmup 1 --no-cpu-baseline --spmv-reps 10 --layout csr ;;
        benchcsr) step benchcsr 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --layout csr ;;
        benchsolo) step benchsolo 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --comm-solo ;;
        benchc1solo) step benchc1solo 300 python bench.py --config C1 --steps 5 --warmup 1 --no-cpu-baseline --comm-solo ;;
        profline) step profline 600 rocprofv3 --kernel-trace --stats -d gpurun_out/profline -o run --output-format csv -- python bench.py --prec line --steps 3 --warmup 1 --no-cpu-baseline ;;
        profc4) step profc4 600 rocprofv3 --kernel-trace --stats -d gpurun_out/profc4 -o run --output-format csv -- python bench.py --config C4 --steps 2 --warmup 1 --no-cpu-baseline --spmv-reps 10 ;;
        profmgs) step profmgs 600 rocprofv3 --kernel-trace --stats -d gpurun_out/profmgs -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --orth mgs ;;
        ab) for v in a cur a cur; do if [ $v = a ]; then L=tools/bin/lib_a/libvtkrylov.so; else L=vt-precondition_amd/vtkrylov/lib/libvtkrylov.so; fi; VTK_LIB=$L step ab_$v 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --spmv-reps 5 || exit $?; grep -o '"value": [0-9.]*' gpurun_out/ab_$v.log; done ;;
        variants) for rep in 1 2; do for v in cur ${VARIANTS:-a}; do if [ $v = cur ]; then L=vt-precondition_amd/vtkrylov/lib/libvtkrylov.so; else L=tools/bin/lib_$v/libvtkrylov.so; fi; VTK_LIB=$L step var_${v}_$rep 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --spmv-reps 5 ${BENCH_ARGS:-} || exit $?; python tools/bench_brief.py gpurun_out/var_${v}_$rep.log; done; done ;;
        abargs) IFS=';' read -ra AL <<< "${ABARGS:-}"; for rep in 1 2; do i=0; for ar in "${AL[@]}"; do i=$((i+1)); step abargs_${i}_$rep 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --spmv-reps 5 $ar || exit $?; echo "[$ar]"; python tools/bench_brief.py gpurun_out/abargs_${i}_$rep.log; done; done ;;
        benchmgs) step benchmgs 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --orth mgs ;;
        benchdc) step benchdc 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --orth dcgs2 ;;
        prof) step prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline ;;
        multirank) step multirank 900 python -m pytest tests/test_gpu_multirank.py -m gpu -x -q -p no:cacheprovider ;;
        bench2host) step bench2host 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --comm host --config C1 --steps 1 --warmup 1 --spmv-reps 3 ;;
        profc1) step profc1 600 rocprofv3 --kernel-trace --stats -d gpurun_out/profc1 -o run --output-format csv -- python bench.py --config C1 --steps 3 --warmup 1 --no-cpu-baseline ;;
        pmcsq) step pmcsq 120 rocprofv3 --pmc ${PMC:-SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES} -d gpurun_out/pmc_sq -o run --output-format csv -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline --spmv-reps 2 ;;
        bench2self) step bench2self 600 python bench.py --gpus 2 --comm host --config C1 --steps 1 --warmup 1 --spmv-reps 3 --no-cpu-baseline ;;
        pmcwc4) step pmcwc4 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write_c4 -o run --output-format csv -- python bench.py --config C4 --steps 1 --warmup 0 --no-cpu-baseline --spmv-reps 3 ;;
        pmcsqc4) step pmcsqc4 300 rocprofv3 --pmc ${PMC:-SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES} -d gpurun_out/pmc_sq_c4 -o run --output-format csv -- python bench.py --config C4 --steps 1 --warmup 0 --no-cpu-baseline --spmv-reps 3 ;;
        pmcfc4) step pmcfc4 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_c4 -o run --output-format csv -- python bench.py --config C4 --steps 1 --warmup 0 --no-cpu-baseline --spmv-reps 3 ;;
        pmcf) step pmcf 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline --spmv-reps 5 ;;
        pmcw) step pmcw 600 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- python bench.py --steps 1 --warmup 1 --no-cpu-baseline --spmv-reps 5 ;;
        profsolo) step profsolo 600 rocprofv3 --kernel-trace --stats -d gpurun_out/profsolo -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --comm-solo --spmv-reps 5 ;;
        profsoloc2) step profsoloc2 600 rocprofv3 --kernel-trace --stats -d gpurun_out/profsoloc2 -o run --output-format csv -- python bench.py --config C2 --steps 2 --warmup 1 --no-cpu-baseline --comm-solo --spmv-reps 5 ;;
        profc2) step profc2 600 rocprofv3 --kernel-trace --stats -d gpurun_out/profc2 -o run --output-format csv -- python bench.py --config C2 --steps 2 --warmup 1 --no-cpu-baseline --spmv-reps 5 ;;
        profall) for C in C3 C4; do c=$(echo $C | tr C c); A="--config $C --steps 1 --warmup 1 --no-cpu-baseline --spmv-reps 5";
                 step prof_$c 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$c -o run --output-format csv -- python bench.py --config $C --steps 2 --warmup 1 --no-cpu-baseline || exit $?;
                 step pmcf_$c 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcf_$c -o run --output-format csv -- python bench.py $A || exit $?;
                 step pmcw_$c 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcw_$c -o run --output-format csv -- python bench.py $A || exit $?;
                 step pmcsq_$c 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES -d gpurun_out/pmcsq_$c -o run --output-format csv -- python bench.py $A || exit $?; done ;;
        slabs) step slab_c3_8 300 python bench.py --config C3 --slab 8 --comm-solo --steps 5 --warmup 1 --no-cpu-baseline || exit $?;
               step slab_c3_4 300 python bench.py --config C3 --slab 4 --comm-solo --steps 5 --warmup 1 --no-cpu-baseline || exit $?;
               step slab_c3_2 300 python bench.py --config C3 --slab 2 --comm-solo --steps 5 --warmup 1 --no-cpu-baseline || exit $?;
               step slab_c3_1 300 python bench.py --config C3 --comm-solo --steps 5 --warmup 1 --no-cpu-baseline || exit $?;
               step slab_c4_8 300 python bench.py --config C4 --slab 8 --comm-solo --steps 3 --warmup 1 --no-cpu-baseline || exit $? ;;
        benchc2full) step benchc2full 600 python bench.py --config C2 ;;
        mrlarge) step mrlarge 900 python -u -m pytest tests/test_gpu_multirank_large.py -x -v -p no:cacheprovider --timeout 600 --timeout-method thread ;;
        bandtests) step bandtests 600 python -u -m pytest tests/test_gpu_band.py tests/test_gpu_multirank.py tests/test_gpu_large.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread ;;
        testsv) step testsv 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread ;;
        large) step large 600 python -u -m pytest tests/test_gpu_large.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider ;;
        *) echo "unknown step $s"; exit 2 ;;
    esac
done
