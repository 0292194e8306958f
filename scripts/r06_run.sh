#!/bin/bash
# Round-6 GPU steps: each stage under its own time limit, stop at the first failure.
#   STAGES="band ab" scripts/r05_run.sh      (AB_ENV / AB_VALUES / AB_SET / AB_CFG pick the A/B)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; grep -v "^Extension\|amdgpu.ids\|^W20\|^E20\|^I20" "gpurun_out/$name.log" | tail -n 3 | cut -c1-800; [ $rc -le 1 ] || { echo "!! $name rc=$rc"; exit $rc; }; [ $rc -eq 0 ] || { echo "!! $name failed"; exit 1; }; }
T="python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread"
for st in ${STAGES:-band}; do case $st in
band) run t_band 600 $T tests/test_gpu_band.py ;;
tests) run t_sel 900 $T ${TESTS} ;;
gpu) run t_gpu 1100 $T tests -m gpu ;;
smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
ab) run ab_${AB_ENV}${AB_TAG:-} 600 python tools/ab_env.py --env "$AB_ENV" --values "${AB_VALUES:-1,0}" --rounds "${AB_ROUNDS:-4}" --config "${AB_CFG:-C3}" --set "${AB_SET:-}" --perj ${AB_EXTRA:-} ${AB_MAXITER:+--maxiter $AB_MAXITER} ;;
bench) run bench 600 python bench.py ${BENCH_ARGS:-} ;;
slabs) for cp in C3:8 C3:4 C3:2 C4:8; do c=${cp%%:*}; p=${cp##*:}
         run slab_${c}_$p 300 python bench.py --config $c --slab $p --comm-solo --steps 5 --warmup 1 --no-cpu-baseline --spmv-reps 2
         grep '^{' gpurun_out/slab_${c}_$p.log | tail -1 >> gpurun_out/slabs.jsonl; done ;;
c4) run bench_c4 600 python bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline ;;
pmcab) for v in ${AB_VALUES//,/ }; do k=0; for ctr in ${PMC_SETS:-FETCH_SIZE TCC_HIT_sum,TCC_MISS_sum}; do k=$((k+1))
         run pmc_${AB_ENV}_${v}_$k 300 rocprofv3 --pmc ${ctr//,/ } -d gpurun_out/pmc_${AB_ENV}_${v}_$k -o run --output-format csv -- python tools/ab_env.py --env "$AB_ENV" --values "$v" --rounds 1 --config "${AB_CFG:-C3}" --set "${AB_SET:-}"; done; done ;;
final3) P="python bench.py --steps 1 --warmup 1 --no-cpu-baseline --spmv-reps 5"
        run bench_c3 600 python bench.py
        run prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- $P
        run pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- $P
        run pmc_write 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- $P
        run bench_upload 600 python bench.py --operator upload --steps 3 --warmup 1 --no-cpu-baseline ;;
final4) P="python bench.py --config C4 --steps 1 --warmup 1 --no-cpu-baseline --spmv-reps 5"
        run bench_c4 600 python bench.py --config C4 --steps 3 --warmup 1 --no-cpu-baseline
        run prof_c4 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c4 -o run --output-format csv -- $P
        run pmcf_c4 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcf_c4 -o run --output-format csv -- $P
        run pmcw_c4 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcw_c4 -o run --output-format csv -- $P ;;
sq) run pmc_sq 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD -d gpurun_out/pmc_sq -o run --output-format csv -- python bench.py ${SQ_ARGS:-} --steps 1 --warmup 1 --no-cpu-baseline --spmv-reps 5 ;;
line) run bench_line 300 python bench.py --prec line --steps 5 --warmup 1 --no-cpu-baseline
      run prof_line 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_line -o run --output-format csv -- python bench.py --prec line --steps 3 --warmup 1 --no-cpu-baseline ;;
linepmc) P="python bench.py --prec line --steps 1 --warmup 1 --no-cpu-baseline --spmv-reps 5"
         run prof_line 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_line -o run --output-format csv -- $P
         run pmcf_line 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcf_line -o run --output-format csv -- $P
         run pmcw_line 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcw_line -o run --output-format csv -- $P ;;
gh2) for v in ${GH_VALUES:-0 15 0 15}; do
       VTK_BAND_OPT=$v run gh2_$v 400 python bench.py --gpus 2 --comm host --config ${GH_CFG:-C3} --steps 3 --warmup 1 --no-cpu-baseline --spmv-reps 2
       grep '^{' gpurun_out/gh2_$v.log | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('band_opt', $v, round(d['value'],1), 'it/s', d.get('kernels',{}).get('band_step'))" >> gpurun_out/gh2.txt; done ;;
cfgs) run bench_c1 300 python bench.py --config C1 --steps 5 --warmup 1
      run bench_c2 300 python bench.py --config C2 --steps 5 --warmup 1
      run prof_c2 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2 -o run --output-format csv -- python bench.py --config C2 --steps 1 --warmup 1 --no-cpu-baseline --spmv-reps 5 ;;
c3x) for r in 1 2; do run bench_c3_$r 300 python bench.py --no-cpu-baseline; done ;;
membench) run build_mb 200 /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -o /tmp/membench_layout tools/membench_layout.hip
          run membench_layout 300 /tmp/membench_layout ;;
*) echo "unknown stage $st"; exit 2 ;;
esac; done
