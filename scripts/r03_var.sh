# process-level A/B of variant libraries (tools/bin/lib_<v>), alternating, REPS rounds
set -o pipefail
for rep in $(seq 1 ${REPS:-4}); do
  for v in ${VARIANTS}; do
    VTK_LIB=tools/bin/lib_$v/libvtkrylov.so timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --spmv-reps 2 ${BENCH_ARGS:-} > gpurun_out/v_${v}_$rep.log 2>&1 || exit $?
    python tools/bench_brief.py gpurun_out/v_${v}_$rep.log | sed 's/spmv_us.*band_step/band_step/' | cut -c1-110
  done
done
