for S in 25 32 50 100 250; do
  timeout -k 10 200 python bench.py --prec line --seg $S --steps 3 --warmup 1 --no-cpu-baseline --spmv-reps 2 > gpurun_out/seg_$S.log 2>&1 || exit $?
  python tools/brief.py gpurun_out/seg_$S.log $S
done
