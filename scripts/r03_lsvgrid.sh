set -o pipefail
timeout -k 10 300 python tools/ab_env.py --env VTK_SELL_CANON --values 1,0 --rounds 6 --prec line > gpurun_out/ab_canon_line2.json 2>gpurun_out/ab_lsvgrid.err || exit $?
cat gpurun_out/ab_canon_line2.json
timeout -k 10 300 python tools/ab_env.py --env VTK_SELL_CANON --values 1,0 --rounds 5 > gpurun_out/ab_canon_bj2.json 2>>gpurun_out/ab_lsvgrid.err || exit $?
cat gpurun_out/ab_canon_bj2.json
