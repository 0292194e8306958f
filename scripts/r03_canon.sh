# GPU check of the canonical SELL / line SpMV: parity tests, then in-process A/B (BJ and line)
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_band.py tests/test_gpu_line.py tests/test_gpu_multirank.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/canon_tests.log 2>&1
rc=$?; tail -3 gpurun_out/canon_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/ab_env.py --env VTK_SELL_CANON --values 1,0 --rounds 6 > gpurun_out/ab_canon_bj.json 2>gpurun_out/ab_canon.err || exit $?
cat gpurun_out/ab_canon_bj.json
timeout -k 10 300 python tools/ab_env.py --env VTK_SELL_CANON --values 1,0 --rounds 8 --prec line > gpurun_out/ab_canon_line.json 2>>gpurun_out/ab_canon.err || exit $?
cat gpurun_out/ab_canon_line.json
