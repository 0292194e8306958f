set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_band.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/band2.log 2>&1
rc=$?; tail -2 gpurun_out/band2.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/ab_env.py --env VTK_BAND_CANON_SL --values 1,0 --rounds 6 > gpurun_out/ab_canonsl.json 2>gpurun_out/ab_canonsl.err || exit $?
cat gpurun_out/ab_canonsl.json
