set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_dropin.py tests/test_gpu_band.py tests/test_gpu_rccl_solo.py tests/test_gpu_multirank.py tests/test_gpu_line.py > gpurun_out/t2.log 2>&1; rc=$?
tail -5 gpurun_out/t2.log
[ $rc -le 1 ] || exit $rc
bash scripts/gpu_steps.sh benchq slabs
