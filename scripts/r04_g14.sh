#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; grep -v "^Extension\|amdgpu.ids" "gpurun_out/$name.log" | tail -n 2 | cut -c1-400; [ $rc -le 1 ] || { echo "!! $name rc=$rc"; exit $rc; }; }
run t14 600 python -u -m pytest tests/test_gpu_band.py tests/test_gpu_line.py tests/test_gpu_x0.py tests/test_gpu_dropin.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread
run bq14 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline
run bq14c4 300 python bench.py --config C4 --steps 2 --warmup 1 --no-cpu-baseline
