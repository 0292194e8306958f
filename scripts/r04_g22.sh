#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; grep -v "^Extension\|amdgpu.ids" "gpurun_out/$name.log" | tail -n 3 | cut -c1-600; [ $rc -le 1 ] || { echo "!! $name rc=$rc"; exit $rc; }; }
run t22 600 python -u -m pytest tests/test_gpu_band.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread
