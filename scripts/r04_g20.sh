#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; grep -v "^Extension\|amdgpu.ids" "gpurun_out/$name.log" | tail -n 1 | cut -c1-300; [ $rc -le 1 ] || { echo "!! $name rc=$rc"; exit $rc; }; }
run t20 300 python -u -m pytest tests/test_gpu_rccl_solo.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread
run slab_c4_8 300 python bench.py --config C4 --slab 8 --comm-solo --steps 3 --warmup 1 --no-cpu-baseline
