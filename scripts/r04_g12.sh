#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; grep -v "^Extension\|amdgpu.ids" "gpurun_out/$name.log" | tail -n 3 | cut -c1-1500; [ $rc -le 1 ] || { echo "!! $name rc=$rc"; exit $rc; }; }
run t12 400 python -u -m pytest tests/test_gpu_dropin.py tests/test_gpu_multirank.py -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "grid4 or S4"
run c4_gr 600 python tools/ab_env.py --config C4 --env g4_gr --values 256,512 --rounds 3
run c4_gr512 600 python tools/ab_env.py --config C4 --env g4_ring --values 1024,2048,4096 --set g4_gr=512 --rounds 2
