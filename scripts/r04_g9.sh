#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; grep -v "^Extension\|amdgpu.ids" "gpurun_out/$name.log" | tail -n 3 | cut -c1-1500; [ $rc -le 1 ] || { echo "!! $name rc=$rc"; exit $rc; }; }
run t9 300 python -u -m pytest tests/test_gpu_dropin.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k grid4
run c4_ring3 600 python tools/ab_env.py --config C4 --env g4_ring --values 0,768,1024,2048 --rounds 2
run c4_pd 600 python tools/ab_env.py --config C4 --env g4_pd --values 1,2,3,4 --set g4_ring=1024 --rounds 2
export VTK_G4_RING=1024
run c4_prof2 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c4p2 -o c4p2 --output-format csv -- python bench.py --config C4 --steps 2 --warmup 1 --no-cpu-baseline
