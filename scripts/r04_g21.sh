#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; grep -v "^Extension\|amdgpu.ids" "gpurun_out/$name.log" | tail -n 1 | cut -c1-1500; [ $rc -le 1 ] || { echo "!! $name rc=$rc"; exit $rc; }; }
run b_j3 600 python tools/ab_env.py --config C3 --env band_j3 --values 2,3,4 --rounds 4 --perj
