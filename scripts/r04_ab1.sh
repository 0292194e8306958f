#!/bin/bash
# round 4 A/Bs (in-process, one operator): plain SpMV order/grid, band-step variants
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; tail -n 3 "gpurun_out/$name.log"; [ $rc -eq 0 ] || { echo "!! $name rc=$rc"; exit $rc; }; }
run spmv_ab 240 python tools/spmv_ab.py --config C3 --settings "sell_swz=0;sell_swz=1;sell_swz=1,plain_grid=1024;sell_swz=1,plain_grid=4096;sell_swz=0,plain_grid=1024"
run band_spf 240 python tools/ab_env.py --env band_opt --values 0,1 --rounds 6 --perj
run band_wpc3 240 python tools/ab_env.py --env band_opt --values 1,3 --rounds 6 --perj --set band_j3=2
run band_j3 240 python tools/ab_env.py --env band_j3 --values 0,1,2,4 --rounds 6 --perj --set band_opt=3
