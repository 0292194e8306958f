#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; [ $rc -le 1 ] || { echo "!! $name rc=$rc"; exit $rc; }; python3 - "gpurun_out/$name.log" <<'PY'
import json,sys
l=[x for x in open(sys.argv[1]) if x.startswith('{')]
if l:
    d=json.loads(l[0]); k=d['kernels']
    print(round(d['value'],1), d['ms_per_step'], {c:k[c]['avg_us'] for c in ('band_step','xupdate','spmv_resid_bj','spmv_bj_dc') if c in k})
PY
}
for rep in 1 2; do
  run xa_def_$rep 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --spmv-reps 3
  VTK_LIB=.abl/lib_xi1.so run xa_xi1_$rep 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --spmv-reps 3
  VTK_LIB=.abl/lib_xi4.so run xa_xi4_$rep 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --spmv-reps 3
done
