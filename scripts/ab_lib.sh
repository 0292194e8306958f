#!/bin/bash
# In-process-free A/B of two library builds: the tree's and vt-precondition_amd/vtkrylov/lib_$1
# (built by scripts/build_variant.sh and copied there so that it travels with the snapshot),
# alternating bench.py runs; prints it/s and the chosen kernel classes per run.
#   scripts/ab_lib.sh NAME [REPS] [BENCH ARGS...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
name=$1; reps=${2:-3}; shift 2 || shift $#
VL=vt-precondition_amd/vtkrylov/lib_$name/libvtkrylov.so
for rep in $(seq 1 "$reps"); do
  for v in base "$name"; do
    if [ "$v" = base ]; then unset VTK_LIB; else export VTK_LIB=$VL; fi
    timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --spmv-reps 2 "$@" > "gpurun_out/abl_${v}_$rep.log" 2>&1 || exit 1
    python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/abl_${v}_$rep.log') if l.startswith('{')][-1])
print('$v', $rep, round(d['value'],1), {k: round(e['avg_us'],1) for k, e in d['kernels'].items() if k in ('band_step','xupdate','spmv_bj','line_dc','dc_scalar','dc_finalize','dc_update','dc_dots')})"
  done
done
