#!/bin/bash
# plain SpMV: FETCH_SIZE per launch and time with and without the XCD-swizzled group order
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() { local name=$1 to=$2; shift 2; echo "== $name"; timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; grep -v "^Extension\|amdgpu.ids\|^W2026\|^E2026\|^I2026" "gpurun_out/$name.log" | tail -n 1 | cut -c1-300; [ $rc -le 1 ] || { echo "!! $name rc=$rc"; exit $rc; }; }
for z in 0 1; do
  export VTK_SELL_SWZ=$z
  run swz_pmc_$z 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/swz_pmc_$z -o run --output-format csv -- python tools/spmv_lib_time.py --lib vt-precondition_amd/vtkrylov/lib/libvtkrylov.so --rounds 2 --reps 10
done
unset VTK_SELL_SWZ
run swz_ab 300 python tools/spmv_ab.py --rounds 6
