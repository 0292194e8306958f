#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 400 --timeout-method thread > gpurun_out/t4.log 2>&1
rc=$?
grep -v "^Extension" gpurun_out/t4.log | tail -n 12
[ $rc -le 1 ] || exit $rc
bash scripts/r04_ab2.sh
