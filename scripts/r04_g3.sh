#!/bin/bash
# full GPU suite on the current tree, then the round-4 in-process A/Bs (scripts/r04_ab1.sh)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 400 --timeout-method thread > gpurun_out/t3.log 2>&1
rc=$?
tail -n 4 gpurun_out/t3.log
[ $rc -le 1 ] || exit $rc
bash scripts/r04_ab1.sh
