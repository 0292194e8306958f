#!/bin/bash
# Two-library A/B over several bench configs: AB_TESTS on the in-tree build first, then for each
# config the bench alternating in-tree (new) and ablib/libvtkrylov_old.so (old), two rounds.
set -e
O=gpurun_out/${AB_OUT:-ab_multi}; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread ${AB_TESTS} > $O/tests.log 2>&1
i=0
while IFS= read -r cfg; do
  [ -z "$cfg" ] && continue; i=$((i+1))
  for r in 1 2; do
    for v in new old; do
      if [ $v = old ]; then export VTK_LIB=$PWD/ablib/libvtkrylov_old.so; else unset VTK_LIB; fi
      timeout -k 10 300 python bench.py $cfg --no-cpu-baseline > $O/b${i}_${v}_$r.log 2>&1
      grep '^{' $O/b${i}_${v}_$r.log | tail -1 | python -c "import json,sys;d=json.loads(sys.stdin.read());print('$i', '$cfg', '$v', $r, round(d['value'],1))"
    done
  done
done <<< "${AB_CFGS}"
