#!/bin/bash
# A/B of two builds of libvtkrylov.so: AB_TESTS on the in-tree build, then the bench
# (AB_BENCH args) alternating in-tree (new) and ablib/libvtkrylov_old.so (old).
set -e
O=gpurun_out/${AB_OUT:-ab_line}; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread ${AB_TESTS:-tests/test_gpu_line.py} > $O/tests.log 2>&1
for r in 1 2; do
  for v in new old; do
    if [ $v = old ]; then export VTK_LIB=$PWD/ablib/libvtkrylov_old.so; else unset VTK_LIB; fi
    timeout -k 10 300 python bench.py ${AB_BENCH:---prec line --steps 5 --warmup 1} --no-cpu-baseline > $O/bench_${v}_$r.log 2>&1
    tail -1 $O/bench_${v}_$r.log | python -c "import json,sys;d=json.loads(sys.stdin.read());r=d['roofline'];print('$v',$r,d['value'],r['avg_us'],r['frac'])"
  done
done
