#!/bin/bash
# K2 build variants (prefetch depth x waves per SIMD): parity subset + c3/c4 stage times per library.
#   tools/k2_variants.sh libA.so libB.so ...
set -e
export TMPDIR=/tmp
O=gpurun_out/k2var
mkdir -p $O
for lib in "$@"; do
  b=$(basename $lib .so)
  PDP_HIP_LIB=$PWD/$lib timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -q -x -k "bound_accumulate and lean" --timeout 60 --timeout-method thread > $O/$b.test.log 2>&1 || { echo "$b tests FAILED"; tail -5 $O/$b.test.log; exit 1; }
  echo "$b tests ok"
  for w in c3 c4; do
    PDP_HIP_LIB=$PWD/$lib timeout -k 10 150 python -u bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline > $O/${b}_$w.json 2> $O/${b}_$w.err
    python -c "import json; d=json.load(open('$O/${b}_$w.json')); print('$b', '$w', round(d['ms_per_step'],2), 'K2', round(d['kernels']['buckets']['ms_per_launch'],2))"
  done
done
