#!/bin/bash
# Round-4 K0 A/B: the bucket-digit histogram as the sum of the tile counts (PDP_HIST_V3=1, default)
# against one more LDS atomic per row (variants/lib_h2.so); parity + full-size tests first.
#   tools/r04z9.sh OUTDIR
N=${1:-r04z9}; O=gpurun_out/$N
mkdir -p "$O"
tools/gpu_check.sh "$N" "tests/test_gpu_parity.py tests/test_gpu_fullsize.py" "" || exit $?
grep -q " passed" "$O/tests.log" && ! grep -q " failed" "$O/tests.log" || { echo "tests failed"; exit 1; }
tools/exp.sh "$N" 'c3 - --workload c3' 'c3h2 variants/lib_h2.so --workload c3' 'c3b - --workload c3' \
  'c3h2b variants/lib_h2.so --workload c3' 'c2 - --workload c2' 'c2h2 variants/lib_h2.so --workload c2' || exit $?
