#!/bin/bash
# Round-4 check: k_lean sorted group sums read kLeanSumBatch LDS entries per
# round trip (default 4; variants/lib_sb1.so = one per row as before, lib_sb8),
# and the sort_recs passes reduce-then-scan (PDP_SORT_TILESCAN=1) at c5 / c3.
#   tools/r04m.sh OUTDIR
N=${1:-r04m}; O=gpurun_out/$N
mkdir -p "$O"
tools/gpu_check.sh "$N" "tests/test_gpu_parity.py tests/test_gpu_analysis.py" "" || exit $?
grep -q " passed" "$O/tests.log" && ! grep -q " failed" "$O/tests.log" || { echo "tests failed"; exit 1; }
tools/envexp.sh "$N" 'c4 -- --workload c4' 'c4sb1 PDP_HIP_LIB=variants/lib_sb1.so -- --workload c4' \
  'c4sb8 PDP_HIP_LIB=variants/lib_sb8.so -- --workload c4' 'c4b -- --workload c4' \
  'c5 -- --workload c5' 'c5rts PDP_SORT_TILESCAN=1 -- --workload c5' 'c3 -- --workload c3' \
  'c3rts PDP_SORT_TILESCAN=1 -- --workload c3' || exit $?
