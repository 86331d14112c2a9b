#!/bin/bash
# Round-4 check: the GPU suite (K4 pair passes and later pid passes now
# reduce-then-scan), then same-box A/B against the look-back forms and of the
# grouped-selection batch width (variants/lib_sel{2,8}.so).
#   tools/r04i.sh OUTDIR
N=${1:-r04i}; O=gpurun_out/$N
mkdir -p "$O"
tools/gpu_check.sh "$N" "tests -m gpu" "" || exit $?
grep -q " passed" "$O/tests.log" && ! grep -q " failed" "$O/tests.log" || { echo "tests failed"; exit 1; }
tools/envexp.sh "$N" 'c4 -- --workload c4' 'c4k4lb PDP_K4_TILESCAN=0 -- --workload c4' \
  'c4lb PDP_K4_TILESCAN=0 PDP_PASS_TILESCAN=0 -- --workload c4' 'c3 -- --workload c3' \
  'c3k4lb PDP_K4_TILESCAN=0 -- --workload c3' 'c2 -- --workload c2' 'c2k4lb PDP_K4_TILESCAN=0 -- --workload c2' \
  'c5 -- --workload c5' 'c5sel8 PDP_HIP_LIB=variants/lib_sel8.so -- --workload c5' \
  'c5sel2 PDP_HIP_LIB=variants/lib_sel2.so -- --workload c5' || exit $?
