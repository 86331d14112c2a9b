#!/bin/bash
# Round-4 check: the analysis tests (new invalid-row test), then c5 with the later sort passes
# reduce-then-scan (PDP_SORT_TILESCAN=1; the fused first pass stays look-back).
#   tools/r04t.sh OUTDIR
N=${1:-r04t}; O=gpurun_out/$N
mkdir -p "$O"
tools/gpu_check.sh "$N" "tests/test_gpu_analysis.py" "" || exit $?
grep -q " passed" "$O/tests.log" && ! grep -q " failed" "$O/tests.log" || { echo "tests failed"; exit 1; }
tools/envexp.sh "$N" 'c5 -- --workload c5' 'c5rts PDP_SORT_TILESCAN=1 -- --workload c5' 'c5b -- --workload c5' \
  'c5rtsb PDP_SORT_TILESCAN=1 -- --workload c5' || exit $?
