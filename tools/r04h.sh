#!/bin/bash
# Round-4 check: the GPU suite, then same-box A/B of the fused analysis pack
# (PDP_ANA_PACK=1: separate k_ana_pack) and of reduce-then-scan pid passes at c4.
#   tools/r04h.sh OUTDIR
N=${1:-r04h}; O=gpurun_out/$N
mkdir -p "$O"
tools/gpu_check.sh "$N" "tests -m gpu" "" || exit $?
grep -q " passed" "$O/tests.log" && ! grep -q " failed" "$O/tests.log" || { echo "tests failed"; exit 1; }
tools/envexp.sh "$N" 'c5 -- --workload c5' 'c5pack PDP_ANA_PACK=1 -- --workload c5' 'c5b -- --workload c5' \
  'c4 -- --workload c4' 'c4rts PDP_PASS_TILESCAN=1 -- --workload c4' || exit $?
