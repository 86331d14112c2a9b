#!/bin/bash
# Round-4 check: K2 / the generic path write 12-byte K4 slots directly (pair
# pass 0 reads 12 B per slot): the GPU suite, then c4 / c3v / c2 against the
# 16-byte form (PDP_K4_P12=0).
#   tools/r04k.sh OUTDIR
N=${1:-r04k}; O=gpurun_out/$N
mkdir -p "$O"
tools/gpu_check.sh "$N" "tests -m gpu" "" || exit $?
grep -q " passed" "$O/tests.log" && ! grep -q " failed" "$O/tests.log" || { echo "tests failed"; exit 1; }
tools/envexp.sh "$N" 'c4 -- --workload c4' 'c4p16 PDP_K4_P12=0 -- --workload c4' 'c4b -- --workload c4' \
  'c4i4 PDP_HIP_LIB=variants/lib_k4i4.so -- --workload c4' 'c3v -- --workload c3v' 'c3vp16 PDP_K4_P12=0 -- --workload c3v' 'c3 -- --workload c3' || exit $?
