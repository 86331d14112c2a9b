#!/bin/bash
# Round-4 check: K4 reduce with the next round's loads issued ahead (default)
# against variants/lib_k4pf0.so (PDP_K4_PREFETCH=0): parity subset, then c4 / c3v.
#   tools/r04j.sh OUTDIR
N=${1:-r04j}; O=gpurun_out/$N
mkdir -p "$O"
tools/gpu_check.sh "$N" "tests/test_gpu_parity.py tests/test_gpu_rccl.py tests/test_gpu_fullsize.py" "" || exit $?
grep -q " passed" "$O/tests.log" && ! grep -q " failed" "$O/tests.log" || { echo "tests failed"; exit 1; }
tools/exp.sh "$N" 'c4 - --workload c4' 'c4pf0 variants/lib_k4pf0.so --workload c4' 'c4b - --workload c4' \
  'c4i4 variants/lib_k4i4.so --workload c4' 'c4i16 variants/lib_k4i16.so --workload c4' 'c3v - --workload c3v' 'c3vpf0 variants/lib_k4pf0.so --workload c3v' || exit $?
