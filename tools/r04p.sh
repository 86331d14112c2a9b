#!/bin/bash
# Round-4 A/B on c4 K2 (k_lean sorted): the flip bitonic network (default) against the
# direction-alternating one (variants/lib_nf.so), and 6 / 7 waves per SIMD
# (variants/lib_lw{6,7}.so); parity suite first.
#   tools/r04p.sh OUTDIR
N=${1:-r04p}; O=gpurun_out/$N
mkdir -p "$O"
tools/gpu_check.sh "$N" "tests/test_gpu_parity.py" "" || exit $?
grep -q " passed" "$O/tests.log" && ! grep -q " failed" "$O/tests.log" || { echo "tests failed"; exit 1; }
tools/exp.sh "$N" 'c4 - --workload c4' 'c4nf variants/lib_nf.so --workload c4' 'c4lw6 variants/lib_lw6.so --workload c4' \
  'c4lw7 variants/lib_lw7.so --workload c4' 'c4b - --workload c4' 'c4nfb variants/lib_nf.so --workload c4' || exit $?
