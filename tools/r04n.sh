#!/bin/bash
# Round-4 check: k_ana_metrics with its per-pair operands staged in LDS (pipelined broadcast reads)
# against variants/lib_prev.so (the previous commit): analysis tests, then c5.
#   tools/r04n.sh OUTDIR
N=${1:-r04n}; O=gpurun_out/$N
mkdir -p "$O"
tools/gpu_check.sh "$N" "tests/test_gpu_analysis.py tests/test_gpu_fullsize.py" "" || exit $?
grep -q " passed" "$O/tests.log" && ! grep -q " failed" "$O/tests.log" || { echo "tests failed"; exit 1; }
tools/exp.sh "$N" 'c5 - --workload c5' 'c5prev variants/lib_prev.so --workload c5' 'c5b - --workload c5' \
  'c5prevb variants/lib_prev.so --workload c5' || exit $?
