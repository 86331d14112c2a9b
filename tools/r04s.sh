#!/bin/bash
# Round-4 check: k_ana_fix plain stores for private chains against variants/lib_prev.so
# (read-add-store); the full GPU suite first (also runs the k_thin cache variants).
#   tools/r04s.sh OUTDIR
N=${1:-r04s}; O=gpurun_out/$N
mkdir -p "$O"
tools/gpu_check.sh "$N" "tests -m gpu" "" || exit $?
grep -q " passed" "$O/tests.log" && ! grep -q " failed" "$O/tests.log" || { echo "tests failed"; exit 1; }
tools/exp.sh "$N" 'c5 - --workload c5' 'c5prev variants/lib_prev.so --workload c5' 'c5b - --workload c5' \
  'c5prevb variants/lib_prev.so --workload c5' || exit $?
