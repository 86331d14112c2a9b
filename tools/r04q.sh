#!/bin/bash
# Round-4 A/B on c4 K2: L_inf selection by in-group ranks (default) against wave minimum
# searches (variants/lib_lr0.so); parity suite first.
#   tools/r04q.sh OUTDIR
N=${1:-r04q}; O=gpurun_out/$N
mkdir -p "$O"
tools/gpu_check.sh "$N" "tests/test_gpu_parity.py" "" || exit $?
grep -q " passed" "$O/tests.log" && ! grep -q " failed" "$O/tests.log" || { echo "tests failed"; exit 1; }
tools/exp.sh "$N" 'c4 - --workload c4' 'c4lr0 variants/lib_lr0.so --workload c4' 'c4b - --workload c4' \
  'c4lr0b variants/lib_lr0.so --workload c4' || exit $?
