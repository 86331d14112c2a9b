#!/bin/bash
# Round-4 A/B: K4 reduce window of 1024 partitions (PDP_K4_SH=10, 4 workgroups per CU) at c4;
# the parity suite runs with it first.
#   tools/r04r.sh OUTDIR
N=${1:-r04r}; O=gpurun_out/$N
mkdir -p "$O"
PDP_K4_SH=10 tools/gpu_check.sh "$N" "tests/test_gpu_parity.py tests/test_gpu_rccl.py" "" || exit $?
grep -q " passed" "$O/tests.log" && ! grep -q " failed" "$O/tests.log" || { echo "tests failed"; exit 1; }
tools/envexp.sh "$N" 'c4 -- --workload c4' 'c4sh10 PDP_K4_SH=10 -- --workload c4' 'c4b -- --workload c4' \
  'c4sh10b PDP_K4_SH=10 -- --workload c4' || exit $?
