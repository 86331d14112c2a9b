#!/bin/bash
# Round-4 A/B: adaptive K4 reduce chunk (about 1024 workgroups; PDP_K4_CHUNK=32768 = the fixed
# chunk) on the per-rank share of c3 at 8 GPUs and on c3 itself; parity + RCCL tests first.
#   tools/r04w.sh OUTDIR
N=${1:-r04w}; O=gpurun_out/$N
mkdir -p "$O"
tools/gpu_check.sh "$N" "tests/test_gpu_parity.py tests/test_gpu_rccl.py" "" || exit $?
grep -q " passed" "$O/tests.log" && ! grep -q " failed" "$O/tests.log" || { echo "tests failed"; exit 1; }
tools/envexp.sh "$N" 'n8 -- --workload c3 --rows 1.25e8 --pids 1.25e6' \
  'n8fix PDP_K4_CHUNK=32768 -- --workload c3 --rows 1.25e8 --pids 1.25e6' \
  'n8b -- --workload c3 --rows 1.25e8 --pids 1.25e6' 'n8fixb PDP_K4_CHUNK=32768 -- --workload c3 --rows 1.25e8 --pids 1.25e6' \
  'c3 -- --workload c3' || exit $?
