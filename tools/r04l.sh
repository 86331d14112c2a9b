#!/bin/bash
# Round-4 check: K0 with 16-byte column loads (two rows per lane) against
# variants/lib_hv1.so (PDP_HIST_V2=0): parity + full-size tests, then c3 / c4 / c2.
#   tools/r04l.sh OUTDIR
N=${1:-r04l}; O=gpurun_out/$N
mkdir -p "$O"
tools/gpu_check.sh "$N" "tests/test_gpu_parity.py tests/test_gpu_fullsize.py" "" || exit $?
grep -q " passed" "$O/tests.log" && ! grep -q " failed" "$O/tests.log" || { echo "tests failed"; exit 1; }
tools/exp.sh "$N" 'c3 - --workload c3' 'c3hv1 variants/lib_hv1.so --workload c3' 'c3b - --workload c3' \
  'c4 - --workload c4' 'c4hv1 variants/lib_hv1.so --workload c4' 'c2 - --workload c2' 'c2hv1 variants/lib_hv1.so --workload c2' || exit $?
