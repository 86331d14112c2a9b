#!/bin/bash
# Round-4 c5 pair extraction: the analysis tests (incl. the n_partitions forms test), then
# c5 with n_partitions from one atomic per pair (default) / the bucketed LDS histogram
# (PDP_ANA_NPART_HIST=1), and timing-only ablations without the atomics (variants/lib_tp1.so)
# and without most pair writes as well (lib_tp2.so).
#   tools/r04z3.sh OUTDIR
N=${1:-r04z3}; O=gpurun_out/$N
mkdir -p "$O"
tools/gpu_check.sh "$N" "tests/test_gpu_analysis.py" "" || exit $?
grep -q " passed" "$O/tests.log" && ! grep -q " failed" "$O/tests.log" || { echo "tests failed"; exit 1; }
tools/envexp.sh "$N" 'c5 -- --workload c5' 'c5h PDP_ANA_NPART_HIST=1 -- --workload c5' || exit $?
tools/exp.sh "$N" 'c5tp1 variants/lib_tp1.so --workload c5' 'c5tp2 variants/lib_tp2.so --workload c5' || exit $?
tools/envexp.sh "$N" 'c5b -- --workload c5' 'c5hb PDP_ANA_NPART_HIST=1 -- --workload c5' || exit $?
