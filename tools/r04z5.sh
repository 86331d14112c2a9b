#!/bin/bash
# Round-4 c5: run-aggregated bucket count / scatter for n_partitions (now the default,
# PDP_ANA_NPART_HIST=0 = one atomic per pair); analysis + parity tests first.
#   tools/r04z5.sh OUTDIR
N=${1:-r04z5}; O=gpurun_out/$N
mkdir -p "$O"
tools/gpu_check.sh "$N" "tests/test_gpu_analysis.py tests/test_gpu_fullsize.py::test_c5_utility_analysis_full_size" "" || exit $?
grep -q " passed" "$O/tests.log" && ! grep -q " failed" "$O/tests.log" || { echo "tests failed"; exit 1; }
tools/envexp.sh "$N" 'c5 -- --workload c5' 'c5a PDP_ANA_NPART_HIST=0 -- --workload c5' 'c5b -- --workload c5' \
  'c5ab PDP_ANA_NPART_HIST=0 -- --workload c5' || exit $?
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d "$O/kt" -o run -- \
  python -u bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline > "$O/kt.out" 2> "$O/kt.err" || { echo "rc=$?"; tail -5 "$O/kt.err"; exit 1; }
grep -h "k_np_\|k_ana_tile" "$O"/kt/run_kernel_stats.csv
