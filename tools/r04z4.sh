#!/bin/bash
# Round-4: kernel trace of c5 with the bucketed n_partitions histogram (PDP_ANA_NPART_HIST=1).
#   tools/r04z4.sh OUTDIR
N=${1:-r04z4}; O=gpurun_out/$N
mkdir -p "$O"
export TMPDIR=/tmp PDP_ANA_NPART_HIST=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d "$O/kt" -o run -- \
  python -u bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline > "$O/kt.out" 2> "$O/kt.err" || { echo "rc=$?"; tail -5 "$O/kt.err"; exit 1; }
f=$(ls "$O"/kt/*/run_kernel_stats.csv 2>/dev/null | head -1); [ -z "$f" ] && f=$(find "$O/kt" -name "*kernel_stats.csv" | head -1)
head -25 "$f"
