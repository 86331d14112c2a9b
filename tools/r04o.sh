#!/bin/bash
# Round-4 probe: c5 k_ana_metrics output stores -- bench with variants/lib_nostore.so (stores
# skipped, results invalid) against the default, and HBM bytes per kernel (PMC).
#   tools/r04o.sh OUTDIR
N=${1:-r04o}; O=gpurun_out/$N
mkdir -p "$O"
export TMPDIR=/tmp
tools/exp.sh "$N" 'c5 - --workload c5' 'c5nostore variants/lib_nostore.so --workload c5' || exit $?
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 240 rocprofv3 --pmc $c -T -f csv -d "$O/pmc_$c" -o run -- python -u bench.py --workload c5 --steps 1 --warmup 1 --no-cpu-baseline --no-profile > "$O/pmc_$c.out" 2> "$O/pmc_$c.err" || { echo "pmc $c rc=$?"; exit 1; }
done
echo done
