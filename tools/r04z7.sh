#!/bin/bash
# Round-4 c4 K4: split slots (keys, then values; PDP_K4_SOA=1, the default) against 12-byte slots
# (PDP_K4_SOA=0). The full GPU suite first (every parity mode runs the split form), then c4 / c3 A/B
# lines and a PMC pass of the c4 pair passes in both forms.
#   tools/r04z7.sh OUTDIR
N=${1:-r04z7}; O=gpurun_out/$N
mkdir -p "$O"
tools/gpu_check.sh "$N" "tests -m gpu" "" || exit $?
grep -q " passed" "$O/tests.log" && ! grep -q " failed" "$O/tests.log" || { echo "tests failed"; exit 1; }
tools/envexp.sh "$N" 'c4 -- --workload c4' 'c4a PDP_K4_SOA=0 -- --workload c4' 'c4b -- --workload c4' \
  'c4ab PDP_K4_SOA=0 -- --workload c4' 'c3 -- --workload c3' 'c3a PDP_K4_SOA=0 -- --workload c3' || exit $?
export TMPDIR=/tmp
for v in 1 0; do
  for c in FETCH_SIZE WRITE_SIZE; do
    PDP_K4_SOA=$v timeout -k 10 240 rocprofv3 --pmc $c -T -f csv -d "$O/pmc_${v}_$c" -o run -- \
      python -u bench.py --workload c4 --steps 1 --warmup 1 --no-cpu-baseline --no-profile > "$O/pmc_${v}_$c.out" 2> "$O/pmc_${v}_$c.err" \
      || { echo "pmc rc=$?"; tail -3 "$O/pmc_${v}_$c.err"; exit 1; }
  done
done
echo done
