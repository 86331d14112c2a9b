#!/bin/bash
# Round-4 check of the 12-byte K4 pair records: the GPU suite, the record-form
# A/B (PDP_K4_P12=0 forces 16-byte records), analysis chunk / lean prefetch
# variants, then bench lines with the CPU baseline for c2 / c4 / c5.
#   tools/r04g.sh OUTDIR
N=${1:-r04g}; O=gpurun_out/$N
mkdir -p "$O"
tools/gpu_check.sh "$N" "tests -m gpu" "" || exit $?
grep -q " passed" "$O/tests.log" && ! grep -q " failed" "$O/tests.log" || { echo "tests failed"; exit 1; }
tools/exp.sh "$N" 'c5 - --workload c5' 'c5ac4k variants/lib_ac4k.so --workload c5' \
  'c5ac8k variants/lib_ac8k.so --workload c5' 'c4 - --workload c4' 'c4pf2 variants/lib_pf2.so --workload c4' || exit $?
tools/envexp.sh "$N" 'c4p16 PDP_K4_P12=0 -- --workload c4' 'c3 -- --workload c3' 'c3p16 PDP_K4_P12=0 -- --workload c3' \
  'c3v -- --workload c3v' || exit $?
for w in c2 c4 c5; do
  timeout -k 10 300 python -u bench.py --workload $w > "$O/cpu_$w.json" 2> "$O/cpu_$w.err" || { echo "cpu $w rc=$?"; tail -5 "$O/cpu_$w.err"; exit 1; }
  python -c "import json; d=json.loads(open('$O/cpu_$w.json').read().strip().splitlines()[-1]); print('$w', round(d['value']/1e9,2), d['cpu_baseline']['value'], d['cpu_baseline']['sample'][:80])"
done
