#!/bin/bash
# Round-4 closing check on the final defaults: smoke(), the full GPU suite, the default bench line.
#   tools/r04_sanity.sh OUTDIR
R=${1:-r04s2}; O=gpurun_out/$R
mkdir -p "$O"
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { echo "smoke failed"; tail -5 "$O/smoke.log"; exit 1; }
tail -1 "$O/smoke.log"
tools/gpu_check.sh "$R" "tests -m gpu" "" || exit $?
grep -q " passed" "$O/tests.log" && ! grep -q " failed" "$O/tests.log" || { echo "tests failed"; exit 1; }
for w in c3 c4 c5; do
  timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline > "$O/bench_$w.json" 2> "$O/bench_$w.err" || { echo "bench $w failed"; tail -5 "$O/bench_$w.err"; exit 1; }
  python -c "import json; d=json.loads(open('$O/bench_$w.json').read().strip().splitlines()[-1]); print('$w', round(d['value']/1e9,2), round(d['ms_per_step'],2), {k: round(v['ms_per_launch'],2) for k,v in d['kernels'].items()})"
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d "$O/kt_c5" -o run -- \
  python -u bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline > "$O/kt_c5.out" 2> "$O/kt_c5.err" || { echo "kt rc=$?"; tail -5 "$O/kt_c5.err"; exit 1; }
grep -h "k_ana\|k_np_" "$O"/kt_c5/run_kernel_stats.csv
