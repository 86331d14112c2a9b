#!/bin/bash
# GPU-box check: parity tests (optionally a subset), then bench lines.  A
# pytest exit code other than 0/1 (crash, abort, time limit) stops the run
# before anything else touches the GPU.
#   tools/gpu_check.sh OUTDIR "pytest args" "bench args; bench args; ..."
O=gpurun_out/$1; T=$2; B=$3
mkdir -p "$O"
if [ -n "$T" ]; then
  timeout -k 10 600 python -u -m pytest $T -x -q --timeout 120 --timeout-method thread > "$O/tests.log" 2>&1
  rc=$?
  echo "tests rc=$rc"; tail -12 "$O/tests.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: tests rc=$rc"; exit $rc; fi
fi
i=0
IFS=';' read -ra RUNS <<< "$B"
for args in "${RUNS[@]}"; do
  [ -z "${args// }" ] && continue
  i=$((i+1))
  timeout -k 10 240 python -u bench.py --no-cpu-baseline $args > "$O/bench$i.json" 2> "$O/bench$i.err"
  rc=$?
  if [ $rc -ne 0 ]; then echo "bench $i ($args) rc=$rc"; tail -5 "$O/bench$i.err"; exit $rc; fi
  python -c "import json; d=json.loads(open('$O/bench$i.json').read().strip().splitlines()[-1]); print('$args', round(d['value']/1e9,2), round(d['ms_per_step'],2), {k: round(v['ms_per_launch'],2) for k,v in d['kernels'].items()})"
done
