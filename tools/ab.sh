#!/bin/bash
# Same-box A/B bench lines: each argument is "ENV=VAL ... -- bench args" (the
# part before "--" is exported for that run only).  One compact line per run;
# stops at the first run that fails.   OUT=<dir> tools/ab.sh "A=1 -- --workload c4" ...
O=gpurun_out/${OUT:-ab}
mkdir -p "$O"
i=0
for spec in "$@"; do
  i=$((i+1))
  envs=${spec%%--*}; args=${spec#*--}
  env $envs timeout -k 10 240 python -u bench.py --no-cpu-baseline $args > "$O/ab$i.json" 2> "$O/ab$i.err"
  rc=$?
  if [ $rc -ne 0 ]; then echo "run $i ($spec) rc=$rc"; tail -5 "$O/ab$i.err"; exit $rc; fi
  python -c "import json; d=json.loads(open('$O/ab$i.json').read().strip().splitlines()[-1]); print('[$spec]', round(d['value']/1e9,2), round(d['ms_per_step'],2), {k: round(v['ms_per_launch']*v['launches_per_step'],2) for k,v in d['kernels'].items()}, d.get('sweep_cycles_per_tile'))"
done
