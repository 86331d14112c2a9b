#!/bin/bash
# GPU-box experiment runner over environment settings: each argument is
# "<name> <VAR=value ...> -- <bench args...>"; one bench.py run per argument
# under its own time limit, stops at the first failure.
#   tools/envexp.sh OUTDIR 'b1024 PDP_K2_BLOCKS=1024 PDP_K2_CACHE=1 -- --workload c3'
O=gpurun_out/$1; shift
mkdir -p "$O"
for spec in "$@"; do
  set -- $spec
  name=$1; shift
  envs=()
  while [ $# -gt 0 ] && [ "$1" != "--" ]; do envs+=("$1"); shift; done
  [ "$1" == "--" ] && shift
  echo "[exp] $name ${envs[*]} $*"
  env "${envs[@]}" timeout -k 10 180 python -u bench.py --no-cpu-baseline "$@" > "$O/$name.json" 2> "$O/$name.err" || { echo "[exp] $name failed rc=$?"; tail -5 "$O/$name.err"; exit 1; }
  python -c "import json,sys; d=json.loads(open('$O/$name.json').read().strip().splitlines()[-1]); print('$name', round(d['value']/1e9,2), round(d['ms_per_step'],2), {k: round(v['ms_per_launch'],2) for k,v in d['kernels'].items()})"
done
