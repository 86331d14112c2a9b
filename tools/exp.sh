#!/bin/bash
# GPU-box experiment runner: each line of the list is "<name> <lib or -> <bench args...>";
# runs bench.py once per line under its own time limit, stops at the first failure.
#   tools/exp.sh OUTDIR 'name1 - --debug-flags 16384' 'name2 variants/lib_x.so' ...
O=gpurun_out/$1; shift
mkdir -p "$O"
for spec in "$@"; do
  set -- $spec
  name=$1; lib=$2; shift 2
  if [ "$lib" != "-" ]; then export PDP_HIP_LIB=$PWD/$lib; else unset PDP_HIP_LIB; fi
  echo "[exp] $name"
  timeout -k 10 180 python -u bench.py --no-cpu-baseline "$@" > "$O/$name.json" 2> "$O/$name.err" || { echo "[exp] $name failed rc=$?"; tail -5 "$O/$name.err"; exit 1; }
  python -c "import json,sys; d=json.loads(open('$O/$name.json').read().strip().splitlines()[-1]); print('$name', round(d['value']/1e9,2), {k: round(v['ms_per_launch'],2) for k,v in d['kernels'].items()}, d['roofline'].get('copy_peak_measured'), d.get('sweep_cycles_per_tile'))"
done
