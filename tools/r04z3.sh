#!/bin/bash
# Round-4 ablation: c5 pair extraction (k_ana_tile_pairs) without the n_partitions atomics
# (variants/lib_tp1.so) and without most pair writes as well (lib_tp2.so); timing only.
#   tools/r04z3.sh OUTDIR
N=${1:-r04z3}
tools/exp.sh "$N" 'c5 - --workload c5' 'c5tp1 variants/lib_tp1.so --workload c5' 'c5tp2 variants/lib_tp2.so --workload c5' \
  'c5b - --workload c5' || exit $?
