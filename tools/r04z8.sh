#!/bin/bash
# Round-4 attribution (timing only, results of the *_ns builds invalid): c5 with the current work units,
# with units snapped to partition starts (variants/lib_snap.so), and each without the direct output
# stores of k_ana_metrics (PDP_ANA_ABLATE_STORES=1: lib_ns.so, lib_snap_ns.so).
#   tools/r04z8.sh OUTDIR
N=${1:-r04z8}
tools/exp.sh "$N" 'c5 - --workload c5' 'c5ns variants/lib_ns.so --workload c5' 'c5snap variants/lib_snap.so --workload c5' \
  'c5snapns variants/lib_snap_ns.so --workload c5' 'c5b - --workload c5' || exit $?
