#!/bin/bash
# Round-4 A/B: k_lean sorted at 5 (default) / 6 / 7 waves per SIMD (variants/lib_lw{6,7}.so) on c4.
#   tools/r04p.sh OUTDIR
N=${1:-r04p}
tools/exp.sh "$N" 'c4 - --workload c4' 'c4lw6 variants/lib_lw6.so --workload c4' 'c4lw7 variants/lib_lw7.so --workload c4' \
  'c4b - --workload c4' 'c4lw6b variants/lib_lw6.so --workload c4' || exit $?
