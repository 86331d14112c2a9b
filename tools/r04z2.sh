#!/bin/bash
# Round-4 A/B on c4 K2 at 6 waves per SIMD: work chunk 1024 / 2048 (default) / 4096 rows per wave
# (variants/lib_lc{1k,4k}.so) and a 16384-block grid (variants/lib_lb16k.so).
#   tools/r04z2.sh OUTDIR
N=${1:-r04z2}
tools/exp.sh "$N" 'c4 - --workload c4' 'c4lc1k variants/lib_lc1k.so --workload c4' 'c4lc4k variants/lib_lc4k.so --workload c4' \
  'c4lb16k variants/lib_lb16k.so --workload c4' 'c4b - --workload c4' || exit $?
