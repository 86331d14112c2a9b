#!/bin/bash
# One GPU running the per-rank share of c3 under strong scaling at N = 1 / 2 / 4 / 8 (rows and
# privacy ids / N, all 1e6 partitions): the compute part of the driver's N-GPU SCALE steps.
#   tools/rank_share.sh OUTDIR
N=${1:-rank_share}
tools/exp.sh "$N" 'n1 - --workload c3' 'n2 - --workload c3 --rows 5e8 --pids 5e6' \
  'n4 - --workload c3 --rows 2.5e8 --pids 2.5e6' 'n8 - --workload c3 --rows 1.25e8 --pids 1.25e6' || exit $?
