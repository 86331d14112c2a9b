#!/bin/bash
# K2 ablations on the GPU box: per-stage times of bench.py under debug flags
# (262144 no accumulator atomics, 1048576 L0 by minimum searches, 8388608 no L_inf
# ranking, 16777216 no kept-row sums, 33554432 LDS cache forced on, 67108864 k_thin v1 (was: 4096-block grid),
# 2097152 segment walk only).  Output: gpurun_out/k2abl/<workload>_<flags>.json
set -e
export TMPDIR=/tmp
O=gpurun_out/k2abl
mkdir -p $O
for spec in "$@"; do
  w=${spec%%:*}; f=${spec##*:}
  timeout -k 10 150 python -u bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline --debug-flags $f > $O/${w}_$f.json 2> $O/${w}_$f.err
  python -c "import json; d=json.load(open('$O/${w}_$f.json')); print('$w', $f, round(d['ms_per_step'],2), {k: round(v['ms_per_launch'],2) for k, v in d['kernels'].items()})"
done
