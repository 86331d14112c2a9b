#!/bin/bash
# Runs on the GPU box (via gpurun): headline bench line, a rocprofv3
# kernel-trace/stats pass, and one PMC pass per HBM counter (FETCH_SIZE and
# WRITE_SIZE cannot share a pass on gfx950), then one bench line for each of
# the other workloads (c2, c4, c5).  Outputs under gpurun_out/prof_<round>/;
# tools/pmc_traffic.py turns them into profiles/.
#   tools/profile_round.sh r02 [extra bench args]
set -e
R=${1:-r01}; shift || true
export TMPDIR=/tmp
O=gpurun_out/prof_$R
mkdir -p "$O"
echo "[profile] bench"
timeout -k 10 420 python -u bench.py "$@" > "$O/bench.json" 2> "$O/bench.err"
cat "$O/bench.json"
echo "[profile] kernel trace"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d "$O/kt" -o run -- \
  python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline "$@" > "$O/kt_bench.json" 2> "$O/kt.err"
for c in FETCH_SIZE WRITE_SIZE; do
  echo "[profile] pmc $c"
  timeout -s KILL 240 rocprofv3 --pmc $c -T -f csv -d "$O/pmc_$c" -o run -- \
    python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-profile "$@" > "$O/pmc_$c.json" 2> "$O/pmc_$c.err"
done
for w in ${PROFILE_WORKLOADS:-c2 c4 c5}; do
  echo "[profile] bench $w"
  timeout -k 10 300 python -u bench.py --workload $w > "$O/bench_$w.json" 2> "$O/bench_$w.err"
  echo "[profile] kernel trace $w"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -f csv -d "$O/kt_$w" -o run -- \
    python -u bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline > "$O/kt_bench_$w.json" 2> "$O/kt_$w.err"
done
echo "[profile] done"
