#!/bin/bash
# Runs on the GPU box (via gpurun).  For each workload W of $PROFILE_WORKLOADS
# (default "c3 c4"): one bench line (with the CPU baseline), a rocprofv3
# kernel-trace/stats pass, one PMC pass per HBM counter (FETCH_SIZE and
# WRITE_SIZE cannot share a pass on gfx950) and one SQ pass (wave cycles,
# waits, VALU, occupancy).  Then bench lines + kernel traces of
# $BENCH_WORKLOADS (default "c2 c5").  Outputs under gpurun_out/prof_<round>/;
# tools/pmc_traffic.py turns them into profiles/.
#   tools/profile_round.sh r03
R=${1:-r01}; shift || true
export TMPDIR=/tmp
O=gpurun_out/prof_$R
mkdir -p "$O"
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE"
run() {  # name timeout cmd...
  local n=$1 t=$2; shift 2
  echo "[profile] $n"
  timeout -k 10 "$t" "$@" > "$O/$n.out" 2> "$O/$n.err"
  local rc=$?
  if [ $rc -ne 0 ]; then echo "[profile] $n rc=$rc"; tail -5 "$O/$n.err"; fi
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  if grep -qi "illegal memory access\|memory access fault" "$O/$n.err"; then echo "[profile] GPU fault"; exit 3; fi
  return 0
}
for w in ${PROFILE_WORKLOADS:-c3 c4}; do
  run "bench_$w" 420 python -u bench.py --workload $w "$@"
  tail -1 "$O/bench_$w.out" | cut -c1-300
  run "kt_$w" 300 rocprofv3 --kernel-trace --stats -T -f csv -d "$O/kt_$w" -o run -- \
    python -u bench.py --workload $w --steps 5 --warmup 2 --no-cpu-baseline "$@"
  for c in FETCH_SIZE WRITE_SIZE; do
    run "pmc_${w}_$c" 240 rocprofv3 --pmc $c -T -f csv -d "$O/pmc_${w}_$c" -o run -- \
      python -u bench.py --workload $w --steps 1 --warmup 1 --no-cpu-baseline --no-profile "$@"
  done
  run "sq_$w" 240 rocprofv3 --pmc $SQ -T -f csv -d "$O/sq_$w" -o run -- \
    python -u bench.py --workload $w --steps 1 --warmup 1 --no-cpu-baseline --no-profile "$@"
done
for w in ${BENCH_WORKLOADS:-c2 c5 c3v}; do
  run "bench_$w" 360 python -u bench.py --workload $w "$@"
  tail -1 "$O/bench_$w.out" | cut -c1-300
  run "kt_$w" 300 rocprofv3 --kernel-trace --stats -T -f csv -d "$O/kt_$w" -o run -- \
    python -u bench.py --workload $w --steps 3 --warmup 1 --no-cpu-baseline "$@"
done
echo "[profile] done"
