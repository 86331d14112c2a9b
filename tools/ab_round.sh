#!/bin/bash
# GPU-box A/B round (one gpurun call): the parity / stream-order / RCCL suites, then bench lines
# (tools/exp.sh specs), then a rocprofv3 kernel trace of one workload.  Stops at the first failure.
#   tools/ab_round.sh OUT TRACE_WORKLOAD 'name lib args...' ...
O=$1; W=$2; shift 2
export TMPDIR=/tmp
mkdir -p gpurun_out/$O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_stream_order.py tests/test_gpu_rccl.py \
  -x -q --timeout 200 --timeout-method thread > gpurun_out/$O/t.log 2>&1 || { tail -5 gpurun_out/$O/t.log; exit 1; }
tail -1 gpurun_out/$O/t.log
tools/exp.sh $O "$@" || exit 1
if [ -n "$W" ] && [ "$W" != "-" ]; then
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -T -f csv -d gpurun_out/$O/kt_$W -o run -- \
    python bench.py --workload $W --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/$O/kt_$W.log 2>&1 || exit 1
  python tools/kt_top.py gpurun_out/$O/kt_$W/run_kernel_stats.csv
fi
