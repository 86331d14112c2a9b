#!/bin/bash
# Round-4 GPU check: smoke, the GPU parity suite, c3 / c3v bench lines, then
# bucket-pass ablations (sort only / linear write / no scatter / phase stamps),
# SoA-group variant builds and the HBM copy probes.  Stops at the first GPU
# failure.   tools/r04_check.sh OUTDIR
O=gpurun_out/${1:-r04}
mkdir -p "$O"
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { echo "smoke failed"; tail -5 "$O/smoke.log"; exit 1; }
tail -1 "$O/smoke.log"
tools/gpu_check.sh "${1:-r04}" "${TESTS-tests -m gpu}" "--workload c3;--workload c3v" || exit $?
tools/exp.sh "${1:-r04}" 'base - --workload c3' 'sortonly - --workload c3 --debug-flags 16384' \
  'linear - --workload c3 --debug-flags 81920' 'noscatter - --workload c3 --debug-flags 18432' \
  'stamps - --workload c3 --debug-flags 8192' 'soa4 variants/lib_soa4.so --workload c3' \
  'soa16 variants/lib_soa16.so --workload c3' 'c4 - --workload c4' 'c4old variants/lib_k2old.so --workload c4' \
  'c4perm variants/lib_k2perm.so --workload c4' || exit $?
timeout -k 10 300 python -u tools/copy_probe.py > "$O/copy.log" 2>&1 || { echo "copy probe failed"; tail -5 "$O/copy.log"; exit 1; }
tail -1 "$O/copy.log" | cut -c1-2000
# the 12-rows-per-thread (3072-row tile) build that faulted in round 3, after the loop-bound fix: parity once
PDP_HIP_LIB=$PWD/variants/lib_items12.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > "$O/items12_tests.log" 2>&1
rc=$?; echo "items12 parity rc=$rc"; tail -3 "$O/items12_tests.log"
[ $rc -eq 0 ] || exit $rc
tools/exp.sh "${1:-r04}" 'items12 variants/lib_items12.so --workload c3' || exit $?
