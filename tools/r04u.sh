#!/bin/bash
# Round-4 re-check of round 3's "gfx950 miscompile" (DESIGN 3.1c): the parity, analysis and
# full-size suites with variants/lib_chk.so (current code + a bounds check on every scatter
# position) and with variants/lib_m6.so (the same plus round 3's mode-6 early return in digit_of).
#   tools/r04u.sh OUTDIR
N=${1:-r04u}; O=gpurun_out/$N
mkdir -p "$O"
for v in chk m6; do
  PDP_HIP_LIB=$PWD/variants/lib_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_analysis.py tests/test_gpu_fullsize.py -x -q --timeout 120 --timeout-method thread > "$O/tests_$v.log" 2>&1
  rc=$?
  echo "$v rc=$rc"; tail -4 "$O/tests_$v.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: rc=$rc"; exit $rc; fi
done
