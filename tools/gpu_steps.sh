#!/bin/bash
# GPU-box step runner: each argument is "SECONDS command..."; output of step i
# goes to gpurun_out/$OUT/step$i.log (OUT from the environment, default
# "steps").  Exit codes 0/1 continue (test failures, mismatches); anything
# else (crash, abort, time limit) ends the run before the GPU is touched again.
O=gpurun_out/${OUT:-steps}
mkdir -p "$O"
i=0
for s in "$@"; do
  i=$((i+1))
  t=${s%% *}; cmd=${s#* }
  echo "== step $i ($t s): $cmd"
  timeout -k 10 "$t" bash -c "$cmd" > "$O/step$i.log" 2>&1
  rc=$?
  echo "   rc=$rc"; tail -n 15 "$O/step$i.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: step $i rc=$rc"; exit $rc; fi
  if grep -qi "illegal memory access\|memory access fault\|hipErrorIllegalAddress" "$O/step$i.log"; then
    echo "stopping: step $i hit a GPU memory fault"; exit 3
  fi
done
