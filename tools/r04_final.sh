#!/bin/bash
# Round-4 final check, as the driver runs it: smoke(), the full GPU suite, the
# default bench line; then the profile round (tools/profile_round.sh).
#   tools/r04_final.sh ROUND
R=${1:-r04z}; O=gpurun_out/$R
mkdir -p "$O"
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { echo "smoke failed"; tail -5 "$O/smoke.log"; exit 1; }
tail -1 "$O/smoke.log"
tools/gpu_check.sh "$R" "tests -m gpu" "" || exit $?
grep -q " passed" "$O/tests.log" && ! grep -q " failed" "$O/tests.log" || { echo "tests failed"; exit 1; }
timeout -k 10 300 python -u bench.py > "$O/bench_default.json" 2> "$O/bench_default.err" || { echo "default bench failed"; tail -5 "$O/bench_default.err"; exit 1; }
tail -1 "$O/bench_default.json" | cut -c1-400
tools/profile_round.sh "$R"
