#!/bin/bash
# Round-end evidence on the final sources: the full check (suite, bench, kernel trace, PMC
# passes), smoke, config 2's size sweep with its kernel trace, and the reference call pattern.
set -u
TAG=${1:-r02z}
bash scripts/gpu_check.sh $TAG || exit 1
O=gpurun_out/$TAG
grep -q "rc=[^0]" $O/status && { echo "check step failed"; cat $O/status; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
  || { echo "smoke rc=$?"; cat $O/smoke.log; exit 1; }
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --sweep --steps 50 --warmup 5 --no-cpu-baseline > $O/sweep.json 2> $O/sweep.err || { echo "sweep rc=$?"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/sweep_kt -o run -- python3 bench.py --sweep --steps 20 --warmup 2 --no-cpu-baseline > $O/sweep_prof.log 2>&1 || { echo "sweep kt rc=$?"; exit 1; }
timeout -k 10 300 python -u scripts/call_pattern.py > $O/call_pattern.json 2> $O/call_pattern.err || { echo "call_pattern rc=$?"; exit 1; }
cat $O/status; tail -1 $O/bench.log | cut -c1-300
