#!/bin/bash
# Round-2 session: the full check (parity suite, bench, kernel trace, PMC passes), smoke, the
# reference call pattern, and the host-path sweeps of configs 1 and 3 (our host runtime and
# the reference ring with the hydra Func), each step under its own timeout.
set -u
TAG=${1:-r02e}
bash scripts/gpu_check.sh $TAG || exit 1
O=gpurun_out/$TAG
grep -q "rc=[^0]" $O/status && { echo "check step failed"; cat $O/status; exit 1; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
  || { echo "smoke rc=$?"; cat $O/smoke.log; exit 1; }
timeout -k 10 300 python -u scripts/call_pattern.py > $O/call_pattern.json 2> $O/call_pattern.err \
  || { echo "call_pattern rc=$?"; tail $O/call_pattern.err; exit 1; }
timeout -k 10 600 python -u scripts/host_path.py > $O/host_path.json 2> $O/host_path.err \
  || { echo "host_path rc=$?"; tail $O/host_path.err; exit 1; }
timeout -k 10 600 python -u scripts/dropin_sweep.py > $O/dropin_sweep.json 2> $O/dropin_sweep.err \
  || { echo "dropin_sweep rc=$?"; tail $O/dropin_sweep.err; exit 1; }
cat $O/status; tail -1 $O/bench.log | cut -c1-400
