#!/bin/bash
# Round check: full parity suite, smoke, bench (N=1), rocprof kernel trace + PMC passes
# (scripts/gpu_check.sh), then the N>1 bench code path at world size 1 (--force-dist).
set -u
TAG=${1:-r01b}
bash scripts/gpu_check.sh $TAG || exit 1
O=gpurun_out/$TAG
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
  || { echo "smoke rc=$?"; cat $O/smoke.log; exit 1; }
timeout -k 10 400 python -u bench.py --force-dist --steps 10 --warmup 2 --no-config5 > $O/force_dist.log 2>&1 \
  || { echo "force-dist rc=$?"; tail -20 $O/force_dist.log; exit 1; }
cat $O/status; tail -1 $O/bench.log; tail -1 $O/force_dist.log | cut -c1-600
