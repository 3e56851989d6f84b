#!/bin/bash
# Round 3, session w (re-entry checkpoint): the whole GPU suite, kernel trace + PMC passes and the
# bench line (scripts/gpu_check.sh, ROUND=r03), then smoke() -- on the tree as committed.
set -u
TAG=${1:-r03w}
O=gpurun_out/$TAG
mkdir -p $O
ROUND=r03 bash scripts/gpu_check.sh $TAG
rc=$?; echo "gpu_check rc=$rc"; cat $O/status; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 $O/smoke.log
exit $rc
