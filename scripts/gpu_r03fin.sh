#!/bin/bash
# Round-3 closing check on a freshly rebuilt tree: scripts/gpu_check.sh (GPU suite, rocprofv3
# kernel trace + FETCH_SIZE / WRITE_SIZE passes, bench line), then smoke().
# bash scripts/gpu_r03fin.sh TAG
set -u
TAG=${1:-r03fin}
O=gpurun_out/$TAG
mkdir -p $O
ROUND=r03 bash scripts/gpu_check.sh $TAG
rc=$?; echo "gpu_check rc=$rc"; cat $O/status
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $O/smoke.log
exit $rc
