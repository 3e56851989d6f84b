#!/bin/bash
# Round 3 closing session: the whole GPU suite + kernel trace + PMC passes + bench
# (scripts/gpu_check.sh, ROUND=r03) and smoke on the final sources; then the failure-detection
# probe across real RCCL ranks (absent peer, dead peer), each bounded.
set -u
TAG=${1:-r03final2}
O=gpurun_out/$TAG
mkdir -p $O
ROUND=r03 bash scripts/gpu_check.sh $TAG
rc=$?; echo "gpu_check rc=$rc"; cat $O/status; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $O/smoke.log; [ $rc -ne 0 ] && exit $rc
for mode in absent dead; do
  timeout -k 10 120 python -u scripts/probe_rank_faults.py $TAG $mode > $O/fault_$mode.log 2>&1
  rc=$?; echo "fault probe $mode rc=$rc"; grep -v amdgpu.ids $O/fault_$mode.log | tail -14
  [ $rc -ne 0 ] && exit $rc
done
exit 0
