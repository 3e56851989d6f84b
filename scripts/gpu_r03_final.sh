#!/bin/bash
# Round 3 evidence session: the RCCL executor's enqueue cost at config 4,
# then scripts/gpu_check.sh (the whole GPU suite on the runtime's default copy path, rocprofv3
# kernel trace + FETCH_SIZE / WRITE_SIZE passes, the bench line).
# bash scripts/gpu_r03_final.sh TAG
set -u
TAG=${1:-r03final}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u scripts/executor_overhead.py > $O/executor_overhead.json 2> $O/executor_overhead.log
rc=$?; echo "executor_overhead rc=$rc"; case $rc in 124|137|134|139|143) exit $rc;; esac
ROUND=r03 bash scripts/gpu_check.sh $TAG
rc=$?; echo "gpu_check rc=$rc"; cat $O/status
exit $rc
