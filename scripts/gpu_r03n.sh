#!/bin/bash
# Round 3, session n: staged calls cut into overlapping rounds (HYDRA_STAGE_SPLIT).
set -u
TAG=${1:-r03n}
O=gpurun_out/$TAG
mkdir -p $O
fatal() { case $1 in 124|137|134|139|143) echo "FATAL $2 rc=$1"; exit $1;; esac; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_resident.py tests/test_gpu_host_map.py \
    tests/test_gpu_host.py tests/test_gpu_reduce.py tests/test_gpu_dropin.py -m gpu -x -q --timeout 200 \
    --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log; fatal $rc pytest; [ $rc -ne 0 ] && exit $rc
for sp in 1 4 8; do
  HYDRA_STAGE_SPLIT=$sp timeout -k 10 200 ./scripts/probe_host_floor 65536 262144 1048576 4194304 16777216 \
      > $O/floor_split$sp.json 2> $O/floor_split$sp.log
  rc=$?; echo "floor split$sp rc=$rc"; fatal $rc floor; [ $rc -ne 0 ] && exit $rc
done
SIZES=${SIZES:-262144,1048576,4194304,16777216,67108864} \
    timeout -k 10 500 python -u scripts/dropin_sweep.py > $O/dropin_sweep.json 2> $O/dropin_sweep.log
rc=$?; echo "dropin_sweep rc=$rc"; tail -2 $O/dropin_sweep.log
exit $rc
