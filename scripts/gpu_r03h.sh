#!/bin/bash
# Round 3, session h: the per-device resident reducer (one instance, leased slots, own queue).
#   1. resident-reducer + host-path GPU tests
#   2. does the persistent grid hold other streams up (own queue vs shared queue)
#   3. C++ per-call floor, resident on / off
#   4. drop-in sweep inside the reference ring (config 1 sizes)
# bash scripts/gpu_r03h.sh TAG
set -u
TAG=${1:-r03h}
O=gpurun_out/$TAG
mkdir -p $O
fatal() { case $1 in 124|137|134|139|143) echo "FATAL $2 rc=$1"; exit $1;; esac; }
timeout -k 10 200 python -u scripts/probe_queue_block.py > $O/queue_block.jsonl 2> $O/queue_block.log
rc=$?; echo "queue_block rc=$rc"; cut -c1-400 $O/queue_block.jsonl; fatal $rc queue; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_resident.py tests/test_gpu_host_map.py \
    tests/test_gpu_host.py tests/test_gpu_reduce.py -m gpu -x -v --timeout 200 \
    --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log; fatal $rc pytest; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 ./scripts/probe_host_floor > $O/floor_cpp.json 2> $O/floor_cpp.log
rc=$?; echo "floor rc=$rc"; fatal $rc floor; [ $rc -ne 0 ] && exit $rc
HYDRA_RESIDENT=0 timeout -k 10 200 ./scripts/probe_host_floor > $O/floor_cpp_launch.json \
    2> $O/floor_cpp_launch.log
rc=$?; echo "floor (launch) rc=$rc"; fatal $rc floor2; [ $rc -ne 0 ] && exit $rc
SIZES=${SIZES:-262144,1048576,4194304,16777216,67108864} \
    timeout -k 10 500 python -u scripts/dropin_sweep.py > $O/dropin_sweep.json 2> $O/dropin_sweep.log
rc=$?; echo "dropin_sweep rc=$rc"; tail -2 $O/dropin_sweep.log
exit $rc
