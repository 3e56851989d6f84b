#!/bin/bash
# Round 3: the host Func's per-call floor and the drop-in inside the reference's ring.
#   1. the resident-reducer and host-mapping GPU tests
#   2. scripts/probe_host_floor (C++, no Python in the loop), resident reducer on and off
#   3. scripts/dropin_sweep.py at the reference's call sizes and config 1's large sizes
# bash scripts/gpu_r03_floor.sh TAG
set -u
TAG=${1:-r03floor}
O=gpurun_out/$TAG
mkdir -p $O
fatal() { case $1 in 124|137|134|139|143) echo "FATAL $2 rc=$1"; exit $1;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_resident.py tests/test_gpu_host_map.py -m gpu \
    -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log; fatal $rc pytest; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 ./scripts/probe_host_floor > $O/floor_cpp.json 2> $O/floor_cpp.log
rc=$?; echo "floor rc=$rc"; fatal $rc floor; [ $rc -ne 0 ] && exit $rc
HYDRA_RESIDENT=0 timeout -k 10 200 ./scripts/probe_host_floor > $O/floor_cpp_launch.json \
    2> $O/floor_cpp_launch.log
rc=$?; echo "floor (launch) rc=$rc"; fatal $rc floor2; [ $rc -ne 0 ] && exit $rc
SIZES=${SIZES:-262144,524288,1048576,2097152,4194304,16777216,67108864} \
    timeout -k 10 500 python -u scripts/dropin_sweep.py > $O/dropin_sweep.json 2> $O/dropin_sweep.log
rc=$?; echo "dropin_sweep rc=$rc"; tail -2 $O/dropin_sweep.log
exit $rc
