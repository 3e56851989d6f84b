#!/bin/bash
# Round-3 development session: a test selection, then the host-call floor probe (resident
# reducer on and off).  bash scripts/gpu_r03.sh TAG [pytest args...]
set -u
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest "$@" -m gpu -x -v --timeout 200 --timeout-method thread \
    -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/host_floor.py > $O/host_floor.json 2> $O/host_floor.log
rc=$?; echo "host_floor rc=$rc"; tail -2 $O/host_floor.log
[ $rc -ne 0 ] && exit $rc
HYDRA_RESIDENT=0 timeout -k 10 300 python -u scripts/host_floor.py > $O/host_floor_launch.json \
    2> $O/host_floor_launch.log
rc=$?; echo "host_floor (HYDRA_RESIDENT=0) rc=$rc"
exit $rc
