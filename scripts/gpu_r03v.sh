#!/bin/bash
# Round 3, session v: resident shape A/B on a GPU-local CPU, interleaved twice; then the drop-in
# sweep with every thread on the GPU's socket (taskset before any GPU use).
set -u
TAG=${1:-r03v}
O=gpurun_out/$TAG
mkdir -p $O
for rep in 1 2; do
  for sh in 128,4,4,2 128,1,4,2 128,4,4,4; do
    HYDRA_RESIDENT_SHAPE=$sh timeout -k 10 120 taskset -c 0 ./scripts/probe_host_floor 1024 4096 16384 65536 262144 1048576 4194304 \
        > $O/floor_${sh}_$rep.json 2> $O/floor_${sh}_$rep.log
    rc=$?; echo "$sh rep $rep rc=$rc"; [ $rc -ne 0 ] && exit $rc
  done
done
SIZES=${SIZES:-262144,1048576,4194304,16777216,67108864} \
    timeout -k 10 500 taskset -c 0-15 python -u scripts/dropin_sweep.py > $O/dropin_sweep.json 2> $O/dropin_sweep.log
rc=$?; echo "dropin_sweep rc=$rc"; tail -2 $O/dropin_sweep.log
exit $rc
