#!/bin/bash
# Round 3, session s: resident reducer shape A/B on one box (HYDRA_RESIDENT_SHAPE =
# blocks,batch,solo,tiles_per_block), the default first and last (drift check).
set -u
TAG=${1:-r03s}
O=gpurun_out/$TAG
mkdir -p $O
i=0
for sh in 128,1,4,2 128,4,4,4 128,4,4,2 128,2,4,2 128,1,1,2 128,4,8,4 128,2,8,4 128,1,4,2; do
  HYDRA_RESIDENT_SHAPE=$sh timeout -k 10 120 ./scripts/probe_host_floor 64 1024 4096 16384 65536 262144 1048576 4194304 \
      > $O/floor_$i.json 2> $O/floor_$i.log
  rc=$?; echo "$i $sh rc=$rc"; [ $rc -ne 0 ] && exit $rc
  echo "$sh" > $O/shape_$i.txt
  i=$((i+1))
done
