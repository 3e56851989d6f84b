#!/bin/bash
# Round 3, session x: the RCCL executor with 2 and 4 real RCCL ranks on the one GPU (per-rank
# NCCL_HOSTID, loopback sockets; tests/test_gpu_rccl_ranks.py), then the whole N>1 bench path
# at world size 2 and 4 the same way (HYDRA_BENCH_SHARED_GPU=1, small buckets: a code-path
# rehearsal of the driver's scale run, not an xGMI rate).
set -u
TAG=${1:-r03x}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_rccl_ranks.py -m gpu -x -v --timeout 300 \
    --timeout-method thread -p no:cacheprovider > $O/pytest_rccl_ranks.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 $O/pytest_rccl_ranks.log; [ $rc -ne 0 ] && exit $rc
for N in 2 4; do
  HYDRA_BENCH_SHARED_GPU=1 NCCL_DEBUG=WARN timeout -k 10 300 python -m torch.distributed.run \
      --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 --master-port $((29611 + N)) \
      bench.py --gpus $N --steps 5 --warmup 2 --elements 4194304 --config5-elements 4194304 \
      --cpu-seconds 2 > $O/bench_rehearsal_n$N.log 2>&1
  rc=$?; echo "bench rehearsal N=$N rc=$rc"; tail -c 1500 $O/bench_rehearsal_n$N.log; echo
  [ $rc -ne 0 ] && exit $rc
done
exit 0
