#!/bin/bash
# The peer kernels' barrier costs on one GPU (P processes): the peer + bench GPU tests on the
# current kernels, then peer_bench.py event times with bit-identity for the shipped kernels
# against measurement variant 2512 (the push with plain stores and an L2 writeback at barrier 2:
# the kernel before r06zd; earlier sessions ran 2064 / 2256 the same way), then back-to-back
# phase clocks.  Output: gpurun_out/$1/
set -u
TAG=${1:?tag}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_peer.py tests/test_gpu_bench.py -m gpu -x -v \
    --timeout 200 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_peer.log" 2>&1 || exit $?
for P in 2 4 8; do
  timeout -k 10 300 python -u scripts/peer_bench.py --P $P --n 65536 16777216 67108864 \
      --algos peer2w peer2 peer1 --variants 0 2512 --iters 50 \
      > "$OUT/bench_p$P.json" 2> "$OUT/bench_p$P.err" || exit $?
done
for P in 2 8; do
  for V in 0 2512; do
    timeout -k 10 240 python -u scripts/peer_phases.py --P $P --algo peer2w --variant $V \
        --back-to-back > "$OUT/phases_p${P}_v$V.json" 2> "$OUT/phases_p${P}_v$V.err" || exit $?
  done
done
echo done > "$OUT/status"
