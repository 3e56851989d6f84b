#!/bin/bash
# A/B of the push schedule's dynamic slabs (measurement variant 2032) against the shipped static
# k = b mod G assignment on one GPU (P processes): event times with bit-identity (peer_bench.py),
# then the phase clocks of both (peer_phases.py).  Output: gpurun_out/$1/
set -u
TAG=${1:?tag}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for P in 2 4 8; do
  timeout -k 10 300 python -u scripts/peer_bench.py --P $P --n 16777216 67108864 --algos peer2w \
      --variants 0 2032 --iters 50 > "$OUT/bench_p$P.json" 2> "$OUT/bench_p$P.err" || exit $?
done
for P in 2 8; do
  for V in 0 2032; do
    timeout -k 10 300 python -u scripts/peer_phases.py --P $P --algo peer2w --variant $V \
        > "$OUT/phases_p${P}_v$V.json" 2> "$OUT/phases_p${P}_v$V.err" || exit $?
  done
done
echo done > "$OUT/status"
