# round 6: the push two-shot schedule -- peer GPU tests (every schedule), then the phase clocks
# of pull and push at P = 2 / 4 / 8 (64 Mi fp32, one-GPU proxy).  Usage: bash scripts/session_r06d.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-r06d}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_peer.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_peer.log 2>&1 || exit $?
for algo in peer2w peer2; do
  for P in 2 4 8; do
    timeout -k 10 240 python -u scripts/peer_phases.py --algo $algo --P $P --n 67108864 --iters 20 > $OUT/phases_${algo}_p$P.json 2> $OUT/phases_${algo}_p$P.err || exit $?
  done
done
