# The peer kernel's phase clocks under a per-rank rocprofv3 kernel trace (csv), one-GPU proxy.
# Usage: bash scripts/session_peer_kt.sh TAG ALGO P [P ...]   (ALGO: peer2 | peer2w)
set -o pipefail
OUT=gpurun_out/${1:?tag}; ALGO=${2:?algo}; shift 2; mkdir -p $OUT; export TMPDIR=/tmp
for P in "$@"; do
  timeout -k 10 300 python -u scripts/peer_phases.py --algo $ALGO --P $P --n 67108864 --iters 20 --rocprof $OUT/kt_${ALGO}_p$P > $OUT/phases_kt_${ALGO}_p$P.json 2> $OUT/phases_kt_${ALGO}_p$P.err || exit $?
done
find $OUT -name '*.db' -delete
