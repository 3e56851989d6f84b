# PMC evidence for the peer kernel (one-GPU proxy): separate FETCH_SIZE and WRITE_SIZE passes,
# every rank wrapped by rocprofv3 --pmc.  Usage: bash scripts/session_peer_pmc.sh TAG ALGO P
set -o pipefail
OUT=gpurun_out/${1:?tag}; ALGO=${2:?algo}; P=${3:?P}; mkdir -p $OUT; export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 python -u scripts/peer_phases.py --algo $ALGO --P $P --n 67108864 --iters 10 --warmup 3 --rocprof $OUT/pmc_${ALGO}_p${P}_$C --pmc $C > $OUT/pmc_${ALGO}_p${P}_$C.json 2> $OUT/pmc_${ALGO}_p${P}_$C.err || exit $?
done
find $OUT -name '*.db' -delete
