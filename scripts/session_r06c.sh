# round 6: the peer kernel's phase clocks at P = 2 / 4 / 8 (64 Mi fp32, one-GPU proxy) and a
# rocprofv3 kernel trace of the P = 2 and P = 8 runs (every rank wrapped), then the peer /
# executor GPU tests.  Usage: bash scripts/session_r06c.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-r06c}; mkdir -p $OUT; export TMPDIR=/tmp
for P in 2 4 8; do
  timeout -k 10 240 python -u scripts/peer_phases.py --P $P --n 67108864 --iters 20 > $OUT/phases_p$P.json 2> $OUT/phases_p$P.err || exit $?
done
for P in 2 8; do
  timeout -k 10 300 python -u scripts/peer_phases.py --P $P --n 67108864 --iters 20 --rocprof $OUT/kt_p$P > $OUT/phases_kt_p$P.json 2> $OUT/phases_kt_p$P.err || exit $?
done
find $OUT -name '*.db' -delete
du -sh $OUT > $OUT/du.txt
