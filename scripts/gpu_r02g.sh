#!/bin/bash
# Full GPU suite on the current kernels; the fold's kernel trace + PMC passes (HBM-resident);
# the N>1 bench path at world size 1; and the watchdog's exit status through the real bench
# (a context phase that stalls: the measured headline is printed flagged, the process exits 3).
set -u
TAG=${1:-r02g}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || exit 1
bash scripts/gpu_fold_pmc.sh $TAG/fold || exit 1
timeout -k 10 400 python -u bench.py --force-dist --steps 10 --warmup 2 --no-config5 > $O/force_dist.log 2>&1 \
  || { echo "force-dist rc=$?"; tail -20 $O/force_dist.log; exit 1; }
HYDRA_BENCH_STALL_CONTEXT=300 timeout -k 10 300 python -u bench.py --force-dist --steps 10 --warmup 2 --no-config5 --watchdog-s 90 > $O/watchdog.log 2>&1
echo "watchdog run rc=$? (expect 3)"
tail -c 400 $O/force_dist.log; echo; tail -c 300 $O/watchdog.log
