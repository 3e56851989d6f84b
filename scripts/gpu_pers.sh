#!/bin/bash
# Persistent pipelined chunk-sum variants: parity first, then the HBM-resident A/B.
set -u
TAG=${1:-r02i}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_reduce.py -x -q -k "variants_equal" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_variants.log 2>&1
rc=$?; tail -2 $O/pytest_variants.log; [ $rc -eq 0 ] || exit 1
VARIANTS=0,45,46,47,41,40 MODES=rotate ROUNDS=5 REPS=40 timeout -k 10 300 python -u scripts/tune.py > $O/tune_pers.json 2> $O/tune.err \
  || { echo "tune rc=$?"; tail $O/tune.err; exit 1; }
echo done
