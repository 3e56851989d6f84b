#!/bin/bash
# Store-policy / block-size chunk-sum variants 48-52: parity, then the A/B HBM-resident (rotate)
# and MALL-assisted (one pair back to back) at 16 Mi and 64 Mi.
set -u
TAG=${1:-r02m}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_reduce.py -x -q -k "variants_equal" --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_variants.log 2>&1
rc=$?; tail -2 $O/pytest_variants.log; [ $rc -eq 0 ] || exit 1
VARIANTS=0,41,42,48,49,50,52 MODES=rotate,inplace SIZES=16777216,67108864 ROUNDS=5 REPS=40 timeout -k 10 400 python -u scripts/tune.py > $O/tune_pol.json 2> $O/tune.err \
  || { echo "tune rc=$?"; tail $O/tune.err; exit 1; }
echo done
