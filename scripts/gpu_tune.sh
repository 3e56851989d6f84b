#!/bin/bash
# HBM-resident A/B sessions: every chunk-sum variant (tune.py rotate mode) and the P-way fold at
# the BASELINE owner blocks (tune_fold.py with 3 rotating source sets).
set -u
TAG=${1:-r02f}
O=gpurun_out/$TAG
mkdir -p $O
VARIANTS=$(python3 -c "print(','.join(map(str, range(45))))") MODES=rotate ROUNDS=4 REPS=40 \
  timeout -k 10 500 python -u scripts/tune.py > $O/tune_rotate_all.json 2> $O/tune.err \
  || { echo "tune rc=$?"; tail $O/tune.err; exit 1; }
ROTATE=3 BASELINE_ONLY=1 timeout -k 10 400 python -u scripts/tune_fold.py > $O/tune_fold_rot.json 2> $O/tune_fold.err \
  || { echo "tune_fold rc=$?"; tail $O/tune_fold.err; exit 1; }
echo done
