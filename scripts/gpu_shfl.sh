#!/bin/bash
# GPU session: full parity suite + smoke, then the misaligned-operand A/B of the chunk-sum
# (variant 40 = tuned default's unaligned dwordx4 loads, 44 = aligned loads + DPP realignment).
# Every GPU step under its own timeout; the first failure ends the script.
set -u
O=gpurun_out/shfl
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider > $O/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
  || { echo "smoke rc=$?"; cat $O/smoke.log; exit 1; }
cat $O/smoke.log
VARIANTS=0,40,44 SIZES=262144,16777216,67108864 MODES=inplace,misalign,cold ROUNDS=5 REPS=20 \
  timeout -k 10 300 python -u scripts/tune.py > $O/tune.json 2> $O/tune.err \
  || { echo "tune rc=$?"; cat $O/tune.err; exit 1; }
cat $O/tune.json
