#!/bin/bash
# Peer C++ class diagnostics + the rest of the GPU suite + the misaligned chunk-sum A/B.
set -u
O=gpurun_out/diag
mkdir -p $O
for i in 1 2; do
  timeout -k 10 120 tests/cpp/peer_algo 2 1000003 $(mktemp -d) > $O/peer_algo_$i.log 2>&1
  rc=$?; echo "peer_algo run $i rc=$rc"; cat $O/peer_algo_$i.log
  case $rc in 124|134|137|139) exit 1;; esac
done
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider -k "not algorithm_class_cpp" > $O/pytest.log 2>&1
rc=$?; tail -5 $O/pytest.log; case $rc in 0|1) ;; *) exit 1;; esac
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
  || { echo "smoke rc=$?"; cat $O/smoke.log; exit 1; }
VARIANTS=0,40,44 SIZES=262144,16777216,67108864 MODES=inplace,misalign,cold ROUNDS=5 REPS=20 \
  timeout -k 10 300 python -u scripts/tune.py > $O/tune.json 2> $O/tune.err \
  || { echo "tune rc=$?"; cat $O/tune.err; exit 1; }
cat $O/tune.json
