#!/bin/bash
# Batched chunk-sum session: its parity tests, the reference call pattern (single / sync / graph
# / batch per 1 MiB segment) with a kernel trace, and the HBM-resident A/B of the chunk-sum
# variants (tune.py rotate mode).  Each GPU step has its own timeout; a crash ends the script.
set -u
TAG=${1:-r02d}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
fatal() { case $1 in 124|137|134|139|143) echo "FATAL step $2 rc=$1" | tee -a "$OUT/status"; exit $1;; esac; }
step() {
  local name=$1 t=$2; shift 2
  echo "== $name: $*" >> "$OUT/status"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc" >> "$OUT/status"
  fatal $rc "$name"
  return $rc
}
step pytest_reduce 300 python -u -m pytest tests/test_gpu_reduce.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider || exit 1
step call_pattern 300 python -u scripts/call_pattern.py || exit 1
export TMPDIR=/tmp
step call_pattern_kt 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/cp_kt" -o run -- python3 "$ROOT/scripts/call_pattern.py" || exit 1
VARIANTS=0,33,40,41,42,43,44,1,17,20,29,30,34,39,24,36,37 MODES=rotate ROUNDS=5 REPS=40 step tune_rotate 400 python -u scripts/tune.py || exit 1
echo done >> "$OUT/status"
