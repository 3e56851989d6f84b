#!/bin/bash
# One GPU-box session: parity tests, rocprofv3 kernel trace + PMC passes (summarised on the box),
# then the bench, which reads that summary for roofline.traffic.
# Every GPU step runs under its own timeout; a crash/timeout/abort ends the script there.
# Usage (via gpurun): bash scripts/gpu_check.sh [tag]
set -u
TAG=${1:-r01}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"

fatal() {  # exit codes that mean the GPU step crashed or hung: stop everything
  case $1 in 124|137|134|139|143) echo "FATAL step $2 rc=$1" | tee -a "$OUT/status"; exit $1;; esac
}
step() {  # step NAME TIMEOUT CMD...
  local name=$1 t=$2; shift 2
  echo "== $name: $*" >> "$OUT/status"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc" >> "$OUT/status"
  fatal $rc "$name"
  return $rc
}

rocminfo 2>/dev/null | grep -m2 -E "gfx|Marketing" > "$OUT/device.txt" || true
nproc > "$OUT/host.txt"; grep -m1 "model name" /proc/cpuinfo >> "$OUT/host.txt" || true
# the chunk-sum kernel sources this session profiles (scripts/pmc_summary.py, bench.py traffic)
(cd hydra_amd/csrc && cat reduce_kernels.hip reduce_ops.h reduce_kernels.h | sha256sum | cut -d' ' -f1) > "$OUT/kernel_src.sha256"

if [ "${SKIP_TESTS:-0}" != "1" ]; then
  step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider
fi
if [ "${SKIP_PROF:-0}" != "1" ]; then
  export TMPDIR=/tmp
  step rocprof_kt 600 rocprofv3 --kernel-trace --stats --output-format csv \
      -d "$OUT/prof_kt" -o run -- python3 "$ROOT/bench.py" --steps 100 --warmup 10 --no-cpu-baseline
  # the headline's own dispatches from that trace (W = 10, S = 100 as above)
  python3 scripts/headline_from_trace.py "$OUT/prof_kt/run_kernel_trace.csv" 10 100 "$TAG" \
      > "$OUT/headline_from_trace.json" 2>&1 || true
  step rocprof_fetch 600 rocprofv3 --pmc FETCH_SIZE --output-format csv \
      -d "$OUT/prof_fetch" -o run -- python3 "$ROOT/bench.py" --steps 20 --warmup 2 --no-cpu-baseline
  step rocprof_write 600 rocprofv3 --pmc WRITE_SIZE --output-format csv \
      -d "$OUT/prof_write" -o run -- python3 "$ROOT/bench.py" --steps 20 --warmup 2 --no-cpu-baseline
  # the PMC summary of THESE kernel sources, written on the box before the bench reads it, so
  # the bench line below carries roofline.traffic (profiles/ itself is not merged back:
  # re-run scripts/pmc_summary.py on gpurun_out/<tag> in the build container to commit it)
  python3 scripts/pmc_summary.py "$OUT" "${ROUND:-r02}" > "$OUT/pmc_summary.json" 2>&1 || true
fi
step bench 600 python bench.py --steps 200 --warmup 20 ${BENCH_ARGS:-}
tail -1 "$OUT/bench.log" > "$OUT/bench.json" 2>/dev/null  # the JSON line alone
echo done >> "$OUT/status"
