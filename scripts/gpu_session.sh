#!/bin/bash
# One GPU-box session, parametrized: the steps named on the command line, in order, each under
# its own timeout; any failing step ends the session there (no later GPU step runs).
# Replaces the per-session gpu_r0*.sh scripts of rounds 1-3.
#
#   bash scripts/gpu_session.sh TAG STEP [STEP ...]
#
# STEP:
#   suite        the whole GPU suite, as the driver runs it (verbose, per-test timeouts)
#   tests        only $TESTS (pytest paths / -k expressions, space separated)
#   smoke        __graft_entry__.smoke()
#   prof         rocprofv3 kernel trace + separate FETCH_SIZE / WRITE_SIZE passes of the N=1
#                bench, the headline's dispatches from the trace, the PMC summary (ROUND=rNN)
#   bench[_X]    python bench.py (BENCH_ARGS), JSON line -> bench[_X].json (bench_2: a second run)
#   rehearseN    the N>1 bench at world size N on this one GPU (HYDRA_BENCH_SHARED_GPU=1: real
#                RCCL ranks over loopback sockets), 4 Mi fp32 / 16 Mi bf16 -> rehearse_nN.json
#                (REHEARSE_ARGS: extra bench.py flags, e.g. "--peer on" for the peer leg)
#   py:NAME      python scripts/NAME.py $PY_ARGS (a measurement script) -> NAME.log
#   pyprof:NAME  scripts/NAME.py under rocprofv3: a kernel trace, then separate FETCH_SIZE and
#                WRITE_SIZE passes -> NAME_{kt,fetch,write}/ (e.g. pyprof:fold_pmc)
#   bin:NAME     scripts/NAME $BIN_ARGS (a built probe) -> NAME.log
# Output: gpurun_out/TAG/{status,<step>.log,...}
set -u
TAG=${1:?usage: gpu_session.sh TAG STEP...}
shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
export TMPDIR=/tmp

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
{ nproc; grep -m1 "model name" /proc/cpuinfo; numactl -H 2>/dev/null | head -4; } > "$OUT/host.txt" 2>&1 || true
(cd hydra_amd/csrc && cat reduce_kernels.hip reduce_ops.h reduce_kernels.h | sha256sum | cut -d' ' -f1) > "$OUT/kernel_src.sha256"

rc_all=0
for s in "$@"; do
  case $s in
    suite)
      step pytest_gpu 1000 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider
      rc=$?; tail -2 "$OUT/pytest_gpu.log";;
    tests)
      # shellcheck disable=SC2086
      step pytest_sel 900 python -u -m pytest ${TESTS:?TESTS=...} -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider
      rc=$?; tail -2 "$OUT/pytest_sel.log";;
    smoke)
      step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
      rc=$?; tail -1 "$OUT/smoke.log";;
    prof)
      step rocprof_kt 600 rocprofv3 --kernel-trace --stats --output-format csv \
          -d "$OUT/prof_kt" -o run -- python3 "$ROOT/bench.py" --steps 100 --warmup 10 --no-cpu-baseline --no-host-path --no-sweep
      rc=$?
      python3 scripts/headline_from_trace.py "$OUT/prof_kt/run_kernel_trace.csv" 10 100 "$TAG" \
          > "$OUT/headline_from_trace.json" 2>&1 || true
      [ $rc -eq 0 ] && step rocprof_fetch 300 timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv \
          -d "$OUT/prof_fetch" -o run -- python3 "$ROOT/bench.py" --steps 20 --warmup 2 --no-cpu-baseline --no-host-path --no-sweep
      rc=$?
      [ $rc -eq 0 ] && step rocprof_write 300 timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv \
          -d "$OUT/prof_write" -o run -- python3 "$ROOT/bench.py" --steps 20 --warmup 2 --no-cpu-baseline --no-host-path --no-sweep
      rc=$?
      python3 scripts/pmc_summary.py "$OUT" "${ROUND:-r04}" > "$OUT/pmc_summary.json" 2>&1 || true;;
    bench|bench_*)
      # shellcheck disable=SC2086
      step "$s" 600 python bench.py ${BENCH_ARGS:-}
      rc=$?; tail -1 "$OUT/$s.log" > "$OUT/$s.json" 2>/dev/null;;
    rehearse*)
      n=${s#rehearse}
      step "rehearse_n$n" 600 env HYDRA_BENCH_SHARED_GPU=1 python -m torch.distributed.run --nnodes=1 \
          --nproc-per-node "$n" --master-addr 127.0.0.1 --master-port $((29600 + n)) bench.py \
          --gpus "$n" --steps 20 --warmup 3 --elements $((4 << 20)) --config5-elements $((16 << 20)) \
          --cpu-seconds 2 ${REHEARSE_ARGS:-}
      rc=$?; grep '^{' "$OUT/rehearse_n$n.log" | tail -1 > "$OUT/rehearse_n$n.json";;
    py:*)
      name=${s#py:}
      # shellcheck disable=SC2086
      step "$name" 900 python -u "scripts/$name.py" ${PY_ARGS:-}
      rc=$?;;
    pyprof:*)
      name=${s#pyprof:}
      # shellcheck disable=SC2086
      step "${name}_kt" 300 rocprofv3 --kernel-trace --stats --output-format csv \
          -d "$OUT/${name}_kt" -o run -- python3 "scripts/$name.py" ${PY_ARGS:-}
      rc=$?
      # shellcheck disable=SC2086
      [ $rc -eq 0 ] && step "${name}_fetch" 200 timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE \
          --output-format csv -d "$OUT/${name}_fetch" -o run -- python3 "scripts/$name.py" ${PY_ARGS:-}
      rc=$?
      # shellcheck disable=SC2086
      [ $rc -eq 0 ] && step "${name}_write" 200 timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE \
          --output-format csv -d "$OUT/${name}_write" -o run -- python3 "scripts/$name.py" ${PY_ARGS:-}
      rc=$?;;
    bin:*)
      name=${s#bin:}
      # shellcheck disable=SC2086
      step "$name" 600 "scripts/$name" ${BIN_ARGS:-}
      rc=$?;;
    *) echo "unknown step $s" >> "$OUT/status"; rc=2;;
  esac
  echo "$s rc=$rc"
  if [ $rc -ne 0 ]; then  # a failed step may hide a GPU fault: nothing more on the GPU
    rc_all=$rc
    echo "stopped after $s rc=$rc" >> "$OUT/status"
    break
  fi
done
echo done >> "$OUT/status"
exit $rc_all
