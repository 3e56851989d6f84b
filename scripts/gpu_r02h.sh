#!/bin/bash
# GPU suite (incl. the extended drop-in harness) and config 2's size sweep with its kernel trace.
set -u
TAG=${1:-r02h}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || exit 1
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --sweep --steps 50 --warmup 5 --no-cpu-baseline > $O/sweep.json 2> $O/sweep.err || { echo "sweep rc=$?"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o run -- python3 bench.py --sweep --steps 20 --warmup 2 --no-cpu-baseline > $O/prof.log 2>&1 || { echo "sweep kt rc=$?"; exit 1; }
echo done
