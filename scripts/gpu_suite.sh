#!/bin/bash
# The full GPU suite, as the driver runs it (plus per-test timeouts and verbose names).
set -u
TAG=${1:-suite}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; grep -E "beyond_32bit|mixed_pinned" $O/pytest_gpu.log | tail -3
exit $rc
