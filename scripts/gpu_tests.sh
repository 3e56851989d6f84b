#!/bin/bash
# A selection of the GPU suite: bash scripts/gpu_tests.sh TAG [pytest args / test paths ...]
# (no args after TAG: the whole suite, as the driver runs it).  One pytest process, per-test
# timeouts, the log under gpurun_out/TAG.
set -u
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p $O
[ $# -eq 0 ] && set -- tests
timeout -k 10 ${SUITE_TIMEOUT:-900} python -u -m pytest "$@" -m gpu -v --timeout 200 \
    --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 $O/pytest_gpu.log
exit $rc
