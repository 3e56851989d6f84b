#!/bin/bash
# Host-runtime GPU tests under both HIP runtime settings: A = the test mitigation
# (host-memory kernel arguments, shader copies; tests/conftest.py), B = the runtime defaults
# (device kernel arguments, SDMA copies).  Test failures (rc 1) go on to the next leg; a crash,
# abort or timeout ends the script.
set -u
TAG=${1:-r02t}
O=gpurun_out/$TAG
mkdir -p $O
run() {
  timeout -k 10 300 python -u -m pytest tests/test_gpu_host.py -q --maxfail=5 --timeout 120 \
    --timeout-method thread -p no:cacheprovider > $O/$1.log 2>&1
  rc=$?; echo "$1 rc=$rc"; tail -3 $O/$1.log
  [ $rc -le 1 ] || exit 1
}
run mitigated
HSA_ENABLE_SDMA=1 HIP_FORCE_DEV_KERNARG=1 run defaults
echo done
