#!/bin/bash
# Mixed pinned/pageable host path: parity (reduce + drop-in), then the host-path measurements
# (isolated incl. the registered-bucket mode, configs 1/3) and the drop-in sweep with and
# without a registered bucket.
set -u
TAG=${1:-r02j}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_reduce.py tests/test_gpu_dropin.py tests/test_gpu_host.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit 1
SIZES=262144,1048576,4194304,16777216,67108864 timeout -k 10 600 python -u scripts/host_path.py > $O/host_path.json 2> $O/host_path.err \
  || { echo "host_path rc=$?"; tail $O/host_path.err; exit 1; }
timeout -k 10 900 python -u scripts/dropin_sweep.py > $O/dropin_sweep.json 2> $O/dropin_sweep.err \
  || { echo "dropin_sweep rc=$?"; tail $O/dropin_sweep.err; exit 1; }
echo done
