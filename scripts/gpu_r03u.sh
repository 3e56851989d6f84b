#!/bin/bash
# Round 3, session u: the final resident shape and the pageable lookup cache, host thread
# pinned to a CPU local to the GPU (socket 0 here; see r03t) and remote from it, against the
# previous shape (128,1,4,2).  Tests first.
set -u
TAG=${1:-r03u}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_resident.py tests/test_gpu_host_map.py \
    tests/test_gpu_host.py tests/test_gpu_reduce.py tests/test_gpu_dropin.py -m gpu -x -q --timeout 200 \
    --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log; case $rc in 0) ;; *) exit $rc;; esac
LOC=$(python3 -c "
import glob,os
bus=os.popen('rocm-smi --showbus 2>/dev/null').read().split('PCI Bus:')[1].split()[0].lower()
print(open('/sys/bus/pci/devices/%s/local_cpulist'%bus).read().split(',')[0].split('-')[0])")
REM=$(python3 -c "
import os
bus=os.popen('rocm-smi --showbus 2>/dev/null').read().split('PCI Bus:')[1].split()[0].lower()
loc=open('/sys/bus/pci/devices/%s/local_cpulist'%bus).read().strip()
def parse(s):
    out=set()
    for p in s.split(','):
        a,_,b=p.partition('-'); out|=set(range(int(a),int(b or a)+1))
    return out
allc=parse(open('/sys/devices/system/cpu/online').read().strip())
print(min(allc-parse(loc)))")
echo "gpu-local cpu $LOC, remote cpu $REM" | tee $O/cpus.txt
for c in $LOC $REM; do
  for sh in default 128,1,4,2; do
    if [ $sh = default ]; then unset HYDRA_RESIDENT_SHAPE; else export HYDRA_RESIDENT_SHAPE=$sh; fi
    timeout -k 10 120 taskset -c $c ./scripts/probe_host_floor 64 1024 4096 16384 65536 262144 1048576 4194304 \
        > $O/floor_cpu${c}_$sh.json 2> $O/floor_cpu${c}_$sh.log
    rc=$?; echo "cpu $c shape $sh rc=$rc"; [ $rc -ne 0 ] && exit $rc
  done
done
unset HYDRA_RESIDENT_SHAPE
SIZES=${SIZES:-262144,1048576,4194304,16777216,67108864} \
    timeout -k 10 500 python -u scripts/dropin_sweep.py > $O/dropin_sweep.json 2> $O/dropin_sweep.log
rc=$?; echo "dropin_sweep rc=$rc"; tail -2 $O/dropin_sweep.log
exit $rc
