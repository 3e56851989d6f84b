#!/bin/bash
# Round 3, session p: the PCIe ceiling of the host-resident path (scripts/probe_pcie.hip), with
# the probe (and so its pinned buffers) on a CPU of the GPU's socket and on one of the other.
set -u
TAG=${1:-r03p}
O=gpurun_out/$TAG
mkdir -p $O
BUS=$(python3 -c "
import os
print(os.popen('rocm-smi --showbus 2>/dev/null').read().split('PCI Bus:')[1].split()[0].lower())")
LOC=$(cut -d, -f1 /sys/bus/pci/devices/$BUS/local_cpulist | cut -d- -f1)
REM=$(python3 -c "
loc=open('/sys/bus/pci/devices/$BUS/local_cpulist').read().strip()
def parse(s):
    out=set()
    for p in s.split(','):
        a,_,b=p.partition('-'); out|=set(range(int(a),int(b or a)+1))
    return out
allc=parse(open('/sys/devices/system/cpu/online').read().strip())
print(min(allc-parse(loc)))")
echo "bus $BUS gpu-local cpu $LOC remote cpu $REM" | tee $O/cpus.txt
[ -n "$LOC" ] && [ -n "$REM" ] || exit 4
for c in $LOC $REM; do
  timeout -k 10 120 taskset -c $c ./scripts/probe_pcie > $O/pcie_cpu$c.jsonl 2> $O/pcie_cpu$c.err
  rc=$?; echo "cpu $c rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
