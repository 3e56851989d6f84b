#!/bin/bash
# Round 3, session t: is the per-call floor's bimodality (~5.8 vs ~8.5 us) the host thread's
# socket?  The GPU's NUMA node and local CPUs from sysfs, then the C++ floor probe pinned to a
# CPU local to the GPU and to one remote from it (taskset starts the probe: no exec after GPU
# initialisation).
set -u
TAG=${1:-r03t}
O=gpurun_out/$TAG
mkdir -p $O
{
  echo "nproc: $(nproc)"; grep Cpus_allowed_list /proc/self/status
  lscpu | grep -E "^NUMA|^Socket|^Model name" || true
  for d in /sys/class/drm/card*/device; do
    [ -f $d/numa_node ] && echo "$d numa=$(cat $d/numa_node) local=$(cat $d/local_cpulist 2>/dev/null)"
  done
  rocm-smi --showbus 2>/dev/null | head -20 || true
} > $O/topology.txt 2>&1
cat $O/topology.txt
ALLOWED=$(grep Cpus_allowed_list /proc/self/status | awk '{print $2}')
echo "allowed=$ALLOWED"
python3 - "$ALLOWED" > $O/cpus.txt <<'PY'
import glob, sys
def parse(s):
    out = []
    for part in s.split(","):
        if "-" in part:
            a, b = part.split("-"); out += range(int(a), int(b) + 1)
        elif part.strip():
            out.append(int(part))
    return out
allowed = set(parse(sys.argv[1]))
# the visible GPU: HIP_VISIBLE_DEVICES / the first card with a numa node
local = None
for d in sorted(glob.glob("/sys/class/drm/card*/device")):
    try:
        node = int(open(d + "/numa_node").read())
        cpus = set(parse(open(d + "/local_cpulist").read().strip()))
    except Exception:
        continue
    local = cpus
    break
loc = sorted(allowed & local) if local else []
rem = sorted(allowed - local) if local else []
print(loc[0] if loc else -1, rem[0] if rem else -1)
PY
read LOC REM < $O/cpus.txt
echo "local_cpu=$LOC remote_cpu=$REM"
for c in $LOC $REM; do
  [ "$c" = "-1" ] && continue
  timeout -k 10 120 taskset -c $c ./scripts/probe_host_floor 64 1024 16384 262144 > $O/floor_cpu$c.json 2> $O/floor_cpu$c.log
  echo "cpu $c rc=$?"
done
timeout -k 10 120 ./scripts/probe_host_floor 64 1024 16384 262144 > $O/floor_unpinned.json 2> $O/floor_unpinned.log
echo "unpinned rc=$?"
