#!/usr/bin/env python3
"""Does the resident reducer's persistent grid hold up other streams' work?  With an instance
alive (idle limit 1 s), time a tiny torch kernel on each of 24 fresh streams and on the default
stream.  Run once per HYDRA_OPT_RESIDENT_QUEUE setting: the default (a non-blocking stream of the
greatest priority), `cumask` (a CU-masked stream: a hardware queue of its own, but blocking)
and `shared` (a plain non-blocking stream, which the runtime may put on a hardware queue another
stream uses); the default once more with 8 of torch's high-priority streams added.  Prints one
JSON line per run.
Usage (GPU box): python scripts/probe_queue_block.py > out.jsonl"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from hydra_amd import _lib  # noqa: E402
from tests.test_gpu_resident import _BLOCKING_PROBE, _with_opts  # noqa: E402

QUEUE = {"priority": 0, "shared": 1, "cumask": 2}  # HYDRA_OPT_RESIDENT_QUEUE
for mode, hi in (("priority", 0), ("cumask", 0), ("shared", 0), ("priority", 8)):
    code = _with_opts(_BLOCKING_PROBE % ROOT, {_lib.OPT_RESIDENT_IDLE_US: 1000000,
                                                _lib.OPT_RESIDENT_QUEUE: QUEUE[mode]})
    p = subprocess.run([sys.executable, "-c", code, str(hi)],
                       capture_output=True, text=True, timeout=120)
    row = {"queue": mode, "torch_high_priority_streams": hi, "rc": p.returncode}
    if p.returncode == 0:
        row.update(json.loads(p.stdout.strip().splitlines()[-1]))
    else:
        row["stderr"] = p.stderr[-1500:]
    print(json.dumps(row), flush=True)
