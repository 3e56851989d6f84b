"""bench.py --gpus N watchdog (benchkit/watchdog.py): a hang after the headline still prints the
measured line, flagged, but the process exits non-zero; a hang before it exits non-zero with no
line.  A hung GPU process must never read as rc 0 to the driver."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

PROG = """
import sys, time
sys.path.insert(0, {root!r})
from benchkit import watchdog
state = {{}}
if {measured}:
    state["result"] = lambda: {{"metric": "m", "value": 1.0}}
watchdog.start({rank}, 0.3, state)
time.sleep(30)  # the hung collective
print("not reached")
"""


def run(measured: bool, rank: int = 0):
    code = PROG.format(root=ROOT, measured=measured, rank=rank)
    return subprocess.run([sys.executable, "-c", code], capture_output=True, text=True,
                          timeout=60)


def test_hang_after_headline_prints_flagged_line_and_fails():
    p = run(True)
    assert p.returncode == 3, p.stderr
    line = json.loads(p.stdout.strip().splitlines()[-1])
    assert line["value"] == 1.0 and "watchdog" in line
    assert "not reached" not in p.stdout


def test_hang_before_headline_fails_without_a_line():
    p = run(False)
    assert p.returncode == 3
    assert p.stdout.strip() == ""


def test_only_rank0_prints():
    p = run(True, rank=1)
    assert p.returncode == 3 and p.stdout.strip() == ""
