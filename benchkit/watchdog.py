"""Watchdog for bench.py --gpus N: a hung collective must END the run, and must never read as
success.  After `seconds` the timer prints (rank 0) the latest measured headline, flagged with
"watchdog", and hard-exits every rank with EXIT_HUNG; before any headline exists it exits with
EXIT_HUNG and prints nothing on stdout.  os._exit: the hung thread is inside a GPU/RCCL call and
cannot be joined."""
import json
import os
import sys
import threading

EXIT_HUNG = 3


def start(rank: int, seconds: float, state: dict) -> threading.Timer:
    """state["result"] (set by the caller once a headline is measured) builds its JSON dict."""

    def _expire():
        done = state.get("result")
        if done is not None:
            sys.stderr.write(f"[hydra bench] rank {rank}: watchdog expired after the headline; "
                             "reporting it flagged, exit status " f"{EXIT_HUNG}\n")
            sys.stderr.flush()
            if rank == 0:
                r = done()
                r["watchdog"] = ("measurements after this headline (autotune, other algorithms, "
                                 "config 5) hung and were cut short; the process exits "
                                 f"{EXIT_HUNG}")
                print(json.dumps(r), flush=True)
        else:
            sys.stderr.write(f"[hydra bench] rank {rank}: watchdog expired before any "
                             "measurement, aborting\n")
            sys.stderr.flush()
        os._exit(EXIT_HUNG)

    dog = threading.Timer(float(seconds), _expire)
    dog.daemon = True
    dog.start()
    return dog
