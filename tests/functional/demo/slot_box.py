#!/usr/bin/env python3
"""Black box for the node-executor tests: appends one JSON line per trial to $SLOT_LOG with
the devices it was given (HIP_VISIBLE_DEVICES), its pid and its wall span, optionally
ignoring SIGTERM (an orphan that outlives its worker), then reports a quadratic objective."""
import argparse
import json
import os
import signal
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.dirname(
    os.path.abspath(__file__))))))
from orion.client import report_results  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("-x", type=float, required=True)
    ap.add_argument("--sleep", type=float, default=0.5)
    ap.add_argument("--ignore-term", action="store_true")
    a = ap.parse_args()
    if a.ignore_term:
        signal.signal(signal.SIGTERM, signal.SIG_IGN)
    t0 = time.time()
    time.sleep(a.sleep)
    t1 = time.time()
    rec = {"dev": os.environ.get("HIP_VISIBLE_DEVICES"), "pid": os.getpid(), "t0": t0, "t1": t1,
           "trial": os.environ.get("ORION_TRIAL_ID")}
    with open(os.environ["SLOT_LOG"], "a") as f:
        f.write(json.dumps(rec) + "\n")
    report_results([dict(name="obj", type="objective", value=(a.x - 1.0) ** 2)])


if __name__ == "__main__":
    main()
