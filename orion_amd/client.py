"""In-script result reporting (component C18, ``src/orion/client/__init__.py``).

A black-box script calls ``report_results(data)`` exactly once.  Under an
orion worker the env var ``METAOPT_RESULTS_PATH`` names an existing file and
the results are JSON-dumped there; standalone, they are printed.  ``data`` is
a list of ``{'name', 'type' in (objective, constraint, gradient), 'value'}``.
In a multi-rank (torchrun) trial only rank 0 writes.
"""
from __future__ import annotations

import json
import os

IS_METAOPT_ON = False
IS_ORION_ON = False
_HAS_REPORTED_RESULTS = False
RESULTS_FILENAME = os.getenv("METAOPT_RESULTS_PATH", None) or os.getenv("ORION_RESULTS_PATH", None)

if RESULTS_FILENAME and os.path.isfile(RESULTS_FILENAME):
    IS_METAOPT_ON = IS_ORION_ON = True

if RESULTS_FILENAME and not IS_METAOPT_ON:
    raise RuntimeWarning("Results file path provided in environmental variable "
                         "does not correspond to an existing file.")


def _plain(v):
    if hasattr(v, "tolist"):
        return v.tolist()
    if hasattr(v, "item"):
        return v.item()
    return v


def report_results(data):
    """Report the trial's evaluation (once)."""
    global _HAS_REPORTED_RESULTS
    if _HAS_REPORTED_RESULTS:
        raise RuntimeWarning("Has already reported evaluation results once.")
    if isinstance(data, list):
        data = [dict(d, value=_plain(d.get("value"))) for d in data]
    if IS_METAOPT_ON:
        rank = int(os.environ.get("RANK", "0"))
        audit = os.environ.get("ORION_REPORT_AUDIT")  # tests: one line per call, any rank
        if audit:
            with open(audit, "a") as f:
                f.write(f"{rank} {os.getpid()}\n")
        if rank == 0:
            with open(RESULTS_FILENAME, "w") as f:
                json.dump(data, f)
    else:
        print(data)
    _HAS_REPORTED_RESULTS = True


def report_objective(value, name="objective"):
    """Shorthand: report a single objective value."""
    report_results([dict(name=name, type="objective", value=float(value))])
