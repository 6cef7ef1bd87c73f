"""Exact trial budget under heavy contention.

The reference's producer counted and then inserted (``src/orion/core/worker/producer.py:35-45``),
so concurrent workers overshot ``max_trials`` by up to workers x pool_size.  Here a producer
takes registration tokens from the experiment's budget counter with a compare-and-swap before
it inserts (``Experiment.claim_budget``), so 16 workers with pool_size 8 on max_trials 24
register and run exactly 24 trials -- every run, not by luck.
"""
import os
import subprocess
import sys

import pytest

from orion_amd.store import Database

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
DEMO = os.path.join(ROOT, "tests", "functional", "demo")
ORION = [sys.executable, os.path.join(ROOT, "bin", "orion")]


@pytest.mark.parametrize("run", range(5))
def test_sixteen_workers_register_exactly_max_trials(tmp_path, run):
    env = dict(os.environ)
    env.update(METAOPT_DB_ADDRESS=str(tmp_path / "orion.sqlite"), METAOPT_DB_TYPE="sqlite",
               XDG_CONFIG_HOME=str(tmp_path), TMPDIR=str(tmp_path), SLOT_LOG=str(tmp_path / "slots.jsonl"))
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "ORION_GPUS"):
        env.pop(k, None)
    rc = subprocess.call(ORION + ["-n", f"race{run}", "--max-trials", "24", "--pool-size", "8",
                                  "--workers", "16", "./slot_box.py", "-x~uniform(-5, 5)", "--sleep=0.05"],
                         cwd=DEMO, env=env, timeout=600)
    assert rc == 0
    store = Database("sqlite", host=str(tmp_path / "orion.sqlite"))
    (exp,) = store.read("experiments", {"name": f"race{run}"})
    trials = store.read("trials", {"experiment": exp["_id"]})
    assert len(trials) == 24, len(trials)
    assert all(t["status"] == "completed" for t in trials), [t["status"] for t in trials]
    assert exp["budget"]["used"] == 24
