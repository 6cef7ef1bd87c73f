"""HPO on the MI355X node (reference process boundary:
src/orion/core/worker/consumer.py:118-130): the ``orion`` CLI with two worker processes
sharing ONE GPU through the node-local lease pool (``--gpus-per-trial 1``), every trial a
real ``train.py`` run of GPT-2-tiny on the HIP kernels.

Checks that the two workers serialise on the single GPU lease (no two trials overlap in
time), that every trial completes with an objective, and records trials/hour and the
per-trial dispatch overhead (trial wall time minus the trainer's own loop time) in
``gpurun_out/hpo_gpu.json`` for docs/PERFORMANCE.md."""
import json
import os
import subprocess
import sys
import time

import pytest

from orion_amd.store import Database

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
ORION = [sys.executable, os.path.join(ROOT, "bin", "orion")]


@pytest.mark.parametrize("runner", ["exec", "fork"])
def test_two_workers_share_one_gpu_lease(tmp_path, runner):
    db = str(tmp_path / "orion.sqlite")
    env = dict(os.environ, METAOPT_DB_ADDRESS=db, METAOPT_DB_TYPE="sqlite",
               XDG_CONFIG_HOME=str(tmp_path), ORION_GPUS="0",
               TMPDIR=str(tmp_path))  # private lease-lock directory for this test
    out = tmp_path / "out"
    t0 = time.time()
    rc = subprocess.call(ORION + ["-n", "gpu-smoke", "--max-trials", "8", "--workers", "2",
                                  "--gpus-per-trial", "1", "--pool-size", "4", "--trial-runner", runner,
                                  os.path.join(ROOT, "train.py"),
                                  "--device=cuda", "--model=gpt2-tiny", "--block_size=64",
                                  "--batch_size=8", "--gradient_accumulation_steps=1",
                                  "--max_iters=20", "--eval_interval=20", "--eval_iters=2",
                                  f"--out_dir={out}", "--dataset=", "--log_interval=10",
                                  "--learning_rate~loguniform(1e-4, 1e-3)"],
                         cwd=str(tmp_path), env=env, timeout=900)
    wall = time.time() - t0
    assert rc == 0
    store = Database("sqlite", host=db)
    (exp,) = store.read("experiments", {"name": "gpu-smoke"})
    trials = store.read("trials", {"experiment": exp["_id"]})
    done = [t for t in trials if t["status"] == "completed"]
    # the trial budget holds: --max-trials 8 with 2 workers and --pool-size 4 runs exactly 8
    # trainings (round 2 ran twice the budget: every idle worker registered a whole pool)
    assert len(trials) == 8 and len(done) == 8, [t["status"] for t in trials]
    for t in done:
        (r,) = [r for r in t["results"] if r["type"] == "objective"]
        assert r["value"] > 0
        assert t.get("gpus") == ["0"], t.get("gpus")
    # start_time = when the trial got its GPU lease (Experiment.record_lease)
    sec = lambda d: d.timestamp() if hasattr(d, "timestamp") else float(d)
    spans = sorted((sec(t["start_time"]), sec(t["end_time"])) for t in done)
    for (s0, e0), (s1, e1) in zip(spans, spans[1:]):
        assert s1 >= e0 - 0.01, "two trials held the single GPU lease at the same time"
    durs = [e - s for s, e in spans]
    busy = sum(durs)
    rec = {"runner": runner, "trials": len(done), "workers": 2, "gpus": 1, "wall_s": round(wall, 2),
           "trials_per_hour": round(len(done) / wall * 3600, 1),
           "trial_s_median": round(sorted(durs)[len(durs) // 2], 2),
           "lease_idle_s": round(max(0.0, (spans[-1][1] - spans[0][0]) - busy), 2),
           "cli_overhead_s": round(wall - (spans[-1][1] - spans[0][0]), 2)}
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", f"hpo_gpu_{runner}.json"), "w") as f:
        json.dump(rec, f)
    print(json.dumps(rec))
