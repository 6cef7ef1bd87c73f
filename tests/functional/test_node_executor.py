"""The node-level multi-slot executor on the CPU (reference process boundary:
src/orion/core/worker/consumer.py:118-130, where GPUs enter in this framework).

* eight concurrent workers on an 8-device node (``ORION_GPUS=0..7``): every slot used, no
  device ever held by two trials at once, exactly ``max_trials`` trials run;
* a SIGKILLed worker: its orphaned trial keeps its GPU lease (the child holds the lock
  file), so the re-queued trial -- or any other -- cannot land on that device while the
  orphan lives;
* a 2-GPU trial goes through ``torch.distributed.run`` (gloo, ``train.py --device=cpu``)
  and reports exactly once, from rank 0.
"""
import json
import os
import signal
import subprocess
import sys
import time

from orion_amd.store import Database

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
DEMO = os.path.join(ROOT, "tests", "functional", "demo")
ORION = [sys.executable, os.path.join(ROOT, "bin", "orion")]


def _env(tmp_path, **kw):
    env = dict(os.environ)
    env.update(METAOPT_DB_ADDRESS=str(tmp_path / "orion.sqlite"), METAOPT_DB_TYPE="sqlite",
               XDG_CONFIG_HOME=str(tmp_path), TMPDIR=str(tmp_path),  # private lease locks
               SLOT_LOG=str(tmp_path / "slots.jsonl"))
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update(kw)
    return env


def _spans(tmp_path):
    p = tmp_path / "slots.jsonl"
    if not p.exists():
        return []
    return [json.loads(ln) for ln in p.read_text().splitlines() if ln.strip()]


def _overlaps(spans):
    """Pairs of trials that held one device at the same time."""
    bad = []
    by_dev = {}
    for s in spans:
        for d in (s["dev"] or "").split(","):
            by_dev.setdefault(d, []).append(s)
    for d, ss in by_dev.items():
        ss = sorted(ss, key=lambda s: s["t0"])
        for a, b in zip(ss, ss[1:]):
            if b["t0"] < a["t1"] - 1e-3:
                bad.append((d, a, b))
    return bad


def test_eight_workers_eight_slots(tmp_path):
    env = _env(tmp_path, ORION_GPUS=",".join(str(i) for i in range(8)))
    t0 = time.time()
    rc = subprocess.call(ORION + ["-n", "eight", "--max-trials", "24", "--pool-size", "8",
                                  "--workers", "8", "--gpus-per-trial", "1", "./slot_box.py",
                                  "-x~uniform(-5, 5)", "--sleep=1.0"],
                         cwd=DEMO, env=env, timeout=600)
    wall = time.time() - t0
    assert rc == 0
    store = Database("sqlite", host=str(tmp_path / "orion.sqlite"))
    (exp,) = store.read("experiments", {"name": "eight"})
    trials = store.read("trials", {"experiment": exp["_id"]})
    assert len(trials) == 24 and all(t["status"] == "completed" for t in trials), \
        [t["status"] for t in trials]
    spans = _spans(tmp_path)
    assert len(spans) == 24
    assert {s["dev"] for s in spans} == {str(i) for i in range(8)}, "not every slot was used"
    assert not _overlaps(spans)
    # each trial's recorded lease matches the device its process saw
    by_trial = {s["trial"]: s["dev"] for s in spans}
    for t in trials:
        assert t["gpus"] == [by_trial[str(t["_id"])]]
    # dispatch overhead per trial: lease -> completion minus the box's own sleep
    sec = lambda d: d.timestamp() if hasattr(d, "timestamp") else float(d)  # noqa: E731
    over = sorted(sec(t["end_time"]) - sec(t["start_time"]) - 1.0 for t in trials)
    rec = {"trials": 24, "workers": 8, "slots": 8, "wall_s": round(wall, 2),
           "dispatch_overhead_s_median": round(over[len(over) // 2], 3),
           "dispatch_overhead_s_max": round(over[-1], 3)}
    print(json.dumps(rec))
    assert over[len(over) // 2] < 5.0


def test_sigkilled_worker_keeps_its_gpu_locked_while_the_orphan_lives(tmp_path):
    env = _env(tmp_path, ORION_GPUS="0", ORION_STALE_AFTER_MIN_S="1")
    args = ORION + ["-n", "orphan", "--max-trials", "2", "--pool-size", "1", "--gpus-per-trial", "1",
                    "--heartbeat", "0.3", "./slot_box.py", "-x~uniform(-5, 5)", "--sleep=6",
                    "--ignore-term"]
    w1 = subprocess.Popen(args, cwd=DEMO, env=env)
    # wait until w1's first trial holds the GPU (its lease is recorded on the trial)
    db = Database("sqlite", host=str(tmp_path / "orion.sqlite"))
    deadline = time.time() + 120
    while time.time() < deadline:
        exps = db.read("experiments", {"name": "orphan"})
        if exps and db.count("trials", {"experiment": exps[0]["_id"], "gpus": ["0"]}):
            break
        time.sleep(0.1)
    else:
        w1.kill()
        raise AssertionError("first trial never started")
    time.sleep(0.5)
    w1.send_signal(signal.SIGKILL)
    w1.wait(timeout=30)
    killed_at = time.time()
    # a second worker resumes the experiment: the reaper re-queues the orphan's trial after
    # ~1 s, but the GPU stays locked until the orphan (which ignores its SIGTERM) exits
    rc = subprocess.call(args, cwd=DEMO, env=env, timeout=300)
    assert rc == 0
    spans = _spans(tmp_path)
    orphan = min(spans, key=lambda s: s["t0"])
    assert orphan["t1"] > killed_at, "the orphan did not outlive its worker"
    assert not _overlaps(spans), _overlaps(spans)
    (exp,) = db.read("experiments", {"name": "orphan"})
    done = db.count("trials", {"experiment": exp["_id"], "status": "completed"})
    assert done == 2


def test_two_gpu_trial_through_torchrun(tmp_path):
    out = tmp_path / "out"
    audit = tmp_path / "reports.txt"
    env = _env(tmp_path, ORION_GPUS="0,1", ORION_REPORT_AUDIT=str(audit))
    rc = subprocess.call(ORION + ["-n", "k2", "--max-trials", "1", "--pool-size", "1",
                                  "--gpus-per-trial", "2", os.path.join(ROOT, "train.py"),
                                  "--device=cpu", "--backend=gloo", "--model=gpt2-tiny",
                                  "--n_layer=1", "--n_head=2", "--n_embd=64", "--block_size=16",
                                  "--batch_size=2", "--gradient_accumulation_steps=2", "--max_iters=2",
                                  "--eval_interval=2", "--eval_iters=1", f"--out_dir={out}",
                                  "--dataset=", "--learning_rate~loguniform(1e-4, 1e-2)"],
                         cwd=str(tmp_path), env=env, timeout=600)
    assert rc == 0
    store = Database("sqlite", host=str(tmp_path / "orion.sqlite"))
    (exp,) = store.read("experiments", {"name": "k2"})
    (t,) = store.read("trials", {"experiment": exp["_id"]})
    assert t["status"] == "completed" and t["gpus"] == ["0", "1"]
    (r,) = [r for r in t["results"] if r["type"] == "objective"]
    assert r["name"] == "val_loss" and r["value"] > 0
    lines = audit.read_text().split("\n")
    reports = [ln for ln in lines if ln.strip()]
    assert len(reports) == 1 and reports[0].split()[0] == "0", reports
