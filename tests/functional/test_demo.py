"""End-to-end CLI scenarios (reference: tests/functional/demo/test_demo.py), on the
SQLite store instead of MongoDB: real ``orion`` subprocesses, real black boxes."""
import os
import subprocess
import sys

import numpy
import pytest

from orion_amd.store import Database

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
DEMO = os.path.join(ROOT, "tests", "functional", "demo")
ORION = [sys.executable, os.path.join(ROOT, "bin", "orion")]


def _env(db):
    env = dict(os.environ)
    env["METAOPT_DB_ADDRESS"] = db
    env["METAOPT_DB_TYPE"] = "sqlite"
    env["XDG_CONFIG_HOME"] = os.path.dirname(db)
    return env


def test_demo_gradient_descent(tmp_path):
    db = str(tmp_path / "orion.sqlite")
    rc = subprocess.call(ORION + ["--config", "./orion_config.yaml", "./black_box.py",
                                  "-x~uniform(-50, 50)"], cwd=DEMO, env=_env(db), timeout=300)
    assert rc == 0
    store = Database("sqlite", host=db)
    (exp,) = store.read("experiments", {"name": "voila_voici"})
    assert exp["pool_size"] == 1 and exp["max_trials"] == 100 and exp["status"] == "done"
    assert exp["algorithms"] == {"gradient_descent": {"learning_rate": 0.1}}
    for k in ("user", "datetime", "orion_version", "user_script"):
        assert k in exp["metadata"]
    assert os.path.isabs(exp["metadata"]["user_script"])
    assert exp["metadata"]["user_args"] == ["-x~uniform(-50, 50)"]
    trials = sorted(store.read("trials", {"experiment": exp["_id"]}), key=lambda t: t["submit_time"])
    assert len(trials) < 15
    last = trials[-1]
    assert last["status"] == "completed"
    for r in last["results"]:
        assert r["type"] != "constraint"
        if r["type"] == "objective":
            assert abs(r["value"] - 23.4) < 1e-6 and r["name"] == "example_objective"
        elif r["type"] == "gradient":
            g = numpy.asarray(r["value"])
            assert 0.1 * numpy.sqrt(g.dot(g)) < 1e-7 and r["name"] == "example_gradient"
    (p,) = last["params"]
    assert p["name"] == "/x" and p["type"] == "real" and abs(p["value"] - 34.56789) < 1e-5


@pytest.mark.slow
def test_demo_two_workers(tmp_path):
    db = str(tmp_path / "orion.sqlite")
    procs = [subprocess.Popen(ORION + ["-n", "two_workers_demo", "--config", "./orion_config_random.yaml",
                                       "./black_box.py", "-x~norm(34, 3)"], cwd=DEMO, env=_env(db))
             for _ in range(2)]
    for p in procs:
        assert p.wait(timeout=900) == 0
    store = Database("sqlite", host=db)
    (exp,) = store.read("experiments", {"name": "two_workers_demo"})
    assert exp["pool_size"] == 2 and exp["max_trials"] == 400 and exp["status"] == "done"
    assert exp["algorithms"] == {"random": {}}
    assert exp["metadata"]["user_args"] == ["-x~norm(34, 3)"]
    trials = store.read("trials", {"experiment": exp["_id"]})
    assert all(t["status"] == "completed" for t in trials)
    assert 400 <= len(trials) <= 402
    assert trials[-1]["params"][0]["name"] == "/x" and trials[-1]["params"][0]["type"] == "real"


def test_resume_by_name(tmp_path):
    db = str(tmp_path / "orion.sqlite")
    args = ORION + ["-n", "resumable", "--max-trials", "3", "--pool-size", "1", "./black_box.py",
                    "-x~uniform(-50, 50)"]
    assert subprocess.call(args, cwd=DEMO, env=_env(db), timeout=300) == 0
    args[args.index("3")] = "6"
    assert subprocess.call(args, cwd=DEMO, env=_env(db), timeout=300) == 0
    store = Database("sqlite", host=db)
    (exp,) = store.read("experiments", {"name": "resumable"})
    assert exp["max_trials"] == 6
    assert store.count("trials", {"experiment": exp["_id"], "status": "completed"}) == 6


def test_broken_trials_stop_worker(tmp_path):
    db = str(tmp_path / "orion.sqlite")
    bad = tmp_path / "bad.py"
    bad.write_text("import sys\nsys.exit(3)\n")
    rc = subprocess.call(ORION + ["-n", "broken", "--max-trials", "5", "--pool-size", "1",
                                  str(bad), "-x~uniform(0, 1)"], env=_env(db), timeout=300)
    assert rc == 0
    store = Database("sqlite", host=db)
    (exp,) = store.read("experiments", {"name": "broken"})
    assert store.count("trials", {"experiment": exp["_id"], "status": "broken"}) == 3


def test_orion_tunes_train_py(tmp_path):
    """SURVEY.md §7.4's end-to-end slice on CPU: the orion CLI searches the trainer's
    learning rate; every trial trains GPT-2-tiny and reports its val loss."""
    db = str(tmp_path / "orion.sqlite")
    out = tmp_path / "out"
    rc = subprocess.call(ORION + ["-n", "lr_sweep", "--max-trials", "2", "--pool-size", "1",
                                  os.path.join(ROOT, "train.py"), "--device=cpu", "--model=gpt2-tiny",
                                  "--n_layer=1", "--n_head=2", "--n_embd=64", "--block_size=16",
                                  "--batch_size=2", "--gradient_accumulation_steps=1", "--max_iters=2",
                                  "--eval_interval=2", "--eval_iters=1", f"--out_dir={out}", "--dataset=",
                                  "--learning_rate~loguniform(1e-4, 1e-2)"],
                         cwd=str(tmp_path), env=_env(db), timeout=600)
    assert rc == 0
    store = Database("sqlite", host=db)
    (exp,) = store.read("experiments", {"name": "lr_sweep"})
    trials = store.read("trials", {"experiment": exp["_id"]})
    assert len(trials) >= 2 and all(t["status"] == "completed" for t in trials)
    for t in trials:
        (p,) = t["params"]
        assert p["name"] == "/learning_rate" and 1e-4 <= p["value"] < 1e-2
        (r,) = [r for r in t["results"] if r["type"] == "objective"]
        assert r["name"] == "val_loss" and r["value"] > 0


def test_cli_workers_flag_with_default_pool_size(tmp_path):
    """``--workers 2`` starts two worker processes that rebuild the experiment from the
    store; with no --pool-size the stored document must carry the default pool size (a
    new experiment's unset attributes must not override the defaults), and a GPU lease
    (--gpus-per-trial 1 on one device id) serialises the trials."""
    db = str(tmp_path / "orion.sqlite")
    env = _env(db)
    env.update(ORION_GPUS="0", TMPDIR=str(tmp_path))
    rc = subprocess.call(ORION + ["-n", "workers_flag", "--max-trials", "6", "--workers", "2",
                                  "--gpus-per-trial", "1", "./black_box.py", "-x~uniform(-50, 50)"],
                         cwd=DEMO, env=env, timeout=600)
    assert rc == 0
    store = Database("sqlite", host=db)
    (exp,) = store.read("experiments", {"name": "workers_flag"})
    assert exp["pool_size"] == 10 and exp["status"] == "done"
    trials = store.read("trials", {"experiment": exp["_id"]})
    done = [t for t in trials if t["status"] == "completed"]
    assert len(done) >= 6
    assert all(t["gpus"] == ["0"] for t in done)
    spans = sorted((t["start_time"], t["end_time"]) for t in done)
    assert all(b[0] >= a[1] for a, b in zip(spans, spans[1:])), "GPU lease held twice"
