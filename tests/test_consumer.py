"""Consumer liveness contract: a reserved trial that waits for its GPU lease
keeps heart-beating, and a trial re-queued by another worker's reaper is abandoned --
never run a second time or completed twice."""
import os
import textwrap
import threading
import time

from orion_amd.core.consumer import Consumer
from orion_amd.core.experiment import Experiment
from orion_amd.core.gpus import GPUSlotPool
from orion_amd.core.producer import Producer
from orion_amd.store import Database


def _experiment(tmp_path, storage):
    marker = tmp_path / "runs.txt"
    script = tmp_path / "bb.py"
    script.write_text(textwrap.dedent(f"""
        import sys
        sys.path.insert(0, {os.getcwd()!r})
        open({str(marker)!r}, "a").write("ran\\n")
        from orion_amd.client import report_results
        report_results([dict(name="o", type="objective", value=1.0)])
    """))
    exp = Experiment("lease", storage, user="u")
    cfg = exp.configuration
    cfg.update(algorithms={"random": {}}, pool_size=1, max_trials=4)
    cfg["metadata"]["user_script"] = str(script)
    cfg["metadata"]["user_args"] = ["-x~uniform(0, 1)"]
    exp.configure(cfg)
    Producer(exp).produce()
    return exp, marker


def test_lease_wait_keeps_heartbeat_and_abandons_stolen_trial(tmp_path):
    storage = Database("memory")
    exp, marker = _experiment(tmp_path, storage)
    lock_dir = str(tmp_path / "locks")
    holder = GPUSlotPool(["0"], lock_dir).try_acquire(1)  # the only GPU is busy
    assert holder is not None
    cons = Consumer(exp, gpu_pool=GPUSlotPool(["0"], lock_dir), gpus_per_trial=1, heartbeat=0.05)
    trial = exp.reserve_trial(worker="w0")
    beats0 = storage.read("trials", {"_id": trial.id})[0]["heartbeat"]

    out = {}
    th = threading.Thread(target=lambda: out.setdefault("status", cons.consume(trial)))
    th.start()
    time.sleep(0.4)
    # still waiting for the lease, but alive: the heartbeat moved
    doc = storage.read("trials", {"_id": trial.id})[0]
    assert doc["status"] == "reserved" and doc["heartbeat"] > beats0
    # another worker's reaper decides this one is dead and re-queues the trial
    storage.write("trials", {"status": "interrupted"}, {"_id": trial.id})
    th.join(timeout=10)
    assert out.get("status") == "lost"
    assert not marker.exists(), "a stolen trial must not be run"
    assert storage.read("trials", {"_id": trial.id})[0]["status"] == "interrupted"
    holder.release()


def test_trial_runs_once_lease_is_free(tmp_path):
    storage = Database("memory")
    exp, marker = _experiment(tmp_path, storage)
    lock_dir = str(tmp_path / "locks")
    holder = GPUSlotPool(["0"], lock_dir).try_acquire(1)
    cons = Consumer(exp, gpu_pool=GPUSlotPool(["0"], lock_dir), gpus_per_trial=1, heartbeat=0.05)
    trial = exp.reserve_trial(worker="w0")
    threading.Timer(0.3, holder.release).start()
    assert cons.consume(trial) == "completed"
    assert marker.read_text() == "ran\n"
    assert storage.read("trials", {"_id": trial.id})[0]["status"] == "completed"
