"""Experiment / producer / reservation protocol on local stores
(reference: tests/unittests/core/test_experiment.py, test_producer.py)."""
import datetime
import os

import pytest

from orion_amd.core.experiment import Experiment, create_experiment, utcnow
from orion_amd.core.producer import Producer
from orion_amd.core.trial import Trial
from orion_amd.store import Database, DuplicateKeyError


@pytest.fixture
def storage():
    return Database("memory")


def _config(exp, algo=None, args=("-x~uniform(-50, 50)",), max_trials=10, pool_size=2):
    cfg = exp.configuration
    cfg["algorithms"] = algo or {"random": {}}
    cfg["pool_size"] = pool_size
    cfg["max_trials"] = max_trials
    cfg["metadata"]["user_script"] = "/bin/true"
    cfg["metadata"]["user_args"] = list(args)
    return cfg


def test_new_experiment_configure(storage):
    exp = Experiment("supernaedo", storage, user="tsirif")
    assert exp.status is None and exp.id is None
    exp.configure(_config(exp))
    assert exp.status == "pending" and exp.id is not None
    doc = storage.read("experiments", {"name": "supernaedo"})[0]
    assert doc["algorithms"] == {"random": {}} and doc["metadata"]["user"] == "tsirif"
    assert list(exp.space.keys()) == ["/x"]
    with pytest.raises(RuntimeError, match="Configuration is done"):
        exp.configure(_config(exp))


def test_resume_same_config(storage):
    exp = Experiment("e", storage, user="u")
    exp.configure(_config(exp))
    exp2 = Experiment("e", storage, user="u")
    assert exp2.id == exp.id and exp2.status == "pending"
    cfg = exp2.configuration
    cfg["max_trials"] = 50  # non-forking attribute: allowed
    exp2.configure(cfg)
    assert storage.read("experiments", {"_id": exp.id})[0]["max_trials"] == 50
    assert storage.count("experiments") == 1


def test_fork_is_rejected(storage):
    exp = Experiment("e", storage, user="u")
    exp.configure(_config(exp))
    exp2 = Experiment("e", storage, user="u")
    cfg = exp2.configuration
    cfg["metadata"]["user_args"] = ["-x~uniform(0, 1)"]
    with pytest.raises(NotImplementedError, match="forking"):
        exp2.configure(cfg)


def test_creation_race_duplicate_key(storage):
    a = Experiment("race", storage, user="u")
    b = Experiment("race", storage, user="u")
    a.configure(_config(a))
    with pytest.raises(DuplicateKeyError):
        b.configure(_config(b))


def test_create_experiment_retries_race(storage):
    a = Experiment("race2", storage, user="u")
    a.configure(_config(a))
    cmdargs = {"metadata": {"user_args": ["-x~uniform(-50, 50)"], "user_script": "/bin/true"},
               "max_trials": 10, "pool_size": 2}
    exp = create_experiment("race2", storage, dict(cmdargs=cmdargs), user="u")
    assert exp.id == a.id


def _ready(storage, **kw):
    exp = Experiment("w", storage, user="u")
    exp.configure(_config(exp, **kw))
    return exp


def test_produce_reserve_complete_cycle(storage):
    exp = _ready(storage)
    prod = Producer(exp)
    assert prod.produce() == 2
    assert exp.count_trials("new") == 2
    t = exp.reserve_trial(score_handle=prod.algorithm.score, worker="w0")
    assert t.status == "reserved" and t.start_time is not None and t.worker == "w0"
    t.results = [Trial.Result(name="o", type="objective", value=3.0)]
    exp.push_completed_trial(t)
    got = exp.fetch_completed_trials()
    assert [x.id for x in got] == [t.id]
    assert exp.fetch_completed_trials() == []  # incremental
    assert prod.update() == 0
    st = exp.stats
    assert st["trials_completed"] == 1 and st["best_evaluation"] == 3.0 and st["best_trials_id"] == t.id


def test_reserve_none_when_empty(storage):
    exp = _ready(storage)
    assert exp.reserve_trial() is None


def test_reserve_rejects_non_callable(storage):
    exp = _ready(storage)
    with pytest.raises(ValueError):
        exp.reserve_trial(score_handle=5)


def test_reserve_lost_race_retries(storage, monkeypatch):
    """Another worker grabs the chosen trial between read and CAS (reference:
    patch_sample_concurrent): the loop retries and gets the other one."""
    exp = _ready(storage)
    Producer(exp).produce()
    import random as _r
    real = _r.sample
    calls = {"n": 0}

    def sneaky(pop, k):
        calls["n"] += 1
        chosen = real(pop, k)
        if calls["n"] == 1:
            storage.write("trials", {"status": "reserved"}, {"_id": chosen[0].id})
        return chosen

    monkeypatch.setattr("orion_amd.core.experiment.random.sample", sneaky)
    t = exp.reserve_trial()
    assert t is not None and calls["n"] == 2
    assert exp.count_trials("reserved") == 2


def test_reserve_all_lost_returns_none(storage, monkeypatch):
    exp = _ready(storage)
    Producer(exp).produce()
    import random as _r
    real = _r.sample

    def always_lose(pop, k):
        chosen = real(pop, k)
        storage.write("trials", {"status": "reserved"}, {"_id": chosen[0].id})
        return chosen

    monkeypatch.setattr("orion_amd.core.experiment.random.sample", always_lose)
    assert exp.reserve_trial() is None


def test_is_done_by_max_trials(storage):
    exp = _ready(storage, max_trials=2)
    Producer(exp).produce()
    for _ in range(2):
        t = exp.reserve_trial()
        t.results = [Trial.Result(name="o", type="objective", value=1.0)]
        exp.push_completed_trial(t)
    assert exp.is_done
    # the query has no side effect; finish_if_done records the status
    assert storage.read("experiments", {"_id": exp.id})[0]["status"] == "pending"
    assert exp.finish_if_done()
    assert storage.read("experiments", {"_id": exp.id})[0]["status"] == "done"


def test_is_done_by_algorithm(storage):
    exp = _ready(storage, algo={"gradient_descent": {"learning_rate": 0.1}}, max_trials=100)
    exp.algorithms.algorithm.gradient = __import__("numpy").array([0.0])
    assert exp.is_done


def test_stats_with_no_completed_trials(storage):
    exp = _ready(storage)
    st = exp.stats
    assert st["trials_completed"] == 0 and st["best_trials_id"] is None


def test_stale_reservation_reaper(storage):
    exp = _ready(storage)
    Producer(exp).produce()
    t = exp.reserve_trial()
    storage.write("trials", {"heartbeat": utcnow() - datetime.timedelta(hours=1)}, {"_id": t.id})
    assert exp.fix_lost_trials(60) == 1
    assert storage.read("trials", {"_id": t.id})[0]["status"] == "interrupted"
    t2 = exp.reserve_trial()  # interrupted trials are reservable again
    assert t2 is not None


def test_fetch_tolerates_clock_skew(storage):
    """A completed trial stamped slightly before our watermark (other host's slow clock)."""
    exp = _ready(storage)
    Producer(exp).produce()
    exp.fetch_completed_trials()
    t = exp.reserve_trial()
    t.results = [Trial.Result(name="o", type="objective", value=1.0)]
    exp.push_completed_trial(t)
    storage.write("trials", {"end_time": utcnow() - datetime.timedelta(minutes=2)}, {"_id": t.id})
    assert [x.id for x in exp.fetch_completed_trials()] == [t.id]


def test_completion_is_a_cas_on_reserved(storage):
    exp = _ready(storage)
    Producer(exp).produce()
    t = exp.reserve_trial(worker="w0")
    # another worker's reaper re-queues the trial (stale heartbeat) and someone re-reserves it
    storage.write("trials", {"status": "interrupted"}, {"_id": t.id})
    t2 = exp.reserve_trial(worker="w1")
    assert t2.id == t.id or exp.reserve_trial(worker="w1") is not None
    t.results = [Trial.Result(name="o", type="objective", value=1.0)]
    assert not exp.push_completed_trial(t, only_if_reserved=True)  # w0 lost it
    doc = storage.read("trials", {"_id": t.id})[0]
    assert doc["status"] in ("reserved", "interrupted") and doc.get("results", []) == []


def test_lost_trial_is_out_of_reach_of_its_first_worker(storage):
    """The reaper re-queues w0's trial and w1 reserves it: w0's heartbeat, lease record and
    'broken' / 'interrupted' writes must all fail and leave w1's reservation untouched
    (they used to check only the status)."""
    exp = _ready(storage)
    exp.pool_size = 1
    Producer(exp).produce()
    t0 = exp.reserve_trial(worker="w0")
    assert t0 is not None and t0.worker == "w0"
    storage.write("trials", {"heartbeat": utcnow() - datetime.timedelta(hours=1)}, {"_id": t0.id})
    assert exp.fix_lost_trials(60) == 1
    t1 = exp.reserve_trial(worker="w1")
    assert t1 is not None and t1.id == t0.id and t1.worker == "w1"
    before = storage.read("trials", {"_id": t0.id})[0]
    assert not exp.update_heartbeat(t0)
    assert not exp.record_lease(t0, [3])
    assert not exp.set_trial_status(t0, "broken", only_if="reserved")
    assert not exp.set_trial_status(t0, "interrupted", only_if="reserved")
    t0.results = [Trial.Result(name="o", type="objective", value=1.0)]
    assert not exp.push_completed_trial(t0, only_if_reserved=True)
    after = storage.read("trials", {"_id": t0.id})[0]
    assert after["status"] == "reserved" and after["worker"] == "w1"
    assert after.get("heartbeat") == before.get("heartbeat") and after.get("gpus") == before.get("gpus")
    # the rightful owner's writes still succeed
    assert exp.update_heartbeat(t1) and exp.record_lease(t1, [0])
    t1.results = [Trial.Result(name="o", type="objective", value=2.0)]
    assert exp.push_completed_trial(t1, only_if_reserved=True)


def test_plan_configuration_is_pure(storage):
    from orion_amd.core.experiment import plan_configuration
    exp = Experiment("p", storage, user="u")
    cfg = _config(exp)
    plan = plan_configuration(None, cfg)
    assert plan.config["algorithms"] == {"random": {}} and list(plan.template.space) == ["/x"]
    assert storage.count("experiments") == 0
    same = dict(plan.config, max_trials=99)
    assert plan_configuration(plan.config, same).config["max_trials"] == 99
    other = copy_cfg = __import__("copy").deepcopy(plan.config)
    copy_cfg["metadata"]["user_args"] = ["-x~uniform(0, 2)"]
    with pytest.raises(NotImplementedError, match="metadata"):
        plan_configuration(plan.config, other)


# ---------------------------------------------------------------- budget claims
def test_slow_suggest_keeps_its_claim(storage, monkeypatch):
    """A producer whose suggest outlasts any grace period keeps its tokens: its owner (this
    process) is alive, so reconcile recovers nothing and the budget never overshoots."""
    exp = _ready(storage, max_trials=3, pool_size=2)
    prod = Producer(exp)
    orig = prod.algorithm.suggest
    other = Producer(exp)

    nested = []

    def slow_suggest(n):
        # while this claim is open: an aggressive reconcile (grace 0) and a second producer
        # (which shares the algorithm object, hence the guard)
        if not nested:
            nested.append(1)
            assert exp.reconcile_budget(grace_s=0.0) == 0
            assert other.produce() == 1  # only 3 - 2 tokens are left
        return orig(n)

    monkeypatch.setattr(prod.algorithm, "suggest", slow_suggest)
    assert prod.produce() == 2
    assert exp.count_trials("new") == 3
    b = storage.read("experiments", {"_id": exp.id})[0]["budget"]
    assert b["used"] == 3 and b["claims"] == {}
    assert Producer(exp).produce() == 0


def test_dead_producer_claim_is_recovered(storage):
    import subprocess
    import sys
    exp = _ready(storage, max_trials=4, pool_size=4)
    k, cid = exp.take_budget(3, owner="dead")
    assert k == 3
    # the claim's owner: a process that has exited
    p = subprocess.Popen([sys.executable, "-c", "pass"])
    p.wait()
    b = storage.read("experiments", {"_id": exp.id})[0]["budget"]
    b["claims"][cid]["pid"] = p.pid
    storage.write("experiments", {"budget": b}, {"_id": exp.id})
    # it inserted one of its three trials before dying
    t = Trial(params=[dict(name="/x", type="real", value=1.0)])
    t._id = exp.claim_trial_id(cid, 0)
    exp.register_trials([t])
    assert exp.reconcile_budget() == 2
    b = storage.read("experiments", {"_id": exp.id})[0]["budget"]
    assert b["used"] == 1 and b["claims"] == {}
    assert Producer(exp).produce() == 3


def test_settle_after_recovery_is_a_noop(storage):
    """A foreign-host claim presumed dead after the grace period is recovered once; when its
    producer turns out to be alive, its confirm fails (it inserts nothing) and its settle
    gives nothing back twice."""
    exp = _ready(storage, max_trials=4, pool_size=2)
    k, cid = exp.take_budget(2, owner="far")
    b = storage.read("experiments", {"_id": exp.id})[0]["budget"]
    b["claims"][cid]["host"] = "some-other-host"
    b["claims"][cid]["t"] = utcnow() - datetime.timedelta(hours=2)
    storage.write("experiments", {"budget": b}, {"_id": exp.id})
    assert exp.reconcile_budget() == 2
    assert storage.read("experiments", {"_id": exp.id})[0]["budget"]["used"] == 0
    assert not exp.confirm_claim(cid)
    exp.settle_budget(cid, 0)
    assert storage.read("experiments", {"_id": exp.id})[0]["budget"]["used"] == 0
    assert exp.take_budget(9)[0] == 4


# ---------------------------------------------------------------- claim owners
def _edit_claim(storage, exp, cid, **kw):
    b = storage.read("experiments", {"_id": exp.id})[0]["budget"]
    b["claims"][cid].update(kw)
    storage.write("experiments", {"budget": b}, {"_id": exp.id})


def test_claim_in_another_pid_namespace_is_not_probed(storage):
    """Same host name, other pid namespace (host-networking containers): a pid that does not
    exist HERE says nothing about the owner, so only the grace period recovers the claim."""
    exp = _ready(storage, max_trials=4, pool_size=2)
    k, cid = exp.take_budget(2, owner="ns")
    _edit_claim(storage, exp, cid, pid=2 ** 22 + 12345, pidns=-1)
    assert exp.reconcile_budget() == 0
    _edit_claim(storage, exp, cid, t=utcnow() - datetime.timedelta(hours=2))
    assert exp.reconcile_budget() == 2


def test_reused_pid_counts_as_dead_owner(storage):
    """The claim's pid is alive but started at another time: a reused pid, the owner is gone."""
    exp = _ready(storage, max_trials=4, pool_size=2)
    k, cid = exp.take_budget(2, owner="reused")
    me = storage.read("experiments", {"_id": exp.id})[0]["budget"]["claims"][cid]
    assert me["pid"] == os.getpid() and me["start"] is not None
    assert exp.reconcile_budget() == 0  # alive, same start time
    _edit_claim(storage, exp, cid, start=me["start"] - 1)
    assert exp.reconcile_budget() == 2


def test_inserting_claim_waits_for_its_grace(storage):
    """A confirmed (insert-stage) claim is never recovered within CLAIM_INSERT_GRACE_S of the
    confirmation, even when its owner probes dead; a broken trial of the claim counts as
    accounted for (it already returned its token)."""
    import subprocess
    import sys
    exp = _ready(storage, max_trials=4, pool_size=4)
    k, cid = exp.take_budget(3, owner="ins")
    assert exp.confirm_claim(cid)
    p = subprocess.Popen([sys.executable, "-c", "pass"])
    p.wait()
    _edit_claim(storage, exp, cid, pid=p.pid)
    ts = []
    for i in range(2):
        t = Trial(params=[dict(name="/x", type="real", value=float(i))])
        t._id = exp.claim_trial_id(cid, i)
        ts.append(t)
    exp.register_trials(ts)
    assert exp.set_trial_status(ts[1], "broken")  # gives its token back: used 3 -> 2
    assert exp.reconcile_budget() == 0
    old = utcnow() - datetime.timedelta(seconds=exp.CLAIM_INSERT_GRACE_S + 5)
    _edit_claim(storage, exp, cid, t=old)
    assert exp.reconcile_budget() == 1  # only the never-inserted third trial
    b = storage.read("experiments", {"_id": exp.id})[0]["budget"]
    assert b["used"] == 1 and b["claims"] == {}


def test_settle_counts_the_store_when_insert_failed(storage, monkeypatch):
    """An insert that raised part-way: settle counts the claim's trials instead of trusting
    the producer's local count (0), so the written trials keep their tokens."""
    exp = _ready(storage, max_trials=4, pool_size=3)
    prod = Producer(exp)
    real = Experiment.register_trials

    def partial(self, trials):
        real(self, trials[:2])
        raise RuntimeError("connection lost")
    monkeypatch.setattr(Experiment, "register_trials", partial)
    with pytest.raises(RuntimeError):
        prod.produce()
    b = storage.read("experiments", {"_id": exp.id})[0]["budget"]
    assert b["used"] == 2 and b["claims"] == {}
    assert exp.count_trials("new") == 2
