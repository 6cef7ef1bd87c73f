"""Document-store conformance (memory, SQLite, MongoDB-if-reachable) and a REAL
multi-process reservation race (reference tests simulated races with patched
random.sample; SURVEY.md §4 'Improve' item 2)."""
import datetime
import multiprocessing as mp
import os

import pytest

from orion_amd.store import Database, DuplicateKeyError, LocalDB, MemoryDB


def _mongo_reachable():
    try:
        import pymongo
        c = pymongo.MongoClient(serverSelectionTimeoutMS=200)
        c.admin.command("ping")
        return True
    except Exception:
        return False


BACKENDS = ["memory", "sqlite"] + (["mongodb"] if _mongo_reachable() else [])


@pytest.fixture(params=BACKENDS)
def db(request, tmp_path):
    if request.param == "sqlite":
        return Database("sqlite", host=str(tmp_path / "t.sqlite"))
    if request.param == "mongodb":
        d = Database("mongodb", name="orion_amd_test")
        for c in ("experiments", "trials", "things"):
            d.drop(c)
        return d
    return Database("memory")


def test_insert_read_count_remove(db):
    docs = [{"a": 1, "b": {"c": 2}}, {"a": 2, "b": {"c": 3}}, {"a": 3, "tags": ["x", "y"]}]
    assert db.write("things", docs) == 3
    assert all("_id" in d for d in docs)
    assert db.count("things") == 3
    assert [d["a"] for d in db.read("things", {"b.c": 3})] == [2]
    assert sorted(d["a"] for d in db.read("things", {"a": {"$in": [1, 3]}})) == [1, 3]
    assert sorted(d["a"] for d in db.read("things", {"a": {"$gte": 2}})) == [2, 3]
    assert [d["a"] for d in db.read("things", {"tags": "x"})] == [3]
    assert db.count("things", {"a": {"$ne": 1}}) == 2
    assert db.remove("things", {"a": 1}) == 1
    assert db.count("things") == 2


def test_projection(db):
    db.write("things", {"a": 1, "b": 2, "c": {"d": 3}})
    (d,) = db.read("things", {}, selection={"a": 1, "c.d": 1})
    assert d["a"] == 1 and "b" not in d and d["c"] == {"d": 3} and "_id" in d


def test_update_and_upsert(db):
    db.write("things", {"a": 1, "s": "new"})
    assert db.write("things", {"s": "old"}, query={"a": 1}) == 1
    assert db.read("things", {"a": 1})[0]["s"] == "old"
    db.write("things", {"s": "fresh"}, query={"a": 42})
    assert db.read("things", {"a": 42})[0]["s"] == "fresh"


def test_datetime_roundtrip(db):
    t = datetime.datetime(2020, 1, 2, 3, 4, 5, 6000)
    db.write("things", {"t": t})
    assert db.read("things", {})[0]["t"] == t
    assert db.count("things", {"t": {"$gte": t}}) == 1
    assert db.count("things", {"t": {"$gt": t}}) == 0


def test_read_and_write_is_cas(db):
    db.write("things", {"k": 1, "status": "new"})
    got = db.read_and_write("things", {"k": 1, "status": "new"}, {"status": "reserved"})
    assert got is not None and got["status"] == "reserved"
    assert db.read_and_write("things", {"k": 1, "status": "new"}, {"status": "reserved"}) is None


def test_unique_index(db):
    db.ensure_index("experiments", [("name", db.ASCENDING), ("metadata.user", db.ASCENDING)], unique=True)
    db.write("experiments", {"name": "a", "metadata": {"user": "u"}})
    db.write("experiments", {"name": "a", "metadata": {"user": "v"}})
    with pytest.raises(DuplicateKeyError):
        db.write("experiments", {"name": "a", "metadata": {"user": "u"}})


def _racer(path, n_trials, out_q):
    db = LocalDB(host=path)
    got = []
    while True:
        cands = db.read("trials", {"status": "new"})
        if not cands:
            break
        for c in cands:
            if db.read_and_write("trials", {"_id": c["_id"], "status": "new"},
                                 {"status": "reserved", "by": os.getpid()}) is not None:
                got.append(c["_id"])
                break
    out_q.put(got)


def test_multiprocess_reservation_race(tmp_path):
    """N real processes reserve from one SQLite store: every trial exactly once."""
    path = str(tmp_path / "race.sqlite")
    db = LocalDB(host=path)
    n = 120
    db.write("trials", [{"i": i, "status": "new"} for i in range(n)])
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_racer, args=(path, n, q)) for _ in range(4)]
    for p in procs:
        p.start()
    results = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    allgot = [x for r in results for x in r]
    assert len(allgot) == n and len(set(allgot)) == n
    assert db.count("trials", {"status": "reserved"}) == n


def test_factory_names():
    assert isinstance(Database("memory"), MemoryDB)
    with pytest.raises(NotImplementedError):
        Database("nosuchdb")


def _reservation_times(path, n_pending, n_reserve=30):
    import time as _t
    from orion_amd.core.experiment import Experiment
    from orion_amd.store import Database
    db = Database("sqlite", host=str(path))
    exp = Experiment("big", db, user="u")
    cfg = exp.configuration
    cfg.update(algorithms={"random": {}}, pool_size=1, max_trials=10**5)
    cfg["metadata"]["user_script"] = "/bin/true"
    cfg["metadata"]["user_args"] = ["-x~uniform(0, 1)"]
    exp.configure(cfg)
    docs = [dict(experiment=exp.id, status="new", params=[dict(name="/x", type="real", value=i / 1e4)])
            for i in range(n_pending)]
    db.write("trials", docs)
    assert db.count("trials", {"experiment": exp.id, "status": "new"}) == n_pending
    times, seen = [], set()
    for _ in range(n_reserve):
        t0 = _t.perf_counter()
        tr = exp.reserve_trial(worker="w")
        times.append(_t.perf_counter() - t0)
        assert tr is not None and tr.id not in seen
        seen.add(tr.id)
    t0 = _t.perf_counter()
    for _ in range(20):
        assert db.read_and_write("trials", {"_id": tr.id, "status": "reserved"}, {"heartbeat": 1})
    cas = (_t.perf_counter() - t0) / 20
    return times, cas


def test_sqlite_reservation_is_constant_time(tmp_path):
    """10^4 pending trials: a reservation is a COUNT + one 64-document page + a one-row CAS
    (indexed ``_id``/status), not a parse of every pending trial.
    Judged against the same reservation with 100 pending trials on the same machine, so a
    loaded test host (parallel workers) does not turn a scaling check into a clock check."""
    import statistics
    small, small_cas = _reservation_times(tmp_path / "small.sqlite", 100)
    big, big_cas = _reservation_times(tmp_path / "big.sqlite", 10**4)
    # a parse of every pending trial would make the 10^4 case ~100x the 100 case -- in every
    # sample, so the fastest samples are compared (the median drifts with disk/CPU contention
    # from parallel test workers)
    assert min(big) < 3 * min(small) + 0.002, (big, small)
    assert statistics.median(big) < 20 * statistics.median(small) + 0.01, (big, small)
    assert big_cas < 3 * small_cas + 0.002, (big_cas, small_cas)
