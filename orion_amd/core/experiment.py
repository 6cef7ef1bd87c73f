"""Experiment manager (component C6).

Parity with ``src/orion/core/worker/experiment.py``: one document in the
``experiments`` collection, primary key ``(name, metadata.user)`` enforced by a
unique index; ``configure`` creates or resumes it (config merge; a differing
configuration of an existing experiment is a "fork" -- rejected, as in the
reference); trials are registered as ``new``, reserved with an atomic
compare-and-swap on their status, completed with their results; completed
trials are fetched incrementally for the algorithm; ``is_done`` marks the
experiment ``done`` when ``max_trials`` completed trials exist or the
algorithm declares itself done; ``stats`` summarises it.

Deliberate fixes of reference quirks:

* explicit storage handle, and the experiment owns its immutable
  :class:`~orion_amd.space.dsl.ScriptTemplate` instead of process singletons
  (item 1); configuration planning is a pure function (:func:`plan_configuration`);
* ``is_done`` is a side-effect-free query; :meth:`Experiment.finish_if_done` records
  the ``done`` status (item 3);
* ``stats`` works with zero completed trials (item 2);
* bounded reservation retry loop instead of unbounded recursion (item 6);
* incremental fetch keeps a set of already-observed trial ids and re-reads a
  clock-skew margin, so a worker with a fast clock cannot drop another
  worker's results (item 5);
* liveness: reserved trials carry a ``heartbeat``; stale reservations of dead
  workers are returned to the pool as ``interrupted`` (SURVEY.md §5 failure
  detection) -- the reference leaves them reserved forever.
"""
from __future__ import annotations

import copy
import datetime
import errno
import getpass
import logging
import os
import random
import socket
import uuid
from dataclasses import dataclass

from ..space.dsl import ScriptTemplate
from ..store import DuplicateKeyError
from .format_trials import trial_to_tuple
from .primary_algo import PrimaryAlgo
from .trial import Trial

log = logging.getLogger(__name__)

FETCH_SKEW_MARGIN = datetime.timedelta(minutes=10)


def utcnow():
    """Naive UTC truncated to milliseconds (what MongoDB stores), so every backend
    round-trips timestamps exactly."""
    n = datetime.datetime.utcnow()
    return n.replace(microsecond=n.microsecond // 1000 * 1000)


def _proc_start_time(pid):
    """Start time of ``pid`` in clock ticks since boot (``/proc/<pid>/stat`` field 22), or
    None where /proc is unavailable."""
    try:
        with open(f"/proc/{pid}/stat", "rb") as f:
            stat = f.read().decode(errors="replace")
        return int(stat[stat.rindex(")") + 2:].split()[19])
    except (OSError, ValueError, IndexError):
        return None


_IDENTITY = {}


def process_identity():
    """Who owns a budget claim: host name, boot id, pid-namespace inode, pid and the pid's
    start time.  Two processes are comparable by pid only when host, boot and pidns agree."""
    pid = os.getpid()
    if pid not in _IDENTITY:
        try:
            with open("/proc/sys/kernel/random/boot_id") as f:
                boot = f.read().strip()
        except OSError:
            boot = None
        try:
            pidns = os.stat("/proc/self/ns/pid").st_ino
        except OSError:
            pidns = None
        _IDENTITY.clear()
        _IDENTITY[pid] = {"host": socket.gethostname(), "boot": boot, "pidns": pidns, "pid": pid,
                          "start": _proc_start_time(pid)}
    return dict(_IDENTITY[pid])


class Experiment:
    __slots__ = ("name", "refers", "metadata", "pool_size", "max_trials", "status", "algorithms",
                 "_db", "_init_done", "_id", "_last_fetched", "_seen", "template", "_user")
    non_forking_attrs = ("status", "pool_size", "max_trials")
    _config_attrs = ("name", "refers", "metadata", "pool_size", "max_trials", "status", "algorithms")
    MAX_RESERVE_ATTEMPTS = 64

    def __init__(self, name, storage, user=None):
        self._init_done = False
        self._db = storage
        self._setup_db()
        self._id = None
        self.name = name
        self.refers = None
        self._user = user or getpass.getuser()
        self.metadata = {"user": self._user, "datetime": utcnow()}
        self.pool_size = None
        self.max_trials = None
        self.status = None
        self.algorithms = None
        self.template = None
        self._seen = set()
        docs = self._db.read("experiments", {"name": name, "metadata.user": self._user})
        if docs:
            if len(docs) > 1:
                log.warning("Many (%s) experiments for (%s, %s); using the most recent one.",
                            len(docs), name, self._user)
            doc = sorted(docs, key=lambda x: x["metadata"]["datetime"], reverse=True)[0]
            for attr in self._config_attrs:
                setattr(self, attr, doc.get(attr))
            self._id = doc["_id"]
        self._last_fetched = self.metadata["datetime"]

    @property
    def storage(self):
        return self._db

    @property
    def id(self):
        return self._id

    def _setup_db(self):
        db = self._db
        db.ensure_index("experiments", [("name", db.ASCENDING), ("metadata.user", db.ASCENDING)],
                        unique=True)
        db.ensure_index("experiments", "status")
        for f in ("experiment", "status", "results", "start_time"):
            db.ensure_index("trials", f)
        db.ensure_index("trials", [("end_time", db.DESCENDING)])

    # ------------------------------------------------------------------ trials
    RESERVE_WINDOW = 64

    def _candidates(self, query, uniform):
        """Reservable trials to choose from.  When every candidate scores the same, a
        random window of ``RESERVE_WINDOW`` of them is enough (one COUNT plus one paged read,
        independent of how many trials are pending); otherwise all of them."""
        if not uniform:
            return Trial.build(self._db.read("trials", query))
        n = self._db.count("trials", query)
        if n == 0:
            return []
        skip = random.randrange(n - self.RESERVE_WINDOW + 1) if n > self.RESERVE_WINDOW else 0
        return Trial.build(self._db.read("trials", query, skip=skip, limit=self.RESERVE_WINDOW))

    def reserve_trial(self, score_handle=None, worker=None):
        """Atomically move one reservable trial to ``reserved``; None if there is none.
        Among the candidates the best-scored ones win (``score_handle``), ties at random."""
        if score_handle is not None and not callable(score_handle):
            raise ValueError("Argument `score_handle` must be callable with a `Trial`.")
        uniform = score_handle is None or bool(
            getattr(getattr(score_handle, "__self__", None), "scores_uniform", False))
        for _ in range(self.MAX_RESERVE_ATTEMPTS):
            query = dict(experiment=self._id, status={"$in": list(Trial.reservable_stati)})
            candidates = self._candidates(query, uniform)
            if not candidates:
                return None
            if score_handle is not None and not uniform and self.space:
                scores = [score_handle(trial_to_tuple(t, self.space)) for t in candidates]
                best = max(scores)
                candidates = [t for s, t in zip(scores, candidates) if s == best]
            elif score_handle is not None and not uniform:
                log.warning("`score_handle` given but the parameter space is not defined yet.")
            sel = random.sample(candidates, 1)[0]
            now = utcnow()
            update = dict(status="reserved", heartbeat=now)
            if worker is not None:
                update["worker"] = worker
            if sel.status == "new":
                update["start_time"] = now
            doc = self._db.read_and_write("trials", {"_id": sel.id, "status": sel.status}, update)
            if doc is not None:
                return Trial(**doc)
            log.debug("lost the reservation race for %s; retrying", sel.id)
        return None

    # ------------------------------------------------------------------ trial budget
    # Trials that count toward ``max_trials``: every status but ``broken``.  The experiment
    # document carries ``budget = {"used": n, "v": version, "t": time, "claims": {...}}``:
    # ``used`` counts the counting trials registered or about to be; a producer takes tokens
    # with a compare-and-swap on the version BEFORE it inserts, as a CLAIM recorded under a
    # fresh claim id with its owner (host, pid, worker) and stage; it inserts its trials under
    # ids derived from the claim id, then settles the claim (gives back what it did not
    # insert, removes the record).  So concurrent producers can never register more than
    # ``max_trials`` counting trials (the reference counted, then inserted: W workers
    # overshot by up to W x pool_size, src/orion/core/worker/producer.py:35-45), a claim of a
    # producer that died is recovered exactly (its inserted trials are found by id), and a
    # settle after such a recovery is a no-op (no double release).
    LIVE_STATI = ("new", "reserved", "suspended", "interrupted", "completed")
    BUDGET_ATTEMPTS = 256
    # a claim whose owner cannot be probed (another host) is presumed dead after this long by
    # the writer's clock; owners on this host are probed by pid and recovered only when dead
    CLAIM_FOREIGN_GRACE_S = 3600.0
    # an inserting claim (its producer passed confirm_claim) is left alone this long after the
    # confirmation even when its owner looks dead: the insert of pool_size documents takes ms
    CLAIM_INSERT_GRACE_S = 120.0

    def _budgeted(self):
        return self.max_trials not in (None, float("inf")) and self._id is not None

    def _budget_doc(self):
        docs = self._db.read("experiments", {"_id": self._id}, selection={"budget": 1})
        return docs[0].get("budget") if docs else None

    def _budget_cas(self, old, used, claims=None):
        """Replace the budget document if it is still ``old`` (compared by version; documents
        from before the version field by ``used`` and ``t``)."""
        q = {"_id": self._id}
        if old is None:
            q["budget"] = {"$exists": False}
            v = 1
        elif "v" in old:
            q["budget.v"] = old["v"]
            v = int(old["v"]) + 1
        else:
            q["budget.used"], q["budget.t"] = old["used"], old["t"]
            v = 1
        if claims is None:
            claims = dict((old or {}).get("claims") or {})
        new = {"used": int(used), "v": v, "t": utcnow(), "claims": claims}
        return self._db.read_and_write("experiments", q, {"budget": new}) is not None

    def _seeded_budget(self):
        b = self._budget_doc()
        if b is None:  # first use (or an experiment from before the counter): seed it
            self._budget_cas(None, self.count_trials(self.LIVE_STATI), {})
            b = self._budget_doc()
        return b

    @staticmethod
    def claim_trial_id(cid, i):
        """The id of the ``i``-th trial inserted under budget claim ``cid``."""
        return f"{cid}.{i}"

    def take_budget(self, n, owner=None):
        """Take up to ``n`` registration tokens as a recorded claim: returns ``(k, cid)``, ``k``
        tokens (0 when the budget is spent) under claim id ``cid`` (None for an unbudgeted
        experiment, which always gets ``n``)."""
        if n <= 0:
            return 0, None
        if not self._budgeted():
            return n, None
        for _ in range(self.BUDGET_ATTEMPTS):
            b = self._seeded_budget()
            if b is None:
                continue
            k = min(n, int(self.max_trials) - int(b["used"]))
            if k <= 0:
                return 0, None
            cid = uuid.uuid4().hex
            claims = dict(b.get("claims") or {})
            claims[cid] = dict(process_identity(), n=int(k), owner=owner, t=utcnow(), stage="suggest")
            if self._budget_cas(b, int(b["used"]) + k, claims):
                return k, cid
        log.warning("trial budget: no token after %d attempts (heavy contention)", self.BUDGET_ATTEMPTS)
        return 0, None

    def _update_claim(self, cid, fn):
        """Apply ``fn(budget, claim) -> (used, claim or None) | None`` to claim ``cid`` under
        the compare-and-swap; returns False when the claim no longer exists."""
        for _ in range(self.BUDGET_ATTEMPTS):
            b = self._budget_doc()
            claims = dict((b or {}).get("claims") or {})
            if cid not in claims:
                return False
            r = fn(b, claims[cid])
            if r is None:
                return True
            used, c = r
            if c is None:
                claims.pop(cid)
            else:
                claims[cid] = c
            if self._budget_cas(b, used, claims):
                return True
        return False

    def confirm_claim(self, cid):
        """Mark claim ``cid`` as inserting; False when it was recovered meanwhile (its owner was
        presumed dead), in which case the caller must not insert its trials."""
        if cid is None:
            return True
        # ``t`` restarts here: an insert-stage claim is recovered only INSERT_GRACE_S after it
        return self._update_claim(cid, lambda b, c: (int(b["used"]), dict(c, stage="insert", t=utcnow())))

    def _claim_trials_found(self, cid, n):
        """How many of claim ``cid``'s ``n`` trials exist, in ANY status: a broken one already
        gave its token back through :meth:`set_trial_status`, so it must not be returned twice."""
        ids = [self.claim_trial_id(cid, i) for i in range(int(n))]
        return self._db.count("trials", {"experiment": self._id, "_id": {"$in": ids}})

    def settle_budget(self, cid, inserted=None):
        """Close claim ``cid`` after ``inserted`` of its trials were registered: the rest of its
        tokens go back.  ``inserted=None`` (the insert raised part-way) counts the claim's trials
        in the store instead of trusting the caller.  A no-op when the claim was already
        recovered."""
        if cid is None:
            return

        def fn(b, c):
            got = self._claim_trials_found(cid, c["n"]) if inserted is None else int(inserted)
            return max(0, int(b["used"]) - max(0, int(c["n"]) - got)), None
        self._update_claim(cid, fn)

    def claim_budget(self, n):
        """Anonymous tokens (no claim record): up to ``n``; see :meth:`take_budget`."""
        k, cid = self.take_budget(n)
        if cid is not None:
            self._update_claim(cid, lambda b, c: (int(b["used"]), None))
        return k

    def release_budget(self, k):
        """Give back ``k`` anonymous tokens (a broken trial, an unclaimed shortfall)."""
        if k <= 0 or not self._budgeted():
            return
        for _ in range(self.BUDGET_ATTEMPTS):
            b = self._budget_doc()
            if b is None:
                return
            if self._budget_cas(b, max(0, int(b["used"]) - k)):
                return

    @classmethod
    def _claim_owner_dead(cls, c, now, grace_s):
        """Whether claim ``c``'s producer is gone.  The owner is probed only when it provably
        shares this process's pid space: same host name, boot id AND pid-namespace inode
        (containers with host networking share a host name but not pids).  A live pid whose
        start time differs from the recorded one is a reused pid, i.e. a dead owner.  Any
        other owner is presumed dead ``grace_s`` after the claim's last stamp.  A claim already
        inserting (stage ``insert``) is never recovered within :attr:`CLAIM_INSERT_GRACE_S` of
        its confirmation, whatever the probe says."""
        t = c.get("t")
        age = None if t is None else (now - t).total_seconds()
        if c.get("stage") == "insert" and (age is None or age <= cls.CLAIM_INSERT_GRACE_S):
            return False
        me = process_identity()
        if (c.get("pid") and all(c.get(k) is not None and c.get(k) == me[k]
                                 for k in ("host", "boot", "pidns"))):
            pid = int(c["pid"])
            try:
                os.kill(pid, 0)
            except OSError as e:
                return e.errno == errno.ESRCH
            start = c.get("start")
            return start is not None and _proc_start_time(pid) not in (None, start)
        return age is not None and age > grace_s

    def reconcile_budget(self, grace_s=None):
        """Recover the tokens of claims whose producer died between taking them and settling:
        an owner on this host is dead when its pid is gone; an owner on another host is
        presumed dead after ``grace_s`` (default :attr:`CLAIM_FOREIGN_GRACE_S`).  A recovered
        claim gives back exactly the tokens its trials (found by their claim-derived ids) do
        not hold.  Returns the number of tokens recovered."""
        if not self._budgeted():
            return 0
        grace_s = self.CLAIM_FOREIGN_GRACE_S if grace_s is None else grace_s
        b = self._budget_doc()
        now = utcnow()
        dead = [cid for cid, c in ((b or {}).get("claims") or {}).items()
                if self._claim_owner_dead(c, now, grace_s)]
        got = 0
        for cid in dead:
            def fn(b, c, cid=cid):
                back = max(0, int(c["n"]) - self._claim_trials_found(cid, c["n"]))
                fn.back = back
                return max(0, int(b["used"]) - back), None
            fn.back = 0
            if self._update_claim(cid, fn) and fn.back:
                log.warning("trial budget: recovered %d token(s) of claim %s (producer dead)", fn.back, cid)
                got += fn.back
        return got

    def register_trials(self, trials):
        stamp = utcnow()
        for t in trials:
            t.experiment = self._id
            t.status = "new"
            t.submit_time = stamp
        docs = [t.to_dict() for t in trials]
        if docs:
            self._db.write("trials", docs)
            for t, d in zip(trials, docs):
                t._id = d["_id"]

    def push_completed_trial(self, trial, only_if_reserved=False):
        """Store ``trial`` as completed.  With ``only_if_reserved`` the write is a
        compare-and-swap on ``status='reserved'`` (and on the reserving worker when the
        trial carries one): a trial that was re-queued meanwhile is not overwritten.
        Returns whether the trial was written."""
        trial.end_time = utcnow()
        trial.status = "completed"
        doc = trial.to_dict()
        if not only_if_reserved:
            self._db.write("trials", doc, query={"_id": trial.id})
            return True
        q = self._owned(trial)
        doc.pop("_id", None)
        return self._db.read_and_write("trials", q, doc) is not None

    @staticmethod
    def _owned(trial, status="reserved"):
        """CAS query for a trial this worker holds: its id, the expected status and -- when
        the trial carries the reserving worker's id -- that worker.  A trial that a reaper
        re-queued and another worker reserved is then out of reach of the first worker's
        heartbeats, leases and status writes."""
        q = {"_id": trial.id, "status": status}
        if getattr(trial, "worker", None) is not None:
            q["worker"] = trial.worker
        return q

    def set_trial_status(self, trial, status, only_if=None):
        """Move ``trial`` to ``status``; with ``only_if`` it is a CAS on the current status
        (and on the reserving worker, see :meth:`_owned`)."""
        q = {"_id": trial.id} if only_if is None else self._owned(trial, only_if)
        if status == "broken":  # only a trial that still counted gives a token back
            q.setdefault("status", {"$in": list(self.LIVE_STATI)})
        trial.status = status
        upd = {"status": status}
        if status in ("broken", "completed"):
            upd["end_time"] = trial.end_time = utcnow()
        ok = self._db.read_and_write("trials", q, upd) is not None
        if ok and status == "broken":
            self.release_budget(1)
        return ok

    def record_lease(self, trial, gpu_ids):
        """The trial got its GPUs and starts executing: record the device ids and move
        ``start_time`` from the reservation to now (a reserved trial may wait for a GPU
        lease first).  False if the trial is no longer ours."""
        now = utcnow()
        ok = self._db.read_and_write("trials", self._owned(trial),
                                     {"gpus": list(gpu_ids), "start_time": now,
                                      "heartbeat": now}) is not None
        if ok:
            trial.gpus, trial.start_time = list(gpu_ids), now
        return ok

    def update_heartbeat(self, trial):
        return self._db.read_and_write("trials", self._owned(trial),
                                       {"heartbeat": utcnow()}) is not None

    def fix_lost_trials(self, timeout_s):
        """Reserved trials whose heartbeat is older than ``timeout_s`` -> ``interrupted``."""
        limit = utcnow() - datetime.timedelta(seconds=timeout_s)
        stale = self._db.read("trials", {"experiment": self._id, "status": "reserved",
                                         "heartbeat": {"$lt": limit}})
        n = 0
        for d in stale:
            if self._db.read_and_write("trials", {"_id": d["_id"], "status": "reserved",
                                                  "heartbeat": d.get("heartbeat")},
                                       {"status": "interrupted"}) is not None:
                n += 1
        if n:
            log.warning("re-queued %d trial(s) whose worker stopped heart-beating", n)
        return n

    def fetch_completed_trials(self):
        """Completed trials this object has not returned before (incremental)."""
        query = dict(experiment=self._id, status="completed",
                     end_time={"$gte": self._last_fetched - FETCH_SKEW_MARGIN})
        now = utcnow()
        trials = [t for t in Trial.build(self._db.read("trials", query)) if t.id not in self._seen]
        self._seen.update(t.id for t in trials)
        self._last_fetched = now
        trials.sort(key=lambda t: t.end_time)
        return trials

    def fetch_trials(self, query=None):
        q = dict(query or {})
        q["experiment"] = self._id
        return Trial.build(self._db.read("trials", q))

    def count_trials(self, status=None):
        q = {"experiment": self._id}
        if status is not None:
            q["status"] = status if isinstance(status, str) else {"$in": list(status)}
        return self._db.count("trials", q)

    # ------------------------------------------------------------------ state
    def _finished(self):
        n_completed = self.count_trials("completed")
        return n_completed >= self.max_trials or bool(self._init_done and self.algorithms.is_done)

    @property
    def is_done(self):
        """True when ``max_trials`` trials completed or the algorithm declares itself done.
        Pure query: recording ``status='done'`` is :meth:`finish_if_done`'s job (the
        reference's property wrote to the database)."""
        return self._finished()

    def finish_if_done(self):
        """:attr:`is_done`, and if so persist ``status='done'`` once."""
        if not self._finished():
            return False
        if self.status != "done":
            self._db.write("experiments", {"status": "done"}, {"_id": self._id})
            self.status = "done"
        return True

    @property
    def space(self):
        return self.algorithms.space if self._init_done else None

    @property
    def space_builder(self):
        """The experiment's :class:`ScriptTemplate` (kept under the old attribute name)."""
        return self.template

    @property
    def configuration(self):
        cfg = {}
        for attr in self._config_attrs:
            val = getattr(self, attr)
            if self._init_done and attr == "algorithms":
                val = val.configuration
            cfg[attr] = val
        return copy.deepcopy(cfg)

    def configure(self, config):
        """Create (unknown ``(name, user)``) or resume (stored, same identity) the experiment.

        The work is split into a pure planning step, :func:`plan_configuration`, which
        overlays ``config`` on the stored document, normalises it by instantiating the
        template and the algorithm, and rejects a changed identity (a "fork"); and the
        adoption + single database write here."""
        if self._init_done:
            raise RuntimeError("Configuration is done; cannot reset an Experiment.")
        creating = self.status is None
        if creating:
            md = config.get("metadata") or {}
            if (config.get("name"), md.get("user"), md.get("datetime")) != \
                    (self.name, self.metadata["user"], self.metadata["datetime"]):
                raise ValueError("Configuration given is inconsistent with this Experiment.")
        plan = plan_configuration(None if creating else self.configuration, config)
        for attr in self._config_attrs:
            setattr(self, attr, plan.config.get(attr))
        self.template = plan.template
        if plan.algorithms is not None:
            self.algorithms = plan.algorithms
        self._init_done = plan.algorithms is not None
        self.status = "pending"
        if creating:
            doc = plan.config
            self._db.write("experiments", doc)  # DuplicateKeyError on a creation race
            self._id = doc["_id"]
        else:
            self._db.write("experiments", {k: v for k, v in plan.config.items() if k != "name"},
                           {"_id": self._id})

    # ------------------------------------------------------------------ stats
    @property
    def stats(self):
        docs = self._db.read("trials", dict(experiment=self._id, status="completed"),
                             selection={"_id": 1, "end_time": 1, "results": 1})
        stats = dict(trials_completed=len(docs), best_trials_id=None, best_evaluation=None,
                     start_time=self.metadata["datetime"], finish_time=self.metadata["datetime"])
        for d in docs:
            t = Trial(**d)
            if t.end_time and t.end_time > stats["finish_time"]:
                stats["finish_time"] = t.end_time
            obj = t.objective
            if obj is None or obj.value is None:
                continue
            if stats["best_evaluation"] is None or obj.value < stats["best_evaluation"]:
                stats["best_evaluation"] = obj.value
                stats["best_trials_id"] = t.id
        stats["duration"] = stats["finish_time"] - stats["start_time"]
        return stats


def create_experiment(name, storage, config, user=None, _retry=True):
    """Bootstrap: load/merge/configure, retrying once on a concurrent-creation race
    (reference ``cli.py:70-120``)."""
    from .config import merge_orion_config, to_plain
    exp = Experiment(name, storage, user=user)
    cfg = to_plain(merge_orion_config(config.get("expconfig", {}), exp.configuration,
                                      config.get("cmdconfig", {}), config.get("cmdargs", {})))
    for k in ("database", "resources", "status", "execution"):
        cfg.pop(k, None)
    cfg["name"] = name
    if not cfg.get("algorithms"):
        cfg["algorithms"] = "random"  # default optimizer when none is configured
    md = cfg.setdefault("metadata", {})
    md.setdefault("user", exp.metadata["user"])
    md.setdefault("datetime", exp.metadata["datetime"])
    if exp.status is None:
        md["user"], md["datetime"] = exp.metadata["user"], exp.metadata["datetime"]
    try:
        exp.configure(cfg)
    except DuplicateKeyError:
        if not _retry:
            raise
        return create_experiment(name, storage, config, user=user, _retry=False)
    return exp


# ---------------------------------------------------------------------------- configuration
CONFIG_ATTRS = Experiment._config_attrs
# sections that may change when an experiment is resumed
MUTABLE_SECTIONS = Experiment.non_forking_attrs
# metadata keys that do not identify an experiment
VOLATILE_METADATA = ("datetime", "orion_version")


@dataclass
class ConfigPlan:
    config: dict            # the document to store (algorithms normalised)
    template: object        # ScriptTemplate or None (no user_args yet)
    algorithms: object      # PrimaryAlgo or None


def _identity(cfg: dict) -> dict:
    """The sections that define WHAT an experiment optimises."""
    ident = {}
    for k in CONFIG_ATTRS:
        if k in MUTABLE_SECTIONS:
            continue
        v = cfg.get(k)
        if k == "metadata":
            v = {mk: mv for mk, mv in (v or {}).items() if mk not in VOLATILE_METADATA}
        ident[k] = v
    return ident


def plan_configuration(stored: dict | None, requested: dict) -> ConfigPlan:
    """Overlay ``requested`` on ``stored`` (None: a new experiment), instantiate the
    script template and the algorithm to normalise the algorithm section, and refuse a
    resume whose identity differs from the stored one.  No side effects on any store."""
    for k in requested:
        if k not in CONFIG_ATTRS:
            log.warning("Found section '%s' in configuration. Experiments do not support "
                        "this option. Ignoring.", k)
    cfg = {k: copy.deepcopy(requested[k] if k in requested else (stored or {}).get(k))
           for k in CONFIG_ATTRS}
    cfg["status"] = "pending"
    template = algorithms = None
    user_args = (cfg.get("metadata") or {}).get("user_args")
    if user_args is not None:
        template = ScriptTemplate.parse(user_args)
        if not template.space:
            raise ValueError("Parameter space is empty. There is nothing to optimize.")
        algorithms = PrimaryAlgo(template.space, cfg.get("algorithms"))
        cfg["algorithms"] = algorithms.configuration
    if stored is not None:
        old, new = _identity(stored), _identity(cfg)
        changed = [k for k in old if old[k] != new[k]]
        if changed:
            for k in changed:
                log.warning("Config given is different from config found in db at section: %s\n"
                            "  stored:    %s\n  requested: %s", k, old[k], new[k])
            raise NotImplementedError(
                f"Experiment '{cfg.get('name')}' exists with a different configuration "
                f"({', '.join(changed)}); forking is not supported -- use a new experiment "
                "name (-n).")
    return ConfigPlan(cfg, template, algorithms)
