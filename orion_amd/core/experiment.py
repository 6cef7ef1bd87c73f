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

* explicit storage handle and the experiment owns its :class:`SpaceBuilder`
  (templates) instead of process singletons (items 1);
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
import getpass
import logging
import random

from ..space.dsl import SpaceBuilder
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


class Experiment:
    __slots__ = ("name", "refers", "metadata", "pool_size", "max_trials", "status", "algorithms",
                 "_db", "_init_done", "_id", "_last_fetched", "_seen", "space_builder", "_user")
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
        self.space_builder = None
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
    def reserve_trial(self, score_handle=None, worker=None):
        """Atomically move one reservable trial to ``reserved``; None if there is none."""
        if score_handle is not None and not callable(score_handle):
            raise ValueError("Argument `score_handle` must be callable with a `Trial`.")
        for _ in range(self.MAX_RESERVE_ATTEMPTS):
            query = dict(experiment=self._id, status={"$in": list(Trial.reservable_stati)})
            candidates = Trial.build(self._db.read("trials", query))
            if not candidates:
                return None
            if score_handle is not None and self.space:
                scores = [score_handle(trial_to_tuple(t, self.space)) for t in candidates]
                best = max(scores)
                candidates = [t for s, t in zip(scores, candidates) if s == best]
            elif score_handle is not None:
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

    def push_completed_trial(self, trial):
        trial.end_time = utcnow()
        trial.status = "completed"
        self._db.write("trials", trial.to_dict(), query={"_id": trial.id})

    def set_trial_status(self, trial, status, only_if=None):
        """Move ``trial`` to ``status``; with ``only_if`` it is a CAS on the current status."""
        trial.status = status
        q = {"_id": trial.id}
        if only_if is not None:
            q["status"] = only_if
        upd = {"status": status}
        if status in ("broken", "completed"):
            upd["end_time"] = trial.end_time = utcnow()
        return self._db.read_and_write("trials", q, upd) is not None

    def update_heartbeat(self, trial):
        return self._db.read_and_write("trials", {"_id": trial.id, "status": "reserved"},
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
    @property
    def is_done(self):
        n_completed = self.count_trials("completed")
        if n_completed >= self.max_trials or (self._init_done and self.algorithms.is_done):
            self._db.write("experiments", {"status": "done"}, {"_id": self._id})
            self.status = "done"
            return True
        return False

    @property
    def space(self):
        return self.algorithms.space if self._init_done else None

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
        """Create (new name) or resume (existing, same configuration) the experiment."""
        if self._init_done:
            raise RuntimeError("Configuration is done; cannot reset an Experiment.")
        shadow = Experiment(self.name, self._db, user=self._user)
        shadow._instantiate_config(self.configuration)
        shadow._instantiate_config(config)
        shadow._init_done = True
        shadow.status = "pending"
        if self.status is None:
            if config["name"] != self.name or \
                    config["metadata"]["user"] != self.metadata["user"] or \
                    config["metadata"]["datetime"] != self.metadata["datetime"]:
                raise ValueError("Configuration given is inconsistent with this Experiment.")
            is_new = True
        else:
            is_new = self._is_different_from(shadow.configuration)
            if is_new:
                self._fork_config(config)
        final = shadow.configuration
        self._instantiate_config(final)
        self._init_done = True
        self.status = "pending"
        if is_new:
            self._db.write("experiments", final)  # DuplicateKeyError on a creation race
            self._id = final["_id"]
        else:
            final.pop("name")
            self._db.write("experiments", final, {"_id": self._id})

    def _instantiate_config(self, config):
        for section, value in config.items():
            if section == "status":
                continue
            if section not in self._config_attrs:
                log.warning("Found section '%s' in configuration. Experiments do not support "
                            "this option. Ignoring.", section)
                continue
            setattr(self, section, value)
        try:
            builder = SpaceBuilder()
            space = builder.build_from(config["metadata"]["user_args"])
            if not space:
                raise ValueError("Parameter space is empty. There is nothing to optimize.")
            self.space_builder = builder
            self.algorithms = PrimaryAlgo(space, self.algorithms)
        except KeyError:
            pass

    def _fork_config(self, config):
        raise NotImplementedError(
            f"Experiment '{self.name}' exists with a different configuration; forking is not "
            "supported -- use a new experiment name (-n).")

    def _is_different_from(self, config):
        for section, value in config.items():
            if section in self.non_forking_attrs or section not in self._config_attrs:
                continue
            item = getattr(self, section)
            if section == "metadata":
                item = {k: v for k, v in (item or {}).items() if k not in ("datetime", "orion_version")}
                value = {k: v for k, v in (value or {}).items() if k not in ("datetime", "orion_version")}
            if item != value:
                log.warning("Config given is different from config found in db at section: %s", section)
                log.warning("Config+ :\n%s", value)
                log.warning("Config- :\n%s", item)
                return True
        return False

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
