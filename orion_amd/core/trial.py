"""Trial record (component C5).

Parity with ``src/orion/core/worker/trial.py``: parameters (``integer`` /
``real`` / ``categorical``), results (``objective`` / ``constraint`` /
``gradient``), the status set ``new, reserved, suspended, completed,
interrupted, broken``, ``to_dict``/``build`` (de)serialisation with ``_id`` as
the database key, and ``objective``/``gradient`` accessors (first one wins
when several are reported, ``trial.py:246-250``).

Additions for the MI355X executor: ``heartbeat`` (liveness of the worker that
reserved the trial, used by the stale-reservation reaper) and ``gpus`` (the
devices the trial ran on).
"""
from __future__ import annotations

import logging

log = logging.getLogger(__name__)


class Trial:
    class Value:
        __slots__ = ("name", "_type", "value")
        allowed_types: tuple = ()

        def __init__(self, **kwargs):
            for a in self.__slots__:
                setattr(self, a, None)
            for k, v in kwargs.items():
                setattr(self, k, v)

        def to_dict(self):
            return dict(name=self.name, type=self._type, value=self.value)

        def __str__(self):
            return "{0}(name={1}, type={2}, value={3})".format(
                type(self).__name__, repr(self.name), repr(self._type), repr(self.value))

        __repr__ = __str__

        def __eq__(self, other):
            return isinstance(other, Trial.Value) and self.to_dict() == other.to_dict()

        @property
        def type(self):
            return self._type

        @type.setter
        def type(self, type_):
            if type_ is not None and type_ not in self.allowed_types:
                raise ValueError("Given type, {0}, not one of: {1}".format(type_, self.allowed_types))
            self._type = type_

    class Result(Value):
        allowed_types = ("objective", "constraint", "gradient")

    class Param(Value):
        allowed_types = ("integer", "real", "categorical")

    __slots__ = ("experiment", "_id", "_status", "worker", "submit_time", "start_time",
                 "end_time", "heartbeat", "gpus", "results", "params")
    allowed_stati = ("new", "reserved", "suspended", "completed", "interrupted", "broken")
    # statuses a worker may (re)reserve
    reservable_stati = ("new", "suspended", "interrupted")
    NoID = None

    def __init__(self, **kwargs):
        for a in self.__slots__:
            setattr(self, a, [] if a in ("results", "params") else None)
        self.status = "new"
        for k, v in kwargs.items():
            if k == "results":
                self.results = [self.Result(**r) for r in v]
            elif k == "params":
                self.params = [self.Param(**p) for p in v]
            elif k == "id":
                self._id = v
            else:
                setattr(self, k, v)

    @classmethod
    def build(cls, entries):
        return [cls(**e) for e in entries]

    def to_dict(self):
        d = {}
        for a in self.__slots__:
            d[a.lstrip("_")] = getattr(self, a)
        d["results"] = [r.to_dict() for r in self.results]
        d["params"] = [p.to_dict() for p in self.params]
        d.pop("id")
        if self.is_registered:
            d["_id"] = self._id
        return d

    def __str__(self):
        return "Trial(experiment={0}, status={1}, params.value={2})".format(
            repr(self.experiment), repr(self._status), [p.value for p in self.params])

    __repr__ = __str__

    @property
    def status(self):
        return self._status

    @status.setter
    def status(self, status):
        if status is not None and status not in self.allowed_stati:
            raise ValueError("Given status, {0}, not one of: {1}".format(status, self.allowed_stati))
        self._status = status

    @property
    def id(self):
        return self._id

    @property
    def objective(self):
        return self._fetch_one("objective")

    @property
    def gradient(self):
        return self._fetch_one("gradient")

    @property
    def constraints(self):
        return [r for r in self.results if r.type == "constraint"]

    @property
    def is_registered(self):
        return self._id is not self.NoID

    @property
    def params_dict(self):
        return {p.name: p.value for p in self.params}

    def _fetch_one(self, result_type):
        vals = [r for r in self.results if r.type == result_type]
        if not vals:
            return None
        if len(vals) > 1:
            log.warning("Found multiple results of '%s' type:\n%s", result_type, vals)
            log.warning("Multi-objective optimization is not currently supported.\n"
                        "Optimizing according to the first one only: %s", vals[0])
        return vals[0]
