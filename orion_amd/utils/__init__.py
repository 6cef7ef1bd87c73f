"""Shared utilities: plugin registries and singletons (component C14).

The reference builds its factories from metaclasses
(``src/orion/core/utils/__init__.py:23-122``: ``SingletonType``, ``Factory``,
``SingletonFactory``) that glob sibling modules, load ``pkg_resources`` entry
points and accept only *immediate* subclasses.  Here the same capabilities are
an explicit :class:`Registry` object:

* case-insensitive name -> class mapping, filled by ``register`` (usable as a
  decorator) or by subclass hooks, at any inheritance depth;
* lazy discovery of third-party implementations from an
  ``importlib.metadata`` entry-point group (same group names as the reference,
  e.g. ``OptimizationAlgorithm``);
* ``create(of_type, *args, **kw)`` raising ``NotImplementedError`` with the
  reference's message when a type is unknown.

:class:`SingletonType` is kept for API compatibility (one instance per class,
resettable in tests: SURVEY.md §2.4 T3), but the framework itself passes
explicit store / experiment handles instead of relying on hidden singletons
(SURVEY.md §5.1 item 1).
"""
from __future__ import annotations

import importlib.metadata
import logging
import threading

log = logging.getLogger(__name__)


class Registry:
    """Named implementations of one abstract type, plus entry-point plugins."""

    def __init__(self, kind: str, entry_point_group: str | None = None, base: type | None = None):
        self.kind = kind
        self.group = entry_point_group
        self.base = base
        self._types: dict[str, type] = {}
        self._ep_loaded = entry_point_group is None
        self._lock = threading.Lock()

    # registration -------------------------------------------------------
    def register(self, obj=None, *, name: str | None = None, aliases=()):
        """Register a class (or a factory callable) under its lower-cased name."""
        def _do(o):
            key = (name or o.__name__).lower()
            self._types[key] = o
            for a in aliases:
                self._types[a.lower()] = o
            return o
        return _do(obj) if obj is not None else _do

    def _load_entry_points(self):
        if self._ep_loaded:
            return
        with self._lock:
            if self._ep_loaded:
                return
            self._ep_loaded = True
            try:
                eps = importlib.metadata.entry_points()
                group = (eps.select(group=self.group) if hasattr(eps, "select")
                         else eps.get(self.group, []))
            except Exception as exc:  # pragma: no cover
                log.debug("entry point discovery failed for %s: %s", self.group, exc)
                return
            for ep in group:
                try:
                    obj = ep.load()
                except Exception as exc:
                    log.warning("could not load %s plugin %s: %s", self.kind, ep, exc)
                    continue
                if self.base is not None and not (isinstance(obj, type) and issubclass(obj, self.base)):
                    log.warning("entry point %s is not a %s subclass; ignored", ep, self.base.__name__)
                    continue
                self._types.setdefault(obj.__name__.lower(), obj)
                self._types.setdefault(ep.name.lower(), obj)

    # lookup -------------------------------------------------------------
    @property
    def types(self):
        self._load_entry_points()
        return list(dict.fromkeys(self._types.values()))

    @property
    def typenames(self):
        self._load_entry_points()
        return sorted(self._types)

    def get(self, of_type: str):
        self._load_entry_points()
        key = str(of_type).lower()
        if key not in self._types:
            raise NotImplementedError(
                "Could not find implementation of {}, type = '{}'\n"
                "Currently, there is an implementation for types:\n{}".format(
                    self.kind, of_type, self.typenames))
        return self._types[key]

    def create(self, of_type: str, *args, **kwargs):
        return self.get(of_type)(*args, **kwargs)

    def __contains__(self, of_type):
        self._load_entry_points()
        return str(of_type).lower() in self._types


class SingletonType(type):
    """Metaclass: one instance per class (``cls.instance``); ``cls.reset()`` drops it."""

    def __init__(cls, name, bases, ns):
        super().__init__(name, bases, ns)
        cls.instance = None

    def __call__(cls, *args, **kwargs):
        if cls.instance is None:
            cls.instance = super().__call__(*args, **kwargs)
        elif args or kwargs:
            raise ValueError("A singleton instance has already been instantiated.")
        return cls.instance

    def reset(cls):
        cls.instance = None

