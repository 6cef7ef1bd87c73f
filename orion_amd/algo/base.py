"""Optimization-algorithm API and plugin registry (component C2).

Parity with ``src/orion/algo/base.py``: ``BaseAlgorithm(space, **hyper)`` with
``suggest(num)``, ``observe(points, results)``, the optional hooks ``is_done``,
``score``, ``judge``, ``should_suspend``, ``configuration`` (nested algorithms
serialise recursively), a ``space`` setter that propagates to nested
algorithms, and ``OptimizationAlgorithm(of_type, space, **kw)`` -- the factory
that resolves an algorithm by lower-case class name.

Discovery (reference: ``Factory`` metaclass + ``pkg_resources``,
``utils/__init__.py:46-116``) is re-done with ``importlib.metadata``:
subclasses register themselves on definition (any depth, not only immediate
subclasses), and third-party packages are loaded from the
``OptimizationAlgorithm`` entry-point group (the same group name as the
reference, so existing plugin packages keep working once they import
``orion_amd.algo.base.BaseAlgorithm``).
"""
from __future__ import annotations

import abc
import logging

from ..utils import Registry

log = logging.getLogger(__name__)

ENTRY_POINT_GROUP = "OptimizationAlgorithm"
ALGORITHMS = Registry("BaseAlgorithm", entry_point_group=ENTRY_POINT_GROUP)


def register_algorithm(cls, name=None):
    return ALGORITHMS.register(cls, name=name)


class BaseAlgorithm(abc.ABC):
    """An optimizer: suggests points of ``space`` and observes their results."""

    requires = None  # reserved for space-transformation requirements

    def __init_subclass__(cls, **kw):
        super().__init_subclass__(**kw)
        if not getattr(cls, "__abstractmethods__", None) and not cls.__name__.startswith("_") \
                and cls.__name__ not in ("OptimizationAlgorithm", "PrimaryAlgo"):
            register_algorithm(cls)

    def __init__(self, space, **kwargs):
        log.debug("Creating %s with parameters %s", type(self).__name__, kwargs)
        self._space = space
        self._param_names = list(kwargs.keys())
        for varname, param in kwargs.items():
            if isinstance(param, dict) and len(param) == 1:
                sub_type = next(iter(param))
                sub_kw = param[sub_type]
                if isinstance(sub_kw, dict) and str(sub_type).lower() in OptimizationAlgorithm.typenames:
                    param = OptimizationAlgorithm(sub_type, space, **sub_kw)
            elif isinstance(param, str) and param.lower() in OptimizationAlgorithm.typenames:
                param = OptimizationAlgorithm(param, space)
            setattr(self, varname, param)

    @abc.abstractmethod
    def suggest(self, num=1):
        """Return ``num`` new points (tuples ordered like ``space``)."""

    @abc.abstractmethod
    def observe(self, points, results):
        """Learn from evaluated ``points``; ``results`` are dicts with ``objective``,
        ``gradient`` (optional) and ``constraint`` (list, optional)."""

    @property
    def is_done(self):
        return False

    def score(self, point):  # noqa: ARG002
        return 0

    def judge(self, point, measurements):  # noqa: ARG002
        return None

    @property
    def should_suspend(self):
        return False

    @property
    def configuration(self):
        d = {}
        for name in self._param_names:
            if name.startswith("_"):
                continue
            attr = getattr(self, name)
            if isinstance(attr, BaseAlgorithm):
                attr = attr.configuration
            d[name] = attr
        return {type(self).__name__.lower(): d}

    @property
    def space(self):
        return self._space

    @space.setter
    def space(self, space_):
        self._space = space_
        for attr in list(self.__dict__.values()):
            if isinstance(attr, BaseAlgorithm):
                attr.space = space_

    # optional persistence of algorithm state (the reference never persisted it)
    @property
    def state_dict(self):
        return {}

    def set_state(self, state):
        pass


ALGORITHMS.base = BaseAlgorithm  # entry points must resolve to BaseAlgorithm subclasses


class _FactoryMeta(abc.ABCMeta):
    @property
    def types(cls):
        return ALGORITHMS.types

    @property
    def typenames(cls):
        return ALGORITHMS.typenames


class OptimizationAlgorithm(metaclass=_FactoryMeta):
    """Factory: ``OptimizationAlgorithm('random', space, **kw)`` -> a ``Random`` instance."""

    def __new__(cls, of_type, space, **kwargs):
        return ALGORITHMS.create(of_type, space, **kwargs)
