"""Search-space dimensions (component C1 of SURVEY.md §2.1).

Parity with ``src/orion/algo/space.py`` of the reference:

* ``Dimension(name, prior, *args, **kwargs)`` -- prior is a scipy.stats
  distribution (name or instance); ``shape`` packs several values in one
  dimension; ``seed``/``random_state``/``size``/``discrete`` are rejected
  (``space.py:65-108``);
* ``Real`` -- optional ``low`` (inclusive) / ``high`` (exclusive) bounds and
  4-try rejection sampling (``space.py:199-276``);
* ``Integer`` -- real prior floored to ``int`` (``space.py:279-347``);
* ``Categorical`` -- finite categories with optional probabilities
  (``space.py:350-446``);
* ``Space`` -- ordered name -> dimension map, positional indexing and
  membership tests (``space.py:449-550``).

Differences by design: no private scipy helpers (``check_random_state``,
``_parse_args_rvs``), ``numpy.object`` replaced by ``object`` (numpy >= 1.24),
and shapes are normalised eagerly.
"""
from __future__ import annotations

import numbers
from collections import OrderedDict

import numpy
from scipy.stats import distributions

_FORBIDDEN_SEED = ("random_state", "seed")


def as_random_state(seed):
    """None -> numpy's global RandomState, int -> fresh RandomState, RandomState -> itself."""
    if seed is None or seed is numpy.random:
        return numpy.random.mtrand._rand
    if isinstance(seed, numbers.Integral):
        return numpy.random.RandomState(int(seed))
    if isinstance(seed, (numpy.random.RandomState, numpy.random.Generator)):
        return seed
    raise ValueError(f"{seed!r} cannot be used to seed a numpy.random.RandomState instance")


def _norm_shape(shape):
    if shape is None:
        return ()
    if isinstance(shape, numbers.Integral):
        return (int(shape),)
    return tuple(int(s) for s in shape)


class Dimension:
    """Base class: a named parameter with a scipy prior."""

    def __init__(self, name, prior, *args, **kwargs):
        self._name = None
        self.name = name
        if any(k in kwargs for k in _FORBIDDEN_SEED):
            raise ValueError("random_state/seed cannot be set in a parameter's definition! "
                             "Set seed globally!")
        if "discrete" in kwargs:
            raise ValueError("Do not use kwarg 'discrete' on `Dimension`, "
                             "use pure `_Discrete` class instead!")
        if "size" in kwargs:
            raise ValueError("Use 'shape' keyword only instead of 'size'.")
        if isinstance(prior, str):
            self._prior_name = prior
            self.prior = getattr(distributions, prior)
        else:
            self._prior_name = prior.name
            self.prior = prior
        self._shape = kwargs.pop("shape", None)
        self._args = args
        self._kwargs = kwargs

    # --------------------------------------------------------------- sampling
    def _rvs(self, rng):
        return self.prior.rvs(*self._args, size=self._shape, random_state=rng, **self._kwargs)

    def sample(self, n_samples=1, seed=None):
        """Draw ``n_samples`` values from the prior (list of length n_samples)."""
        rng = seed if seed is not None else None
        return [self._rvs(rng) for _ in range(n_samples)]

    def interval(self, alpha=1.0):
        """(low, high) containing ``alpha`` of the prior mass; low inclusive, high exclusive."""
        return self.prior.interval(alpha, *self._args, **self._kwargs)

    def __contains__(self, point):
        low, high = self.interval()
        p = numpy.asarray(point)
        if p.shape != self.shape:
            return False
        return bool(numpy.all(p < high) and numpy.all(p >= low))

    def __repr__(self):
        return "{0}(name={1}, prior={{{2}: {3}, {4}}}, shape={5})".format(
            type(self).__name__, self.name, self._prior_name, self._args, self._kwargs, self.shape)

    # --------------------------------------------------------------- properties
    @property
    def name(self):
        return self._name

    @name.setter
    def name(self, value):
        if value is not None and not isinstance(value, str):
            raise TypeError("Dimension's name must be either string or None. "
                            "Provided: {}, of type: {}".format(value, type(value)))
        self._name = value

    @property
    def type(self):
        return type(self).__name__.lower()

    @property
    def shape(self):
        return _norm_shape(self._shape)

    @property
    def prior_name(self):
        return self._prior_name

    def get_prior_string(self):
        """DSL expression that rebuilds this dimension (used in experiment documents)."""
        args = list(self._args)
        kw = dict(self._kwargs)
        if self._shape is not None:
            kw["shape"] = self._shape
        parts = [repr(a) for a in args] + [f"{k}={v!r}" for k, v in kw.items()]
        return f"{self._prior_name}({', '.join(parts)})"


class Real(Dimension):
    """Real-valued dimension with optional hard bounds ``low`` <= x < ``high``."""

    MAX_TRIES = 4

    def __init__(self, name, prior, *args, **kwargs):
        self._low = kwargs.pop("low", -numpy.inf)
        self._high = kwargs.pop("high", numpy.inf)
        if self._high <= self._low:
            raise ValueError("Lower bound {} has to be less than upper bound {}".format(
                self._low, self._high))
        super().__init__(name, prior, *args, **kwargs)

    def interval(self, alpha=1.0):
        lo, hi = super().interval(alpha)
        return (max(lo, self._low), min(hi, self._high))

    def sample(self, n_samples=1, seed=None):
        out = []
        for _ in range(n_samples):
            for _ in range(self.MAX_TRIES):
                s = self._draw_one(seed)
                if s in self:
                    out.append(s)
                    break
            else:
                raise ValueError("Improbable bounds: (low={0}, high={1}). "
                                 "Please make interval larger.".format(self._low, self._high))
        return out

    def _draw_one(self, seed):
        return Dimension.sample(self, 1, seed)[0]


class _Discrete(Dimension):
    """Mixin: floor real draws to integers; integer-valued interval."""

    def _draw_one(self, seed):
        v = super()._draw_one(seed)
        return numpy.floor(v).astype(int)

    def sample(self, n_samples=1, seed=None):
        return super().sample(n_samples, seed)

    def interval(self, alpha=1.0):
        lo, hi = super().interval(alpha)
        try:
            ilo = int(numpy.floor(lo))
        except OverflowError:
            ilo = -numpy.inf
        try:
            ihi = int(numpy.floor(hi))
        except OverflowError:
            ihi = numpy.inf
        if ihi < hi:  # exclusive upper bound
            ihi += 1
        return (ilo, ihi)


class Integer(_Discrete, Real):
    """Integer-valued dimension (real prior, floored)."""

    def __contains__(self, point):
        p = numpy.asarray(point)
        if not numpy.all(numpy.equal(numpy.mod(p, 1), 0)):
            return False
        return super().__contains__(point)

    def _draw_one(self, seed):
        v = Real._draw_one(self, seed)
        return numpy.floor(v).astype(int)


class Categorical(Dimension):
    """Finite set of categories; dict input gives per-category probabilities."""

    def __init__(self, name, categories, **kwargs):
        if isinstance(categories, dict):
            self.categories = tuple(categories.keys())
            self._probs = tuple(float(p) for p in categories.values())
        else:
            self.categories = tuple(categories)
            n = len(self.categories)
            self._probs = tuple(numpy.tile(1.0 / n, n))
        prior = distributions.rv_discrete(values=(list(range(len(self.categories))), self._probs))
        super().__init__(name, prior, **kwargs)

    def sample(self, n_samples=1, seed=None):
        rng = as_random_state(seed)
        cats = numpy.empty(len(self.categories), dtype=object)
        cats[:] = list(self.categories)
        return [rng.choice(cats, p=self._probs, size=self._shape) for _ in range(n_samples)]

    def interval(self, alpha=1.0):
        raise RuntimeError("Categories have no ``interval`` (as they are not ordered).\n"
                           "Use ``self.categories`` instead.")

    def __contains__(self, point):
        p = numpy.empty(numpy.shape(point) if not isinstance(point, str) else (), dtype=object)
        if p.shape == ():
            p = numpy.asarray(point, dtype=object)
        else:
            p[...] = point
        if p.shape != self.shape:
            return False
        check = numpy.vectorize(lambda x: x in self.categories, otypes=[bool])
        return bool(numpy.all(check(p)))

    @property
    def probabilities(self):
        return self._probs

    def __repr__(self):
        if len(self.categories) > 5:
            pairs = list(zip(self.categories[:2] + self.categories[-2:],
                             self._probs[:2] + self._probs[-2:]))
            items = ["{}: {:.2f}".format(c, p) for c, p in pairs]
            items.insert(2, "...")
        else:
            items = ["{}: {:.2f}".format(c, p) for c, p in zip(self.categories, self._probs)]
        return "Categorical(name={0}, prior={{{1}}}, shape={2})".format(
            self.name, ", ".join(items), self.shape)

    def get_prior_string(self):
        cats = dict(zip(self.categories, self._probs))
        return f"choices({cats!r})"


class Space(OrderedDict):
    """Ordered collection of named dimensions: the problem's search space."""

    def register(self, dimension):
        self[dimension.name] = dimension

    def sample(self, n_samples=1, seed=None):
        """``n_samples`` points, each a tuple ordered like the dimensions."""
        rng = as_random_state(seed)
        cols = [dim.sample(n_samples, rng) for dim in self.values()]
        return list(zip(*cols))

    def interval(self, alpha=1.0):
        return [dim.categories if dim.type == "categorical" else dim.interval(alpha)
                for dim in self.values()]

    def __getitem__(self, key):
        if isinstance(key, str):
            return super().__getitem__(key)
        return list(self.values())[key]

    def __setitem__(self, key, value):
        if not isinstance(key, str):
            raise TypeError("Keys registered to Space must be string types. "
                            "Provided: {}".format(key))
        if not isinstance(value, Dimension):
            raise TypeError("Values registered to Space must be Dimension types. "
                            "Provided: {}".format(value))
        if key in self:
            raise ValueError("There is already a Dimension registered with this name. "
                             "Register it with another name. Provided: {}".format(key))
        super().__setitem__(key, value)

    def __contains__(self, value):
        if isinstance(value, str):
            return super().__contains__(value)
        try:
            len(value)
        except TypeError as exc:
            raise TypeError("Can check only for dimension names or "
                            "for tuples with parameter values.") from exc
        if not self:
            return False
        return all(component in dim for component, dim in zip(value, self.values()))

    def __repr__(self):
        return "Space([{}])".format(",\n       ".join(map(str, self.values())))

    def configuration(self):
        """name -> DSL prior string (what is stored with an experiment)."""
        return {name: dim.get_prior_string() for name, dim in self.items()}
