"""Random search (component C3): ``suggest`` draws from the space's priors.
Parity with ``src/orion/algo/random.py``; adds an optional ``seed``."""
from __future__ import annotations

import numpy

from .base import BaseAlgorithm


class Random(BaseAlgorithm):
    def __init__(self, space, seed=None):
        kw = {} if seed is None else {"seed": seed}
        super().__init__(space, **kw)
        self.seed = seed
        self._rng = numpy.random.RandomState(seed) if seed is not None else None

    def suggest(self, num=1):
        return self.space.sample(num, seed=self._rng)

    def observe(self, points, results):
        pass
