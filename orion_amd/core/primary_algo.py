"""Sanitising wrapper around the configured algorithm (component C4,
``src/orion/core/worker/primary_algo.py``): every point going in or out must
lie in the space; everything else is delegated."""
from __future__ import annotations

from ..algo.base import BaseAlgorithm


class PrimaryAlgo(BaseAlgorithm):
    def __init__(self, space, algorithm_config):
        self.algorithm = None
        super().__init__(space, algorithm=algorithm_config)
        if not isinstance(self.algorithm, BaseAlgorithm):
            raise TypeError(f"unknown algorithm configuration: {algorithm_config!r}")

    def suggest(self, num=1):
        points = self.algorithm.suggest(num)
        for p in points:
            assert p in self._space, f"suggested point {p} is outside the space"
        return points

    def observe(self, points, results):
        for p in points:
            assert p in self._space, f"observed point {p} is outside the space"
        assert len(points) == len(results)
        self.algorithm.observe(points, results)

    @property
    def is_done(self):
        return self.algorithm.is_done

    def score(self, point):
        assert point in self._space
        return self.algorithm.score(point)

    @property
    def scores_uniform(self):
        """True when the algorithm keeps the default ``score`` (every point ties), so a
        reservation may pick among a random window of candidates instead of scoring all."""
        from ..algo.base import BaseAlgorithm
        return type(self.algorithm).score is BaseAlgorithm.score

    def judge(self, point, measurements):
        assert point in self._space
        return self.algorithm.judge(point, measurements)

    @property
    def should_suspend(self):
        return self.algorithm.should_suspend

    @property
    def configuration(self):
        return self.algorithm.configuration

    @property
    def space(self):
        return self._space
