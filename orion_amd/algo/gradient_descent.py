"""Gradient descent on a black box that reports its gradient (plugin P1).

Behaviour of the reference's test plugin
(``tests/functional/gradient_descent_algo/src/orion/algo/gradient_descent.py``):
the first suggestion is random; afterwards ``x <- x - lr * grad`` using the
last observed point and gradient; done when ``lr * ||grad|| <= 1e-7``.
Shipped in-tree (still discoverable through the entry-point group too).
"""
from __future__ import annotations

import numpy

from .base import BaseAlgorithm


class Gradient_Descent(BaseAlgorithm):  # noqa: N801 (name kept for plugin/config parity)
    dx_tolerance = 1e-7

    def __init__(self, space, learning_rate=1.0):
        super().__init__(space, learning_rate=learning_rate)
        self.current_point = None
        self.gradient = numpy.array([numpy.inf])

    def suggest(self, num=1):
        assert num == 1, "gradient descent suggests one point at a time"
        if self.current_point is None:
            return self.space.sample(1)
        return [tuple(numpy.asarray(self.current_point) - self.learning_rate * self.gradient)]

    def observe(self, points, results):
        self.current_point = numpy.asarray(points[-1])
        grad = results[-1].get("gradient")
        self.gradient = numpy.asarray(grad if grad is not None else [0.0] * len(points[-1]))

    @property
    def is_done(self):
        dx = self.learning_rate * numpy.sqrt(numpy.sum(self.gradient ** 2))
        return bool(dx <= self.dx_tolerance)


GradientDescent = Gradient_Descent
