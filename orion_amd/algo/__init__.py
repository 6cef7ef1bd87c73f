"""Optimization algorithms.  Importing this package registers the built-ins."""
from .base import BaseAlgorithm, OptimizationAlgorithm, register_algorithm  # noqa: F401
from .random import Random  # noqa: F401
from .gradient_descent import Gradient_Descent  # noqa: F401
