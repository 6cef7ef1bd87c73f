"""``orion.algo.base`` -> :mod:`orion_amd.algo.base`."""
from orion_amd.algo.base import BaseAlgorithm, OptimizationAlgorithm  # noqa: F401
