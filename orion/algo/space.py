"""``orion.algo.space`` -> :mod:`orion_amd.space.dimensions`."""
from orion_amd.space.dimensions import Categorical, Dimension, Integer, Real, Space  # noqa: F401
