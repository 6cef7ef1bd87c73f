"""``orion.algo.random`` (reference `src/orion/algo/random.py:15`) -> :mod:`orion_amd.algo.random`."""
from orion_amd.algo.random import Random  # noqa: F401
