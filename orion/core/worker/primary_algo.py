"""``orion.core.worker.primary_algo`` (reference `src/orion/core/worker/primary_algo.py:17-119`)
-> :mod:`orion_amd.core.primary_algo`."""
from orion_amd.core.primary_algo import PrimaryAlgo  # noqa: F401
