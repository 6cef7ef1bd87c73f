"""``orion.core.worker`` (reference `src/orion/core/worker/__init__.py:21-53`) -> :mod:`orion_amd.core.worker`."""
from orion_amd.core.worker import workon, workon_pool  # noqa: F401
