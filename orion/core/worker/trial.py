"""``orion.core.worker.trial`` (reference `src/orion/core/worker/trial.py:17-252`) -> :mod:`orion_amd.core.trial`."""
from orion_amd.core.trial import Trial  # noqa: F401
