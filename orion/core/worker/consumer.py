"""``orion.core.worker.consumer`` (reference `src/orion/core/worker/consumer.py:24-130`)
-> :mod:`orion_amd.core.consumer`."""
from orion_amd.core.consumer import Consumer, TrialInterrupted  # noqa: F401
