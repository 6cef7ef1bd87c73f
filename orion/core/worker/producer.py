"""``orion.core.worker.producer`` (reference `src/orion/core/worker/producer.py:18-67`)
-> :mod:`orion_amd.core.producer`."""
from orion_amd.core.producer import Producer  # noqa: F401
