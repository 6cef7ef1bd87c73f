"""``orion.core.worker.experiment`` (reference `src/orion/core/worker/experiment.py:27-473`)
-> :mod:`orion_amd.core.experiment`."""
from orion_amd.core.experiment import Experiment, create_experiment  # noqa: F401
