"""Orchestration core: trials, experiments, producer/consumer, worker loop, CLI."""
from .trial import Trial  # noqa: F401
from .experiment import Experiment, create_experiment  # noqa: F401
from .worker import workon, workon_pool  # noqa: F401
