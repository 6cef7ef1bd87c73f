"""``orion.core.cli`` (reference `src/orion/core/cli.py:28-128`) -> :mod:`orion_amd.core.cli`."""
from orion_amd.core.cli import *  # noqa: F401,F403
from orion_amd.core.cli import main  # noqa: F401
