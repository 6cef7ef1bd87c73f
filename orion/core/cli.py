"""``orion.core.cli`` -> :mod:`orion_amd.core.cli`."""
from orion_amd.core.cli import main  # noqa: F401
