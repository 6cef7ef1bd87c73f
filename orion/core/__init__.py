"""``orion.core`` entry points -> :mod:`orion_amd.core`."""
from orion_amd import __version__  # noqa: F401
