"""``orion.core.io.space_builder`` (reference `src/orion/core/io/space_builder.py:69-389`)
-> :mod:`orion_amd.space.dsl`."""
from orion_amd.space.dsl import DimensionBuilder, SpaceBuilder  # noqa: F401
