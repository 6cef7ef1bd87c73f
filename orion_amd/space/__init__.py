"""Search spaces: typed dimensions and the ``~`` prior DSL."""
from .dimensions import Categorical, Dimension, Integer, Real, Space  # noqa: F401
from .dsl import DimensionBuilder, SpaceBuilder  # noqa: F401
