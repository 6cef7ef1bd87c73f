"""``orion.core.utils`` (reference `src/orion/core/utils/__init__.py:23-122`) -> :mod:`orion_amd.utils`.

The reference's ``Factory`` metaclass is replaced by :class:`orion_amd.utils.Registry`
(entry-point discovery via ``importlib.metadata``).
"""
from orion_amd.utils import Registry, SingletonType  # noqa: F401
