"""``orion.core.io.database`` (reference `src/orion/core/io/database/__init__.py:21-235`) -> :mod:`orion_amd.store`.

``Database(of_type=...)`` is a plain factory here (no singleton): pass the handle explicitly.
"""
from orion_amd.store import (  # noqa: F401
    AbstractDB, Database, DatabaseError, DuplicateKeyError, LocalDB, MemoryDB, MongoDB)
