"""Document stores with compare-and-swap: the coordination medium between workers.

``Database(of_type, **options)`` picks a backend by (case-insensitive) name --
the reference's ``Database(of_type=...)`` factory (``cli.py:53-56``) without the
process-wide singleton: callers pass the returned handle explicitly.

=============  ==================================================================
type           backend
=============  ==================================================================
``sqlite``     :class:`~orion_amd.store.local.LocalDB` (default; aliases ``local``,
               ``localdb``, ``pickleddb``) -- one file, cross-process atomic
``memory``     :class:`~orion_amd.store.memory.MemoryDB` -- in-process only
``mongodb``    :class:`~orion_amd.store.mongodb.MongoDB` -- pymongo + server
=============  ==================================================================
"""
from __future__ import annotations

from .base import AbstractDB, DatabaseError, DuplicateKeyError  # noqa: F401
from .local import LocalDB
from .memory import MemoryDB
from .mongodb import MongoDB

from ..utils import Registry

# third-party backends can join through the "Database" entry-point group
BACKENDS = Registry("AbstractDB", entry_point_group="Database", base=AbstractDB)
BACKENDS.register(LocalDB, name="sqlite", aliases=("local", "localdb", "pickleddb"))
BACKENDS.register(MemoryDB, name="memory", aliases=("memorydb", "ephemeraldb"))
BACKENDS.register(MongoDB, name="mongodb", aliases=("mongo",))


def Database(of_type="sqlite", **options):  # noqa: N802  (reference factory name)
    return BACKENDS.create(of_type, **options)


def backend_names():
    return BACKENDS.typenames
