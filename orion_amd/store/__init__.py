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

_BACKENDS = {
    "sqlite": LocalDB, "local": LocalDB, "localdb": LocalDB, "pickleddb": LocalDB,
    "memory": MemoryDB, "memorydb": MemoryDB, "ephemeraldb": MemoryDB,
    "mongodb": MongoDB, "mongo": MongoDB,
}


def Database(of_type="sqlite", **options):  # noqa: N802  (reference factory name)
    try:
        klass = _BACKENDS[str(of_type).lower()]
    except KeyError as exc:
        raise NotImplementedError(f"Could not find implementation of AbstractDB, type = "
                                  f"'{of_type}' (known: {sorted(set(_BACKENDS))})") from exc
    return klass(**options)


def backend_names():
    return sorted(_BACKENDS)
