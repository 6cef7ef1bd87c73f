"""``orion.core.io.database.mongodb`` (reference `src/orion/core/io/database/mongodb.py:64-255`)
-> :mod:`orion_amd.store.mongodb`."""
from orion_amd.store.mongodb import MongoDB, mongodb_exception_wrapper  # noqa: F401
