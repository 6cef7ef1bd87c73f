"""Document-store API with compare-and-swap (component C9).

Parity with ``src/orion/core/io/database/__init__.py``: ``AbstractDB`` with
``ensure_index / write / read / read_and_write / count / remove`` plus
connection management, ``DatabaseError`` and ``DuplicateKeyError``.

The two primitives every worker relies on:

* ``read_and_write(collection, query, data)`` -- atomically find ONE document
  matching ``query`` and ``$set`` ``data`` on it, returning the updated
  document or ``None``.  With a status precondition in ``query`` this is the
  trial-reservation compare-and-swap.
* unique indexes -> concurrent duplicate inserts raise ``DuplicateKeyError``
  (experiment-creation race).

Backends: :mod:`memory` (in-process), :mod:`local` (SQLite file, cross-process
atomic, the default), :mod:`mongodb` (pymongo, multi-node).
"""
from __future__ import annotations

import abc


class DatabaseError(RuntimeError):
    """Exception type used to delegate responsibility from any database implementation."""


class DuplicateKeyError(DatabaseError):
    """A write violates a unique index."""


class AbstractDB(abc.ABC):
    ASCENDING = 1
    DESCENDING = -1

    def __init__(self, host=None, name=None, port=None, username=None, password=None, **kwargs):
        self.host = host
        self.name = name
        self.port = port
        self.username = username
        self.password = password
        self.options = kwargs
        self._db = None
        self._conn = None
        self.initiate_connection()

    @property
    @abc.abstractmethod
    def is_connected(self):
        ...

    @abc.abstractmethod
    def initiate_connection(self):
        ...

    @abc.abstractmethod
    def close_connection(self):
        ...

    @abc.abstractmethod
    def ensure_index(self, collection_name, keys, unique=False):
        """keys: field name or list of (field, ASCENDING|DESCENDING)."""

    @abc.abstractmethod
    def write(self, collection_name, data, query=None):
        """Insert ``data`` (dict or list of dicts; ``_id`` added in place) when ``query`` is
        None, else ``$set`` it on every matching document (upsert).  Returns #docs written."""

    @abc.abstractmethod
    def read(self, collection_name, query=None, selection=None, skip=0, limit=None):
        """Matching documents in insertion order; ``skip``/``limit`` page through them."""

    @abc.abstractmethod
    def read_and_write(self, collection_name, query, data, selection=None):
        ...

    @abc.abstractmethod
    def count(self, collection_name, query=None):
        ...

    @abc.abstractmethod
    def remove(self, collection_name, query):
        ...

    def drop(self, collection_name):
        return self.remove(collection_name, {})


def normalize_index_keys(keys):
    if isinstance(keys, str):
        return [(keys, AbstractDB.ASCENDING)]
    return [(k, d) for k, d in keys]
