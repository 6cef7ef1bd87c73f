"""MongoDB backend (multi-node coordination), parity with
``src/orion/core/io/database/mongodb.py``.

Maps ``write`` to ``insert_many`` / ``update_many(upsert=True)``,
``read_and_write`` to ``find_one_and_update(..., return_document=AFTER)``,
``count`` to ``count_documents`` (``Collection.count`` was removed in
pymongo 4), and converts pymongo errors into
:class:`DatabaseError` / :class:`DuplicateKeyError`.
"""
from __future__ import annotations

import functools

from .base import AbstractDB, DatabaseError, DuplicateKeyError, normalize_index_keys

try:
    import pymongo
    from pymongo import errors as _perr
except ImportError:  # pragma: no cover - pymongo is optional
    pymongo = None
    _perr = None


def mongodb_exception_wrapper(method):
    """Convert pymongo exceptions into the backend-neutral ones."""

    @functools.wraps(method)
    def _inner(*args, **kwargs):
        try:
            return method(*args, **kwargs)
        except _perr.DuplicateKeyError as exc:
            raise DuplicateKeyError(str(exc)) from exc
        except _perr.BulkWriteError as exc:
            codes = {e.get("code") for e in exc.details.get("writeErrors", [])}
            if 11000 in codes:
                raise DuplicateKeyError(str(exc)) from exc
            raise DatabaseError(str(exc)) from exc
        except _perr.ConnectionFailure as exc:
            raise DatabaseError("Connection Failure: database not found on specified uri") from exc
        except _perr.OperationFailure as exc:
            if "Authentication failed" in str(exc) or getattr(exc, "code", None) == 18:
                raise DatabaseError("Authentication Failure: bad credentials") from exc
            raise DatabaseError(str(exc)) from exc

    return _inner


class MongoDB(AbstractDB):
    """``host`` may be a hostname or a full ``mongodb://user:pw@host:port/db`` URI; fields
    given explicitly (``port=``, ``name=``, ``username=``, ``password=``) override the
    URI's (reference ``mongodb.py:237-255``).  ``check_connection=False`` skips the
    initial round trip (pymongo connects lazily), e.g. to inspect a configuration."""

    DEFAULT_PORT = 27017

    @mongodb_exception_wrapper
    def initiate_connection(self):
        if pymongo is None:
            raise DatabaseError("pymongo is not installed")
        check = self.options.pop("check_connection", True)
        self._sanitize_attrs()
        kw = dict(self._uri_options)
        kw.update(self.options)
        kw.setdefault("serverSelectionTimeoutMS", 5000)
        if self.username:
            kw.update(username=self.username, password=self.password, authSource=self.name)
        self._conn = pymongo.MongoClient(host=self.host, port=self.port, **kw)
        self._db = self._conn[self.name]
        if check:
            self._conn.admin.command("ping")

    def _sanitize_attrs(self):
        self._uri_options = {}
        if self.host and str(self.host).startswith(("mongodb://", "mongodb+srv://")):
            from pymongo.uri_parser import parse_uri
            info = parse_uri(self.host, validate=False)
            nodes = info.get("nodelist") or [("localhost", self.DEFAULT_PORT)]
            self.host = nodes[0][0]
            self.port = self.port if self.port is not None else nodes[0][1]
            self.username = self.username or info.get("username")
            self.password = self.password or info.get("password")
            self.name = self.name or info.get("database")
            self._uri_options = dict(info.get("options") or {})
        self.host = self.host or "localhost"
        self.port = int(self.port) if self.port is not None else self.DEFAULT_PORT
        self.name = self.name or "orion"

    @property
    def is_connected(self):
        if self._conn is None:
            return False
        try:
            self._conn.admin.command("ping")
            return True
        except Exception:
            return False

    def close_connection(self):
        if self._conn is not None:
            self._conn.close()

    @mongodb_exception_wrapper
    def ensure_index(self, collection_name, keys, unique=False):
        keys = normalize_index_keys(keys)
        self._db[collection_name].create_index(keys, unique=unique, background=True)

    @mongodb_exception_wrapper
    def write(self, collection_name, data, query=None):
        coll = self._db[collection_name]
        if query is None:
            docs = data if isinstance(data, list) else [data]
            return len(coll.insert_many(docs).inserted_ids)
        upd = data if "$set" in data else {"$set": data}
        res = coll.update_many(query, upd, upsert=True)
        return res.modified_count or (1 if res.upserted_id is not None else 0)

    @mongodb_exception_wrapper
    def read(self, collection_name, query=None, selection=None, skip=0, limit=None):
        cur = self._db[collection_name].find(query or {}, selection)
        if skip:
            cur = cur.skip(int(skip))
        if limit is not None:
            cur = cur.limit(int(limit))
        return list(cur)

    @mongodb_exception_wrapper
    def read_and_write(self, collection_name, query, data, selection=None):
        upd = data if "$set" in data else {"$set": data}
        return self._db[collection_name].find_one_and_update(
            query, upd, projection=selection, return_document=pymongo.ReturnDocument.AFTER)

    @mongodb_exception_wrapper
    def count(self, collection_name, query=None):
        return self._db[collection_name].count_documents(query or {})

    @mongodb_exception_wrapper
    def remove(self, collection_name, query):
        return self._db[collection_name].delete_many(query).deleted_count
