"""SQLite-file document store: the default, zero-dependency backend.

Cross-PROCESS atomicity (several ``orion`` workers on one node, or on nodes
sharing a POSIX filesystem with working locks) comes from SQLite's database
lock: every mutation runs in a ``BEGIN IMMEDIATE`` transaction, so the
trial-reservation compare-and-swap (``read_and_write`` with a status
precondition) and unique-index checks are serialised exactly like MongoDB's
single-document atomic ``find_one_and_update``.
WAL journaling keeps readers unblocked while a writer holds the lock.

Documents are stored as JSON (datetimes as ``{"$date": iso}``); the queried
fields ``experiment`` and ``status`` are mirrored into indexed columns so a
worker's poll does not parse every trial document.
"""
from __future__ import annotations

import datetime
import json
import os
import sqlite3
import threading
import time
import uuid

import numpy

from .base import AbstractDB, DatabaseError, DuplicateKeyError, normalize_index_keys
from .query import apply_set, get_path, match, project

_INDEXED = ("experiment", "status")


def _default(o):
    if isinstance(o, datetime.datetime):
        return {"$date": o.isoformat()}
    if isinstance(o, numpy.generic):
        return o.item()
    if isinstance(o, numpy.ndarray):
        return o.tolist()
    raise TypeError(f"not JSON serializable: {type(o)}")


def _hook(d):
    if len(d) == 1 and "$date" in d:
        return datetime.datetime.fromisoformat(d["$date"])
    return d


def dumps(doc):
    return json.dumps(doc, default=_default)


def loads(s):
    return json.loads(s, object_hook=_hook)


def _col_value(doc, field):
    v = doc.get(field)
    return None if v is None else json.dumps(v, default=_default)


class LocalDB(AbstractDB):
    """``host`` = path of the SQLite file (created if missing); ``name`` is informational."""

    def initiate_connection(self):
        path = self.host or self.options.get("path")
        if not path:
            from ..core.config import DIRS
            os.makedirs(DIRS.user_data_dir, exist_ok=True)
            path = os.path.join(DIRS.user_data_dir, f"{self.name or 'orion'}.sqlite")
        self.path = os.path.abspath(os.path.expanduser(path))
        os.makedirs(os.path.dirname(self.path), exist_ok=True)
        self._local = threading.local()
        self._unique_cache = {}
        self._tables = set()
        try:
            conn = self._connect()
            conn.execute("PRAGMA journal_mode=WAL")
            conn.execute("CREATE TABLE IF NOT EXISTS _orion_indexes "
                         "(coll TEXT, fields TEXT, uniq INTEGER, PRIMARY KEY (coll, fields))")
        except sqlite3.Error as exc:
            raise DatabaseError(f"cannot open local database {self.path}: {exc}") from exc
        self._open = True

    def _connect(self):
        conn = getattr(self._local, "conn", None)
        if conn is None:
            conn = sqlite3.connect(self.path, timeout=60.0, isolation_level=None,
                                   check_same_thread=False)
            conn.execute("PRAGMA busy_timeout=60000")
            self._local.conn = conn
        return conn

    @property
    def is_connected(self):
        return self._open

    def close_connection(self):
        conn = getattr(self._local, "conn", None)
        if conn is not None:
            conn.close()
            self._local.conn = None
        self._open = False

    # ------------------------------------------------------------ schema helpers
    def _table(self, conn, coll):
        if coll in self._tables:
            return
        q = '"' + coll.replace('"', '') + '"'
        conn.execute(f"CREATE TABLE IF NOT EXISTS {q} (id TEXT PRIMARY KEY, experiment TEXT, "
                     f"status TEXT, doc TEXT NOT NULL)")
        conn.execute(f"CREATE INDEX IF NOT EXISTS \"{coll}_exp_status\" ON {q} (experiment, status)")
        self._tables.add(coll)

    def _q(self, coll):
        return '"' + coll.replace('"', '') + '"'

    def _begin(self, conn):
        for attempt in range(200):
            try:
                conn.execute("BEGIN IMMEDIATE")
                return
            except sqlite3.OperationalError as exc:
                if "locked" not in str(exc) and "busy" not in str(exc):
                    raise DatabaseError(str(exc)) from exc
                time.sleep(0.01 * (1 + attempt % 10))
        raise DatabaseError("database is locked")

    def _uniques(self, conn, coll):
        rows = conn.execute("SELECT fields FROM _orion_indexes WHERE coll=? AND uniq=1", (coll,)).fetchall()
        return [tuple(json.loads(r[0])) for r in rows]

    def _prefilter(self, query):
        """SQL WHERE for the mirrored columns when the query pins them by equality / $in."""
        where, args = [], []
        for f in _INDEXED:
            if not query or f not in query:
                continue
            cond = query[f]
            if isinstance(cond, dict) and set(cond) == {"$in"}:
                vals = [json.dumps(v, default=_default) for v in cond["$in"]]
                where.append(f"{f} IN ({','.join('?' * len(vals))})")
                args.extend(vals)
            elif not isinstance(cond, (dict, list)):
                where.append(f"{f} = ?")
                args.append(json.dumps(cond, default=_default))
        return (" WHERE " + " AND ".join(where)) if where else "", args

    def _select(self, conn, coll, query):
        self._table(conn, coll)
        w, a = self._prefilter(query)
        rows = conn.execute(f"SELECT doc FROM {self._q(coll)}{w}", a).fetchall()
        docs = (loads(r[0]) for r in rows)
        return [d for d in docs if match(d, query)]

    def _check_unique(self, conn, coll, doc, exclude_id=None):
        for fields in self._uniques(conn, coll):
            key = tuple(get_path(doc, f) for f in fields)
            for other in self._select(conn, coll, None):
                if other["_id"] == exclude_id:
                    continue
                if tuple(get_path(other, f) for f in fields) == key:
                    raise DuplicateKeyError(f"duplicate key {dict(zip(fields, map(repr, key)))} "
                                            f"in {coll}")

    def _put(self, conn, coll, doc, insert):
        vals = (doc["_id"], _col_value(doc, "experiment"), _col_value(doc, "status"), dumps(doc))
        if insert:
            try:
                conn.execute(f"INSERT INTO {self._q(coll)} (id, experiment, status, doc) VALUES (?,?,?,?)", vals)
            except sqlite3.IntegrityError as exc:
                raise DuplicateKeyError(str(exc)) from exc
        else:
            conn.execute(f"UPDATE {self._q(coll)} SET experiment=?, status=?, doc=? WHERE id=?",
                         (vals[1], vals[2], vals[3], vals[0]))

    # ------------------------------------------------------------ API
    def ensure_index(self, collection_name, keys, unique=False):
        keys = normalize_index_keys(keys)
        fields = json.dumps([k for k, _ in keys])
        conn = self._connect()
        self._begin(conn)
        try:
            self._table(conn, collection_name)
            conn.execute("INSERT OR IGNORE INTO _orion_indexes (coll, fields, uniq) VALUES (?,?,?)",
                         (collection_name, fields, int(bool(unique))))
            if unique:
                conn.execute("UPDATE _orion_indexes SET uniq=1 WHERE coll=? AND fields=?",
                             (collection_name, fields))
            conn.execute("COMMIT")
        except BaseException:
            conn.execute("ROLLBACK")
            raise

    def write(self, collection_name, data, query=None):
        conn = self._connect()
        self._begin(conn)
        try:
            self._table(conn, collection_name)
            if query is None:
                docs = data if isinstance(data, list) else [data]
                for d in docs:
                    d.setdefault("_id", uuid.uuid4().hex)
                    self._check_unique(conn, collection_name, d)
                    self._put(conn, collection_name, d, insert=True)
                n = len(docs)
            else:
                hits = self._select(conn, collection_name, query)
                if not hits:
                    new = {k: v for k, v in query.items() if not isinstance(v, dict) and "." not in k}
                    apply_set(new, data)
                    new.setdefault("_id", uuid.uuid4().hex)
                    self._check_unique(conn, collection_name, new)
                    self._put(conn, collection_name, new, insert=True)
                    n = 1
                else:
                    for d in hits:
                        apply_set(d, data)
                        self._check_unique(conn, collection_name, d, exclude_id=d["_id"])
                        self._put(conn, collection_name, d, insert=False)
                    n = len(hits)
            conn.execute("COMMIT")
            return n
        except BaseException:
            conn.execute("ROLLBACK")
            raise

    def read(self, collection_name, query=None, selection=None):
        conn = self._connect()
        return [project(d, selection) for d in self._select(conn, collection_name, query)]

    def read_and_write(self, collection_name, query, data, selection=None):
        conn = self._connect()
        self._begin(conn)
        try:
            hits = self._select(conn, collection_name, query)
            if not hits:
                conn.execute("COMMIT")
                return None
            d = apply_set(hits[0], data)
            self._check_unique(conn, collection_name, d, exclude_id=d["_id"])
            self._put(conn, collection_name, d, insert=False)
            conn.execute("COMMIT")
            return project(d, selection)
        except BaseException:
            conn.execute("ROLLBACK")
            raise

    def count(self, collection_name, query=None):
        conn = self._connect()
        return len(self._select(conn, collection_name, query))

    def remove(self, collection_name, query):
        conn = self._connect()
        self._begin(conn)
        try:
            hits = self._select(conn, collection_name, query)
            for d in hits:
                conn.execute(f"DELETE FROM {self._q(collection_name)} WHERE id=?", (d["_id"],))
            conn.execute("COMMIT")
            return len(hits)
        except BaseException:
            conn.execute("ROLLBACK")
            raise
