"""SQLite-file document store: the default, zero-dependency backend.

Cross-PROCESS atomicity (several ``orion`` workers on one node, or on nodes
sharing a POSIX filesystem with working locks) comes from SQLite's database
lock: every mutation runs in a ``BEGIN IMMEDIATE`` transaction, so the
trial-reservation compare-and-swap (``read_and_write`` with a status
precondition) and unique-index checks are serialised exactly like MongoDB's
single-document atomic ``find_one_and_update``.
WAL journaling keeps readers unblocked while a writer holds the lock.

Documents are stored as JSON (datetimes as ``{"$date": iso}``).  Hot paths are
indexed, so their cost does not grow with the number of trials:

* ``_id`` is the primary key and ``experiment`` / ``status`` are mirrored into
  indexed columns: a query that pins them by equality or ``$in`` is answered in
  SQL (the reservation compare-and-swap ``{_id, status}`` touches one row);
* ``count`` of such a query is ``SELECT COUNT(*)``; ``read(skip=, limit=)`` becomes
  ``LIMIT/OFFSET``;
* unique indexes are kept in a key table with a primary key on
  ``(collection, fields, key)``, so an insert checks uniqueness with one index probe
  instead of a scan of the collection.
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
_SQL_FIELDS = {"_id": "id", "experiment": "experiment", "status": "status"}


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
            conn.execute("CREATE TABLE IF NOT EXISTS _orion_unique "
                         "(coll TEXT, fields TEXT, key TEXT, id TEXT, PRIMARY KEY (coll, fields, key))")
            conn.execute("CREATE INDEX IF NOT EXISTS _orion_unique_id ON _orion_unique (coll, id)")
        except sqlite3.Error as exc:
            raise DatabaseError(f"cannot open local database {self.path}: {exc}") from exc
        self._open = True

    def _connect(self):
        conn = getattr(self._local, "conn", None)
        if conn is None:
            conn = sqlite3.connect(self.path, timeout=60.0, isolation_level=None,
                                   check_same_thread=False)
            conn.execute("PRAGMA busy_timeout=60000")
            # WAL + NORMAL: commits are atomic and crash-safe; only an OS crash may lose the
            # last transactions (no fsync per reservation)
            conn.execute("PRAGMA synchronous=NORMAL")
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

    @staticmethod
    def _sql_value(field, v):
        return v if field == "_id" else json.dumps(v, default=_default)

    def _prefilter(self, query):
        """SQL WHERE for ``_id`` and the mirrored columns where the query pins them by
        equality / ``$in``; ``covered`` says whether SQL alone decides the match."""
        where, args, covered = [], [], True
        for f, cond in (query or {}).items():
            col = _SQL_FIELDS.get(f)
            if col is None:
                covered = False
                continue
            if isinstance(cond, dict) and set(cond) == {"$in"} and \
                    all(not isinstance(v, (dict, list)) for v in cond["$in"]):
                vals = [self._sql_value(f, v) for v in cond["$in"]]
                where.append(f"{col} IN ({','.join('?' * len(vals))})" if vals else "0")
                args.extend(vals)
            elif not isinstance(cond, (dict, list)) and cond is not None:
                where.append(f"{col} = ?")
                args.append(self._sql_value(f, cond))
            else:
                covered = False
        return (" WHERE " + " AND ".join(where)) if where else "", args, covered

    def _select(self, conn, coll, query, skip=0, limit=None):
        self._table(conn, coll)
        w, a, covered = self._prefilter(query)
        page = ""
        if covered and (skip or limit is not None):
            page = f" LIMIT {int(limit) if limit is not None else -1} OFFSET {int(skip)}"
        rows = conn.execute(f"SELECT doc FROM {self._q(coll)}{w}{page}", a).fetchall()
        docs = (loads(r[0]) for r in rows)
        hits = [d for d in docs if match(d, query)]
        if not page and (skip or limit is not None):
            hits = hits[skip: None if limit is None else skip + limit]
        return hits

    def _unique_keys(self, conn, coll, doc):
        return [(json.dumps(list(fields)), json.dumps([get_path(doc, f) for f in fields], default=_default))
                for fields in self._uniques(conn, coll)]

    def _claim_keys(self, conn, coll, doc, replace=False):
        """Record ``doc``'s unique keys; DuplicateKeyError if another document holds one."""
        if replace:
            conn.execute("DELETE FROM _orion_unique WHERE coll=? AND id=?", (coll, doc["_id"]))
        for fields, key in self._unique_keys(conn, coll, doc):
            try:
                conn.execute("INSERT INTO _orion_unique (coll, fields, key, id) VALUES (?,?,?,?)",
                             (coll, fields, key, doc["_id"]))
            except sqlite3.IntegrityError as exc:
                raise DuplicateKeyError(f"duplicate key {fields}={key} in {coll}") from exc

    def _put(self, conn, coll, doc, insert):
        self._claim_keys(conn, coll, doc, replace=not insert)
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
                # documents written before the index existed get their keys now
                have = conn.execute("SELECT COUNT(*) FROM _orion_unique WHERE coll=? AND fields=?",
                                    (collection_name, fields)).fetchone()[0]
                total = conn.execute(f"SELECT COUNT(*) FROM {self._q(collection_name)}").fetchone()[0]
                if have != total:
                    conn.execute("DELETE FROM _orion_unique WHERE coll=? AND fields=?",
                                 (collection_name, fields))
                    flds = json.loads(fields)
                    for d in self._select(conn, collection_name, None):
                        key = json.dumps([get_path(d, f) for f in flds], default=_default)
                        try:
                            conn.execute("INSERT INTO _orion_unique (coll, fields, key, id) "
                                         "VALUES (?,?,?,?)", (collection_name, fields, key, d["_id"]))
                        except sqlite3.IntegrityError as exc:
                            raise DuplicateKeyError(f"existing documents violate unique index "
                                                    f"{fields} in {collection_name}") from exc
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
                    self._put(conn, collection_name, d, insert=True)
                n = len(docs)
            else:
                hits = self._select(conn, collection_name, query)
                if not hits:
                    new = {k: v for k, v in query.items() if not isinstance(v, dict) and "." not in k}
                    apply_set(new, data)
                    new.setdefault("_id", uuid.uuid4().hex)
                    self._put(conn, collection_name, new, insert=True)
                    n = 1
                else:
                    for d in hits:
                        apply_set(d, data)
                        self._put(conn, collection_name, d, insert=False)
                    n = len(hits)
            conn.execute("COMMIT")
            return n
        except BaseException:
            conn.execute("ROLLBACK")
            raise

    def read(self, collection_name, query=None, selection=None, skip=0, limit=None):
        conn = self._connect()
        return [project(d, selection)
                for d in self._select(conn, collection_name, query, skip, limit)]

    def read_and_write(self, collection_name, query, data, selection=None):
        conn = self._connect()
        self._begin(conn)
        try:
            hits = self._select(conn, collection_name, query, limit=1)
            if not hits:
                conn.execute("COMMIT")
                return None
            d = apply_set(hits[0], data)
            self._put(conn, collection_name, d, insert=False)
            conn.execute("COMMIT")
            return project(d, selection)
        except BaseException:
            conn.execute("ROLLBACK")
            raise

    def count(self, collection_name, query=None):
        conn = self._connect()
        self._table(conn, collection_name)
        w, a, covered = self._prefilter(query)
        if covered:
            return conn.execute(f"SELECT COUNT(*) FROM {self._q(collection_name)}{w}", a).fetchone()[0]
        return len(self._select(conn, collection_name, query))

    def remove(self, collection_name, query):
        conn = self._connect()
        self._begin(conn)
        try:
            hits = self._select(conn, collection_name, query)
            for d in hits:
                conn.execute(f"DELETE FROM {self._q(collection_name)} WHERE id=?", (d["_id"],))
                conn.execute("DELETE FROM _orion_unique WHERE coll=? AND id=?", (collection_name, d["_id"]))
            conn.execute("COMMIT")
            return len(hits)
        except BaseException:
            conn.execute("ROLLBACK")
            raise
