"""In-process document store (tests, single-process runs).  Thread-safe."""
from __future__ import annotations

import copy
import threading
import uuid

from .base import AbstractDB, DuplicateKeyError, normalize_index_keys
from .query import apply_set, get_path, match, project


class MemoryDB(AbstractDB):
    def initiate_connection(self):
        self._lock = threading.RLock()
        self._colls = {}
        self._unique = {}  # collection -> list of key tuples
        self._open = True

    @property
    def is_connected(self):
        return self._open

    def close_connection(self):
        self._open = False

    def _coll(self, name):
        return self._colls.setdefault(name, {})

    def ensure_index(self, collection_name, keys, unique=False):
        keys = normalize_index_keys(keys)
        if unique:
            with self._lock:
                fields = tuple(k for k, _ in keys)
                lst = self._unique.setdefault(collection_name, [])
                if fields not in lst:
                    lst.append(fields)

    def _check_unique(self, collection_name, doc, exclude_id=None):
        for fields in self._unique.get(collection_name, []):
            key = tuple(repr(get_path(doc, f)) for f in fields)
            for other in self._coll(collection_name).values():
                if other["_id"] == exclude_id:
                    continue
                if tuple(repr(get_path(other, f)) for f in fields) == key:
                    raise DuplicateKeyError(f"duplicate key {dict(zip(fields, key))} in "
                                            f"{collection_name}")

    def write(self, collection_name, data, query=None):
        with self._lock:
            coll = self._coll(collection_name)
            if query is None:
                docs = data if isinstance(data, list) else [data]
                staged = []
                for d in docs:
                    d.setdefault("_id", uuid.uuid4().hex)
                    if d["_id"] in coll:
                        raise DuplicateKeyError(f"duplicate _id {d['_id']}")
                    self._check_unique(collection_name, d)
                    staged.append(copy.deepcopy(d))
                for d in staged:
                    coll[d["_id"]] = d
                return len(staged)
            hits = [d for d in coll.values() if match(d, query)]
            if not hits:  # upsert
                new = {k: copy.deepcopy(v) for k, v in query.items()
                       if not isinstance(v, dict) and "." not in k}
                apply_set(new, data)
                new.setdefault("_id", uuid.uuid4().hex)
                self._check_unique(collection_name, new)
                coll[new["_id"]] = new
                return 1
            for d in hits:
                cand = apply_set(copy.deepcopy(d), data)
                self._check_unique(collection_name, cand, exclude_id=d["_id"])
                coll[d["_id"]] = cand
            return len(hits)

    def read(self, collection_name, query=None, selection=None, skip=0, limit=None):
        with self._lock:
            hits = [d for d in self._coll(collection_name).values() if match(d, query)]
            hits = hits[skip: None if limit is None else skip + limit]
            return [project(copy.deepcopy(d), selection) for d in hits]

    def read_and_write(self, collection_name, query, data, selection=None):
        with self._lock:
            for d in self._coll(collection_name).values():
                if match(d, query):
                    cand = apply_set(copy.deepcopy(d), data)
                    self._check_unique(collection_name, cand, exclude_id=d["_id"])
                    self._coll(collection_name)[d["_id"]] = cand
                    return project(copy.deepcopy(cand), selection)
            return None

    def count(self, collection_name, query=None):
        with self._lock:
            return sum(1 for d in self._coll(collection_name).values() if match(d, query))

    def remove(self, collection_name, query):
        with self._lock:
            coll = self._coll(collection_name)
            ids = [i for i, d in coll.items() if match(d, query)]
            for i in ids:
                del coll[i]
            return len(ids)
