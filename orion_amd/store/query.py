"""Mongo-style query / projection / $set evaluation for the local document stores.

The subset the framework (and the reference's protocol) uses:
equality on dotted keys (a list field matches if it contains the value),
``$in $nin $eq $ne $gt $gte $lt $lte $exists``, include/exclude projections,
and ``$set`` updates with dotted keys.
"""
from __future__ import annotations

import copy

_MISSING = object()


def get_path(doc, key):
    cur = doc
    for part in key.split("."):
        if isinstance(cur, dict) and part in cur:
            cur = cur[part]
        elif isinstance(cur, list) and part.isdigit() and int(part) < len(cur):
            cur = cur[int(part)]
        else:
            return _MISSING
    return cur


def set_path(doc, key, value):
    parts = key.split(".")
    cur = doc
    for part in parts[:-1]:
        nxt = cur.get(part)
        if not isinstance(nxt, dict):
            nxt = {}
            cur[part] = nxt
        cur = nxt
    cur[parts[-1]] = value


def _cmp(op, a, b):
    try:
        if op == "$gt":
            return a > b
        if op == "$gte":
            return a >= b
        if op == "$lt":
            return a < b
        if op == "$lte":
            return a <= b
    except TypeError:
        return False
    raise ValueError(op)


def _eq(val, target):
    if val is _MISSING:
        return target is None
    if isinstance(val, list) and not isinstance(target, list):
        return target in val
    return val == target


def _match_cond(val, cond):
    if isinstance(cond, dict) and cond and all(k.startswith("$") for k in cond):
        for op, arg in cond.items():
            if op == "$in":
                if not any(_eq(val, a) for a in arg):
                    return False
            elif op == "$nin":
                if any(_eq(val, a) for a in arg):
                    return False
            elif op == "$eq":
                if not _eq(val, arg):
                    return False
            elif op == "$ne":
                if _eq(val, arg):
                    return False
            elif op == "$exists":
                if (val is not _MISSING) != bool(arg):
                    return False
            elif op in ("$gt", "$gte", "$lt", "$lte"):
                if val is _MISSING or not _cmp(op, val, arg):
                    return False
            else:
                raise ValueError(f"unsupported query operator {op}")
        return True
    return _eq(val, cond)


def match(doc, query):
    if not query:
        return True
    for key, cond in query.items():
        if key == "$or":
            if not any(match(doc, q) for q in cond):
                return False
            continue
        if key == "$and":
            if not all(match(doc, q) for q in cond):
                return False
            continue
        if not _match_cond(get_path(doc, key), cond):
            return False
    return True


def project(doc, selection):
    if not selection:
        return doc
    include = {k for k, v in selection.items() if v}
    exclude = {k for k, v in selection.items() if not v}
    if include:
        out = {}
        if "_id" not in exclude and "_id" in doc:
            out["_id"] = doc["_id"]
        for k in include:
            v = get_path(doc, k)
            if v is not _MISSING:
                set_path(out, k, v)
        return out
    out = copy.deepcopy(doc)
    for k in exclude:
        parts = k.split(".")
        cur = out
        for p in parts[:-1]:
            cur = cur.get(p, {}) if isinstance(cur, dict) else {}
        if isinstance(cur, dict):
            cur.pop(parts[-1], None)
    return out


def apply_set(doc, data):
    """Apply an update: plain dict = $set; also accepts {'$set': {...}}."""
    if "$set" in data:
        data = data["$set"]
    for k, v in data.items():
        if k == "_id":
            continue
        set_path(doc, k, copy.deepcopy(v))
    return doc
