"""MongoDB backend paths that need no server (reference tests/unittests/core/mongodb_test.py:
connection failure, exception normalisation, URI handling).  CRUD against a live mongod is
parity-unpinned here: no server exists on either box."""
import pymongo
import pytest
from pymongo import errors as perr

from orion_amd.store import Database, DatabaseError, DuplicateKeyError
from orion_amd.store.mongodb import MongoDB, mongodb_exception_wrapper


def test_unresolvable_host_is_a_connection_database_error():
    with pytest.raises(DatabaseError, match="Connection"):
        MongoDB(host="asdfada.invalid", port=123, name="orion", username="u", password="p",
                serverSelectionTimeoutMS=1)


def test_unwrapped_method_raises_raw_pymongo_error(monkeypatch):
    monkeypatch.setattr(MongoDB, "initiate_connection", MongoDB.initiate_connection.__wrapped__)
    with pytest.raises(perr.ConnectionFailure):
        MongoDB(host="asdfada.invalid", port=123, serverSelectionTimeoutMS=1)


def _raising(exc):
    @mongodb_exception_wrapper
    def f():
        raise exc
    return f


@pytest.mark.parametrize("exc,kind,text", [
    (perr.DuplicateKeyError("E11000 duplicate key"), DuplicateKeyError, "duplicate"),
    (perr.BulkWriteError({"writeErrors": [{"code": 11000, "errmsg": "dup"}]}), DuplicateKeyError, None),
    (perr.BulkWriteError({"writeErrors": [{"code": 121, "errmsg": "validation"}]}), DatabaseError, None),
    (perr.OperationFailure("Authentication failed.", code=18), DatabaseError, "Authentication"),
    (perr.OperationFailure("not authorized", code=13), DatabaseError, "not authorized"),
    (perr.ServerSelectionTimeoutError("no servers"), DatabaseError, "Connection"),
])
def test_exception_normalisation(exc, kind, text):
    with pytest.raises(kind, match=text) as info:
        _raising(exc)()
    assert info.type is kind
    assert isinstance(info.value.__cause__, perr.PyMongoError)


def test_uri_is_parsed():
    db = MongoDB("mongodb://user:pass@localhost/orion_test", check_connection=False)
    assert (db.host, db.port, db.username, db.password, db.name) == \
        ("localhost", 27017, "user", "pass", "orion_test")


def test_explicit_fields_override_uri():
    db = MongoDB("mongodb://lala:pass@localhost:1231/orion", port=27017, name="orion_test",
                 username="user", password="pass", check_connection=False)
    assert (db.host, db.port, db.username, db.password, db.name) == \
        ("localhost", 27017, "user", "pass", "orion_test")


def test_factory_name_and_defaults():
    db = Database("mongodb", check_connection=False)
    assert isinstance(db, MongoDB) and (db.host, db.port, db.name) == ("localhost", 27017, "orion")


class _Coll:
    """Records the pymongo calls the backend makes (the CRUD mapping, not the server)."""

    def __init__(self):
        self.calls = []

    def insert_many(self, docs):
        self.calls.append(("insert_many", docs))
        return type("R", (), {"inserted_ids": [1] * len(docs)})()

    def update_many(self, q, upd, upsert):
        self.calls.append(("update_many", q, upd, upsert))
        return type("R", (), {"modified_count": 2, "upserted_id": None})()

    def find_one_and_update(self, q, upd, projection, return_document):
        self.calls.append(("find_one_and_update", q, upd, return_document))
        return {"_id": 1}

    def count_documents(self, q):
        self.calls.append(("count_documents", q))
        return 7


def test_crud_mapping():
    db = MongoDB(check_connection=False)
    coll = _Coll()
    db._db = {"trials": coll}
    assert db.write("trials", [{"a": 1}, {"a": 2}]) == 2
    assert db.write("trials", {"status": "done"}, {"_id": 3}) == 2
    assert db.read_and_write("trials", {"_id": 1, "status": "new"}, {"status": "reserved"}) == {"_id": 1}
    assert db.count("trials", {"status": "new"}) == 7
    kinds = [c[0] for c in coll.calls]
    assert kinds == ["insert_many", "update_many", "find_one_and_update", "count_documents"]
    assert coll.calls[1][2] == {"$set": {"status": "done"}} and coll.calls[1][3] is True
    assert coll.calls[2][3] == pymongo.ReturnDocument.AFTER
