"""In-tree Postgres client against a protocol-level fake server, and the
Postgres store's claim/complete statement wiring.

No Postgres server exists in this image, so the SQL *semantics* of
store/postgres.py (SKIP LOCKED claim, triggers, views) are parity-unpinned
here; what is pinned is the wire protocol (auth, framing, parameter
encoding, type decoding, errors, LISTEN/NOTIFY) and that every store call
sends well-formed parameterised statements and maps rows back to the same
dict shapes MemoryStore returns."""
import json
import time

import pytest

from llm_mcp_amd.store.pgwire import Connection, PGError, Pool, encode_param, parse_dsn
from tests.pg_fake import FakePG

OIDS = {"int": 23, "float": 701, "bool": 16, "json": 3802, "ts": 1184, "text": 25, "arr": 1009}


def _typed(sql, params):
    if "SELECT typed" in sql:
        cols = [("i", OIDS["int"]), ("f", OIDS["float"]), ("b", OIDS["bool"]),
                ("j", OIDS["json"]), ("t", OIDS["ts"]), ("s", OIDS["text"]), ("a", OIDS["arr"]),
                ("n", OIDS["text"])]
        return cols, [[7, 2.5, "t", '{"x": [1, 2]}', "2026-05-01 12:00:00.5+00", "héllo",
                       '{a,"b,c",NULL}', None]], "SELECT 1"
    if "boom" in sql:
        raise ValueError("relation boom does not exist")
    if sql.startswith("SELECT $1"):
        return [("v", OIDS["text"])], [[params[0]]], "SELECT 1"
    return [], [], "OK"


@pytest.mark.parametrize("auth", ["md5", "scram", "trust"])
def test_auth_and_types(auth):
    srv = FakePG(_typed, auth=auth)
    try:
        c = Connection(srv.dsn)
        r = c.one("SELECT typed")
        assert r["i"] == 7 and r["f"] == 2.5 and r["b"] is True
        assert r["j"] == {"x": [1, 2]} and r["s"] == "héllo" and r["n"] is None
        assert abs(r["t"] - 1777636800.5) < 1e-6
        assert r["a"] == ["a", "b,c", None]
        assert c.scalar("SELECT $1", {"k": 1}) == '{"k": 1}'
        with pytest.raises(PGError) as ei:
            c.query("SELECT boom")
        assert ei.value.code == "42000"
        assert c.scalar("SELECT $1", "still alive") == "still alive"
        c.close()
    finally:
        srv.close()


def test_bad_password_rejected():
    srv = FakePG(_typed, auth="scram")
    try:
        with pytest.raises(PGError):
            Connection(srv.dsn.replace(":pw@", ":nope@"))
    finally:
        srv.close()


def test_listen_notify_and_pool():
    srv = FakePG(_typed, auth="md5")
    try:
        c = Connection(srv.dsn)
        c.listen("job_update")
        assert c.wait_notify(0.05) == []
        srv.notify("job_update", "abc")
        got = c.wait_notify(2.0)
        assert got == [("job_update", "abc")]
        pool = Pool(srv.dsn, size=2)
        with pool.conn() as a, pool.conn() as b:
            assert a is not b
        with pool.conn() as a2:
            assert a2 in (a, b)
        pool.close()
        c.close()
    finally:
        srv.close()


def test_param_encoding_and_dsn():
    assert encode_param(None) is None
    assert encode_param(True) == b"t"
    assert encode_param(["a", 'q"t', None]) == b'{"a","q\\"t",NULL}'
    assert json.loads(encode_param({"a": 1})) == {"a": 1}
    d = parse_dsn("postgres://u:p%40ss@db:5433/core?sslmode=disable")
    assert (d["user"], d["password"], d["host"], d["port"], d["database"]) == \
        ("u", "p@ss", "db", 5433, "core")


class _StoreHandler:
    """Answers the statements PostgresStore issues with canned rows."""

    JOB = [("id", 25), ("kind", 25), ("payload", 3802), ("status", 25), ("attempts", 23),
           ("max_attempts", 23), ("lease_until", 1184), ("deadline_at", 1184), ("result", 3802),
           ("error", 25), ("priority", 23), ("queued_at", 1184), ("updated_at", 1184),
           ("source", 25), ("device_id", 25), ("worker_id", 25)]

    def __init__(self):
        self.seen = []

    def __call__(self, sql, params):
        self.seen.append((sql, params))
        s = " ".join(sql.split())
        if s.startswith("INSERT INTO jobs"):
            return [("id", 25)], [["0b7f8c2e-0000-4000-8000-000000000001"]], "INSERT 0 1"
        if "WITH running_per_device" in s:
            row = ["0b7f8c2e-0000-4000-8000-000000000001", "engine.generate",
                   '{"model": "llama-3-8b"}', "running", 1, 3, "2026-05-01 12:01:00+00", None,
                   None, None, 0, "2026-05-01 12:00:00+00", "2026-05-01 12:00:00+00", "api",
                   "n:gpu0", "w1", "11111111-2222-4333-8444-555555555555"]
            return self.JOB + [("attempt_id", 25)], [row], "UPDATE 1"
        if "FROM devices WHERE tags ? 'capacity'" in s:
            return [("id", 25), ("cap", 23)], [["n:gpu0", 256]], "SELECT 1"
        if s.startswith("UPDATE jobs SET status = 'done'"):
            return [("tok", 25)], [["11111111-2222-4333-8444-555555555555"]], "UPDATE 1"
        if s.startswith("SELECT status, COUNT(*)"):
            return [("status", 25), ("n", 23)], [["running", 1], ["queued", 4]], "SELECT 2"
        return [], [], "OK"


def test_postgres_store_statement_wiring():
    from llm_mcp_amd.store.postgres import PostgresStore
    h = _StoreHandler()
    srv = FakePG(h, auth="md5")
    try:
        st = PostgresStore(srv.dsn)
        assert any("CREATE TABLE IF NOT EXISTS jobs" in q for q, _ in h.seen)   # migration ran
        jid = st.submit_job("engine.generate", {"model": "llama-3-8b", "device_id": "n:gpu0"},
                            priority=2, source="api", deadline_at=1777636800.0)
        assert jid.startswith("0b7f8c2e")
        sql, p = next(x for x in h.seen if x[0].startswith("INSERT INTO jobs"))
        assert json.loads(p[1]) == {"model": "llama-3-8b", "device_id": "n:gpu0"}
        assert p[2] == "2" and p[7] == "n:gpu0"
        j = st.claim_job("w1", ["engine.generate"], 60, worker_device="n:gpu0")
        assert j["status"] == "running" and j["payload"]["model"] == "llama-3-8b"
        assert j["attempt_id"].startswith("11111111") and j["queued_at"] == 1777636800.0
        sql, p = next(x for x in h.seen if "WITH running_per_device" in x[0])
        assert "FOR UPDATE OF j SKIP LOCKED" in sql
        assert p[1] == '{"engine.generate"}' and json.loads(p[5]) == {"n:gpu0": 256}
        assert any(q.startswith("INSERT INTO job_attempts") for q, _ in h.seen)
        # the claim transaction takes no row locks outside SKIP LOCKED: the
        # deadline / attempts sweeps moved to the maintenance loop
        assert not any("deadline_exceeded" in q or "attempts_exhausted" in q for q, _ in h.seen)
        assert "deadline_at >= now()" in sql
        st.expire_deadlines()
        st.sweep_exhausted()
        sweeps = [q for q, _ in h.seen if "deadline_exceeded" in q or "attempts_exhausted" in q]
        assert len(sweeps) == 2 and all("FOR UPDATE SKIP LOCKED" in q for q in sweeps)
        assert st.complete_job(jid, "w1", {"ok": True}, {"ms": 5}, token=j["attempt_id"])
        assert st.job_counts() == {"queued": 4, "running": 1, "done": 0, "error": 0}
        v = st.job_version()
        srv.notify("job_update", jid)
        assert st.wait_job_change(v, 3.0) > v
        st.close()
    finally:
        srv.close()
