"""One job-store contract, run against every backend: the native MemoryStore
always, the PostgresStore when a server is reachable (``LMX_TEST_PG_DSN``,
e.g. postgres://lmx:pw@127.0.0.1:5432/lmx_test -- there is no Postgres in
this image, so that leg is skipped here and Postgres parity with the
reference's claim (core/internal/api/handlers.go:173-293) stays unpinned
until a server runs it; tests/test_pgwire.py pins the statements sent).

Covered: no double claim under concurrent claimers, expired-lease reclaim
(and the old lease token losing ownership), the attempts bound, priority
then FIFO order, per-device concurrency, deadline filtering + the
maintenance sweep."""
import os
import threading
import time

import pytest

BACKENDS = ["memory", "postgres"]


@pytest.fixture(params=BACKENDS)
def store(request):
    if request.param == "memory":
        from llm_mcp_amd.store.memory import MemoryStore
        yield MemoryStore()
        return
    dsn = os.environ.get("LMX_TEST_PG_DSN", "")
    if not dsn:
        pytest.skip("no Postgres server (set LMX_TEST_PG_DSN): Postgres parity unpinned")
    from llm_mcp_amd.store.postgres import PostgresStore
    st = PostgresStore(dsn)
    st._n("DELETE FROM job_attempts")
    st._n("DELETE FROM jobs")
    yield st
    st.close()


def _kind(tag):
    return f"contract.{tag}.{os.getpid()}.{time.time_ns()}"


def test_no_double_claim_under_concurrency(store):
    kind = _kind("race")
    ids = {store.submit_job(kind, {"i": i}) for i in range(40)}
    got, lock = [], threading.Lock()

    def worker(w):
        while True:
            j = store.claim_job(f"w{w}", [kind], 60)
            if j is None:
                return
            with lock:
                got.append(j["id"])

    ts = [threading.Thread(target=worker, args=(w,)) for w in range(8)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert sorted(got) == sorted(ids)          # every job exactly once


def test_expired_lease_is_reclaimed_and_old_token_loses(store):
    kind = _kind("lease")
    jid = store.submit_job(kind, {})
    a = store.claim_job("w1", [kind], 1)
    assert a["id"] == jid and store.claim_job("w2", [kind], 1) is None
    time.sleep(1.3)
    b = store.claim_job("w2", [kind], 60)
    assert b is not None and b["id"] == jid and b["attempts"] == 2
    assert not store.complete_job(jid, "w1", {"ok": 1}, {}, token=a["attempt_id"])
    assert not store.heartbeat(jid, "w1", 30, token=a["attempt_id"])
    assert store.heartbeat(jid, "w2", 30, token=b["attempt_id"])
    assert store.complete_job(jid, "w2", {"ok": 2}, {}, token=b["attempt_id"])
    j = store.get_job(jid)
    assert j["status"] == "done" and j["result"] == {"ok": 2}


def test_attempts_bound(store):
    kind = _kind("attempts")
    jid = store.submit_job(kind, {}, max_attempts=2)
    a = store.claim_job("w", [kind], 60)
    assert store.fail_job(jid, "w", "boom", {}, token=a["attempt_id"]) == "queued"
    b = store.claim_job("w", [kind], 60)
    assert store.fail_job(jid, "w", "boom", {}, token=b["attempt_id"]) == "error"
    assert store.claim_job("w", [kind], 60) is None
    j = store.get_job(jid)
    assert j["status"] == "error" and j["attempts"] == 2


def test_lapsed_final_attempt_is_retired(store):
    kind = _kind("lapse")
    jid = store.submit_job(kind, {}, max_attempts=1)
    assert store.claim_job("w", [kind], 1)["id"] == jid
    time.sleep(1.3)
    assert store.claim_job("w", [kind], 60) is None      # attempts exhausted
    store.sweep_exhausted()
    j = store.get_job(jid)
    assert j["status"] == "error" and "attempts" in (j["error"] or ""), j


def test_priority_then_fifo(store):
    kind = _kind("order")
    low1 = store.submit_job(kind, {}, priority=0)
    time.sleep(0.01)
    high = store.submit_job(kind, {}, priority=5)
    time.sleep(0.01)
    low2 = store.submit_job(kind, {}, priority=0)
    order = [store.claim_job("w", [kind], 60)["id"] for _ in range(3)]
    assert order == [high, low1, low2]


def test_device_concurrency(store):
    kind = _kind("dev")
    dev = f"node-{os.getpid()}:gpu0"
    store.upsert_device(dev, status="online")
    j1 = store.submit_job(kind, {"device_id": dev})
    j2 = store.submit_job(kind, {"device_id": dev})
    a = store.claim_job("w", [kind], 60, worker_device=dev, device_max_concurrency=1)
    assert a["id"] == j1
    assert store.claim_job("w", [kind], 60, worker_device=dev, device_max_concurrency=1) is None
    assert store.complete_job(j1, "w", {}, {}, token=a["attempt_id"])
    b = store.claim_job("w", [kind], 60, worker_device=dev, device_max_concurrency=1)
    assert b["id"] == j2


def test_deadline_filtered_and_swept(store):
    kind = _kind("deadline")
    jid = store.submit_job(kind, {}, deadline_at=time.time() - 5)
    assert store.claim_job("w", [kind], 60) is None
    store.expire_deadlines()
    j = store.get_job(jid)
    assert j["status"] == "error" and "deadline" in (j["error"] or "")


def test_requeued_job_is_not_stuck_on_its_failed_device(store):
    """A claim records where the job runs (device_id), but only the
    submitter's pin restricts placement: after a failure or a lapsed lease
    the job goes to another device, while a pinned job stays on its pin."""
    kind = _kind("move")
    a_dev, b_dev = f"n{os.getpid()}:gpu0.r1", f"n{os.getpid()}:gpu0"
    for d in (a_dev, b_dev):
        store.upsert_device(d, status="online")
    free = store.submit_job(kind, {})
    a = store.claim_job("wa", [kind], 60, worker_device=a_dev)
    assert a["id"] == free and store.get_job(free)["device_id"] == a_dev
    assert store.fail_job(free, "wa", "HIP error", {}, token=a["attempt_id"]) == "queued"
    b = store.claim_job("wb", [kind], 60, worker_device=b_dev)
    assert b is not None and b["id"] == free and store.get_job(free)["device_id"] == b_dev
    # lease lapse on b: c on a_dev takes it over
    store.complete_job(free, "wb", {}, {}, token=b["attempt_id"])
    lapsing = store.submit_job(kind, {})
    assert store.claim_job("wb", [kind], 1, worker_device=b_dev)["id"] == lapsing
    time.sleep(1.3)
    c = store.claim_job("wa", [kind], 60, worker_device=a_dev)
    assert c is not None and c["id"] == lapsing
    assert store.complete_job(lapsing, "wa", {}, {}, token=c["attempt_id"])
    # pinned: never moves
    pinned = store.submit_job(kind, {"device_id": a_dev})
    p = store.claim_job("wa", [kind], 60, worker_device=a_dev)
    assert p["id"] == pinned
    assert store.fail_job(pinned, "wa", "boom", {}, token=p["attempt_id"]) == "queued"
    assert store.claim_job("wb", [kind], 60, worker_device=b_dev) is None
