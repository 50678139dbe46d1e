"""Property-based test of the native lease queue (SURVEY §7.3 step 1:
'property tests'): random interleavings of submit / claim / heartbeat /
complete / fail / lease expiry / device release checked against a plain
Python model of the reference's SQL semantics plus this build's fixes
(lease tokens, attempt bound, reclaim of expired leases)."""
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from llm_mcp_amd.store.memory import MemoryStore

OPS = st.lists(st.tuples(st.sampled_from(["submit", "claim", "complete", "fail", "heartbeat",
                                          "tick", "stale_complete", "release"]),
                         st.integers(0, 5), st.integers(0, 3)),
               min_size=1, max_size=60)


@settings(max_examples=150, deadline=None, suppress_health_check=[HealthCheck.too_slow])
@given(OPS)
def test_lease_queue_matches_model(ops):
    now = [1000.0]
    q = MemoryStore(clock=lambda: now[0])
    model: dict[str, dict] = {}     # id -> {status, attempts, max, lease_until, token, prio, seq}
    leases: list[tuple[str, str, str]] = []   # (job, worker, token) ever handed out
    seq = 0
    for op, a, b in ops:
        if op == "submit":
            jid = q.submit_job("echo", {"device_id": f"d{b}"} if b == 3 else {}, priority=a % 3,
                               max_attempts=1 + a % 3)
            model[jid] = {"status": "queued", "attempts": 0, "max": 1 + a % 3,
                          "lease": 0.0, "token": None, "prio": a % 3, "seq": seq,
                          "dev": f"d{b}" if b == 3 else ""}
            seq += 1
        elif op == "claim":
            j = q.claim_job(f"w{a}", [], 10, check_online=False)
            def live_on(dev, but):
                return sum(1 for k2, m2 in model.items() if k2 != but and m2["dev"] == dev
                           and m2["status"] == "running" and m2["lease"] >= now[0])
            # the claim walks queued / lease-lapsed rows by (priority, FIFO):
            # rows that exhausted max_attempts are retired ('attempts_exhausted')
            # as the walk passes them (the Postgres store retires them in its
            # maintenance sweep instead); per-device concurrency
            # (DEVICE_MAX_CONCURRENCY = 1) for pinned jobs
            best = None
            for k in sorted((k for k, m in model.items() if m["status"] in ("queued", "running")),
                            key=lambda k: (-model[k]["prio"], model[k]["seq"])):
                m = model[k]
                if m["status"] == "running" and m["lease"] >= now[0]:
                    continue
                if m["attempts"] >= m["max"]:
                    m.update(status="error", lease=0.0, token=None)
                    continue
                if m["dev"] and live_on(m["dev"], k) >= 1:
                    continue
                best = k
                break
            if best is None:
                assert j is None
                continue
            assert j is not None and j["id"] == best
            m = model[best]
            m.update(status="running", attempts=m["attempts"] + 1, lease=now[0] + 10,
                     token=j["attempt_id"])
            assert j["attempts"] == m["attempts"]
            leases.append((best, f"w{a}", j["attempt_id"]))
        elif op in ("complete", "fail", "heartbeat") and leases:
            jid, w, tok = leases[a % len(leases)]
            m = model[jid]
            owner = m["status"] == "running" and m["token"] == tok
            if op == "complete":
                assert q.complete_job(jid, w, {"ok": True}, {}, tok) == owner
                if owner:
                    m.update(status="done", lease=0.0)
            elif op == "fail":
                r = q.fail_job(jid, w, "boom", {}, tok)
                if owner:
                    m["status"] = "queued" if m["attempts"] < m["max"] else "error"
                    m.update(lease=0.0, token=None)
                    assert r == m["status"]
                else:
                    assert r is None
            else:
                assert q.heartbeat(jid, w, 10, tok) == owner
                if owner:
                    m["lease"] = now[0] + 10
        elif op == "stale_complete" and leases:
            jid, w, _ = leases[a % len(leases)]
            assert not q.complete_job(jid, w, {}, {}, "not-a-token")
        elif op == "tick":
            now[0] += 4.0 * (a + 1)
        elif op == "release":
            q.release_device_leases(f"d{b}")
            for k, m in model.items():
                if m["status"] == "running" and q.get_job(k)["device_id"] == f"d{b}":
                    m["lease"] = 0.0
        # invariants
        for k, m in model.items():
            got = q.get_job(k)
            if m["status"] == "queued" and m["attempts"] >= m["max"]:
                assert got["status"] in ("queued", "error")   # swept at next claim
            elif m["status"] == "running" and m["lease"] < now[0] and m["attempts"] >= m["max"]:
                # expired with no attempt left: a claim may sweep it to error
                assert got["status"] in ("running", "error")
                if got["status"] == "error":
                    m.update(status="error", token=None)
            else:
                assert got["status"] == m["status"], (k, got, m)
            assert got["attempts"] == m["attempts"]
