"""Lookahead (one-step asynchronous) stepping of the native scheduler.

The engine's GPU path launches step n+1 before it reads step n's tokens
(engine.LLMEngine._step_la): ``update_lookahead()`` consumes a launched plan
with placeholder tokens, the next plan names the rows that read them
(``input_src``), ``patch()`` fills them and reports stop-token finishes one
step late.  Driven here by a deterministic "model" whose sample depends on the
sequence, its context length and the row's INPUT token, the lookahead protocol
must produce exactly the token streams and finish reasons of the synchronous
``update()`` protocol -- through stop tokens, length limits, preemption by a
small KV cache, aborts and late arrivals -- and return every KV page."""
import numpy as np
import pytest

from llm_mcp_amd.native import runtime

STOP = 7


def model(plan, ids):
    """Token sampled for each sample row: a hash of (sequence, context, input
    token of the sampled row); STOP about once in 23 draws."""
    out = []
    for i, row in enumerate(plan["sample_rows"]):
        sid = int(plan["seq_ids"][plan["sample_seq"][i]])
        ctx = int(plan["positions"][row]) + 1
        h = (sid * 1000003 + ctx * 7919 + int(ids[row]) * 104729) % 2311
        out.append(STOP if h % 23 == 0 else 10 + h % 500)
    return np.asarray(out, np.int32)


def make(num_blocks):
    return runtime().Scheduler(num_blocks, 16, 8, 96, 512, True)


def script():
    """(step, action, args): arrivals over time and two aborts."""
    rng = np.random.default_rng(3)
    ev = []
    for j in range(14):
        plen = int(rng.integers(3, 70))
        prompt = [int(x) for x in rng.integers(20, 900, plen)]
        ev.append((int(rng.integers(0, 30)), "add", (100 + j, prompt, int(rng.integers(1, 40)),
                                                     bool(j % 5 == 0))))
    ev.append((9, "abort", (103,)))
    ev.append((17, "abort", (110,)))
    return ev


def collect(plan, toks, outs, finished):
    for i in range(len(plan["sample_rows"])):
        sid = int(plan["seq_ids"][plan["sample_seq"][i]])
        if sid in finished:       # a sample of an already finished sequence: dropped
            continue
        outs.setdefault(sid, []).append(int(toks[i]))


def run_sync(num_blocks):
    s, ev = make(num_blocks), script()
    outs, finished = {}, {}
    for step in range(400):
        for st, kind, args in ev:
            if st == step:
                if kind == "add":
                    sid, prompt, mx, ign = args
                    s.add(sid, prompt, mx, [STOP], ign, 0)
                elif s.abort(args[0]):
                    finished[args[0]] = "abort"
        if not s.has_work and step > 30:
            break
        plan = s.schedule(16)
        if plan["num_tokens"] == 0:
            continue
        assert plan["num_pending_inputs"] == 0
        toks = model(plan, plan["input_ids"])
        collect(plan, toks, outs, finished)
        for sid, r in s.update(toks):
            finished[sid] = r
    return outs, finished, s


def run_lookahead(num_blocks):
    s, ev = make(num_blocks), script()
    outs, finished = {}, {}
    la = None                     # (plan, toks) launched, not yet read back
    for step in range(400):
        for st, kind, args in ev:
            if st == step:
                if kind == "add":
                    sid, prompt, mx, ign = args
                    s.add(sid, prompt, mx, [STOP], ign, 0)
                elif s.abort(args[0]):
                    finished[args[0]] = "abort"
        if not s.has_work and la is None and step > 30:
            break
        if la is not None:
            s.update_lookahead()
        plan = s.schedule(16)
        if plan["num_tokens"] == 0:
            if la is not None:
                fin = s.patch(la[1])
                collect(la[0], la[1], outs, finished)
                finished.update(dict(fin))
                la = None
            continue
        ids = plan["input_ids"].copy()
        src = plan["input_src"]
        if la is not None:
            m = src >= 0
            ids[m] = la[1][src[m]]        # the device-side gather of ids_from_prev
        else:
            assert (src < 0).all()
        toks = model(plan, ids)
        if la is not None:                # read back step n after launching n+1
            fin = s.patch(la[1])
            collect(la[0], la[1], outs, finished)
            finished.update(dict(fin))
        la = (plan, toks)
    return outs, finished, s


@pytest.mark.parametrize("num_blocks", [200, 14])
def test_lookahead_matches_synchronous_protocol(num_blocks):
    o1, f1, s1 = run_sync(num_blocks)
    o2, f2, s2 = run_lookahead(num_blocks)
    aborted = {103, 110}
    # an abort lands one step later in the lookahead protocol (the launched
    # step's sample of the aborted sequence is dropped): prefix, not equality
    for sid in aborted:
        a, b = o1.get(sid, []), o2.get(sid, [])
        assert b == a[:len(b)] and len(a) - len(b) <= 1, (sid, a, b)
    assert {k: v for k, v in f1.items() if k not in aborted} == \
        {k: v for k, v in f2.items() if k not in aborted}
    assert {k: v for k, v in o1.items() if k not in aborted} == \
        {k: v for k, v in o2.items() if k not in aborted}
    assert len(f1) == len(f2) == 14
    assert 1 in f1.values() and 2 in f1.values()      # stop and length finishes both seen
    for s in (s1, s2):
        assert not s.has_work
        assert s.kv_usage == 0.0                  # every page back (free or cached)
        assert s.num_inflight_samples == 0
    if num_blocks == 14:
        assert s1.preemptions > 0 and s2.preemptions > 0


def test_discard_lookahead_releases_state():
    s = make(64)
    s.add(1, list(range(20, 40)), 10, [STOP], False, 0)
    plan = s.schedule(16)
    assert plan["num_tokens"] == 20
    s.update_lookahead()
    assert s.num_inflight_samples == 1
    plan = s.schedule(16)
    assert plan["num_pending_inputs"] == 1 and list(plan["input_src"]) == [0]
    s.discard_lookahead()
    assert s.num_inflight_samples == 0
    assert s.abort(1)
    assert not s.has_work


def test_stop_in_flight_makes_a_zombie_row():
    """A sequence that samples STOP at step n is already in step n+1's plan:
    patch() finishes it, update_lookahead() of n+1 drops its extra sample and
    frees the object; abort of it in between is refused."""
    s = make(64)
    s.add(1, [11, 12, 13], 10, [STOP], False, 0)
    s.add(2, [21, 22, 23], 10, [STOP], False, 0)
    p0 = s.schedule(16)
    s.update_lookahead()
    p1 = s.schedule(16)
    assert list(p1["input_src"]) == [0, 1]
    fin = s.patch(np.asarray([STOP, 50], np.int32))
    assert fin == [(1, 1)]
    assert not s.abort(1)                 # finished, still referenced by plan 1
    s.update_lookahead()                  # sequence 1's extra sample dropped
    p2 = s.schedule(16)
    assert list(p2["seq_ids"]) == [2] and list(p2["input_src"]) == [1]
    assert s.patch(np.asarray([0, 60], np.int32)) == []
    assert p0["num_tokens"] == 6


def test_stop_of_a_preempted_sequence_leaves_the_waiting_queue():
    """the plan after a sampled step can preempt a sequence
    whose in-flight sample turns out to be STOP.  patch() must take it out of
    the waiting queue before freeing it, or the next schedule() reads a freed
    Seq.  3 pages of 16: both 16-token prompts fill a page each, the decode
    step needs a second page for each and only one is free, so sequence 2
    (running_.back()) preempts itself."""
    s = make(3)
    s.add(1, list(range(100, 116)), 10, [STOP], False, 0)
    s.add(2, list(range(200, 216)), 10, [STOP], False, 0)
    p0 = s.schedule(16)
    assert p0["num_tokens"] == 32
    s.update_lookahead()
    p1 = s.schedule(16)
    assert list(p1["seq_ids"]) == [1] and list(p1["preempted"]) == [2]
    fin = s.patch(np.asarray([50, STOP], np.int32))
    assert fin == [(2, 1)]
    s.update_lookahead()                  # consumes p1 (sequence 1 only)
    p2 = s.schedule(16)
    assert list(p2["seq_ids"]) == [1]     # the freed sequence 2 is gone from every queue
    assert s.patch(np.asarray([60], np.int32)) == []
    s.discard_lookahead()
    assert s.abort(1)
    assert not s.has_work
    assert s.kv_usage == 0.0


def test_mixed_step_prefill_cap():
    """With >= min_decodes decode rows running, a step's prompt tokens are
    capped (set_mixed_prefill_cap), so a long prompt arriving mid-stream is
    split into capped chunks instead of stalling every decoding stream for a
    max_batched_tokens step; an idle engine (no decode rows) still takes the
    full budget."""
    s = runtime().Scheduler(4096, 32, 64, 4096, 8192, False)
    s.set_mixed_prefill_cap(256, 4)
    for i in range(8):
        s.add(i, [10 + i] * 40, 50, [], True, 0)
    p = s.schedule(16)
    assert p["num_decode"] == 0 and p["num_tokens"] == 8 * 40       # burst: full budget
    s.update(np.full(len(p["sample_rows"]), 11, np.int32))
    s.add(100, list(range(20, 1020)), 10, [], True, 0)             # a 1000-token prompt
    steps = []
    while True:
        p = s.schedule(16)
        steps.append((p["num_decode"], p["num_tokens"] - p["num_decode"]))
        s.update(np.full(len(p["sample_rows"]), 11, np.int32))
        if steps[-1][1] == 0:
            break
    assert [pf for _, pf in steps[:-1]] == [256, 256, 256, 232]
    assert all(nd >= 8 for nd, _ in steps)                          # the decodes keep running
    # below min_decodes the cap does not apply
    s2 = runtime().Scheduler(4096, 32, 64, 4096, 8192, False)
    s2.set_mixed_prefill_cap(256, 16)
    for i in range(8):
        s2.add(i, [10 + i] * 40, 50, [], True, 0)
    p = s2.schedule(16)
    s2.update(np.full(len(p["sample_rows"]), 11, np.int32))
    s2.add(100, list(range(20, 1020)), 10, [], True, 0)
    p = s2.schedule(16)
    assert p["num_tokens"] - p["num_decode"] == 1000


def test_block_manager_hands_out_lowest_free_pages():
    """KV pages come from a min-heap: a prompt's pages are one ascending run and a
    new wave reuses the lowest freed pages, in order (block_manager.h)."""
    bm = runtime().BlockManager(64, 16, False)
    assert bm.ensure(1, 16 * 5) and bm.ensure(2, 16 * 3)
    assert list(bm.table(1)) == [0, 1, 2, 3, 4] and list(bm.table(2)) == [5, 6, 7]
    bm.free_seq(1)
    assert bm.ensure(3, 16 * 6)
    assert list(bm.table(3)) == [0, 1, 2, 3, 4, 8]
    bm.free_seq(2)
    bm.free_seq(3)
    assert bm.ensure(4, 16 * 9)
    assert list(bm.table(4)) == list(range(9))
    assert bm.num_free == 64 - 9
