"""Engine (paged KV, continuous batching, chunked prefill, prefix cache) on the
CPU reference ops against a dense full-recompute forward."""
import torch

from llm_mcp_amd.engine.engine import EngineConfig, LLMEngine, SamplingParams
from tests.dense_ref import assert_greedy_consistent, dense_logits


def _engine(**kw):
    cfg = dict(model="tiny-llama", max_num_seqs=8, max_batched_tokens=64, max_model_len=512,
               use_graphs=False, kv_cache_gb=None)
    cfg.update(kw)
    return LLMEngine(EngineConfig(**cfg), device="cpu")


def test_greedy_matches_dense_reference():
    e = _engine()
    prompts = [list(range(10, 50)), list(range(5, 100)), [7] * 33, [3]]
    outs = e.generate(prompts, SamplingParams(temperature=0, max_tokens=6, ignore_eos=True))
    for p, o in zip(prompts, outs):
        assert len(o) == 6
        assert_greedy_consistent(e.model, p, o)


def test_chunked_prefill_and_prefix_cache_consistent():
    # token budget 64 forces chunked prefill of the 95-token prompt
    e = _engine(max_batched_tokens=40)
    p = list(range(1, 96))
    a = e.generate([p], SamplingParams(temperature=0, max_tokens=4, ignore_eos=True))[0]
    # second request with the same prefix reuses cached pages
    b = e.generate([p], SamplingParams(temperature=0, max_tokens=4, ignore_eos=True))[0]
    assert a == b
    assert_greedy_consistent(e.model, p, a)
    assert e.sched.prefix_hits > 0


def test_prefix_cache_switch(monkeypatch):
    """LMX_PREFIX_CACHE=0: finished pages go straight back to the free list, a
    repeated prompt is recomputed (no hits) and gives the same tokens."""
    monkeypatch.setenv("LMX_PREFIX_CACHE", "0")
    assert EngineConfig().prefix_cache is False
    e = _engine(max_batched_tokens=40)
    p = list(range(1, 96))
    a = e.generate([p], SamplingParams(temperature=0, max_tokens=4, ignore_eos=True))[0]
    b = e.generate([p], SamplingParams(temperature=0, max_tokens=4, ignore_eos=True))[0]
    assert a == b and e.sched.prefix_hits == 0
    monkeypatch.setenv("LMX_PREFIX_CACHE", "1")
    assert EngineConfig().prefix_cache is True


def test_preemption_recompute_keeps_outputs():
    # tiny KV: 16 blocks x 32 tokens; 4 sequences of ~120 tokens cannot all fit
    e = _engine(kv_cache_gb=None)
    e2 = LLMEngine(EngineConfig(model="tiny-llama", max_num_seqs=8, max_batched_tokens=512,
                                max_model_len=512, use_graphs=False, kv_cache_gb=16 * 2 * 2 * 2
                                * 32 * 128 * 2 / (1 << 30)), device="cpu", weights=e.model.w)
    assert e2.num_blocks == 16
    prompts = [list(range(i, i + 100)) for i in range(4)]
    sp = SamplingParams(temperature=0, max_tokens=30, ignore_eos=True)
    outs = e2.generate(prompts, sp)
    assert e2.sched.preemptions > 0
    for p, o in zip(prompts, outs):
        assert len(o) == 30
        assert_greedy_consistent(e2.model, p, o)


def test_logits_close_to_dense():
    e = _engine()
    p = list(range(20, 60))
    from llm_mcp_amd.models.llama import StepInputs
    import numpy as np
    e.sched.add(999, p, 1, [], True, 0)
    plan = e.sched.schedule(e.q_per_tile)
    S = len(plan["seq_ids"])
    t = lambda a, dt=torch.int32: torch.as_tensor(np.asarray(a), dtype=dt)
    inp = StepInputs(t(plan["input_ids"]), t(plan["positions"]), t(plan["slots"]),
                     plan["num_decode"], t(plan["block_tables"]).view(S, -1),
                     t(plan["context_lens"]), t(plan["cu_q"]), t(plan["prefill_tiles"]),
                     t(plan["sample_rows"], torch.int64), plan["num_tokens"], S)
    logits = e.model.forward(inp, e.k_caches, e.v_caches, None)
    ref = dense_logits(e.model, p)
    assert torch.allclose(logits[0].float(), ref, atol=5e-2, rtol=5e-2)


def test_qwen2_biased_qkv_group7_matches_dense():
    """Qwen2-style model: biased q/k/v and a GQA group of 7 (not a divisor of
    16) through the engine vs the dense fp32 reference."""
    e = _engine(model="tiny-qwen")
    assert e.cfg.qkv_bias and e.Hq // e.Hkv == 7
    prompts = [list(range(10, 50)), [7] * 33, [3]]
    outs = e.generate(prompts, SamplingParams(temperature=0, max_tokens=5, ignore_eos=True))
    for p, o in zip(prompts, outs):
        assert len(o) == 5
        assert_greedy_consistent(e.model, p, o)


def test_qwen3_qk_norm_matches_dense():
    """Qwen3-style model: per-head q/k RMSNorm before RoPE and
    num_heads * head_dim (512) != hidden (256), vs the dense fp32 reference."""
    e = _engine(model="tiny-qwen3")
    assert e.cfg.qk_norm and e.Hq * e.D != e.cfg.hidden_size
    assert "q_norm" in e.model.w["layers"][0]
    prompts = [list(range(10, 50)), [7] * 33, [3]]
    outs = e.generate(prompts, SamplingParams(temperature=0, max_tokens=5, ignore_eos=True))
    for p, o in zip(prompts, outs):
        assert len(o) == 5
        assert_greedy_consistent(e.model, p, o)


def test_waiting_sequences_do_not_pin_prefix_pages():
    """Regression: preempted sequences sharing a cached prefix used to keep the
    pages matched at (failed) re-admission, filling the KV cache with waiting
    sequences and admitting nobody -- every request stalled forever."""
    import threading
    e = LLMEngine(EngineConfig(model="tiny-llama", max_num_seqs=16, max_batched_tokens=2048,
                               max_model_len=1024, use_graphs=False), device="cpu")
    assert e.num_blocks == 64
    shared = list(range(100, 140))
    prompts = [shared + [200 + i, 300 + i] for i in range(8)]
    out = {}
    t = threading.Thread(target=lambda: out.setdefault("o", e.generate(
        prompts, SamplingParams(temperature=0.7, max_tokens=300, ignore_eos=True, seed=3))),
        daemon=True)
    t.start()
    t.join(timeout=240)
    assert not t.is_alive(), (e.sched.num_running, e.sched.num_waiting, e.sched.kv_usage)
    assert [len(o) for o in out["o"]] == [300] * 8
    assert e.sched.preemptions > 0


def test_lookahead_stepping_matches_synchronous(monkeypatch):
    """Lookahead stepping (engine._step_la: step n+1 scheduled before step n's
    tokens are read; forced on here, the GPU default) gives the synchronous
    engine's tokens: seeded sampling, stop tokens seen one step late,
    preemption by a 16-page KV cache, ragged prompt lengths."""
    monkeypatch.setenv("LMX_LOOKAHEAD", "0")
    base = _engine()
    kv = 16 * 2 * 2 * 2 * 32 * 128 * 2 / (1 << 30)
    prompts = [list(range(i, i + 20 + 17 * i)) for i in range(6)]

    def run(la, stops):
        monkeypatch.setenv("LMX_LOOKAHEAD", la)
        e = LLMEngine(EngineConfig(model="tiny-llama", max_num_seqs=8, max_batched_tokens=96,
                                   max_model_len=512, use_graphs=False, kv_cache_gb=kv),
                      device="cpu", weights=base.model.w)
        assert e.lookahead == (la == "1")
        sp = SamplingParams(temperature=0.9, top_p=0.9, max_tokens=24, seed=5,
                            stop_token_ids=stops)
        out = e.generate(prompts, sp)
        assert not e.sched.has_work
        return out, e.sched.preemptions

    free, pre0 = run("0", [])
    free_la, pre1 = run("1", [])
    assert free_la == free and pre0 > 0 and pre1 > 0   # through preemption
    stops = [free[0][4], free[3][9]]           # tokens the streams do sample
    sync, _ = run("0", stops)
    ahead, _ = run("1", stops)
    assert ahead == sync
    assert any(len(o) < 24 for o in ahead)     # streams ended on a stop token


def test_lookahead_abort_and_late_arrivals(monkeypatch):
    """Lookahead stepping with an abort of a running request (its in-flight
    row becomes a dropped sample), a request arriving while a step is in
    flight, and the engine draining to idle: every other stream completes
    with its full token count and exactly one finish event."""
    from llm_mcp_amd.engine.engine import GenRequest
    monkeypatch.setenv("LMX_LOOKAHEAD", "1")
    e = _engine()
    assert e.lookahead
    evs = {}
    e.event_sink = lambda batch: [evs.setdefault(x.req.id, []).append(x) for x in batch]
    sp = SamplingParams(temperature=0, max_tokens=10, ignore_eos=True)
    reqs = [e.submit(GenRequest(list(range(i, i + 30)), sp)) for i in range(3)]
    for _ in range(4):
        e.step()
    e.abort(reqs[1].id)
    late = e.submit(GenRequest(list(range(100, 140)), sp))
    for _ in range(200):
        if not e.step() and e._la is None:
            break
    assert not e.sched.has_work and e._la is None
    for r in (reqs[0], reqs[2], late):
        toks = [x for x in evs[r.id] if x.token >= 0]
        fins = [x for x in evs[r.id] if x.finish is not None]
        assert len(toks) == 10 and len(fins) == 1 and fins[0].finish == "length"
    assert [x.finish for x in evs[reqs[1].id] if x.finish is not None] == ["abort"]
    assert e.num_active == 0


def test_kv_page_layouts_roundtrip():
    """The CPU reference writes / gathers the kernels' page layouts: K pages
    token-major [NB, Hkv, BS, D]; V pages key-quad [NB, Hkv, BS/4, D, 4]
    (v_cache[blk, h, key // 4, d, key % 4]), the layout that keeps one
    token's V inside D/16 128-B lines of its page."""
    from llm_mcp_amd.ops import ref
    NB, Hkv, BS, D, n = 6, 2, 32, 64, 70
    kc = torch.zeros(NB, Hkv, BS, D)
    vc = torch.zeros(NB, Hkv, BS // 4, D, 4)
    k, v = torch.randn(n, Hkv, D), torch.randn(n, Hkv, D)
    table = torch.tensor([4, 1, 5], dtype=torch.int32)
    slots = torch.tensor([int(table[i // BS]) * BS + i % BS for i in range(n)],
                         dtype=torch.int32)
    ref.write_cache(k, v, slots, kc, vc)
    k2, v2 = ref.gather_kv(kc, vc, table, n)
    assert torch.equal(k2, k) and torch.equal(v2, v)
    # flat offset of (block, head, key, d) in the V page = ((key // 4) * D + d) * 4 + key % 4
    blk, h, key, d = 1, 1, 37 - 32, 9
    flat = vc.reshape(NB, Hkv, BS * D)[blk, h, ((key // 4) * D + d) * 4 + key % 4]
    assert flat == v[37, h, d]


def test_lookahead_recovers_after_a_step_failure(monkeypatch):
    """A step that raises while a lookahead step is in flight (as a HIP error
    would): the engine fails the in-flight requests (the _loop path) and
    serves new ones afterwards."""
    from llm_mcp_amd.engine.engine import GenRequest
    monkeypatch.setenv("LMX_LOOKAHEAD", "1")
    e = _engine()
    evs = []
    e.event_sink = evs.extend
    sp = SamplingParams(temperature=0, max_tokens=8, ignore_eos=True)
    for i in range(3):
        e.submit(GenRequest(list(range(i, i + 20)), sp))
    real, calls = e._run_eager, [0]

    def flaky(plan):
        calls[0] += 1
        if calls[0] == 4:
            raise RuntimeError("HIP error: injected")
        return real(plan)
    monkeypatch.setattr(e, "_run_eager", flaky)
    for _ in range(50):
        try:
            e.step()
        except RuntimeError:
            e._fail_all("engine_error")
            break
    assert sum(1 for x in evs if x.finish == "error") == 3 and e.num_active == 0
    outs = e.generate([list(range(50, 80))], sp)
    assert len(outs[0]) == 8


def test_admission_window_gathers_a_burst(monkeypatch):
    """An idle engine that sees its first request waits while more keep
    arriving (LMX_ADMIT_QUIET_MS / LMX_ADMIT_MAX_MS) before the first step,
    so a burst is prefilled together instead of the first arrival alone;
    with the window off the first step holds what had arrived."""
    import threading
    import time as _t
    from llm_mcp_amd.engine.engine import GenRequest
    sp = SamplingParams(temperature=0, max_tokens=2, ignore_eos=True)

    def run(quiet_ms):
        monkeypatch.setenv("LMX_STEP_TRACE", "1")
        monkeypatch.setenv("LMX_ADMIT_QUIET_MS", str(quiet_ms))
        monkeypatch.setenv("LMX_ADMIT_MAX_MS", "400")
        e = _engine(max_batched_tokens=512)
        e.submit(GenRequest(list(range(1, 21)), sp))

        def later():
            for i in range(5):            # the rest of the burst, 10 ms apart
                _t.sleep(0.01)
                e.submit(GenRequest(list(range(30 + i, 50 + i)), sp))
        th = threading.Thread(target=later)
        th.start()
        e.step()
        th.join()
        return e.step_trace[0]

    first = run(40.0)
    assert first[3] == 6 * 20           # all six prompts in the first step
    first = run(0.0)
    assert first[3] < 6 * 20            # window off: only what had arrived


def test_peer_failure_withholds_that_steps_tokens():
    """A TP peer collective that timed out (its error word set) during step n:
    the error is raised where step n's tokens are read back, so none of them
    reaches the scheduler or the event sink -- only the earlier, sound steps'
    tokens were emitted (the check used to run at launch and read
    an older step's word)."""
    import pytest
    from llm_mcp_amd.engine.engine import GenRequest

    class StubPeer:
        # the word goes bad during the armed step's kernels: it is visible
        # only through the copy enqueued behind that step (check_async)
        armed = bad = False

        def failed(self):
            return self.bad

        def check_async(self, stream):
            self.bad = self.bad or self.armed

    e = _engine()
    peer = StubPeer()
    e.tp.peer = peer
    got = []
    e.event_sink = got.extend
    e.submit(GenRequest(list(range(10, 30)), SamplingParams(temperature=0, max_tokens=8,
                                                            ignore_eos=True)))
    ok_steps = 0
    for _ in range(3):
        assert e.step()
        ok_steps += 1
    peer.armed = True
    with pytest.raises(RuntimeError, match="peer all-reduce"):
        e.step()
    # step k's events are flushed during step k + 1: every sound step's token
    # and none of the failing step's
    assert len(got) == ok_steps
    assert e.stats["generated_tokens"] == ok_steps
