"""Tensor parallelism on CPU (gloo, world_size 2): a TP group of engines fed
by the leader's plan mailbox must generate what one process generates from
the same (unsharded) weights, and the HF safetensors loader must produce the
same shards as slicing the full weights."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from llm_mcp_amd.engine.engine import EngineConfig, LLMEngine, SamplingParams
from llm_mcp_amd.models import config as mc
from llm_mcp_amd.models.llama import LlamaModel
from llm_mcp_amd.models.weights import load_llama_weights, save_hf_llama, shard_llama
from llm_mcp_amd.parallel.plan_channel import PlanChannel, decode_plan, encode_plan
from tests.dense_ref import assert_greedy_consistent

PROMPTS = [list(range(10, 50)), list(range(5, 100)), [7] * 33, [3]]


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _ecfg(model="tiny-llama"):
    return EngineConfig(model=model, max_num_seqs=8, max_batched_tokens=64,
                        max_model_len=512, use_graphs=False)


def _rank_main(rank, size, port, ckpt, tag, q, sp_min_tokens=0, model="tiny-llama",
               lookahead="0", microbatch="0"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(size), LOCAL_RANK=str(rank),
                      LMX_SP_MIN_TOKENS=str(sp_min_tokens), LMX_TP_PROBE_STEPS="3",
                      LMX_LOOKAHEAD=lookahead, LMX_TP_MICROBATCH=microbatch)
    torch.set_num_threads(2 if size <= 2 else 1)
    import torch.distributed as dist

    from llm_mcp_amd.parallel.tp_worker import build_tp_engine, init_group
    tp = init_group("cpu")
    eng = build_tp_engine(_ecfg(model), "cpu", tp, tag, weights_path=ckpt)
    try:
        if rank == 0:
            greedy = eng.generate(PROMPTS, SamplingParams(temperature=0, max_tokens=6,
                                                          ignore_eos=True))
            sampled = eng.generate(PROMPTS[:2], SamplingParams(temperature=0.8, top_p=0.9,
                                                               max_tokens=5, seed=7,
                                                               ignore_eos=True))
            eng.release_followers()
            q.put(("leader", greedy, sampled, eng.num_blocks, eng.tp_comm_live))
        else:
            q.put(("follower", eng.run_follower(), eng.num_blocks))
    finally:
        eng.chan.close()
        dist.destroy_process_group()


@pytest.fixture(scope="module")
def full_model(tmp_path_factory):
    cfg = mc.resolve("tiny-llama")
    m = LlamaModel(cfg, "cpu", seed=3)
    path = str(tmp_path_factory.mktemp("ckpt"))
    save_hf_llama(m, cfg, path)
    return m, path


def test_loader_matches_slicing(full_model):
    m, path = full_model
    cfg = m.cfg
    for size in (1, 2):
        for rank in range(size):
            a = load_llama_weights(path, cfg, "cpu", rank, size)
            b = shard_llama(m.w, cfg, rank, size)
            for k in ("embed", "norm", "lm_head"):
                assert torch.equal(a[k], b[k]), (size, rank, k)
            for la, lb in zip(a["layers"], b["layers"]):
                for k in la:
                    assert torch.equal(la[k], lb[k]), (size, rank, k)


def test_plan_roundtrip(tmp_path):
    import numpy as np
    e = LLMEngine(_ecfg(), device="cpu")
    e.sched.add(1, list(range(40)), 4, [], True, 0)
    plan = e.sched.schedule(e.q_per_tile)
    leader = PlanChannel(str(tmp_path / "mb"), 0, 2, capacity=1 << 20, create=True)
    follower = PlanChannel(str(tmp_path / "mb"), 1, 2, capacity=1 << 20, create=False)
    leader.publish(encode_plan(plan, None))
    got, bucket = decode_plan(follower.receive())
    assert bucket is None
    for k in ("input_ids", "positions", "slots", "block_tables", "prefill_tiles", "temp"):
        assert np.array_equal(got[k], plan[k]), k
    leader.publish({"cmd": "stop"})   # waits for the follower's ack of msg 1
    assert follower.receive()["cmd"] == "stop"
    follower.close()
    leader.close()


@pytest.mark.parametrize("sp_min_tokens,lookahead,microbatch",
                         [(0, "0", "0"), (7, "0", "0"), (0, "1", "0"), (0, "0", "1")])
def test_tp2_generation_matches_single_process(full_model, sp_min_tokens, lookahead, microbatch):
    """sp_min_tokens=7: every prefill / mixed step of >= 7 tokens runs
    sequence-parallel (reduce-scatter + row-sharded RMSNorm + all-gather),
    odd token counts included (padded rows); pure decode steps stay on the
    all-reduce path.  lookahead=1: the leader launches step n+1 before it
    reads step n back; every rank samples the all-gathered logits itself
    (engine.sample_all) and gathers its inputs from its own samples.
    microbatch=1: pure-prefill steps of >= 2 sequences run as two
    micro-batches whose all-reduces alternate (LlamaModel._forward_tp_mb)."""
    m, path = full_model
    # the TP group samples vocab-sharded (race form): the single-process
    # reference draws with the same sampler over whole rows
    os.environ["LMX_SAMPLER"] = "race"
    try:
        single = LLMEngine(_ecfg(), device="cpu", model_cfg=m.cfg, weights=m.w)
    finally:
        del os.environ["LMX_SAMPLER"]
    ref_sampled = single.generate(PROMPTS[:2], SamplingParams(temperature=0.8, top_p=0.9,
                                                              max_tokens=5, seed=7,
                                                              ignore_eos=True))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port, tag = _free_port(), f"test-{os.getpid()}-{_free_port()}"
    procs = [ctx.Process(target=_rank_main,
                         args=(r, 2, port, path, tag, q, sp_min_tokens, "tiny-llama", lookahead,
                               microbatch),
                         daemon=True)
             for r in range(2)]
    for p in procs:
        p.start()
    try:
        res = [q.get(timeout=240) for _ in procs]
        for p in procs:
            p.join(timeout=60)
            assert p.exitcode == 0
    finally:
        for p in procs:
            if p.is_alive():
                p.kill()
    leader = next(r for r in res if r[0] == "leader")
    follower = next(r for r in res if r[0] == "follower")
    _, greedy, sampled, nb, live = leader
    assert follower[2] == nb                     # agreed KV page count
    # in-service all-reduce samples every 3 steps, run collectively by both ranks
    assert live.get("seq", 0) >= 1 and live["us"].get("rccl", 0) > 0, live
    assert follower[1] > 0                       # follower executed the steps
    for p, o in zip(PROMPTS, greedy):
        assert len(o) == 6
        assert_greedy_consistent(m, p, o)
    # same seeds + same logits (up to bf16 reduction order) -> same samples:
    # the race keys of a row do not depend on how the vocabulary is sharded
    agree = sum(a == b for x, y in zip(sampled, ref_sampled) for a, b in zip(x, y))
    assert agree >= 8, (sampled, ref_sampled)


def test_qwen_loader_roundtrip_with_bias(tmp_path):
    cfg = mc.resolve("tiny-qwen")
    m = LlamaModel(cfg, "cpu", seed=5)
    save_hf_llama(m, cfg, str(tmp_path))
    assert mc.from_hf_config(str(tmp_path / "config.json")).qkv_bias
    a = load_llama_weights(str(tmp_path), cfg, "cpu")
    for la, lb in zip(a["layers"], m.w["layers"]):
        assert torch.equal(la["bqkv"], lb["bqkv"]) and torch.equal(la["wqkv"], lb["wqkv"])


def test_qwen3_loader_roundtrip_and_tp_shards(tmp_path):
    cfg = mc.resolve("tiny-qwen3")
    m = LlamaModel(cfg, "cpu", seed=9)
    save_hf_llama(m, cfg, str(tmp_path))
    hf = mc.from_hf_config(str(tmp_path / "config.json"))
    assert hf.qk_norm and not hf.qkv_bias and hf.family == "qwen3"
    for size in (1, 2):
        for rank in range(size):
            a = load_llama_weights(str(tmp_path), cfg, "cpu", rank, size)
            b = shard_llama(m.w, cfg, rank, size)
            for la, lb in zip(a["layers"], b["layers"]):
                assert set(la) == set(lb)
                assert torch.equal(la["q_norm"], lb["q_norm"]) and torch.equal(la["wqkv"], lb["wqkv"])



@pytest.fixture(scope="module")
def full_model_tp8(tmp_path_factory):
    cfg = mc.resolve("tiny-llama-tp8")
    m = LlamaModel(cfg, "cpu", seed=5)
    path = str(tmp_path_factory.mktemp("ckpt8"))
    save_hf_llama(m, cfg, path)
    return m, path


@pytest.mark.timeout(600)
def test_tp8_generation_with_sp_matches_dense(full_model_tp8):
    """World size 8 (the 70B TP=8 layout: 2 q heads and 1 kv head per rank,
    vocab-parallel LM head gathered to the leader only), sequence-parallel
    forced on every step of >= 5 tokens, 8 gloo ranks on the CPU."""
    m, path = full_model_tp8
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port, tag = _free_port(), f"test8-{os.getpid()}-{_free_port()}"
    procs = [ctx.Process(target=_rank_main, args=(r, 8, port, path, tag, q, 5, "tiny-llama-tp8"),
                         daemon=True) for r in range(8)]
    for p in procs:
        p.start()
    try:
        res = [q.get(timeout=500) for _ in procs]
        for p in procs:
            p.join(timeout=60)
            assert p.exitcode == 0
    finally:
        for p in procs:
            if p.is_alive():
                p.kill()
    leader = next(r for r in res if r[0] == "leader")
    followers = [r for r in res if r[0] == "follower"]
    assert len(followers) == 7 and all(f[1] > 0 and f[2] == leader[3] for f in followers)
    for p, o in zip(PROMPTS, leader[1]):
        assert len(o) == 6
        assert_greedy_consistent(m, p, o)


def _leader_then_die(path, q):
    ch = PlanChannel(path, 0, 2, capacity=1 << 20, create=True)
    ch.publish({"cmd": "step-noop"})
    q.put("published")
    import time
    time.sleep(600)          # killed by the test


def _follower(path, q):
    os.environ["LMX_TP_LEADER_TIMEOUT_S"] = "20"
    from llm_mcp_amd.parallel.plan_channel import LeaderLost
    ch = PlanChannel(path, 1, 2, capacity=1 << 20, create=False)
    assert ch.receive()["cmd"] == "step-noop"
    q.put("first")
    try:
        ch.receive()          # the leader is killed while we wait here
    except LeaderLost as e:
        q.put(f"lost: {e}")
        raise SystemExit(3)
    q.put("unexpected message")


def test_follower_exits_when_the_leader_dies(tmp_path):
    """A killed TP leader must not strand its followers: the mailbox carries
    the leader's pid and a heartbeat, and a waiting follower raises
    LeaderLost (the TP worker then exits non-zero) within seconds."""
    import signal
    import time
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    path = str(tmp_path / "mb")
    lead = ctx.Process(target=_leader_then_die, args=(path, q), daemon=True)
    lead.start()
    assert q.get(timeout=60) == "published"
    fol = ctx.Process(target=_follower, args=(path, q), daemon=True)
    fol.start()
    try:
        assert q.get(timeout=60) == "first"
        t0 = time.time()
        os.kill(lead.pid, signal.SIGKILL)
        msg = q.get(timeout=30)
        fol.join(timeout=30)
        assert msg.startswith("lost:") and "gone" in msg, msg
        assert fol.exitcode == 3 and time.time() - t0 < 30
    finally:
        for p in (lead, fol):
            if p.is_alive():
                p.kill()


def test_follower_exits_on_stale_heartbeat(tmp_path):
    """Leader process alive but wedged (no heartbeat): the follower gives up
    after LMX_TP_LEADER_TIMEOUT_S."""
    import time
    leader = PlanChannel(str(tmp_path / "mb"), 0, 2, capacity=1 << 20, create=True)
    leader._beat_stop.set()                     # freeze the heartbeat
    leader._beat_thread.join()
    leader.ctl[2] = time.time_ns() - int(60e9)  # last beat a minute ago
    follower = PlanChannel(str(tmp_path / "mb"), 1, 2, capacity=1 << 20, create=False)
    from llm_mcp_amd.parallel.plan_channel import LeaderLost
    t0 = time.time()
    with pytest.raises(LeaderLost, match="heartbeat"):
        follower.receive(timeout_s=5)
    assert time.time() - t0 < 10
    follower.close()
    leader.close()


def test_prefill_microbatches_match_one_batch(full_model, monkeypatch):
    """The micro-batch split of a pure-prefill step (LlamaModel._microbatch):
    the two halves' rows, rebased cu_q / tile lists / sampled rows, run through
    the per-micro-batch pipeline, give the logits of the unsplit forward
    (single process: the all-reduces are no-ops, the split is what is tested)."""
    import numpy as np
    from llm_mcp_amd import ops
    from llm_mcp_amd.models.llama import StepInputs
    m, _ = full_model
    cfg = m.cfg
    lens = [7, 12, 5, 9]
    BS, D = 32, cfg.head_dim
    nb = 8
    kc = [torch.zeros(nb, cfg.num_kv_heads, BS, D, dtype=torch.bfloat16) for _ in range(cfg.num_layers)]
    vc = [torch.zeros(nb, cfg.num_kv_heads, BS // 4, D, 4, dtype=torch.bfloat16)
          for _ in range(cfg.num_layers)]
    ids = torch.arange(sum(lens), dtype=torch.int32) % 400 + 3
    cu = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
    pos = torch.cat([torch.arange(n, dtype=torch.int32) for n in lens])
    bt = torch.arange(len(lens), dtype=torch.int32).view(-1, 1)
    slots = torch.cat([torch.arange(n, dtype=torch.int32) + 32 * i for i, n in enumerate(lens)])
    qpt = ops.prefill_q_per_tile(cfg.num_heads, cfg.num_kv_heads, D)
    tiles = np.array([v for s_, n in enumerate(lens) for q0 in range(0, n, qpt) for v in (s_, q0)],
                     np.int32)
    rows = (cu[1:] - 1).astype(np.int64)
    inp = StepInputs(ids, pos, slots, 0, bt, torch.tensor(lens, dtype=torch.int32),
                     torch.from_numpy(cu), torch.from_numpy(tiles), torch.from_numpy(rows),
                     int(cu[-1]), len(lens),
                     host={"cu_q": cu, "tiles": tiles, "rows": rows})
    ref = m.forward(inp, kc, vc, None).float()
    # the split the model would take, then the micro-batched path itself
    j = 2
    a, b = m._microbatch(inp, 0, j), m._microbatch(inp, j, len(lens))
    assert a.num_tokens + b.num_tokens == inp.num_tokens
    assert a.host["cu_q"].tolist() == [0, 7, 19] and b.host["cu_q"].tolist() == [0, 5, 14]
    assert b.prefill_tiles.view(-1, 2)[:, 0].tolist() == sorted(b.prefill_tiles.view(-1, 2)[:, 0].tolist())
    assert b.sample_rows.tolist() == [4, 13]
    got = m._forward_tp_mb(inp, j, kc, vc).float()
    torch.testing.assert_close(got, ref, atol=1e-2, rtol=1e-2)


def test_all_reduce_async_takes_rccl_beside_the_peer_kernel(monkeypatch):
    """An RCCL TP group with the peer all-reduce installed (the 8-GPU default):
    messages the peer slot holds run on the peer kernel, anything larger (the
    prefill micro-batch all-reduces) must go to RCCL with async_op=True, or
    the two micro-batches of _forward_tp_mb serialise."""
    import torch.distributed as dist
    from llm_mcp_amd.models.llama import TPContext, _Done

    calls = []

    class StubPeer:
        slot = 1 << 10

        def supports(self, t):
            return t.numel() * t.element_size() <= self.slot

        def __call__(self, t):
            calls.append(("peer", t.numel()))
            return t

    class Handle:
        def wait(self):
            return True

    def fake_all_reduce(t, group=None, async_op=False, **kw):
        calls.append(("rccl_async" if async_op else "rccl_sync", t.numel()))
        return Handle() if async_op else None

    monkeypatch.setattr(dist, "get_backend", lambda group=None: "nccl")
    monkeypatch.setattr(dist, "all_reduce", fake_all_reduce)
    tp = TPContext(rank=0, size=8, group=object())
    tp.peer = StubPeer()
    small = torch.zeros(256)            # 1 KB fp32: inside the slot
    big = torch.zeros(64, 1024)         # 256 KB: prefill-sized
    h_small = tp.all_reduce_async(small)
    h_big = tp.all_reduce_async(big)
    assert isinstance(h_small, _Done) and isinstance(h_big, Handle)
    assert calls == [("peer", 256), ("rccl_async", 64 * 1024)]


def test_fused_norm_grid_plan():
    """PeerAllReduce.norm_plan: a rank's few decode rows split over column
    chunks (>= 256 16-B columns each, LMX_AR_NORM_CS at most), at most 128
    blocks per rank alone on its GPU and 256 / ranks-per-card when a one-GPU
    rehearsal puts the whole group on one card (all blocks must co-reside)."""
    from llm_mcp_amd.parallel.peer_allreduce import PeerAllReduce

    def plan(world, T, cols, two, co=1, mcs=2):
        p = PeerAllReduce.__new__(PeerAllReduce)
        p.world, p.norm_max_cs, p.co_resident = world, mcs, co
        return p.norm_plan(T, cols, two)

    assert plan(8, 256, 8192, 1) == (32, 2)            # 32 rows per rank -> 64 blocks
    assert plan(8, 256, 8192, 1, mcs=4) == (32, 4)
    assert plan(8, 256, 8192, 1, mcs=1) == (32, 1)
    assert plan(2, 256, 4096, 1) == (128, 1)           # the grid is already full
    assert plan(8, 37, 1024, 0) == (37, 1)             # 128 columns: no split
    assert plan(8, 256, 8192, 1, co=8, mcs=4) == (32, 1)   # 8 ranks on one card: 32 blocks
    g, cs = plan(8, 16, 8192, 0, co=8, mcs=4)
    assert g * cs <= 32 and cs == 2
    for world, T, cols, two, co, mcs in [(2, 300, 4096, 1, 1, 4), (4, 64, 8192, 1, 4, 4),
                                        (8, 1, 8192, 0, 1, 4)]:
        g, cs = plan(world, T, cols, two, co, mcs)
        assert g * cs <= max(32, min(128, 256 // co)) and (cols // 8) % cs == 0
