"""Engine on the GPU (HIP kernels + hipGraph decode) against the dense fp32
reference forward."""
import pytest
import torch

from llm_mcp_amd import ops
from llm_mcp_amd.engine.engine import EngineConfig, GenRequest, LLMEngine, SamplingParams
from tests.dense_ref import assert_greedy_consistent

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("graphs", [False, True])
def test_tiny_llama_engine_matches_dense(graphs):
    ops.native()
    e = LLMEngine(EngineConfig(model="tiny-llama", max_num_seqs=16, max_batched_tokens=128,
                               max_model_len=1024, use_graphs=graphs, kv_cache_gb=0.05),
                  device="cuda")
    prompts = [list(range(10, 50)), list(range(5, 300)), [7] * 33, [3]]
    outs = e.generate(prompts, SamplingParams(temperature=0, max_tokens=12, ignore_eos=True))
    for p, o in zip(prompts, outs):
        assert len(o) == 12
        assert_greedy_consistent(e.model, p, o)
    if graphs:
        assert e.stats["graph_steps"] > 0


def test_llama3_8b_decode_step_runs():
    ops.native()
    e = LLMEngine(EngineConfig(model="llama-3-8b", max_num_seqs=8, max_batched_tokens=1024,
                               max_model_len=2048, use_graphs=True, kv_cache_gb=4),
                  device="cuda")
    outs = e.generate([list(range(100, 400)), list(range(7, 40))],
                      SamplingParams(temperature=0.8, top_p=0.95, max_tokens=16, ignore_eos=True,
                                     seed=1))
    assert all(len(o) == 16 for o in outs)
    assert all(0 <= t < 128256 for o in outs for t in o)
    assert e.stats["graph_steps"] > 0
    torch.cuda.synchronize()


@pytest.mark.gpu
@pytest.mark.parametrize("preset", ["tiny-nomic", "nomic-2layer"])
def test_nomic_bert_gpu_matches_cpu_reference(preset):
    """Encoder on the HIP kernels (K13 large-M GEMM incl. the fused SwiGLU
    epilogue -- gemm_nt for the tiny shapes K13 does not take -- tiled
    rope/cache, bidirectional paged prefill, LayerNorm, mean-pool) vs the same
    weights on the fp32-reference CPU path."""
    import dataclasses

    from llm_mcp_amd.models import config as mc
    from llm_mcp_amd.models.nomic_bert import NomicBertModel
    cfg = mc.resolve("tiny-nomic") if preset == "tiny-nomic" else \
        dataclasses.replace(mc.resolve("nomic-embed-text"), num_layers=2)
    g = NomicBertModel(cfg, "cuda", seed=3)
    wc = {k: (v.cpu() if hasattr(v, "cpu") else [{kk: vv.cpu() for kk, vv in L.items()}
                                                  for L in v]) for k, v in g.w.items()}
    c = NomicBertModel(cfg, "cpu", weights=wc)
    lens = [30, 1, 39, 70]
    ids = torch.randint(0, 500, (sum(lens),), dtype=torch.int32)
    cu = torch.tensor([0] + list(torch.cumsum(torch.tensor(lens), 0)), dtype=torch.int32)
    before = ops.PGEMM_CALLS[0]
    a = g.forward(ids.cuda(), cu.cuda(), lens).cpu()
    if preset == "nomic-2layer":
        assert ops.PGEMM_CALLS[0] - before == 2 * 4     # every projection on K13
    b = c.forward(ids, cu, lens)
    cos = torch.nn.functional.cosine_similarity(a, b, dim=-1)
    assert float(cos.min()) > 0.999, cos
    assert float((a - b).abs().max()) < 2e-2


@pytest.mark.gpu
@pytest.mark.parametrize("preset", ["tiny-bert", "tiny-bert-mean", "mxbai-2layer"])
def test_bert_gpu_matches_cpu_reference(preset):
    """BERT encoder on the HIP kernels (K13 with fused bias / exact GELU --
    gemm_nt with the residual for the tiny shapes -- kv_write, bidirectional
    paged prefill, LayerNorm, CLS or mean pooling) vs the same weights on the
    fp32-reference CPU path."""
    import dataclasses

    from llm_mcp_amd.models import config as mc
    from llm_mcp_amd.models.bert import BertModel
    cfg = mc.resolve(preset) if preset.startswith("tiny") else \
        dataclasses.replace(mc.resolve("mxbai-embed-large"), num_layers=2)
    g = BertModel(cfg, "cuda", seed=3)
    wc = {k: (v.cpu() if hasattr(v, "cpu") else [{kk: vv.cpu() for kk, vv in L.items()}
                                                  for L in v]) for k, v in g.w.items()}
    c = BertModel(cfg, "cpu", weights=wc)
    lens = [30, 1, 39, 70]
    ids = torch.randint(0, 500, (sum(lens),), dtype=torch.int32)
    cu = torch.tensor([0] + list(torch.cumsum(torch.tensor(lens), 0)), dtype=torch.int32)
    before = ops.PGEMM_CALLS[0]
    a = g.forward(ids.cuda(), cu.cuda(), lens).cpu()
    if preset == "mxbai-2layer":
        assert ops.PGEMM_CALLS[0] - before == 2 * 4     # every projection on K13
    b = c.forward(ids, cu, lens)
    cos = torch.nn.functional.cosine_similarity(a, b, dim=-1)
    assert float(cos.min()) > 0.999, cos
    assert float((a - b).abs().max()) < 2e-2


@pytest.mark.gpu
def test_qwen2_group7_on_gpu_kernels():
    e = LLMEngine(EngineConfig(model="tiny-qwen", max_num_seqs=8, max_batched_tokens=128,
                               max_model_len=512, kv_cache_gb=0.05), device="cuda")
    prompts = [list(range(10, 80)), [7] * 33, [3]]
    outs = e.generate(prompts, SamplingParams(temperature=0, max_tokens=6, ignore_eos=True))
    for p, o in zip(prompts, outs):
        assert len(o) == 6
        assert_greedy_consistent(e.model, p, o)


@pytest.mark.gpu
def test_qwen3_qk_norm_on_gpu_kernels():
    e = LLMEngine(EngineConfig(model="tiny-qwen3", max_num_seqs=8, max_batched_tokens=128,
                               max_model_len=512, kv_cache_gb=0.05), device="cuda")
    prompts = [list(range(10, 80)), [7] * 33, [3]]
    outs = e.generate(prompts, SamplingParams(temperature=0, max_tokens=6, ignore_eos=True))
    for p, o in zip(prompts, outs):
        assert len(o) == 6
        assert_greedy_consistent(e.model, p, o)


@pytest.mark.gpu
def test_penalties_in_graph_and_eager():
    """Penalised rows inside the captured decode graph (penalty block uploaded,
    pen_on flag) and on the eager path: greedy tokens never repeat one of the
    last 64 context tokens; unpenalised rows in the same batch are unchanged."""
    e = LLMEngine(EngineConfig(model="tiny-llama", max_num_seqs=8, max_batched_tokens=256,
                               max_model_len=512, kv_cache_gb=0.05), device="cuda")
    assert e.graphs, "decode graphs expected"
    prompts = [list(range(5, 45)), [9] * 20 + list(range(100, 120))]
    base = e.generate(prompts, SamplingParams(temperature=0, max_tokens=40, ignore_eos=True))
    pen = SamplingParams(temperature=0, max_tokens=40, ignore_eos=True, repetition_penalty=1e4,
                         presence_penalty=1e3, penalty_last_n=64)
    reqs = [e.submit(GenRequest(list(prompts[0]), pen)),
            e.submit(GenRequest(list(prompts[1]), SamplingParams(temperature=0, max_tokens=40,
                                                                 ignore_eos=True)))]
    outs = {r.id: [] for r in reqs}
    done = set()

    def sink(evs):
        for ev in evs:
            if ev.token >= 0:
                outs[ev.req.id].append(ev.token)
            if ev.finish is not None:
                done.add(ev.req.id)
    e.event_sink = sink
    while len(done) < 2:
        e.step()
    ctx = list(prompts[0])
    for t in outs[reqs[0].id]:
        assert t not in ctx[-64:]
        ctx.append(t)
    assert outs[reqs[1].id] == base[1]
    assert e.stats["graph_steps"] > 0


@pytest.mark.parametrize("graphs", [False, True])
def test_llama3_8b_shapes_on_decode_gemm_match_dense(graphs):
    """Two layers of Llama-3-8B (the served d=4096 / I=14336 / vocab 128256
    shapes, so the measured K11 table applies): prefill of 48 prompts in one
    step (T <= 256) and decode at M = 48 run on the decode GEMM -- fused
    SwiGLU gate/up, split-K partials summed inside the residual-add RMSNorm --
    and every greedy token is (near-)argmax of the dense fp32 forward."""
    import dataclasses

    from llm_mcp_amd.models import config as mc
    ops.native()
    cfg = dataclasses.replace(mc.resolve("llama-3-8b"), num_layers=2)
    n0 = ops.DGEMM_CALLS[0]
    e = LLMEngine(EngineConfig(model="llama-3-8b", max_num_seqs=64, max_batched_tokens=512,
                               max_model_len=512, use_graphs=graphs, kv_cache_gb=1),
                  device="cuda", model_cfg=cfg)
    # 16: the in-register epilogue over 16-column gate/up pairs (epi 3 table
    # entries); BN/2 of the LDS hand-off form (epi 1) when only those exist
    assert e.model.gu_block == ops.swiglu_block(2 * cfg.intermediate_size, cfg.hidden_size) > 0, \
        "fused SwiGLU layout not selected from the table"
    prompts = [[(17 * i + 3 * j) % 120000 + 100 for j in range(4)] for i in range(48)]
    outs = e.generate(prompts, SamplingParams(temperature=0, max_tokens=3, ignore_eos=True))
    assert ops.DGEMM_CALLS[0] > n0
    for p, o in list(zip(prompts, outs))[::7]:
        assert_greedy_consistent(e.model, p, o, tol=0.08)


@pytest.mark.parametrize("preset", ["qwen3-8b", "qwen2.5-7b", "llama-3.2-3b"])
def test_family_shapes_on_decode_gemm_match_dense(preset):
    """Two layers of the other served chat families at their real shapes
    (Qwen3 q/k-norm, Qwen2.5 GQA-7 with QKV bias, Llama-3.2-3B): the round-6
    family sweep's K11 table entries (bench/dgemm_bench.py, tools/dg_merge.py)
    put the decode projections on the hand-written GEMM -- fused SwiGLU
    gate/up, split-K partials summed in the residual-add RMSNorm -- in captured
    graphs, and greedy tokens stay (near-)argmax of the dense fp32 forward."""
    import dataclasses

    from llm_mcp_amd.models import config as mc
    ops.native()
    cfg = dataclasses.replace(mc.resolve(preset), num_layers=2)
    n0 = ops.DGEMM_CALLS[0]
    e = LLMEngine(EngineConfig(model=preset, max_num_seqs=64, max_batched_tokens=512,
                               max_model_len=512, use_graphs=True, kv_cache_gb=1),
                  device="cuda", model_cfg=cfg)
    assert e.model.gu_block == ops.SWIGLU16, "fused SwiGLU layout not selected from the table"
    prompts = [[(17 * i + 3 * j) % 120000 + 100 for j in range(4)] for i in range(48)]
    outs = e.generate(prompts, SamplingParams(temperature=0, max_tokens=3, ignore_eos=True))
    assert ops.DGEMM_CALLS[0] > n0
    assert e.stats["graph_steps"] > 0
    for p, o in list(zip(prompts, outs))[::7]:
        assert_greedy_consistent(e.model, p, o, tol=0.08)


@pytest.mark.parametrize("preset", ["qwen3-8b", "llama-3.2-3b"])
def test_family_shapes_200_rows(preset):
    """The same families at a 200-row batch: K13 prefill of 200 x 4 tokens
    and 200-row decode steps on the K11 entries (fused SwiGLU gate/up, down
    partials summed in the norm) in captured graphs.  Their MLP weights stay
    row-major (no packed-only K14 entries for these shapes: K11 serves every
    batch size), and greedy tokens stay (near-)argmax of the dense fp32
    forward."""
    import dataclasses

    from llm_mcp_amd.models import config as mc
    ops.native()
    cfg = dataclasses.replace(mc.resolve(preset), num_layers=2)
    n0 = ops.DGEMM_CALLS[0]
    e = LLMEngine(EngineConfig(model=preset, max_num_seqs=224, max_batched_tokens=1024,
                               max_model_len=256, use_graphs=True, kv_cache_gb=1),
                  device="cuda", model_cfg=cfg)
    assert not ops.is_packed_only(e.model.w["layers"][0]["w_down"])
    prompts = [[(13 * i + 5 * j) % 120000 + 100 for j in range(4)] for i in range(200)]
    outs = e.generate(prompts, SamplingParams(temperature=0, max_tokens=3, ignore_eos=True))
    assert ops.DGEMM_CALLS[0] > n0
    assert e.stats["graph_steps"] > 0
    for p, o in list(zip(prompts, outs))[::37]:
        assert_greedy_consistent(e.model, p, o, tol=0.08)


@pytest.mark.parametrize("graphs", [False, True])
def test_llama3_8b_shapes_k13_prefill_and_sk_lm_head(graphs):
    """Two layers of Llama-3-8B at a 200-row batch: the one-step prefill of
    200 x 4 tokens (M = 800) runs the projections on K13 (fused SwiGLU gate/up)
    and the 200-row decode steps run the LM head on K13-SK (config "sk") and
    gate/up / down on K14 (config "rs"), in
    captured graphs too (bucket 224); greedy tokens stay (near-)argmax of the dense fp32
    forward."""
    import dataclasses

    from llm_mcp_amd.models import config as mc
    ops.native()
    cfg = dataclasses.replace(mc.resolve("llama-3-8b"), num_layers=2)
    assert ops.sk_choice(200, cfg.vocab_size, cfg.hidden_size) is not None
    n0, r0 = ops.PGEMM_CALLS[0], ops.RSGEMM_CALLS[0]
    e = LLMEngine(EngineConfig(model="llama-3-8b", max_num_seqs=224, max_batched_tokens=1024,
                               max_model_len=256, use_graphs=graphs, kv_cache_gb=1),
                  device="cuda", model_cfg=cfg)
    prompts = [[(13 * i + 5 * j) % 120000 + 100 for j in range(4)] for i in range(200)]
    outs = e.generate(prompts, SamplingParams(temperature=0, max_tokens=3, ignore_eos=True))
    assert ops.PGEMM_CALLS[0] > n0
    # 200-row decode steps: gate/up + SwiGLU and down partials on K14 (packed
    # weights, 128-row tiles; config "rs") when the table has those entries
    if ops.rs_choice(200, 2 * cfg.intermediate_size, cfg.hidden_size, 3,
                     w=e.model.w["layers"][0]["w_gate_up"]) is not None:
        assert ops.RSGEMM_CALLS[0] > r0
    if graphs:
        assert e.stats["graph_steps"] > 0
    for p, o in list(zip(prompts, outs))[::37]:
        assert_greedy_consistent(e.model, p, o, tol=0.08)


@pytest.mark.parametrize("M", [300, 512, 640])
def test_rows_split_products_match_dense(M):
    """257-1024-row products on the narrow Llama-3-8B projections (QKV, O,
    down; fewer than 128 K13 tiles): a row-major weight takes the library
    (K13's tile wave would be mostly empty), a packed-only one equal <= 256-row
    pieces on K14 (ops.rows_split); both give the fp32 product."""
    ops.native()
    torch.manual_seed(M)
    for N, K in ((6144, 4096), (4096, 4096), (4096, 14336)):
        assert ops.rows_split(M, N)
        x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
        w = (torch.randn(N, K, device="cuda") * K ** -0.5).to(torch.bfloat16)
        ops.rs_prepare(w)
        assert not ops.rows_split(M, N, K, 0, w)
        want = x.float() @ w.float().t()
        forms = [w]
        if ops.rs_single_ok(w):
            wp = ops.rs_pack_only(w.clone())
            assert ops.rows_split(M, N, K, 0, wp)
            forms.append(wp)
        for ww in forms:
            torch.testing.assert_close(ops.linear(x, ww).float(), want, atol=3e-2, rtol=3e-2)
            d = ops.linear(x, ww, defer=True)
            d = d.sum() if isinstance(d, ops.Partials) else d
            torch.testing.assert_close(d.float(), want, atol=3e-2, rtol=3e-2)


def test_llama3_8b_400_stream_decode_in_row_pieces():
    """Two layers of Llama-3-8B with 400 streams: the decode steps (graph
    bucket above 256 rows) run QKV / O / down off K13, whose tile waves would
    be mostly empty (library for row-major weights, <= 256-row K14 pieces for
    packed-only ones), in captured graphs; greedy tokens stay (near-)argmax of
    the dense fp32 forward."""
    import dataclasses

    from llm_mcp_amd.models import config as mc
    ops.native()
    cfg = dataclasses.replace(mc.resolve("llama-3-8b"), num_layers=2)
    d0, r0 = ops.DGEMM_CALLS[0], ops.RSGEMM_CALLS[0]      # decode graphs capture at load
    e = LLMEngine(EngineConfig(model="llama-3-8b", max_num_seqs=512, max_batched_tokens=2048,
                               max_model_len=256, use_graphs=True, kv_cache_gb=2),
                  device="cuda", model_cfg=cfg)
    prompts = [[(11 * i + 3 * j) % 120000 + 100 for j in range(4)] for i in range(400)]
    outs = e.generate(prompts, SamplingParams(temperature=0, max_tokens=3, ignore_eos=True))
    assert ops.DGEMM_CALLS[0] + ops.RSGEMM_CALLS[0] > d0 + r0
    assert e.stats["graph_steps"] > 0
    for p, o in list(zip(prompts, outs))[::61]:
        assert_greedy_consistent(e.model, p, o, tol=0.08)


def test_lookahead_graph_steps_match_synchronous(monkeypatch):
    """Lookahead stepping on the captured decode graphs (input tokens gathered
    on the device by ops.ids_from_prev from the previous step's samples) gives
    the synchronous engine's tokens: seeded top-p sampling, stop tokens, rows
    joining while others decode, and the greedy streams stay consistent with
    the dense fp32 forward."""
    ops.native()
    base = None
    prompts = [list(range(10, 50)), list(range(5, 300)), [7] * 33, [3], list(range(40, 41 + 70))]

    def run(la, sp):
        nonlocal base
        monkeypatch.setenv("LMX_LOOKAHEAD", la)
        e = LLMEngine(EngineConfig(model="tiny-llama", max_num_seqs=16, max_batched_tokens=96,
                                   max_model_len=1024, use_graphs=True, kv_cache_gb=0.05),
                      device="cuda", weights=None if base is None else base.model.w)
        base = base or e
        assert e.lookahead == (la == "1")
        out = e.generate(prompts, sp)
        torch.cuda.synchronize()
        assert e.stats["graph_steps"] > 0
        return out, e

    greedy = SamplingParams(temperature=0, max_tokens=16, ignore_eos=True)
    g0, _ = run("0", greedy)
    g1, e1 = run("1", greedy)
    assert g1 == g0
    for p, o in zip(prompts, g1):
        assert_greedy_consistent(e1.model, p, o)
    free, _ = run("0", SamplingParams(temperature=0.8, top_p=0.9, max_tokens=16, seed=3))
    stops = [free[0][3], free[2][7]]
    sp = SamplingParams(temperature=0.8, top_p=0.9, max_tokens=16, seed=3, stop_token_ids=stops)
    s0, _ = run("0", sp)
    s1, _ = run("1", sp)
    assert s1 == s0
    assert any(len(o) < 16 for o in s1)
