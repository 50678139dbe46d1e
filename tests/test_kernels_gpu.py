"""Numerics of every gfx950 HIP kernel against the plain PyTorch fp32
reference of the same op (ops/ref.py)."""
import math

import pytest
import torch

from llm_mcp_amd import ops
from llm_mcp_amd.ops import ref

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(autouse=True)
def _native():
    ops.native()  # GPU tests must exercise the HIP path: fail if it is missing
    torch.manual_seed(0)


def _bf(*shape, scale=1.0):
    return (torch.randn(*shape, device=DEV) * scale).to(torch.bfloat16)


@pytest.mark.parametrize("rows,cols", [(1, 4096), (7, 4096), (300, 768), (64, 8192), (3, 256)])
def test_rms_norm(rows, cols):
    x, w = _bf(rows, cols), _bf(cols)
    y = ops.rms_norm(x, w, 1e-5)
    torch.testing.assert_close(y.float(), ref.rms_norm(x, w, 1e-5).float(), atol=2e-2, rtol=2e-2)
    r = _bf(rows, cols)
    r_ref = r.clone()
    y2 = ops.rms_norm(x, w, 1e-5, residual=r)
    y2_ref = ref.rms_norm(x, w, 1e-5, residual=r_ref)
    torch.testing.assert_close(r.float(), r_ref.float(), atol=1e-2, rtol=1e-2)
    torch.testing.assert_close(y2.float(), y2_ref.float(), atol=3e-2, rtol=3e-2)


def test_rms_norm_strided_input():
    x = _bf(16, 6144)[:, 1024:5120]
    w = _bf(4096)
    torch.testing.assert_close(ops.rms_norm(x, w, 1e-5).float(),
                               ref.rms_norm(x.contiguous(), w, 1e-5).float(), atol=2e-2, rtol=2e-2)


def test_layer_norm():
    x, w, b, r = _bf(33, 768), _bf(768), _bf(768), _bf(33, 768)
    torch.testing.assert_close(ops.layer_norm(x, w, b, 1e-12, r).float(),
                               ref.layer_norm(x, w, b, 1e-12, r).float(), atol=3e-2, rtol=3e-2)


def _cache(NB, Hkv, D, BS=32):
    k = _bf(NB, Hkv, BS, D)
    v = _bf(NB, Hkv, BS // 4, D, 4)      # key-quad V pages
    return k, v


@pytest.mark.parametrize("Hq,Hkv,D", [(32, 8, 128), (8, 1, 128), (12, 12, 64), (4, 2, 128)])
@pytest.mark.parametrize("layout", ["scattered", "chunks"])
@pytest.mark.parametrize("tile_from", [None, 5, 1000])
def test_rope_and_cache(Hq, Hkv, D, layout, tile_from):
    _rope_case(Hq, Hkv, D, layout, tile_from, qk_norm=False)


@pytest.mark.parametrize("Hq,Hkv", [(32, 8), (16, 8), (4, 2)])
@pytest.mark.parametrize("tile_from", [None, 5, 1000])
def test_rope_and_cache_qk_norm(Hq, Hkv, tile_from):
    """Qwen3: per-head q/k RMSNorm fused before the rotation (both kernels)."""
    _rope_case(Hq, Hkv, 128, "chunks", tile_from, qk_norm=True)


def _rope_case(Hq, Hkv, D, layout, tile_from, qk_norm):
    T, NB = 77, 8
    qkv = _bf(T, (Hq + 2 * Hkv) * D)
    pos = torch.randint(0, 4000, (T,), device=DEV, dtype=torch.int32)
    cs = ref.rope_cos_sin(4096, D, 500000.0, DEV)
    if layout == "scattered":
        slots = torch.randperm(NB * 32, device=DEV)[:T].to(torch.int32)
    else:   # prefill-like runs: consecutive slots starting mid-page, page jumps
        slots = torch.cat([torch.arange(45, 45 + 40), torch.arange(160, 160 + 37)]).to(
            torch.int32).to(DEV)
    slots[3] = -1
    kc, vc = torch.zeros(NB, Hkv, 32, D, device=DEV, dtype=torch.bfloat16), \
        torch.zeros(NB, Hkv, 8, D, 4, device=DEV, dtype=torch.bfloat16)
    qkv0, kc0, vc0 = qkv.cpu(), kc.cpu(), vc.cpu()
    qn = kn = None
    if qk_norm:
        qn = (1 + 0.2 * torch.randn(D, device=DEV)).to(torch.bfloat16)
        kn = (1 + 0.2 * torch.randn(D, device=DEV)).to(torch.bfloat16)
        qkv.mul_(3.0)                      # the norm must really rescale
        qkv0 = qkv.cpu()
    ops.rope_and_cache(qkv, pos, cs, Hq, Hkv, D, slots, kc, vc, tile_from=tile_from,
                       q_norm=qn, k_norm=kn, eps=1e-6)
    ref.rope_cache(qkv0, pos.cpu(), cs.cpu(), Hq, Hkv, D, slots.cpu(), kc0, vc0, False,
                   None if qn is None else qn.cpu(), None if kn is None else kn.cpu(), 1e-6)
    torch.testing.assert_close(qkv[:, :Hq * D].float().cpu(), qkv0[:, :Hq * D].float(),
                               atol=2e-2, rtol=2e-2)
    torch.testing.assert_close(kc.cpu().float(), kc0.float(), atol=2e-2, rtol=2e-2)
    assert torch.equal(vc.cpu(), vc0)


def _random_tables(B, ctxs, NB, BS=32):
    maxb = max(math.ceil(c / BS) for c in ctxs)
    perm = torch.randperm(NB)
    bt = torch.zeros(B, maxb, dtype=torch.int32)
    k = 0
    for b, c in enumerate(ctxs):
        nb = math.ceil(c / BS)
        bt[b, :nb] = perm[k:k + nb]
        k += nb
    return bt.to(DEV)


@pytest.mark.parametrize("Hq,Hkv,D", [(32, 8, 128), (8, 1, 128), (64, 8, 128), (16, 16, 64),
                                     (28, 4, 128), (14, 2, 64), (24, 8, 128)])
@pytest.mark.parametrize("ctxs", [[1, 17, 32, 33, 500], [1024, 2047, 3000], [5000]])
def test_paged_decode(Hq, Hkv, D, ctxs):
    B = len(ctxs)
    NB = sum(math.ceil(c / 32) for c in ctxs) + 4
    kc, vc = _cache(NB, Hkv, D)
    bt = _random_tables(B, ctxs, NB)
    ctx = torch.tensor(ctxs, dtype=torch.int32, device=DEV)
    q = _bf(B, (Hq + 2 * Hkv) * D)  # rows strided like the fused qkv buffer
    out = torch.empty(B, Hq * D, dtype=torch.bfloat16, device=DEV)
    ws = ops.DecodeWorkspace(B, Hq, D, 4, DEV)
    scale = 1 / math.sqrt(D)
    ops.paged_decode_attention(q, kc, vc, bt, ctx, scale, out, ws, part_tokens=512, Hq=Hq)
    expect = ref.paged_decode(q[:, :Hq * D].reshape(B, Hq, D), kc, vc, bt, ctx, scale)
    torch.testing.assert_close(out.float().view(B, Hq, D), expect.float(), atol=2e-2, rtol=2e-2)


@pytest.fixture(params=[0, 2, 3], ids=["nst-default", "nst2", "nst3"])
def prefill_ring(request):
    """LDS ring slots of the prefill kernel: default per head dim, 2, 3."""
    ops.native().set_prefill_stages(request.param)
    yield request.param
    ops.native().set_prefill_stages(0)


@pytest.fixture(params=[4, 8], ids=["w4", "w8"])
def prefill_waves(request, monkeypatch):
    """Waves per prefill workgroup at head dim 128 (the tile list follows)."""
    monkeypatch.setenv("LMX_PREFILL_WAVES", str(request.param))
    yield request.param


@pytest.mark.parametrize("Hq,Hkv,D", [(32, 8, 128), (8, 1, 128), (12, 12, 64), (4, 4, 128),
                                     (28, 4, 128), (7, 1, 64), (24, 8, 128)])
def test_paged_prefill_varlen_with_prefix(Hq, Hkv, D, prefill_ring, prefill_waves):
    qlens = [1, 70, 33, 256]
    prefix = [0, 40, 0, 100]
    ctxs = [q + p for q, p in zip(qlens, prefix)]
    S = len(qlens)
    NB = sum(math.ceil(c / 32) for c in ctxs) + 2
    kc, vc = _cache(NB, Hkv, D)
    bt = _random_tables(S, ctxs, NB)
    cu = torch.tensor([0] + list(torch.cumsum(torch.tensor(qlens), 0)), dtype=torch.int32,
                      device=DEV)
    T = int(cu[-1])
    q = _bf(T, (Hq + 2 * Hkv) * D)
    qpt = ops.prefill_q_per_tile(Hq, Hkv, D)
    tiles = []
    for s, ql in enumerate(qlens):
        for q0 in range(0, ql, qpt):
            tiles += [s, q0]
    tiles = torch.tensor(tiles, dtype=torch.int32, device=DEV)
    ctx = torch.tensor(ctxs, dtype=torch.int32, device=DEV)
    out = torch.zeros(T, Hq * D, dtype=torch.bfloat16, device=DEV)
    scale = 1 / math.sqrt(D)
    ops.paged_prefill_attention(q, kc, vc, bt, cu, ctx, tiles, scale, out, causal=True, Hq=Hq)
    expect = ref.paged_prefill(q[:, :Hq * D].reshape(T, Hq, D), kc, vc, bt, cu, ctx, scale)
    torch.testing.assert_close(out.float().view(T, Hq, D), expect.float(), atol=2e-2, rtol=2e-2)
    # bidirectional (encoder) mode
    out2 = torch.zeros_like(out)
    ops.paged_prefill_attention(q, kc, vc, bt, cu, ctx, tiles, scale, out2, causal=False, Hq=Hq)
    expect2 = ref.paged_prefill(q[:, :Hq * D].reshape(T, Hq, D), kc, vc, bt, cu, ctx, scale,
                                causal=False)
    torch.testing.assert_close(out2.float().view(T, Hq, D), expect2.float(), atol=2e-2, rtol=2e-2)


@pytest.mark.gpu
def test_paged_decode_dispatch_order_and_loop_modes():
    """The persistent grid (default, one partition per sequence), the
    longest-first order (ops.decode_order), the pipelined loop form (mode 1)
    and the one-workgroup-per-segment grid (mode 4) give bitwise the same
    result."""
    Hq, Hkv, D = 32, 8, 128
    ctxs = [535, 791, 1, 640, 33, 700, 64, 600] * 4
    B = len(ctxs)
    NB = sum(math.ceil(c / 32) for c in ctxs) + 4
    kc, vc = _cache(NB, Hkv, D)
    bt = _random_tables(B, ctxs, NB)
    ctx = torch.tensor(ctxs, dtype=torch.int32, device=DEV)
    q = _bf(B, (Hq + 2 * Hkv) * D)
    scale = 1 / math.sqrt(D)
    base = torch.empty(B, Hq * D, dtype=torch.bfloat16, device=DEV)
    ops.paged_decode_attention(q, kc, vc, bt, ctx, scale, base, Hq=Hq)
    order = torch.from_numpy(ops.decode_order(ctxs)).to(DEV)
    assert sorted(order.tolist()) == list(range(B)) and ctxs[int(order[0])] == 791
    got = torch.empty_like(base)
    ops.paged_decode_attention(q, kc, vc, bt, ctx, scale, got, Hq=Hq, order=order)
    assert torch.equal(got, base)
    for mode in (1, 4, 9, 10):   # pipelined pages; one workgroup per segment; register ring
        try:
            ops.native().set_decode_mode(mode)
            ops.paged_decode_attention(q, kc, vc, bt, ctx, scale, got, Hq=Hq, order=order)
        finally:
            ops.native().set_decode_mode(0)
        if mode >= 9:   # PV as two 16x16x16 MFMAs: fp32 sums in another order
            torch.testing.assert_close(got.float(), base.float(), atol=4e-3, rtol=1e-2)
        else:
            assert torch.equal(got, base), mode
    expect = ref.paged_decode(q[:, :Hq * D].reshape(B, Hq, D), kc, vc, bt, ctx, scale)
    torch.testing.assert_close(base.float().view(B, Hq, D), expect.float(), atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("Hq,Hkv,D", [(32, 8, 128), (8, 1, 128), (16, 16, 64), (28, 4, 128)])
@pytest.mark.parametrize("parts", [1, 4])
@pytest.mark.parametrize("mode", [0, 1, 4, 9, 10])
def test_paged_decode_fused_rope(Hq, Hkv, D, parts, mode):
    """K2 + K5 fused into K4 (rope=...): the kernel rotates q in registers and
    writes the step's rotated k / transposed v into the cache itself.  Same
    output and cache as rope_and_cache followed by the plain decode kernel,
    and as the fp32 reference; padding rows (slot -1, context 1) write nothing."""
    ctxs = [535, 791, 1, 33, 32, 700, 1024, 64, 2000, 17]
    B = len(ctxs)
    NB = sum(math.ceil(c / 32) for c in ctxs) + 4
    kc, vc = _cache(NB, Hkv, D)
    bt = _random_tables(B, ctxs, NB)
    ctx = torch.tensor(ctxs, dtype=torch.int32, device=DEV)
    pos = (ctx - 1).to(torch.int32)
    slots = torch.tensor([int(bt[b, (c - 1) // 32]) * 32 + (c - 1) % 32 for b, c in enumerate(ctxs)],
                         dtype=torch.int32, device=DEV)
    slots[2] = -1                        # a padding row of a captured bucket
    cs = ref.rope_cos_sin(4096, D, 500000.0, DEV)
    qkv = _bf(B, (Hq + 2 * Hkv) * D)
    scale = 1 / math.sqrt(D)
    ws = ops.DecodeWorkspace(B, Hq, D, parts, DEV) if parts > 1 else None
    order = torch.from_numpy(ops.decode_order(ctxs)).to(DEV)
    # unfused: rope/cache kernel, then the decode kernel on the rotated rows
    q_u, kc_u, vc_u = qkv.clone(), kc.clone(), vc.clone()
    ops.rope_and_cache(q_u, pos, cs, Hq, Hkv, D, slots, kc_u, vc_u, tile_from=B)
    out_u = torch.empty(B, Hq * D, dtype=torch.bfloat16, device=DEV)
    out_f = torch.empty_like(out_u)
    q_f, kc_f, vc_f = qkv.clone(), kc.clone(), vc.clone()
    try:
        ops.native().set_decode_mode(mode)
        ops.paged_decode_attention(q_u, kc_u, vc_u, bt, ctx, scale, out_u, ws, 256, Hq=Hq,
                                   order=order)
        ops.paged_decode_attention(q_f, kc_f, vc_f, bt, ctx, scale, out_f, ws, 256, Hq=Hq,
                                   order=order, rope=(pos, cs, slots))
    finally:
        ops.native().set_decode_mode(0)
    torch.cuda.synchronize()
    assert torch.equal(q_f, qkv)                      # the fused kernel leaves the rows alone
    assert torch.equal(vc_f, vc_u)
    torch.testing.assert_close(kc_f.float(), kc_u.float(), atol=1e-2, rtol=1e-2)
    torch.testing.assert_close(out_f.float(), out_u.float(), atol=1e-2, rtol=1e-2)
    # fp32 reference of the whole step
    q0, kc0, vc0 = qkv.cpu(), kc.cpu(), vc.cpu()
    ref.rope_cache(q0, pos.cpu(), cs.cpu(), Hq, Hkv, D, slots.cpu(), kc0, vc0, False)
    expect = ref.paged_decode(q0[:, :Hq * D].reshape(B, Hq, D), kc0, vc0, bt.cpu(), ctx.cpu(),
                              scale)
    live = [b for b in range(B) if b != 2]
    torch.testing.assert_close(out_f.float().cpu().view(B, Hq, D)[live], expect.float()[live],
                               atol=2e-2, rtol=2e-2)


def test_paged_decode_spike_rescale():
    """Force the online-softmax rescale: one key scores far above the rest in a
    late page (guide §5.4 rule 26)."""
    Hq, Hkv, D, c = 32, 8, 128, 1500
    NB = 64
    kc, vc = _cache(NB, Hkv, D)
    bt = _random_tables(1, [c], NB)
    q = _bf(1, (Hq + 2 * Hkv) * D)
    blk = int(bt[0, 1400 // 32])
    kc[blk, :, 1400 % 32, :] = (q[0, :Hq * D].view(Hkv, Hq // Hkv, D)[:, 0, :] * 8).to(kc.dtype)
    ctx = torch.tensor([c], dtype=torch.int32, device=DEV)
    out = torch.empty(1, Hq * D, dtype=torch.bfloat16, device=DEV)
    ws = ops.DecodeWorkspace(1, Hq, D, 8, DEV)
    ops.paged_decode_attention(q, kc, vc, bt, ctx, 1 / math.sqrt(D), out, ws, 256, Hq=Hq)
    expect = ref.paged_decode(q[:, :Hq * D].reshape(1, Hq, D), kc, vc, bt, ctx, 1 / math.sqrt(D))
    torch.testing.assert_close(out.float().view(1, Hq, D), expect.float(), atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("Hq,Hkv,D", [(32, 8, 128), (12, 12, 64)])
@pytest.mark.parametrize("causal", [True, False])
def test_paged_prefill_lazy_rescale(Hq, Hkv, D, causal):
    """The prefill softmax raises its running max only past a threshold (guide
    T13).  Force the rescale branch: key 700 scores far above every other key
    for the queries after it (and, bidirectional, for all of them), in a late
    tile.  The shipped threshold and threshold 0 (rescale on every growth)
    agree to rounding and both match the fp32 reference (guide §5.4 rule 26)."""
    L, S = 900, 2
    NB = S * math.ceil(L / 32) + 2
    kc, vc = _cache(NB, Hkv, D)
    bt = _random_tables(S, [L] * S, NB)
    cu = torch.tensor([0, L, 2 * L], dtype=torch.int32, device=DEV)
    ctx = torch.tensor([L] * S, dtype=torch.int32, device=DEV)
    q = _bf(S * L, (Hq + 2 * Hkv) * D)
    G = Hq // Hkv
    # key 700 of sequence 0 = 6 x (query 800's head-0 vector of each kv group)
    qv = q[800, :Hq * D].view(Hkv, G, D)[:, 0, :]
    blk = int(bt[0, 700 // 32])
    kc[blk, :, 700 % 32, :] = (qv * 6).to(kc.dtype)
    qpt = ops.prefill_q_per_tile(Hq, Hkv, D)
    tiles = torch.tensor([v for s_ in range(S) for q0 in range(0, L, qpt) for v in (s_, q0)],
                         dtype=torch.int32, device=DEV)
    scale = 1 / math.sqrt(D)
    outs = []
    try:
        for thr in (8.0, 0.0):
            ops.native().set_prefill_rescale_thr(thr)
            o = torch.zeros(S * L, Hq * D, dtype=torch.bfloat16, device=DEV)
            ops.paged_prefill_attention(q, kc, vc, bt, cu, ctx, tiles, scale, o, causal=causal,
                                        Hq=Hq)
            outs.append(o)
    finally:
        ops.native().set_prefill_rescale_thr(8.0)
    torch.testing.assert_close(outs[0].float(), outs[1].float(), atol=1e-2, rtol=1e-2)
    expect = ref.paged_prefill(q[:, :Hq * D].reshape(S * L, Hq, D), kc, vc, bt, cu, ctx, scale,
                               causal=causal)
    torch.testing.assert_close(outs[0].float().view(S * L, Hq, D), expect.float(), atol=2e-2,
                               rtol=2e-2)


def _params(B, t=1.0, k=0, p=1.0):
    f = lambda v, dt: torch.full((B,), v, dtype=dt, device=DEV)
    return (f(t, torch.float32), f(k, torch.int32), f(p, torch.float32),
            torch.arange(B, dtype=torch.int64, device=DEV) * 7 + 1, f(0, torch.int32))


@pytest.mark.parametrize("fn", ["sample", "sample_race"])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_sample_greedy_and_logprob(dtype, fn):
    B, V = 5, 128256
    lg = (torch.randn(B, V, device=DEV) * 3).to(dtype)
    tok, lp = getattr(ops, fn)(lg, *_params(B, t=0.0))
    assert torch.equal(tok.long(), lg.float().argmax(-1))
    ref_lp = torch.log_softmax(lg.float(), -1).gather(1, tok.long()[:, None])[:, 0]
    torch.testing.assert_close(lp, ref_lp, atol=1e-3, rtol=1e-3)


@pytest.mark.parametrize("fn", ["sample", "sample_race"])
def test_sample_distribution_matches_softmax(fn):
    V, B = 8, 4096
    base = torch.tensor([2.0, 1.0, 0.5, 0.0, -1.0, -2.0, 0.3, 1.5], device=DEV)
    lg = base.repeat(B, 1)
    t, k, p, _, off = _params(B, t=0.7)
    seeds = torch.arange(B, dtype=torch.int64, device=DEV) * 977 + 3
    tok, _ = getattr(ops, fn)(lg, t, k, p, seeds, off)
    freq = torch.bincount(tok.long(), minlength=V).float() / B
    expect = torch.softmax(base / 0.7, -1)
    assert torch.allclose(freq, expect, atol=0.03), (freq, expect)


@pytest.mark.parametrize("fn", ["sample", "sample_race"])
def test_sample_distribution_full_vocab(fn):
    """A draw over the whole 128k vocabulary (inverse CDF; the race form's
    Gumbel keys): five hot tokens placed
    in different threads' element sets (a flat tail carries the remaining
    ~0.7 % of the mass) are drawn at their softmax frequencies; with top_p
    0.8 only the nucleus (mass strictly above < 0.8) is ever drawn."""
    V, B = 128256, 4096
    hot = torch.tensor([3, 40001, 77777, 100000, 128255], device=DEV)
    lg = torch.zeros(V, device=DEV)
    lg[hot] = torch.tensor([16.0, 15.5, 15.0, 14.0, 13.0], device=DEV)
    lg = lg.repeat(B, 1).to(torch.bfloat16)
    seeds = torch.arange(B, dtype=torch.int64, device=DEV) * 131 + 7
    t, k, p, _, off = _params(B, t=1.0)
    tok, _ = getattr(ops, fn)(lg, t, k, p, seeds, off)
    probs = torch.softmax(lg[0].float(), -1)
    cnt = torch.bincount(tok.long(), minlength=V).float() / B
    torch.testing.assert_close(cnt[hot], probs[hot], atol=0.03, rtol=0)
    t, k, p, _, off = _params(B, t=1.0, p=0.8)
    tok, _ = getattr(ops, fn)(lg, t, k, p, seeds, off)
    order = probs.argsort(descending=True)
    above = torch.cumsum(probs[order], 0) - probs[order]
    nucleus = set(order[above < 0.8].tolist())
    assert nucleus == set(hot[:3].tolist())
    assert set(tok.tolist()) == nucleus


@pytest.mark.parametrize("fn", ["sample", "sample_race"])
def test_sample_top_k_top_p_support(fn):
    V, B = 1000, 2048
    lg = torch.randn(V, device=DEV).repeat(B, 1) * 2
    order = lg[0].argsort(descending=True)
    seeds = torch.arange(B, dtype=torch.int64, device=DEV) * 31 + 5
    t, k, p, _, off = _params(B, t=1.0, k=5)
    tok, _ = getattr(ops, fn)(lg, t, k, p, seeds, off)
    assert set(tok.tolist()) <= set(order[:5].tolist())
    assert len(set(tok.tolist())) > 1
    # nucleus: expected support = smallest prefix with mass >= 0.5
    probs = torch.softmax(lg[0], -1)[order]
    above = torch.cumsum(probs, 0) - probs
    nucleus = set(order[above < 0.5].tolist())
    t, k, p, _, off = _params(B, t=1.0, p=0.5)
    tok, _ = getattr(ops, fn)(lg, t, k, p, seeds, off)
    assert set(tok.tolist()) <= nucleus
    # determinism: same seeds -> same tokens
    tok2, _ = getattr(ops, fn)(lg, t, k, p, seeds, off)
    assert torch.equal(tok, tok2)


@pytest.mark.parametrize("rows,I", [(77, 14336 // 4), (256, 14336), (3, 16), (1, 8 * 257)])
def test_silu_mul_gelu_mul(rows, I):
    x = _bf(rows, 2 * I)
    torch.testing.assert_close(ops.silu_mul(x).float(), ref.silu_mul(x).float(), atol=2e-2,
                               rtol=2e-2)
    torch.testing.assert_close(ops.gelu_mul(x).float(), ref.gelu_mul(x).float(), atol=2e-2,
                               rtol=2e-2)


def test_embed_gather_vocab_shard():
    table = _bf(1000, 256)
    ids = torch.randint(0, 2000, (50,), device=DEV, dtype=torch.int32)
    y = ops.embed_gather(table, ids, vocab_start=500)
    local = ids.long() - 500
    own = (local >= 0) & (local < 1000)
    expect = table[local.clamp(0, 999)] * own[:, None].to(table.dtype)
    assert torch.equal(y, expect)


def test_mean_pool_l2_matryoshka():
    h = _bf(100, 768)
    cu = torch.tensor([0, 10, 11, 100], dtype=torch.int32, device=DEV)
    for dims in (768, 256):
        y = ops.mean_pool_l2(h, cu, dims)
        torch.testing.assert_close(y, ref.mean_pool_l2(h, cu, dims), atol=1e-3, rtol=1e-3)


@pytest.mark.parametrize("d", [768, 1024])
def test_mean_pool_l2_row_tiled(d):
    """Two-stage (row-tiled + atomics) path: long sequences, an empty one, a
    sequence boundary inside a row tile, and padding rows past cu[-1]."""
    lens = [512, 0, 45, 1, 700, 300]
    cu = torch.tensor([0] + list(torch.tensor(lens).cumsum(0)), dtype=torch.int32, device=DEV)
    h = _bf(int(cu[-1]) + 40, d)
    assert 2 * (len(lens)) < (h.shape[0] + ops.POOL_ROWS - 1) // ops.POOL_ROWS
    for dims, norm in ((d, True), (256, True), (d, False)):
        y = ops.mean_pool_l2(h, cu, dims, norm)
        torch.testing.assert_close(y, ref.mean_pool_l2(h, cu, dims, norm), atol=1e-3, rtol=1e-3)


@pytest.mark.parametrize("M,N,K", [(1, 128, 64), (77, 768, 768), (256, 2304, 768),
                                   (1000, 3072, 768), (130, 768, 3072), (512, 4096, 4096)])
@pytest.mark.parametrize("act", [0, 1, 2, 4])
def test_gemm_nt(M, N, K, act):
    a, w, b = _bf(M, K), _bf(N, K, scale=K ** -0.5), _bf(N)
    r = _bf(M, N)
    y = ops.gemm_nt(a, w, b, act, residual=r)
    expect = ref.gemm_nt(a, w, b, act, r)
    torch.testing.assert_close(y.float(), expect.float(), atol=3e-2, rtol=3e-2)


def test_gemm_nt_identity_asymmetric():
    """A = I with an asymmetric B catches a transposed C write (guide §3)."""
    n = 128
    a = torch.eye(n, device=DEV, dtype=torch.bfloat16)
    w = torch.arange(n * n, device=DEV, dtype=torch.float32).view(n, n).remainder(97).to(
        torch.bfloat16)
    y = ops.gemm_nt(a, w)
    assert torch.equal(y, w.t().contiguous())


@pytest.mark.gpu
@pytest.mark.parametrize("Hq,Hkv,D", [(32, 8, 128), (12, 12, 64)])
def test_paged_prefill_long_multi_tile(Hq, Hkv, D):
    """Several 64-key LDS tiles per workgroup, a ragged last page and a long
    cached prefix (chunked prefill continuation)."""
    qlens, prefix = [517, 190], [300, 0]
    ctxs = [q + p for q, p in zip(qlens, prefix)]
    S = len(qlens)
    NB = sum(math.ceil(c / 32) for c in ctxs) + 3
    kc, vc = _cache(NB, Hkv, D)
    bt = _random_tables(S, ctxs, NB)
    cu = torch.tensor([0] + list(torch.cumsum(torch.tensor(qlens), 0)), dtype=torch.int32,
                      device=DEV)
    T = int(cu[-1])
    q = _bf(T, (Hq + 2 * Hkv) * D)
    qpt = ops.prefill_q_per_tile(Hq, Hkv, D)
    tiles = [v for s, ql in enumerate(qlens) for q0 in range(0, ql, qpt) for v in (s, q0)]
    tiles = torch.tensor(tiles, dtype=torch.int32, device=DEV)
    ctx = torch.tensor(ctxs, dtype=torch.int32, device=DEV)
    scale = 1 / math.sqrt(D)
    for causal in (True, False):
        out = torch.zeros(T, Hq * D, dtype=torch.bfloat16, device=DEV)
        ops.paged_prefill_attention(q, kc, vc, bt, cu, ctx, tiles, scale, out, causal=causal,
                                    Hq=Hq)
        expect = ref.paged_prefill(q[:, :Hq * D].reshape(T, Hq, D), kc, vc, bt, cu, ctx, scale,
                                   causal=causal)
        torch.testing.assert_close(out.float().view(T, Hq, D), expect.float(), atol=2e-2,
                                   rtol=2e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("M", [1, 7, 64, 100, 256])
@pytest.mark.parametrize("N,K,splits", [(384, 1024, 1), (6144, 4096, 2), (1024, 3584, 4),
                                        (640, 2048, 8)])
def test_gemm_splitk_vs_fp32(M, N, K, splits):
    a = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    w = (torch.randn(N, K, device=DEV) * K ** -0.5).to(torch.bfloat16)
    out = ops.gemm_splitk(a, w, splits=splits)
    expect = a.float() @ w.float().t()
    torch.testing.assert_close(out.float(), expect, atol=2e-2, rtol=2e-2)
    # twice in a row: tickets re-armed, slabs reused
    out2 = ops.gemm_splitk(a, w, splits=splits)
    assert torch.equal(out, out2)


@pytest.mark.gpu
def test_gemm_splitk_in_graph_strided_input():
    M, K, N = 48, 4096, 6144
    x = torch.randn(M, K + 64, device=DEV).to(torch.bfloat16)[:, :K]   # row stride K + 64
    w = (torch.randn(N, K, device=DEV) * K ** -0.5).to(torch.bfloat16)
    out = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    ops.gemm_splitk(x, w, out)                       # allocates the workspace eagerly
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        ops.gemm_splitk(x, w, out)
    torch.cuda.current_stream().wait_stream(s)
    with torch.cuda.graph(g, stream=s):
        ops.gemm_splitk(x, w, out)
    x.copy_(torch.randn(M, K + 64, device=DEV).to(torch.bfloat16)[:, :K])
    g.replay()
    torch.cuda.synchronize()
    torch.testing.assert_close(out.float(), x.float() @ w.float().t(), atol=2e-2, rtol=2e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("M", [5, 128, 333])
def test_gemm_nt_fused_swiglu(M):
    K, I = 768, 3072
    a = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    w = (torch.randn(2 * I, K, device=DEV) * K ** -0.5).to(torch.bfloat16)
    out = ops.gemm_nt(a, ops.interleave_gate_up(w), act=ops.ACT_SWIGLU)
    y = a.float() @ w.float().t()
    expect = torch.nn.functional.silu(y[:, :I]) * y[:, I:]
    torch.testing.assert_close(out.float(), expect, atol=2e-2, rtol=2e-2)



@pytest.mark.gpu
def test_apply_penalties_vs_reference():
    B, V, W = 37, 128256, 64
    g = torch.Generator().manual_seed(3)
    logits = (torch.randn(B, V, generator=g) * 3).to(torch.bfloat16)
    win = torch.randint(0, 300, (B, W), generator=g, dtype=torch.int32)   # many repeats
    win[::3, : W // 2] = -1                                               # short windows
    ngen = torch.randint(0, W + 1, (B,), generator=g, dtype=torch.int32)
    pen = torch.stack([torch.rand(B, generator=g) + 0.5, torch.rand(B, generator=g),
                       torch.rand(B, generator=g)], 1).float()
    pen[::5] = torch.tensor([1.0, 0.0, 0.0])                              # neutral rows
    expect = ref.apply_penalties(logits.float().clone(), win, ngen, pen)
    got = ops.apply_penalties(logits.cuda(), win.cuda(), ngen.cuda(), pen.cuda()).float().cpu()
    torch.testing.assert_close(got, expect.to(torch.bfloat16).float(), atol=1e-2, rtol=1e-2)
    off = torch.zeros(1, dtype=torch.int32, device=DEV)
    lg = logits.cuda()
    assert torch.equal(ops.apply_penalties(lg.clone(), win.cuda(), ngen.cuda(), pen.cuda(), on=off),
                       lg)


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", list(range(len(ops.DGEMM_CONFIGS))) +
                         [c | 32 for c in (1, 4, 6, 13, 19, 23)])
@pytest.mark.parametrize("M", [1, 37, 64, 130, 256])
def test_dgemm_configs_vs_fp32(cfg, M):
    """K11 decode GEMM: every tile configuration (and some with the
    non-temporal weight stream, cfg | DGEMM_NT), split-K 1/2/4, every
    epilogue (plain; SwiGLU with the LDS hand-off, epi 1; SwiGLU on 16-column
    pairs, epi 3, where the wave tile allows), against an fp32 PyTorch
    reference (rows past M masked); 96-column tiles take N = 1536."""
    bm, bn = ops.DGEMM_CONFIGS[cfg & ops.DGEMM_CFG_MASK]
    K, N = 1024, {96: 1536}.get(bn, 2 * 1024)
    a = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    w = (torch.randn(N, K, device=DEV) * K ** -0.5).to(torch.bfloat16)
    y = a.float() @ w.float().t()
    for s in (1, 2, 4):
        out = ops.dgemm(a, w, cfg, s)
        torch.testing.assert_close(out.float(), y, atol=2e-2, rtol=2e-2)
        out2 = ops.dgemm(a, w, cfg, s)            # tickets re-armed by the last arriver
        assert torch.equal(out, out2)
        # fused SwiGLU on weights interleaved per BN-column tile
        I = N // 2
        wil = w.view(2, I // (bn // 2), bn // 2, K).transpose(0, 1).reshape(N, K).contiguous()
        g = torch.nn.functional.silu(y[:, :I]) * y[:, I:]
        out3 = ops.dgemm(a, wil, cfg, s, epi=1)
        torch.testing.assert_close(out3.float(), g, atol=2e-2, rtol=2e-2)
        if ops.swiglu16_ok(cfg):
            out4 = ops.dgemm(a, ops.interleave_gate_up(w, ops.SWIGLU16), cfg, s, epi=3)
            torch.testing.assert_close(out4.float(), g, atol=2e-2, rtol=2e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("cfg", [6, 1, 0, 19, 23, 26, 31])
@pytest.mark.parametrize("M,N,K,groups", [(1, 2048, 1024, 0), (37, 2048, 1024, 7),
                                          (128, 2048, 1024, 0), (130, 2048, 2048, 300),
                                          (256, 2048, 1024, 64)])
def test_dgemm_stream_k_vs_fp32(cfg, M, N, K, groups):
    """K11 stream-K form (cfg | DGEMM_SK): equal runs of K-steps per
    workgroup crossing tile boundaries (runs shorter and longer than a tile,
    a grid smaller than the tile count), pieces summed by the reduction
    kernel, against an fp32 reference; bitwise repeatable."""
    bm, bn = ops.DGEMM_CONFIGS[cfg]
    if bn == 96:
        N = 1536
    a = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    w = (torch.randn(N, K, device=DEV) * K ** -0.5).to(torch.bfloat16)
    y = a.float() @ w.float().t()
    for c in (cfg | ops.DGEMM_SK, cfg | ops.DGEMM_SK | ops.DGEMM_NT):
        out = ops.dgemm(a, w, c, groups)
        torch.testing.assert_close(out.float(), y, atol=2e-2, rtol=2e-2)
        assert torch.equal(out, ops.dgemm(a, w, c, groups))


@pytest.mark.gpu
def test_dgemm_in_graph_strided_input_long_k():
    M, K, N = 96, 14336, 4096
    x = torch.randn(M, K + 64, device=DEV).to(torch.bfloat16)[:, :K]   # row stride K + 64
    w = (torch.randn(N, K, device=DEV) * K ** -0.5).to(torch.bfloat16)
    out = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    ops.dgemm(x, w, 0, 8, out=out)                # allocates the workspace eagerly
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        ops.dgemm(x, w, 0, 8, out=out)
    torch.cuda.current_stream().wait_stream(s)
    with torch.cuda.graph(g, stream=s):
        ops.dgemm(x, w, 0, 8, out=out)
    for _ in range(3):
        x.copy_(torch.randn(M, K + 64, device=DEV).to(torch.bfloat16)[:, :K])
        g.replay()
        torch.cuda.synchronize()
        torch.testing.assert_close(out.float(), x.float() @ w.float().t(), atol=2e-2, rtol=2e-2)


@pytest.mark.gpu
@pytest.mark.parametrize("cfg,splits", [(0, 8), (5, 1), (1, 4), (13, 16), (1 | 32, 4), (23, 16), (21, 8),
                                       (31, 2), (20, 2)])
def test_dgemm_partials_into_rmsnorm(cfg, splits):
    """K11 partials-only epilogue summed by the residual-add RMSNorm equals the
    fp32 reference of norm(residual + x @ w^T)."""
    M, K, N = 200, 4096, 4096
    a = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    w = (torch.randn(N, K, device=DEV) * K ** -0.5).to(torch.bfloat16)
    g = (1.0 + 0.1 * torch.randn(N, device=DEV)).to(torch.bfloat16)
    res = torch.randn(M, N, device=DEV).to(torch.bfloat16)
    r_ref = (res.float() + a.float() @ w.float().t()).to(torch.bfloat16)
    expect = ref.rms_norm(r_ref.float(), g.float(), 1e-5)
    p = ops.dgemm_partials(a, w, cfg, splits)
    assert p.slabs.shape == (splits, M, N)
    torch.testing.assert_close(p.sum(), a.float() @ w.float().t(), atol=2e-2, rtol=2e-2)
    r2 = res.clone()
    out = ops.rms_norm(p, g, 1e-5, residual=r2)
    torch.testing.assert_close(r2.float(), r_ref.float(), atol=3e-2, rtol=2e-2)
    torch.testing.assert_close(out.float(), expect.float(), atol=3e-2, rtol=3e-2)


@pytest.mark.parametrize("M,N,K", [(256, 512, 192), (300, 768, 768), (1000, 2304, 768),
                                   (4096, 1024, 1024), (77, 256, 4096)])
@pytest.mark.parametrize("grid", [0, 3])
def test_pgemm_vs_fp32(M, N, K, grid):
    """K13 persistent large-M GEMM (csrc/kernels/pgemm.hip): plain, bias +
    GELU(erf) (BERT FFN), bias only, SwiGLU on 16-row gate/up pairs, against
    an fp32 PyTorch reference; ragged M (rows >= M dropped by the buffer
    range), grid 3 (several tiles per workgroup: the cross-tile load stream and
    the epilogue stores interleaved into the next tile's first K-step)."""
    a = _bf(M, K)
    w = _bf(N, K, scale=K ** -0.5)
    b = _bf(N)
    y = a.float() @ w.float().t()
    before = ops.PGEMM_CALLS[0]
    out = ops.pgemm(a, w, grid=grid)
    torch.testing.assert_close(out.float(), y, atol=2e-2, rtol=2e-2)
    assert torch.equal(out, ops.pgemm(a, w, grid=grid))            # deterministic
    yb = y + b.float()
    torch.testing.assert_close(ops.pgemm(a, w, bias=b, grid=grid).float(), yb, atol=2e-2,
                               rtol=2e-2)
    torch.testing.assert_close(ops.pgemm(a, w, bias=b, act=ops.ACT_GELU_ERF, grid=grid).float(),
                               torch.nn.functional.gelu(yb), atol=2e-2, rtol=2e-2)
    wil = ops.interleave_gate_up(w, 16)
    I = N // 2
    g = torch.nn.functional.silu(y[:, :I]) * y[:, I:]
    torch.testing.assert_close(ops.pgemm(a, wil, act=ops.ACT_SWIGLU, grid=grid).float(), g,
                               atol=2e-2, rtol=2e-2)
    # strided output rows (a view into a wider buffer)
    big = torch.zeros(M, N + 64, dtype=torch.bfloat16, device=DEV)
    ops.pgemm(a, w, out=big[:, 32:32 + N], grid=grid)
    torch.testing.assert_close(big[:, 32:32 + N].float(), y, atol=2e-2, rtol=2e-2)
    assert big[:, :32].abs().sum().item() == 0 and big[:, 32 + N:].abs().sum().item() == 0
    assert ops.PGEMM_CALLS[0] - before == 6


@pytest.mark.parametrize("M,N,K", [(256, 512, 192), (300, 768, 768), (1000, 2304, 768),
                                   (4096, 1024, 4096), (77, 256, 4096)])
@pytest.mark.parametrize("grid", [0, 3])
def test_pgemm_residual_epilogue_vs_fp32(M, N, K, grid):
    """K13 residual epilogue (pre-norm block): residual = bf16(residual +
    bf16(a @ w^T)) in place -- the rounding of the separate residual-add pass
    it replaces -- against the fp32 product; ragged M (rows >= M untouched),
    a residual that is a strided view into a wider buffer (columns outside it
    untouched), several tiles per workgroup (grid 3), repeatable."""
    a = _bf(M, K)
    w = _bf(N, K, scale=K ** -0.5)
    big = _bf(M + 5, N + 64)
    keep = big.clone()
    res = big[:M, 32:32 + N]
    want = (res.float() + (a.float() @ w.float().t()).to(torch.bfloat16).float()).to(torch.bfloat16)
    before = ops.PGEMM_CALLS[0]
    out = ops.pgemm(a, w, grid=grid, residual=res)
    assert out.data_ptr() == res.data_ptr()
    torch.testing.assert_close(res.float(), want.float(), atol=3e-2, rtol=2e-2)
    assert torch.equal(big[:, :32], keep[:, :32]) and torch.equal(big[:, 32 + N:], keep[:, 32 + N:])
    assert torch.equal(big[M:], keep[M:])
    # same inputs again: bitwise the same result
    res2 = keep[:M, 32:32 + N].clone()
    ops.pgemm(a, w, grid=grid, residual=res2)
    assert torch.equal(res2, res)
    assert ops.PGEMM_CALLS[0] - before == 2


@pytest.mark.parametrize("M,N,K", [(256, 1024, 4096), (200, 768, 1536), (37, 512, 512),
                                   (300, 512, 1024)])
@pytest.mark.parametrize("splits", [1, 2, 3, 4])
def test_pgemm_sk_vs_fp32(M, N, K, splits):
    """K13-SK (split-K 256x256 decode tile): in-kernel ticketed combine (plain,
    GELU, 16-row SwiGLU), the fp32 partials form summed by the norm, ragged M,
    repeated calls (counters re-armed), bitwise deterministic."""
    if not ops.pgemm_sk_supported(M, N, K, splits):
        pytest.skip("shape outside K13-SK")
    a = _bf(M, K)
    w = _bf(N, K, scale=K ** -0.5)
    y = a.float() @ w.float().t()
    out = ops.pgemm_sk(a, w, splits)
    torch.testing.assert_close(out.float(), y, atol=2e-2, rtol=2e-2)
    for _ in range(3):
        assert torch.equal(out, ops.pgemm_sk(a, w, splits))
    torch.testing.assert_close(ops.pgemm_sk(a, w, splits, act=ops.ACT_GELU).float(),
                               torch.nn.functional.gelu(y, approximate="tanh"), atol=2e-2, rtol=2e-2)
    wil = ops.interleave_gate_up(w, 16)
    g = torch.nn.functional.silu(y[:, :N // 2]) * y[:, N // 2:]
    torch.testing.assert_close(ops.pgemm_sk(a, wil, splits, act=ops.ACT_SWIGLU).float(), g,
                               atol=2e-2, rtol=2e-2)
    p = ops.pgemm_sk(a, w, splits, epi=2)
    assert p.slabs.shape == (splits, M, N)
    torch.testing.assert_close(p.sum(), y, atol=2e-3, rtol=2e-3)
    if splits not in (1, 2, 4, 8, 16):
        return                               # rmsnorm_slabs instantiates power-of-two S
    # through the residual-add RMSNorm that consumes partials
    res = _bf(M, N)
    nw = _bf(N)
    ref_res = res.float() + y
    ref_out = ref_res * torch.rsqrt(ref_res.pow(2).mean(-1, keepdim=True) + 1e-5) * nw.float()
    got = ops.rms_norm(p, nw, 1e-5, residual=res)
    torch.testing.assert_close(res.float(), ref_res, atol=3e-2, rtol=2e-2)
    torch.testing.assert_close(got.float(), ref_out, atol=5e-2, rtol=3e-2)


def test_linear_large_m_runs_k13(monkeypatch):
    """Prefill-sized projections: ops.linear / linear_swiglu route M >= 512 to
    K13 (LMX_LARGE_GEMM=k13), bias and the 16-row gate/up SwiGLU included,
    and match the library / GLU-kernel path."""
    monkeypatch.setenv("LMX_LARGE_GEMM", "k13")
    M, K, N = 1100, 1024, 2048          # above ops.ROWS_SPLIT_MAX: one K13 product
    x = _bf(M, K)
    w = _bf(N, K, scale=K ** -0.5)
    b = _bf(N)
    before = ops.PGEMM_CALLS[0]
    y = ops.linear(x, w, bias=b)
    torch.testing.assert_close(y.float(), torch.nn.functional.linear(x, w, b).float(),
                               atol=2e-2, rtol=2e-2)
    wil = ops.interleave_gate_up(w, ops.SWIGLU16)
    g = ops.linear_swiglu(x, wil, ops.SWIGLU16)
    ref_g = ops.silu_mul(torch.nn.functional.linear(x, wil), block=ops.SWIGLU16)
    torch.testing.assert_close(g.float(), ref_g.float(), atol=2e-2, rtol=2e-2)
    assert ops.PGEMM_CALLS[0] - before == 2
    monkeypatch.setenv("LMX_LARGE_GEMM", "lib")
    ops.linear(x, w)
    assert ops.PGEMM_CALLS[0] - before == 2


def test_linear_decode_lm_head_runs_k13_sk():
    """The decode table's K13-SK entry (config "sk": Llama-3-8B LM head at
    M 129..256) is what ops.linear runs there, and it matches the library."""
    N, K = 128256, 4096
    assert ops.sk_choice(256, N, K) == 1 and ops.sk_choice(128, N, K) is None
    x = _bf(256, K)
    w = _bf(N, K, scale=K ** -0.5)
    before = ops.PGEMM_CALLS[0]
    y = ops.linear(x, w)
    assert ops.PGEMM_CALLS[0] - before == 1
    torch.testing.assert_close(y.float(), torch.nn.functional.linear(x, w).float(),
                               atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("lead", [0, 5])
@pytest.mark.parametrize("Hq,Hkv,D", [(32, 8, 128), (12, 12, 64), (28, 4, 128)])
def test_prefill_fused_q_rope(Hq, Hkv, D, lead, prefill_waves):
    """Prefill rows with the q rotation inside the attention kernel: the
    rope/cache kernel with skip_q leaves q untouched and writes the same K/V
    cache; the attention over the unrotated q with rope=(positions, cos_sin)
    matches the fp32 reference over the rotated q.  ``lead`` > 0: the batch
    starts with decode-style rows (the Llama mixed-step call: the whole qkv,
    every row's position, cu_q starting at ``lead``), so the kernel must take
    each query's position by its absolute row."""
    qlens, prefix = [70, 33, 256], [40, 0, 100]
    ctxs = [q + p for q, p in zip(qlens, prefix)]
    S = len(qlens)
    NB = sum(math.ceil(c / 32) for c in ctxs) + 2
    kc, vc = _cache(NB, Hkv, D)
    bt = _random_tables(S, ctxs, NB)
    T = sum(qlens)
    qkv = _bf(T, (Hq + 2 * Hkv) * D)
    pos = torch.cat([torch.arange(p, p + q) for q, p in zip(qlens, prefix)]).to(torch.int32).to(DEV)
    # slot of the token at position p of sequence s: page bt[s][p // 32], offset p % 32
    slots = torch.cat([bt[s].long()[torch.arange(p, p + q, device=DEV) // 32] * 32 +
                       torch.arange(p, p + q, device=DEV) % 32
                       for s, (q, p) in enumerate(zip(qlens, prefix))]).to(torch.int32)
    cs = ref.rope_cos_sin(4096, D, 500000.0, DEV)
    kc2, vc2, qkv2 = kc.clone(), vc.clone(), qkv.clone()
    q0 = qkv[:, :Hq * D].clone()
    ops.rope_and_cache(qkv, pos, cs, Hq, Hkv, D, slots, kc, vc, tile_from=0, skip_q=True)
    ops.rope_and_cache(qkv2, pos, cs, Hq, Hkv, D, slots, kc2, vc2, tile_from=0)
    assert torch.equal(qkv[:, :Hq * D], q0)              # q left unrotated
    assert torch.equal(kc, kc2) and torch.equal(vc, vc2)
    cu = torch.tensor([0] + list(torch.cumsum(torch.tensor(qlens), 0)), dtype=torch.int32,
                      device=DEV)
    qpt = ops.prefill_q_per_tile(Hq, Hkv, D)
    tiles = torch.tensor([v for s, ql in enumerate(qlens) for q0 in range(0, ql, qpt)
                          for v in (s, q0)], dtype=torch.int32, device=DEV)
    ctx = torch.tensor(ctxs, dtype=torch.int32, device=DEV)
    scale = 1 / math.sqrt(D)
    out = torch.zeros(T, Hq * D, dtype=torch.bfloat16, device=DEV)
    if lead:
        # leading rows with their own (unrelated) positions; the prefill
        # kernel must neither read their positions for its rows nor write them
        qkv_l = torch.cat([_bf(lead, qkv.shape[1]), qkv])
        pos_l = torch.cat([torch.randint(0, 4000, (lead,), dtype=torch.int32, device=DEV), pos])
        out_l = torch.zeros(T + lead, Hq * D, dtype=torch.bfloat16, device=DEV)
        ops.paged_prefill_attention(qkv_l, kc, vc, bt, cu + lead, ctx, tiles, scale, out_l,
                                    causal=True, Hq=Hq, rope=(pos_l, cs))
        assert torch.count_nonzero(out_l[:lead]) == 0
        out.copy_(out_l[lead:])
    else:
        ops.paged_prefill_attention(qkv, kc, vc, bt, cu, ctx, tiles, scale, out, causal=True,
                                    Hq=Hq, rope=(pos, cs))
    out2 = torch.zeros_like(out)
    ops.paged_prefill_attention(qkv2, kc2, vc2, bt, cu, ctx, tiles, scale, out2, causal=True,
                                Hq=Hq)
    # same bf16 rounding of the rotated q in both paths
    torch.testing.assert_close(out.float(), out2.float(), atol=1e-2, rtol=1e-2)
    expect = ref.paged_prefill(qkv2[:, :Hq * D].reshape(T, Hq, D), kc2, vc2, bt, cu, ctx, scale)
    torch.testing.assert_close(out.float().view(T, Hq, D), expect.float(), atol=2e-2, rtol=2e-2)


# ---- K14: register-streamed decode GEMM (csrc/kernels/rsgemm.hip) ----
@pytest.mark.parametrize("cfg", [2, 2 | 32, 0, 0 | 32, 2 | 4 | 32, 0 | 4, 2 | 8 | 32])
@pytest.mark.parametrize("M", [256, 200, 129, 17])
def test_rsgemm_vs_fp32(cfg, M):
    """K14 against the fp32 reference: row-major and packed weights, every
    epilogue (bf16 with the in-kernel split-K combine, SwiGLU over 16-row
    gate/up pairs, fp32 partials), split-K 1/2/4, ring shapes D4/D6/D8 with and
    without the non-temporal stream; padded rows (M < 256) never stored."""
    K, N = {3: 3072, 2: 2048}[ops.RS_U[cfg & 3]], 1024   # K slices = whole ring blocks
    a = _bf(M, K)
    w = _bf(N, K, scale=K ** -0.5)
    wp = ops.rsgemm_pack(w)
    y = a.float() @ w.float().t()
    wil = ops.interleave_gate_up(w, ops.SWIGLU16)
    yil = a.float() @ wil.float().t()
    g = (torch.nn.functional.silu(yil.view(M, N // 32, 2, 16)[:, :, 0]) *
         yil.view(M, N // 32, 2, 16)[:, :, 1]).reshape(M, N // 2)
    for s in (1, 2, 4):
        if ops.rsgemm_supported(M, N, K, cfg, s):
            for packed in (False, True):
                out = ops.rsgemm(a, wp if packed else w, cfg, s, packed=packed)
                torch.testing.assert_close(out.float(), y, atol=2e-2, rtol=2e-2)
                assert torch.equal(out, ops.rsgemm(a, wp if packed else w, cfg, s, packed=packed))
        if ops.rsgemm_supported(M, N, K, cfg, s, 3):
            out3 = ops.rsgemm(a, wil, cfg, s, epi=3)
            torch.testing.assert_close(out3.float(), g, atol=2e-2, rtol=2e-2)
        if not ops.rsgemm_supported(M, N, K, cfg, s, 2):
            continue
        p = ops.rsgemm(a, w, cfg, s, epi=2)
        torch.testing.assert_close(p.slabs.sum(0), y, atol=2e-2, rtol=2e-2)


def test_rsgemm_llama_shapes_and_graph():
    """The Llama-3-8B decode shapes at 256 rows (gate/up + SwiGLU S 2, QKV S 8,
    O / down partials S 16) vs fp32, then replayed in a captured graph with new
    activations (tickets re-armed in-kernel, no memset node)."""
    M = 256
    for N, K, epi, s in [(28672, 4096, 3, 2), (6144, 4096, 0, 8), (4096, 4096, 2, 16),
                         (4096, 14336, 2, 16)]:
        cfg = 2 | 4 | 32
        if not ops.rsgemm_supported(M, N, K, cfg, s, epi):
            continue
        a = _bf(M, K)
        w = _bf(N, K, scale=K ** -0.5)
        y = a.float() @ w.float().t()
        if epi == 3:
            y = (torch.nn.functional.silu(y.view(M, N // 32, 2, 16)[:, :, 0]) *
                 y.view(M, N // 32, 2, 16)[:, :, 1]).reshape(M, N // 2)
        r = ops.rsgemm(a, w, cfg, s, epi=epi)
        got = r.slabs.sum(0) if epi == 2 else r.float()
        torch.testing.assert_close(got, y, atol=3e-2, rtol=3e-2)
        if epi == 2:
            continue
        out = torch.empty_like(r)
        st = torch.cuda.Stream()
        st.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(st):
            ops.rsgemm(a, w, cfg, s, epi=epi, out=out)
        torch.cuda.current_stream().wait_stream(st)
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr, stream=st):
            ops.rsgemm(a, w, cfg, s, epi=epi, out=out)
        for _ in range(2):
            a.copy_(_bf(M, K))
            gr.replay()
            torch.cuda.synchronize()
            y = a.float() @ w.float().t()
            if epi == 3:
                y = (torch.nn.functional.silu(y.view(M, N // 32, 2, 16)[:, :, 0]) *
                     y.view(M, N // 32, 2, 16)[:, :, 1]).reshape(M, N // 2)
            torch.testing.assert_close(out.float(), y, atol=3e-2, rtol=3e-2)


@pytest.mark.parametrize("M", [16, 64, 160, 256])
def test_tp8_lm_head_shard_served_hand_written(M):
    """The 70B TP = 8 LM-head shard (padded to 16128 rows) through ``ops.linear``
    at decode batch sizes: the table serves it on K11 (round 5: 1.03-1.37x of
    hipBLASLt below 160 rows, stream-K above), the logits match fp32 and the
    padding rows (zero weights) give zero logits."""
    from llm_mcp_amd.models.weights import vocab_shard
    N, K = vocab_shard(128256, 8), 8192
    assert N == 16128
    w = _bf(N, K, scale=K ** -0.5)
    w[N - 768:] = 0                          # rows past the vocabulary on the last rank
    assert ops.dgemm_choice(M, N, K) is not None, "no K11 entry for the TP8 LM head"
    a = _bf(M, K)
    before = ops.DGEMM_CALLS[0]
    y = ops.linear(a, w)
    assert ops.DGEMM_CALLS[0] == before + 1
    torch.testing.assert_close(y.float(), a.float() @ w.float().t(), atol=3e-2, rtol=3e-2)
    assert y[:, N - 768:].abs().max().item() == 0
