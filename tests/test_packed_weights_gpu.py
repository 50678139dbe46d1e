"""One copy of the MLP weights: a packed-only weight (K14's layout, no
row-major copy) serves every product the Llama forward asks of it -- K14 at
decode batch sizes (table entry or ops.rs_default), K13 with packed W above
256 rows (plain, residual epilogue, SwiGLU) -- against the fp32 reference
and against the same call on the row-major weight."""
import pytest
import torch

from llm_mcp_amd import ops

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(autouse=True)
def _native():
    ops.native()
    torch.manual_seed(0)


def _bf(*shape, scale=1.0):
    return (torch.randn(*shape, device=DEV) * scale).to(torch.bfloat16)


@pytest.mark.parametrize("M", [300, 513, 1024])
@pytest.mark.parametrize("N,K", [(512, 256), (1024, 1536)])
def test_pgemm_packed_w_matches_row_major(M, N, K):
    """K13 with packed W (pgemm.hip WP) is bitwise the row-major K13: the same
    fragments reach the same MFMAs in the same order."""
    a = _bf(M, K)
    w = _bf(N, K, scale=K ** -0.5)
    wp = ops.rsgemm_pack(w)
    y = ops.pgemm(a, w)
    torch.testing.assert_close(y.float(), a.float() @ w.float().t(), atol=2e-2, rtol=2e-2)
    assert torch.equal(ops.pgemm(a, wp, packed=True), y)
    wil = ops.interleave_gate_up(w, ops.SWIGLU16)
    g = ops.pgemm(a, wil, act=ops.ACT_SWIGLU)
    assert torch.equal(ops.pgemm(a, ops.rsgemm_pack(wil), act=ops.ACT_SWIGLU, packed=True), g)
    r0 = _bf(M, N)
    r1, r2 = r0.clone(), r0.clone()
    ops.pgemm(a, w, residual=r1)
    ops.pgemm(a, wp, residual=r2, packed=True)
    assert torch.equal(r1, r2)
    torch.testing.assert_close(r1.float(), (r0.float() + y.float()), atol=3e-2, rtol=2e-2)


@pytest.mark.parametrize("M", [1, 16, 64, 100, 200, 256, 300, 700])
def test_packed_only_weights_every_batch_size(M):
    """linear / linear_swiglu / the residual product on packed-only weights of
    the Llama-3-8B MLP shapes, at decode and prefill batch sizes."""
    d, inter = 4096, 14336
    gu = ops.interleave_gate_up(_bf(2 * inter, d, scale=d ** -0.5), ops.SWIGLU16)
    dn = _bf(d, inter, scale=inter ** -0.5)
    if not (ops.rs_single_ok(gu, True) and ops.rs_single_ok(dn)):
        pytest.skip("the K14 table has no packed entries for these shapes")
    gup, dnp = ops.rs_pack_only(gu), ops.rs_pack_only(dn)
    assert ops.is_packed_only(gup) and torch.equal(ops.dense_weight(gup), gu)
    h = _bf(M, d)
    yil = h.float() @ gu.float().t()
    g = (torch.nn.functional.silu(yil.view(M, inter // 16, 2, 16)[:, :, 0]) *
         yil.view(M, inter // 16, 2, 16)[:, :, 1]).reshape(M, inter)
    a = ops.linear_swiglu(h, gup, ops.SWIGLU16)
    torch.testing.assert_close(a.float(), g, atol=3e-2, rtol=3e-2)
    y = a.float() @ dn.float().t()
    x = ops.linear(a, dnp)
    torch.testing.assert_close(x.float(), y, atol=3e-2, rtol=3e-2)
    p = ops.linear(a, dnp, defer=True)
    got = p.slabs.sum(0) if isinstance(p, ops.Partials) else p.float()
    torch.testing.assert_close(got, y, atol=3e-2, rtol=3e-2)
    res = _bf(M, d)
    if ops.residual_gemm_ok(a, dnp, res):
        r = res.clone()
        ops.pgemm(a, dnp, residual=r)
        torch.testing.assert_close(r.float(), res.float() + y, atol=5e-2, rtol=3e-2)
    else:      # decode sizes, and 257-1024 rows split into decode-kernel pieces
        assert M <= 256 or ops.rows_split(M, d, inter, 0, dnp)


def test_gpu_model_export_round_trip(tmp_path):
    """A TP = 1 model built on the GPU folds its norm gains, interleaves
    gate/up and stores the MLP weights packed-only -- in its own copies: the
    caller's weight dict is untouched, and ``save_hf_llama(model)`` exports
    the served weights (unpacked, de-interleaved) so a model loaded from the
    export serves bitwise the same weights and the same logits."""
    from llm_mcp_amd.models import config as mc
    from llm_mcp_amd.models.llama import LlamaModel, StepInputs
    from llm_mcp_amd.models.weights import load_llama_weights, save_hf_llama
    cfg = mc.resolve("llama-3-8b@L2")
    src = LlamaModel(cfg, DEV, seed=3)
    given = src.export_weights()
    # non-unit gains, so the fold is visible
    for L in given["layers"]:
        L["ln1"] = (1 + 0.1 * torch.randn_like(L["ln1"].float())).to(L["ln1"].dtype)
        L["ln2"] = (1 + 0.1 * torch.randn_like(L["ln2"].float())).to(L["ln2"].dtype)
    before = {(i, k): v for i, L in enumerate(given["layers"]) for k, v in L.items()}
    m = LlamaModel(cfg, DEV, weights=given)
    assert all(given["layers"][i][k] is v for (i, k), v in before.items())
    if any(ops.is_packed_only(v) for L in m.w["layers"] for v in L.values()):
        with pytest.raises(ValueError, match="packed"):
            save_hf_llama(m.w, cfg, str(tmp_path / "raw"))
    save_hf_llama(m, cfg, str(tmp_path))
    m2 = LlamaModel(cfg, DEV, weights=load_llama_weights(str(tmp_path), cfg, DEV))
    e1, e2 = m.export_weights(), m2.export_weights()
    for L1, L2 in zip(e1["layers"], e2["layers"]):
        for k in L1:
            assert torch.equal(L1[k], L2[k]), k
    # and the two models give bitwise the same logits
    T = 7
    ids = torch.arange(100, 100 + T, dtype=torch.int32, device=DEV)
    pos = torch.arange(T, dtype=torch.int32, device=DEV)
    nb = 4
    D = cfg.head_dim
    kc = [torch.zeros(nb, cfg.num_kv_heads, 32, D, dtype=torch.bfloat16, device=DEV)
          for _ in range(cfg.num_layers)]
    vc = [torch.zeros(nb, cfg.num_kv_heads, 8, D, 4, dtype=torch.bfloat16, device=DEV)
          for _ in range(cfg.num_layers)]
    qpt = ops.prefill_q_per_tile(cfg.num_heads, cfg.num_kv_heads, D)
    tiles = torch.tensor([v for q0 in range(0, T, qpt) for v in (0, q0)], dtype=torch.int32,
                         device=DEV)
    inp = StepInputs(ids, pos, pos.clone(), 0, torch.zeros(1, 1, dtype=torch.int32, device=DEV),
                     torch.tensor([T], dtype=torch.int32, device=DEV),
                     torch.tensor([0, T], dtype=torch.int32, device=DEV), tiles,
                     torch.tensor([T - 1], dtype=torch.int64, device=DEV), T, 1)
    l1 = m.forward(inp, kc, vc, None).float()
    l2 = m2.forward(inp, [k.zero_() for k in kc], [v.zero_() for v in vc], None).float()
    assert torch.equal(l1, l2)
