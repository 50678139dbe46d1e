"""The RMSNorm folded into the K13 projections on the GPU (pgemm.hip NRM):
the residual epilogue's per-64-column sums of squares, the row-scale kernel,
and the row-scaled plain / SwiGLU products (row-major and packed W), against
the fp32 reference; then a Llama prefill step through the folded path against
the same step with the norms."""
import dataclasses

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


@pytest.mark.parametrize("M", [512, 700, 1024])
@pytest.mark.parametrize("packed", [False, True])
def test_residual_epilogue_sums_of_squares(M, packed):
    N, K = 1024, 1536
    a = _bf(M, K)
    w = _bf(N, K, scale=K ** -0.5)
    wk = ops.rsgemm_pack(w) if packed else w
    r0 = _bf(M, N)
    r1, r2 = r0.clone(), r0.clone()
    ops.pgemm(a, wk, residual=r1, packed=packed)
    part = torch.full((M, N // 64), float("nan"), device=DEV)
    ops.pgemm(a, wk, residual=r2, packed=packed, ssq=part)
    assert torch.equal(r1, r2)                       # the residual itself is unchanged
    want = r2.float().pow(2).view(M, N // 64, 64).sum(-1)
    torch.testing.assert_close(part, want, atol=1e-3, rtol=1e-4)
    s = ops.row_scale(1e-5, part=part, cols=N)
    torch.testing.assert_close(s, torch.rsqrt(r2.float().pow(2).mean(-1) + 1e-5),
                               atol=1e-5, rtol=1e-4)
    torch.testing.assert_close(ops.row_scale(1e-5, x=r2), s, atol=1e-5, rtol=1e-4)


@pytest.mark.parametrize("M", [512, 777])
@pytest.mark.parametrize("packed", [False, True])
def test_row_scaled_products(M, packed):
    N, K = 1024, 512
    x = _bf(M, K)
    s = torch.rand(M, device=DEV) + 0.5
    w = _bf(N, K, scale=K ** -0.5)
    y = (x.float() @ w.float().t()) * s[:, None]
    got = ops.pgemm(x, ops.rsgemm_pack(w) if packed else w, row_scale=s, packed=packed)
    torch.testing.assert_close(got.float(), y, atol=2e-2, rtol=2e-2)
    wil = ops.interleave_gate_up(w, ops.SWIGLU16)
    yi = ((x.float() @ wil.float().t()) * s[:, None]).view(M, N // 32, 2, 16)
    g = (torch.nn.functional.silu(yi[:, :, 0]) * yi[:, :, 1]).reshape(M, N // 2)
    got3 = ops.pgemm(x, ops.rsgemm_pack(wil) if packed else wil, act=ops.ACT_SWIGLU,
                     row_scale=s, packed=packed)
    torch.testing.assert_close(got3.float(), g, atol=2e-2, rtol=2e-2)


def test_llama_prefill_folded_norm_matches_norm_pass(monkeypatch):
    """A 2-layer Llama-3-8B prefill step of 2,400 tokens (every projection
    fills >= 60 % of K13's tile wave, so all four run on K13): the folded path
    (no norm pass) against the same weights run with the norm kernels."""
    from llm_mcp_amd.models import config as mc
    from llm_mcp_amd.models.llama import LlamaModel
    from tests.test_norm_fold_cpu import _prefill_inputs
    monkeypatch.setenv("LMX_NORM_FOLD", "1")
    cfg = dataclasses.replace(mc.resolve("llama-3-8b"), num_layers=2)
    m = LlamaModel(cfg, DEV, seed=1)
    assert m.norm_folded
    lens = [1400, 700, 300]
    inp, kc, vc = _prefill_inputs(cfg, lens)
    to = lambda t: t.to(DEV) if isinstance(t, torch.Tensor) else t  # noqa: E731
    inp = dataclasses.replace(inp, **{f.name: to(getattr(inp, f.name))
                                      for f in dataclasses.fields(inp) if f.name != "host"})
    kc = [t.to(DEV) for t in kc]
    vc = [t.to(DEV) for t in vc]
    assert m._norm_fold_step(inp.num_tokens, True)
    got = m.forward(inp, kc, vc, None).float()
    monkeypatch.setattr(m, "_norm_fold_step", lambda T, fold: False)
    kc2 = [torch.zeros_like(t) for t in kc]
    vc2 = [torch.zeros_like(t) for t in vc]
    want = m.forward(inp, kc2, vc2, None).float()
    torch.testing.assert_close(got, want, atol=5e-2, rtol=5e-2)
    assert (got.argmax(-1) == want.argmax(-1)).float().mean() >= 0.66
