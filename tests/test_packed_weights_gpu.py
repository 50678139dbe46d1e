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
    else:
        assert M <= 256
