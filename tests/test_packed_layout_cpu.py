"""The packed weight layout (K14's rsgemm_pack, also read by K13 with WP)
and its inverse, on the CPU: ops.rs_unpack undoes a plain-torch model of the
packing kernel (csrc/kernels/rsgemm.hip rsgemm_pack_kernel)."""
import torch

from llm_mcp_amd import ops


def _pack_model(w: torch.Tensor) -> torch.Tensor:
    """Element-wise statement of the packed order: run (tile T, wave w, K32
    block kb, half j) is 64 lanes x 8 values, lane l holding
    W[256 T + 32 w + 16 j + (l & 15)][32 kb + 8 (l >> 4) .. + 8]."""
    N, K = w.shape
    out = torch.empty(N * K, dtype=w.dtype)
    KB = K // 32
    c = 0
    for T in range(N // 256):
        for wv in range(8):
            for kb in range(KB):
                for j in range(2):
                    for lane in range(64):
                        n = T * 256 + wv * 32 + j * 16 + (lane & 15)
                        k = kb * 32 + (lane >> 4) * 8
                        out[c * 8:(c + 1) * 8] = w[n, k:k + 8]
                        c += 1
    return out.view(N, K)


def test_rs_unpack_inverts_the_packing():
    w = torch.arange(512 * 64, dtype=torch.float32).view(512, 64).to(torch.bfloat16)
    p = _pack_model(w)
    assert not torch.equal(p, w)
    assert torch.equal(ops.rs_unpack(p), w)


def test_packed_only_marker_and_dense_weight():
    w = torch.randn(256, 64).to(torch.bfloat16)
    p = _pack_model(w)
    assert not ops.is_packed_only(p) and ops.dense_weight(w) is w
    p._lmx_packed_only = True
    assert ops.is_packed_only(p)
    assert torch.equal(ops.dense_weight(p), w)
    # a packed-only weight is its own packed copy for the K14 dispatch
    assert ops._rs_packed_of(p) is p


def test_rs_default_configurations():
    # 64-row tiles to 64 rows, 128-row beyond; enough K slices for >= 192 workgroups
    cfg, s = ops.rs_default(16, 28672, 4096, 3)
    assert cfg & ops.RS_BM64 and s == 2 and ops.rsgemm_supported(16, 28672, 4096, cfg, s, 3)
    cfg, s = ops.rs_default(200, 4096, 14336, 2)
    assert cfg & ops.RS_BM128 and 2 * 16 * s >= 192
    assert ops.rsgemm_supported(200, 4096, 14336, cfg, s, 2)
    assert ops.rs_default(300, 4096, 14336, 0) is None       # K14 stops at 256 rows
