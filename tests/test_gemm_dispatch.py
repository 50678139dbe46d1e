"""CPU tests of the measured GEMM dispatch tables (config/dgemm_gfx950.json):
the gate/up interleave block, the K13-SK entries and the large-M backend pick."""
from llm_mcp_amd import ops


def test_swiglu_block_follows_the_largest_batch_bucket(monkeypatch):
    # 64-row buckets won at BN 128 (cfg 16 -> (64, 128)), the 128-row bucket at
    # BN 256 (cfg 11 -> (128, 256)): one interleave for all, the big batch wins
    table = {(57344, 8192, 1): [(64, 16 | ops.DGEMM_NT, 1), (128, 11, 1), (256, -1, 0)]}
    monkeypatch.setattr(ops, "DGEMM_TABLE", table)
    monkeypatch.setattr(ops, "_SK_TABLE", {})
    monkeypatch.setattr(ops, "_RS_TABLE", {})
    assert ops.swiglu_block(57344, 8192) == 128
    assert ops.dgemm_choice(128, 57344, 8192, epi=1) == (11, 1)
    assert ops.dgemm_choice(200, 57344, 8192, epi=1) is None     # library bucket
    # epi-3 entries (16-row pairs, any tile width) take precedence
    table[(57344, 8192, 3)] = [(128, 17, 1)]
    assert ops.swiglu_block(57344, 8192) == ops.SWIGLU16
    assert ops.swiglu_block(1000, 1000) == 0


def test_sk_choice_and_large_gemm_backend(monkeypatch):
    monkeypatch.setattr(ops, "_SK_TABLE", {(128256, 4096, 0): [(176, 256, 1)],
                                           (4096, 4096, 2): [(129, 256, 3)]})
    assert ops.sk_choice(256, 128256, 4096) == 1
    assert ops.sk_choice(175, 128256, 4096) is None
    assert ops.sk_choice(200, 4096, 4096, epi=2) is None      # S 3: no rmsnorm_slabs instance
    monkeypatch.setattr(ops, "_ENC_TABLE", {(6144, 4096): {"k13_tflops": 1560.0, "lib_tflops": 1600.0},
                                            (768, 3072): {"k13_tflops": 1100.0, "lib_tflops": 1300.0}})
    monkeypatch.delenv("LMX_LARGE_GEMM", raising=False)
    assert ops.large_gemm_backend(16384, 6144, 4096) == "k13"   # within the 5 % margin
    assert ops.large_gemm_backend(16384, 768, 3072) == "lib"
    assert ops.large_gemm_backend(100, 6144, 4096) == "lib"     # decode-sized M
    assert ops.large_gemm_backend(16384, 4096, 4096) == "k13"   # unmeasured
    monkeypatch.setenv("LMX_LARGE_GEMM", "lib")
    assert ops.large_gemm_backend(16384, 6144, 4096) == "lib"


def test_pgemm_sk_cpu_reference_forms():
    """ops.pgemm_sk on CPU tensors (the fp32 reference of the K13-SK forms):
    plain, 16-row SwiGLU pairs, fp32 partials summed by the consumer."""
    import torch
    torch.manual_seed(0)
    a = torch.randn(37, 512).to(torch.bfloat16)
    w = (torch.randn(512, 512) * 512 ** -0.5).to(torch.bfloat16)
    y = a.float() @ w.float().t()
    torch.testing.assert_close(ops.pgemm_sk(a, w, 2).float(), y, atol=2e-2, rtol=2e-2)
    p = ops.pgemm_sk(a, w, 4, epi=2)
    assert isinstance(p, ops.Partials) and p.slabs.shape == (4, 37, 512)
    torch.testing.assert_close(p.sum(), y, atol=1e-4, rtol=1e-4)
    wil = ops.interleave_gate_up(w, ops.SWIGLU16)
    g = torch.nn.functional.silu(y[:, :256]) * y[:, 256:]
    torch.testing.assert_close(ops.pgemm_sk(a, wil, 2, act=ops.ACT_SWIGLU).float(), g,
                               atol=2e-2, rtol=2e-2)
    assert not ops.pgemm_sk_supported(37, 500, 512, 2)          # N not a 256 multiple
    assert not ops.pgemm_sk_supported(37, 512, 512, 8)          # one K-step per slice


def test_rsgemm_shape_rules_and_cpu_reference(monkeypatch, tmp_path):
    """K14 (csrc/kernels/rsgemm.hip) shape rules, its measured-table dispatch
    ("rs" entries) and the CPU reference forms of its three epilogues."""
    import json
    import torch
    from llm_mcp_amd import ops
    # ring blocks: D4 (cfg 2) takes K slices of 2 K64 steps, D6 (cfg 0) of 3
    assert ops.rsgemm_supported(256, 28672, 4096, 2 | 4, 2)
    assert not ops.rsgemm_supported(256, 28672, 4096, 0 | 4, 2)    # 32 K64 steps % 3
    assert ops.rsgemm_supported(256, 4096, 14336, 2 | 32, 16, 2)   # 14 K64 steps
    assert not ops.rsgemm_supported(257, 4096, 4096, 2 | 4, 1)
    assert not ops.rsgemm_supported(256, 4000, 4096, 2 | 4, 1)
    # all-rows tiles: the partials epilogue only (bf16 / SwiGLU spill there, not built)
    assert not ops.rsgemm_supported(256, 28672, 4096, 2, 2)
    assert not ops.rsgemm_supported(256, 28672, 4096, 2, 2, 3)
    assert ops.rsgemm_supported(256, 28672, 4096, 2, 2, 2)
    table = {"entries": [], "rs": [{"N": 28672, "K": 4096, "epi": 3, "m_min": 129,
                                    "m_max": 256, "cfg": 102, "splits": 2},
                                   {"N": 4096, "K": 4096, "epi": 2, "m_min": 129,
                                    "m_max": 256, "cfg": 102, "splits": 16},
                                   {"N": 4096, "K": 14336, "epi": 2, "m_min": 129,
                                    "m_max": 256, "cfg": 38, "splits": 8}]}
    p = tmp_path / "t.json"
    p.write_text(json.dumps(table))
    monkeypatch.setenv("LMX_DGEMM_TABLE", str(p))
    monkeypatch.setattr(ops, "_RS_TABLE", None)
    assert ops.rs_choice(256, 28672, 4096, 3) == (102, 2)           # row-major entry
    assert ops.rs_choice(128, 28672, 4096, 3) is None
    assert ops.rs_choice(200, 4096, 4096, 2) == (102, 16)
    assert ops.rs_choice(200, 4096, 4096, 0) is None
    # a packed-weight entry applies only to a weight rs_prepare packed
    assert ops.rs_choice(256, 4096, 14336, 2) is None
    w_cpu = torch.zeros(4096, 14336, dtype=torch.bfloat16)
    assert not ops.rs_prepare(w_cpu)                                # CPU weights: never packed
    assert ops.rs_choice(256, 4096, 14336, 2, w=w_cpu) is None
    monkeypatch.setattr(ops, "_RS_TABLE", None)
    a = torch.randn(5, 2048).to(torch.bfloat16)
    w = (torch.randn(512, 2048) * 0.02).to(torch.bfloat16)
    y = a.float() @ w.float().t()
    torch.testing.assert_close(ops.rsgemm(a, w, 2 | 4, 2).float(), y, atol=2e-2, rtol=2e-2)
    part = ops.rsgemm(a, w, 2, 4, epi=2)
    assert part.slabs.shape == (4, 5, 512)
    torch.testing.assert_close(part.slabs.sum(0), y, atol=1e-3, rtol=1e-3)
    g = ops.rsgemm(a, w, 2 | 4, 1, epi=3)
    yy = y.view(5, 16, 2, 16)
    torch.testing.assert_close(g.float(), (torch.nn.functional.silu(yy[:, :, 0]) * yy[:, :, 1])
                               .reshape(5, 256), atol=2e-2, rtol=2e-2)


def test_pgemm_residual_cpu_reference_and_gate(monkeypatch):
    """ops.pgemm(residual=) on CPU (the reference of K13's residual epilogue:
    residual = bf16(residual + a @ w^T), in place, returned) and the gate that
    sends only prefill-sized, K13-claimed shapes there (CPU tensors, decode
    shapes and LMX_RESIDUAL_EPILOGUE=0 keep the separate residual-add pass)."""
    import torch
    torch.manual_seed(0)
    a = torch.randn(37, 512).to(torch.bfloat16)
    w = (torch.randn(256, 512) * 512 ** -0.5).to(torch.bfloat16)
    r = torch.randn(37, 256).to(torch.bfloat16)
    want = (r.float() + a.float() @ w.float().t()).to(torch.bfloat16)
    out = ops.pgemm(a, w, residual=r)
    assert out is r
    torch.testing.assert_close(r.float(), want.float(), atol=1e-2, rtol=1e-2)
    assert not ops.residual_gemm_ok(a, w, r)              # CPU tensors
    assert not ops.residual_gemm_ok(a, w, None)
    monkeypatch.setattr(ops, "RESIDUAL_EPILOGUE", False)
    assert not ops.residual_gemm_ok(a, w, r)


def test_rs_prepare_all_packs_whole_shapes_or_none(monkeypatch):
    import torch
    """ADVICE r4: the K14 packed-copy budget (LMX_RS_PACK_GB) is decided per
    weight SHAPE, all or nothing -- never the first layers of a shape packed and
    the rest left row-major."""
    packed = []

    def attach(w):
        w._lmx_rs_packed = w
        ops._RS_PACKED_BYTES[0] += w.numel() * w.element_size()
        packed.append(w)

    monkeypatch.setattr(ops, "_rs_wants_packed", lambda w: True)
    monkeypatch.setattr(ops, "_rs_attach_packed", attach)
    monkeypatch.setattr(ops, "_RS_PACKED_BYTES", [0])
    mib = 1 << 20
    small = [torch.empty(256, 1024, dtype=torch.bfloat16) for _ in range(4)]      # 0.5 MiB each
    big = [torch.empty(1024, 1024, dtype=torch.bfloat16) for _ in range(4)]       # 2 MiB each
    other = [torch.empty(512, 1024, dtype=torch.bfloat16) for _ in range(2)]      # 1 MiB each
    layers = [t for trio in zip(small, big) for t in trio] + other
    res = ops.rs_prepare_all(layers, budget_gb=5 * mib / 2**30)
    assert res == {(256, 1024): True, (1024, 1024): False, (512, 1024): True}
    assert all(ops._rs_packed_of(w) is not None for w in small + other)
    assert all(ops._rs_packed_of(w) is None for w in big)          # 8 MiB: none of them
    assert ops._RS_PACKED_BYTES[0] == 4 * mib


def test_rows_split_for_cu_starved_decode_batches(monkeypatch):
    """256 < M <= 1024 rows on a narrow projection (fewer than 128 K13 tiles)
    of a packed-only weight runs as equal <= 256-row pieces on K14; wide
    products (gate/up, LM head) and prefill-sized batches stay one product.
    A row-major weight there takes the library: K13's tile waves would be
    mostly empty (k13_wave_fill)."""
    import torch
    assert ops.rows_split(256, 4096) == 0                 # the decode kernels' own range
    assert ops.rows_split(512, 4096) == 256
    assert ops.rows_split(300, 6144) == 150               # two equal pieces, not 256 + 44
    assert ops.rows_split(640, 4096) == 214
    assert ops.rows_split(512, 28672) == 0                # 224 tiles: K13 fills the chip
    assert ops.rows_split(1024, 8192) == 0                # 128 tiles
    assert ops.rows_split(1100, 4096) == 0                # prefill-sized
    # given K: only for a packed-only weight (a row-major one takes the library)
    assert ops.rows_split(512, 4096, 14336) == 0
    assert ops.rows_split(512, 4096, 14336, 0, torch.empty(0)) == 0
    x = torch.randn(300, 64)
    w = torch.randn(32, 64)
    y = ops._by_rows(x, ops.rows_split(300, 4096), 32, lambda xs, o: torch.mm(xs, w.t(), out=o))
    torch.testing.assert_close(y, x @ w.t())
    assert ops.k13_wave_fill(512, 4096) == 32 / 256
    assert ops.k13_wave_fill(512, 28672) == 224 / 256
    assert ops.k13_wave_fill(768, 28672) == 336 / 512
    assert ops.k13_wave_fill(36864, 4096) == 1.0
    monkeypatch.delenv("LMX_LARGE_GEMM", raising=False)
    monkeypatch.setattr(ops, "_ENC_TABLE", {})
    assert ops.large_gemm_backend(512, 4096, 14336) == "lib"       # 32 tiles
    assert ops.large_gemm_backend(1024, 6144, 4096) == "lib"       # 96 of 256
    assert ops.large_gemm_backend(1536, 6144, 4096) == "k13"       # above ROWS_SPLIT_MAX
    assert ops.large_gemm_backend(2304, 6144, 4096) == "k13"       # 216 of 256
    assert ops.large_gemm_backend(512, 28672, 4096, ops.ACT_SWIGLU) == "k13"
    assert ops.large_gemm_backend(36864, 4096, 14336) == "k13"
    monkeypatch.setenv("LMX_LARGE_GEMM", "k13")
    assert ops.large_gemm_backend(512, 4096, 14336) == "k13"

