"""The RMSNorm folded into the projections (prefill, TP = 1): gains folded
into QKV / gate-up at load, no norm pass -- the residual epilogues' per-64-column
sums of squares become row scales (ops.row_scale) that QKV and gate/up apply
to their output rows.  On the CPU reference kernels, against the unfolded
forward of the same weights (models/llama.py _norm_fold_step)."""
import numpy as np
import torch

from llm_mcp_amd import ops
from llm_mcp_amd.models import config as mc
from llm_mcp_amd.models.llama import LlamaModel, StepInputs


def _prefill_inputs(cfg, lens):
    BS, D = 32, cfg.head_dim
    nb = sum(-(-n // BS) for n in lens) + 1
    kc = [torch.zeros(nb, cfg.num_kv_heads, BS, D, dtype=torch.bfloat16) for _ in range(cfg.num_layers)]
    vc = [torch.zeros(nb, cfg.num_kv_heads, BS // 4, D, 4, dtype=torch.bfloat16)
          for _ in range(cfg.num_layers)]
    ids = torch.arange(sum(lens), dtype=torch.int32) % 400 + 3
    cu = np.concatenate([[0], np.cumsum(lens)]).astype(np.int32)
    pos = torch.cat([torch.arange(n, dtype=torch.int32) for n in lens])
    pages = [-(-n // BS) for n in lens]
    first = np.concatenate([[0], np.cumsum(pages)])
    bt = torch.zeros(len(lens), max(pages), dtype=torch.int32)
    for i, n in enumerate(pages):
        bt[i, :n] = torch.arange(first[i], first[i] + n, dtype=torch.int32)
    slots = torch.cat([bt[i].long()[torch.arange(n) // BS] * BS + torch.arange(n) % BS
                       for i, n in enumerate(lens)]).to(torch.int32)
    qpt = ops.prefill_q_per_tile(cfg.num_heads, cfg.num_kv_heads, D)
    tiles = np.array([v for s_, n in enumerate(lens) for q0 in range(0, n, qpt) for v in (s_, q0)],
                     np.int32)
    rows = (cu[1:] - 1).astype(np.int64)
    inp = StepInputs(ids, pos, slots, 0, bt, torch.tensor(lens, dtype=torch.int32),
                     torch.from_numpy(cu), torch.from_numpy(tiles), torch.from_numpy(rows),
                     int(cu[-1]), len(lens), host={"cu_q": cu, "tiles": tiles, "rows": rows})
    return inp, kc, vc


def test_row_scale_matches_rms():
    x = torch.randn(300, 256).to(torch.bfloat16)
    s = ops.row_scale(1e-5, x=x)
    torch.testing.assert_close(s, torch.rsqrt(x.float().pow(2).mean(-1) + 1e-5))
    part = x.float().pow(2).view(300, 4, 64).sum(-1)
    torch.testing.assert_close(ops.row_scale(1e-5, part=part, cols=256), s)


def test_folded_norm_prefill_matches_unfolded(monkeypatch):
    monkeypatch.setenv("LMX_LARGE_GEMM", "k13")     # tiny shapes: K13's tile waves mostly empty
    cfg = mc.resolve("tiny-llama")
    g = torch.Generator().manual_seed(7)
    ref_m = LlamaModel(cfg, "cpu", seed=3)
    for L in ref_m.w["layers"]:           # non-trivial gains
        for k in ("ln1", "ln2"):
            L[k] = (1.0 + 0.2 * torch.randn(cfg.hidden_size, generator=g)).to(torch.bfloat16)
    lens = [300, 231, 40]                  # T >= 512: the K13 regime of the folded norm
    inp, kc, vc = _prefill_inputs(cfg, lens)
    want = ref_m.forward(inp, kc, vc, None).float()

    m = LlamaModel(cfg, "cpu", seed=3, weights={
        "embed": ref_m.w["embed"], "norm": ref_m.w["norm"], "lm_head": ref_m.w["lm_head"],
        "layers": [dict(L) for L in ref_m.w["layers"]]})
    for L in m.w["layers"]:               # what the GPU load does (LlamaModel.__init__)
        for gk, wk in (("ln1", "wqkv"), ("ln2", "w_gate_up")):
            L[wk] = (L[wk].float() * L[gk].float()[None, :]).to(L[wk].dtype)
            L[gk] = torch.ones_like(L[gk])
        L["w_gate_up"] = ops.interleave_gate_up(L["w_gate_up"], ops.SWIGLU16)
    m.gu_block, m.norm_folded = ops.SWIGLU16, True
    assert m._norm_fold_step(inp.num_tokens, True)
    assert not m._norm_fold_step(200, True)          # decode-sized steps keep the norms
    inp2, kc2, vc2 = _prefill_inputs(cfg, lens)
    got = m.forward(inp2, kc2, vc2, None).float()
    torch.testing.assert_close(got, want, atol=3e-2, rtol=3e-2)
    for a, b in zip(kc, kc2):                         # the same K/V cache
        torch.testing.assert_close(a.float(), b.float(), atol=3e-2, rtol=3e-2)
