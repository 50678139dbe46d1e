"""Dense (non-paged, full-recompute) fp32 reference of the Llama forward, used
to check the engine's paged / incremental / batched execution."""
import math

import torch

from llm_mcp_amd.ops import dense_weight, ref


def dense_logits(model, tokens: list[int]) -> torch.Tensor:
    cfg, w = model.cfg, model.w
    Hq, Hkv, D = model.Hq, model.Hkv, model.D
    dev = w["embed"].device
    ids = torch.tensor(tokens, device=dev)
    pos = torch.arange(len(tokens), device=dev, dtype=torch.int32)
    x = w["embed"][ids].float()
    for L in w["layers"]:
        h = ref.rms_norm(x, L["ln1"].float(), cfg.rms_eps)
        qkv = h @ L["wqkv"].float().t()
        if "bqkv" in L:
            qkv = qkv + L["bqkv"].float()
        T = qkv.shape[0]
        q = qkv[:, :Hq * D].view(T, Hq, D)
        k = qkv[:, Hq * D:(Hq + Hkv) * D].view(T, Hkv, D)
        v = qkv[:, (Hq + Hkv) * D:].view(T, Hkv, D)
        if "q_norm" in L:     # Qwen3 per-head q/k RMSNorm
            q = ref.head_norm(q, L["q_norm"], cfg.rms_eps)
            k = ref.head_norm(k, L["k_norm"], cfg.rms_eps)
        q = ref.apply_rope(q, pos, model.cos_sin).float()
        k = ref.apply_rope(k, pos, model.cos_sin).float()
        a = ref.attention_dense(q, k, v, 1.0 / math.sqrt(D), 0).reshape(T, Hq * D)
        x = x + a @ L["wo"].float().t()
        h = ref.rms_norm(x, L["ln2"].float(), cfg.rms_eps)
        gu = h @ dense_weight(L["w_gate_up"]).float().t()
        if getattr(model, "gu_block", 0):      # fused-SwiGLU weight layout (K11)
            from llm_mcp_amd.ops import deinterleave_gate_up
            gu = deinterleave_gate_up(gu, model.gu_block)
        x = x + ref.silu_mul(gu) @ dense_weight(L["w_down"]).float().t()
    h = ref.rms_norm(x[-1:], w["norm"].float(), cfg.rms_eps)
    return (h @ w["lm_head"].float().t())[0]


def dense_greedy(model, prompt: list[int], n: int) -> list[int]:
    toks = list(prompt)
    out = []
    for _ in range(n):
        j = int(torch.argmax(dense_logits(model, toks)))
        out.append(j)
        toks.append(j)
    return out


def assert_greedy_consistent(model, prompt: list[int], out: list[int], tol: float = 0.05):
    """Each generated token must be (near-)argmax of the dense fp32 logits on
    the engine's own trajectory (bf16 execution may flip exact near-ties)."""
    toks = list(prompt)
    for i, j in enumerate(out):
        lg = dense_logits(model, toks)
        m = float(lg.max())
        assert float(lg[j]) >= m - tol * max(1.0, abs(m)), (i, j, float(lg[j]), m)
        toks.append(j)
