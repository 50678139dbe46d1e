"""nomic-embed-text (NomicBert) encoder for ``/v1/embeddings`` and embed jobs.

What the reference delegated to Ollama ``/api/embed``
(core/internal/api/handlers.go:1942-2015, worker/llm_worker/main.py:246-261)
runs in-process on the GPU:

  embed_gather(word) + token_type row -> LayerNorm
  per layer (post-norm BERT with rotary and SwiGLU):
      QKV = x . Wqkv^T                                      [T, 3d]
      rope + scatter K/V into a per-batch paged scratch cache (K2/K5)
      bidirectional varlen attention on the paged kernel (K3, causal=0)
      h = LayerNorm(x + attn . Wo^T)                        (fused residual LN)
      g = silu(h . Wgate^T) * (h . Wup^T)                   (SwiGLU in the GEMM epilogue)
      x = LayerNorm(h + g . Wfc2^T)
  masked mean pool + Matryoshka truncation + L2 normalise (K9)

Every projection runs on the hand-written large-M GEMM (K13,
csrc/kernels/pgemm.hip) by default -- ``ops.encoder_backend``; with
LMX_ENCODER_LIBRARY=1 hipBLASLt takes the shapes where the encoder table
(config/dgemm_gfx950.json "encoder", bench/dgemm_bench.py --encoder)
measured it faster -- and the gate/up projection carries the SwiGLU in
K13's epilogue (gate/up rows interleaved per 16 channels).  The sequences of
a batch are packed (cu_seqlens), never padded.
"""
from __future__ import annotations

import math
import os

import numpy as np
import torch

from .. import ops
from ..ops import ref
from .config import NomicBertConfig

PAGE = 32


class NomicBertModel:
    def __init__(self, cfg: NomicBertConfig, device="cuda", dtype=torch.bfloat16, seed: int = 0,
                 weights: dict | None = None):
        self.cfg = cfg
        self.device = torch.device(device)
        self.dtype = dtype
        self.H, self.D = cfg.num_heads, cfg.head_dim
        self.scale = 1.0 / math.sqrt(self.D)
        self.cos_sin = ref.rope_cos_sin(cfg.max_position, self.D, cfg.rope_theta, self.device)
        # q rotation inside the attention kernel: off by default for the
        # encoder (one A/B: 2,674 fused vs 2,760 emb/s unfused on nomic)
        self.fuse_q_rope = os.environ.get("LMX_FUSED_ENCODER_ROPE", "0") == "1"
        self.w = weights or self._random_weights(seed)
        # gate/up rows interleaved for the fused SwiGLU epilogue: per 16
        # channels for K13 (the large-M GEMM; the default), per BN/2 channels
        # of the K11 tile where the encoder table picks K11, else per 64
        # channels (gemm_nt act=3)
        I2, d = self.w["layers"][0]["w_gate_up"].shape
        cuda = self.device.type == "cuda"
        self.gu_k13 = cuda and ops.encoder_backend(I2, d, ops.ACT_SWIGLU)[0] == "k13"
        self.gu_cfg = ops.encoder_choice(I2, d) if cuda and not self.gu_k13 else None
        self.gu_block = (ops.SWIGLU16 if self.gu_k13 else
                         ops.DGEMM_CONFIGS[self.gu_cfg & ops.DGEMM_CFG_MASK][1] // 2
                         if self.gu_cfg is not None else 64)
        for L in self.w["layers"]:
            L.pop("w_gu_il", None)      # always this model's own layout (never a copy's)
            if ops.gemm_nt_supported(*L["w_gate_up"].shape) and I2 // 2 % self.gu_block == 0:
                L["w_gu_il"] = ops.interleave_gate_up(L["w_gate_up"], self.gu_block)

    def _random_weights(self, seed):
        cfg, dev, dt = self.cfg, self.device, self.dtype
        g = torch.Generator(device=dev)
        g.manual_seed(seed + 77)
        d, I = cfg.hidden_size, cfg.intermediate_size

        def rnd(*shape, std=0.02):
            t = torch.empty(shape, dtype=dt, device=dev)
            t.normal_(0.0, std, generator=g)
            return t

        ones = lambda: torch.ones(d, dtype=dt, device=dev)
        zeros = lambda: torch.zeros(d, dtype=dt, device=dev)
        layers = [{"wqkv": rnd(3 * d, d), "wo": rnd(d, d), "w_gate_up": rnd(2 * I, d),
                   "w_down": rnd(d, I), "ln1_w": ones(), "ln1_b": zeros(), "ln2_w": ones(),
                   "ln2_b": zeros()} for _ in range(cfg.num_layers)]
        return {"word": rnd(cfg.vocab_size, d, std=1.0), "type": rnd(cfg.type_vocab_size, d),
                "emb_ln_w": ones(), "emb_ln_b": zeros(), "layers": layers}

    def _linear(self, x, w, residual=None):
        """Plain projection on the backend ops.encoder_backend picks for its
        shape: K13 (default), K11, gemm_nt, or hipBLASLt (LMX_ENCODER_LIBRARY=1
        where measured faster)."""
        kind, cfg = ops.encoder_backend(w.shape[0], w.shape[1]) if x.is_cuda else ("lib", None)
        if kind == "k13" and residual is None and ops.pgemm_operands_ok(x, w):
            return ops.pgemm(x, w)
        if kind == "k11" and residual is None:
            return ops.dgemm(x, w, cfg, 1)
        if kind == "gemm_nt" and ops.gemm_nt_supported(w.shape[0], w.shape[1]):
            return ops.gemm_nt(x, w, residual=residual)
        y = torch.nn.functional.linear(x, w)
        return y if residual is None else y + residual

    @torch.no_grad()
    def forward(self, ids: torch.Tensor, cu: torch.Tensor, lens: list[int],
                dims: int | None = None, normalize: bool = True) -> torch.Tensor:
        """ids int32 [T] packed, cu int32 [S+1] -> fp32 [S, dims] embeddings."""
        cfg, w = self.cfg, self.w
        H, D, d = self.H, self.D, cfg.hidden_size
        T, S = ids.numel(), len(lens)
        dev = self.device
        # per-sequence page-aligned slots in a scratch paged K/V cache, built
        # with array ops (no per-token Python work on the host critical path)
        ln = np.asarray(lens, dtype=np.int64)
        pages = np.maximum(1, -(-ln // PAGE))
        page_off = np.concatenate([[0], np.cumsum(pages)])
        NB = int(page_off[-1])
        cu_h = np.concatenate([[0], np.cumsum(ln)])
        within = np.arange(T, dtype=np.int64) - np.repeat(cu_h[:-1], ln)
        slots = np.repeat(page_off[:-1] * PAGE, ln) + within
        qpt = ops.prefill_q_per_tile(H, H, D)
        nt = -(-ln // qpt)
        tile_seq = np.repeat(np.arange(S), nt)
        tile_q0 = (np.arange(int(nt.sum())) - np.repeat(np.concatenate([[0], np.cumsum(nt)])[:-1],
                                                        nt)) * qpt
        tiles = np.stack([tile_seq, tile_q0], 1).reshape(-1)
        maxp = int(pages.max())
        bt_np = np.zeros((S, maxp), dtype=np.int32)
        col = np.arange(maxp)
        mask = col[None, :] < pages[:, None]
        bt_np[mask] = np.arange(NB, dtype=np.int32)
        meta = torch.from_numpy(np.concatenate([slots, within, tiles]).astype(np.int32))
        meta = meta.pin_memory().to(dev, non_blocking=True) if dev.type == "cuda" else meta
        slots_t, pos_t, tiles_t = meta[:T], meta[T:2 * T], meta[2 * T:]
        bt = torch.from_numpy(bt_np).to(dev, non_blocking=True)
        ctx = torch.tensor(lens, dtype=torch.int32).to(dev, non_blocking=True)
        kc = torch.zeros((NB, H, PAGE, D), dtype=self.dtype, device=dev)
        vc = torch.zeros((NB, H, PAGE // 4, D, 4), dtype=self.dtype, device=dev)   # key-quad

        x = ops.embed_gather(w["word"], ids)
        x = ops.layer_norm(x, w["emb_ln_w"], w["emb_ln_b"], cfg.ln_eps,
                           residual=w["type"][0:1].expand(T, d).contiguous())
        attn = torch.empty((T, H * D), dtype=self.dtype, device=dev)
        for L in w["layers"]:
            qkv = self._linear(x, L["wqkv"])
            # q rotated inside the attention kernel when LMX_FUSED_ENCODER_ROPE=1
            fq = self.fuse_q_rope and qkv.is_cuda
            ops.rope_and_cache(qkv, pos_t, self.cos_sin, H, H, D, slots_t, kc, vc, skip_q=fq)
            ops.paged_prefill_attention(qkv, kc, vc, bt, cu, ctx, tiles_t, self.scale, attn,
                                        causal=False, Hq=H,
                                        rope=(pos_t, self.cos_sin) if fq else None)
            o = self._linear(attn, L["wo"])
            h = ops.layer_norm(o, L["ln1_w"], L["ln1_b"], cfg.ln_eps, residual=x)
            if "w_gu_il" in L and self.gu_k13 and h.is_cuda:
                g = ops.pgemm(h, L["w_gu_il"], act=ops.ACT_SWIGLU)          # K13 + fused SwiGLU
            elif "w_gu_il" in L and self.gu_cfg is not None and h.is_cuda:
                g = ops.dgemm(h, L["w_gu_il"], self.gu_cfg, 1, epi=1)   # K11 + fused K8
            elif "w_gu_il" in L and self.gu_block == 64:   # K8 fused into gemm_nt
                g = ops.gemm_nt(h, L["w_gu_il"], act=ops.ACT_SWIGLU)
            else:
                g = ops.silu_mul(self._linear(h, L["w_gate_up"]))
            m = self._linear(g, L["w_down"])
            x = ops.layer_norm(m, L["ln2_w"], L["ln2_b"], cfg.ln_eps, residual=h)
        return ops.mean_pool_l2(x, cu, dims or cfg.embed_dim, normalize)


def load_nomic_weights(path: str, cfg: NomicBertConfig, device, dtype=torch.bfloat16) -> dict:
    """HF nomic-embed-text(-v1.5) safetensors -> NomicBertModel weights.
    The gated MLP computes fc11(x) * silu(fc12(x)) (fc12 is the gate), so the
    fused projection is [fc12; fc11]."""
    from .weights import _Reader
    r = _Reader(path)

    def t(name):
        return r.rows(name).to(device=device, dtype=dtype).contiguous()

    layers = []
    for i in range(cfg.num_layers):
        b = f"encoder.layers.{i}."
        layers.append({
            "wqkv": t(b + "attn.Wqkv.weight"), "wo": t(b + "attn.out_proj.weight"),
            "w_gate_up": torch.cat([t(b + "mlp.fc12.weight"), t(b + "mlp.fc11.weight")]),
            "w_down": t(b + "mlp.fc2.weight"),
            "ln1_w": t(b + "norm1.weight"), "ln1_b": t(b + "norm1.bias"),
            "ln2_w": t(b + "norm2.weight"), "ln2_b": t(b + "norm2.bias")})
    return {"word": t("embeddings.word_embeddings.weight"),
            "type": t("embeddings.token_type_embeddings.weight"),
            "emb_ln_w": t("emb_ln.weight"), "emb_ln_b": t("emb_ln.bias"), "layers": layers}
