"""Classic BERT encoders for ``/v1/embeddings``: mxbai-embed-large,
bge-large/base, snowflake-arctic-embed and other BertModel checkpoints.

The reference serves whatever embedding model its Ollama hosts carry
(``OLLAMA_EMBED_MODEL``, worker/llm_worker/main.py:248; ``/api/embed``,
core/internal/api/handlers.go:1942-2015); besides nomic-bert (models/nomic_bert.py)
the common Ollama embedders are BERT-architecture models.  Here they run
in-process on the same gfx950 kernels as the nomic encoder:

  x = LayerNorm(word[ids] + pos[p] + type[0])                     (K10 gather, LN)
  per layer (post-norm):
      QKV = gemm_nt(x, Wqkv, bias)                                (K7, fused bias)
      K/V scattered into a per-batch paged scratch cache          (K5)
      bidirectional varlen attention on the paged prefill kernel  (K3, causal=0)
      h = LayerNorm(gemm_nt(attn, Wo, bias, residual=x))          (K7 + fused residual)
      x = LayerNorm(gemm_nt(gelu(gemm_nt(h, W1, b1)), W2, b2, residual=h))
          (exact-erf GELU fused into the first FFN GEMM's epilogue)
  pooling: CLS row (mxbai / bge / arctic) or masked mean (MiniLM-style), then
  Matryoshka truncation + L2 normalisation in the pooling kernel (K9).
Sequences are packed (cu_seqlens), never padded.
"""
from __future__ import annotations

import math

import numpy as np

import torch

from .. import ops
from .config import BertConfig

PAGE = 32


class BertModel:
    def __init__(self, cfg: BertConfig, device="cuda", dtype=torch.bfloat16, seed: int = 0,
                 weights: dict | None = None):
        self.cfg = cfg
        self.device = torch.device(device)
        self.dtype = dtype
        self.H, self.D = cfg.num_heads, cfg.head_dim
        self.scale = 1.0 / math.sqrt(self.D)
        self.w = weights or self._random_weights(seed)

    def _random_weights(self, seed):
        cfg, dev, dt = self.cfg, self.device, self.dtype
        g = torch.Generator(device=dev)
        g.manual_seed(seed + 91)
        d, I = cfg.hidden_size, cfg.intermediate_size

        def rnd(*shape, std=0.02):
            t = torch.empty(shape, dtype=dt, device=dev)
            t.normal_(0.0, std, generator=g)
            return t

        ones = lambda: torch.ones(d, dtype=dt, device=dev)
        layers = [{"wqkv": rnd(3 * d, d), "bqkv": rnd(3 * d), "wo": rnd(d, d), "bo": rnd(d),
                   "ln1_w": ones(), "ln1_b": rnd(d), "w1": rnd(I, d), "b1": rnd(I),
                   "w2": rnd(d, I), "b2": rnd(d), "ln2_w": ones(), "ln2_b": rnd(d)}
                  for _ in range(cfg.num_layers)]
        return {"word": rnd(cfg.vocab_size, d, std=1.0), "pos": rnd(cfg.max_position, d),
                "type": rnd(cfg.type_vocab_size, d), "emb_ln_w": ones(), "emb_ln_b": rnd(d),
                "layers": layers}

    def weight_bytes(self) -> int:
        n = sum(t.numel() * t.element_size() for k, t in self.w.items() if k != "layers")
        for L in self.w["layers"]:
            n += sum(t.numel() * t.element_size() for t in L.values())
        return n

    def _linear(self, x, w, b=None, act=0, residual=None):
        """Projection + bias (+ GELU) on the backend ops.encoder_backend picks
        for the shape (K13 by default).  Returns (y, residual still to add):
        the K7 epilogue fuses the residual, K13 and the library leave it to
        the following LayerNorm's fused residual add."""
        if x.is_cuda:
            kind, _ = ops.encoder_backend(w.shape[0], w.shape[1], act, b is not None)
            if kind == "k13" and ops.pgemm_operands_ok(x, w):
                # bias + GELU in K13's epilogue; the residual goes to the next LayerNorm
                return ops.pgemm(x, w, bias=b, act=act), residual
            if kind == "lib" or not ops.gemm_nt_supported(w.shape[0], w.shape[1]):
                y = torch.nn.functional.linear(x, w, b)
                if act == ops.ACT_GELU_ERF:
                    y = torch.nn.functional.gelu(y)
                return y, residual
            return ops.gemm_nt(x, w, b, act, residual=residual), None
        from ..ops import ref
        return ref.gemm_nt(x, w, b, act, residual), None

    @torch.no_grad()
    def forward(self, ids: torch.Tensor, cu: torch.Tensor, lens: list[int],
                dims: int | None = None, normalize: bool = True) -> torch.Tensor:
        """ids int32 [T] packed, cu int32 [S+1] -> fp32 [S, dims] embeddings."""
        cfg, w = self.cfg, self.w
        H, D, d = self.H, self.D, cfg.hidden_size
        T, S = ids.numel(), len(lens)
        dev = self.device
        ln = np.asarray(lens, dtype=np.int64)
        if int(ln.max()) > cfg.max_position:
            raise ValueError(f"sequence longer than {cfg.max_position} positions")
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
        mask = np.arange(maxp)[None, :] < pages[:, None]
        bt_np[mask] = np.arange(NB, dtype=np.int32)
        meta = torch.from_numpy(np.concatenate([slots, within, tiles, cu_h[:-1]]).astype(np.int32))
        meta = meta.pin_memory().to(dev, non_blocking=True) if dev.type == "cuda" else meta
        slots_t, pos_t = meta[:T], meta[T:2 * T]
        tiles_t, first_t = meta[2 * T:2 * T + tiles.size], meta[2 * T + tiles.size:]
        bt = torch.from_numpy(bt_np).to(dev, non_blocking=True)
        ctx = torch.tensor(lens, dtype=torch.int32).to(dev, non_blocking=True)
        kc = torch.zeros((NB, H, PAGE, D), dtype=self.dtype, device=dev)
        vc = torch.zeros((NB, H, PAGE // 4, D, 4), dtype=self.dtype, device=dev)   # key-quad

        x = ops.embed_gather(w["word"], ids)
        # absolute position + token-type rows enter as the LayerNorm's fused residual
        pe = (w["pos"].index_select(0, pos_t.long()) + w["type"][0]).contiguous()
        x = ops.layer_norm(x, w["emb_ln_w"], w["emb_ln_b"], cfg.ln_eps, residual=pe)
        attn = torch.empty((T, H * D), dtype=self.dtype, device=dev)
        for L in w["layers"]:
            qkv, _ = self._linear(x, L["wqkv"], L["bqkv"])
            k = qkv[:, d:2 * d].view(T, H, D)
            v = qkv[:, 2 * d:].view(T, H, D)
            ops.kv_write(k, v, slots_t, kc, vc)
            ops.paged_prefill_attention(qkv, kc, vc, bt, cu, ctx, tiles_t, self.scale, attn,
                                        causal=False, Hq=H)
            o, r = self._linear(attn, L["wo"], L["bo"], residual=x)
            h = ops.layer_norm(o, L["ln1_w"], L["ln1_b"], cfg.ln_eps, residual=r)
            f, _ = self._linear(h, L["w1"], L["b1"], act=ops.ACT_GELU_ERF)
            m, r = self._linear(f, L["w2"], L["b2"], residual=h)
            x = ops.layer_norm(m, L["ln2_w"], L["ln2_b"], cfg.ln_eps, residual=r)
        if cfg.pooling == "cls":
            x = x.index_select(0, first_t.long()).contiguous()
            cu = torch.arange(S + 1, dtype=torch.int32, device=dev)
        return ops.mean_pool_l2(x, cu, dims or cfg.embed_dim, normalize)


def load_bert_weights(path: str, cfg: BertConfig, device, dtype=torch.bfloat16) -> dict:
    """HF BertModel safetensors (``bert.`` prefix optional) -> BertModel weights;
    Q/K/V are concatenated into one [3d, d] projection."""
    from .weights import _Reader
    r = _Reader(path)
    pre = "bert." if r.has("bert.embeddings.word_embeddings.weight") else ""

    def t(name):
        return r.rows(pre + name).to(device=device, dtype=dtype).contiguous()

    layers = []
    for i in range(cfg.num_layers):
        b = f"encoder.layer.{i}."
        a = b + "attention."
        layers.append({
            "wqkv": torch.cat([t(a + f"self.{n}.weight") for n in ("query", "key", "value")]),
            "bqkv": torch.cat([t(a + f"self.{n}.bias") for n in ("query", "key", "value")]),
            "wo": t(a + "output.dense.weight"), "bo": t(a + "output.dense.bias"),
            "ln1_w": t(a + "output.LayerNorm.weight"), "ln1_b": t(a + "output.LayerNorm.bias"),
            "w1": t(b + "intermediate.dense.weight"), "b1": t(b + "intermediate.dense.bias"),
            "w2": t(b + "output.dense.weight"), "b2": t(b + "output.dense.bias"),
            "ln2_w": t(b + "output.LayerNorm.weight"), "ln2_b": t(b + "output.LayerNorm.bias")})
    e = "embeddings."
    return {"word": t(e + "word_embeddings.weight"), "pos": t(e + "position_embeddings.weight"),
            "type": t(e + "token_type_embeddings.weight"), "emb_ln_w": t(e + "LayerNorm.weight"),
            "emb_ln_b": t(e + "LayerNorm.bias"), "layers": layers}
