"""Llama weights: HF safetensors loading and Megatron-style TP sharding.

The reference never holds weights (Ollama pulls GGUF blobs out of tree;
worker/llm_worker/main.py:222-261).  Here a GPU worker (or every rank of a TP
group) builds its own shard directly:

* ``load_llama_weights(path, cfg, device, rank, size)`` reads HF
  ``model*.safetensors`` with ``safe_open(...).get_slice`` so each rank only
  touches its slice of every tensor (no full-model host copy per rank; a 70B
  checkpoint is ~140 GB).  q/k/v and gate/up are fused on load into the
  layouts ``LlamaModel.forward`` expects ([q | k | v] rows, [gate | up] rows).
* ``shard_llama(full, cfg, rank, size)`` slices an already materialised
  full (TP=1) weight dict the same way -- used by tests to check that a TP
  group computes exactly what one process computes.

Sharding (per rank r of T):  wqkv rows = this rank's q heads + its kv head
group (kv heads replicated when T > num_kv_heads); wo / w_down split by
input columns (row-parallel, followed by an all-reduce); w_gate_up split by
output rows; lm_head split by vocab rows, each shard zero-padded to
``vocab_shard(V, T)`` rows (ceil(V/T) rounded up to whole 256-row GEMM tiles,
so the all-gather is uniform and the per-rank LM head runs on the hand-written
decode kernels); embeddings and norms replicated.
"""
from __future__ import annotations

import glob
import json
import os

import torch

from .config import LlamaConfig


def vocab_shard(vocab: int, size: int) -> int:
    """Rows of one rank's LM-head shard: ceil(V/T) rounded up to a multiple of
    256 under TP (whole K13 / K14 column tiles: Llama-3's 128256 / 8 = 16032
    -> 16128); the whole vocabulary at T = 1."""
    if size <= 1:
        return vocab
    return -(-(-(-vocab // size)) // 256) * 256


def _geometry(cfg: LlamaConfig, size: int):
    if cfg.num_heads % size or cfg.intermediate_size % size:
        raise ValueError("TP size must divide heads and intermediate size")
    if cfg.num_kv_heads % size and size % cfg.num_kv_heads:
        raise ValueError("TP size incompatible with kv heads")
    hq = cfg.num_heads // size
    hkv = max(1, cfg.num_kv_heads // size)
    rep = max(1, size // cfg.num_kv_heads)
    inter = cfg.intermediate_size // size
    vs = vocab_shard(cfg.vocab_size, size)
    return hq, hkv, rep, inter, vs


def _ranges(cfg: LlamaConfig, rank: int, size: int):
    """Row/col ranges of rank's shard in the unsharded tensors."""
    hq, hkv, rep, inter, vs = _geometry(cfg, size)
    D = cfg.head_dim
    kv0 = (rank // rep) * hkv
    return {
        "q": (rank * hq * D, (rank + 1) * hq * D),
        "kv": (kv0 * D, (kv0 + hkv) * D),
        "i": (rank * inter, (rank + 1) * inter),
        "v": (rank * vs, min(cfg.vocab_size, (rank + 1) * vs)),
        "vs": vs,
    }


def shard_llama(full: dict, cfg: LlamaConfig, rank: int, size: int) -> dict:
    """Slice a full fused weight dict (``LlamaModel`` layout) for one rank."""
    if size == 1:
        return full
    r = _ranges(cfg, rank, size)
    D = cfg.head_dim
    qn, kvn = cfg.num_heads * D, cfg.num_kv_heads * D
    I = cfg.intermediate_size
    layers = []
    for L in full["layers"]:
        wqkv = L["wqkv"]
        q = wqkv[r["q"][0]:r["q"][1]]
        k = wqkv[qn + r["kv"][0]:qn + r["kv"][1]]
        v = wqkv[qn + kvn + r["kv"][0]:qn + kvn + r["kv"][1]]
        gu = L["w_gate_up"]
        extra = {k: L[k] for k in ("q_norm", "k_norm") if k in L}   # per-head: replicated
        if "bqkv" in L:
            b = L["bqkv"]
            extra["bqkv"] = torch.cat([
                b[r["q"][0]:r["q"][1]], b[qn + r["kv"][0]:qn + r["kv"][1]],
                b[qn + kvn + r["kv"][0]:qn + kvn + r["kv"][1]]]).contiguous()
        layers.append({
            **extra,
            "ln1": L["ln1"], "ln2": L["ln2"],
            "wqkv": torch.cat([q, k, v]).contiguous(),
            "wo": L["wo"][:, r["q"][0]:r["q"][1]].contiguous(),
            "w_gate_up": torch.cat([gu[r["i"][0]:r["i"][1]],
                                    gu[I + r["i"][0]:I + r["i"][1]]]).contiguous(),
            "w_down": L["w_down"][:, r["i"][0]:r["i"][1]].contiguous(),
        })
    head = full["lm_head"][r["v"][0]:r["v"][1]]
    if head.shape[0] < r["vs"]:
        head = torch.cat([head, head.new_zeros(r["vs"] - head.shape[0], head.shape[1])])
    return {"embed": full["embed"], "norm": full["norm"], "lm_head": head.contiguous(),
            "layers": layers}


# ----------------------------------------------------------- safetensors ----
def _index(path: str) -> dict[str, str]:
    """tensor name -> file, from model.safetensors.index.json or by scanning."""
    idx = os.path.join(path, "model.safetensors.index.json")
    if os.path.exists(idx):
        with open(idx) as f:
            wm = json.load(f)["weight_map"]
        return {k: os.path.join(path, v) for k, v in wm.items()}
    from safetensors import safe_open
    out = {}
    for fn in sorted(glob.glob(os.path.join(path, "*.safetensors"))):
        with safe_open(fn, framework="pt") as f:
            for k in f.keys():
                out[k] = fn
    if not out:
        raise FileNotFoundError(f"no safetensors files under {path}")
    return out


class _Reader:
    def __init__(self, path: str):
        from safetensors import safe_open
        self._safe_open = safe_open
        self.where = _index(path)
        self.files: dict[str, object] = {}

    def _f(self, name: str):
        fn = self.where.get(name)
        if fn is None:
            raise KeyError(f"checkpoint has no tensor {name!r}")
        if fn not in self.files:
            self.files[fn] = self._safe_open(fn, framework="pt")
        return self.files[fn]

    def has(self, name: str) -> bool:
        return name in self.where

    def rows(self, name: str, lo: int | None = None, hi: int | None = None):
        sl = self._f(name).get_slice(name)
        return sl[lo:hi] if lo is not None else sl[:]

    def cols(self, name: str, lo: int, hi: int):
        return self._f(name).get_slice(name)[:, lo:hi]


def load_llama_weights(path: str, cfg: LlamaConfig, device, rank: int = 0, size: int = 1,
                       dtype=torch.bfloat16) -> dict:
    """Load this rank's shard of a HF Llama checkpoint directory."""
    rd = _Reader(path)
    r = _ranges(cfg, rank, size)
    dev = torch.device(device)

    def put(t):
        return t.to(dtype).contiguous().to(dev, non_blocking=True)

    layers = []
    for i in range(cfg.num_layers):
        p = f"model.layers.{i}."
        q = rd.rows(p + "self_attn.q_proj.weight", *r["q"])
        k = rd.rows(p + "self_attn.k_proj.weight", *r["kv"])
        v = rd.rows(p + "self_attn.v_proj.weight", *r["kv"])
        g = rd.rows(p + "mlp.gate_proj.weight", *r["i"])
        u = rd.rows(p + "mlp.up_proj.weight", *r["i"])
        extra = {}
        if cfg.qk_norm:
            extra["q_norm"] = put(rd.rows(p + "self_attn.q_norm.weight"))
            extra["k_norm"] = put(rd.rows(p + "self_attn.k_norm.weight"))
        if cfg.qkv_bias:
            extra["bqkv"] = put(torch.cat([rd.rows(p + "self_attn.q_proj.bias", *r["q"]),
                                           rd.rows(p + "self_attn.k_proj.bias", *r["kv"]),
                                           rd.rows(p + "self_attn.v_proj.bias", *r["kv"])]))
        layers.append({
            **extra,
            "ln1": put(rd.rows(p + "input_layernorm.weight")),
            "ln2": put(rd.rows(p + "post_attention_layernorm.weight")),
            "wqkv": put(torch.cat([q, k, v])),
            "wo": put(rd.cols(p + "self_attn.o_proj.weight", *r["q"])),
            "w_gate_up": put(torch.cat([g, u])),
            "w_down": put(rd.cols(p + "mlp.down_proj.weight", *r["i"])),
        })
    embed = put(rd.rows("model.embed_tokens.weight"))
    head_name = "lm_head.weight" if rd.has("lm_head.weight") else "model.embed_tokens.weight"
    head = rd.rows(head_name, *r["v"]) if size > 1 else rd.rows(head_name)
    if head.shape[0] < r["vs"]:
        head = torch.cat([head, head.new_zeros(r["vs"] - head.shape[0], head.shape[1])])
    return {"embed": embed, "norm": put(rd.rows("model.norm.weight")), "lm_head": put(head),
            "layers": layers}


def save_hf_llama(full: dict, cfg: LlamaConfig, path: str) -> None:
    """Write a full fused weight dict as a HF-layout safetensors checkpoint
    (tests, and exporting random-init models for other tools).  ``full`` may
    be a ``LlamaModel``: its served weights are exported
    (``LlamaModel.export_weights``: packed copies unpacked, gate/up rows
    de-interleaved).  A raw model dict with packed-only tensors is refused."""
    from safetensors.torch import save_file
    from .. import ops
    if hasattr(full, "export_weights"):
        full = full.export_weights()
    if any(ops.is_packed_only(v) for L in full["layers"] for v in L.values()):
        raise ValueError("packed weights: export LlamaModel.export_weights(), not model.w")
    os.makedirs(path, exist_ok=True)
    D = cfg.head_dim
    qn, kvn, I = cfg.num_heads * D, cfg.num_kv_heads * D, cfg.intermediate_size
    out = {"model.embed_tokens.weight": full["embed"], "model.norm.weight": full["norm"],
           "lm_head.weight": full["lm_head"][:cfg.vocab_size]}
    for i, L in enumerate(full["layers"]):
        p = f"model.layers.{i}."
        out[p + "input_layernorm.weight"] = L["ln1"]
        out[p + "post_attention_layernorm.weight"] = L["ln2"]
        out[p + "self_attn.q_proj.weight"] = L["wqkv"][:qn]
        out[p + "self_attn.k_proj.weight"] = L["wqkv"][qn:qn + kvn]
        out[p + "self_attn.v_proj.weight"] = L["wqkv"][qn + kvn:]
        out[p + "self_attn.o_proj.weight"] = L["wo"]
        out[p + "mlp.gate_proj.weight"] = L["w_gate_up"][:I]
        out[p + "mlp.up_proj.weight"] = L["w_gate_up"][I:]
        out[p + "mlp.down_proj.weight"] = L["w_down"]
        if "q_norm" in L:
            out[p + "self_attn.q_norm.weight"] = L["q_norm"]
            out[p + "self_attn.k_norm.weight"] = L["k_norm"]
        if "bqkv" in L:
            out[p + "self_attn.q_proj.bias"] = L["bqkv"][:qn]
            out[p + "self_attn.k_proj.bias"] = L["bqkv"][qn:qn + kvn]
            out[p + "self_attn.v_proj.bias"] = L["bqkv"][qn + kvn:]
    save_file({k: v.detach().to("cpu").contiguous() for k, v in out.items()},
              os.path.join(path, "model.safetensors"))
    arch = ("Qwen3ForCausalLM" if cfg.qk_norm else
            "Qwen2ForCausalLM" if cfg.qkv_bias else "LlamaForCausalLM")
    hf = {"architectures": [arch], "vocab_size": cfg.vocab_size,
          "hidden_size": cfg.hidden_size, "intermediate_size": cfg.intermediate_size,
          "num_hidden_layers": cfg.num_layers, "num_attention_heads": cfg.num_heads,
          "num_key_value_heads": cfg.num_kv_heads, "head_dim": cfg.head_dim,
          "rope_theta": cfg.rope_theta, "rms_norm_eps": cfg.rms_eps,
          "max_position_embeddings": cfg.max_position, "bos_token_id": cfg.bos_token_id,
          "eos_token_id": list(cfg.eos_token_ids), "tie_word_embeddings": cfg.tie_embeddings,
          "_name_or_path": cfg.name}
    with open(os.path.join(path, "config.json"), "w") as f:
        json.dump(hf, f)
