"""Model architecture configs (public HF config.json values) and the local
model registry entries derived from them.

The reference infers tier / thinking / context / kind from model *names*
(core/internal/discovery/discovery.go:482-649).  Here they are derived from the
architecture itself (`params_b`, `context_k`, `kind`), and the name heuristics
are kept only for foreign names (policy/inference.py)."""
from __future__ import annotations

import json
from dataclasses import asdict, dataclass, field
from pathlib import Path


@dataclass
class LlamaConfig:
    name: str = "llama-3-8b"
    vocab_size: int = 128256
    hidden_size: int = 4096
    intermediate_size: int = 14336
    num_layers: int = 32
    num_heads: int = 32
    num_kv_heads: int = 8
    head_dim: int = 128
    rope_theta: float = 500000.0
    rope_scaling: dict | None = None
    rms_eps: float = 1e-5
    max_position: int = 8192
    tie_embeddings: bool = False
    bos_token_id: int = 128000
    eos_token_ids: tuple = (128001, 128009)
    family: str = "llama"
    kind: str = "chat"
    qkv_bias: bool = False          # Qwen2 / Qwen2.5: biased q/k/v projections
    qk_norm: bool = False           # Qwen3: per-head RMSNorm of q and k before RoPE
    # > 1: a one-GPU stand-in for ONE rank of a TP group of this size (the
    # preset's shapes are already the per-rank shard): the O / down GEMMs
    # produce bf16 as a TP rank does before its all-reduce (no split-K
    # partials handed to the norm, no residual epilogue), so the proxy runs
    # exactly the rank's kernels; the all-reduces themselves are not run
    proxy_tp: int = 0

    @property
    def params(self) -> int:
        d, I, L, V = self.hidden_size, self.intermediate_size, self.num_layers, self.vocab_size
        qkv = d * (self.num_heads + 2 * self.num_kv_heads) * self.head_dim
        if self.qkv_bias:
            qkv += (self.num_heads + 2 * self.num_kv_heads) * self.head_dim
        o = self.num_heads * self.head_dim * d
        mlp = 3 * d * I
        emb = V * d * (1 if self.tie_embeddings else 2)
        qkn = 2 * self.head_dim if self.qk_norm else 0
        return L * (qkv + o + mlp + 2 * d + qkn) + emb + d

    @property
    def params_b(self) -> float:
        return round(self.params / 1e9, 2)

    @property
    def context_k(self) -> int:
        return self.max_position // 1024

    def kv_bytes_per_token(self, tp: int = 1, dtype_bytes: int = 2) -> int:
        kvh = max(1, self.num_kv_heads // tp)
        return self.num_layers * 2 * kvh * self.head_dim * dtype_bytes

    def to_dict(self) -> dict:
        return asdict(self)


@dataclass
class NomicBertConfig:
    """nomic-embed-text(-v1.5): post-norm BERT with rotary, SwiGLU, mean pool."""
    name: str = "nomic-embed-text"
    vocab_size: int = 30528
    hidden_size: int = 768
    intermediate_size: int = 3072
    num_layers: int = 12
    num_heads: int = 12
    head_dim: int = 64
    rope_theta: float = 1000.0
    ln_eps: float = 1e-12
    max_position: int = 8192
    type_vocab_size: int = 2
    qkv_bias: bool = False
    mlp_bias: bool = False
    family: str = "nomic-bert"
    kind: str = "embed"
    embed_dim: int = 768

    @property
    def params(self) -> int:
        d, I, L = self.hidden_size, self.intermediate_size, self.num_layers
        return L * (4 * d * d + 3 * d * I + 4 * d) + (self.vocab_size + self.type_vocab_size) * d

    @property
    def params_b(self) -> float:
        return round(self.params / 1e9, 3)

    @property
    def context_k(self) -> int:
        return self.max_position // 1024

    def to_dict(self) -> dict:
        return asdict(self)


@dataclass
class BertConfig:
    """Classic BERT encoder (absolute positions, post-norm, exact-GELU FFN with
    biases); ``pooling`` = "cls" (mxbai / bge / arctic) or "mean"."""
    name: str = "mxbai-embed-large"
    vocab_size: int = 30522
    hidden_size: int = 1024
    intermediate_size: int = 4096
    num_layers: int = 24
    num_heads: int = 16
    head_dim: int = 64
    ln_eps: float = 1e-12
    max_position: int = 512
    type_vocab_size: int = 2
    pooling: str = "cls"
    family: str = "bert"
    kind: str = "embed"
    embed_dim: int = 1024

    @property
    def params(self) -> int:
        d, I, L = self.hidden_size, self.intermediate_size, self.num_layers
        return (L * (4 * d * d + 2 * d * I + 9 * d + I)
                + (self.vocab_size + self.max_position + self.type_vocab_size + 2) * d)

    @property
    def params_b(self) -> float:
        return round(self.params / 1e9, 3)

    @property
    def context_k(self) -> int:
        return max(1, self.max_position // 1024)

    def to_dict(self) -> dict:
        return asdict(self)


_LLAMA32_ROPE = {"rope_type": "llama3", "factor": 32.0, "low_freq_factor": 1.0,
                 "high_freq_factor": 4.0, "original_max_position_embeddings": 8192}


def _qwen3(name, **kw):
    base = dict(name=name, vocab_size=151936, head_dim=128, rope_theta=1000000.0, rms_eps=1e-6,
                max_position=40960, bos_token_id=151643, eos_token_ids=(151645, 151643),
                family="qwen3", qk_norm=True)
    base.update(kw)
    return LlamaConfig(**base)


PRESETS: dict[str, object] = {
    "llama-3-8b": LlamaConfig(),
    "llama-3-70b": LlamaConfig(name="llama-3-70b", hidden_size=8192, intermediate_size=28672,
                               num_layers=80, num_heads=64, num_kv_heads=8),
    "llama-3.1-8b": LlamaConfig(name="llama-3.1-8b", max_position=131072,
                                rope_scaling={"rope_type": "llama3", "factor": 8.0,
                                              "low_freq_factor": 1.0, "high_freq_factor": 4.0,
                                              "original_max_position_embeddings": 8192}),
    "llama-3.2-1b": LlamaConfig(name="llama-3.2-1b", hidden_size=2048, intermediate_size=8192,
                                num_layers=16, num_heads=32, num_kv_heads=8, head_dim=64,
                                tie_embeddings=True, max_position=131072,
                                rope_scaling=_LLAMA32_ROPE),
    # the reference's default OLLAMA_MODEL (llama3.2:3b); GQA group 3
    "llama-3.2-3b": LlamaConfig(name="llama-3.2-3b", hidden_size=3072, intermediate_size=8192,
                                num_layers=28, num_heads=24, num_kv_heads=8, head_dim=128,
                                tie_embeddings=True, max_position=131072,
                                rope_scaling=_LLAMA32_ROPE),
    # tiny configs for tests / smoke (same code paths, D = 128 heads)
    "tiny-llama": LlamaConfig(name="tiny-llama", vocab_size=512, hidden_size=256,
                              intermediate_size=512, num_layers=2, num_heads=4, num_kv_heads=2,
                              head_dim=128, max_position=2048, bos_token_id=506,
                              eos_token_ids=(510,)),
    # the Llama-3-70B head layout shrunk (64 q / 8 kv heads -> 16 / 8): splits
    # over TP = 8 like 70B does (per rank 2 q heads and 1 kv head, I / 8 = 128)
    "tiny-llama-tp8": LlamaConfig(name="tiny-llama-tp8", vocab_size=1024, hidden_size=512,
                                  intermediate_size=1024, num_layers=2, num_heads=16,
                                  num_kv_heads=8, head_dim=128, max_position=2048,
                                  bos_token_id=1018, eos_token_ids=(1022,)),
    # one rank of Llama-3-70B at TP = 8 (config 4) as a TP = 1 model: 8 q / 1 kv
    # heads, FFN 28672 / 8, the vocab shard 16128 (128256 / 8 padded to 256-row
    # tiles), 80 layers -- QKV 1280 x 8192, O 8192 x 1024, gate/up 7168 x 8192,
    # down 8192 x 3584, LM head 16128 x 8192 per decode step, measured on one GPU
    "llama-3-70b-tp8-rank": LlamaConfig(name="llama-3-70b-tp8-rank", vocab_size=16128,
                                        hidden_size=8192, intermediate_size=3584,
                                        num_layers=80, num_heads=8, num_kv_heads=1,
                                        bos_token_id=16122, eos_token_ids=(16123,),
                                        proxy_tp=8),
    # Qwen2.5 (biased QKV, GQA group 7 / 7 -- not a divisor of 16)
    "qwen2.5-7b": LlamaConfig(name="qwen2.5-7b", vocab_size=152064, hidden_size=3584,
                              intermediate_size=18944, num_layers=28, num_heads=28,
                              num_kv_heads=4, head_dim=128, rope_theta=1000000.0, rms_eps=1e-6,
                              max_position=32768, bos_token_id=151643,
                              eos_token_ids=(151643, 151645), family="qwen2", qkv_bias=True),
    "qwen2.5-0.5b": LlamaConfig(name="qwen2.5-0.5b", vocab_size=151936, hidden_size=896,
                                intermediate_size=4864, num_layers=24, num_heads=14,
                                num_kv_heads=2, head_dim=64, rope_theta=1000000.0, rms_eps=1e-6,
                                max_position=32768, tie_embeddings=True, bos_token_id=151643,
                                eos_token_ids=(151643, 151645), family="qwen2", qkv_bias=True),
    "tiny-qwen": LlamaConfig(name="tiny-qwen", vocab_size=512, hidden_size=448,
                             intermediate_size=512, num_layers=2, num_heads=7, num_kv_heads=1,
                             head_dim=64, rope_theta=1000000.0, rms_eps=1e-6, max_position=2048,
                             bos_token_id=506, eos_token_ids=(510,), family="qwen2",
                             qkv_bias=True),
    # Qwen3 (per-head q/k RMSNorm; num_heads x head_dim may differ from hidden)
    "qwen3-8b": _qwen3("qwen3-8b", hidden_size=4096, intermediate_size=12288, num_layers=36,
                       num_heads=32, num_kv_heads=8),
    "qwen3-32b": _qwen3("qwen3-32b", hidden_size=5120, intermediate_size=25600, num_layers=64,
                        num_heads=64, num_kv_heads=8),
    "qwen3-0.6b": _qwen3("qwen3-0.6b", hidden_size=1024, intermediate_size=3072, num_layers=28,
                         num_heads=16, num_kv_heads=8, tie_embeddings=True),
    "tiny-qwen3": _qwen3("tiny-qwen3", vocab_size=512, hidden_size=256, intermediate_size=512,
                         num_layers=2, num_heads=4, num_kv_heads=2, max_position=2048,
                         bos_token_id=506, eos_token_ids=(510,)),
    "nomic-embed-text": NomicBertConfig(),
    # BERT-architecture embedders (Ollama: mxbai-embed-large, bge-large, snowflake-arctic-embed)
    "mxbai-embed-large": BertConfig(),
    "bge-large-en-v1.5": BertConfig(name="bge-large-en-v1.5"),
    "bge-base-en-v1.5": BertConfig(name="bge-base-en-v1.5", hidden_size=768,
                                   intermediate_size=3072, num_layers=12, num_heads=12,
                                   embed_dim=768),
    "snowflake-arctic-embed-m": BertConfig(name="snowflake-arctic-embed-m", hidden_size=768,
                                           intermediate_size=3072, num_layers=12, num_heads=12,
                                           embed_dim=768),
    "tiny-bert": BertConfig(name="tiny-bert", vocab_size=512, hidden_size=256,
                            intermediate_size=512, num_layers=2, num_heads=4, head_dim=64,
                            embed_dim=256, max_position=256),
    "tiny-bert-mean": BertConfig(name="tiny-bert-mean", vocab_size=512, hidden_size=256,
                                 intermediate_size=512, num_layers=2, num_heads=2, head_dim=128,
                                 embed_dim=256, max_position=256, pooling="mean"),
    "tiny-nomic": NomicBertConfig(name="tiny-nomic", vocab_size=512, hidden_size=256,
                                  intermediate_size=512, num_layers=2, num_heads=2, head_dim=128,
                                  embed_dim=256, max_position=2048),
}

# OpenAI-style aliases (Ollama tags used by the reference's defaults)
ALIASES = {
    "llama3": "llama-3-8b", "llama3:8b": "llama-3-8b", "llama-3-8b-instruct": "llama-3-8b",
    "meta-llama-3-8b": "llama-3-8b", "llama3:70b": "llama-3-70b",
    "llama3.2:1b": "llama-3.2-1b", "llama3.2:3b": "llama-3.2-3b", "llama3.2": "llama-3.2-3b",
    "nomic-embed-text:latest": "nomic-embed-text",
    "qwen3:8b": "qwen3-8b", "qwen3:32b": "qwen3-32b", "qwen3:0.6b": "qwen3-0.6b",
    "qwen3": "qwen3-8b",
    "nomic-embed-text-v1.5": "nomic-embed-text",
    "qwen2.5:7b": "qwen2.5-7b", "qwen2.5:0.5b": "qwen2.5-0.5b",
    "qwen2.5-7b-instruct": "qwen2.5-7b",
    "mxbai-embed-large:latest": "mxbai-embed-large", "mxbai-embed-large:335m": "mxbai-embed-large",
    "mixedbread-ai/mxbai-embed-large-v1": "mxbai-embed-large",
    "bge-large": "bge-large-en-v1.5", "bge-large:335m": "bge-large-en-v1.5",
    "snowflake-arctic-embed:110m": "snowflake-arctic-embed-m",
}


def resolve(name: str):
    """Preset by name or alias.  ``<name>@L<n>`` keeps the preset's shapes
    with only n layers (e.g. ``llama-3-70b@L8``: one-GPU rehearsals of the
    70B TP layout; never a number for the full model)."""
    base, _, layers = name.partition("@L")
    key = ALIASES.get(base, base)
    if key not in PRESETS:
        raise KeyError(f"unknown model {name!r}; known: {sorted(PRESETS)}")
    cfg = PRESETS[key]
    if layers:
        import dataclasses
        n = int(layers)
        if n < 1 or n > cfg.num_layers:
            raise KeyError(f"{name!r}: layer count must be 1..{cfg.num_layers}")
        cfg = dataclasses.replace(cfg, name=name, num_layers=n)
    return cfg


def from_hf_config(path: str | Path):
    """Build a config from a HF config.json (local file; no network)."""
    cfg = json.loads(Path(path).read_text())
    arch = (cfg.get("architectures") or [""])[0]
    if "Llama" in arch or "Qwen2" in arch or "Qwen3" in arch or "Mistral" in arch:
        qwen = "Qwen2" in arch
        qwen3 = "Qwen3" in arch
        return LlamaConfig(
            name=cfg.get("_name_or_path", "llama"), vocab_size=cfg["vocab_size"],
            hidden_size=cfg["hidden_size"], intermediate_size=cfg["intermediate_size"],
            num_layers=cfg["num_hidden_layers"], num_heads=cfg["num_attention_heads"],
            num_kv_heads=cfg.get("num_key_value_heads", cfg["num_attention_heads"]),
            head_dim=cfg.get("head_dim", cfg["hidden_size"] // cfg["num_attention_heads"]),
            rope_theta=cfg.get("rope_theta", 10000.0), rope_scaling=cfg.get("rope_scaling"),
            rms_eps=cfg.get("rms_norm_eps", 1e-5),
            max_position=cfg.get("max_position_embeddings", 8192),
            tie_embeddings=cfg.get("tie_word_embeddings", False),
            bos_token_id=cfg.get("bos_token_id", 128000),
            eos_token_ids=tuple(cfg["eos_token_id"]) if isinstance(cfg.get("eos_token_id"), list)
            else (cfg.get("eos_token_id", 128001),),
            family="qwen2" if qwen else ("qwen3" if qwen3 else
                                         ("mistral" if "Mistral" in arch else "llama")),
            qkv_bias=qwen or bool(cfg.get("attention_bias", False)), qk_norm=qwen3)
    if "NomicBert" in arch or cfg.get("model_type") == "nomic_bert":
        return NomicBertConfig(
            vocab_size=cfg["vocab_size"], hidden_size=cfg["n_embd"],
            intermediate_size=cfg["n_inner"], num_layers=cfg["n_layer"],
            num_heads=cfg["n_head"], head_dim=cfg["n_embd"] // cfg["n_head"],
            rope_theta=cfg.get("rotary_emb_base", 1000.0),
            ln_eps=cfg.get("layer_norm_epsilon", 1e-12),
            max_position=cfg.get("n_positions", 8192),
            qkv_bias=cfg.get("qkv_proj_bias", False), mlp_bias=cfg.get("mlp_fc1_bias", False),
            embed_dim=cfg["n_embd"])
    if arch in ("BertModel", "BertForMaskedLM") or cfg.get("model_type") == "bert":
        d, H = cfg["hidden_size"], cfg["num_attention_heads"]
        return BertConfig(
            name=cfg.get("_name_or_path", "bert"), vocab_size=cfg["vocab_size"], hidden_size=d,
            intermediate_size=cfg["intermediate_size"], num_layers=cfg["num_hidden_layers"],
            num_heads=H, head_dim=d // H, ln_eps=cfg.get("layer_norm_eps", 1e-12),
            max_position=cfg.get("max_position_embeddings", 512),
            type_vocab_size=cfg.get("type_vocab_size", 2), embed_dim=d,
            pooling=cfg.get("pooling", "cls"))
    raise ValueError(f"unsupported architecture {arch!r}")
