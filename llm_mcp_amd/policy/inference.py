"""Model metadata inference.

Local models served by this node get their metadata from the architecture
config (params_b, context_k, kind -- models/config.py).  The name heuristics
of the reference's discovery (core/internal/discovery/discovery.go:482-649)
are kept for foreign / catalog model names."""
from __future__ import annotations

THINKING_PREFIXES = ("qwen3:",)
THINKING_SUBSTR = ("deepseek-r1", "phi4-reasoning", "lfm2.5-thinking", "deepscaler",
                   "exaone-deep")


def parse_params_b(raw: str | None) -> float | None:
    """'8B' -> 8.0, '137M' -> 0.137, '500K' -> 0.0005."""
    raw = (raw or "").strip()
    if not raw:
        return None
    mult = 1.0
    if raw[-1] in "Bb":
        raw = raw[:-1]
    elif raw[-1] in "Mm":
        raw, mult = raw[:-1], 0.001
    elif raw[-1] in "Kk":
        raw, mult = raw[:-1], 0.000001
    try:
        return float(raw) * mult
    except ValueError:
        return None


def infer_tier(params_b: float | None, name: str) -> str:
    if "embed" in name.lower():
        return "embed"
    if params_b is None:
        return ""
    b = params_b
    if b <= 1.2:
        return "tiny"
    if b <= 2.0:
        return "small"
    if b <= 4.5:
        return "medium"
    if b <= 10.0:
        return "large"
    return "xl"


def infer_thinking(name: str, family: str = "") -> bool:
    n = name.lower()
    return n.startswith(THINKING_PREFIXES) or any(s in n for s in THINKING_SUBSTR)


def infer_context_k(name: str, family: str = "") -> int:
    n = name.lower()
    if n.startswith("tinyllama"):
        return 2
    if n.startswith("yi:"):
        return 4
    if n.startswith(("qwen3:", "qwen2.5:", "qwen2.5-coder:", "exaone-deep:", "granite4:",
                     "lfm2.5-thinking:", "falcon3:", "smollm2:")):
        return 32
    if n.startswith(("llama3.2:", "phi3.5:", "phi3:", "qwen2.5vl:", "qwen3-vl:")):
        return 128
    if n.startswith("phi4-reasoning"):
        return 16
    if "embed" in n:
        return 8
    if n.startswith("gemma"):
        return 8
    return 4


def infer_kind(name: str) -> str:
    return "embed" if "embed" in name.lower() else "chat"


def model_record(model_id: str, cfg=None) -> dict:
    """Catalog fields for a model, from its architecture config when known."""
    if cfg is not None:
        params_b = float(getattr(cfg, "params_b", 0) or 0) or None
        kind = getattr(cfg, "kind", infer_kind(model_id))
        return {"provider": "local", "family": getattr(cfg, "family", ""), "kind": kind,
                "params_b": params_b, "context_k": getattr(cfg, "context_k", None),
                "size_gb": round(getattr(cfg, "params", 0) * 2 / 2 ** 30, 2) or None,
                "quant": "bf16", "tier": "embed" if kind == "embed" else
                infer_tier(params_b, model_id),
                "thinking": infer_thinking(model_id), "status": "active"}
    return {"provider": "local", "kind": infer_kind(model_id),
            "context_k": infer_context_k(model_id), "tier": "",
            "thinking": infer_thinking(model_id), "status": "active"}
