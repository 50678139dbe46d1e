"""Device <-> model admission (reference: core/internal/limits/limits.go).

* ``load_device_limit_specs`` -- DEVICE_LIMITS_JSON / DEVICE_LIMITS_FILE,
  ``"*"`` is the default spec.
* ``derive_device_limits`` -- the reference thresholds for host RAM/VRAM
  (<=8 GB -> 5B params / 4096 ctx, <=16 GB -> 12B / 8192, else
  floor(mem*0.75*2)/2 and 16384; max_size floor(mem*0.8*10)/10), plus an HBM
  branch for GPUs with ``hbm_gb``: bf16 weights must fit in 85 % of HBM
  (TP-group devices multiply by the group size).
* ``model_allowed`` -- (ok, reason) with the reference's reason codes.
"""
from __future__ import annotations

import json
import math
import os


def load_device_limit_specs(env=None) -> tuple[dict, dict | None]:
    env = os.environ if env is None else env
    raw = (env.get("DEVICE_LIMITS_JSON") or "").strip()
    path = (env.get("DEVICE_LIMITS_FILE") or "").strip()
    if not raw and path:
        with open(path) as f:
            raw = f.read().strip()
    if not raw:
        return {}, None
    data = json.loads(raw)
    specs, default = {}, None
    for k, v in data.items():
        k = k.strip()
        if not k:
            continue
        if k == "*":
            default = dict(v)
        else:
            specs[k] = dict(v)
    return specs, default


def derive_device_limits(spec: dict) -> dict:
    s = dict(spec)
    hbm = s.get("hbm_gb")
    if hbm:
        tp = int(s.get("tp", 1) or 1)
        usable = float(hbm) * tp * 0.85
        s.setdefault("vram_gb", float(hbm) * tp)
        if s.get("max_params_b") is None:
            s["max_params_b"] = math.floor(usable / 2.0 * 2) / 2  # bf16: 2 bytes/param
        if s.get("max_size_gb") is None:
            s["max_size_gb"] = math.floor(usable * 10) / 10
        if s.get("max_context_k") is None:
            s["max_context_k"] = 128
        return s
    mem = 0.0
    if s.get("vram_gb"):
        mem = float(s["vram_gb"])
    elif s.get("ram_gb"):
        mem = float(s["ram_gb"])
    if mem > 0:
        if s.get("max_params_b") is None:
            s["max_params_b"] = 5.0 if mem <= 8 else (12.0 if mem <= 16 else
                                                      math.floor(mem * 0.75 * 2) / 2)
        if s.get("max_size_gb") is None:
            s["max_size_gb"] = math.floor(mem * 0.8 * 10) / 10
        if s.get("max_context_k") is None:
            s["max_context_k"] = 4096 if mem <= 8 else (8192 if mem <= 16 else 16384)
    return s


def _list(v) -> list[str]:
    if not v:
        return []
    if isinstance(v, str):
        try:
            v = json.loads(v)
        except ValueError:
            return []
    return [x.strip() for x in v if isinstance(x, str) and x.strip()]


def strict_mode() -> bool:
    return os.environ.get("STRICT_MODEL_LIMITS", "0") == "1"


def model_allowed(store, device_id: str, model: str, strict: bool | None = None) -> tuple[bool, str]:
    device_id, model = (device_id or "").strip(), (model or "").strip()
    if not device_id or not model:
        return True, ""
    strict = strict_mode() if strict is None else strict
    dm = [d for d in store.list_device_models(device_id) if d["model_id"] == model]
    if not dm:
        return False, "model_not_on_device"
    if not dm[0].get("available", True):
        return False, "model_not_available"
    m = store.get_model(model) or {}
    lim = store.get_device_limits(device_id) or {}
    allow = _list(lim.get("allow_models"))
    if allow and model not in allow:
        return False, "model_not_in_allowlist"
    deny = _list(lim.get("deny_models"))
    if deny and model in deny:
        return False, "model_denied"
    for lk, mk, code in (("max_params_b", "params_b", "params"), ("max_size_gb", "size_gb", "size"),
                         ("max_context_k", "context_k", "context")):
        if lim.get(lk) is None:
            continue
        if m.get(mk) is None:
            if strict:
                return False, f"model_{code}_unknown"
            continue
        if float(m[mk]) > float(lim[lk]):
            return False, f"model_{code}_too_large"
    return True, ""


def apply_device_limits(store, env=None) -> int:
    """Upsert derived limits for every configured device (and, with a "*"
    default, every GPU/engine device)."""
    specs, default = load_device_limit_specs(env)
    if not specs and default is None:
        return 0
    ids = list(specs)
    if default is not None:
        for d in store.list_devices():
            tags = d.get("tags") or {}
            if (tags.get("rocm") or tags.get("engine") or tags.get("ollama")) and d["id"] not in specs:
                ids.append(d["id"])
    for i in ids:
        spec = specs.get(i, default or {})
        if default is None and i not in specs:
            continue
        d = store.get_device(i) or {}
        hb = (d.get("tags") or {}).get("hbm_gb")
        spec = dict(spec)
        if hb and "hbm_gb" not in spec and "vram_gb" not in spec and "ram_gb" not in spec:
            spec["hbm_gb"] = hb
        store.upsert_device_limits(i, derive_device_limits(spec))
    return len(ids)
