"""Smart model selection for ``/v1/chat/completions`` with an empty model
(reference: core/internal/api/handlers.go:3040-3144, selectModel).

Score = catScore * accWeight - costFactor * log10(price_in_1m * 1000 + 1) * 10
with accuracy low/medium/high/critical -> (0.3, 3.0) / (0.6, 1.5) / (0.9, 0.5)
/ (1.0, 0.0); candidates must fit the context (chars/4 vs context_k*1000) and
the max cost.  Extended: locally served models are candidates too (price 0,
category score from their ranking row or 50), and cloud rankings only count
when cloud is enabled."""
from __future__ import annotations

import math

from ..policy.router import cloud_enabled

ACCURACY = {"low": (0.3, 3.0), "medium": (0.6, 1.5), "high": (0.9, 0.5), "critical": (1.0, 0.0)}


def select_model(rankings: list[dict], local_models: list[dict], task_type: str, accuracy: str,
                 max_cost: float, messages: list) -> str | None:
    chars = sum(len(m.get("content", "")) for m in messages
                if isinstance(m, dict) and isinstance(m.get("content"), str))
    est = chars / 4.0
    acc_w, cost_f = ACCURACY.get(accuracy, ACCURACY["medium"])
    cands = []
    by_id = {r["model_id"]: r for r in rankings}
    pool = []
    for lm in local_models:
        r = by_id.get(lm["id"], {})
        pool.append({"model_id": lm["id"], "category_scores": r.get("category_scores") or {},
                     "context_k": lm.get("context_k"), "price_in_1m": 0.0, "price_out_1m": 0.0})
    if cloud_enabled():
        pool += [r for r in rankings if r.get("provider") == "openrouter"]
    for r in pool:
        ck = r.get("context_k")
        if ck and est > float(ck) * 1000:
            continue
        pin, pout = float(r.get("price_in_1m") or 0), float(r.get("price_out_1m") or 0)
        if max_cost > 0 and (est / 1e6) * pin + (est / 1e6) * pout > max_cost:
            continue
        scores = r.get("category_scores") or {}
        cat = float(scores.get(task_type) or 0)
        if cat == 0:
            cat = (sum(scores.values()) / len(scores)) if scores else 50.0
        tier = math.log10(pin * 1000 + 1) * 10 if pin > 0 else 0.0
        cands.append((cat * acc_w - cost_f * tier, r["model_id"]))
    if not cands:
        return None
    return max(cands, key=lambda c: c[0])[1]
