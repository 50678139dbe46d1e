"""Model catalogue planner: cloud catalogue sync and job retention.

* ``sync_openrouter(store)`` -- ``POST /v1/models/sync`` (reference
  handlers.go:3176-3287): pulls ``/models?category=`` for six categories,
  upserts ``model_rankings`` (per-token price x 1e6 -> per-1M), gives listed
  models a membership score of 75 in each category they appear in, and seeds
  ``model_stats`` rows.  Only reachable with ``LMX_ALLOW_CLOUD=1`` -- the
  serving hot path never depends on it.
* ``sync_curated(store, path)`` -- the reference's offline script
  (scripts/sync_openrouter_models.py:80-320): curated YAML ids -> ``models``
  + ``model_pricing`` (context_k = context_length // 1024) + a JSON snapshot.
* ``RetentionPlanner`` -- the "planner/" the reference documents but never
  shipped: periodic purge of finished jobs older than
  ``LMX_JOB_RETENTION_DAYS`` and expiry of missed deadlines.
"""
from __future__ import annotations

import asyncio
import json
import logging
import os
import time

log = logging.getLogger("lmx.planner")

CATEGORIES = ("programming", "science", "technology", "translation", "finance", "academia")
DEFAULT_BASE = "https://openrouter.ai/api/v1"


def _price_1m(v) -> float:
    try:
        return round(float(v) * 1e6, 6)
    except (TypeError, ValueError):
        return 0.0


def rankings_from_catalog(per_category: dict[str, list[dict]]) -> dict[str, dict]:
    """Merge per-category model lists into ranking rows (pure; unit-tested)."""
    out: dict[str, dict] = {}
    for cat, models in per_category.items():
        for m in models:
            mid = m.get("id")
            if not mid:
                continue
            r = out.setdefault(mid, {
                "provider": "openrouter", "display_name": m.get("name") or mid,
                "category_scores": {},
                "context_k": int(m.get("context_length") or 0) // 1000,
                "price_in_1m": _price_1m((m.get("pricing") or {}).get("prompt")),
                "price_out_1m": _price_1m((m.get("pricing") or {}).get("completion")),
                "modalities": (m.get("architecture") or {}).get("input_modalities") or ["text"],
                "supports_tools": "tools" in (m.get("supported_parameters") or []),
                "supports_vision": "image" in ((m.get("architecture") or {})
                                               .get("input_modalities") or []),
                "is_local": False})
            r["category_scores"][cat] = 75
    return out


async def _fetch_json(session, url: str, key: str) -> dict:
    async with session.get(url, headers={"Authorization": f"Bearer {key}"}) as r:
        if r.status != 200:
            raise RuntimeError(f"{url}: HTTP {r.status}")
        return await r.json()


async def sync_openrouter(store, api_key: str | None = None, base: str | None = None,
                          categories=CATEGORIES) -> dict:
    import aiohttp
    key = api_key or os.environ.get("OPENROUTER_API_KEY", "")
    if not key or key == "not-used":
        raise RuntimeError("OPENROUTER_API_KEY not configured")
    base = (base or os.environ.get("OPENROUTER_BASE_URL", DEFAULT_BASE)).rstrip("/")
    per: dict[str, list[dict]] = {}
    timeout = aiohttp.ClientTimeout(total=30)
    async with aiohttp.ClientSession(timeout=timeout) as s:
        res = await asyncio.gather(*[_fetch_json(s, f"{base}/models?category={c}", key)
                                     for c in categories], return_exceptions=True)
    for c, r in zip(categories, res):
        if isinstance(r, Exception):
            log.warning("category %s: %s", c, r)
            continue
        per[c] = r.get("data") or []
    rows = rankings_from_catalog(per)
    existing = {m["model_id"] for m in store.model_stats()}
    for mid, r in rows.items():
        store.upsert_model_ranking(mid, **r)
        store.upsert_model(mid, provider="openrouter", kind="chat",
                           context_k=r["context_k"] or None)
        store.set_pricing(mid, r["price_in_1m"], r["price_out_1m"])
        if mid not in existing:
            store.update_model_stats(mid, 0, 0, 0, 0.0, True)   # seed the row
    return {"status": "ok", "synced": len(rows), "categories": sorted(per)}


def load_curated(path: str) -> list[str]:
    import yaml
    with open(path) as f:
        doc = yaml.safe_load(f) or {}
    return [m["id"] for m in doc.get("models") or [] if isinstance(m, dict) and m.get("id")]


def apply_curated(store, ids: list[str], catalog: list[dict], snapshot_dir: str = "") -> dict:
    """Upsert the curated subset of a fetched ``/models`` list (pure w.r.t. IO
    besides the store and the optional snapshot)."""
    by_id = {m.get("id"): m for m in catalog}
    done, missing = [], []
    for mid in ids:
        m = by_id.get(mid)
        if m is None:
            missing.append(mid)
            continue
        p = m.get("pricing") or {}
        store.upsert_model(mid, provider="openrouter", kind="chat",
                           context_k=int(m.get("context_length") or 0) // 1024 or None,
                           meta={"name": m.get("name"), "curated": True})
        store.set_pricing(mid, _price_1m(p.get("prompt")), _price_1m(p.get("completion")))
        done.append(mid)
    snap = ""
    if snapshot_dir:
        os.makedirs(snapshot_dir, exist_ok=True)
        snap = os.path.join(snapshot_dir, time.strftime("openrouter-%Y%m%d-%H%M%S.json"))
        with open(snap, "w") as f:
            json.dump({"synced": done, "missing": missing,
                       "models": [by_id[m] for m in done]}, f, indent=1)
    return {"synced": done, "missing": missing, "snapshot": snap}


async def sync_curated(store, path: str | None = None, snapshot_dir: str = "") -> dict:
    import aiohttp
    path = path or os.path.join(os.path.dirname(__file__), "..", "config",
                                "curated_cloud_models.yaml")
    key = os.environ.get("OPENROUTER_API_KEY", "")
    base = os.environ.get("OPENROUTER_BASE_URL", DEFAULT_BASE).rstrip("/")
    async with aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=30)) as s:
        data = await _fetch_json(s, f"{base}/models", key)
    return apply_curated(store, load_curated(path), data.get("data") or [], snapshot_dir)


class RetentionPlanner:
    """Periodic store hygiene (run from the core's maintenance loop)."""

    def __init__(self, store, retention_days: float | None = None):
        self.store = store
        days = retention_days if retention_days is not None else \
            float(os.environ.get("LMX_JOB_RETENTION_DAYS", "30"))
        self.retention_s = days * 86400

    def tick(self) -> dict:
        expired = self.store.expire_deadlines()
        exhausted = self.store.sweep_exhausted()
        purged = self.store.purge_jobs(self.retention_s) if self.retention_s > 0 else 0
        return {"deadline_expired": expired, "attempts_exhausted": exhausted, "purged": purged}
