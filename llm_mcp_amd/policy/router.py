"""Provider / model / device routing (reference: core/internal/routing/router.go).

Behaviour kept:
  * ``route_llm`` classic routing: embed -> local; force_cloud -> openrouter >
    openai > local; prefer_local with a local device -> local; otherwise cloud
    keys first -- *but* cloud providers only count when ``LMX_ALLOW_CLOUD=1``
    (the north star forbids cloud on the hot path, so by default everything
    routes to the local GPUs); max_latency_ms checked against the latest
    benchmark; an explicit ``payload`` bypasses payload construction; an
    explicit ``provider`` is not overridden.
  * smart routing (``quality`` set, ``model`` empty): token estimate (chars/4,
    min 256), context buckets <=4K / 4-32K / >32K, the quality-tier tables,
    thinking preference for task=reason, local models first, cloud fallback,
    ``_tier`` / ``_price_in_1m`` / ``_price_out_1m`` / ``thinking`` injected.
Local provider = this node's engines: provider ``local`` with kinds
``engine.generate`` / ``engine.embed``; the reference names ``ollama`` /
``ollama.generate`` / ``ollama.embed`` are accepted as aliases.
Fixed defect: ``select_device`` consults the circuit breaker and the device's
live capacity (the reference's SelectOllamaDevice did neither).
"""
from __future__ import annotations

import os

from ..models.tokenizer import messages_to_prompt
from . import limits as lim

QUALITY_TIERS = {
    #            <=4K                 4K-32K              >32K
    "turbo": (["tiny"], ["tiny", "small"], []),
    "economy": (["tiny", "small"], ["small", "medium"], []),
    "standard": (["small", "medium"], ["medium", "large"], []),
    "premium": (["medium", "large"], ["large", "xl"], []),
    "ultra": (["large", "xl"], ["xl"], []),
    "max": ([], [], []),
}

CLOUD_FALLBACK_TIERS = {
    "turbo": ["cloud_economy"], "economy": ["cloud_economy"], "standard": ["cloud_economy"],
    "premium": ["cloud_economy", "cloud_premium"], "ultra": ["cloud_premium", "cloud_economy"],
    "max": ["cloud_premium", "cloud_economy"],
}

QUALITY_TIMEOUTS = {"turbo": 15, "economy": 30, "standard": 60, "premium": 90, "ultra": 120,
                    "max": 180}

LOCAL_ALIASES = {"ollama", "local", "engine", "gpu"}


class RoutingError(Exception):
    pass


def estimate_tokens(prompt: str = "", messages: list | None = None) -> int:
    total = len(prompt or "")
    for m in messages or []:
        c = m.get("content", "") if isinstance(m, dict) else ""
        total += len(c) if isinstance(c, str) else 0
    return max(256, total // 4)


def parse_payload_model_device(payload) -> tuple[str, str]:
    if not isinstance(payload, dict):
        return "", ""
    model = payload.get("model")
    dev = payload.get("device_id")
    return (model.strip() if isinstance(model, str) else "",
            dev.strip() if isinstance(dev, str) else "")


def cloud_enabled() -> bool:
    return os.environ.get("LMX_ALLOW_CLOUD", "0") == "1"


def has_openrouter() -> bool:
    k = os.environ.get("OPENROUTER_API_KEY", "")
    return cloud_enabled() and bool(k) and k != "not-used"


def has_openai() -> bool:
    k = os.environ.get("OPENAI_API_KEY", "")
    return cloud_enabled() and bool(k) and k != "not-used"


class Router:
    def __init__(self, store, circuit, capacity_of=None):
        """capacity_of(device_id) -> max concurrent jobs (engine slots) or None."""
        self.store = store
        self.circuit = circuit
        self.capacity_of = capacity_of or (lambda dev: None)

    # ------------------------------------------------------------ devices ---
    def has_local(self) -> bool:
        return any(d.get("status") == "online" and (d.get("tags") or {}).get("engine")
                   for d in self.store.list_devices())

    def meets_latency(self, model: str, task: str, max_ms: int) -> bool:
        b = self.store.latest_benchmark(model, task)
        return bool(b) and 0 < b["latency_ms"] <= max_ms

    def select_device(self, model: str, task: str, strict: bool | None = None) -> dict | None:
        """Best online engine device serving ``model``: limits pass, circuit not
        degraded, capacity left; ordered by latest benchmark tps desc, latency
        asc, last_seen desc."""
        model = (model or "").strip()
        if not model:
            return None
        strict = lim.strict_mode() if strict is None else strict
        cands = []
        for dm in self.store.list_device_models(available_only=True):
            if dm["model_id"] != model:
                continue
            d = self.store.get_device(dm["device_id"])
            if not d or d.get("status") != "online" or not (d.get("tags") or {}).get("engine"):
                continue
            ok, _ = lim.model_allowed(self.store, d["id"], model, strict)
            if not ok:
                continue
            if self.circuit is not None and self.circuit.is_degraded(d["id"]):
                continue
            cap = self.capacity_of(d["id"])
            if cap is None:
                cap = (d.get("tags") or {}).get("capacity")
            load = self.store.active_jobs_on(d["id"])
            if cap and load >= int(cap):
                continue
            b = self.store.latest_benchmark(model, task, d["id"]) or {}
            cands.append((-(b.get("tps") or 0.0), b.get("latency_ms") or 1 << 30,
                          -(d.get("last_seen") or 0), load, d))
        if not cands:
            return None
        cands.sort(key=lambda c: c[:4])
        d = cands[0][-1]
        tags = d.get("tags") or {}
        return {"id": d["id"], "addr": tags.get("engine_addr", ""), "host": tags.get("host", "")}

    # ---------------------------------------------------------- classic -----
    def route_llm(self, req: dict) -> tuple[str, str, dict]:
        model = (req.get("model") or "").strip()
        quality = (req.get("quality") or "").strip()
        if not model and quality:
            return self.route_smart(req)
        task = (req.get("task") or "chat").strip().lower() or "chat"
        provider = (req.get("provider") or "auto").strip().lower() or "auto"
        cons = req.get("constraints") or {}
        local = self.has_local()
        alias = provider if provider in LOCAL_ALIASES else None
        if provider == "auto":
            if task == "embed":
                provider = "local"
            elif cons.get("force_cloud"):
                provider = "openrouter" if has_openrouter() else (
                    "openai" if has_openai() else "local")
            elif cons.get("prefer_local") and local:
                provider = "local"
            elif has_openrouter():
                provider = "openrouter"
            elif has_openai():
                provider = "openai"
            else:
                provider = "local"
        elif provider in LOCAL_ALIASES:
            provider = "local"
        if provider == "local" and int(cons.get("max_latency_ms") or 0) > 0 and model:
            if not self.meets_latency(model, task, int(cons["max_latency_ms"])):
                if has_openrouter():
                    provider = "openrouter"
                elif has_openai():
                    provider = "openai"
        if provider == "local":
            prefix = "ollama" if alias == "ollama" else "engine"
            kind = f"{prefix}.embed" if task == "embed" else f"{prefix}.generate"
        elif provider == "openai":
            kind = "openai.chat"
        elif provider == "openrouter":
            kind = "openrouter.chat"
        else:
            raise RoutingError("provider_not_supported")

        if req.get("payload"):
            payload = req["payload"]
            if isinstance(payload, dict) and provider == "local":
                m, dev = parse_payload_model_device(payload)
                if m and dev:
                    ok, why = lim.model_allowed(self.store, dev, m)
                    if not ok:
                        raise RoutingError("model_not_allowed:" + why)
            return provider, kind, payload

        payload: dict = {}
        if kind.endswith(".generate"):
            prompt = req.get("prompt") or ""
            if not prompt and req.get("messages"):
                prompt = messages_to_prompt(req["messages"])
                payload["messages"] = req["messages"]
            if not prompt:
                raise RoutingError("prompt_required")
            if model:
                payload["model"] = model
            payload["prompt"] = prompt
            self._copy_gen_options(req, payload)
            if model:
                self._place(payload, model, "generate")
        elif kind.endswith(".embed"):
            prompt = req.get("prompt") or ""
            if not prompt:
                raise RoutingError("prompt_required")
            if model:
                payload["model"] = model
            payload["prompt"] = prompt
            if model:
                self._place(payload, model, "embed")
        else:
            msgs = req.get("messages") or []
            if not msgs and req.get("prompt"):
                msgs = [{"role": "user", "content": req["prompt"]}]
            if not msgs:
                raise RoutingError("messages_required")
            if model:
                payload["model"] = model
            payload["messages"] = msgs
            if req.get("temperature") is not None:
                payload["temperature"] = req["temperature"]
            if req.get("max_tokens") is not None:
                payload["max_tokens"] = req["max_tokens"]
        return provider, kind, payload

    @staticmethod
    def _copy_gen_options(req, payload):
        opts = dict(req.get("options") or {})
        for k in ("temperature", "max_tokens", "top_p", "top_k", "stop", "seed"):
            if req.get(k) is not None:
                opts[k] = req[k]
        if opts:
            payload["options"] = opts

    def _place(self, payload, model, task):
        t = self.select_device(model, task)
        if t is not None:
            payload["device_id"] = t["id"]
            if t.get("addr"):
                payload["engine_addr"] = t["addr"]
        elif lim.strict_mode():
            raise RoutingError("no_eligible_device")

    # ------------------------------------------------------------ smart -----
    def find_local_model(self, tiers: list[str], min_context_k: int, prefer_thinking: bool):
        cands = []
        for m in self.store.list_models():
            if m.get("provider") not in ("local", "ollama") or m.get("kind") == "embed":
                continue
            if (m.get("status") or "active") != "active" or m.get("tier") not in tiers:
                continue
            if (m.get("context_k") or 4) < min_context_k:
                continue
            for dm in self.store.list_device_models(available_only=True):
                if dm["model_id"] != m["id"]:
                    continue
                d = self.store.get_device(dm["device_id"])
                if not d or d.get("status") != "online" or not (d.get("tags") or {}).get("engine"):
                    continue
                if self.circuit is not None and self.circuit.is_degraded(d["id"]):
                    continue
                think = bool(m.get("thinking"))
                cands.append(((0 if prefer_thinking and think else 1), tiers.index(m["tier"]),
                              self.store.active_jobs_on(d["id"]), -(m.get("params_b") or 0),
                              -(d.get("last_seen") or 0), m, d))
        if not cands:
            return None
        cands.sort(key=lambda c: c[:5])
        m, d = cands[0][5], cands[0][6]
        return {"model": m["id"], "provider": "local", "device_id": d["id"], "tier": m["tier"],
                "thinking": bool(m.get("thinking")), "reason": "local_match",
                "addr": (d.get("tags") or {}).get("engine_addr", "")}

    def find_cloud_model(self, tiers: list[str], min_context_k: int, prefer_thinking: bool):
        cands = []
        for m in self.store.list_models():
            if m.get("provider") not in ("openrouter", "openai") or m.get("kind") == "embed":
                continue
            if (m.get("status") or "active") != "active" or m.get("tier") not in tiers:
                continue
            if (m.get("context_k") or 128) < min_context_k:
                continue
            cands.append(((0 if prefer_thinking and m.get("thinking") else 1),
                          tiers.index(m["tier"]), -(m.get("context_k") or 0), m))
        if not cands:
            return None
        cands.sort(key=lambda c: c[:3])
        m = cands[0][3]
        if m["provider"] == "openrouter" and not has_openrouter():
            return None
        if m["provider"] == "openai" and not has_openai():
            return None
        return {"model": m["id"], "provider": m["provider"], "device_id": "",
                "tier": m["tier"], "thinking": bool(m.get("thinking")),
                "reason": "cloud_fallback"}

    def lookup_pricing(self, model_id: str) -> tuple[float, float]:
        p = self.store.get_pricing(model_id)
        return (0.0, 0.0) if p is None else (float(p[0]), float(p[1]))

    def route_smart(self, req: dict) -> tuple[str, str, dict]:
        quality = (req.get("quality") or "").strip().lower()
        task = (req.get("task") or "chat").strip().lower() or "chat"
        if quality not in QUALITY_TIERS:
            raise RoutingError(f"invalid_quality: {quality} "
                               "(use turbo|economy|standard|premium|ultra|max)")
        est = estimate_tokens(req.get("prompt") or "", req.get("messages"))
        bucket = 2 if est > 32000 else (1 if est > 4000 else 0)
        min_ctx = max(1, est // 1000)
        think = task == "reason"
        sel = None
        tiers = QUALITY_TIERS[quality][bucket]
        if tiers:
            sel = self.find_local_model(tiers, min_ctx, think)
        if sel is None and CLOUD_FALLBACK_TIERS.get(quality):
            sel = self.find_cloud_model(CLOUD_FALLBACK_TIERS[quality], min_ctx, think)
        if sel is None:
            raise RoutingError("no_model_available: quality=" + quality)
        if sel["provider"] == "local":
            kind = "engine.embed" if task == "embed" else "engine.generate"
        else:
            kind = f"{sel['provider']}.chat"
        payload: dict = {}
        if sel["provider"] == "local":
            prompt = req.get("prompt") or ""
            if not prompt and req.get("messages"):
                prompt = messages_to_prompt(req["messages"])
                payload["messages"] = req["messages"]
            if not prompt:
                raise RoutingError("prompt_required")
            payload.update(model=sel["model"], prompt=prompt)
            self._copy_gen_options(req, payload)
            if sel.get("device_id"):
                payload["device_id"] = sel["device_id"]
            if sel.get("addr"):
                payload["engine_addr"] = sel["addr"]
        else:
            msgs = req.get("messages") or ([{"role": "user", "content": req["prompt"]}]
                                           if req.get("prompt") else [])
            if not msgs:
                raise RoutingError("messages_required")
            payload.update(model=sel["model"], messages=msgs)
            if req.get("temperature") is not None:
                payload["temperature"] = req["temperature"]
            if req.get("max_tokens") is not None:
                payload["max_tokens"] = req["max_tokens"]
        payload["_tier"] = sel["tier"]
        pin, pout = self.lookup_pricing(sel["model"])
        payload["_price_in_1m"] = pin
        payload["_price_out_1m"] = pout
        if req.get("thinking") is not None:
            payload["thinking"] = bool(req["thinking"])
        elif sel["thinking"]:
            payload["thinking"] = True
        return sel["provider"], kind, payload
