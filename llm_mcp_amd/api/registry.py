"""Local model registry: which model runs on which GPU (or TP group) of this
node, and device selection among replicas.

This is the in-process replacement of the reference's ``SelectOllamaDevice``
(core/internal/routing/router.go:277-331), which picked the Ollama host with
the best benchmark tps and ignored both the circuit breaker and concurrency.
Here selection
  * skips replicas whose device circuit is degraded (policy/circuit.py),
  * skips replicas at capacity (continuous-batching slots / KV pages),
  * prefers the least loaded replica, breaking ties by measured tokens/s.
"""
from __future__ import annotations

import threading
from dataclasses import dataclass, field

from ..models import config as mc


@dataclass
class LocalModel:
    model_id: str
    kind: str                 # "chat" | "embed"
    device_id: str
    engine: object            # AsyncEngine (chat) or EmbeddingEngine (embed)
    tokenizer: object
    cfg: object
    max_model_len: int = 8192
    capacity: int = 256       # concurrent sequences admitted by the engine
    tps: float = 0.0          # last measured decode tokens/s (benchmarks)
    inflight: int = 0
    tags: dict = field(default_factory=dict)
    lb_slot: int = -1         # column in the front door's SharedLoad (-1: local count only)

    def load(self) -> float:
        return self.inflight / max(1, self.capacity)

    def info(self) -> dict:
        eng = getattr(self.engine, "engine", self.engine)
        sched = getattr(eng, "sched", None)
        d = {"model": self.model_id, "kind": self.kind, "device_id": self.device_id,
             "inflight": self.inflight, "capacity": self.capacity, "tps": self.tps,
             "params_b": getattr(self.cfg, "params_b", None),
             "context_k": getattr(self.cfg, "context_k", None)}
        if sched is not None:
            d.update(kv_usage=round(sched.kv_usage, 4), running=sched.num_running,
                     waiting=sched.num_waiting)
        else:
            # engine in a worker process: the link's last polled info (api/serve.py)
            live = self.tags.get("live") or {}
            if "kv_usage" in live:
                d.update(kv_usage=round(float(live["kv_usage"]), 4),
                         running=int(live.get("running", 0)),
                         waiting=int(live.get("waiting", 0)))
        comm = getattr(eng, "tp_comm", None) or self.tags.get("tp_comm")
        if comm:
            d["tp_comm"] = comm       # TP all-reduce probe, us by message size
        live = getattr(eng, "tp_comm_live", None) or \
            (self.tags.get("live") or {}).get("tp_comm_live")
        if live:
            d["tp_comm_live"] = live  # latest in-service sample (engine._comm_probe)
        return d


class ModelRegistry:
    def __init__(self):
        self._lock = threading.Lock()
        self._models: dict[str, list[LocalModel]] = {}
        # api/shared_load.SharedLoad when several API processes share the
        # engines: selection then balances on the node-wide in-flight counts
        self.balancer = None

    @staticmethod
    def canonical(name: str) -> str:
        return mc.ALIASES.get(name, name)

    def add(self, m: LocalModel) -> None:
        with self._lock:
            self._models.setdefault(self.canonical(m.model_id), []).append(m)

    def remove(self, m: LocalModel) -> None:
        """Drop one replica (by identity), e.g. when its worker died."""
        with self._lock:
            k = self.canonical(m.model_id)
            lst = [x for x in self._models.get(k, []) if x is not m]
            if lst:
                self._models[k] = lst
            else:
                self._models.pop(k, None)

    def remove_device(self, device_id: str) -> None:
        with self._lock:
            for k in list(self._models):
                self._models[k] = [m for m in self._models[k] if m.device_id != device_id]
                if not self._models[k]:
                    del self._models[k]

    def replicas(self, model: str) -> list[LocalModel]:
        return list(self._models.get(self.canonical(model), []))

    def all(self) -> list[LocalModel]:
        with self._lock:
            return [m for v in self._models.values() for m in v]

    def model_ids(self, kind: str | None = None) -> list[str]:
        return sorted({k for k, v in self._models.items()
                       if any(kind is None or m.kind == kind for m in v)})

    def select(self, model: str, kind: str, circuit=None,
               exclude: set | None = None, acquire: bool = False) -> LocalModel | None:
        """Least-loaded healthy replica with a free slot (else least loaded),
        ties by measured tokens/s.  ``acquire``: count the request against
        the pick in the same step (atomically across the API processes of a
        shared front door); pair with ``release``."""
        cands = [m for m in self.replicas(model) if m.kind == kind
                 and (not exclude or m.device_id not in exclude)]
        if circuit is not None:
            healthy = [m for m in cands if not circuit.is_degraded(m.device_id)]
            cands = healthy or []
        if not cands:
            return None
        bal = self.balancer
        if bal is None or all(m.lb_slot < 0 for m in cands):
            free = [m for m in cands if m.inflight < m.capacity] or cands
            m = min(free, key=lambda m: (m.load(), -m.tps))
            if acquire:
                m.inflight += 1
            return m
        with bal.locked():
            tot = bal.totals()

            def count(m):
                return int(tot[m.lb_slot]) if m.lb_slot >= 0 else m.inflight
            free = [m for m in cands if count(m) < m.capacity] or cands
            m = min(free, key=lambda m: (count(m) / max(1, m.capacity), -m.tps))
            if acquire:
                m.inflight += 1
                if m.lb_slot >= 0:
                    bal.add(m.lb_slot, 1)
        return m

    def acquire(self, m: LocalModel) -> None:
        m.inflight += 1
        if self.balancer is not None and m.lb_slot >= 0:
            with self.balancer.locked():
                self.balancer.add(m.lb_slot, 1)

    def release(self, m: LocalModel) -> None:
        m.inflight -= 1
        if self.balancer is not None and m.lb_slot >= 0:
            self.balancer.release(m.lb_slot)
