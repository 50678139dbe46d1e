"""Deterministic fault injection for failure-path tests.

``LMX_FAULT="job_crash:0.2,gpu_error:0.05,claim_drop:0.1,step_hang:0.01"``
(probabilities) with ``LMX_FAULT_SEED``, or a fixed schedule
``LMX_FAULT="gpu_error@40/200"``: the fault fires on the 40th and 200th call
of its hook in this process (1-based; e.g. engine steps), so repeated runs of
a benchmark fail at the same points and differ only in performance.  The reference has no fault
injection; its failure paths (lease expiry, requeue, device offline) were
only exercised by real outages.

Hook points:
  job_crash   worker/agent.py, before a claimed job runs   -> job fails, requeued
  gpu_error   engine step                                  -> "HIP error" -> in-flight
                                                              requests fail, device offline
  claim_drop  worker/agent.py, after a claim               -> the job is dropped without a
                                                              heartbeat: its lease expires
  step_hang   engine step                                  -> the step sleeps LMX_FAULT_HANG_S
                                                              (hung-GPU watchdog test)
"""
from __future__ import annotations

import os
import random
import threading


class InjectedFault(RuntimeError):
    pass


class Faults:
    def __init__(self, spec: str | None = None, seed: int | None = None):
        spec = os.environ.get("LMX_FAULT", "") if spec is None else spec
        self.p: dict[str, float] = {}
        self.at: dict[str, set[int]] = {}     # name -> call indices that fire
        self.calls: dict[str, int] = {}
        for part in spec.split(","):
            if "@" in part:
                k, v = part.split("@", 1)
                self.at[k.strip()] = {int(x) for x in v.split("/") if x.strip()}
            elif ":" in part:
                k, v = part.split(":", 1)
                self.p[k.strip()] = float(v)
        seed = int(os.environ.get("LMX_FAULT_SEED", "0")) if seed is None else seed
        self._rng = random.Random(seed)
        self._lock = threading.Lock()
        self.fired: dict[str, int] = {}

    def __bool__(self) -> bool:
        return bool(self.p) or bool(self.at)

    def hit(self, name: str) -> bool:
        sched = self.at.get(name)
        if sched is not None:
            with self._lock:
                n = self.calls[name] = self.calls.get(name, 0) + 1
                fire = n in sched
                if fire:
                    self.fired[name] = self.fired.get(name, 0) + 1
            return fire
        p = self.p.get(name, 0.0)
        if p <= 0.0:
            return False
        with self._lock:
            fire = self._rng.random() < p
            if fire:
                self.fired[name] = self.fired.get(name, 0) + 1
        return fire

    def maybe_raise(self, name: str, msg: str | None = None) -> None:
        if self.hit(name):
            raise InjectedFault(msg or f"injected fault: {name}")


_GLOBAL: Faults | None = None


def faults() -> Faults:
    global _GLOBAL
    if _GLOBAL is None:
        _GLOBAL = Faults()
    return _GLOBAL


def set_faults(f: Faults | None) -> None:
    global _GLOBAL
    _GLOBAL = f
