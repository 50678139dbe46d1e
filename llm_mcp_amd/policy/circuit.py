"""Per-device circuit breaker (reference: core/internal/routing/router.go:21-89).

3 consecutive failures -> "degraded" for 5 minutes -> "probe" (traffic allowed
again) -> any success deletes the entry.  Unlike the reference, which only
consulted it in findLocalModel, every selection path here consults it
(registry.select, Router.select_device, smart routing)."""
from __future__ import annotations

import threading
import time

FAILURE_THRESHOLD = 3
DEGRADED_SECONDS = 300.0


class CircuitBreaker:
    def __init__(self, clock=time.time, threshold: int = FAILURE_THRESHOLD,
                 degraded_s: float = DEGRADED_SECONDS):
        self.clock = clock
        self.threshold = threshold
        self.degraded_s = degraded_s
        self._lock = threading.RLock()
        self._c: dict[str, dict] = {}
        # ok -> degraded transitions per device since start (observability:
        # a trip can be shorter than any dashboard poll, e.g. a restarted
        # worker's first success closes it again)
        self.trips: dict[str, int] = {}

    def record(self, device_id: str, success: bool) -> None:
        if not device_id:
            return
        with self._lock:
            if success:
                self._c.pop(device_id, None)
                return
            c = self._c.setdefault(device_id, {"failures": 0, "degraded_at": 0.0})
            c["failures"] += 1
            if c["failures"] >= self.threshold:
                if c["failures"] == self.threshold:
                    self.trips[device_id] = self.trips.get(device_id, 0) + 1
                c["degraded_at"] = self.clock()

    # reference name
    record_device_result = record

    def is_degraded(self, device_id: str) -> bool:
        with self._lock:
            c = self._c.get(device_id)
            if c is None or c["failures"] < self.threshold:
                return False
            return self.clock() - c["degraded_at"] <= self.degraded_s

    def status(self, device_id: str) -> str:
        with self._lock:
            c = self._c.get(device_id)
            if c is None or c["failures"] < self.threshold:
                return "ok"
            if self.clock() - c["degraded_at"] > self.degraded_s:
                return "probe"
            return "degraded"

    def snapshot(self) -> dict:
        with self._lock:
            return {k: dict(v) for k, v in self._c.items()}

    def _set(self, device_id: str, failures: int, degraded_at: float) -> None:
        """Test hook: write the state directly (the reference's tests do this)."""
        with self._lock:
            self._c[device_id] = {"failures": failures, "degraded_at": degraded_at}
