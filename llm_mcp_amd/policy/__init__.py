"""Routing policy: circuit breaker, device limits/admission, provider/model
/device selection (reference: core/internal/routing, core/internal/limits)."""
