"""Alerting loop with pluggable sinks (reference: telemetry/llm_telemetry)."""
