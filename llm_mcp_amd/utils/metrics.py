"""Prometheus metrics.

Every series of the reference is kept under its name
(core/internal/metrics/metrics.go:8-116): llmcore_embedding_requests_total,
_embedding_duration_seconds, _jobs_created_total (now actually incremented),
_devices_online, _discovery_runs_total, _discovery_duration_seconds,
_embedding_input_tokens_total, _chat_requests_total, _chat_duration_seconds,
_chat_tokens_total, _chat_cost_usd_total, _openrouter_balance_usd.

Serving series added: llm_ttft_seconds, llm_inter_token_seconds,
llm_generated_tokens_total, llm_batch_size, llm_kv_cache_usage_ratio,
llm_queue_wait_seconds, gpu_hbm_used_bytes, gpu_util, rccl_allreduce_seconds.
"""
from __future__ import annotations

from prometheus_client import (CollectorRegistry, Counter, Gauge, Histogram,
                               generate_latest)
from prometheus_client import CONTENT_TYPE_LATEST  # noqa: F401


class Metrics:
    def __init__(self, registry: CollectorRegistry | None = None):
        r = self.registry = registry or CollectorRegistry()
        self.embedding_requests = Counter("llmcore_embedding_requests_total",
                                          "Embedding requests", ["model", "device", "status"],
                                          registry=r)
        self.embedding_duration = Histogram(
            "llmcore_embedding_duration_seconds", "Embedding latency", ["model", "device"],
            buckets=(0.01, 0.025, 0.05, 0.1, 0.25, 0.5, 1, 2, 5, 10, 30, 60), registry=r)
        self.jobs_created = Counter("llmcore_jobs_created_total", "Jobs created", ["kind"],
                                    registry=r)
        self.devices_online = Gauge("llmcore_devices_online", "Devices online", registry=r)
        self.discovery_runs = Counter("llmcore_discovery_runs_total", "Discovery runs",
                                      ["status"], registry=r)
        self.discovery_duration = Histogram("llmcore_discovery_duration_seconds",
                                            "Discovery duration", registry=r)
        self.embedding_tokens = Counter("llmcore_embedding_input_tokens_total",
                                        "Embedding input tokens", ["model", "device"], registry=r)
        self.chat_requests_c = Counter("llmcore_chat_requests_total", "Chat requests",
                                       ["model", "provider", "status"], registry=r)
        self.chat_duration_h = Histogram(
            "llmcore_chat_duration_seconds", "Chat latency", ["model", "provider"],
            buckets=(0.05, 0.1, 0.25, 0.5, 1, 2, 5, 10, 20, 30, 60, 120), registry=r)
        self.chat_tokens_c = Counter("llmcore_chat_tokens_total", "Chat tokens",
                                     ["model", "provider", "direction"], registry=r)
        self.chat_cost = Counter("llmcore_chat_cost_usd_total", "Chat cost (USD)",
                                 ["model", "provider"], registry=r)
        self.openrouter_balance = Gauge("llmcore_openrouter_balance_usd", "OpenRouter balance",
                                        registry=r)
        # serving
        self.ttft_h = Histogram("llm_ttft_seconds", "Time to first token", ["model"],
                                buckets=(0.005, 0.01, 0.025, 0.05, 0.1, 0.25, 0.5, 1, 2, 5, 10),
                                registry=r)
        self.itl_h = Histogram("llm_inter_token_seconds", "Mean inter-token latency per request",
                               ["model"], buckets=(0.002, 0.005, 0.01, 0.02, 0.03, 0.05, 0.1,
                                                   0.2, 0.5), registry=r)
        self.generated = Counter("llm_generated_tokens_total", "Generated tokens", ["model"],
                                 registry=r)
        self.batch_size = Histogram("llm_batch_size", "Sequences per engine step", ["device"],
                                    buckets=(1, 2, 4, 8, 16, 32, 64, 128, 256, 512), registry=r)
        self.kv_usage = Gauge("llm_kv_cache_usage_ratio", "KV cache pages in use", ["device"],
                              registry=r)
        self.queue_wait = Histogram("llm_queue_wait_seconds", "Job queue wait", ["kind"],
                                    registry=r)
        self.hbm_used = Gauge("gpu_hbm_used_bytes", "HBM in use", ["device"], registry=r)
        self.gpu_util = Gauge("gpu_util", "GPU busy percent", ["device"], registry=r)
        self.allreduce = Histogram("rccl_allreduce_seconds", "TP all-reduce latency", ["group"],
                                   buckets=(1e-5, 3e-5, 1e-4, 3e-4, 1e-3, 3e-3, 1e-2),
                                   registry=r)

    # convenience recorders used by the handlers
    def chat_requests(self, model, provider, status):
        self.chat_requests_c.labels(model, provider, status).inc()

    def chat_duration(self, model, provider, seconds):
        self.chat_duration_h.labels(model, provider).observe(seconds)

    def chat_tokens(self, model, provider, n_in, n_out):
        self.chat_tokens_c.labels(model, provider, "input").inc(n_in)
        self.chat_tokens_c.labels(model, provider, "output").inc(n_out)
        self.generated.labels(model).inc(n_out)

    def ttft(self, model, s):
        self.ttft_h.labels(model).observe(s)

    def inter_token(self, model, s):
        self.itl_h.labels(model).observe(s)

    def render(self) -> bytes:
        return generate_latest(self.registry)
