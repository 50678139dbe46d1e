"""Typed settings: every environment variable the framework reads, with its
type, default and meaning.

The reference is configured by environment variables only, scattered over
the Go core, the Python worker, the bridge and telemetry
(core/internal/config/config.go:9-34, worker/llm_worker/main.py:52-539,
mcp/src/index.ts:7-10, telemetry/llm_telemetry/main.py:139-145).  The same
names are honoured here (compatibility), the dead ones are dropped, and the
new ones carry the LMX_ prefix.  ``python -m llm_mcp_amd config`` prints the
table with the current values (secrets masked); ``validate()`` type-checks
the environment at process start.
"""
from __future__ import annotations

import os
from dataclasses import dataclass


@dataclass(frozen=True)
class Var:
    name: str
    type: type
    default: object
    doc: str
    secret: bool = False


VARS: list[Var] = [
    # ---- control plane (reference names) ----
    Var("CORE_HTTP_ADDR", str, ":8080", "core HTTP listen address"),
    Var("CORE_GRPC_ADDR", str, ":9090", "core gRPC address (listen on core, dial on workers)"),
    Var("CORE_HTTP_URL", str, "http://127.0.0.1:8080", "core URL used by workers / bridge"),
    Var("CORE_VERSION", str, "0.1.0", "version reported by /health (falls back to LLM_MCP_VERSION)"),
    Var("DB_DSN", str, "", "Postgres DSN (postgres://user:pass@host:5432/db?sslmode=disable)",
        secret=True),
    Var("DISCOVERY_INTERVAL", int, 0, "seconds between discovery runs (0 = off)"),
    Var("DEVICE_LIMITS_INTERVAL", int, 0, "seconds between device-limit refreshes"),
    Var("DEVICE_MAX_CONCURRENCY", int, 1, "jobs per device for devices without a capacity tag"),
    Var("DEVICE_LIMITS_JSON", str, "", "per-device limit specs (JSON, '*' = default)"),
    Var("DEVICE_LIMITS_FILE", str, "", "file with the device limit specs"),
    Var("STRICT_MODEL_LIMITS", int, 0, "1: unknown model size/context counts as too large"),
    Var("OPENROUTER_API_KEY", str, "", "cloud catalogue / cloud provider key", secret=True),
    Var("OPENROUTER_BASE_URL", str, "https://openrouter.ai/api/v1", "OpenRouter API base"),
    Var("OPENAI_API_KEY", str, "", "OpenAI key (cloud provider)", secret=True),
    Var("OPENAI_BASE_URL", str, "https://api.openai.com/v1", "OpenAI API base"),
    Var("CLOUD_EMBED_DIMENSIONS", int, 0, "Matryoshka truncation for cloud embeddings"),
    Var("LIGHTRAG_URL", str, "", "knowledge ingest target (LightRAG)"),
    Var("LIGHTRAG_API_KEY", str, "", "LightRAG key (no built-in default)", secret=True),
    Var("MEM0_URL", str, "", "knowledge ingest target (mem0)"),
    # ---- worker (reference names) ----
    Var("WORKER_ID", str, "", "worker id (default worker-<device>)"),
    Var("WORKER_LEASE_SECONDS", int, 60, "lease length; heartbeat every max(5, lease/2) s"),
    Var("WORKER_KINDS", str, "", "comma list of job kinds this worker claims (empty = all)"),
    # ---- bridge / MCP / telemetry (reference names) ----
    Var("MCP_HTTP_ADDR", str, "0.0.0.0:3333", "HTTP bridge listen address"),
    Var("BACKEND_URL", str, "http://localhost:3333", "MCP tool server -> bridge URL"),
    Var("MCP_PORT", int, 8765, "MCP streamable-HTTP port (mcp --http)"),
    Var("TELEMETRY_CHECK_INTERVAL", int, 30, "alert loop period (s)"),
    Var("ALERT_FAIL_THRESHOLD", int, 3, "attempts before a failed job is alerted"),
    Var("TELEGRAM_BOT_TOKEN", str, "", "Telegram alert sink", secret=True),
    Var("TELEGRAM_CHAT_ID", str, "", "Telegram chat (REPORT_CHAT_ID also accepted)"),
    Var("TELEGRAM_USE_MCP", bool, False, "send alerts through a telegram-mcp gateway"),
    Var("TELEGRAM_MCP_BASE_URL", str, "http://tgapi:8000", "telegram-mcp gateway URL"),
    Var("TELEGRAM_MCP_CHAT_ID", str, "", "chat for the gateway route (else TELEGRAM_CHAT_ID)"),
    Var("TELEGRAM_MCP_BOT_ID", int, 0, "gateway bot id (optional)"),
    Var("TELEGRAM_MCP_FALLBACK_DIRECT", bool, True,
        "fall back to the Bot API when the gateway fails"),
    Var("ALERT_WEBHOOK_URL", str, "", "webhook alert sink"),
    Var("LOG_LEVEL", str, "INFO", "python logging level"),
    # ---- MI355X serving (new) ----
    Var("LMX_STORE", str, "memory", "memory[:journal] | postgres"),
    Var("LMX_JOURNAL", str, "", "native queue journal file (crash durability, memory store)"),
    Var("LMX_SNAPSHOT", str, "", "catalog snapshot file (memory store)"),
    Var("LMX_GPUS", str, "", "GPUs served by `serve` (e.g. 0-7); default all enumerated"),
    Var("LMX_CHAT_MODEL", str, "llama-3-8b", "chat model preset / alias"),
    Var("LMX_EMBED_MODEL", str, "", "embedding model preset (e.g. nomic-embed-text)"),
    Var("LMX_EMBED_BATCH_TOKENS", int, 65536, "tokens per embedding-engine forward (whole requests packed up to this many tokens)"),
    Var("LMX_TP", int, 1, "tensor-parallel degree of a chat-model group"),
    Var("LMX_WEIGHTS", str, "", "safetensors dir of the chat model's real weights (`serve`)"),
    Var("LMX_MODEL_REGISTRY", str, "", "per-GPU placement 'GPUS:[tpN:|embed:]MODEL;...' "
        "(overrides LMX_CHAT_MODEL / LMX_TP for `serve`)"),
    Var("LMX_MAX_BATCH", int, 256, "max concurrent sequences per engine"),
    Var("LMX_MAX_BATCHED_TOKENS", int, 36864, "tokens per engine step (an idle engine takes a burst of prompts in steps this large); bench.py and serve share it"),
    Var("LMX_MIXED_PREFILL_TOKENS", int, 2048, "prompt tokens per step while >= LMX_MIXED_MIN_DECODES decode rows of earlier-arrived streams run (bounds the stall a new request's prefill puts on every decoding stream; burst-aware, see LMX_MIXED_LATER_STEPS); 0 = no cap"),
    Var("LMX_PREFIX_CACHE", int, 1, "1: full KV pages are hashed and kept (LRU) for reuse by later prompts with the same prefix; 0: pages return to the free list when their sequence ends"),
    Var("LMX_MIXED_MIN_DECODES", int, 32, "decode rows that make a step 'mixed' for LMX_MIXED_PREFILL_TOKENS"),
    Var("LMX_MIXED_LATER_STEPS", int, 8, "LMX_MIXED_PREFILL_TOKENS counts only decode rows whose request came >= this many scheduler steps before the newest request with prompt tokens left (streams interrupted by later arrivals); 0 = every decode row"),
    Var("LMX_AR_NORM_CS", int, 2, "fused TP all-reduce + RMSNorm: column chunks per row (blocks per row, >= 256 16-B columns each), so a rank's few decode rows spread over more CUs; 1 = one block per row"),
    Var("LMX_AR_SPIN", int, 1 << 25, "peer all-reduce: polls (s_sleep 1 each) a kernel waits for a TP peer before it gives up and sets the error word (the engine then fails the step)"),
    Var("LMX_ALLOW_CLOUD", int, 0, "1: allow cloud providers (never on the GPU hot path)"),
    Var("LMX_JOB_RETENTION_DAYS", float, 7.0, "purge finished jobs older than this"),
    Var("LMX_MAINTENANCE_INTERVAL", int, 60, "seconds between store maintenance ticks"),
    Var("LMX_JOB_STREAM_MAX_S", int, 3600, "max duration of one /v1/jobs/{id}/stream"),
    Var("LMX_SP_MIN_TOKENS", int, 0, "TP: steps with at least this many tokens run sequence-parallel (reduce-scatter/all-gather residual stream); 0 disables (default until the RCCL branch is measured on a multi-GPU node)"),
    Var("LMX_TP_MICROBATCH", str, "auto", "TP prefill micro-batches (two halves whose async RCCL all-reduces overlap the other half's compute): auto = RCCL groups at >= LMX_TP_MICROBATCH_MIN tokens, 1 always (also gloo), 0 off"),
    Var("LMX_TP_MICROBATCH_MIN", int, 2048, "step tokens from which LMX_TP_MICROBATCH=auto splits a pure-prefill TP step"),
    Var("LMX_LOOKAHEAD", str, "", "engine lookahead stepping (step n+1 scheduled and launched before step n's tokens are read back; input tokens gathered on the device): default on for GPU engines and one-GPU (gloo) TP rehearsals, opt-in (1) on RCCL TP groups until a multi-GPU run covers it; 1 forces it (also on CPU), 0 off"),
    Var("LMX_TP_SAMPLER", str, "race", "TP sampling: race = vocab-sharded exponential-race sampler (every rank samples its logits shard, B x 32-B record exchanges, no logits gathered); gather = the logits gathered to the sampling ranks and the K6 kernel"),
    Var("LMX_SAMPLER", str, "", "race: the vocab-sharded race sampler at TP = 1 too (the tokens a TP group draws for the same seeds); default: the K6 inverse-CDF kernel"),
    Var("LMX_RACE_ROUNDS", int, 4, "race sampler rejection rounds before the argmax fallback (top-p 0.95: ~0.05^rounds of rows)"),
    Var("LMX_FUSED_PREFILL_ROPE", str, "1", "1: prefill rows' q rotation runs inside the prefill attention kernel (the rope/cache kernel only rotates k and writes the cache); 0: the rope/cache kernel rotates q in place"),
    Var("LMX_FUSED_ENCODER_ROPE", str, "0", "1: the embedding encoders (nomic) rotate q inside the attention kernel as LMX_FUSED_PREFILL_ROPE does for Llama (measured slower once: off)"),
    Var("LMX_FUSED_DECODE_ROPE", str, "1", "1: decode rows' rotary embedding and KV-cache write run inside the paged decode attention kernel; 0: separate rope/cache kernel"),
    Var("LMX_ENCODER_LIBRARY", str, "0", "1: encoder (embedding-model) projections may run on hipBLASLt where the encoder table measured it faster than K13; 0 (default) keeps them on the hand-written kernels"),
    Var("LMX_LARGE_GEMM", str, "auto", "large-M (prefill) projections: k13 = the hand-written persistent GEMM, lib = hipBLASLt, auto = the faster of the two per the encoder table (K13 where unmeasured)"),
    Var("LMX_TP_PROBE_STEPS", int, 2000, "TP engines: every N steps all ranks time one decode-sized all-reduce (rccl_allreduce_seconds live samples; 0 = off)"),
    Var("LMX_TP_LEADER_TIMEOUT_S", float, 30.0, "TP follower: exit when the leader's mailbox heartbeat is older than this (or its pid is gone)"),
    Var("LMX_ENGINE_INFO_S", float, 5.0, "API process: cadence of live engine info polls (KV usage, running, waiting)"),
    Var("LMX_RESTART_BACKOFF_S", float, 1.0, "serve: first restart delay of a dead GPU worker (doubles per consecutive death)"),
    Var("LMX_RESTART_MAX_S", float, 60.0, "serve: cap of the worker restart backoff"),
    Var("LMX_STOP_GRACE_S", float, 20.0, "serve: seconds a worker gets to exit after SIGTERM at shutdown before SIGKILL"),
    Var("LMX_SOCKET_DIR", str, "", "serve: directory of the engine sockets (default /tmp)"),
    Var("LMX_DGEMM", str, "1", "0 disables the decode GEMM (K11) dispatch table (hipBLASLt everywhere)"),
    Var("LMX_PREFILL_WAVES", int, 4, "waves per prefill-attention workgroup at head dim 128 (4 or 8)"),
    Var("LMX_SK", str, "1", "0 disables the K13-SK (split-K 256x256 tile) entries of the decode GEMM table"),
    Var("LMX_ADMIT_QUIET_MS", float, 2.0, "idle engine: wait for more arrivals until this long passes without one (0: schedule at once)"),
    Var("LMX_ADMIT_MAX_MS", float, 25.0, "idle engine: longest wait for a burst of arrivals before the first step"),
    Var("LMX_STEP_TRACE", int, 0, "record the engine's eager (prefill / mixed) steps; bench.py logs each wave's steps"),
    Var("LMX_RESIDUAL_EPILOGUE", int, 1, "prefill O / down projections on K13 add into the residual stream in their epilogue (0: separate residual-add pass in the norm)"),
    Var("LMX_NORM_FOLD", str, "1", "TP = 1: fold the RMSNorm gains into QKV / gate-up at load; prefill steps on K13 then run no norm pass (row scales from the residual epilogue's sums of squares); 0 keeps the norm kernels"),
    Var("LMX_RS_SINGLE", str, "auto", "one copy of the MLP weights: gate/up and down stored only in K14's packed layout (K14 decode, K13 prefill with packed W) when the table runs them packed; auto = only when the weights take > 25 % of the GPU's memory (a small model keeps its row-major copy for K11 below 129 rows), 1 always, 0 never"),
    Var("LMX_K13_MIN_FILL", float, 0.6, "decode-sized projections (512..LMX_ROWS_SPLIT_MAX rows): below this fraction of K13's last 256-CU tile wave filled the product runs on hipBLASLt (0: K13 whenever the encoder table allows)"),
    Var("LMX_ROWS_SPLIT_MAX", int, 1024, "decode batches of 257..N rows: a projection with fewer than 128 K13 tiles runs as <= 256-row pieces on the decode kernels (0 disables: one K13 / library product)"),
    Var("LMX_RS_PACK_GB", float, 24.0, "budget for K14's packed copies of decode weights that are not stored packed-only (beside the row-major weights prefill reads)"),
    Var("LMX_RS", str, "1", "0 disables the K14 (register-streamed weights, csrc/kernels/rsgemm.hip) entries of the decode GEMM table"),
    Var("LMX_TP_SELFTEST_S", float, 180.0, "TP engines: seconds the start-up collective self-test may wait before the rank exits (code 3) instead of hanging"),
    Var("LMX_DGEMM_TABLE", str, "", "decode GEMM dispatch table (default llm_mcp_amd/config/dgemm_gfx950.json)"),
    Var("LMX_FAULT_LIVES", int, 0, "apply LMX_FAULT only in the first N lives of a supervised worker (0 = every life); the serve supervisor numbers lives in LMX_WORKER_LIFE"),
    Var("LMX_WORKER_LIFE", int, 1, "set by the serve supervisor: 1-based life of this worker slot (restarts + 1)"),
    Var("LMX_FAULT_DEVICE", str, "", "apply LMX_FAULT only in the worker whose device id ends with this (e.g. gpu0.r1)"),
    Var("LMX_WATCHDOG_S", float, 1.0, "worker: engine health check cadence; an unhealthy engine makes the worker exit for a restart"),
    Var("LMX_WATCHDOG_GRACE_S", float, 2.0, "worker: delay between detecting a broken engine and exiting"),
    Var("LMX_PROGRESS_S", float, 2.0, "worker: cadence of job progress reports (tokens so far)"),
    Var("LMX_PEER_NODES", str, "", "other nodes' core URLs polled by discovery"),
    Var("LMX_PEER_PORTS", str, "8080", "core ports probed on mesh / subnet hosts"),
    Var("LMX_DISCOVERY_TAILSCALE", int, 1, "probe Tailscale peers when the tailscale CLI exists"),
    Var("LMX_TAILSCALE_STATUS_FILE", str, "", "saved 'tailscale status --json' document to use instead of the CLI"),
    Var("DISCOVERY_EXTRA_ENDPOINTS", str, "", "extra peer host:port list (alias OLLAMA_EXTRA_ENDPOINTS)"),
    Var("OLLAMA_EXTRA_ENDPOINTS", str, "", "reference name of DISCOVERY_EXTRA_ENDPOINTS"),
    Var("DISCOVERY_SCAN_SUBNETS", int, 0, "scan DISCOVERY_SUBNETS for peer cores"),
    Var("DISCOVERY_SUBNETS", str, "", "CIDR list scanned when DISCOVERY_SCAN_SUBNETS=1 (max 1024 hosts)"),
    Var("LMX_NODE_ID", str, "", "host id used in device ids (default hostname)"),
    Var("LMX_FAKE_GPUS", int, 0, "enumerate N fake GPUs (tests / CPU hosts)"),
    Var("LMX_ALERT_TEMP_C", float, 95.0, "GPU temperature alert threshold"),
    Var("LMX_STEP_TIMEOUT", float, 120.0, "engine watchdog: a longer step marks the GPU hung"),
    Var("LMX_TORCH_PROFILE", str, "", "dir[:steps] -- torch.profiler timeline of engine steps"),
    Var("LMX_FAULT", str, "", "fault injection spec (job_crash:p,claim_drop:p,gpu_error:p,...)"),
    Var("LMX_FAULT_SEED", int, 0, "fault injection RNG seed"),
    Var("LMX_AUTOBUILD", int, 1, "build missing native extensions on import"),
    Var("LMX_DEBUG_SYNC", int, 0, "synchronize after every HIP kernel launch and name the faulting kernel (disables graphs)"),
    Var("LMX_CUSTOM_AR", int, 1, "TP all-reduce over IPC-mapped peer memory for decode sizes (0 = RCCL only)"),
    Var("LMX_AR_SLOT_MB", float, 16.0, "peer all-reduce: largest message (MB) per rank region slot"),
    Var("LMX_AR_ONESHOT_MAX", int, 524288, "peer all-reduce: one-shot up to this many bytes, two-shot above"),
    Var("LMX_TUNABLEOP", int, 1, "load the cold-cache hipBLASLt solution table at engine start"),
    Var("LMX_TUNABLEOP_FILE", str, "", "solution table (default llm_mcp_amd/config/tunableop_gfx950.csv)"),
    Var("LMX_OFFLOAD_ARCH", str, "gfx950", "hipcc --offload-arch for the kernels"),
    Var("HSA_ENABLE_IPC_MODE_LEGACY", str, "0", "keep 0: dmabuf IPC for RCCL between ranks"),
]

_BY_NAME = {v.name: v for v in VARS}


class SettingsError(ValueError):
    pass


def get(name: str):
    """Typed value of a registered variable (environment or default)."""
    v = _BY_NAME[name]
    raw = os.environ.get(name)
    if raw is None or raw == "":
        if name == "CORE_VERSION" and os.environ.get("LLM_MCP_VERSION"):
            return os.environ["LLM_MCP_VERSION"]
        return v.default
    if v.type is bool:
        s = raw.strip().lower()
        if s in ("1", "true", "yes", "y", "on"):
            return True
        if s in ("0", "false", "no", "n", "off"):
            return False
        raise SettingsError(f"{name}={raw!r} is not a valid bool")
    try:
        return v.type(raw)
    except ValueError as e:
        raise SettingsError(f"{name}={raw!r} is not a valid {v.type.__name__}") from e


def validate() -> dict:
    """Type-check every registered variable present in the environment."""
    return {v.name: get(v.name) for v in VARS}


def table(mask: bool = True) -> str:
    rows = ["| variable | type | default | current | meaning |", "|---|---|---|---|---|"]
    for v in VARS:
        cur = os.environ.get(v.name, "")
        if cur and v.secret and mask:
            cur = "***"
        rows.append(f"| `{v.name}` | {v.type.__name__} | `{v.default}` | `{cur}` | {v.doc} |")
    return "\n".join(rows)
