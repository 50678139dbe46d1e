"""llm_mcp_amd -- an MI355X-native LLM router, lease job queue and in-process
serving stack with the capabilities of plagness/LLM-MCP.

Layers (see SURVEY.md §1 for the reference's layer map):
  api/        OpenAI-compatible HTTP API, job API, SSE, dashboard, debug
  rpc/        llmmcp.v1.Core gRPC contract (server + client)
  mcp/        MCP tool server (JSON-RPC 2.0, stdio + HTTP) and HTTP bridge
  policy/     routing, circuit breaker, device limits / admission
  devices/    ROCm GPU enumerator (replaces Tailscale/Ollama discovery)
  store/      durable state: native lease queue, SQLite, Postgres wire client
  worker/     per-GPU worker: claim -> heartbeat -> execute -> complete
  engine/     continuous-batching engine over the paged KV cache
  models/     Llama-3 decoder, nomic-bert encoder, tokenizers
  ops/        gfx950 HIP kernels (csrc/kernels) + PyTorch references
  parallel/   process groups, tensor parallel, RCCL collectives
  telemetry/  alert loop and sinks
"""
__version__ = "2026.10.15"
