"""Engine-only benchmark (no HTTP): prefill throughput and decode step time
per batch size, with the engine's host-side phase breakdown.  Used to separate
GPU/kernel cost from API/SSE cost when profiling (rocprofv3 wraps this)."""
from __future__ import annotations

import argparse
import json
import time

import torch


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama-3-8b")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--prompt-len", type=int, default=512)
    ap.add_argument("--max-tokens", type=int, default=128)
    ap.add_argument("--temperature", type=float, default=0.8)
    ap.add_argument("--top-p", type=float, default=0.95)
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--max-batched-tokens", type=int, default=16384)
    a = ap.parse_args(argv)
    from llm_mcp_amd.engine.engine import EngineConfig, LLMEngine, SamplingParams
    e = LLMEngine(EngineConfig(model=a.model, max_num_seqs=a.batch,
                               max_batched_tokens=a.max_batched_tokens,
                               max_model_len=a.prompt_len + a.max_tokens + 64,
                               use_graphs=not a.no_graphs, kv_cache_gb=24), device="cuda")
    g = torch.Generator().manual_seed(0)
    prompts = [torch.randint(0, 128000, (a.prompt_len,), generator=g).tolist()
               for _ in range(a.batch)]
    sp = SamplingParams(temperature=a.temperature, top_p=a.top_p, max_tokens=a.max_tokens,
                        ignore_eos=True, seed=1)
    e.generate(prompts[:8], SamplingParams(max_tokens=4, ignore_eos=True))  # warm
    for k in list(e.stats):
        e.stats[k] = 0 if isinstance(e.stats[k], int) else 0.0
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    outs = e.generate(prompts, sp)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    st = dict(e.stats)
    ntok = sum(len(o) for o in outs)
    dsteps = max(1, st["graph_steps"])
    res = {"batch": a.batch, "elapsed_s": round(el, 3), "gen_tokens": ntok,
           "tok_s": round(ntok / el, 1), **{k: (round(v, 4) if isinstance(v, float) else v)
                                            for k, v in st.items()},
           "ms_per_step_avg": round(st["step_time_s"] / max(1, st["steps"]) * 1e3, 3)}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
