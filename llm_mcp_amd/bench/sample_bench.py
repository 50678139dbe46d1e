"""Sampling kernel micro-benchmark at the decode shape (B rows x 128256
logits, bf16): greedy, temperature, temperature + top-p."""
import json

import torch

from llm_mcp_amd import ops
from llm_mcp_amd.bench.gemm_bench import timeit


def main():
    for B in (64, 256):
        lg = (torch.randn(B, 128256, device="cuda") * 2).to(torch.bfloat16)
        seeds = torch.arange(B, dtype=torch.int64, device="cuda")
        off = torch.zeros(B, dtype=torch.int32, device="cuda")
        k = torch.zeros(B, dtype=torch.int32, device="cuda")
        for name, t, p in (("greedy", 0.0, 1.0), ("temp0.8", 0.8, 1.0),
                           ("temp0.8_top_p0.95", 0.8, 0.95)):
            tt = torch.full((B,), t, device="cuda")
            pp = torch.full((B,), p, device="cuda")
            us = timeit(lambda: ops.sample(lg, tt, k, pp, seeds, off))
            print(json.dumps({"B": B, "mode": name, "us": round(us, 1),
                              "GBps": round(lg.numel() * 2 / us / 1e3, 1)}), flush=True)


if __name__ == "__main__":
    main()
