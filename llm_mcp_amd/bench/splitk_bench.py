"""Decode-shape GEMMs with cold weights: hipBLASLt (F.linear) vs the split-K
MFMA kernel (ops.gemm_splitk).  Weights rotate over enough copies (> 512 MB)
that every call streams them from HBM, as inside a decode step where 16 GB
of weights pass once per step (an isolated loop over one weight would hit
the 256 MB Infinity Cache).  Interleaved in one process (guide §5.4 rule 24)."""
import json

import torch
import torch.nn.functional as F

from llm_mcp_amd import ops

import argparse

SHAPES = {"llama-3-8b": {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096),
                        "down": (4096, 14336)},
          "llama-3-70b": {"qkv": (10240, 8192), "o": (8192, 8192), "gate_up": (57344, 8192),
                         "down": (8192, 28672)}}


def timed(fn, ws, iters=30):
    for i in range(3):
        fn(ws[i % len(ws)])
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for i in range(iters):
        fn(ws[i % len(ws)])
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama-3-8b", choices=sorted(SHAPES))
    ap.add_argument("--ms", default="1,16,64,128,256")
    a = ap.parse_args()
    for name, (N, K) in SHAPES[a.model].items():
        copies = max(2, int(600e6 // (N * K * 2)) + 1)
        ws = [(torch.randn(N, K, device="cuda") * K ** -0.5).to(torch.bfloat16)
              for _ in range(copies)]
        for M in [int(v) for v in a.ms.split(",")]:
            x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
            out = torch.empty(M, N, dtype=torch.bfloat16, device="cuda")
            t_lt = timed(lambda w: F.linear(x, w), ws)
            t_sk = timed(lambda w: ops.gemm_splitk(x, w, out), ws)
            print(json.dumps({"model": a.model, "gemm": name, "M": M, "N": N, "K": K,
                              "splits": ops.splitk_splits(N, K),
                              "hipblaslt_us": round(t_lt, 1), "splitk_us": round(t_sk, 1),
                              "splitk_weight_TBps": round(N * K * 2 / t_sk / 1e6, 2)}),
                  flush=True)
        del ws


if __name__ == "__main__":
    main()
