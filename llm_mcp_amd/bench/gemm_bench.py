"""GEMM micro-benchmark for the Llama-3 / nomic projection shapes:
hipBLASLt (torch F.linear, optionally through TunableOp) vs the hand-written
gfx950 MFMA GEMM (ops.gemm_nt).  Interleaved rounds in one process
(guide §5.4 rule 24), random operands (rule 25)."""
from __future__ import annotations

import argparse
import json

import torch
import torch.nn.functional as F

LLAMA8B = [(6144, 4096), (4096, 4096), (28672, 4096), (4096, 14336), (128256, 4096)]
NOMIC = [(2304, 768), (768, 768), (6144, 768), (768, 3072)]


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3  # us


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--ms", default="64,128,256,2048,16384")
    ap.add_argument("--model", default="llama", choices=["llama", "nomic"])
    ap.add_argument("--ours", action="store_true")
    a = ap.parse_args(argv)
    from llm_mcp_amd import ops
    shapes = LLAMA8B if a.model == "llama" else NOMIC
    for M in [int(x) for x in a.ms.split(",")]:
        for N, K in shapes:
            x = torch.rand(M, K, device="cuda", dtype=torch.bfloat16) * 2 - 1
            w = (torch.rand(N, K, device="cuda", dtype=torch.bfloat16) * 2 - 1) * K ** -0.5
            t = timeit(lambda: F.linear(x, w))
            rec = {"M": M, "N": N, "K": K, "hipblaslt_us": round(t, 1),
                   "hipblaslt_tflops": round(2 * M * N * K / t / 1e6, 1),
                   "hipblaslt_weight_tbs": round(N * K * 2 / t / 1e6, 2)}
            if a.ours and ops.gemm_nt_supported(N, K):
                t2 = timeit(lambda: ops.gemm_nt(x, w))
                rec.update(ours_us=round(t2, 1), ours_tflops=round(2 * M * N * K / t2 / 1e6, 1))
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
