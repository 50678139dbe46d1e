"""Decode products of 257-1024 rows on the Llama-3-8B projections: one
product (K13 from 512 rows, the library below) against ops.rows_split's
<= 256-row pieces on the decode kernels, per shape and row count, on 8
rotating weight copies (cold, as in the engine).  Checks the ROWS_SPLIT_TILES
threshold.

    python tools/rows_split_probe.py [--iters 100]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from llm_mcp_amd import ops  # noqa: E402

SHAPES = (("qkv", 6144, 4096), ("o", 4096, 4096), ("down", 4096, 14336), ("gate_up", 28672, 4096))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=100)
    ap.add_argument("--copies", type=int, default=6)
    ap.add_argument("--rows", default="320,384,448,512,640,768,896,1024,1280,1536")
    a = ap.parse_args()
    ops.native()
    torch.manual_seed(0)
    split_max = ops.ROWS_SPLIT_MAX
    for name, N, K in SHAPES:
        ws = []
        for _ in range(a.copies):
            w = (torch.randn(N, K, device="cuda") * K ** -0.5).to(torch.bfloat16)
            if name == "gate_up":
                w = ops.interleave_gate_up(w, ops.SWIGLU16)
            ops.rs_prepare(w)
            ws.append(w)

        def run(x, w):
            if name == "gate_up":
                return ops.linear_swiglu(x, w, ops.SWIGLU16)
            return ops.linear(x, w)

        for M in (int(v) for v in a.rows.split(",")):
            x = (torch.randn(M, K, device="cuda") * 0.1).to(torch.bfloat16)
            res = {}
            for mode in ("one", "split", "lib"):
                ops.ROWS_SPLIT_MAX = 0 if mode == "one" else split_max
                fn = run if mode != "lib" else (
                    (lambda x, w: ops.silu_mul(torch.nn.functional.linear(x, w), block=ops.SWIGLU16))
                    if name == "gate_up" else (lambda x, w: torch.nn.functional.linear(x, w)))
                y = fn(x, ws[0])
                res[mode + "_y"] = y
                for i in range(5):
                    fn(x, ws[i % a.copies])
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                e0.record()
                for i in range(a.iters):
                    fn(x, ws[i % a.copies])
                e1.record()
                torch.cuda.synchronize()
                res[mode] = e0.elapsed_time(e1) * 1000 / a.iters
            ops.ROWS_SPLIT_MAX = split_max
            piece = ops.rows_split(M, N, K, 3 if name == "gate_up" else 0, ws[0])
            tiles = -(-M // 256) * (N // 256)
            diff = (res["one_y"].float() - res["split_y"].float()).abs().max().item()
            print(f"{name:8s} M {M:5d} tiles {tiles:4d} piece {piece:3d}: one {res['one']:7.2f} us"
                  f"  pieces {res['split']:7.2f} us  ({res['one'] / res['split']:.2f}x)  library {res['lib']:7.2f} us"
                  f"  max diff {diff:.3g}",
                  flush=True)


if __name__ == "__main__":
    main()
