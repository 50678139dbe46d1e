"""K13 (ops.pgemm) vs hipBLASLt (torch F.linear) on the encoder / prefill
shapes, uniform [-1, 1) operands, interleaved rounds in one process; TFLOP/s.

  python tools/pgemm_probe.py [--m 32768] [--rounds 5] [--only nomic]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from llm_mcp_amd import ops  # noqa: E402

SHAPES = {"nomic.qkv": (2304, 768), "nomic.o": (768, 768), "nomic.gate_up": (6144, 768),
          "nomic.down": (768, 3072), "l8b.qkv": (6144, 4096), "l8b.o": (4096, 4096),
          "l8b.gate_up": (28672, 4096), "l8b.down": (4096, 14336), "bert.qkv": (3072, 1024),
          "bert.o": (1024, 1024), "bert.w1": (4096, 1024), "bert.w2": (1024, 4096),
          "l70b.qkv": (10240, 8192), "l70b.o": (8192, 8192), "l70b.gate_up": (57344, 8192),
          "l70b.down": (8192, 28672)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", default="32768")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--only", default="")
    ap.add_argument("--grid", type=int, default=0)
    a = ap.parse_args()
    ops.native()
    torch.manual_seed(0)
    for M in [int(v) for v in a.m.split(",")]:
        for name, (N, K) in SHAPES.items():
            if a.only and not any(o in name for o in a.only.split(",")):
                continue
            x = torch.rand(M, K, device="cuda", dtype=torch.bfloat16) * 2 - 1
            w = (torch.rand(N, K, device="cuda", dtype=torch.bfloat16) * 2 - 1) * K ** -0.5
            out = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
            ref = torch.nn.functional.linear(x, w)
            ops.pgemm(x, w, out=out, grid=a.grid)
            err = (out.float() - ref.float()).abs().max().item()
            fl = 2.0 * M * N * K
            iters = max(3, min(50, int(3e12 / fl)))
            ev = lambda: torch.cuda.Event(enable_timing=True)
            t = {"lib": [], "k13": []}
            for _ in range(a.rounds):
                for kind in ("lib", "k13"):
                    s, e = ev(), ev()
                    fn = (lambda: torch.nn.functional.linear(x, w)) if kind == "lib" else \
                        (lambda: ops.pgemm(x, w, out=out, grid=a.grid))
                    fn()
                    s.record()
                    for _ in range(iters):
                        fn()
                    e.record()
                    torch.cuda.synchronize()
                    t[kind].append(s.elapsed_time(e) / iters * 1e3)
            med = {k: sorted(v)[len(v) // 2] for k, v in t.items()}
            print(f"{name:14s} M={M:6d} lib {fl / med['lib'] / 1e6:6.0f} TF | K13 "
                  f"{fl / med['k13'] / 1e6:6.0f} TF ({med['k13']:8.1f} us, "
                  f"{med['lib'] / med['k13']:.3f}x)  maxerr {err:.3g}", flush=True)


if __name__ == "__main__":
    main()
