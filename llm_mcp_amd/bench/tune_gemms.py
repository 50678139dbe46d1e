"""Cold-cache GEMM tuning of the served projection shapes (hipBLASLt solution
choice via PyTorch TunableOp).

hipBLASLt's default heuristic picks, at decode batch 256, 48-96 workgroup
tilings for the QKV / O projections that run 2-4x off the weight-streaming
roofline inside a decode step (profiles/r1_gemm_decode_shapes.md).  TunableOp
times every hipBLASLt solution for a shape; with a rotating buffer larger
than the 256 MB Infinity Cache each candidate streams its weights from HBM,
as in the real step.  The winners are written to a CSV that the engine loads
at start (engine/engine.py, LMX_TUNABLEOP_FILE), tuning disabled at serve
time.

    python -m llm_mcp_amd.bench.tune_gemms --model llama-3-8b \\
        --out llm_mcp_amd/config/tunableop_gfx950.csv
"""
from __future__ import annotations

import argparse
import os
import time

import torch
import torch.nn.functional as F

DECODE_M = [1, 2, 4, 8, 16, 24, 32, 40, 48, 56, 64, 80, 96, 112, 128, 160, 192, 224, 256]


def shapes_for(model: str, tp: int = 1) -> list[tuple[int, int]]:
    from ..models import config as mc
    c = mc.resolve(model)
    D = c.head_dim
    hq, hkv, inter = c.num_heads // tp, max(1, c.num_kv_heads // tp), c.intermediate_size // tp
    d = c.hidden_size
    vocab = (c.vocab_size + tp - 1) // tp
    return [((hq + 2 * hkv) * D, d), (d, hq * D), (2 * inter, d), (d, inter), (vocab, d)]


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama-3-8b")
    ap.add_argument("--tp", type=int, default=1)
    ap.add_argument("--ms", default=",".join(map(str, DECODE_M)))
    ap.add_argument("--prefill-ms", default="16384", help="prefill chunk sizes (projections only)")
    ap.add_argument("--out", default="llm_mcp_amd/config/tunableop_gfx950.csv")
    ap.add_argument("--rotating-mb", type=int, default=1024)
    ap.add_argument("--max-ms", type=int, default=60, help="tuning time budget per shape")
    a = ap.parse_args(argv)
    tun = torch.cuda.tunable
    tun.enable(True)
    tun.tuning_enable(True)
    tun.set_filename(os.path.abspath(a.out), insert_device_ordinal=False)
    tun.set_rotating_buffer_size(a.rotating_mb)
    tun.set_max_tuning_duration(a.max_ms)
    tun.set_max_tuning_iterations(100)
    ms = [int(x) for x in a.ms.split(",")]
    pms = [int(x) for x in a.prefill_ms.split(",") if x]
    t0 = time.time()
    shapes = shapes_for(a.model, a.tp)
    for si, (N, K) in enumerate(shapes):
        w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * K ** -0.5
        lm_head = si == len(shapes) - 1
        for M in ms + ([] if lm_head else pms):
            x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
            F.linear(x, w)
            torch.cuda.synchronize()
        print(f"[tune] N={N} K={K}: {len(ms)} shapes tuned ({time.time() - t0:.0f}s)",
              flush=True)
    # TunableOp writes the results file when the process exits
    print(f"[tune] {len(tun.get_results())} tuned GEMMs -> {a.out} at exit", flush=True)


if __name__ == "__main__":
    main()
