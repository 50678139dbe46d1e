"""K13-SK (ops.pgemm_sk: 256x256 ping-pong tile, split-K) vs the paths that
serve the decode projections now (hipBLASLt via F.linear, K11 table entries)
at decode batch sizes; cold weights by default, as in a decode graph replay (the whole
model's weights cycle through HBM between two uses, so the tested weight is
rotated over copies > 512 MB); us per call, median of interleaved rounds.

  python tools/pgemm_sk_probe.py [--m 256] [--splits 1,2,3,4] [--only gate_up]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from llm_mcp_amd import ops  # noqa: E402

# name: (N, K, act, epi)  -- gate_up runs the SwiGLU epilogue (vs library + GLU
# kernel); o / down the partials form read by the residual-add RMSNorm
SHAPES = {"l8b.qkv": (6144, 4096, 0, 0), "l8b.o": (4096, 4096, 0, 2),
          "l8b.gate_up": (28672, 4096, ops.ACT_SWIGLU, 0), "l8b.down": (4096, 14336, 0, 2),
          "l8b.lm_head": (128256, 4096, 0, 0),
          "l70b.qkv": (10240, 8192, 0, 0), "l70b.gate_up": (57344, 8192, ops.ACT_SWIGLU, 0),
          "l70b.down": (8192, 28672, 0, 2), "l70b.o": (8192, 8192, 0, 2),
          # Llama-3-70B TP = 8 per-rank shapes (LM head shard padded to 256-row tiles)
          "l70b.tp8_lm_head": (16128, 8192, 0, 0), "l70b.tp8_qkv": (1280, 8192, 0, 0)}


def bench(fn, iters, rounds_out, ws):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn(ws[0])
    s.record()
    for i in range(iters):
        fn(ws[i % len(ws)])
    e.record()
    torch.cuda.synchronize()
    rounds_out.append(s.elapsed_time(e) / iters * 1e3)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", default="256")
    ap.add_argument("--splits", default="1,2,3,4")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--only", default="")
    ap.add_argument("--warm", action="store_true", help="one weight copy (re-read from the Infinity Cache)")
    a = ap.parse_args()
    ops.native()
    torch.manual_seed(0)
    for M in [int(v) for v in a.m.split(",")]:
        for name, (N, K, act, epi) in SHAPES.items():
            if a.only and not any(o in name for o in a.only.split(",")):
                continue
            ncopy = 1 if a.warm else max(2, int(6e8 // (N * K * 2)) + 1)
            x = (torch.rand(M, K, device="cuda", dtype=torch.bfloat16) * 2 - 1)
            ws = [(torch.rand(N, K, device="cuda", dtype=torch.bfloat16) * 2 - 1) * K ** -0.5
                  for _ in range(ncopy)]
            # fp32 reference of copy 0
            y = x.float() @ ws[0].float().t()
            if act == ops.ACT_SWIGLU:
                y4 = y.view(M, N // 32, 2, 16)
                ref = (torch.nn.functional.silu(y4[:, :, 0]) * y4[:, :, 1]).reshape(M, N // 2)
                lib = lambda w: ops.silu_mul(torch.nn.functional.linear(x, w), block=16)  # noqa: E731
            else:
                ref = y
                lib = lambda w: torch.nn.functional.linear(x, w)  # noqa: E731
            cands = {"lib": lib}
            for S in [int(v) for v in a.splits.split(",")]:
                if not ops.pgemm_sk_supported(M, N, K, S):
                    continue
                if epi == 2:
                    cands[f"sk{S}p"] = (lambda w, S=S: ops.pgemm_sk(x, w, S, epi=2))
                cands[f"sk{S}"] = (lambda w, S=S: ops.pgemm_sk(x, w, S, act=act))
            errs = {}
            for k, fn in cands.items():
                out = fn(ws[0])
                if isinstance(out, ops.Partials):
                    out = out.slabs.sum(0)
                errs[k] = ((out.float() - ref).abs().max() / ref.abs().max()).item()
                # second call: re-armed counters
                out = fn(ws[0])
                if isinstance(out, ops.Partials):
                    out = out.slabs.sum(0)
                errs[k] = max(errs[k], ((out.float() - ref).abs().max() / ref.abs().max()).item())
            iters = 30
            t = {k: [] for k in cands}
            for _ in range(a.rounds):
                for k, fn in cands.items():
                    bench(fn, iters, t[k], ws)
            med = {k: sorted(v)[len(v) // 2] for k, v in t.items()}
            wb = N * K * 2
            line = " | ".join(f"{k} {med[k]:7.1f} us ({wb / med[k] / 1e6:4.2f} TB/s, err {errs[k]:.1e})"
                              for k in cands)
            print(f"{name:13s} M={M:4d} {line}", flush=True)


if __name__ == "__main__":
    main()
