"""Down projection + its residual RMSNorm at the headline decode shape
(256 rows, Llama-3-8B: N 4096, K 14336): K14 partials (rsgemm epi 2) over
S split-K slabs, then rmsnorm_slabs reading the S fp32 slabs.  The table's
S was picked on the GEMM's time alone; this times the pair per S, on 8
rotating weight copies (cold as in the engine, where 32 layers' weights
stream through), with hipEvents over graph-free launches.

    python tools/down_norm_probe.py [--m 256] [--iters 200]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from llm_mcp_amd import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=256)
    ap.add_argument("--n", type=int, default=4096)
    ap.add_argument("--k", type=int, default=14336)
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--copies", type=int, default=8)
    a = ap.parse_args()
    ops.native()
    M, N, K = a.m, a.n, a.k
    torch.manual_seed(0)
    x = (torch.randn(M, K, device="cuda") * 0.1).to(torch.bfloat16)
    ws = []
    for _ in range(a.copies):
        w = (torch.randn(N, K, device="cuda") * K ** -0.5).to(torch.bfloat16)
        ws.append((w, ops.rsgemm_pack(w)))
    g = torch.ones(N, device="cuda", dtype=torch.bfloat16)
    res = torch.zeros(M, N, device="cuda", dtype=torch.bfloat16)
    ref = x.float() @ ws[0][0].float().t()
    print(f"M {M} N {N} K {K}; table choice {ops.rs_choice(M, N, K, 2, w=ws[0][0])}", flush=True)
    for cfg in (38, 42):
        for S in (2, 4, 8, 16):
            if not ops.rsgemm_supported(M, N, K, cfg, S, 2):
                continue
            p = ops.rsgemm(x, ws[0][1], cfg, S, epi=2, packed=True)
            err = (p.slabs.sum(0) - ref).abs().max().item()
            times = {}
            for what in ("gemm", "pair"):
                for _ in range(10):
                    ops.rsgemm(x, ws[0][1], cfg, S, epi=2, packed=True)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                e0.record()
                for i in range(a.iters):
                    p = ops.rsgemm(x, ws[i % a.copies][1], cfg, S, epi=2, packed=True)
                    if what == "pair":
                        ops.rms_norm(p, g, 1e-5, residual=res)
                e1.record()
                torch.cuda.synchronize()
                times[what] = e0.elapsed_time(e1) * 1000 / a.iters
            print(f"cfg {cfg} S {S:2d}: gemm {times['gemm']:6.2f} us  gemm+norm {times['pair']:6.2f} us"
                  f"  (norm {times['pair'] - times['gemm']:5.2f})  max err {err:.3g}", flush=True)


if __name__ == "__main__":
    main()
