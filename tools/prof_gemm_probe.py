"""Minimal driver for rocprofv3 --pmc passes over the hand-written GEMM:
five gemm_nt calls on a prefill-sized problem (uniform [-1,1) operands).
Usage: rocprofv3 --pmc <counters> -- python tools/prof_gemm_probe.py [M N K]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from llm_mcp_amd import ops  # noqa: E402

M, N, K = (int(v) for v in sys.argv[1:4]) if len(sys.argv) >= 4 else (16384, 4096, 4096)
x = torch.rand(M, K, device="cuda", dtype=torch.bfloat16) * 2 - 1
w = (torch.rand(N, K, device="cuda", dtype=torch.bfloat16) * 2 - 1) * K ** -0.5
for _ in range(5):
    ops.gemm_nt(x, w)
torch.cuda.synchronize()
