"""Driver for rocprofv3 --pmc passes over the decode GEMM (K11) and the
library GEMM on one projection shape, cold weights (rotating copies), so the
per-dispatch counters of both kernels land in one counter_collection.csv.

    rocprofv3 --pmc <counters> -d DIR -o run --output-format csv -- \
        python tools/prof_dgemm_probe.py N K M CFG SPLITS EPI
"""
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from llm_mcp_amd import ops  # noqa: E402

N, K, M, CFG, S, EPI = (int(v) for v in sys.argv[1:7])
os.environ["LMX_DGEMM"] = "0"
dev = torch.device("cuda", 0)
ncopy = max(2, math.ceil((640 << 20) / (N * K * 2)))
ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02 for _ in range(ncopy)]
x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
for i in range(20):
    if EPI == 2:
        ops.dgemm_partials(x, ws[i % ncopy], CFG, S)
    else:
        ops.dgemm(x, ws[i % ncopy], CFG, S, EPI)
torch.cuda.synchronize()
for i in range(20):
    torch.nn.functional.linear(x, ws[i % ncopy])
torch.cuda.synchronize()
