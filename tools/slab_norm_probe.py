"""RMSNorm over split-K partials (K1 over K11 epi-2 slabs) at the decode shape:
256 rows x 4096, S = 4 (O) and 8 (down) fp32 slabs + residual, per workgroup
size cap (ops.native().set_slab_norm_threads).  Slabs rotate over copies
larger than the L2 so every call reads HBM / MALL like the decode step."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_mcp_amd import ops  # noqa: E402


def main():
    nat = ops.native()
    dev = torch.device("cuda", 0)
    rows, cols = 256, 4096
    w = torch.randn(cols, device=dev, dtype=torch.bfloat16)
    out = torch.empty(rows, cols, device=dev, dtype=torch.bfloat16)
    res = torch.randn(rows, cols, device=dev, dtype=torch.bfloat16)
    st = torch.cuda.current_stream().cuda_stream
    for S in (4, 8):
        ncopy = 16
        slabs = [torch.randn(S, rows, cols, device=dev) for _ in range(ncopy)]
        for th in (256, 512, 256, 512):
            nat.set_slab_norm_threads(th)
            for i in range(ncopy):
                nat.rmsnorm_slabs(out.data_ptr(), res.data_ptr(), slabs[i].data_ptr(), S,
                                  rows * cols, w.data_ptr(), rows, cols, cols, 1e-5, st)
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            n = 200
            s.record()
            for i in range(n):
                nat.rmsnorm_slabs(out.data_ptr(), res.data_ptr(), slabs[i % ncopy].data_ptr(), S,
                                  rows * cols, w.data_ptr(), rows, cols, cols, 1e-5, st)
            e.record()
            torch.cuda.synchronize()
            print(f"S={S} threads<={th}: {s.elapsed_time(e) / n * 1e3:.2f} us", flush=True)
    nat.set_slab_norm_threads(512)


if __name__ == "__main__":
    main()
