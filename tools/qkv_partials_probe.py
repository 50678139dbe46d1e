"""QKV projection at the headline decode shape (M = 256, N = 6144, K = 4096):
hipBLASLt (served TunableOp table) vs K11 partials-only (epi 2: S fp32 slabs,
the reduction left to the consumer), cold weights rotated over > 640 MB."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from llm_mcp_amd import ops  # noqa: E402
from llm_mcp_amd.engine.engine import _load_gemm_tuning  # noqa: E402


def t(fn, n=60):
    for i in range(5):
        fn(i)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for i in range(n):
        fn(i)
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3


def main():
    _load_gemm_tuning()
    dev = torch.device("cuda", 0)
    M, N, K = 256, 6144, 4096
    ws = [torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02 for _ in range(14)]
    x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    print(f"lib {t(lambda i: torch.nn.functional.linear(x, ws[i % 14])):.1f} us", flush=True)
    for cfg, (bm, bn) in enumerate(ops.DGEMM_CONFIGS):
        if N % bn or bm < 128:
            continue
        for S in (2, 4, 8):
            if K % (64 * S) or (-(-M // bm)) * (N // bn) * S > 1024:
                continue
            try:
                us = t(lambda i: ops.dgemm_partials(x, ws[i % 14], cfg, S))
            except Exception as e:   # noqa: BLE001
                print(f"cfg {cfg} S={S}: {e}", flush=True)
                continue
            print(f"partials cfg {cfg} ({bm}x{bn}) S={S}: {us:.1f} us", flush=True)


if __name__ == "__main__":
    main()
