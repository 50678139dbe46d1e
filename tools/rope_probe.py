"""Decode rope/cache kernel cost split (1 GPU): the per-token kernel at the
decode-graph shape (256 tokens, Llama-3-8B heads), timed whole, without the
transposed-V scatter, and without any cache write.

    python tools/rope_probe.py [--tokens 256] [--bs 32]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from llm_mcp_amd import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=256)
    ap.add_argument("--bs", type=int, default=32)
    ap.add_argument("--iters", type=int, default=400)
    a = ap.parse_args()
    T, Hq, Hkv, D, BS = a.tokens, 32, 8, 128, a.bs
    dev = torch.device("cuda", 0)
    nb = T * 24
    qkv = torch.randn(T, (Hq + 2 * Hkv) * D, device=dev).to(torch.bfloat16)
    pos = torch.randint(0, 4000, (T,), device=dev, dtype=torch.int32)
    cs = torch.randn(4096, D, device=dev)
    pages = torch.randperm(nb, device=dev)[:T].to(torch.int32)
    slots = pages * BS + torch.randint(0, BS, (T,), device=dev, dtype=torch.int32)
    kc = torch.zeros(nb, Hkv, BS, D, device=dev, dtype=torch.bfloat16)
    vc = torch.zeros(nb, Hkv, BS // 4, D, 4, device=dev, dtype=torch.bfloat16)
    nat = ops.native()
    st = torch.cuda.current_stream().cuda_stream

    def call(slot_p, k_p, v_p):
        nat.rope_cache(qkv.data_ptr(), qkv.stride(0), pos.data_ptr(), cs.data_ptr(), T, Hq, Hkv, D,
                       slot_p, k_p, v_p, BS, 0, T, 0, 0, 1e-6, 0, st)

    variants = {
        "full": (slots.data_ptr(), kc.data_ptr(), vc.data_ptr()),
        "no V scatter": (slots.data_ptr(), kc.data_ptr(), 0),
        "no cache write": (0, 0, 0),
    }
    # prefill rows: 16,384 tokens of 32 prompts with consecutive slots (tiled kernel)
    TP = 16384
    qkvp = torch.randn(TP, (Hq + 2 * Hkv) * D, device=dev).to(torch.bfloat16)
    posp = (torch.arange(TP, device=dev, dtype=torch.int32) % 512)
    slotsp = torch.arange(TP, device=dev, dtype=torch.int32)
    kcp = torch.zeros(TP // BS, Hkv, BS, D, device=dev, dtype=torch.bfloat16)
    vcp = torch.zeros(TP // BS, Hkv, BS // 4, D, 4, device=dev, dtype=torch.bfloat16)
    for skip_q in (0, 1):      # 1: the engine's prefill form (q rotated in attention)
        for _ in range(5):
            nat.rope_cache(qkvp.data_ptr(), qkvp.stride(0), posp.data_ptr(), cs.data_ptr(), TP,
                           Hq, Hkv, D, slotsp.data_ptr(), kcp.data_ptr(), vcp.data_ptr(), BS, 0,
                           0, 0, 0, 1e-6, skip_q, st)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(50):
            nat.rope_cache(qkvp.data_ptr(), qkvp.stride(0), posp.data_ptr(), cs.data_ptr(), TP,
                           Hq, Hkv, D, slotsp.data_ptr(), kcp.data_ptr(), vcp.data_ptr(), BS, 0,
                           0, 0, 0, 1e-6, skip_q, st)
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) / 50 * 1e3
        nbytes = TP * Hkv * D * 2 * 4 + (0 if skip_q else TP * Hq * D * 2 * 2)
        print(f"rope_cache tiled T={TP} skip_q={skip_q} {us:7.2f} us "
              f"({nbytes / us / 1e6:.2f} TB/s of q/k/v/cache bytes)", flush=True)
    for name, args in variants.items():
        for _ in range(10):
            call(*args)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(a.iters):
            call(*args)
        e.record()
        torch.cuda.synchronize()
        print(f"rope_cache T={T} {name:15s} {s.elapsed_time(e) / a.iters * 1e3:7.2f} us", flush=True)


if __name__ == "__main__":
    main()
