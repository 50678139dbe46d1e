"""Paged prefill / encoder attention (K3) at the served shapes, TFLOP/s:
nomic-embed-text (32 x 1024 tokens, 12 heads x 64, bidirectional),
mxbai-embed-large (64 x 512, 16 x 64, bidirectional) and a Llama-3-8B
prefill chunk (30 prompts x 546 tokens, 32 q / 8 kv x 128, causal).

    python tools/prefill_attn_probe.py [--iters 20]
"""
import argparse
import math
import os
import sys

# --pkg-root DIR: import llm_mcp_amd from DIR instead (a same-box A/B against another build)
_root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if "--pkg-root" in sys.argv:
    _i = sys.argv.index("--pkg-root")
    _root = os.path.abspath(sys.argv[_i + 1])
    del sys.argv[_i:_i + 2]
sys.path.insert(0, _root)
import torch  # noqa: E402

from llm_mcp_amd import ops  # noqa: E402

SHAPES = {"nomic": (32, 1024, 12, 12, 64, False), "mxbai": (64, 512, 16, 16, 64, False),
          "llama8b": (30, 546, 32, 8, 128, True),
          # long-context prefill steps (one 24576-token step of 2K / 7.7K prompts)
          "llama8b_2k": (12, 2048, 32, 8, 128, True),
          "llama8b_8k": (3, 7680, 32, 8, 128, True)}


def run(name, S, L, Hq, Hkv, D, causal, iters, ng=0, tag="", waves=4):
    dev = torch.device("cuda", 0)
    BS = 32
    T = S * L
    pages = -(-L // BS)
    NB = S * pages
    kc = torch.randn(NB, Hkv, BS, D, device=dev).to(torch.bfloat16)
    vc = torch.randn(NB, Hkv, BS // 4, D, 4, device=dev).to(torch.bfloat16)   # key-quad V pages
    bt = torch.randperm(NB, device=dev).to(torch.int32).view(S, pages)
    q = torch.randn(T, (Hq + 2 * Hkv) * D, device=dev).to(torch.bfloat16)
    cu = torch.arange(0, T + 1, L, dtype=torch.int32, device=dev)
    ctx = torch.full((S,), L, dtype=torch.int32, device=dev)
    if D != 128:
        waves = 4
    os.environ["LMX_PREFILL_WAVES"] = str(waves)
    qpt = 4 * ng * (16 // (Hq // Hkv)) if ng else ops.prefill_q_per_tile(Hq, Hkv, D)
    tiles = torch.tensor([v for s in range(S) for q0 in range(0, L, qpt) for v in (s, q0)],
                         dtype=torch.int32, device=dev)
    out = torch.empty(T, Hq * D, dtype=torch.bfloat16, device=dev)
    scale = 1 / math.sqrt(D)

    def call():
        ops.paged_prefill_attention(q, kc, vc, bt, cu, ctx, tiles, scale, out, causal=causal,
                                    Hq=Hq, q_per_tile=qpt)
    for _ in range(3):
        call()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        call()
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) / iters * 1e3
    flops = 4.0 * S * L * L * D * Hq * (0.5 if causal else 1.0)
    print(f"prefill attn {name:8s} {tag} {us:8.1f} us  {flops / us / 1e6:6.0f} TF/s", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--shapes", default="nomic,mxbai,llama8b",
                    help="comma list of " + ", ".join(SHAPES))
    ap.add_argument("--ng", type=int, default=0,
                    help="column groups per wave of the loaded build (A/B of an older .so)")
    ap.add_argument("--thr", default="8",
                    help="comma list of softmax lazy-rescale thresholds to interleave")
    ap.add_argument("--waves", default="4,8", help="comma list of waves per workgroup (head dim 128)")
    ap.add_argument("--xcd", default="2", help="comma list of workgroup orders (2 XCD-aware + reversed tile list, 1 XCD-aware, 0 hardware)")
    ap.add_argument("--stages", default="0",
                    help="comma list of LDS ring slot counts to interleave (0 = default)")
    a = ap.parse_args()
    thrs = [float(t) for t in a.thr.split(",")]
    stages = [int(t) for t in a.stages.split(",")]
    xcds = [int(t) for t in a.xcd.split(",")]
    wl = [int(t) for t in a.waves.split(",")]
    nat = ops.native()
    for _ in range(2):
        for name, shp in [(n, SHAPES[n]) for n in a.shapes.split(",")]:
            for thr in thrs:
                for st, xo, w in [(st, xo, w) for st in stages for xo in xcds for w in wl]:
                    if shp[4] != 128 and w != wl[0]:
                        continue
                    if hasattr(nat, "set_prefill_xcd"):
                        nat.set_prefill_xcd(xo)
                    if hasattr(nat, "set_prefill_rescale_thr"):
                        nat.set_prefill_rescale_thr(thr)
                    if hasattr(nat, "set_prefill_stages"):
                        nat.set_prefill_stages(st)
                    run(name, *shp, a.iters, a.ng,
                        tag=f"thr={thr:g} nst={st} xcd={xo} w={w}", waves=w)
    nat.set_prefill_stages(0)
    nat.set_prefill_xcd(2)


if __name__ == "__main__":
    main()
