"""Paged decode attention (K4) at the headline decode shape: 256 sequences,
Llama-3-8B heads (32 q / 8 kv x 128), contexts 535-791 (the bench wave's
range), random page tables over a 40 GB cache.  Times each loop form of the
kernel (ops.native().set_decode_mode) and reports the K/V stream in TB/s.

    python tools/decode_attn_probe.py [--batch 256] [--iters 50]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from llm_mcp_amd import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--hq", type=int, default=32, help="query heads (8 kv heads): 64 = Llama-3-70B")
    ap.add_argument("--hkv", type=int, default=8, help="kv heads (1 = a Llama-3-70B TP = 8 rank)")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--ctx-lo", type=int, default=535)
    ap.add_argument("--ctx-hi", type=int, default=791)
    ap.add_argument("--parts", type=int, default=1, help="split-K partitions per sequence")
    ap.add_argument("--part-tokens", type=int, default=256)
    ap.add_argument("--order", choices=("random", "desc", "asc"), default="random",
                    help="sequence order = workgroup dispatch order (longest-first test)")
    ap.add_argument("--layout", choices=("random", "contig", "engine"), default="random",
                    help="page placement: random pages; each sequence's pages contiguous; or the "
                         "engine's wave pattern (prompt pages contiguous per sequence, decode "
                         "pages handed out one per sequence in turn)")
    ap.add_argument("--pages", type=int, default=20000, help="pages in the cache")
    ap.add_argument("--rope", action="store_true",
                    help="the engine's fused form: q rows are whole unrotated QKV rows, the "
                         "kernel rotates q and writes the step's k/v at ctx-1")
    ap.add_argument("--modes", default="4,0,5,4,0,5")
    ap.add_argument("--head-major", action="store_true",
                    help="emulate a head-major cache ([kv head][block] pages): each (sequence, "
                         "kv head) becomes its own 1-kv-head sequence of the same context, so with "
                         "--layout contig every segment streams one contiguous run of pages")
    a = ap.parse_args()
    B, Hq, Hkv, D, BS = a.batch, a.hq, a.hkv, 128, 32
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    ctx = torch.randint(a.ctx_lo, a.ctx_hi + 1, (B,), dtype=torch.int32)
    if a.head_major:
        ctx = ctx.repeat_interleave(Hkv)
        B, Hq, a.pages, Hkv = B * Hkv, Hq // Hkv, a.pages * Hkv, 1
    if a.order != "random":
        ctx = ctx.sort(descending=a.order == "desc").values
    maxb = (a.ctx_hi + BS - 1) // BS
    nb = a.pages                                # 20000 pages x 64 KB x 2 = 2.6 GB (> MALL)
    k_cache = (torch.randn(nb, Hkv, BS, D, device=dev) * 0.5).to(torch.bfloat16)
    v_cache = torch.randn(nb, Hkv, BS // 4, D, 4, device=dev).to(torch.bfloat16)
    q = torch.randn(B, (Hq + 2 * Hkv if a.rope else Hq) * D, device=dev).to(torch.bfloat16)
    cl = ctx.to(dev)
    # page tables rotated per call over disjoint page sets: a call's K/V were
    # last read >= 640 MB of other pages ago, so they come from HBM (as in a
    # decode step, where the whole model streams between two calls of a layer)
    nrot = max(1, min(8, nb // (B * maxb)))
    def table(base):
        if a.layout == "random":
            return torch.randperm(nb)[:B * maxb].to(torch.int32).view(B, maxb)
        if a.layout == "contig":
            return (base + torch.arange(B * maxb, dtype=torch.int32)).view(B, maxb)
        # engine wave: prompt pages (ctx_lo tokens) contiguous per sequence,
        # then one page per sequence in turn as decode crosses page boundaries
        npr = (a.ctx_lo + BS - 1) // BS
        t = torch.empty(B, maxb, dtype=torch.int32)
        t[:, :npr] = (base + torch.arange(B * npr, dtype=torch.int32)).view(B, npr)
        nxt = base + B * npr
        for j in range(npr, maxb):
            t[:, j] = nxt + torch.arange(B, dtype=torch.int32)
            nxt += B
        return t
    tables = [table(i * B * maxb).to(dev) for i in range(nrot)]
    if a.layout == "random":
        tables = [p.view(B, maxb).to(dev) for p in
                  torch.randperm(nb)[:nrot * B * maxb].to(torch.int32).chunk(nrot)]
    bt = tables[0]
    out = torch.empty(B, Hq * D, device=dev, dtype=torch.bfloat16)
    kv_bytes = int(ctx.sum()) * Hkv * D * 2 * 2
    ws = ops.DecodeWorkspace(B, Hq, D, a.parts, dev) if a.parts > 1 else None
    order = torch.from_numpy(ops.decode_order(ctx.numpy())).to(dev)
    scale = D ** -0.5
    ref = None
    nat = ops.native()
    ropes = [None] * len(tables)
    if a.rope:
        from llm_mcp_amd.ops import ref as opsref
        cs = opsref.rope_cos_sin(8192, D, 500000.0, dev)
        pos = (cl - 1).to(torch.int32)
        ropes = [(pos, cs, (t[torch.arange(B, device=dev), (pos // BS).long()] * BS + pos % BS)
                  .to(torch.int32)) for t in tables]
    for mode in map(int, a.modes.split(",")):
        nat.set_decode_mode(mode)
        ops.paged_decode_attention(q, k_cache, v_cache, bt, cl, scale, out, ws, a.part_tokens,
                                   order=order, Hq=Hq, rope=ropes[0])
        torch.cuda.synchronize()
        if ref is None:
            ref = out.clone()
        same = "-" if mode in (2, 3) else ("bitwise" if torch.equal(out, ref) else
                                      f"max diff {(out.float() - ref.float()).abs().max():.3g}")
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for i in range(a.iters):
            ops.paged_decode_attention(q, k_cache, v_cache, tables[i % nrot], cl, scale, out, ws,
                                       a.part_tokens, order=order, Hq=Hq, rope=ropes[i % nrot])
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) / a.iters * 1e3
        print(f"decode attn {'rope ' if a.rope else ''}{'head-major ' if a.head_major else ''}{a.layout} pages={nb} B={B} parts {a.parts}x{a.part_tokens} {a.order} mode {mode}: {us:7.1f} us  {kv_bytes / us / 1e6:5.2f} TB/s  "
              f"vs first mode: {same}", flush=True)
    nat.set_decode_mode(0)
    if a.rope:
        # the unfused form: the per-token rope / cache kernel, then attention without rope
        pos_, cs_, _ = ropes[0]
        for rep in range(2):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for i in range(a.iters):
                _, _, sl = ropes[i % nrot]
                ops.rope_and_cache(q, pos_, cs_, Hq, Hkv, D, sl, k_cache, v_cache, tile_from=B)
                ops.paged_decode_attention(q, k_cache, v_cache, tables[i % nrot], cl, scale,
                                           out, ws, a.part_tokens, order=order, Hq=Hq)
            e.record()
            torch.cuda.synchronize()
            print(f"decode attn rope split (rope_cache kernel + attention): "
                  f"{s.elapsed_time(e) / a.iters * 1e3:7.1f} us", flush=True)


if __name__ == "__main__":
    main()
