"""Can decode attention (HBM-bound) run under the decode GEMMs (bound by the
per-CU vector-L1 fill rate)?  Times, at a half batch (--rows, default 128):

  * K14 gate/up + SwiGLU (Llama-3-8B 28672 x 4096, packed, cold: copies rotate)
  * paged decode attention (32 q / 8 kv heads, contexts 535-791, random pages)
  * both serially on one stream, and the two on two streams at once.

If "two streams" is well under "serial", a two-half-batch decode step whose
halves are shifted by one phase (attention of one half under the GEMMs of
the other) pays; if it is ~serial, the kernels do not share the chip.

    python tools/overlap_probe.py [--rows 128] [--iters 40]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from llm_mcp_amd import ops  # noqa: E402


def timed(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    fn(iters)
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=128)
    ap.add_argument("--iters", type=int, default=40)
    ap.add_argument("--copies", type=int, default=4)
    ap.add_argument("--what", default="gateup", choices=("gateup", "down", "qkv"))
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    M = a.rows
    N, K, epi = {"gateup": (28672, 4096, 3), "down": (4096, 14336, 0),
                 "qkv": (6144, 4096, 0)}[a.what]
    x = (torch.randn(M, K, device=dev) * 0.5).to(torch.bfloat16)
    ws = []
    for _ in range(a.copies):
        w = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
        ws.append(ops.rs_pack_only(w) if ops.rs_single_ok(w, epi == 3) else w)
        del w

    def gemm(i):
        w = ws[i % len(ws)]
        if epi == 3:
            return ops.linear_swiglu(x, w, ops.SWIGLU16)
        return ops.linear(x, w)

    # attention: M sequences, Llama-3-8B heads, random pages over a 2.6 GB cache
    Hq, Hkv, D, BS = 32, 8, 128, 32
    ctx = torch.randint(535, 792, (M,), dtype=torch.int32)
    maxb = (791 + BS - 1) // BS
    nb = 20000
    k_cache = (torch.randn(nb, Hkv, BS, D, device=dev) * 0.5).to(torch.bfloat16)
    v_cache = torch.randn(nb, Hkv, BS // 4, D, 4, device=dev).to(torch.bfloat16)
    q = torch.randn(M, Hq * D, device=dev).to(torch.bfloat16)
    cl = ctx.to(dev)
    nrot = max(1, min(8, nb // (M * maxb)))
    tables = [p.view(M, maxb).to(dev) for p in
              torch.randperm(nb)[:nrot * M * maxb].to(torch.int32).chunk(nrot)]
    out = torch.empty(M, Hq * D, device=dev, dtype=torch.bfloat16)
    order = torch.from_numpy(ops.decode_order(ctx.numpy())).to(dev)
    scale = D ** -0.5
    kv_bytes = int(ctx.sum()) * Hkv * D * 2 * 2

    def attn(i):
        ops.paged_decode_attention(q, k_cache, v_cache, tables[i % nrot], cl, scale, out, None,
                                   256, order=order, Hq=Hq)

    def run_gemm(n):
        for i in range(n):
            gemm(i)

    def run_attn(n):
        for i in range(n):
            attn(i)

    def run_serial(n):
        for i in range(n):
            gemm(i)
            attn(i)

    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def run_two(n):
        cur = torch.cuda.current_stream()
        s1.wait_stream(cur)
        s2.wait_stream(cur)
        with torch.cuda.stream(s1):
            run_gemm(n)
        with torch.cuda.stream(s2):
            run_attn(n)
        cur.wait_stream(s1)
        cur.wait_stream(s2)

    def run_pingpong(n):
        # the pipeline form: each stream alternates gemm / attention, the
        # second one phase behind, so one stream's attention meets the other's GEMM
        cur = torch.cuda.current_stream()
        s1.wait_stream(cur)
        s2.wait_stream(cur)
        with torch.cuda.stream(s2):
            attn(n + 1)
        for i in range(n):
            with torch.cuda.stream(s1):
                gemm(i)
                attn(i)
            with torch.cuda.stream(s2):
                gemm(i + 1)
                attn(i + 2)
        cur.wait_stream(s1)
        cur.wait_stream(s2)

    for f in (run_gemm, run_attn, run_serial, run_two):
        f(3)
    torch.cuda.synchronize()
    for rep in range(2):
        tg = timed(run_gemm, a.iters)
        ta = timed(run_attn, a.iters)
        ts = timed(run_serial, a.iters)
        tt = timed(run_two, a.iters)
        tp = timed(run_pingpong, a.iters) / 2
        print(f"[overlap] {a.what} M={M}: gemm {tg:6.1f} us, attention {ta:6.1f} us "
              f"({kv_bytes / ta / 1e6:4.2f} TB/s); serial {ts:6.1f} us/pair, two streams "
              f"{tt:6.1f} us/pair ({ts / tt:4.2f}x), ping-pong {tp:6.1f} us/pair", flush=True)


if __name__ == "__main__":
    main()
