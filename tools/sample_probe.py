"""K6 sampling at the headline decode shape: 256 rows x 128256 bf16 logits
(Llama-3), temperature 0.8 / top-p 0.95 (the bench's), plus greedy.  Logits
rotate over copies so each call reads its rows from HBM / the MALL as after
the LM head.  Prints us per call.

    python tools/sample_probe.py [--rows 256] [--iters 50] [--fns sample,sample_race]

sample_race (one shard, the TP-decomposable form) is timed eagerly and, with
--graph, replayed from a captured graph (its 9 launches, as in a decode graph).
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from llm_mcp_amd import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=256)
    ap.add_argument("--vocab", type=int, default=128256)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--fns", default="sample,sample_race")
    ap.add_argument("--graph", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    B, V = a.rows, a.vocab
    copies = [(torch.randn(B, V, device=dev) * 1.3).to(torch.bfloat16) for _ in range(6)]
    seeds = torch.arange(B, device=dev, dtype=torch.int64) + 7
    off = torch.zeros(B, device=dev, dtype=torch.int32)
    for name, t, p in (("temperature 0.8 top-p 0.95", 0.8, 0.95), ("temperature 0.8", 0.8, 1.0),
                       ("greedy", 0.0, 1.0)):
        tt = torch.full((B,), t, device=dev)
        kk = torch.zeros(B, device=dev, dtype=torch.int32)
        pp = torch.full((B,), p, device=dev)
        for fn in a.fns.split(","):
            f = getattr(ops, fn)
            tok0, _ = f(copies[0], tt, kk, pp, seeds, off)
            torch.cuda.synchronize()
            run = lambda i: f(copies[i % len(copies)], tt, kk, pp, seeds, off)  # noqa: E731
            if a.graph:
                gs = []
                st = torch.cuda.Stream()
                st.wait_stream(torch.cuda.current_stream())
                for c in range(len(copies)):
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g, stream=st):
                        f(copies[c], tt, kk, pp, seeds, off)
                    gs.append(g)
                torch.cuda.synchronize()
                run = lambda i: gs[i % len(gs)].replay()  # noqa: E731
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for i in range(a.iters):
                run(i)
            e.record()
            torch.cuda.synchronize()
            print(f"[{fn}{' graph' if a.graph else ''}] {name}: B={B} V={V}: "
                  f"{s.elapsed_time(e) / a.iters * 1e3:7.1f} us per call; "
                  f"first tokens {tok0[:4].tolist()}", flush=True)

if __name__ == "__main__":
    main()
