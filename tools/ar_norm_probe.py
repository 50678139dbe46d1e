"""Local cost of the fused TP all-reduce + residual + RMSNorm
(allreduce.hip allreduce_norm_kernel) at world W with every rank on ONE GPU:
the W processes share the card, so this times the kernel's own work and the
peer-memory protocol through local HBM, not xGMI.  Column chunks per row
(LMX_AR_NORM_CS) 1 vs the split grid, decode shapes of Llama-3-70B TP = 8
(8192 columns) and Llama-3-8B TP = 2 (4096).  Rank 0 prints us per call.
Ranks sharing one card must all be resident at once, so the per-rank grid is
capped at 256 / W blocks here (PeerAllReduce.norm_plan): world 2 shows the
full 128-block grids, world 8 the capped ones.

    python tools/ar_norm_probe.py [--worlds 2,8] [--iters 50]
"""
import argparse
import os
import socket
import sys

import torch
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _rank(rank, world, port, iters, shapes, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    import torch.distributed as dist

    from llm_mcp_amd.parallel.peer_allreduce import PeerAllReduce
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("gloo")
    ar = PeerAllReduce(dist.group.WORLD, rank, world, dev, slot_bytes=16 << 20)
    out = []
    try:
        for T, cols in shapes:
            x = torch.randn(T, cols, device=dev).to(torch.bfloat16)
            res = torch.randn(T, cols, device=dev).to(torch.bfloat16)
            w = torch.ones(cols, device=dev, dtype=torch.bfloat16)
            h = torch.empty_like(x)
            for mcs in (1, 2, 4):
                ar.norm_max_cs = mcs
                two = int(T * cols * 2 > ar.oneshot_max and T >= world)
                plan = ar.norm_plan(T, cols, two)
                for _ in range(10):
                    ar.all_reduce_norm(x, w, 1e-5, res, out=h)
                torch.cuda.synchronize()
                dist.barrier()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(iters):
                    ar.all_reduce_norm(x, w, 1e-5, res, out=h)
                e.record()
                torch.cuda.synchronize()
                us = s.elapsed_time(e) / iters * 1e3
                dist.barrier()
                out.append((T, cols, mcs, plan, two, us))
                if rank == 0:
                    print(f"  world {world} T {T} cols {cols} max cs {mcs} grid {plan}: "
                          f"{us:.1f} us (rank 0)", flush=True)
        err = ar.error(clear=True)
        q.put((rank, out, err))
    finally:
        dist.barrier()
        ar.close()
        dist.destroy_process_group()


def run(world, iters, shapes):
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_rank, args=(r, world, port, iters, shapes, q), daemon=True)
             for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in procs:
        r, out, err = q.get(timeout=600)
        res[r] = (out, err)
    for p in procs:
        p.join(timeout=60)
    print(f"\nworld {world} on one GPU (local cost, not xGMI); us per call, max over ranks")
    print("| T | cols | two-shot | max cs | grid (groups x cs) | us |\n|---:|---:|---:|---:|---|---:|")
    for i, (T, cols, mcs, plan, two, _) in enumerate(res[0][0]):
        us = max(res[r][0][i][5] for r in res)
        print(f"| {T} | {cols} | {two} | {mcs} | {plan[0]} x {plan[1]} | {us:.1f} |")
    print("error words:", [res[r][1] for r in sorted(res)], flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--worlds", default="2,8")
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    shapes = [(256, 8192), (128, 8192), (64, 8192), (16, 8192), (256, 4096)]
    for w in a.worlds.split(","):
        run(int(w), a.iters, shapes)


if __name__ == "__main__":
    main()
