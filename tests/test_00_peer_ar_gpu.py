"""Peer-memory all-reduce and all-gather kernel (csrc/kernels/allreduce.hip) on the GPU.

The 1-GPU box maps every rank's IPC region into the other ranks' processes on
the same device, so the full protocol runs for real: IPC export/open, the
flag rendezvous, one-shot and two-shot, in place and out of place, and
hipGraph replay (device-side epochs).  Each rank checks its result against
the fp32 sum of every rank's seeded input computed on the host; the
all-gather (the TP logits path) against torch.cat of the shards.  Runs before
anything in this pytest process touches the GPU (ranks are spawned)."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _inputs(world, n, salt):
    return [(torch.randn(n, generator=torch.Generator().manual_seed(salt * 97 + r)) * (r + 1))
            .to(torch.bfloat16) for r in range(world)]


def _rank(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    import torch.distributed as dist

    from llm_mcp_amd.parallel.peer_allreduce import PeerAllReduce
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("gloo")
    errs, ar = [], None
    try:
        ar = PeerAllReduce(dist.group.WORLD, rank, world, dev, slot_bytes=8 << 20,
                           oneshot_max=256 << 10)
        cases = [(8 * world, False), (4096, False), (40000 * world, False), (1 << 20, False),
                 (3 << 20, True), (1 << 20, True)]
        for salt, (n, inplace) in enumerate(cases):
            xs = _inputs(world, n, salt)
            want = torch.stack([x.float() for x in xs]).sum(0)
            x = xs[rank].to(dev)
            out = ar(x) if inplace else ar(x, torch.empty_like(x))
            torch.cuda.synchronize()
            got = out.float().cpu()
            err = (got - want).abs().max().item()
            tol = 1e-2 * max(1.0, want.abs().max().item())
            if not err <= tol:
                errs.append(f"n={n} inplace={inplace} err={err}")
            two, _ = ar.plan(n * 2)
            errs += [f"n={n}: error word set"] if ar.error(clear=True) else []
            q.put(("case", rank, n, two))
        # hipGraph: capture once, replay with new inputs (epochs advance on the device)
        n = 64 << 10
        buf = torch.zeros(n, dtype=torch.bfloat16, device=dev)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            ar(buf)            # warm-up outside capture
        torch.cuda.synchronize()
        dist.barrier()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            ar(buf)
        for salt in range(100, 104):
            xs = _inputs(world, n, salt)
            buf.copy_(xs[rank].to(dev))
            torch.cuda.synchronize()
            dist.barrier()
            g.replay()
            torch.cuda.synchronize()
            want = torch.stack([x.float() for x in xs]).sum(0)
            err = (buf.float().cpu() - want).abs().max().item()
            if not err <= 1e-2 * max(1.0, want.abs().max().item()):
                errs.append(f"graph replay {salt}: err={err}")
        errs += ["graph: error word set"] if ar.error(clear=True) else []
        # all-gather (the TP logits path): to every rank and to rank 0 only,
        # eagerly and interleaved with all-reduces inside one captured graph
        for salt, (n, to_all) in enumerate([(8, True), (4096, False), (16032 * 4, True),
                                            (300000, False)], start=200):
            xs = _inputs(world, n, salt)
            want = torch.cat(xs)
            got = ar.all_gather(xs[rank].to(dev), None, to_all=to_all)
            torch.cuda.synchronize()
            if to_all or rank == 0:
                if got is None or not torch.equal(got.cpu(), want):
                    errs.append(f"all_gather n={n} to_all={to_all} mismatch")
            elif got is not None:
                errs.append("all_gather: a follower received the gather")
        errs += ["all_gather: error word set"] if ar.error(clear=True) else []
        n = 16032
        src = torch.zeros(n, dtype=torch.bfloat16, device=dev)
        red = torch.zeros(4096, dtype=torch.bfloat16, device=dev)
        gout = torch.zeros(world * n, dtype=torch.bfloat16, device=dev)
        with torch.cuda.stream(s):
            ar(red)
            ar.all_gather(src, gout)
        torch.cuda.synchronize()
        dist.barrier()
        g2 = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g2, stream=s):
            ar(red)
            ar.all_gather(src, gout)
        for salt in range(300, 303):
            xs, rs = _inputs(world, n, salt), _inputs(world, 4096, salt + 50)
            src.copy_(xs[rank].to(dev))
            red.copy_(rs[rank].to(dev))
            torch.cuda.synchronize()
            dist.barrier()
            g2.replay()
            torch.cuda.synchronize()
            if not torch.equal(gout.cpu(), torch.cat(xs)):
                errs.append(f"graph all_gather {salt} mismatch")
            want = torch.stack([x.float() for x in rs]).sum(0)
            if not (red.float().cpu() - want).abs().max().item() <= 1e-2 * max(
                    1.0, want.abs().max().item()):
                errs.append(f"graph all_reduce after gather {salt}")
        errs += ["graph all_gather: error word set"] if ar.error(clear=True) else []
        # fused all-reduce + residual add + RMSNorm (a TP sub-layer's tail):
        # bitwise equal to the all-reduce followed by ops.rms_norm(residual=),
        # one-shot and row-sharded two-shot (T not a multiple of the world too)
        from llm_mcp_amd import ops
        # column-split grids (up to 4 chunks; 2 by default) and one block per row
        shapes = [(1, 8192), (16, 8192), (37, 1024), (256, 8192), (300, 4096)]
        for salt, (T, cols, mcs) in enumerate([(T, c, m) for m in (4, 1) for T, c in shapes],
                                              start=400):
            ar.norm_max_cs = mcs
            xs = [x.view(T, cols) for x in _inputs(world, T * cols, salt)]
            res0 = _inputs(1, T * cols, salt + 7)[0].view(T, cols)
            wgt = (1 + 0.1 * torch.randn(cols, generator=torch.Generator().manual_seed(salt))
                   ).to(torch.bfloat16)
            x, res, wd = xs[rank].to(dev), res0.to(dev), wgt.to(dev)
            h = ar.all_reduce_norm(x, wd, 1e-5, res)
            res_u = res0.to(dev)
            h_u = ops.rms_norm(ar(x.clone()), wd, 1e-5, residual=res_u)
            torch.cuda.synchronize()
            # the residual stream bitwise; h up to the order of the sum of squares
            # (512 vs 256 threads per row): a last-bit difference of the scale
            if not (torch.equal(res, res_u) and torch.allclose(h.float(), h_u.float(),
                                                                atol=1e-2, rtol=1e-2)):
                errs.append(f"fused norm T={T} cols={cols} cs<={mcs}: differs from all-reduce "
                            "+ rms_norm")
            o = torch.stack([v.float() for v in xs]).sum(0).to(torch.bfloat16)
            r = (o.float() + res0.float()).to(torch.bfloat16).float()
            want = (r * torch.rsqrt(r.pow(2).mean(-1, keepdim=True) + 1e-5) * wgt.float())
            if not torch.allclose(h.float().cpu(), want, atol=3e-2, rtol=3e-2):
                errs.append(f"fused norm T={T} cols={cols} cs<={mcs}: vs fp32 reference")
        errs += ["fused norm: error word set"] if ar.error(clear=True) else []
        ar.norm_max_cs = 4
        # ... and inside a captured graph (device epochs), new inputs per replay
        T, cols = 64, 8192
        x = torch.zeros(T, cols, dtype=torch.bfloat16, device=dev)
        res = torch.zeros_like(x)
        wd = torch.ones(cols, dtype=torch.bfloat16, device=dev)
        hg = torch.empty_like(x)
        with torch.cuda.stream(s):
            ar.all_reduce_norm(x, wd, 1e-5, res, out=hg)
        torch.cuda.synchronize()
        dist.barrier()
        g3 = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g3, stream=s):
            ar.all_reduce_norm(x, wd, 1e-5, res, out=hg)
        for salt in range(500, 503):
            xs = [v.view(T, cols) for v in _inputs(world, T * cols, salt)]
            res0 = _inputs(1, T * cols, salt + 7)[0].view(T, cols)
            x.copy_(xs[rank].to(dev))
            res.copy_(res0.to(dev))
            torch.cuda.synchronize()
            dist.barrier()
            g3.replay()
            torch.cuda.synchronize()
            o = torch.stack([v.float() for v in xs]).sum(0).to(torch.bfloat16)
            r = (o.float() + res0.float()).to(torch.bfloat16).float()
            want = r * torch.rsqrt(r.pow(2).mean(-1, keepdim=True) + 1e-5)
            if not torch.allclose(hg.float().cpu(), want, atol=3e-2, rtol=3e-2):
                errs.append(f"graph fused norm {salt} mismatch")
        errs += ["graph fused norm: error word set"] if ar.error(clear=True) else []
        q.put(("done", rank, errs))
    except Exception as ex:   # report instead of hanging the parent
        q.put(("done", rank, [f"{type(ex).__name__}: {ex}"]))
    finally:
        if ar is not None:
            dist.barrier()
            ar.close()
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4, 8])
def test_peer_allreduce_matches_fp32_sum(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, world, port, q), daemon=True)
             for r in range(world)]
    for p in procs:
        p.start()
    done, modes = {}, set()
    try:
        while len(done) < world:
            msg = q.get(timeout=300)
            if msg[0] == "done":
                done[msg[1]] = msg[2]
            else:
                modes.add(msg[3])
        for p in procs:
            p.join(timeout=60)
            assert p.exitcode == 0
    finally:
        for p in procs:
            if p.is_alive():
                p.kill()
    assert modes == {0, 1}                        # both one-shot and two-shot ran
    assert all(not e for e in done.values()), done


def _race_rank(rank, world, port, q):
    """Vocab-sharded sampling (ops.sample_race) at TP = world on the one GPU:
    each rank holds its vocabulary shard of the logits, the records travel
    through the peer slots, and every rank gets the tokens of the one-shard
    run over the full rows -- eagerly and in a captured graph."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    import torch.distributed as dist

    from llm_mcp_amd import ops
    from llm_mcp_amd.models.llama import TPContext
    from llm_mcp_amd.models.weights import vocab_shard
    from llm_mcp_amd.parallel.peer_allreduce import PeerAllReduce
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("gloo")
    errs, ar = [], None
    try:
        ops.native()
        ar = PeerAllReduce(dist.group.WORLD, rank, world, dev, slot_bytes=4 << 20)
        tp = TPContext(rank, world, dist.group.WORLD)
        tp.peer = ar
        V, B = 128256, 256
        vs = vocab_shard(V, world)
        lo, hi = rank * vs, min(V, (rank + 1) * vs)

        def params(salt):
            g = torch.Generator().manual_seed(salt)
            t = torch.full((B,), 0.8)
            t[::17] = 0.0                               # greedy rows
            k = torch.zeros(B, dtype=torch.int32)
            k[1::5] = 40                                # top-k rows
            p = torch.full((B,), 0.95)
            p[2::7] = 0.5
            seeds = torch.randint(0, 1 << 40, (B,), generator=g)
            off = torch.randint(0, 1000, (B,), generator=g, dtype=torch.int32)
            return [x.to(dev) for x in (t, k, p, seeds, off)]

        def logits(salt):
            g = torch.Generator().manual_seed(1000 + salt)
            # a peaked head over a flat tail: nucleus sizes from 1 to thousands
            x = torch.randn(B, V, generator=g) * torch.linspace(0.5, 4.0, B)[:, None]
            return x.to(torch.bfloat16).to(dev)

        for salt in range(3):
            full, prm = logits(salt), params(salt)
            want_t, want_lp = ops.sample_race(full, *prm)
            shard = full[:, lo:hi].contiguous()
            got_t, got_lp = ops.sample_race(shard, *prm, exchange=tp.all_gather_records,
                                            v0=lo, vocab=V, world=world)
            torch.cuda.synchronize()
            if not torch.equal(got_t, want_t):
                n = int((got_t != want_t).sum())
                errs.append(f"salt {salt}: {n}/{B} tokens differ from the one-shard run")
            if not torch.allclose(got_lp, want_lp, atol=1e-3, rtol=1e-3):
                errs.append(f"salt {salt}: logprobs differ")
        # captured: new logits / params per replay
        buf = torch.zeros(B, hi - lo, dtype=torch.bfloat16, device=dev)
        pb = params(0)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            out = ops.sample_race(buf, *pb, exchange=tp.all_gather_records, v0=lo, vocab=V,
                                  world=world)
        torch.cuda.synchronize()
        dist.barrier()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            out = ops.sample_race(buf, *pb, exchange=tp.all_gather_records, v0=lo, vocab=V,
                                  world=world)
        for salt in range(10, 13):
            full, prm = logits(salt), params(salt)
            buf.copy_(full[:, lo:hi])
            for dst, src in zip(pb, prm):
                dst.copy_(src)
            want_t, _ = ops.sample_race(full, *prm)
            torch.cuda.synchronize()
            dist.barrier()
            g.replay()
            torch.cuda.synchronize()
            if not torch.equal(out[0], want_t):
                errs.append(f"graph salt {salt}: tokens differ")
        errs += ["race: error word set"] if ar.error(clear=True) else []
        q.put(("done", rank, errs))
    except Exception as ex:   # report instead of hanging the parent
        q.put(("done", rank, [f"{type(ex).__name__}: {ex}"]))
    finally:
        if ar is not None:
            dist.barrier()
            ar.close()
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4, 8])
def test_vocab_sharded_sampling_matches_one_shard(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_race_rank, args=(r, world, port, q), daemon=True)
             for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = [q.get(timeout=300) for _ in procs]
        for p in procs:
            p.join(timeout=60)
    finally:
        for p in procs:
            if p.is_alive():
                p.kill()
    errs = [e for r in res for e in r[2]]
    assert not errs, errs
