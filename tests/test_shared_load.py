"""Front-door balancing across API processes (api/shared_load.py): two
registries standing in for two API processes of one port, each with its own
row of the shared counts, spread an uneven split of streams exactly evenly
over the replicas and never past a replica's slots."""
import os
import multiprocessing as mp

import pytest

from llm_mcp_amd.api.registry import LocalModel, ModelRegistry
from llm_mcp_amd.api.shared_load import SharedLoad


def _registry(path, row, rows, n, cap):
    reg = ModelRegistry()
    reg.balancer = SharedLoad(path, row, rows, n)
    for i in range(n):
        reg.add(LocalModel("tiny-llama", "chat", f"gpu{i}", None, None, None, capacity=cap,
                           lb_slot=i))
    return reg


def test_two_processes_fill_every_replica_exactly(tmp_path):
    path = str(tmp_path / "load")
    n, cap = 8, 5
    a, b = _registry(path, 0, 2, n, cap), _registry(path, 1, 2, n, cap)
    # uneven connection split (SO_REUSEPORT hashing): 23 vs 17 of 40 streams
    picks = [a.select("tiny-llama", "chat", acquire=True).device_id for _ in range(23)]
    picks += [b.select("tiny-llama", "chat", acquire=True).device_id for _ in range(17)]
    per = {f"gpu{i}": picks.count(f"gpu{i}") for i in range(n)}
    assert set(per.values()) == {cap}, per          # without sharing: up to cap + 1
    # releases free the node-wide slot for the other process
    victim = next(m for m in a.replicas("tiny-llama") if m.device_id == "gpu3")
    a.release(victim)
    assert b.select("tiny-llama", "chat", acquire=True).device_id == "gpu3"


def test_private_counts_would_overfill():
    """The failure the shared table prevents: two independent balancers give
    their remainders to the same first replicas."""
    n, cap = 8, 5
    regs = []
    for _ in range(2):
        reg = ModelRegistry()
        for i in range(n):
            reg.add(LocalModel("m", "chat", f"gpu{i}", None, None, None, capacity=cap))
        regs.append(reg)
    picks = [regs[0].select("m", "chat", acquire=True).device_id for _ in range(23)]
    picks += [regs[1].select("m", "chat", acquire=True).device_id for _ in range(17)]
    assert max(picks.count(f"gpu{i}") for i in range(n)) > cap


def _worker(path, row, k, q):
    reg = _registry(path, row, 4, 4, 1000)
    got = [reg.select("tiny-llama", "chat", acquire=True).lb_slot for _ in range(k)]
    q.put(got)


def test_concurrent_processes(tmp_path):
    """Four real processes selecting at once: the flock keeps the node-wide
    counts exact (no lost updates), so the split stays within one stream."""
    path = str(tmp_path / "load")
    SharedLoad(path, 0, 4, 4)             # shape the file once
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ks = [150, 90, 120, 40]
    ps = [ctx.Process(target=_worker, args=(path, r, k, q)) for r, k in enumerate(ks)]
    for p in ps:
        p.start()
    got = [x for _ in ps for x in q.get(timeout=120)]
    for p in ps:
        p.join(timeout=60)
    per = [got.count(i) for i in range(4)]
    assert sum(per) == sum(ks)
    assert max(per) - min(per) <= 1, per


def test_shape_mismatch_rejected(tmp_path):
    path = str(tmp_path / "load")
    SharedLoad(path, 0, 2, 4)
    with pytest.raises(ValueError):
        SharedLoad(path, 0, 2, 8)
