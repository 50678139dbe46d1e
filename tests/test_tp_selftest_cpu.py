"""TP group start-up self-test (parallel/tp_worker.group_self_test) on gloo:
a healthy group passes; a group whose peer never joins the collective ends
the waiting rank with exit code 3 and a clear message instead of a hang."""
import os
import socket
import subprocess
import sys
import textwrap

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = textwrap.dedent("""
    import os, sys, time
    sys.path.insert(0, {root!r})
    import torch, torch.distributed as dist
    from llm_mcp_amd.models.llama import TPContext
    from llm_mcp_amd.parallel.tp_worker import group_self_test
    rank = int(os.environ["RANK"])
    dist.init_process_group("gloo")
    tp = TPContext(rank, 2, dist.group.WORLD)
    if rank == 1 and os.environ.get("SKIP_PEER") == "1":
        time.sleep(30)           # never joins the collectives
        sys.exit(0)
    print("RESULT", group_self_test(tp, torch.device("cpu"), timeout_s=float(os.environ["TMO"])),
          flush=True)
    dist.destroy_process_group()
""")


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _launch(skip_peer: bool, tmo: float):
    port = _port()
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), SKIP_PEER="1" if skip_peer else "0", TMO=str(tmo),
                   GLOO_SOCKET_IFNAME="lo")
        procs.append(subprocess.Popen([sys.executable, "-c", SCRIPT.format(root=ROOT)], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    return procs


def test_group_self_test_passes_on_a_healthy_group():
    procs = _launch(False, 60)
    outs = [p.communicate(timeout=120)[0] for p in procs]
    assert all(p.returncode == 0 for p in procs), outs
    assert all("RESULT {'backend': 'gloo'" in o for o in outs), outs


def test_group_self_test_exits_instead_of_hanging():
    procs = _launch(True, 3)
    try:
        out0 = procs[0].communicate(timeout=60)[0]
        assert procs[0].returncode == 3, out0
        assert "exiting instead of hanging" in out0
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
            p.communicate()
