"""The driver's scaling command path, on the CPU: ``python bench.py --gpus N``
started WITHOUT a launcher takes ``bench.self_launch`` (torch.distributed.run
with N child ranks on 127.0.0.1), every rank serves its engine behind the one
front door, and rank 0 prints the single JSON line of the driver contract.

``--cpu`` runs each rank's engine on the CPU (gloo) with a tiny model, so the
same code path -- self-launch, rendezvous, front door, load generators,
timed waves, max-over-ranks, the JSON line -- runs here with no GPU.  The
``--tp`` case builds TP groups through the same launcher (config 4's shape)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args, timeout=240):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["GLOO_SOCKET_IFNAME"] = "lo"
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--cpu", "--model", "tiny-llama",
           "--steps", "2", "--warmup", "1", "--concurrency", "4", "--max-tokens", "4",
           "--prompt-len", "32", "--max-batched-tokens", "512"] + list(args)
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]        # ONE JSON line, from rank 0 only
    return json.loads(lines[0]), p.stderr


@pytest.mark.parametrize("gpus,tp", [(2, 1), (4, 2)])
def test_bench_self_launch_json_contract(gpus, tp):
    out, err = _run("--gpus", str(gpus), "--tp", str(tp))
    assert "launching" in err                      # the self_launch branch ran
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
              "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config"):
        assert k in out, k
    assert out["n_gpus"] == gpus and out["steps"] == 2 and out["warmup"] == 1
    assert out["higher_is_better"] is True and out["scaling"] == "weak"
    assert out["dtype"] == "bf16" and out["cpu_plumbing"] is True
    n_eng = gpus // tp
    assert out["config"]["global_batch"] == 4 * n_eng
    par = out["config"]["parallelism"]
    assert par.startswith(f"dp{gpus}" if tp == 1 else f"dp{n_eng}xtp{tp}")
    # every engine served streams: tokens = steps x streams x max_tokens
    assert out["value"] > 0 and len(out["per_gpu_tok_s"]) == n_eng
    assert all(v > 0 for v in out["per_gpu_tok_s"])
    assert len(out["decode_step_ms"]) == gpus      # one entry per rank (max over ranks)
    if tp > 1:     # the TP group's start-up collective self-test ran and passed
        assert out["config"]["tp_group"]["startup_selftest"]["backend"] == "gloo"
    tokens = out["value"] * out["ms_per_step"] * out["steps"] / 1e3
    assert abs(tokens - 2 * (4 * n_eng) * 4) <= 0.02 * tokens


def test_bench_gpus_mismatch_exits_nonzero():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--cpu"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=120)
    assert p.returncode != 0 and "WORLD_SIZE=2" in p.stderr
