"""BASELINE config 4 through the production launcher, on the CPU.

``python -m llm_mcp_amd serve --cpu --gpus 0-7 --tp 8 --weights CKPT`` starts
one ``torch.distributed.run`` group of 8 worker ranks (worker/main.py ->
parallel/tp_worker.run_tp_worker: leader serves the engine socket and the job
agent, followers execute its plans; gloo instead of RCCL).  Checked here:

* a greedy SSE chat through the core's /v1/chat/completions streams exactly
  the tokens of the dense fp32 forward of the same checkpoint (tests/dense_ref.py),
  within bf16 near-ties;
* killing the TP leader makes the followers exit (plan-channel liveness),
  the supervisor starts a fresh group, and the next chat succeeds.

Reference surface: /root/reference/core/internal/api/handlers.go:2087-2189
(chat completions), :2427-2587 (streamed Ollama chat)."""
import asyncio
import json
import os
import signal
import socket
import subprocess
import sys
import tempfile

import aiohttp
import pytest

from llm_mcp_amd.models import config as mc
from llm_mcp_amd.models.llama import LlamaModel
from llm_mcp_amd.models.tokenizer import apply_chat_template, for_model
from llm_mcp_amd.models.weights import save_hf_llama
from tests.dense_ref import assert_greedy_consistent

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ENV = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="1", LMX_RESTART_BACKOFF_S="0.5",
           LMX_STORE="memory", DISCOVERY_INTERVAL="0", LMX_FAKE_GPUS="8",
           LMX_TP_PROBE_STEPS="0", LOG_LEVEL="WARNING")


def _port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


async def _ready(url: str, timeout: float) -> dict:
    loop = asyncio.get_event_loop()
    end = loop.time() + timeout
    async with aiohttp.ClientSession() as s:
        while loop.time() < end:
            try:
                async with s.get(url + "/v1/models") as r:
                    if r.status == 200:
                        body = await r.json()
                        if any(m.get("id") == "tiny-llama-tp8" for m in body.get("data", [])):
                            return body
            except aiohttp.ClientError:
                pass
            await asyncio.sleep(1.0)
    raise TimeoutError("TP group never registered with the core")


async def _chat(url: str, content: str, max_tokens: int) -> list[int]:
    """Greedy SSE chat; the streamed token ids (logprobs entries with
    return_tokens_as_token_ids: one chunk per token)."""
    body = {"model": "tiny-llama-tp8", "messages": [{"role": "user", "content": content}],
            "stream": True, "max_tokens": max_tokens, "temperature": 0, "ignore_eos": True,
            "logprobs": True, "return_tokens_as_token_ids": True}
    ids = []
    async with aiohttp.ClientSession(timeout=aiohttp.ClientTimeout(total=240)) as s:
        async with s.post(url + "/v1/chat/completions", json=body) as r:
            assert r.status == 200, await r.text()
            async for line in r.content:
                if line.startswith(b"data: ") and line[6:].strip() != b"[DONE]":
                    ch = json.loads(line[6:]).get("choices") or []
                    for e in ((ch[0].get("logprobs") or {}).get("content") or []) if ch else []:
                        ids.append(int(e["token"].split(":")[1]))
    return ids


@pytest.mark.timeout(900)
def test_serve_tp8_chat_matches_dense_and_survives_a_leader_kill():
    import psutil

    cfg = mc.resolve("tiny-llama-tp8")
    model = LlamaModel(cfg, "cpu", seed=11)
    ckpt = tempfile.mkdtemp()
    save_hf_llama(model, cfg, ckpt)
    d = tempfile.mkdtemp()
    http, grpc = _port(), _port()
    url = f"http://127.0.0.1:{http}"
    core = subprocess.Popen(
        [sys.executable, "-m", "llm_mcp_amd", "serve", "--cpu", "--gpus", "0-7", "--tp", "8",
         "--chat-model", "tiny-llama-tp8", "--weights", ckpt, "--max-num-seqs", "8",
         "--socket-dir", d, "--http", f"127.0.0.1:{http}", "--grpc", f"127.0.0.1:{grpc}"],
        cwd=ROOT, env=ENV, start_new_session=True)

    def ranks():
        out = []
        for c in psutil.Process(core.pid).children(recursive=True):
            try:
                cl = " ".join(c.cmdline())
            except psutil.Error:
                continue
            if "llm_mcp_amd.worker.main" in cl and "torch.distributed.run" not in cl:
                out.append(c)
        return out

    try:
        async def go():
            await _ready(url, timeout=420)
            content = "tp eight"
            out = await _chat(url, content, 6)
            # the engine's prompt: the chat template over the model's tokenizer
            prompt = apply_chat_template(for_model(cfg), [{"role": "user", "content": content}])
            assert len(out) == 6, out
            assert_greedy_consistent(model, prompt, out)

            procs = ranks()
            assert len(procs) == 8, [p.cmdline() for p in procs]
            leader = next(p for p in procs if p.environ().get("RANK") == "0")
            old = {p.pid for p in procs}
            leader.send_signal(signal.SIGKILL)
            # the followers notice (leader pid gone / stale heartbeat) and exit
            gone, alive = psutil.wait_procs([p for p in procs if p.pid != leader.pid],
                                            timeout=120)
            assert not alive, [p.pid for p in alive]
            # a fresh group registers; chat works again
            loop = asyncio.get_event_loop()
            end = loop.time() + 420
            while loop.time() < end:
                new = ranks()
                if len(new) == 8 and not ({p.pid for p in new} & old):
                    break
                await asyncio.sleep(1.0)
            else:
                raise AssertionError("supervisor did not start a new TP group")
            await _ready(url, timeout=420)
            out2 = None
            for _ in range(60):
                try:
                    out2 = await _chat(url, content, 6)
                    break
                except (AssertionError, aiohttp.ClientError):
                    await asyncio.sleep(2.0)
            assert out2 == out              # same weights, same greedy stream
        asyncio.new_event_loop().run_until_complete(go())
    finally:
        try:
            os.killpg(core.pid, signal.SIGTERM)
        except ProcessLookupError:
            pass
        try:
            core.wait(timeout=60)
        except subprocess.TimeoutExpired:
            os.killpg(core.pid, signal.SIGKILL)
