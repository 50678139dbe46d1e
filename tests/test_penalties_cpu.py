"""Repetition / presence / frequency penalties (K6 prologue): reference
semantics, the native scheduler's penalty window, the engine end to end on
the CPU path, and the request mappings (OpenAI body, Ollama options, job
payloads with Ollama's repeat_penalty default for ``ollama.*`` kinds)."""
import numpy as np
import torch

from llm_mcp_amd.api.openai_chat import sampling_from_body
from llm_mcp_amd.engine.engine import EngineConfig, LLMEngine, SamplingParams
from llm_mcp_amd.native import runtime
from llm_mcp_amd.ops import ref
from llm_mcp_amd.worker.jobs import sampling_from_payload


def test_reference_semantics_by_hand():
    logits = torch.tensor([[2.0, -1.0, 0.5, 3.0, 1.0]])
    # window (right-aligned, W=6): prompt tokens 0, 1, then generated 3, 3, 2
    win = torch.tensor([[-1, 0, 1, 3, 3, 2]], dtype=torch.int32)
    ngen = torch.tensor([3], dtype=torch.int32)
    pen = torch.tensor([[2.0, 0.5, 0.25]])
    out = ref.apply_penalties(logits.clone(), win, ngen, pen)
    # token 0 (prompt only): 2 / 2 = 1; token 1 (prompt only, negative): -1 * 2
    # token 3: 3 / 2 - 0.25 * 2 - 0.5 = 0.5; token 2: 0.5 / 2 - 0.25 - 0.5 = -0.5
    # token 4 (not in window) untouched
    assert torch.allclose(out, torch.tensor([[1.0, -2.0, -0.5, 0.5, 1.0]]))


def test_scheduler_emits_right_aligned_window():
    rt = runtime()
    s = rt.Scheduler(64, 16, 4, 256, 512, True)
    s.add(1, list(range(100, 200)), 8, [], True, 0)
    s.add(2, [5, 6, 7], 8, [], True, 0)
    assert s.set_penalties(1, 1.3, 0.2, 0.1, 8)
    p = s.schedule(16)
    assert p["any_penalty"] and p["pen_window_len"] == 64
    W = p["pen_window_len"]
    win = p["pen_window"].reshape(-1, W)
    rows = {int(p["seq_ids"][p["sample_seq"][i]]): i for i in range(len(p["sample_rows"]))}
    r1, r2 = win[rows[1]], win[rows[2]]
    assert list(r1[-8:]) == list(range(192, 200)) and (r1[:-8] == -1).all()
    assert (r2 == -1).all()                                # unpenalised row: empty window
    prm = p["pen_params"].reshape(-1, 3)
    assert np.allclose(prm[rows[1]], [1.3, 0.2, 0.1]) and prm[rows[2]][0] == 1.0
    s.update(np.array([0, 0], dtype=np.int32))
    p = s.schedule(16)
    i1 = [i for i in range(len(p["sample_rows"])) if int(p["seq_ids"][p["sample_seq"][i]]) == 1][0]
    assert p["pen_ngen"][i1] == 1 and p["pen_window"].reshape(-1, W)[i1][-1] == 0


def test_engine_penalty_blocks_recent_tokens():
    e = LLMEngine(EngineConfig(model="tiny-llama", max_num_seqs=4, max_batched_tokens=128,
                               max_model_len=256), device="cpu")
    prompt = list(range(5, 25))
    sp = SamplingParams(temperature=0, max_tokens=30, ignore_eos=True,
                        repetition_penalty=1e4, presence_penalty=1e3, penalty_last_n=64)
    out = e.generate([prompt], sp)[0]
    ctx = list(prompt)
    for t in out:
        assert t not in ctx[-64:], (t, ctx[-64:])
        ctx.append(t)
    # neutral penalties leave greedy decoding unchanged
    a = e.generate([prompt], SamplingParams(temperature=0, max_tokens=8, ignore_eos=True))[0]
    b = e.generate([prompt], SamplingParams(temperature=0, max_tokens=8, ignore_eos=True,
                                            repetition_penalty=1.0, penalty_last_n=64))[0]
    assert a == b


def test_request_mappings():
    sp = sampling_from_body({"presence_penalty": 0.5, "frequency_penalty": 0.3}, 100)
    assert (sp.presence_penalty, sp.frequency_penalty, sp.repetition_penalty) == (0.5, 0.3, 1.0)
    assert sp.penalized()
    sp = sampling_from_body({"options": {"repeat_penalty": 1.2, "repeat_last_n": -1}}, 100)
    assert sp.repetition_penalty == 1.2 and sp.penalty_last_n == 64
    assert not sampling_from_body({}, 100).penalized()
    assert sampling_from_payload({"prompt": "x"}, ollama_defaults=True).repetition_penalty == 1.1
    assert sampling_from_payload({"prompt": "x"}).repetition_penalty == 1.0
    sp = sampling_from_payload({"options": {"repeat_penalty": 1.0, "repeat_last_n": 0}},
                               ollama_defaults=True)
    assert not sp.penalized()
