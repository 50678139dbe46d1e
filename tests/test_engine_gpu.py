"""Engine on the GPU (HIP kernels + hipGraph decode) against the dense fp32
reference forward."""
import pytest
import torch

from llm_mcp_amd import ops
from llm_mcp_amd.engine.engine import EngineConfig, LLMEngine, SamplingParams
from tests.dense_ref import assert_greedy_consistent

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("graphs", [False, True])
def test_tiny_llama_engine_matches_dense(graphs):
    ops.native()
    e = LLMEngine(EngineConfig(model="tiny-llama", max_num_seqs=16, max_batched_tokens=128,
                               max_model_len=1024, use_graphs=graphs, kv_cache_gb=0.05),
                  device="cuda")
    prompts = [list(range(10, 50)), list(range(5, 300)), [7] * 33, [3]]
    outs = e.generate(prompts, SamplingParams(temperature=0, max_tokens=12, ignore_eos=True))
    for p, o in zip(prompts, outs):
        assert len(o) == 12
        assert_greedy_consistent(e.model, p, o)
    if graphs:
        assert e.stats["graph_steps"] > 0


def test_llama3_8b_decode_step_runs():
    ops.native()
    e = LLMEngine(EngineConfig(model="llama-3-8b", max_num_seqs=8, max_batched_tokens=1024,
                               max_model_len=2048, use_graphs=True, kv_cache_gb=4),
                  device="cuda")
    outs = e.generate([list(range(100, 400)), list(range(7, 40))],
                      SamplingParams(temperature=0.8, top_p=0.95, max_tokens=16, ignore_eos=True,
                                     seed=1))
    assert all(len(o) == 16 for o in outs)
    assert all(0 <= t < 128256 for o in outs for t in o)
    assert e.stats["graph_steps"] > 0
    torch.cuda.synchronize()
