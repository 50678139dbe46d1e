"""Model presets that stand in for other deployments."""
import torch

from llm_mcp_amd.models import config as mc
from llm_mcp_amd.models.llama import LlamaModel
from llm_mcp_amd.models.weights import vocab_shard


def test_tp8_rank_proxy_has_the_rank_shapes():
    """llama-3-70b-tp8-rank is ONE rank of Llama-3-70B at TP = 8 as a TP = 1
    model (config 4 measured on one GPU): every decode GEMM has the rank's
    shape, and the O / down outputs stay bf16 (proxy_tp) as before an all-reduce."""
    full = mc.resolve("llama-3-70b")
    cfg = mc.resolve("llama-3-70b-tp8-rank@L1")
    assert cfg.proxy_tp == 8 and cfg.num_layers == 1
    assert cfg.vocab_size == vocab_shard(full.vocab_size, 8) == 16128
    assert cfg.intermediate_size == full.intermediate_size // 8
    assert (cfg.num_heads, cfg.num_kv_heads) == (full.num_heads // 8, full.num_kv_heads // 8)
    m = LlamaModel(cfg, "cpu", dtype=torch.bfloat16)
    L = m.w["layers"][0]
    assert tuple(L["wqkv"].shape) == (1280, 8192)
    assert tuple(L["wo"].shape) == (8192, 1024)
    assert tuple(L["w_gate_up"].shape) == (7168, 8192)
    assert tuple(L["w_down"].shape) == (8192, 3584)
    assert tuple(m.w["lm_head"].shape) == (16128, 8192)
    assert mc.resolve("llama-3-70b-tp8-rank").num_layers == 80
