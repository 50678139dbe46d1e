"""BERT-architecture embedders (models/bert.py) and the HF checkpoint loaders
of both encoder families, on the CPU reference path:

* the packed varlen forward (paged scratch K/V, bidirectional attention,
  fused-residual LayerNorms, exact GELU, CLS / mean pooling, Matryoshka
  truncation) against an independent dense fp32 BERT written here;
* HF ``BertModel`` / nomic-bert safetensors -> loader -> same embeddings as
  the in-memory weights they were written from;
* ``from_hf_config`` for a BERT config.json and the embedding engine."""
import json

import torch
from safetensors.torch import save_file

from llm_mcp_amd.engine.embed_engine import EmbeddingEngine
from llm_mcp_amd.models import config as mc
from llm_mcp_amd.models.bert import BertModel, load_bert_weights
from llm_mcp_amd.models.nomic_bert import NomicBertModel, load_nomic_weights


def dense_bert(w, cfg, seq):
    """Plain fp32 BERT over one sequence (no packing, no paging)."""
    f = {k: v.float() for k, v in w.items() if k != "layers"}
    n, d, H, D = len(seq), cfg.hidden_size, cfg.num_heads, cfg.head_dim
    ids = torch.tensor(seq)
    x = f["word"][ids] + f["pos"][:n] + f["type"][0]
    ln = lambda t, g, b: torch.nn.functional.layer_norm(t, (d,), g.float(), b.float(),
                                                        cfg.ln_eps)
    x = ln(x, f["emb_ln_w"], f["emb_ln_b"]).bfloat16().float()
    for L in w["layers"]:
        L = {k: v.float() for k, v in L.items()}
        qkv = x @ L["wqkv"].t() + L["bqkv"]
        q, k, v = (qkv[:, i * d:(i + 1) * d].view(n, H, D).transpose(0, 1) for i in range(3))
        a = torch.softmax(q @ k.transpose(1, 2) / D ** 0.5, -1) @ v
        a = a.transpose(0, 1).reshape(n, d)
        h = ln(a @ L["wo"].t() + L["bo"] + x, L["ln1_w"], L["ln1_b"])
        g = torch.nn.functional.gelu(h @ L["w1"].t() + L["b1"])
        x = ln(g @ L["w2"].t() + L["b2"] + h, L["ln2_w"], L["ln2_b"])
    p = x[0] if cfg.pooling == "cls" else x.mean(0)
    return p / p.norm()


def _packed(lens, seed=0):
    g = torch.Generator().manual_seed(seed)
    ids = torch.randint(0, 500, (sum(lens),), generator=g, dtype=torch.int32)
    cu = torch.tensor([0] + list(torch.cumsum(torch.tensor(lens), 0)), dtype=torch.int32)
    return ids, cu


def test_bert_packed_forward_matches_dense_cls_and_mean():
    for preset in ("tiny-bert", "tiny-bert-mean"):
        cfg = mc.resolve(preset)
        m = BertModel(cfg, "cpu", seed=5)
        lens = [7, 1, 40, 33]
        ids, cu = _packed(lens)
        out = m.forward(ids, cu, lens)
        assert out.shape == (len(lens), cfg.embed_dim)
        for i, n in enumerate(lens):
            ref = dense_bert(m.w, cfg, ids[int(cu[i]):int(cu[i]) + n].tolist())
            cos = torch.nn.functional.cosine_similarity(out[i], ref, dim=0)
            assert float(cos) > 0.999, (preset, i, float(cos))
        # Matryoshka truncation re-normalises the leading dims
        t = m.forward(ids, cu, lens, dims=64)
        assert t.shape == (len(lens), 64)
        assert torch.allclose(t.norm(dim=-1), torch.ones(len(lens)), atol=1e-4)


def _hf_bert_state(w, cfg):
    sd = {}
    d = cfg.hidden_size
    e = "bert.embeddings."
    sd[e + "word_embeddings.weight"] = w["word"]
    sd[e + "position_embeddings.weight"] = w["pos"]
    sd[e + "token_type_embeddings.weight"] = w["type"]
    sd[e + "LayerNorm.weight"], sd[e + "LayerNorm.bias"] = w["emb_ln_w"], w["emb_ln_b"]
    for i, L in enumerate(w["layers"]):
        b = f"bert.encoder.layer.{i}."
        for j, n in enumerate(("query", "key", "value")):
            sd[b + f"attention.self.{n}.weight"] = L["wqkv"][j * d:(j + 1) * d]
            sd[b + f"attention.self.{n}.bias"] = L["bqkv"][j * d:(j + 1) * d]
        sd[b + "attention.output.dense.weight"], sd[b + "attention.output.dense.bias"] = \
            L["wo"], L["bo"]
        sd[b + "attention.output.LayerNorm.weight"] = L["ln1_w"]
        sd[b + "attention.output.LayerNorm.bias"] = L["ln1_b"]
        sd[b + "intermediate.dense.weight"], sd[b + "intermediate.dense.bias"] = L["w1"], L["b1"]
        sd[b + "output.dense.weight"], sd[b + "output.dense.bias"] = L["w2"], L["b2"]
        sd[b + "output.LayerNorm.weight"], sd[b + "output.LayerNorm.bias"] = \
            L["ln2_w"], L["ln2_b"]
    return {k: v.contiguous().clone() for k, v in sd.items()}


def test_hf_bert_checkpoint_roundtrip(tmp_path):
    cfg = mc.resolve("tiny-bert")
    m = BertModel(cfg, "cpu", seed=9)
    save_file(_hf_bert_state(m.w, cfg), str(tmp_path / "model.safetensors"))
    (tmp_path / "config.json").write_text(json.dumps({
        "architectures": ["BertModel"], "model_type": "bert", "vocab_size": cfg.vocab_size,
        "hidden_size": cfg.hidden_size, "intermediate_size": cfg.intermediate_size,
        "num_hidden_layers": cfg.num_layers, "num_attention_heads": cfg.num_heads,
        "max_position_embeddings": cfg.max_position, "layer_norm_eps": 1e-12}))
    cfg2 = mc.from_hf_config(tmp_path / "config.json")
    assert isinstance(cfg2, mc.BertConfig) and cfg2.head_dim == cfg.head_dim
    m2 = BertModel(cfg2, "cpu", weights=load_bert_weights(str(tmp_path), cfg2, "cpu"))
    lens = [12, 30]
    ids, cu = _packed(lens, 1)
    assert torch.allclose(m.forward(ids, cu, lens), m2.forward(ids, cu, lens), atol=1e-6)


def test_hf_nomic_checkpoint_roundtrip(tmp_path):
    cfg = mc.resolve("tiny-nomic")
    m = NomicBertModel(cfg, "cpu", seed=4)
    I = cfg.intermediate_size
    sd = {"embeddings.word_embeddings.weight": m.w["word"],
          "embeddings.token_type_embeddings.weight": m.w["type"],
          "emb_ln.weight": m.w["emb_ln_w"], "emb_ln.bias": m.w["emb_ln_b"]}
    for i, L in enumerate(m.w["layers"]):
        b = f"encoder.layers.{i}."
        sd.update({b + "attn.Wqkv.weight": L["wqkv"], b + "attn.out_proj.weight": L["wo"],
                   b + "mlp.fc12.weight": L["w_gate_up"][:I], b + "mlp.fc11.weight":
                   L["w_gate_up"][I:], b + "mlp.fc2.weight": L["w_down"],
                   b + "norm1.weight": L["ln1_w"], b + "norm1.bias": L["ln1_b"],
                   b + "norm2.weight": L["ln2_w"], b + "norm2.bias": L["ln2_b"]})
    save_file({k: v.contiguous().clone() for k, v in sd.items()},
              str(tmp_path / "model.safetensors"))
    m2 = NomicBertModel(cfg, "cpu", weights=load_nomic_weights(str(tmp_path), cfg, "cpu"))
    lens = [20, 3]
    ids, cu = _packed(lens, 2)
    assert torch.allclose(m.forward(ids, cu, lens), m2.forward(ids, cu, lens), atol=1e-6)


def test_embedding_engine_serves_bert():
    e = EmbeddingEngine(mc.resolve("tiny-bert"), device="cpu", max_batch_tokens=64)
    out = e.embed_sync([[1, 2, 3], list(range(10, 60)), [7]], dims=128)
    assert len(out) == 3 and all(len(v) == 128 for v in out)
    assert abs(sum(x * x for x in out[0]) - 1.0) < 1e-3
    assert mc.resolve("mxbai-embed-large:latest").pooling == "cls"
    assert 0.3 < mc.resolve("mxbai-embed-large").params_b < 0.4
