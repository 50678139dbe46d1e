"""Embedding engine throughput without HTTP (nomic-embed-text or a BERT
embedder, bf16): docs of
--doc-len tokens in batches of --batch-tokens; reports embeddings/s, tok/s."""
import argparse
import json
import time

import torch

from llm_mcp_amd.engine.embed_engine import EmbeddingEngine
from llm_mcp_amd.models import config as mc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--docs", type=int, default=512)
    ap.add_argument("--doc-len", type=int, default=1024)
    ap.add_argument("--batch-tokens", type=int, default=None,
                    help="tokens per forward (default: the engine's, LMX_EMBED_BATCH_TOKENS)")
    ap.add_argument("--model", default="nomic-embed-text")
    a = ap.parse_args()
    cfg = mc.resolve(a.model)
    a.doc_len = min(a.doc_len, cfg.max_position)
    e = EmbeddingEngine(cfg, device="cuda", max_batch_tokens=a.batch_tokens)
    a.batch_tokens = e.max_batch_tokens
    g = torch.Generator().manual_seed(0)
    docs = [torch.randint(1000, 30000, (a.doc_len,), generator=g).tolist()
            for _ in range(a.docs)]
    per = max(1, a.batch_tokens // a.doc_len)
    e.embed_sync(docs[:per])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(0, a.docs, per):
        e.embed_sync(docs[i:i + per])
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    print(json.dumps({"model": a.model, "docs": a.docs, "doc_len": a.doc_len, "batch_docs": per,
                      "emb_per_s": round(a.docs / el, 1),
                      "tok_per_s": round(a.docs * a.doc_len / el, 1)}), flush=True)


if __name__ == "__main__":
    main()
