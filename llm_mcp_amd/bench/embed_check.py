import time, torch, json
from llm_mcp_amd.engine.embed_engine import EmbeddingEngine
from llm_mcp_amd.models import config as mc
from llm_mcp_amd.models.nomic_bert import NomicBertModel
torch.cuda.set_device(0)
e = EmbeddingEngine(mc.resolve("nomic-embed-text"), device="cuda", max_batch_tokens=65536)
seqs = [[(i*7+j)%30000+1000 for i in range(256)] for j in range(256)]
e.embed_sync(seqs[:8])
torch.cuda.synchronize()
for n in (1, 32, 256):
    t0 = time.time(); out = e.embed_sync(seqs[:n]); torch.cuda.synchronize(); dt = time.time()-t0
    print(json.dumps({"seqs": n, "tokens": n*256, "ms": round(dt*1e3,2), "emb_per_s": round(n/dt,1), "norm": round(sum(x*x for x in out[0]),4)}), flush=True)
# CPU-reference parity on a tiny model on GPU vs CPU
tm = mc.resolve("tiny-nomic")
g = NomicBertModel(tm, "cuda", seed=3)
wc = {k: (v.cpu() if hasattr(v, "cpu") else [{kk: vv.cpu() for kk, vv in L.items()} for L in v]) for k, v in g.w.items()}
c = NomicBertModel(tm, "cpu", weights=wc)
ids = torch.randint(0, 500, (70,), dtype=torch.int32)
cu = torch.tensor([0, 30, 31, 70], dtype=torch.int32)
a = g.forward(ids.cuda(), cu.cuda(), [30, 1, 39])
b = c.forward(ids, cu, [30, 1, 39])
print("max abs diff gpu vs cpu-ref", float((a.cpu()-b).abs().max()))
