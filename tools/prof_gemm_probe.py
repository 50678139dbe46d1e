import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch, sys
from llm_mcp_amd import ops
M,N,K=16384,4096,4096
x=(torch.rand(M,K,device='cuda',dtype=torch.bfloat16)*2-1)
w=(torch.rand(N,K,device='cuda',dtype=torch.bfloat16)*2-1)*K**-0.5
for impl in sys.argv[1].split(","):
    for _ in range(5): ops.gemm_nt(x,w,impl=impl)
torch.cuda.synchronize()
