# round 4, call 42: dgemm_bench on the buckets call40 left out -- the 8B QKV / O /
# down at 80 and 112 rows, the 70B gate/up (+ SwiGLU) and down at 64-128 rows
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m llm_mcp_amd.bench.dgemm_bench --only qkv,o,down --m 16,32,48,80,112 \
    --json gpurun_out/b42_8b_rows.json > gpurun_out/b42_8b.log 2>&1 || exit $?
grep -v "^ *!!" gpurun_out/b42_8b.log | tail -30
timeout -k 10 900 python -u -m llm_mcp_amd.bench.dgemm_bench --model llama-3-70b --only gate_up,down --m 64,96,128 \
    --json gpurun_out/b42_70b_rows.json > gpurun_out/b42_70b.log 2>&1 || exit $?
grep -v "^ *!!" gpurun_out/b42_70b.log | tail -12
