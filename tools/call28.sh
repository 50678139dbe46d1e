# round 4, call 28: (1) K11 64 x 96 tiles on the Llama-3-8B QKV at 160-256
# rows (lab); (2) Llama-3-70B on one GPU (TP = 1), 128 streams x 128 tokens:
# the current stack, then with the K14 gate/up entry allowed its 75 GB packed
# copy (LMX_RS_PACK_GB=80)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m llm_mcp_amd.bench.dgemm_bench --only qkv --m 128,160,192,224,256 \
    --json gpurun_out/dg96_rows.json > gpurun_out/dg96_bench.log 2>&1 || exit $?
grep -i "qkv" gpurun_out/dg96_bench.log | tail -12
timeout -k 10 900 python bench.py --model llama-3-70b --concurrency 128 --max-tokens 128 --steps 2 --warmup 1 \
    > gpurun_out/l70_tp1.log 2>&1 || exit $?
tail -1 gpurun_out/l70_tp1.log | cut -c1-400
LMX_RS_PACK_GB=80 timeout -k 10 900 python bench.py --model llama-3-70b --concurrency 128 --max-tokens 128 --steps 2 --warmup 1 \
    > gpurun_out/l70_tp1_rs.log 2>&1 || exit $?
tail -1 gpurun_out/l70_tp1_rs.log | cut -c1-400
