# round 4, call 33: K11 stream-K form (cfg bit 6) -- lab timing on the
# Llama-3-70B QKV (M = 128) and Llama-3-8B QKV (M = 256) against the split-K
# forms, its GPU numerics tests, then dgemm_bench (vs hipBLASLt) on the 70B QKV
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/qkv_sk.log
: > $L
echo "== l70 qkv M=128" >> $L
timeout -k 10 120 tools/labbin/rsgemm_lab 10240 8192 128 0 dg:0x26:4,dg:0x66:0,dg:0x46:0,dg:0x61:0,dg:0x76:0,dg:0x60:0,dg:0x66:128,dg:0x61:512 >> $L 2>&1 || exit $?
echo "== l70 qkv M=96" >> $L
timeout -k 10 120 tools/labbin/rsgemm_lab 10240 8192 96 0 dg:0x66:0,dg:0x61:0,dg:0x76:0 >> $L 2>&1 || exit $?
echo "== l8b qkv M=256" >> $L
timeout -k 10 120 tools/labbin/rsgemm_lab 6144 4096 256 0 dg:0x23:2,dg:0x66:0,dg:0x61:0,dg:0x60:0,dg:0x76:0,dg:0x63:0 >> $L 2>&1 || exit $?
cat $L
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
    -k "stream_k or dgemm_configs" -p no:cacheprovider > gpurun_out/sk_tests.log 2>&1 || { tail -30 gpurun_out/sk_tests.log; exit 1; }
tail -2 gpurun_out/sk_tests.log
timeout -k 10 600 python -u -m llm_mcp_amd.bench.dgemm_bench --model llama-3-70b --only qkv --m 96,112,128,160,192 \
    --json gpurun_out/sk_rows.json > gpurun_out/sk_bench.log 2>&1 || exit $?
grep -i "qkv" gpurun_out/sk_bench.log | tail -12
