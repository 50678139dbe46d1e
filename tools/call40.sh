# round 4, call 40: K11 cfg 31 (64 x 128, 128-deep K-steps) -- numerics tests,
# then dgemm_bench on the Llama-3-8B QKV / O / down (+ partials forms) at
# 64-256 rows and the Llama-3-70B QKV / O at 64-128 rows against the table
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
    -k "stream_k or dgemm_configs" -p no:cacheprovider > gpurun_out/k11_tests.log 2>&1 || { tail -30 gpurun_out/k11_tests.log; exit 1; }
tail -2 gpurun_out/k11_tests.log
timeout -k 10 900 python -u -m llm_mcp_amd.bench.dgemm_bench --only qkv,o,down --m 64,96,128,160,192,224,256 \
    --json gpurun_out/bk128_8b_rows.json > gpurun_out/bk128_8b.log 2>&1 || exit $?
grep -v "^ *!!" gpurun_out/bk128_8b.log | tail -30
timeout -k 10 900 python -u -m llm_mcp_amd.bench.dgemm_bench --model llama-3-70b --only qkv,o --m 64,96,128 \
    --json gpurun_out/bk128_70b_rows.json > gpurun_out/bk128_70b.log 2>&1 || exit $?
grep -v "^ *!!" gpurun_out/bk128_70b.log | tail -12
