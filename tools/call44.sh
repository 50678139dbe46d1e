# round 4, call 44: K11 ids 19-25 now 128-deep tiles (the 32-deep and 224-column
# tiles they held lost every shape) -- numerics, then dgemm_bench on the 8B and
# 70B decode shapes
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
    -k "stream_k or dgemm_configs" -p no:cacheprovider > gpurun_out/k11_tests.log 2>&1 || { tail -30 gpurun_out/k11_tests.log; exit 1; }
tail -2 gpurun_out/k11_tests.log
timeout -k 10 800 python -u -m llm_mcp_amd.bench.dgemm_bench --only qkv,o,down,gate_up --m 16,64,128,160,192,224,256 \
    --json gpurun_out/b44_8b_rows.json > gpurun_out/b44_8b.log 2>&1 || exit $?
grep -v "^ *!!" gpurun_out/b44_8b.log | tail -45
timeout -k 10 600 python -u -m llm_mcp_amd.bench.dgemm_bench --model llama-3-70b --only qkv,o,gate_up,down --m 64,128 \
    --json gpurun_out/b44_70b_rows.json > gpurun_out/b44_70b.log 2>&1 || exit $?
grep -v "^ *!!" gpurun_out/b44_70b.log | tail -14
