# round 4, call 38: K11 64 x 96 tiles with 128-deep K-steps (cfg 29 / 30) on the
# Llama-3-8B QKV at 160-256 rows -- lab against the 64-deep form, the tile
# numerics tests, then dgemm_bench against hipBLASLt
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/qkv_bk128.log
: > $L
for M in 256 192; do
  echo "== l8b qkv M=$M" >> $L
  timeout -k 10 120 tools/labbin/rsgemm_lab 6144 4096 $M 0 dg:0x3a:1,dg:0x3d:1,dg:0x3e:1,dg:0x1d:1,dg:0x3a:1,dg:0x3d:1,dg:0x3e:1 >> $L 2>&1 || exit $?
done
cat $L
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
    -k "stream_k or dgemm_configs" -p no:cacheprovider > gpurun_out/k11_tests.log 2>&1 || { tail -30 gpurun_out/k11_tests.log; exit 1; }
tail -2 gpurun_out/k11_tests.log
timeout -k 10 600 python -u -m llm_mcp_amd.bench.dgemm_bench --only qkv --m 160,192,224,256 \
    --json gpurun_out/qkv128_rows.json > gpurun_out/qkv128_bench.log 2>&1 || exit $?
grep -i "qkv" gpurun_out/qkv128_bench.log | tail -12
