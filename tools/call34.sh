# round 4, call 34: K11 256 x 96 tiles (cfg 29 / 30; S 4 = 256 workgroups) on
# the Llama-3-8B QKV at 160-256 rows -- lab, then dgemm_bench against
# hipBLASLt -- and the numerics tests of the new tiles
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/qkv_256x96.log
: > $L
for M in 256 224 192; do
  echo "== l8b qkv M=$M" >> $L
  timeout -k 10 120 tools/labbin/rsgemm_lab 6144 4096 $M 0 dg:0x3d:4,dg:0x3e:4,dg:0x3d:2,dg:0x3e:8,dg:0x7d:0,dg:0x7e:0,dg:0x3a:1 >> $L 2>&1 || exit $?
done
cat $L
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
    -k "stream_k or dgemm_configs" -p no:cacheprovider > gpurun_out/k11_tests.log 2>&1 || { tail -30 gpurun_out/k11_tests.log; exit 1; }
tail -2 gpurun_out/k11_tests.log
timeout -k 10 600 python -u -m llm_mcp_amd.bench.dgemm_bench --only qkv --m 160,192,224,256 \
    --json gpurun_out/qkv96_rows.json > gpurun_out/qkv96_bench.log 2>&1 || exit $?
grep -i "qkv" gpurun_out/qkv96_bench.log | tail -12
