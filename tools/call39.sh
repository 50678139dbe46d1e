# round 4, call 39: the headline bench with the Llama-3-8B QKV at 129-256 rows on
# K11 (64 x 96, 128-deep K-steps) against the library QKV table
# (tools/dgemm_libqkv.json), alternating, one box
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 > gpurun_out/qkv_k11_$r.log 2>&1 || exit $?
  tail -1 gpurun_out/qkv_k11_$r.log | cut -c1-300
  LMX_DGEMM_TABLE=tools/dgemm_libqkv.json timeout -k 10 300 python bench.py --steps 3 --warmup 1 \
      > gpurun_out/qkv_lib_$r.log 2>&1 || exit $?
  tail -1 gpurun_out/qkv_lib_$r.log | cut -c1-300
done
