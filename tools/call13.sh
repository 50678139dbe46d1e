# round 4, call 13: decode GEMMs with the weights warm in the Infinity Cache
# (LAB_COPIES=1: the same copy every call) vs cold (default rotation) -- what a
# prefetch of the next projection's weights during the latency-bound slab norms
# could buy
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/mall_lab.log
for c in 0 1 2; do
  for spec in "6144 4096 256 0 rs:42:2,dg:3:2" "4096 4096 256 2 rs:38:8,dg:1:4" \
              "4096 14336 256 2 rs:38:8" "28672 4096 256 3 rs:38:1"; do
    echo "== copies=$c $spec" >> gpurun_out/mall_lab.log
    if [ $c -eq 0 ]; then
      timeout -k 10 120 tools/labbin/rsgemm_lab $spec >> gpurun_out/mall_lab.log 2>&1 || exit $?
    else
      LAB_COPIES=$c timeout -k 10 120 tools/labbin/rsgemm_lab $spec >> gpurun_out/mall_lab.log 2>&1 || exit $?
    fi
  done
done
cat gpurun_out/mall_lab.log
# Llama-3-70B (TP=1) at 128 rows: K14 straight from the row-major weights
# (cfg bit 6) -- one 128-row tile per column tile, so no L2 sharing to lose --
# vs packed and K11
: > gpurun_out/l70_rowmajor.log
for spec in "57344 8192 128 3 rs:102:1,rs:38:1,dg:50:1" "8192 28672 128 2 rs:102:8,rs:38:8,dg:38:8" \
            "10240 8192 128 0 rs:102:4,rs:38:4" "8192 8192 128 2 rs:102:8,rs:38:8,dg:42:4"; do
  echo "== $spec" >> gpurun_out/l70_rowmajor.log
  timeout -k 10 150 tools/labbin/rsgemm_lab $spec >> gpurun_out/l70_rowmajor.log 2>&1 || exit $?
done
cat gpurun_out/l70_rowmajor.log
