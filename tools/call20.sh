# round 4, call 20: prefill step budget 16384 vs 24576 tokens (96 whole 256-row
# tiles: every prefill projection's tile count divides into full rounds over
# 256 CUs; the median request of a 256 x 513-token wave completes in step 3
# instead of step 5), alternating, one box
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for B in 24576 16384; do
    timeout -k 10 300 python bench.py --steps 3 --warmup 1 --max-batched-tokens $B \
        > gpurun_out/mbt_${B}_$r.log 2>&1 || exit $?
    tail -1 gpurun_out/mbt_${B}_$r.log | cut -c1-300
  done
done
