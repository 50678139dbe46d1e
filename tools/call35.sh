# round 4, call 35: (1) prefill step budget 24576 vs 33792 / 34816 tokens (132 /
# 136 whole 256-row tiles: two steps hold the median request #129 of a
# 256 x 513-token wave, against three at 24576), alternating, one box;
# (2) Llama-3-70B TP = 1 with the stream-K QKV and the corrected decode-step time
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for B in 24576 33792 34816; do
    LMX_STEP_TRACE=1 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --max-batched-tokens $B \
        > gpurun_out/mbt2_${B}_$r.log 2>&1 || exit $?
    tail -1 gpurun_out/mbt2_${B}_$r.log | cut -c1-330
  done
done
timeout -k 10 900 python bench.py --model llama-3-70b --concurrency 128 --max-tokens 128 --steps 2 --warmup 1 \
    > gpurun_out/l70_sk.log 2>&1 || exit $?
tail -1 gpurun_out/l70_sk.log | cut -c1-400
