# round 4, call 22: the eager-step trace of headline waves at the 24576 and
# 16384 prefill budgets (step sizes, decode rows, waiting sequences)
set -o pipefail
mkdir -p gpurun_out
for B in 24576 16384; do
  LMX_STEP_TRACE=1 timeout -k 10 300 python bench.py --steps 2 --warmup 1 --max-batched-tokens $B \
      > gpurun_out/steptrace_$B.log 2>&1 || exit $?
  grep "eager steps\|ttft" gpurun_out/steptrace_$B.log | cut -c1-1500
done
