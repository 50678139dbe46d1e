# round 4, call 23: the engine's admission window (idle -> busy: wait for the
# burst) on vs off, with the eager-step trace, alternating
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for Q in 2 0; do
    LMX_STEP_TRACE=1 LMX_ADMIT_QUIET_MS=$Q timeout -k 10 300 python bench.py --steps 3 --warmup 1 \
        > gpurun_out/admit_${Q}_$r.log 2>&1 || exit $?
    grep "step 2 eager\|step 2:" gpurun_out/admit_${Q}_$r.log | cut -c1-400
    tail -1 gpurun_out/admit_${Q}_$r.log | cut -c1-300
  done
done
