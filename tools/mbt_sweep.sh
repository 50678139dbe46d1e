# headline bench at several prefill chunk budgets (tokens per engine step)
set -o pipefail
for m in "$@"; do
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --max-batched-tokens $m > gpurun_out/bench_mbt_$m.log 2>&1 || exit $?
done
