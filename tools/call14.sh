# round 4, call 14: front-door process counts in the headline bench (A/B,
# alternating, one box): 1 API + 1 load generator (the default) vs 2 + 2 vs 4 + 4
set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for cfg in "1 1" "2 2" "4 4"; do
    set -- $cfg
    timeout -k 10 300 python bench.py --steps 3 --warmup 1 --api-procs $1 --loadgen-procs $2 \
        > gpurun_out/fd_${1}x${2}_$r.log 2>&1 || exit $?
    tail -1 gpurun_out/fd_${1}x${2}_$r.log | cut -c1-400
  done
done
