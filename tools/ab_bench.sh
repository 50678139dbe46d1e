# A/B of the headline bench under two environments, alternating, one box:
#   bash tools/ab_bench.sh NAME_A "ENV_A" NAME_B "ENV_B" [rounds]
set -o pipefail
na=$1; ea=$2; nb=$3; eb=$4; rounds=${5:-2}
for r in $(seq 1 $rounds); do
  env $ea timeout -k 10 300 python bench.py --steps 3 --warmup 1 > gpurun_out/ab_${na}_$r.log 2>&1 || exit $?
  env $eb timeout -k 10 300 python bench.py --steps 3 --warmup 1 > gpurun_out/ab_${nb}_$r.log 2>&1 || exit $?
done
