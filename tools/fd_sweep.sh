set -o pipefail
for cfg in "1 1" "2 1" "1 4" "2 4" "4 4"; do
  set -- $cfg
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --api-procs $1 --loadgen-procs $2 > gpurun_out/fd_a$1_l$2.log 2>&1 || exit $?
done
