# round 4, call 43: the K11 table after call42 -- GPU suite, smoke, the headline
# bench twice
set -o pipefail
bash tools/gpu_session.sh tests smoke || exit $?
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 > gpurun_out/t42_$r.log 2>&1 || exit $?
  tail -1 gpurun_out/t42_$r.log | cut -c1-300
done
