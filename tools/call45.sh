# round 4, call 45: the K11 table after call44 -- GPU suite, then the headline
# bench against the call43 table (tools/dgemm_pre44.json), alternating
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_session.sh tests || exit $?
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 > gpurun_out/t44_new_$r.log 2>&1 || exit $?
  tail -1 gpurun_out/t44_new_$r.log | cut -c1-200
  LMX_DGEMM_TABLE=tools/dgemm_pre44.json timeout -k 10 300 python bench.py --steps 3 --warmup 1 \
      > gpurun_out/t44_old_$r.log 2>&1 || exit $?
  tail -1 gpurun_out/t44_old_$r.log | cut -c1-200
done
