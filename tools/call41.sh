# round 4, call 41: the K11 table after call40 (stream-K QKV / O / down at the
# ramp and tail buckets, 128-deep 64 x 128 O partials at 224-256 rows, 70B QKV
# / O) -- GPU suite, then the headline bench against the previous table
# (tools/dgemm_pre40.json), alternating, and the 70B bench
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_session.sh tests || exit $?
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 > gpurun_out/t40_new_$r.log 2>&1 || exit $?
  tail -1 gpurun_out/t40_new_$r.log | cut -c1-300
  LMX_DGEMM_TABLE=tools/dgemm_pre40.json timeout -k 10 300 python bench.py --steps 3 --warmup 1 \
      > gpurun_out/t40_old_$r.log 2>&1 || exit $?
  tail -1 gpurun_out/t40_old_$r.log | cut -c1-300
done
timeout -k 10 900 python bench.py --model llama-3-70b --concurrency 128 --max-tokens 128 --steps 2 --warmup 1 \
    > gpurun_out/l70_t40.log 2>&1 || exit $?
tail -1 gpurun_out/l70_t40.log | cut -c1-400
