# round 4, call 18: Llama-3-70B TP = 8 per-rank decode shapes on the hand-written
# kernels: the LM head shard padded to 16128 rows (K13-SK / K14) and QKV 1280 x 8192
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/pgemm_sk_probe.py --m 64,128,192,256 --splits 1,2,4,8,16 \
    --only tp8_lm_head,tp8_qkv --rounds 3 > gpurun_out/tp8_sk.log 2>&1 || exit $?
cat gpurun_out/tp8_sk.log
: > gpurun_out/tp8_rs.log
for M in 64 128 192 256; do
  echo "== M=$M" >> gpurun_out/tp8_rs.log
  timeout -k 10 150 tools/labbin/rsgemm_lab 16128 8192 $M 0 rs:38:1,rs:38:2,rs:38:4,rs:42:1,rs:42:2,rs:34:2 >> gpurun_out/tp8_rs.log 2>&1 || exit $?
done
cat gpurun_out/tp8_rs.log
