# round 4, call 47: decode attention at the Llama-3-70B TP=1 shape with the
# context split in two partitions (2048 half segments + the reduce kernel)
# against one partition per sequence
set -o pipefail
mkdir -p gpurun_out
for P in 1 2; do
  timeout -k 10 300 python -u tools/decode_attn_probe.py --batch 128 --hq 64 --ctx-lo 512 --ctx-hi 640 \
      --layout engine --rope --modes 0,0,0 --iters 40 --parts $P --part-tokens 384 > gpurun_out/attn_l70_p$P.log 2>&1 || exit $?
  grep "decode attn" gpurun_out/attn_l70_p$P.log
done
