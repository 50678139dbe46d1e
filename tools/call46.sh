# round 4, call 46: decode attention at the Llama-3-70B TP=1 shape (128 rows x
# 8 kv heads = 1024 segments: 1.33 rounds of the 768 resident workgroups at 3 per
# CU, one round at 4 per CU) -- persistent 3 / CU (mode 0), 4 / CU (mode 8), one
# workgroup per segment (mode 4), alternating
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/decode_attn_probe.py --batch 128 --hq 64 --ctx-lo 512 --ctx-hi 640 \
    --layout engine --rope --modes 0,8,4,0,8,4 --iters 40 > gpurun_out/attn_l70.log 2>&1 || exit $?
grep "decode attn" gpurun_out/attn_l70.log
