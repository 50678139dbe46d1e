# round 4, call 36: decode attention at 4 resident workgroups per CU (mode 8:
# VGPRs capped at 128, 4 spilled) against the default 3 (146 VGPRs), headline
# shape, engine page layout, fused rope, alternating
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/decode_attn_probe.py --layout engine --rope --modes 0,8,0,8,0,8 --iters 40 \
    > gpurun_out/attn_occ4.log 2>&1 || exit $?
grep "decode attn" gpurun_out/attn_occ4.log
