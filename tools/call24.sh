# round 4, call 24: decode attention MODE 7 (half-page software pipeline: the
# next page's K loads issued after the QK MFMAs, its V after the PV MFMAs) vs
# the default MODE 0, headline shape, engine page layout, fused rope
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 150 python -u tools/decode_attn_probe.py --layout engine --rope --modes 0,7,0,7,0,7 \
    --iters 40 > gpurun_out/attn_mode7.log 2>&1 || exit $?
cat gpurun_out/attn_mode7.log
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "decode" -x -q --timeout 120 \
    --timeout-method thread -p no:cacheprovider > gpurun_out/attn_tests.log 2>&1; tail -2 gpurun_out/attn_tests.log
