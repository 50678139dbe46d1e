set -o pipefail
bash tools/rsgemm_lab.sh g1 "28672 4096 256 3 rs:2:2,rs:34:2,rs:98:2,rs:66:2,rs:34:1,rs:98:1,rs:34:4,dg:6:1" "6144 4096 256 0 rs:34:8,rs:98:8,rs:34:4,rs:34:16,dg:3:2" "4096 4096 256 2 rs:34:16,rs:98:16,rs:34:8,dg:1:4" "4096 14336 256 2 rs:34:16,rs:98:16,rs:34:8,dg:0:8" "128256 4096 256 0 rs:34:1,rs:98:1" || exit $?
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k rsgemm -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/rs_tests.log 2>&1
rc=$?; echo "rs tests exit $rc"; tail -5 gpurun_out/rs_tests.log
# 0 = passed, 1 = assertion failures: the GPU is fine; anything else ends the call
if [ $rc -gt 1 ]; then exit $rc; fi
bash tools/gpu_session.sh tp_tests bench1 pmc_attn
