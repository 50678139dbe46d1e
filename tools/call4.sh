set -o pipefail
bash tools/rsgemm_lab.sh g2 "28672 4096 256 3 rs:34:2,rs:98:2,rs:2:2,rs:66:2,rs:34:4,rs:98:4,dg:6:1" "6144 4096 256 0 rs:34:4,rs:98:4,rs:34:8,rs:98:8,rs:34:2,dg:3:2" "28672 4096 192 3 rs:34:2,rs:98:2,dg:6:1" "6144 4096 160 0 rs:98:4,rs:98:8,dg:3:2" || exit $?
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k rsgemm -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/rs_tests.log 2>&1
rc=$?; echo "rs tests exit $rc"; tail -5 gpurun_out/rs_tests.log
exit $rc
