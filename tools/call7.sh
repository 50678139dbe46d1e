set -o pipefail
bash tools/rsgemm_lab.sh g5 "6144 4096 256 0 rs:42:2,rs:42:1,rs:42:4,rs:38:4" "4096 4096 256 2 rs:42:4,rs:42:2,rs:42:8,rs:38:8,dg:1:4" "4096 14336 256 2 rs:42:4,rs:42:2,rs:38:8" "28672 4096 256 3 rs:42:1,rs:38:1" "128256 4096 256 0 rs:38:1,rs:42:1" || exit $?
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k rsgemm -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/rs_tests3.log 2>&1
rc=$?; echo "rs tests exit $rc"; tail -3 gpurun_out/rs_tests3.log; exit $rc
