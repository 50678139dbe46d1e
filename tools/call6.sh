set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -k "rsgemm or llama3_8b_shapes" -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/rs_tests2.log 2>&1
rc=$?; echo "rs tests exit $rc"; tail -5 gpurun_out/rs_tests2.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash tools/rsgemm_lab.sh g4 "28672 4096 224 3 rs:38:1,dg:6:1" "28672 4096 192 3 rs:38:1,dg:6:1" "28672 4096 160 3 rs:38:1,dg:6:1" "4096 14336 192 2 rs:38:8,dg:0:8" "4096 14336 160 2 rs:38:8,dg:0:8" || exit $?
bash tools/ab_bench.sh rs1 "LMX_RS=1" rs0 "LMX_RS=0" 2
