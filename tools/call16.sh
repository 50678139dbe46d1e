# round 4, call 16: K13 residual epilogue tests, then the front-door process
# counts (1+1 / 2+2 / 4+4 API processes + load generators) and the residual
# epilogue on / off in the headline bench, one box
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -k "pgemm or llama or qwen or prefill or engine" -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/res_tests.log 2>&1
rc=$?; tail -3 gpurun_out/res_tests.log; if [ $rc -ne 0 ]; then exit $rc; fi
for cfg in "1 1" "2 2" "4 4"; do
  set -- $cfg
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --api-procs $1 --loadgen-procs $2 \
      > gpurun_out/fd_${1}x${2}.log 2>&1 || exit $?
  tail -1 gpurun_out/fd_${1}x${2}.log | cut -c1-330
done
for r in 1 2; do
  LMX_RESIDUAL_EPILOGUE=0 timeout -k 10 300 python bench.py --steps 3 --warmup 1 > gpurun_out/res0_$r.log 2>&1 || exit $?
  tail -1 gpurun_out/res0_$r.log | cut -c1-330
  LMX_RESIDUAL_EPILOGUE=1 timeout -k 10 300 python bench.py --steps 3 --warmup 1 > gpurun_out/res1_$r.log 2>&1 || exit $?
  tail -1 gpurun_out/res1_$r.log | cut -c1-330
done
