set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -k "rope or cache or prefill or qwen3 or llama3_8b_shapes" -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/rope_tests.log 2>&1
rc=$?; echo "rope tests exit $rc"; tail -3 gpurun_out/rope_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 120 python -u tools/rope_probe.py > gpurun_out/rope_probe.log 2>&1; tail -5 gpurun_out/rope_probe.log
bash tools/gpu_session.sh config5b
