# round 4, call 17: traced headline bench with the K13 residual epilogue on
# (default) and off: prefill step time and the per-kernel split
set -o pipefail
bash tools/gpu_session.sh prof_bench || exit $?
LMX_RESIDUAL_EPILOGUE=0 PROF_TAG=prof_res0 bash tools/gpu_session.sh prof_bench || exit $?
