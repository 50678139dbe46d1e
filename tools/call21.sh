# round 4, call 21: traced headline bench at the 24576-token prefill budget
set -o pipefail
bash tools/gpu_session.sh prof_bench || exit $?
