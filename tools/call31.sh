# round 4, call 31: kernel trace of the Llama-3-70B TP = 1 bench (128 streams x
# 128 tokens): the graph-replayed decode step measures 46.7 ms where round 3's
# per-kernel table summed to ~36 ms at short contexts -- find where it goes
set -o pipefail
PROF_TAG=prof_l70 PROF_ARGS="--model llama-3-70b --concurrency 128 --max-tokens 128" \
    bash tools/gpu_session.sh prof_bench || exit $?
