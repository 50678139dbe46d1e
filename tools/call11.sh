# round 4, call 11: full GPU suite + smoke after the lab-kernel move, a fresh
# headline timeline, and a traced A/B of QKV on K14 (64-row tiles, S 2)
set -o pipefail
bash tools/gpu_session.sh tests smoke prof_bench || exit $?
LMX_DGEMM_TABLE=tools/dgemm_qkvrs.json PROF_TAG=prof_qkvrs bash tools/gpu_session.sh prof_bench || exit $?
