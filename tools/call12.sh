# round 4, call 12: the headline timeline and the traced QKV-on-K14 A/B again
# (call 11's trace databases overflowed the copy-back), then the kv-head-major
# cache emulation in the decode attention probe
set -o pipefail
bash tools/gpu_session.sh prof_bench || exit $?
LMX_DGEMM_TABLE=tools/dgemm_qkvrs.json PROF_TAG=prof_qkvrs bash tools/gpu_session.sh prof_bench || exit $?
bash tools/gpu_session.sh attn_layout || exit $?
