# round 4, call 19: the whole GPU suite + smoke after the residual epilogue,
# the padded TP LM-head shards and the TP8 LM-head K14 entry; then the TP8
# launcher rehearsal (70B layer shapes, padded vocab shards) and one headline run
set -o pipefail
bash tools/gpu_session.sh tests smoke tp8s bench1 || exit $?
