# round 4, call 29: end-of-round validation -- the whole GPU suite, smoke, the
# headline bench at the defaults, and config 2 (/v1/embeddings over HTTP)
set -o pipefail
bash tools/gpu_session.sh tests smoke bench1 embed_http || exit $?
