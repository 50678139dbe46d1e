set -o pipefail
bash tools/rsgemm_lab.sh l70 "10240 8192 128 0 rs:38:4,rs:38:8,rs:42:2,rs:42:4" "8192 8192 128 2 rs:38:4,rs:38:8,rs:42:4,dg:42:4" "8192 28672 128 2 rs:38:8,rs:38:4,rs:42:4,dg:38:8" "57344 8192 128 3 rs:38:1,rs:42:1,dg:50:1" "1280 8192 256 0 rs:38:8,rs:42:4,rs:42:8" "1280 8192 128 0 rs:38:16,rs:42:8" || exit $?
bash tools/gpu_session.sh rehearse8s
