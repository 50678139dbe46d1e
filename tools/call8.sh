set -o pipefail
bash tools/gpu_session.sh rehearse4s tp8s
