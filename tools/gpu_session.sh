#!/bin/bash
# One gpurun session: each GPU step under its own time limit, chained so the
# first failure ends the call.  Usage (on the GPU box, from the repo root):
#   bash tools/gpu_session.sh STEP [STEP...]
# Steps: tests | bench1 | rehearse2 | prof
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "[gpu_session] $name: $*" >&2
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[gpu_session] $name exit $rc" >&2
  tail -n 3 "gpurun_out/$name.log" >&2
  return $rc
}
for step in "$@"; do
  case $step in
    tests)
      run gpu_tests 900 python -u -m pytest tests -m gpu -x -v --timeout 120 \
          --timeout-method thread -p no:cacheprovider || exit $? ;;
    bench1)
      run bench1 600 python bench.py --steps 3 --warmup 1 || exit $? ;;
    rehearse2)
      run rehearse2 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
          --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus 2 --steps 2 --warmup 1 \
          --concurrency 64 --rehearse-on-one-gpu || exit $? ;;
    dgemm_tests)
      run dgemm_tests 600 python -u -m pytest tests/test_kernels_gpu.py -k dgemm -x -q --timeout 120 \
          --timeout-method thread -p no:cacheprovider || exit $? ;;
    dgemm_bench)
      run dgemm_bench 900 python -u -m llm_mcp_amd.bench.dgemm_bench --json gpurun_out/dgemm_rows.json \
          --write || exit $?
      cp llm_mcp_amd/config/dgemm_gfx950.json gpurun_out/ ;;
    smoke)
      run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $? ;;
    *)
      echo "unknown step $step" >&2; exit 2 ;;
  esac
done
