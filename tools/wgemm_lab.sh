#!/bin/bash
# K12 lab session on the GPU box: each shape under its own time limit, chained
# so the first failure ends the call.  Binary built on the CPU side:
#   hipcc --offload-arch=gfx950 -O3 -std=c++17 -DLMX_WGEMM_LAB \
#     -I llm_mcp_amd/csrc/kernels -I tools/lab_kernels tools/wgemm_lab.cpp -o tools/labbin/wgemm_lab
# Usage: bash tools/wgemm_lab.sh TAG "N K M EPI LIST" ["N K M EPI LIST" ...]
set -o pipefail
mkdir -p gpurun_out
tag=$1; shift
out=gpurun_out/wgemm_$tag.log
: > $out
for spec in "$@"; do
  echo "== $spec" | tee -a $out
  timeout -k 10 120 tools/labbin/wgemm_lab $spec >> $out 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "exit $rc" | tee -a $out; tail -5 $out; exit $rc; fi
done
cat $out
