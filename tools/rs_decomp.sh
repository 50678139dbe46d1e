#!/bin/bash
# K14 / K14W at the Llama-3-8B M = 256 MLP shapes (rsgemm_lab, cold weights),
# with the RS_LAB decomposition builds (1: no MFMA, 6: weights + activations
# L1-hot, 7: both): bash tools/rs_decomp.sh [variants]
mkdir -p gpurun_out
: > gpurun_out/rs_decomp.log
for v in ${1:-0 1 6 7}; do
  echo "== RS_LAB=$v" >> gpurun_out/rs_decomp.log
  timeout -k 10 100 tools/labbin/rsgemm_lab_v$v 28672 4096 256 3 ${GU_SPECS:-rs:38:1,rs:52:1,rs:56:1} \
      >> gpurun_out/rs_decomp.log 2>&1 || exit $?
  timeout -k 10 100 tools/labbin/rsgemm_lab_v$v 4096 14336 256 2 ${DN_SPECS:-rs:38:8,rs:52:8,rs:52:4,rs:56:4,rs:56:8} \
      >> gpurun_out/rs_decomp.log 2>&1 || exit $?
done
grep -v amdgpu.ids gpurun_out/rs_decomp.log
