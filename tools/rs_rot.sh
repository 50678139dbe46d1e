#!/bin/bash
# K14 K-order rotation (cfg bit 7) and activation row padding (LAB_LDA_PAD) at
# the Llama-3-8B M = 256 MLP shapes (rsgemm_lab, cold weights)
mkdir -p gpurun_out
out=gpurun_out/rs_rot.log
: > $out
for pad in 0 64; do
  echo "== LAB_LDA_PAD=$pad" >> $out
  LAB_LDA_PAD=$pad timeout -k 10 100 tools/labbin/rsgemm_lab_v0 28672 4096 256 3 \
      rs:38:1,rs:166:1,rs:52:1,rs:38:1,rs:166:1 >> $out 2>&1 || exit $?
  LAB_LDA_PAD=$pad timeout -k 10 100 tools/labbin/rsgemm_lab_v0 4096 14336 256 2 \
      rs:38:8,rs:166:8,rs:38:8,rs:166:8 >> $out 2>&1 || exit $?
done
grep -v amdgpu.ids $out
