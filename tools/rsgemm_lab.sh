#!/bin/bash
# K14 lab session on the GPU box (binary built on the CPU side, see
# tools/rsgemm_lab.cpp): each shape under its own time limit, chained so the
# first failure ends the call.
#   bash tools/rsgemm_lab.sh TAG "N K M EPI SPECS" ["N K M EPI SPECS" ...]
set -o pipefail
mkdir -p gpurun_out
tag=$1; shift
out=gpurun_out/rsgemm_$tag.log
: > $out
for spec in "$@"; do
  echo "== $spec" | tee -a $out
  timeout -k 10 150 tools/labbin/rsgemm_lab $spec >> $out 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "exit $rc" | tee -a $out; tail -5 $out; exit $rc; fi
done
cat $out
