#!/bin/bash
# tools/stream_lab.cpp on the GPU box: page-size / order / in-flight matrix.
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/stream_lab.log
: > $out
for spec in "16 0 1 3" "16 1 1 3" "8 1 1 3" "4 1 1 3" "2 1 1 3" "16 0 2 2" "16 1 2 2" \
            "8 1 2 2" "8 2 1 3" "16 2 1 3" "8 1 1 4" "8 1 1 2" "8 0 1 3" "8 1 1 3" "16 0 1 3"; do
  timeout -k 10 60 tools/labbin/stream_lab $spec >> $out 2>&1 || { echo "exit $? on $spec"; cat $out; exit 1; }
done
cat $out
