#!/bin/bash
# tools/stream_lab.cpp on the GPU box: page-size / order / pattern matrix.
# STREAM_SPECS: ';'-separated "PAGE_KB PATTERN INFLIGHT WGS_PER_CU" specs.
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/stream_lab.log
: > $out
IFS=';' read -ra specs <<< "${STREAM_SPECS:-16 0 1 3;16 1 1 3;8 1 1 3;4 1 1 3;2 1 1 3;16 0 2 2;16 1 2 2;8 1 2 2;8 2 1 3;16 2 1 3;8 1 1 4;8 1 1 2;8 0 1 3;8 1 1 3;16 0 1 3}"
for spec in "${specs[@]}"; do
  timeout -k 10 60 tools/labbin/stream_lab $spec >> $out 2>&1 || { echo "exit $? on $spec"; cat $out; exit 1; }
done
cat $out
