# round 4, call 27: K14 128-row pairs with the second tile's K order rotated
# RS_ROT K64 steps behind the first (its weight reads become L2 hits of lines
# the partner just fetched): 0 (shipped), 2, 4, 8
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/rs_rot.log
for r in 0 2 4 8 0 2 4 8; do
  for spec in "28672 4096 256 3 rs:38:1" "4096 14336 256 2 rs:38:8" "4096 4096 256 2 rs:38:8"; do
    echo "== rot$r $spec" >> gpurun_out/rs_rot.log
    timeout -k 10 120 tools/labbin/rsgemm_lab_rot$r $spec >> gpurun_out/rs_rot.log 2>&1 || exit $?
  done
done
grep "==\|rs cfg" gpurun_out/rs_rot.log
