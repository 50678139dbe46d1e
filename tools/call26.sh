# round 4, call 26: K14 A-fragment read-ahead depth (pairs of ds_read_b128
# ahead of the MFMAs: 1 = shipped, 2, 3) on the served 128-row forms
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/rs_apf.log
for pf in 1 2 3 1 2 3; do
  for spec in "28672 4096 256 3 rs:38:1" "4096 14336 256 2 rs:38:8" "6144 4096 256 0 rs:42:2,rs:38:4"; do
    echo "== pf$pf $spec" >> gpurun_out/rs_apf.log
    timeout -k 10 120 tools/labbin/rsgemm_lab_pf$pf $spec >> gpurun_out/rs_apf.log 2>&1 || exit $?
  done
done
grep "==\|rs cfg" gpurun_out/rs_apf.log
