# round 4, call 30: K11 64 x 96 tiles (256 workgroups, no split-K) on the
# Llama-3-8B QKV at 160-256 rows, vs the K11 config the table had (3, S 2)
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/dg96.log
for r in 1 2; do
  for M in 256 224 192 160; do
    echo "== M=$M" >> gpurun_out/dg96.log
    timeout -k 10 120 tools/labbin/rsgemm_lab 6144 4096 $M 0 dg:26:1,dg:27:1,dg:28:1,dg:58:1,dg:59:1,dg:60:1,dg:3:2,dg:35:2 >> gpurun_out/dg96.log 2>&1 || exit $?
  done
done
grep "==\|dg cfg\|stream" gpurun_out/dg96.log
