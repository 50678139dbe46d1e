# round 4, call 32: split-K partial costs on the QKV shapes -- K11 with the
# in-kernel last-arriver reduction (epi 0) vs partials only (epi 2, the sum
# left to another kernel): Llama-3-70B QKV at M = 128, Llama-3-8B QKV at M = 256
set -o pipefail
mkdir -p gpurun_out
L=gpurun_out/qkv_split.log
: > $L
for e in 0 2; do
  echo "== l70 qkv M=128 epi=$e" >> $L
  timeout -k 10 120 tools/labbin/rsgemm_lab 10240 8192 128 $e dg:38:2,dg:38:4,dg:38:8,dg:38:16,dg:42:4,dg:42:8,dg:42:16,dg:33:8,dg:54:8,dg:50:8,dg:40:8,dg:40:16 >> $L 2>&1 || exit $?
  echo "== l8b qkv M=256 epi=$e" >> $L
  timeout -k 10 120 tools/labbin/rsgemm_lab 6144 4096 256 $e dg:38:2,dg:38:4,dg:38:8,dg:42:4,dg:42:8,dg:44:4,dg:44:8,dg:35:2,dg:35:4,dg:40:4,dg:40:8 >> $L 2>&1 || exit $?
done
cat $L
