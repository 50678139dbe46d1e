# round 4, call 25: K14 all-rows tiles (BM 256) with split-K -- where the time
# goes: partials only (epi 2, no combine) vs the in-kernel combine (epi 0 / 3),
# S 1 / 2 / 4, gate/up shape (cold weights)
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/bm256_split.log
for spec in "28672 4096 256 2 rs:34:1,rs:34:2,rs:34:4,rs:32:2" "28672 4096 256 0 rs:34:1,rs:34:2,rs:34:4" \
            "28672 4096 256 3 rs:34:1,rs:34:2,rs:38:1"; do
  echo "== $spec" >> gpurun_out/bm256_split.log
  timeout -k 10 150 tools/labbin/rsgemm_lab $spec >> gpurun_out/bm256_split.log 2>&1 || exit $?
done
cat gpurun_out/bm256_split.log
