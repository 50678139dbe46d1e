# round 4, call 48: dgemm_bench on the Llama-3-8B LM head (128256 x 4096) at
# 192 / 256 rows -- K11 split-K, 128-deep and stream-K forms against hipBLASLt
# (K13-SK serves it now: 260 us per call in the headline trace)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m llm_mcp_amd.bench.dgemm_bench --only lm_head --m ${LM_M:-192,256} \
    --json gpurun_out/b48_rows.json > gpurun_out/b48.log 2>&1 || exit $?
grep -v "^ *!!" gpurun_out/b48.log | tail -4
python - <<'PY'
import json
rows = [r for r in json.load(open("gpurun_out/b48_rows.json")) if "us" in r]
for M in sorted({r["M"] for r in rows}):
    rs = sorted((r["us"], r["cfg"], r["splits"]) for r in rows if r["M"] == M)[:6]
    print(M, rs)
PY
