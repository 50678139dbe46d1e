# A/B/C... of the headline bench, alternating, one box:
#   bash tools/ab_multi.sh ROUNDS NAME_A "ENV_A" NAME_B "ENV_B" ...
# ("-" for no extra environment); logs gpurun_out/ab_<name>_<round>.log
set -o pipefail
rounds=$1; shift
mkdir -p gpurun_out
args=("$@")
for r in $(seq 1 $rounds); do
  for ((i = 0; i < ${#args[@]}; i += 2)); do
    n=${args[i]}; e=${args[i+1]}
    [ "$e" = "-" ] && e=""
    env $e timeout -k 10 300 python bench.py --steps 3 --warmup 1 > gpurun_out/ab_${n}_$r.log 2>&1 || exit $?
    echo "[ab] $n round $r: $(grep -o '"value": [0-9.]*' gpurun_out/ab_${n}_$r.log) $(grep -o '"ttft_p50_ms": [0-9.]*' gpurun_out/ab_${n}_$r.log) $(grep -o '"decode_step_ms": \[[0-9.]*' gpurun_out/ab_${n}_$r.log)" >&2
  done
done
