mkdir -p gpurun_out
: > gpurun_out/rs_decomp.log
for v in 0 1 2 4 6 7; do
  echo "== RS_LAB=$v" >> gpurun_out/rs_decomp.log
  timeout -k 10 100 tools/labbin/rsgemm_lab_v$v 28672 4096 256 3 rs:38:1 >> gpurun_out/rs_decomp.log 2>&1 || exit $?
  timeout -k 10 100 tools/labbin/rsgemm_lab_v$v 4096 14336 256 2 rs:38:8 >> gpurun_out/rs_decomp.log 2>&1 || exit $?
done
