#!/bin/bash
# PMC passes over the K13 probe (tools/pgemm_probe.py: K13 and hipBLASLt on the
# same shapes, one process per pass).  Usage: bash tools/pgemm_pmc.sh TAG PROBE_ARGS...
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=$1; shift
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INSTS_LDS GRBM_GUI_ACTIVE"
P3="TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum GRBM_GUI_ACTIVE"
n=0
for pass in "$P1" "$P2" "$P3"; do
  n=$((n+1))
  d=gpurun_out/pmc_${tag}_${n}
  rm -rf $d
  echo "[pmc] pass $n" >&2
  timeout -s KILL 120 rocprofv3 --pmc $pass --kernel-trace -d $d -o run --output-format csv \
      -- python3 tools/pgemm_probe.py "$@" > $d.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "rc $rc"; tail -5 $d.log; exit $rc; fi
done
echo done
