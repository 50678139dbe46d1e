#!/bin/bash
# PMC passes over single K12 lab configurations (one process per config and
# pass).  Usage: bash tools/wgemm_pmc.sh TAG "N K M EPI CFG:S" ...
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=$1; shift
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM SQ_INST_LEVEL_VMEM SQ_INSTS_LDS GRBM_GUI_ACTIVE"
P2="TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_UTCL1_TRANSLATION_MISS_sum GRBM_GUI_ACTIVE"
P3="TCC_HIT_sum TCC_MISS_sum TCC_TAG_STALL_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE"
i=0
for spec in "$@"; do
  i=$((i+1))
  n=0
  for pass in "$P1" "$P2" "$P3"; do
    n=$((n+1))
    d=gpurun_out/pmc_${tag}_${i}_${n}
    rm -rf $d
    echo "[pmc] $spec pass $n" >&2
    timeout -s KILL 90 rocprofv3 --pmc $pass --kernel-trace -d $d -o run --output-format csv \
        -- tools/labbin/wgemm_lab $spec 5 > $d.log 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "rc $rc"; tail -5 $d.log; exit $rc; fi
  done
done
echo done
