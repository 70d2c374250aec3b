#!/bin/bash
# PMC passes (one rocprofv3 --pmc run each, no trace domains) for one kernel of a command:
#   bash tools/pmc_kernel.sh TAG KERNEL_REGEX python tools/run_tsdf_once.py
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
TAG=$1; RX=$2; shift 2
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
i=0
for PASS in "GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_SALU" \
            "GRBM_GUI_ACTIVE TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum" \
            "GRBM_GUI_ACTIVE TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum" \
            "FETCH_SIZE TCC_HIT_sum" "WRITE_SIZE TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $PASS --kernel-include-regex "$RX" --output-format csv -d $OUT/p$i -o p -- "$@" > $OUT/log$i.txt 2>&1 || { echo "pass $i failed"; grep -v "^W20\|^I20" $OUT/log$i.txt | tail -5; exit 1; }
done
python tools/pmc_summary.py $OUT | tee $OUT/summary.txt
