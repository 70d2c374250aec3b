# usage: bash tools/pmc_tsdf_deep.sh <tag> : memory-pipeline counters for tsdf_kernel
# (one rocprofv3 counter pass each; no trace domains)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
TAG=$1
mkdir -p gpurun_out/pmc_$TAG
i=0
for PASS in "GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum" \
            "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum" \
            "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum" \
            "TCP_UTCL1_STALL_MULTI_MISS_sum TCP_UTCL1_SERIALIZATION_STALL_sum" \
            "TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum" \
            "TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum" \
            "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum" \
            "TD_TD_BUSY_sum TD_TC_STALL_sum" \
            "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCP_LATENCY_sum" \
            "SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES" \
            "FETCH_SIZE"; do
  i=$((i+1))
  NF=48 REPS=1 timeout -k 10 300 rocprofv3 --pmc $PASS --kernel-include-regex tsdf_kernel --output-format csv -d gpurun_out/pmc_$TAG/p$i -o p -- python tools/run_tsdf_once.py > gpurun_out/pmc_$TAG/log$i.txt 2>&1 || { echo "pass $i failed"; grep -v "^W20\|^I20" gpurun_out/pmc_$TAG/log$i.txt | tail -5; }
done
echo done
