# usage: bash tools/pmc.sh <tag> <kernel-regex> <script>
# One rocprofv3 run per PMC pass (counters only; no trace domains), restricted
# to the kernels matching the regex so the CSVs stay small.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
TAG=$1; RX=$2; SCRIPT=$3
mkdir -p gpurun_out/pmc_$TAG
i=0
for PASS in "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_LDS" \
            "GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $PASS --kernel-include-regex "$RX" --output-format csv -d gpurun_out/pmc_$TAG/p$i -o p -- python $SCRIPT > gpurun_out/pmc_$TAG/log$i.txt 2>&1 || { echo "pass $i failed"; grep -v "^W20\|^I20" gpurun_out/pmc_$TAG/log$i.txt | tail -5; exit 1; }
done
du -sh gpurun_out/pmc_$TAG
echo done
