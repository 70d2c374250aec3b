# usage: bash tools/pmc_tsdf_prepass.sh <tag> : issue / wait counters of the TSDF cull and refine
# pre-passes on the full C5 call (one rocprofv3 counter pass each; no trace domains)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
TAG=$1
mkdir -p gpurun_out/pmc_$TAG
i=0
for PASS in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAVES" \
            "GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum" \
            "FETCH_SIZE"; do
  i=$((i+1))
  REPS=1 timeout -k 10 -s KILL 120 rocprofv3 --pmc $PASS --kernel-include-regex "tsdf_cull_kernel|tsdf_refine_kernel" --output-format csv -d gpurun_out/pmc_$TAG/p$i -o p -- python tools/run_tsdf_once.py > gpurun_out/pmc_$TAG/log$i.txt 2>&1 || { echo "pass $i failed"; grep -v "^W20\|^I20" gpurun_out/pmc_$TAG/log$i.txt | tail -5; exit 1; }
done
python tools/pmc_summary.py gpurun_out/pmc_$TAG > gpurun_out/pmc_$TAG/summary.txt 2>&1 || true
find gpurun_out/pmc_$TAG -name "*counter_collection.csv" | head -3
cat gpurun_out/pmc_$TAG/summary.txt | head -60
