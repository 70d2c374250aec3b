# f16 MFMA subnormal inputs: kept or flushed?
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 60 tools/mfma_f16_denorm 2>&1 | tee gpurun_out/mfma_f16_denorm_r3ao.txt
