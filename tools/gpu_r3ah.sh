# matcher MFMA ceilings with the two-candidate (pair) epilogue: random operands, d = 256 / 128
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 120 tools/mfma_peak 2000 1 > gpurun_out/mfma_peak_r3ah.txt 2>&1 || { tail -5 gpurun_out/mfma_peak_r3ah.txt; exit 1; }
cat gpurun_out/mfma_peak_r3ah.txt
