# PMC traffic re-measured for the kernels changed late in round 5 (BA solve records, the exact-mode
# resolve), as tools/gpu_traffic_r5.sh does; then: python tools/traffic_r2.py r5b r5
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=r5b
REPS=1 bash tools/pmc.sh ba_$TAG "ba_trf_kernel" tools/run_ba_once.py || exit 1
REPS=1 bash tools/pmc.sh match_$TAG "match_kernel|resolve" tools/run_match_once.py || exit 1
for k in ba match; do
  python tools/pmc_summary.py gpurun_out/pmc_${k}_$TAG > gpurun_out/pmc_${k}_$TAG.txt 2>&1 || true
done
find gpurun_out/pmc_*_$TAG -name "*.txt" -path "*log*" -delete
du -sh gpurun_out
