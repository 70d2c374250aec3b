# PMC traffic of the round-6 tree (separate rocprofv3 --pmc passes per counter group, tools/pmc.sh):
# the C3 exact match launch writing the int16 graph, the int8-mode launch, one C5 TSDF call, one
# render launch, one BA solve, one vq call; then (here): python tools/traffic_r2.py r6 r6
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=r6
REPS=1 bash tools/pmc.sh match_$TAG "match_kernel|resolve" tools/run_match_once.py || exit 1
EXACT=0 REPS=1 bash tools/pmc.sh match_int8_$TAG "match_kernel" tools/run_match_once.py || exit 1
REPS=1 bash tools/pmc.sh tsdf_$TAG "tsdf_|depth_blockmax|coarse_table" tools/run_tsdf_once.py || exit 1
bash tools/pmc.sh render_$TAG "render_kernel" tools/run_render_once.py || exit 1
REPS=1 bash tools/pmc.sh ba_$TAG "ba_trf_kernel" tools/run_ba_once.py || exit 1
bash tools/pmc.sh vq_$TAG "vq_" tools/run_vq_once.py || exit 1
for k in match match_int8 tsdf render ba vq; do
  python tools/pmc_summary.py gpurun_out/pmc_${k}_$TAG > gpurun_out/pmc_${k}_$TAG.txt 2>&1 || true
done
find gpurun_out/pmc_*_$TAG -name "*.txt" -path "*log*" -delete
du -sh gpurun_out
