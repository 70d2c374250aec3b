# PMC passes (round 2 onwards; TAG names the run) (tools/pmc.sh: SQ, clock + L2, FETCH_SIZE, WRITE_SIZE, each its own run)
# for the C3 match launch, the C5 TSDF call and the V2+V4 render launch; summaries per kind.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r2}
REPS=1 bash tools/pmc.sh tsdf_$TAG "tsdf|blockmax|coarse" tools/run_tsdf_once.py || exit 1
REPS=2 bash tools/pmc.sh render_$TAG "render_kernel" tools/run_render_once.py || exit 1
REPS=1 bash tools/pmc.sh match_$TAG "match_kernel" tools/run_match_once.py || exit 1
for k in tsdf render match; do
  python tools/pmc_summary.py gpurun_out/pmc_${k}_$TAG > gpurun_out/pmc_${k}_$TAG.txt 2>&1 || true
done
find gpurun_out/pmc_*_$TAG -name "*.txt" -path "*log*" -delete
du -sh gpurun_out
