# PMC traffic passes (tools/pmc.sh: SQ, clock + L2, FETCH_SIZE, WRITE_SIZE, each its own run) for the
# dominant kernels of every bench line that carries `traffic`: the C3 exact-float match launch, one C5
# TSDF call (every pre-pass + the fusion), the V2+V4 render launch, the BA solve, the vq call.
# Then: python tools/traffic_r2.py $TAG r5  ->  profiles/r5/traffic.json + pmc_<kind>.txt
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r5}
REPS=1 bash tools/pmc.sh tsdf_$TAG "tsdf|blockmax|coarse" tools/run_tsdf_once.py || exit 1
REPS=2 bash tools/pmc.sh render_$TAG "render_kernel" tools/run_render_once.py || exit 1
REPS=1 bash tools/pmc.sh ba_$TAG "ba_trf_kernel" tools/run_ba_once.py || exit 1
REPS=1 bash tools/pmc.sh vq_$TAG "vq_" tools/run_vq_once.py || exit 1
REPS=1 bash tools/pmc.sh match_$TAG "match_kernel|match_resolve" tools/run_match_once.py || exit 1
for k in tsdf render ba vq match; do
  python tools/pmc_summary.py gpurun_out/pmc_${k}_$TAG > gpurun_out/pmc_${k}_$TAG.txt 2>&1 || true
done
find gpurun_out/pmc_*_$TAG -name "*.txt" -path "*log*" -delete
du -sh gpurun_out
