# PMC passes (SQ, clock + L2, FETCH_SIZE, WRITE_SIZE; separate runs) for the vq call and the render launch
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-r3be}
REPS=2 bash tools/pmc.sh vq_$TAG "vq_f16s_kernel|vq_exact_kernel" tools/run_vq_once.py || exit 1
REPS=2 bash tools/pmc.sh render_$TAG "render_kernel|render_key_kernel|render_scatter_kernel" tools/run_render_once.py || exit 1
for k in vq render; do
  python tools/pmc_summary.py gpurun_out/pmc_${k}_$TAG > gpurun_out/pmc_${k}_$TAG.txt 2>&1 || true
  cat gpurun_out/pmc_${k}_$TAG.txt
done
find gpurun_out/pmc_*_$TAG -name "*.txt" -path "*log*" -delete
