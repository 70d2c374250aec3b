set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
bash tools/pmc_tsdf_deep.sh deep_v2 > gpurun_out/deep_v2.log 2>&1 || { tail -5 gpurun_out/deep_v2.log; exit 1; }
python tools/pmc_summary.py gpurun_out/pmc_deep_v2 > gpurun_out/deep_v2_summary.txt && cat gpurun_out/deep_v2_summary.txt
sed -i 's/^for FR in 1 4; do/for FR in 1 4; do export SFMHIP_TSDF_CHUNK=512;/' tools/gpu_tsdf_prof.sh
bash tools/gpu_tsdf_prof.sh
