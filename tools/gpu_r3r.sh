# TSDF fusion per-wave timeline (tool-only probe build)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/tsdf_wave_prof.py > gpurun_out/tsdf_wave_prof.txt 2>&1 || { tail -5 gpurun_out/tsdf_wave_prof.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/tsdf_wave_prof.txt
