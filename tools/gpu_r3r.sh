# TSDF fusion per-wave timeline (tool-only probe build); slabs again with the resident waves
# capped by dynamic LDS (64 KB: 2 workgroups = 8 waves per CU; 40 KB: 4 workgroups = 16 waves)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/tsdf_wave_prof.py > gpurun_out/tsdf_wave_prof.txt 2>&1 || { tail -5 gpurun_out/tsdf_wave_prof.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/tsdf_wave_prof.txt
for L in 65536 40960; do
  SFMHIP_TSDF_PROF_LDS=$L timeout -k 10 300 python tools/tsdf_wave_prof.py > gpurun_out/tsdf_wave_prof_lds$L.txt 2>&1 || { tail -5 gpurun_out/tsdf_wave_prof_lds$L.txt; exit 1; }
  echo "LDS $L"; grep -v amdgpu.ids gpurun_out/tsdf_wave_prof_lds$L.txt
done
