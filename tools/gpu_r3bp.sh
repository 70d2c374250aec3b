# TSDF refine pass grid: 2048 (2 waves/SIMD) vs larger grids (the kernel fits 6 waves/SIMD); identical grids checked
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python tools/bench_tsdf_variants.py "REFINE_WG=2048;REFINE_WG=4096;REFINE_WG=6144;REFINE_WG=8192;REFINE_WG=16384" > gpurun_out/tsdf_refine_wg_r3bp.txt 2>&1 || { cat gpurun_out/tsdf_refine_wg_r3bp.txt; exit 1; }
cat gpurun_out/tsdf_refine_wg_r3bp.txt
for wg in 2048 6144; do
  SFMHIP_TSDF_REFINE_WG=$wg REPS=3 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_wg$wg -o run -- python tools/run_tsdf_once.py > /dev/null 2>&1 || exit 1
  grep -h "refine\|cull_kernel\|tsdf_kernel" gpurun_out/kt_wg$wg/*kernel_stats.csv gpurun_out/kt_wg$wg/*/*kernel_stats.csv 2>/dev/null | cut -d, -f1-4 | sed "s/^/wg$wg /" | cut -c1-160
done
rm -rf gpurun_out/kt_wg*
