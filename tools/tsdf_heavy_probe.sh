# Heavy-kernel timing probes (tool-only build ab/lib_probe.so, make EXTRA=-DSFMHIP_PROBES):
# kernel traces of one N=8 centre slab with SFMHIP_TSDF_HEAVY_PROBE = 0 (as built), 1 (producers
# skip the frame evaluation), 2 (the consumer skips the application), 3 (both).  The product
# library is restored at the end.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
L=3d_reconstruction_amd/libsfmhip.so
cp ab/lib_probe.so $L
for pr in 0 1 2 3; do
  ( export SFMHIP_TSDF_HEAVY=200 SFMHIP_TSDF_HEAVY_MODE=2 SFMHIP_TSDF_HEAVY_PROBE=$pr
    timeout -k 10 120 rocprofv3 --kernel-trace --kernel-include-regex "tsdf_kernel|tsdf_heavy_kernel" --output-format csv -d gpurun_out/hp_$pr -o run -- python tools/tsdf_slab_trace.py > /dev/null 2>&1 ) || { cp ab/lib_prod.so $L; exit 1; }
  python tools/trace_summary.py gpurun_out/hp_$pr/run_kernel_trace.csv "tsdf_kernel|tsdf_heavy" 2 gpurun_out/hprobe_$pr.txt > /dev/null && rm -rf gpurun_out/hp_$pr
  echo "== probe $pr"; cat gpurun_out/hprobe_$pr.txt
done
cp ab/lib_prod.so $L
