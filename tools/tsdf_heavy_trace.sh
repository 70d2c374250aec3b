# Kernel traces of one N=8 centre slab (tools/tsdf_slab_trace.py) under several heavy-path
# settings; each summary (fusion kernels' start / duration) goes to gpurun_out/htrace_<name>.txt
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
run() {   # name, env assignments...
  name=$1; shift
  ( export "$@"; timeout -k 10 120 rocprofv3 --kernel-trace --kernel-include-regex "tsdf_kernel|tsdf_heavy_kernel" --output-format csv -d gpurun_out/ht_$name -o run -- python tools/tsdf_slab_trace.py > /dev/null 2>&1 ) || return 1
  python tools/trace_summary.py gpurun_out/ht_$name/run_kernel_trace.csv "tsdf_kernel|tsdf_heavy" 4 gpurun_out/htrace_$name.txt > /dev/null && rm -rf gpurun_out/ht_$name
  echo "== $name"; cat gpurun_out/htrace_$name.txt
}
run off SFMHIP_TSDF_HEAVY=0 &&
run h96k1 SFMHIP_TSDF_HEAVY=96 SFMHIP_TSDF_HEAVY_MODE=2 SFMHIP_TSDF_HEAVY_K=1 &&
run h96k4 SFMHIP_TSDF_HEAVY=96 SFMHIP_TSDF_HEAVY_MODE=2 SFMHIP_TSDF_HEAVY_K=4 &&
run h96k8 SFMHIP_TSDF_HEAVY=96 SFMHIP_TSDF_HEAVY_MODE=2 SFMHIP_TSDF_HEAVY_K=8 &&
run h200k4 SFMHIP_TSDF_HEAVY=200 SFMHIP_TSDF_HEAVY_MODE=2 SFMHIP_TSDF_HEAVY_K=4 &&
run h200k4wg256 SFMHIP_TSDF_HEAVY=200 SFMHIP_TSDF_HEAVY_MODE=2 SFMHIP_TSDF_HEAVY_K=4 SFMHIP_TSDF_HEAVY_WG=256
