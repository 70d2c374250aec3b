# Kernel trace of the C5 whole-grid call with the pre-pass pipeline (SFMHIP_TSDF_PREPIPE=$1):
# the block / cull / refine / fusion dispatches of the last call, start offsets and durations.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
G=${1:-4}
( export SFMHIP_TSDF_PREPIPE=$G
  timeout -k 10 120 rocprofv3 --kernel-trace --kernel-include-regex "tsdf|depth|coarse" --output-format csv -d gpurun_out/pp_$G -o run -- python tools/run_tsdf_once.py > /dev/null 2>&1 ) || exit 1
python tools/trace_summary.py gpurun_out/pp_$G/run_kernel_trace.csv "tsdf|depth|coarse" $((4 + 3 * G)) gpurun_out/prepipe_trace_$G.txt && rm -rf gpurun_out/pp_$G
