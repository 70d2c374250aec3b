# Adam access-pattern microbenchmark (grid-stride block counts, contiguous chunks), two processes
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r3l}
for m in sep rev; do
  timeout -k 10 120 tools/adam_layout_micro $m >> gpurun_out/adam_micro_$TAG.txt 2>&1 || { tail -5 gpurun_out/adam_micro_$TAG.txt; exit 1; }
done
cat gpurun_out/adam_micro_$TAG.txt
