# BA solve PMC passes for variants 0 (AoS) and 1 (field-major)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out
for v in 0 1; do
  SFMHIP_BA_VARIANT=$v bash tools/pmc.sh ba_v$v ba_trf_kernel tools/bench_ba_solve.py > gpurun_out/pmc_ba_v$v.log 2>&1 || { tail -5 gpurun_out/pmc_ba_v$v.log; exit 1; }
  python tools/pmc_summary.py gpurun_out/pmc_ba_v$v > gpurun_out/pmc_ba_v$v.txt
  cat gpurun_out/pmc_ba_v$v.txt
  find gpurun_out/pmc_ba_v$v -name "*.csv" -size +2M -delete
done
