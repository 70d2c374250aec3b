# Fused TSDF pre-pass A/B (round 6): the C5 call (tools/tsdf_ab_once.py) with the separate
# pre-pass launches (default) and the fused persistent pre-pass (SFMHIP_AB=3).  Every form must
# give the same grid digest.  (The task-granularity sweep of profiles/r6/tsdf_fused_prepass_r6.txt
# ran with a temporary SFMHIP_PRE=rows,bpw,lag override, since removed.)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
out=gpurun_out/ab_tsdf_prepass.txt
: > $out
for rep in 1 2; do
  for ab in 0 3; do
    SFMHIP_AB=$ab timeout -k 10 120 python tools/tsdf_ab_once.py > gpurun_out/abp.log 2>&1 || { tail -5 gpurun_out/abp.log; exit 1; }
    echo "SFMHIP_AB=$ab: $(tail -1 gpurun_out/abp.log)" | tee -a $out
  done
done
