# Env-only sweep of the TSDF launch shape for N = 8 slabs (same library, bit-identical
# grids by construction): super-brick shape, XCD dealing, longest-first order, pipe.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in "" "SBX=4 SBY=4" "SBX=2 SBY=2" "SBX=1 SBY=1 SBZ=1" "IL=0" "ORDER=0" "PIPE=0" "SBX=8 SBY=8 SBZ=1" ""; do
  ENVS=""; for kv in $cfg; do ENVS="$ENVS SFMHIP_TSDF_$kv"; done
  env $ENVS timeout -k 10 200 python tools/bench_tsdf_slabs.py > gpurun_out/sweep.txt 2>&1 || { tail -5 gpurun_out/sweep.txt; exit 1; }
  echo "[$cfg] $(grep '^N=8 equal' gpurun_out/sweep.txt | cut -c1-50) $(grep '^N=8 equal' gpurun_out/sweep.txt | grep -o 'ms \[.*')"
done
