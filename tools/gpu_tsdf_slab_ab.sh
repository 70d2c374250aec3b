#!/bin/bash
# Kernel traces of one N=8 C5 slab (rank 3) per knob config: SCONFIGS="LATENCY=0;LATENCY=1" (SFMHIP_TSDF_ prefix)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp
TAG=${1:-r5}; OUT=gpurun_out/$TAG; mkdir -p $OUT
i=0
IFS=';' read -ra CF <<< "${SCONFIGS:--}"
for c in "${CF[@]}"; do
  i=$((i+1)); ENVS="X=1"
  if [ "$c" != "-" ]; then IFS=',' read -ra KV <<< "$c"; for kv in "${KV[@]}"; do ENVS="$ENVS SFMHIP_TSDF_$kv"; done; fi
  env $ENVS timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/sl$i -o run -- \
      python tools/run_tsdf_slab.py ${SLABN:-8} ${SLABR:-3} 5 > $OUT/sl$i.log 2>&1 || { echo "slab $c failed"; tail -5 $OUT/sl$i.log; exit 1; }
  find $OUT/sl$i -type f ! -name "*stats*" -delete
  python tools/trace_stats_line.py "$OUT/sl$i" "slab $c"
done
