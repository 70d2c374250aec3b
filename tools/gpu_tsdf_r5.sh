#!/bin/bash
# Round-5 TSDF iteration on the GPU box: TSDF parity tests (TESTS=0 skips), whole-grid +
# N-way slab timings (SLABS="" skips), kernel traces of one C5 call per knob config
# (CONFIGS="LATENCY=0,SHARE=40;SHARE=1000", SFMHIP_TSDF_ prefix added; "-" = defaults).
# Usage (from the repo root): bash tools/gpu_tsdf_r5.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=${1:-r5}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ "${TESTS:-1}" != "0" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_voxel.py -k "tsdf" -x -q --timeout 300 --timeout-method thread \
      -p no:cacheprovider > $OUT/pytest_tsdf.log 2>&1
  rc=$?; echo "pytest exit $rc" >> $OUT/pytest_tsdf.log; tail -3 $OUT/pytest_tsdf.log
  [ $rc -eq 0 ] || exit $rc
fi
if [ -n "${SLABS-8}" ]; then
  timeout -k 10 300 python -u tools/bench_tsdf_slabs.py ${SLABS-8} > $OUT/slabs.log 2>&1 || exit $?
  head -12 $OUT/slabs.log
fi
i=0
IFS=';' read -ra CF <<< "${CONFIGS:--}"
for c in "${CF[@]}"; do
  i=$((i+1))
  ENVS="REPS=4"
  if [ "$c" != "-" ]; then IFS=',' read -ra KV <<< "$c"; for kv in "${KV[@]}"; do case $kv in SFMHIP_*) ENVS="$ENVS $kv";; *) ENVS="$ENVS SFMHIP_TSDF_$kv";; esac; done; fi
  env $ENVS timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt$i -o run -- \
      python tools/run_tsdf_once.py > $OUT/kt$i.log 2>&1 || { echo "prof $c failed"; tail -5 $OUT/kt$i.log; exit 1; }
  find $OUT/kt$i -type f ! -name "*stats*" -delete
  python tools/trace_stats_line.py "$OUT/kt$i" "$c"
done
