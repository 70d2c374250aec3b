# Exact-mode resolve A/B on a GPU box: the match GPU tests with abl/lib_rx.so, then rocprofv3
# kernel stats of tools/run_match_once.py (C3, 2 reps) for abl/lib_base.so and abl/lib_rx.so
# (two library builds copied there beforehand; abl/ is scratch, not part of the tree).
set -o pipefail
mkdir -p gpurun_out
L=3d_reconstruction_amd/libsfmhip.so
cp abl/lib_rx.so $L
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_match.py tests/test_gpu_pipeline.py > gpurun_out/rx_t.log 2>&1; tail -2 gpurun_out/rx_t.log
export TMPDIR=/tmp
for v in base rx; do
  cp abl/lib_$v.so $L
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_rx_$v -o run -- python tools/run_match_once.py > gpurun_out/rx_$v.txt 2>&1 || exit 1
  grep -v amdgpu.ids gpurun_out/rx_$v.txt | grep matches
  python -c "
import csv,glob
f=glob.glob('gpurun_out/prof_rx_$v/**/*kernel_stats.csv',recursive=True)[0]
for r in csv.DictReader(open(f)):
    if any(w in r['Name'] for w in ('resolve', 'collect', 'match_kernel')): print('  ', r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')
"
  find gpurun_out/prof_rx_$v -type f ! -name "*kernel_stats*" -delete
done
