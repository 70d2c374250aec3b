# rocprofv3 kernel stats + one SQ counter pass of tools/bench_dlt.py
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
TAG=${TAG:-dlt}
mkdir -p gpurun_out/pmc_$TAG
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python tools/bench_dlt.py > gpurun_out/prof_$TAG.txt 2>&1 || exit 1
find gpurun_out/prof_$TAG -type f ! -name "*stats*" -delete
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_SALU --kernel-include-regex dlt --output-format csv -d gpurun_out/pmc_$TAG/p1 -o p -- python tools/bench_dlt.py > gpurun_out/pmc_$TAG/log1.txt 2>&1 || exit 1
python tools/pmc_summary.py gpurun_out/pmc_$TAG 2>/dev/null || true
grep -i dlt gpurun_out/prof_$TAG/run_kernel_stats.csv | cut -d, -f1,2,4 | sed 's/(double[^"]*//'
cat gpurun_out/prof_$TAG.txt | grep DLT
