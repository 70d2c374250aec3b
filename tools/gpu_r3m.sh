# BA solve after the pass merges (X move in the Jacobian pass; |s2| with the subspace products):
# parity for every variant, timing, phase profile of the default
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r3m}
for v in 1 0 2 3; do
  SFMHIP_BA_VARIANT=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_ba.py tests/test_gpu_geometry.py tests/test_gpu_sfm.py -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_ba_v${v}_$TAG.log 2>&1
  rc=$?; echo "v$v: $(tail -1 gpurun_out/pytest_ba_v${v}_$TAG.log)"; grep -E "^E  " gpurun_out/pytest_ba_v${v}_$TAG.log | head -3
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
done
for v in 1 0 2 3 1 0 2 3; do
  SFMHIP_BA_VARIANT=$v timeout -k 10 120 python tools/bench_ba_solve.py >> gpurun_out/ba_variants_$TAG.txt 2>&1 || { tail -5 gpurun_out/ba_variants_$TAG.txt; exit 1; }
done
grep variant gpurun_out/ba_variants_$TAG.txt
timeout -k 10 120 python tools/ba_phase_prof.py 1 > gpurun_out/ba_phase_$TAG.txt 2>&1 || { tail -5 gpurun_out/ba_phase_$TAG.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/ba_phase_$TAG.txt
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_train_$TAG.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_train_$TAG.log; [ $rc -eq 0 ] || exit 1
for m in fresh after fresh; do
  timeout -k 10 300 python tools/adam_probe.py $m >> gpurun_out/adam_probe_$TAG.txt 2>&1 || { tail -5 gpurun_out/adam_probe_$TAG.txt; exit 1; }
done
grep -v amdgpu.ids gpurun_out/adam_probe_$TAG.txt
timeout -k 10 120 tools/adam_layout_micro sep > gpurun_out/adam_micro_$TAG.txt 2>&1 || exit 1
head -1 gpurun_out/adam_micro_$TAG.txt
bash tools/gpu_dlt_probe.sh
