# Matcher: wave index made uniform (scalar LDS-DMA addresses): GPU match tests, then C3 / C2 timing of the
# new build vs ab/lib_prev.so (separate processes, alternating), identical graphs required
set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
mkdir -p gpurun_out
L=3d_reconstruction_amd/libsfmhip.so
cp $L ab/lib_new.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_match_exact.py -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_match_r3ay.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_match_r3ay.log; grep -E "^E  " gpurun_out/pytest_match_r3ay.log | head -3; [ $rc -eq 0 ] || exit 1
for v in new prev new prev; do
  cp ab/lib_$v.so $L
  timeout -k 10 300 python tools/bench_match_ab.py 2>&1 | grep -v amdgpu.ids | sed "s/^/$v /" || { cp ab/lib_new.so $L; exit 1; }
done
cp ab/lib_new.so $L
