"""CPU: the host C++ of the C-ABI (track bookkeeping, tracks.hip) built with
AddressSanitizer and run against a randomized driver that also
checks it against a plain restatement (tools/asan_tracks.cpp)."""
import os
import subprocess

from conftest import ROOT


def test_tracks_host_code_under_asan():
    csrc = os.path.join(ROOT, "3d_reconstruction_amd", "csrc")
    subprocess.run(["make", "-C", csrc, "asan"], check=True, capture_output=True, timeout=600)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1")
    r = subprocess.run([os.path.join(ROOT, "build", "asan_tracks")], capture_output=True, text=True, timeout=300,
                       env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "asan tracks OK" in r.stdout
