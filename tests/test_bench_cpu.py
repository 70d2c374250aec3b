"""CPU checks of bench.py's CPU-baseline legs (BASELINE.md §2 methodology) and of
the oracle's z-slab mode they use for the all-threads TSDF run."""
import importlib

import numpy as np

import bench
from oracle import voxel as ov

syn = importlib.import_module("3d_reconstruction_amd.synthetic")


def test_tsdf_oracle_slab_mode_equals_whole_grid():
    depth, poses, K = syn.tsdf_scene(3, 40, 56, focal=50.0, seed=31)
    R = 24
    args = (depth.numpy(), poses.numpy(), K.numpy(), (-1, -1, -1), (1, 1, 1), np.float32(0.25))
    Tw, Ww = ov.tsdf_integrate(np.zeros((R, R, R), np.float32), np.zeros((R, R, R), np.float32), *args)
    for z0, z1 in ((0, 7), (7, 16), (16, 24)):
        Ts, Ws = ov.tsdf_integrate(np.zeros((z1 - z0, R, R), np.float32), np.zeros((z1 - z0, R, R), np.float32),
                                   *args, z0=z0, z1=z1, grid_depth=R)
        np.testing.assert_array_equal(Ts, Tw[z0:z1])
        np.testing.assert_array_equal(Ws, Ww[z0:z1])
    assert (Ww > 0).any()


def test_cpu_leg_reports_both_thread_counts():
    calls = []

    def run(k, nt):
        calls.append((k, nt))
        np.linalg.norm(np.ones(1000))
    leg = bench.cpu_leg(run, 8, 2, "units/s", "port", "toy", scale=10.0)
    assert leg["cores"] == bench.host_threads()
    assert leg["value"] > 0 and leg["value_1thread"] > 0
    # 1 warm-up + 3 timed runs on each leg
    assert calls == [(8, bench.host_threads())] * 4 + [(2, 1)] * 4
    assert "median of 3" in leg["timing"]


def test_gemm_form_baseline_matches_exact_oracle_away_from_ties():
    """The headline's CPU baseline (numpy f32 GEMM form) does the
    same matching as the exact oracle: identical matches0 on C3-like descriptors
    except rows whose ratio test sits within f32 rounding of the threshold."""
    from oracle import match as om
    x = syn.superpoint_like(2, 512, 256, seed=5).numpy()
    a, b = x[0], x[1]
    g = om.bf_match_gemm_f32(a, b, (3, 4))
    m, d1, d2 = om.bf_match_exact(a, b, (3, 4), return_dist=True)
    near = np.abs(16 * d1 - 9 * d2) <= 1e-4 * d2
    assert (m >= 0).sum() > 20
    np.testing.assert_array_equal(g[~near], m[~near])
    assert om.bf_match_gemm_f32(a[:0], b).shape == (0,)
    assert (om.bf_match_gemm_f32(a[:3], b[:1]) == -1).all()


def test_pool_map_keeps_order():
    assert bench.pool_map(lambda i: i * i, range(10), 4) == [i * i for i in range(10)]
    assert bench.pool_map(lambda i: i + 1, [3, 1], 1) == [4, 2]


def test_composite_line_arithmetic():
    res = {"config": {"pairs": 100}, "ms_per_step": 10.0}
    match_cpu = {"value": 10.0, "value_1thread": 1.0, "cores": 16}
    ba = {"ms_per_step": 1.0, "cpu_baseline": {"value": bench.BA_PAIRS * bench.BA_OBS / 2.0,
                                               "value_1thread": bench.BA_PAIRS * bench.BA_OBS / 4.0}}
    upd = bench.TSDF_R ** 3 * bench.TSDF_F / 1e6
    tsdf = {"ms_per_step": 9.0, "cpu_baseline": {"value": upd / 3.0, "value_1thread": upd / 6.0}}
    c = bench.composite_line(res, match_cpu, ba, tsdf)
    assert abs(c["gpu_s"] - 0.02) < 1e-12
    assert abs(c["cpu_s"] - (10.0 + 2.0 + 3.0)) < 1e-9
    assert abs(c["value"] - 15.0 / 0.02) < 1e-6
    # a part whose 1-thread run is faster counts at that rate
    ba["cpu_baseline"]["value_1thread"] = bench.BA_PAIRS * bench.BA_OBS / 1.0
    c = bench.composite_line(res, match_cpu, ba, tsdf)
    assert abs(c["cpu_s"] - (10.0 + 1.0 + 3.0)) < 1e-9
    assert abs(c["cpu_s_1thread"] - (100.0 + 1.0 + 6.0)) < 1e-9
    assert bench.composite_line(res, None, ba, tsdf) is None


def _run_bench(args, env_extra=None, timeout=120):
    import json
    import os
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT", "MASTER_ADDR")}
    env.update(env_extra or {})
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py")] + args, env=env, capture_output=True,
                       text=True, timeout=timeout)
    return p, [json.loads(ln) for ln in p.stdout.splitlines() if ln.startswith("{")]


def test_bench_gpus_flag_launches_ranks():
    """bench.py --gpus 2 (no torch.distributed launcher) starts two fresh rank
    processes; rank 0 prints one JSON line with n_gpus 2 and both ranks."""
    p, lines = _run_bench(["--gpus", "2", "--dist-backend", "gloo", "--dry-run"])
    assert p.returncode == 0, p.stderr
    assert len(lines) == 1
    ln = lines[0]
    assert ln["n_gpus"] == 2 and ln["dry_run"] is True
    assert [r["rank"] for r in ln["ranks"]] == [0, 1]
    assert [r["local_rank"] for r in ln["ranks"]] == [0, 1]
    assert len({r["pid"] for r in ln["ranks"]}) == 2


def test_bench_gpus_must_match_world():
    p, lines = _run_bench(["--gpus", "4", "--dry-run"], {"WORLD_SIZE": "2", "RANK": "0"})
    assert p.returncode != 0 and not lines
    assert "does not match" in p.stderr


def test_bench_single_rank_default():
    p, lines = _run_bench(["--dry-run"])
    assert p.returncode == 0, p.stderr
    assert lines[0]["n_gpus"] == 1


def test_bench_launcher_propagates_rank_failure():
    p, lines = _run_bench(["--gpus", "2", "--dist-backend", "no_such_backend", "--dry-run"])
    assert p.returncode != 0 and not lines
