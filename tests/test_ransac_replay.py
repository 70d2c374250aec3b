"""CPU check of the load-balanced findEssentialMat schedule (ransac.hip, ess_* kernels) against
OpenCV's sequential RANSAC loop (ptsetreg.cpp RANSACPointSetRegistrator::run, restated in
oracle/ransac.py): chunks of hypotheses evaluated in rounds with bounded speculation, each chunk
reduced to its records (models whose count exceeds max(4, every earlier count of the chunk)),
models that cannot beat the best of earlier rounds dropped before they are counted exactly, and
the records replayed per pair.  The claim: the same best model, inlier count and iteration count
as the sequential loop, for any counts.  Pure Python on random count sequences (the device kernels
are checked bit for bit against the one-workgroup kernel in tests/test_gpu_verify.py)."""
import numpy as np
import pytest

from oracle.ransac import update_num_iters

M_PTS = 5          # model points (essential matrix)
CONF = 0.999


def sequential(models, n, max_iters):
    """ptsetreg.cpp's loop over precomputed per-hypothesis model counts."""
    niters, maxgood, best, it = max(max_iters, 1), 0, None, 0
    while it < niters:
        for m, good in enumerate(models[it]):
            if good > max(maxgood, M_PTS - 1):
                best, maxgood = (it, m), good
                niters = update_num_iters(CONF, (n - good) / n, M_PTS, niters)
        it += 1
    return best, maxgood, it


def balanced(models, n, max_iters, ch, caps, drop):
    """The ess_* schedule: gen / chunk / replay rounds (caps in hypotheses, last round: all)."""
    caps = tuple(-(-c // ch) * ch for c in caps)   # whole chunks, as the host rounds them
    st = dict(niters=max(max_iters, 1), maxgood=0, eval_upto=0, rc=0, cur_k=-1, kp=-1, best=None, done=False)
    recs = {}
    for rnd in range(len(caps) + 1):
        if st["done"]:
            break
        target = min(st["niters"], caps[rnd]) if rnd < len(caps) else st["niters"]
        c0, c1 = st["eval_upto"] // ch, -(-target // ch)
        bound = max(st["maxgood"], 4) if rnd > 0 else 4
        for c in range(c0, c1):   # chunk items: hypotheses below target only
            seq = []
            for h in range(ch):
                k = c * ch + h
                if k >= target:
                    break
                for m, good in enumerate(models[k]):
                    # early termination: some (drop 2) or all (drop 1) models at or below the bound
                    # are never counted exactly (the device drops those its partial count proves so)
                    gone = drop and good <= bound and (drop == 1 or (k + m) % 3 != 0)
                    seq.append((k, m, -1 if gone else good))
            pm, rl = 4, []
            for k, m, good in seq:
                if good > pm:
                    rl.append((k, m, good))
                    pm = good
            recs[c] = rl
        st["eval_upto"] = max(st["eval_upto"], c1 * ch)
        nit, done, c = st["niters"], False, st["rc"]
        while c < st["eval_upto"] // ch and not done:
            for k, m, good in recs[c]:
                if k != st["cur_k"]:
                    if k >= nit:
                        done = True
                        break
                    st["cur_k"] = k
                st["kp"] = k
                if good > max(st["maxgood"], 4):
                    st["maxgood"], st["best"] = good, (k, m)
                    nit = update_num_iters(CONF, (n - good) / n, M_PTS, nit)
            c += 1
        st["rc"], st["niters"] = c, nit
        if done or nit <= st["eval_upto"]:
            st["done"] = True
            st["last"] = max(nit, st["kp"] + 1) - 1
    assert st["done"], "the last round must complete every pair"
    return st["best"], st["maxgood"], st["last"] + 1


def random_models(rng, n, n_hyp, inlier):
    """Per-hypothesis model counts: up to 10 models, mostly poor, some near the inlier count."""
    out = []
    for _ in range(n_hyp):
        nm = int(rng.choice([0, 1, 2, 3, 4, 5, 6, 10], p=[.05, .1, .2, .25, .2, .1, .05, .05]))
        good = []
        for _ in range(nm):
            if rng.random() < 0.15:
                good.append(int(np.clip(rng.normal(inlier * n, 0.03 * n), 0, n)))
            else:
                good.append(int(rng.integers(0, max(2, int(0.1 * n)))))
        out.append(good)
    return out


@pytest.mark.parametrize("seed", range(40))
def test_records_replay_equals_sequential(seed):
    rng = np.random.default_rng(seed)
    n = int(rng.choice([6, 9, 40, 300, 2048, 5000]))
    inlier = float(rng.uniform(0.2, 1.0))
    max_iters = int(rng.choice([1, 7, 40, 77, 1000]))
    models = random_models(rng, n, max(max_iters, 1) + 64, inlier)
    ref = sequential(models, n, max_iters)
    for ch in (16, 32):
        for drop in (0, 1, 2):
            for caps in ((64, 128), (64, 256), (64, 1000), (16, 256), (32, 256), (48, 256), (96, 96), (40, 300)):
                got = balanced(models, n, max_iters, ch, caps=caps, drop=drop)
                assert got == ref, (seed, ch, drop, caps, got, ref)


def test_records_replay_adversarial_increasing_counts():
    """Strictly increasing counts inside every chunk (every model a record) and ties."""
    n = 4000
    for models in ([[5 + 10 * k + m for m in range(10)] for k in range(1100)],
                   [[7, 7, 7] for _ in range(1100)],
                   [[3, 4, 5, 5, 6] for _ in range(1100)]):
        ref = sequential(models, n, 1000)
        for ch in (16, 32):
            for drop in (0, 1, 2):
                for caps in ((64, 128), (64, 256)):
                    assert balanced(models, n, 1000, ch, caps=caps, drop=drop) == ref
