"""Offline model (CPU, numpy): how many C3 rows would a block-scaled FP6 (e2m3) or FP4 (e2m1)
MFMA pass decide under the exact-float certificate that the int8 pass uses (csrc/match.hip
certify: |x_a - x_b| within E = |delta_a| + E_img[b] of the quantised distance)?  The
undecided rows would need the exact re-score, so the share decided bounds the use of the
2x-rate MX formats.  Prints the decided shares of int8 (today), FP6, FP4.
python tools/sim_mx_certify.py [n_img] [rows]"""
import importlib
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
syn = importlib.import_module("3d_reconstruction_amd.synthetic")


def grid_values(kind):
    if kind == "e2m3":   # FP6: bias 1, 3 mantissa bits, max 7.5
        sub = [m / 8 for m in range(8)]
        nor = [2.0 ** (e - 1) * (1 + m / 8) for e in (1, 2, 3) for m in range(8)]
    else:                # FP4 e2m1: {0, .5, 1, 1.5, 2, 3, 4, 6}
        sub = [0.0, 0.5]
        nor = [2.0 ** (e - 1) * (1 + m / 2) for e in (1, 2, 3) for m in range(2)]
    v = np.array(sorted(set(sub + nor)))
    return np.concatenate([-v[::-1], v])


def mx_quantise(x, kind, block=32):
    g = grid_values(kind)
    vmax = g.max()
    xb = x.reshape(x.shape[0], -1, block)
    amax = np.abs(xb).max(-1, keepdims=True)
    s = 2.0 ** np.ceil(np.log2(np.maximum(amax, 1e-30) / vmax))      # E8M0 block scale
    y = xb / s
    idx = np.clip(np.searchsorted(g, y), 1, len(g) - 1)
    lo, hi = g[idx - 1], g[idx]
    q = np.where(np.abs(y - lo) <= np.abs(hi - y), lo, hi)            # nearest (ties either way: a model)
    return (q * s).reshape(x.shape)


def certify(d1, d2, E, rn2=9.0, rd2=16.0):
    s1, s2 = np.sqrt(d1), np.sqrt(d2)
    a1, b1 = np.maximum(s1 - E, 0), s1 + E
    a2, b2 = np.maximum(s2 - E, 0), s2 + E
    rej = rd2 * a1 * a1 >= rn2 * b2 * b2
    acc = (b1 < a2) & (rd2 * b1 * b1 < rn2 * a2 * a2)
    return rej, acc


def main():
    n_img = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    rows = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    x = syn.superpoint_like(n_img, 4096, 256, seed=1).numpy().astype(np.float64)
    forms = {"int8 (q/127, today)": lambda v: np.clip(np.rint(127 * v), -127, 127) / 127,
             "FP6 e2m3, 32-block E8M0": lambda v: mx_quantise(v, "e2m3"),
             "FP4 e2m1, 32-block E8M0": lambda v: mx_quantise(v, "e2m1")}
    pairs = [(i, i + 1) for i in range(n_img - 1)] + [(0, n_img - 1)]
    for name, qf in forms.items():
        q = np.stack([qf(x[i]) for i in range(n_img)])
        E_row = np.linalg.norm(x - q, axis=-1)
        E_img = E_row.max(-1)
        dec = tot = acc_n = 0
        for a, b in pairs:
            qa, qb = q[a, :rows], q[b]
            D = (qa * qa).sum(1)[:, None] + (qb * qb).sum(1)[None, :] - 2 * qa @ qb.T
            D = np.maximum(D, 0)
            p = np.argpartition(D, 1, axis=1)[:, :2]
            d = np.sort(np.take_along_axis(D, p, 1), 1)
            rej, acc = certify(d[:, 0], d[:, 1], E_row[a, :rows] + E_img[b])
            dec += int((rej | acc).sum())
            acc_n += int(acc.sum())
            tot += rows
        print(f"{name:26s}: residual |delta| row median {np.median(E_row):.4f}, decided {dec / tot * 100:7.3f} % "
              f"(accepted {acc_n / tot * 100:.2f} %), undecided {(1 - dec / tot) * 100:.3f} %", flush=True)


if __name__ == "__main__":
    main()
