"""M1/M2: brute-force L2 matching + ratio test, and scipy-compatible ``vq``.

Drop-in surfaces:

* :class:`Matcher` — callable with the LightGlue contract used at
  ``matching.py:20,122-128`` (input dict of ``image0``/``image1`` feature dicts,
  output dict ``lightglue/lightglue.py:442-450``: ``matches0``, ``matches1``,
  ``matching_scores0/1``, ``matches`` (list of (S,2) int64), ``scores``,
  ``stop``), so ``rbd`` (``lightglue/utils.py:64-67``) and the consumer at
  ``matching.py:123-128`` run unchanged.
* :class:`DescriptorBank` — all images' descriptors resident in HBM as int8 and
  matched pair-batched: ``bank.match(pairs)`` -> ``matches0`` (P, m_pad) int32.
* :func:`vq` — ``scipy.cluster.vq.vq`` signature (``matching.py:27``).

Semantics of the BF matcher are build-defined (the reference has no BF
matcher) and pinned by ``oracle/match.py``: best index = lowest on ties, Lowe
ratio test ``den^2 * d1 < num^2 * d2`` evaluated exactly, optional mutual
check with LightGlue's ``filter_matches`` semantics
(``lightglue/lightglue.py:235-254``).  Two distance definitions:

* exact float (the default for float descriptors -- ``MODE_FLOAT``, the DISK /
  SuperPoint descriptors of matching.py:111-122 -- in :class:`Matcher`,
  :meth:`DescriptorBank.from_float`, :func:`bf_match` and so in
  ``pipeline.matching_stage`` / ``dist.match_all_pairs_sharded``): squared L2 of
  the f32 descriptors summed in f64 in k order.  The int8 MFMA pass runs with a
  proven bound on the quantisation residual and certifies most rows; the rest
  are re-scored exactly (DESIGN.md "exact float mode");
* quantised (``exact=False``; and ``MODE_SIFT``, whose integer 0..255 values
  quantise exactly): exact integer squared L2 of the int8 quantisation (SIFT:
  q = x - 128; float: q = rint(127 x)).
"""
from __future__ import annotations

import os
from fractions import Fraction

import numpy as np
import torch

from ._abi import call, dev, ptr, require_gpu, stream_ptr

MODE_SIFT = 0    # integer-valued 0..255 descriptors (SIFT): q = x - 128
MODE_FLOAT = 1   # float descriptors (SuperPoint / DISK, L2-normalised): q = rint(127 x)
_JB = 128        # m_pad granularity required by the kernel
_SHIFTS = (48, 64)   # operand shifts of the matcher, in order of preference (sfmhip_desc_prepare_shifted)


def _ratio(ratio) -> tuple[int, int]:
    if isinstance(ratio, tuple):
        num, den = ratio
    else:
        fr = Fraction(str(ratio)).limit_denominator(65535)
        num, den = fr.numerator, fr.denominator
    if not (0 < num and 0 < den <= 65535 and num <= 65535):
        raise ValueError(f"ratio must be a positive fraction, got {ratio!r}")
    return int(num), int(den)


class DescriptorBank:
    """Quantised descriptors of ``n_img`` images resident on the GPU.

    Layout in HBM: int8 ``[n_img][m_pad][d]`` (rows past ``n_kpts[img]`` zero),
    int32 row norms ``[n_img][m_pad]`` and int32 packed candidate keys
    ``[n_img][m_pad]`` (DESIGN.md "packed key").
    """

    def __init__(self, q: torch.Tensor, n_kpts: torch.Tensor, x: torch.Tensor | None = None,
                 mode: int = MODE_FLOAT):
        require_gpu()
        if q.dtype != torch.int8 or q.dim() != 3:
            raise ValueError("q must be an int8 tensor [n_img, m_pad, d]")
        n_img, m_pad, d = q.shape
        if m_pad % _JB:
            raise ValueError(f"m_pad must be a multiple of {_JB}")
        if d not in (64, 128, 256):
            raise ValueError(f"descriptor dim {d} not in (64, 128, 256)")
        self.q = q.contiguous()
        self.n_kpts = n_kpts.to(device=q.device, dtype=torch.int32).contiguous()
        self.n_img, self.m_pad, self.d = int(n_img), int(m_pad), int(d)
        self.norms = torch.empty((n_img, m_pad), dtype=torch.int32, device=q.device)
        self.keys = torch.empty((n_img, m_pad), dtype=torch.int32, device=q.device)
        # Matcher operands: q itself, or (default, when every value fits) q + c with
        # adjusted norms/keys -- identical results; non-negative operands in a narrow
        # bit band run the int8 array at a higher clock.  c = 48 puts
        # zero-mean descriptors in [32, 64) (bit 5 set, bit 6 clear: only the low bits
        # toggle; measured 105.3 vs 109.9 ms for c = 64 and 115 ms unshifted on C3);
        # c = 64 when the values reach below -48.  SFMHIP_MATCH_SHIFT: 0 off, 1 auto,
        # >= 2 that shift (A/B runs).
        self.qm = self.q
        env = int(os.environ.get("SFMHIP_MATCH_SHIFT", "1"))
        qmin, qmax = (int(self.q.min()), int(self.q.max())) if self.q.numel() else (0, 0)
        cands = () if env == 0 else (_SHIFTS if env == 1 else (env,))
        shift = next((c for c in cands if qmin >= -c and qmax <= 127 - c), 0)
        self.shift = shift
        if shift:
            self.qm = torch.empty_like(self.q)
            call("sfmhip_desc_prepare_shifted", ptr(self.q), self.n_img, self.m_pad, self.d, ptr(self.n_kpts),
                 shift, ptr(self.qm), ptr(self.norms), ptr(self.keys), stream_ptr())
        else:
            call("sfmhip_desc_prepare", ptr(self.q), self.n_img, self.m_pad, self.d, ptr(self.n_kpts),
                 ptr(self.norms), ptr(self.keys), stream_ptr())
        # exact float mode: the f32 descriptors and the per-row residual bounds
        self.mode = int(mode)
        self.x = None
        self.last_resolved = None
        if x is not None:
            if x.dtype != torch.float32 or tuple(x.shape) != tuple(self.q.shape):
                raise ValueError("x must be float32 of the bank's shape [n_img, m_pad, d]")
            self.x = x.contiguous()
            self.erow = torch.empty((self.n_img, self.m_pad), dtype=torch.float64, device=q.device)
            self.eimg = torch.empty(self.n_img, dtype=torch.float64, device=q.device)
            call("sfmhip_desc_residual", ptr(self.x), ptr(self.q), self.n_img, self.m_pad, self.d, ptr(self.n_kpts),
                 self.mode, ptr(self.erow), ptr(self.eimg), stream_ptr())
            self._nres = torch.zeros(1, dtype=torch.int32, device=q.device)

    @property
    def device(self) -> torch.device:
        return self.q.device

    @property
    def exact(self) -> bool:
        """True when the bank holds the float descriptors (exact float mode available)."""
        return self.x is not None

    # -- construction -------------------------------------------------------
    @classmethod
    def from_float(cls, desc, n_kpts=None, mode: int = MODE_FLOAT, exact: bool | None = None) -> "DescriptorBank":
        """``desc``: f32 [n_img, M, d] array/tensor or a list of (K_i, d) arrays
        (the ``all_descriptors.npy`` object-array format, ``feature_extraction.py:50``).
        ``exact``: keep the f32 descriptors for the exact float mode (finite
        values required; padding rows are zeroed); default: True for
        ``MODE_FLOAT``, False for ``MODE_SIFT`` (integer values: the int8
        distances are the exact ones)."""
        exact = (mode == MODE_FLOAT) if exact is None else bool(exact)
        d0 = require_gpu()
        if isinstance(desc, (list, tuple)) or (isinstance(desc, np.ndarray) and desc.dtype == object):
            rows = [dev(r, torch.float32) for r in desc]
            n_img = len(rows)
            d = rows[0].shape[1]
            m = max(r.shape[0] for r in rows)
            m_pad = max(_JB, -(-m // _JB) * _JB)
            x = torch.zeros((n_img, m_pad, d), dtype=torch.float32, device=d0)
            for i, r in enumerate(rows):
                x[i, :r.shape[0]] = r
            nk = torch.tensor([r.shape[0] for r in rows], dtype=torch.int32)
        else:
            x = dev(desc, torch.float32)
            n_img, m, d = x.shape
            m_pad = max(_JB, -(-m // _JB) * _JB)
            if m_pad != m:
                x = torch.nn.functional.pad(x, (0, 0, 0, m_pad - m))
            nk = torch.full((n_img,), m, dtype=torch.int32) if n_kpts is None else torch.as_tensor(n_kpts)
        nk = nk.to(device=d0, dtype=torch.int32).contiguous()
        x = x.contiguous()
        q = torch.empty((n_img, m_pad, d), dtype=torch.int8, device=d0)
        call("sfmhip_desc_quantize", ptr(x), n_img, m_pad, d, ptr(nk), int(mode), ptr(q), stream_ptr())
        if not exact:
            return cls(q, nk)
        valid = torch.arange(m_pad, device=d0)[None, :] < nk[:, None].long()
        x = torch.where(valid[:, :, None], x, torch.zeros((), dtype=x.dtype, device=d0)).contiguous()
        if not bool(torch.isfinite(x).all()):
            raise ValueError("exact matching needs finite descriptors")
        return cls(q, nk, x=x, mode=mode)

    # -- matching ------------------------------------------------------------
    def match(self, pairs, ratio=0.75, mutual: bool = False, with_dist: bool = False,
              out: torch.Tensor | None = None, exact: bool | None = None):
        """Match every pair (a, b): for each row of a, its ratio-tested nearest row of b.

        Returns ``matches0`` int32 [P, m_pad] on the device (-1 = no match); with
        ``with_dist`` also int32 squared distances ``dist1``, ``dist2`` (of the
        int8 quantisation); with ``mutual`` also the backward ``matches1``
        after the mutual filter.  ``exact`` (default: the bank's mode) selects
        the exact float distance (module docstring).  ``out``: a caller-owned
        contiguous [P, m_pad] int32 or int16 tensor (int16: m_pad <= 32767, the
        kernels write the int16 graph directly — dist.match_all_pairs_sharded's
        all-gathered form — without distances or the mutual filter).
        """
        exact = self.exact if exact is None else bool(exact)
        if exact and self.x is None:
            raise ValueError("exact float matching needs a bank built with from_float(..., exact=True)")
        self._exact_now = exact
        num, den = _ratio(ratio)
        pr = dev(pairs, torch.int32).reshape(-1, 2)
        P = pr.shape[0]
        dv = self.q.device
        m0 = out if out is not None else torch.empty((P, self.m_pad), dtype=torch.int32, device=dv)
        if m0.dtype == torch.int16:
            if with_dist or mutual:
                raise ValueError("an int16 graph has no distance outputs or mutual filter: use an int32 out")
            if self.m_pad > 32767:
                raise ValueError(f"an int16 graph needs m_pad <= 32767, got {self.m_pad}")
        elif m0.dtype != torch.int32:
            raise ValueError(f"out must be int32 or int16, got {m0.dtype}")
        if tuple(m0.shape) != (P, self.m_pad) or not m0.is_contiguous() or m0.device != dv:
            raise ValueError(f"out must be a contiguous ({P}, {self.m_pad}) tensor on {dv}")
        d1 = torch.empty_like(m0) if with_dist else None
        d2 = torch.empty_like(m0) if with_dist else None
        self._launch(pr, num, den, m0, d1, d2)
        if not mutual:
            return (m0, d1, d2) if with_dist else m0
        m1 = torch.empty_like(m0)
        e1 = torch.empty_like(m0) if with_dist else None
        e2 = torch.empty_like(m0) if with_dist else None
        self._launch(pr.flip(1).contiguous(), num, den, m1, e1, e2)
        call("sfmhip_mutual_filter", ptr(m0), ptr(m1), P, self.m_pad, stream_ptr())
        return (m0, m1, d1, d2, e1, e2) if with_dist else (m0, m1)

    def _launch(self, pr, num, den, m0, d1, d2, exact: bool | None = None):
        exact = getattr(self, "_exact_now", False) if exact is None else exact
        i16 = m0.dtype == torch.int16
        if exact and i16:
            call("sfmhip_match_pairs_exact_i16", ptr(self.qm), ptr(self.norms), ptr(self.keys), ptr(self.q),
                 ptr(self.x), ptr(self.erow), ptr(self.eimg), self.mode, ptr(self.n_kpts), self.n_img, self.m_pad,
                 self.d, ptr(pr), int(pr.shape[0]), num, den, ptr(m0), ptr(self._nres), stream_ptr())
            self.last_resolved = self._nres
            return
        if i16:
            call("sfmhip_match_pairs_i16", ptr(self.qm), ptr(self.norms), ptr(self.keys), ptr(self.n_kpts),
                 self.n_img, self.m_pad, self.d, ptr(pr), int(pr.shape[0]), num, den, ptr(m0), stream_ptr())
            return
        if exact:
            call("sfmhip_match_pairs_exact", ptr(self.qm), ptr(self.norms), ptr(self.keys), ptr(self.q), ptr(self.x),
                 ptr(self.erow), ptr(self.eimg), self.mode, ptr(self.n_kpts), self.n_img, self.m_pad, self.d,
                 ptr(pr), int(pr.shape[0]), num, den, ptr(m0), ptr(d1), ptr(d2), ptr(self._nres), stream_ptr())
            self.last_resolved = self._nres
            return
        call("sfmhip_match_pairs", ptr(self.qm), ptr(self.norms), ptr(self.keys), ptr(self.n_kpts),
             self.n_img, self.m_pad, self.d, ptr(pr), int(pr.shape[0]), num, den,
             ptr(m0), ptr(d1), ptr(d2), stream_ptr())


def all_pairs(n_img: int) -> np.ndarray:
    """Exhaustive (a < b) pair list, int32 (P, 2), P = n(n-1)/2, a-major order."""
    a, b = np.triu_indices(n_img, k=1)
    return np.stack([a, b], 1).astype(np.int32)


def bf_match(desc0, desc1, ratio=0.75, mutual: bool = False, mode: int = MODE_FLOAT, exact: bool | None = None):
    """One pair, numpy in / numpy out: ``matches0`` int64 (M,), -1 = no match."""
    d0 = np.asarray(desc0, dtype=np.float32)
    d1 = np.asarray(desc1, dtype=np.float32)
    bank = DescriptorBank.from_float([d0, d1], mode=mode, exact=exact)
    res = bank.match(np.array([[0, 1]], dtype=np.int32), ratio=ratio, mutual=mutual)
    m0 = res[0] if mutual else res
    torch.cuda.synchronize()
    return m0[0, :d0.shape[0]].cpu().numpy().astype(np.int64)


def _exact_scores(x0: torch.Tensor, x1: torch.Tensor, m0: torch.Tensor) -> torch.Tensor:
    """1 - sqrt(d1/d2) for the matched rows of x0 from the exact mode's metric:
    d = sum_k (f64(a_k) - f64(b_k))^2 summed in k order, one IEEE op per step
    (oracle/match.py:sq_dist_exact, bit for bit); d1 to the match, d2 the best
    other row of x1; 0 for unmatched rows.  Only the matched rows are scored, in
    row chunks of <= 32 MB of f64 distances."""
    sc = torch.zeros(x0.shape[0], dtype=torch.float32, device=x0.device)
    rows = torch.nonzero(m0 >= 0).flatten()
    if rows.numel() == 0:
        return sc
    a, bt = x0[rows].float().double(), x1.float().double().t().contiguous()
    n, d = bt.shape[1], bt.shape[0]
    step = max(1, (32 << 20) // (8 * max(1, n)))
    for r0 in range(0, a.shape[0], step):
        ar = a[r0:r0 + step]
        D = torch.zeros((ar.shape[0], n), dtype=torch.float64, device=a.device)
        t = torch.empty_like(D)
        for k in range(d):   # k order, one IEEE op per step (sub, mul, add: no fused form)
            torch.sub(ar[:, k:k + 1], bt[k][None, :], out=t)
            t.mul_(t)
            D.add_(t)
        ri = torch.arange(ar.shape[0], device=a.device)
        j = m0[rows[r0:r0 + step]]
        d1 = D[ri, j]
        D[ri, j] = float("inf")
        d2 = D.min(dim=1).values if n > 1 else torch.full_like(d1, float("inf"))
        sc[rows[r0:r0 + step]] = (1.0 - torch.sqrt(d1 / d2.clamp_min(1e-300))).float()
    return sc


class Matcher(torch.nn.Module):
    """Brute-force L2 + ratio-test matcher with LightGlue's call/return contract.

    ``Matcher(ratio=0.75, mutual=True, mode=MODE_FLOAT)(data)`` where ``data`` is
    ``{'image0': {'descriptors': (1,M,d), ...}, 'image1': {...}}`` as built at
    ``matching.py:107-120``.  ``matching_scores0`` = 1 - sqrt(d1/d2) (the Lowe
    margin) for matched keypoints, 0 otherwise: from the f64 difference-form
    distances of the descriptors as given in the exact mode, from the int8
    distances otherwise (matching.py reads only ``matches``).  ``exact``
    (default True): the exact float distance on the descriptors as given; it
    needs finite descriptors and raises ValueError on NaN / inf, where
    LightGlue would pass them through (``exact=False`` matches the int8
    quantisation, which maps non-finite values like any out-of-range value).
    """

    default_conf = {"ratio": 0.75, "mutual": True, "mode": MODE_FLOAT, "exact": True}

    def __init__(self, features: str | None = None, **conf):
        super().__init__()
        self.conf = {**self.default_conf, **conf}
        if features == "sift" and "mode" not in conf:
            self.conf["mode"] = MODE_SIFT

    def forward(self, data: dict) -> dict:
        desc0 = data["image0"]["descriptors"]
        desc1 = data["image1"]["descriptors"]
        if desc0.dim() != 3 or desc0.shape[0] != 1 or desc1.shape[0] != 1:
            raise ValueError("Matcher expects batch size 1 descriptors (1, M, d)")
        out_dev = desc0.device
        M, N = desc0.shape[1], desc1.shape[1]
        bank = DescriptorBank.from_float([desc0[0].detach(), desc1[0].detach()], mode=self.conf["mode"],
                                         exact=self.conf["exact"])
        pr = np.array([[0, 1]], dtype=np.int32)
        if self.conf["mutual"]:
            m0, m1, d1, d2, e1, e2 = bank.match(pr, ratio=self.conf["ratio"], mutual=True, with_dist=True)
        else:
            m0, d1, d2 = bank.match(pr, ratio=self.conf["ratio"], with_dist=True)
            m1 = torch.full_like(m0, -1)
            e1 = e2 = None
        m0 = m0[:, :M].long()
        m1 = m1[:, :N].long()
        if not self.conf["mutual"]:
            # matches1 from the forward result (first i claiming each j).
            i_idx = torch.nonzero(m0[0] >= 0).flatten()
            m1[0].scatter_reduce_(0, m0[0, i_idx], i_idx, reduce="amin", include_self=False)
        if self.conf["exact"]:
            sc0 = _exact_scores(desc0[0].detach(), desc1[0].detach(), m0[0].to(desc0.device))[None].to(m0.device)
        else:
            d1f = d1[:, :M].double().clamp_min(0)
            d2f = d2[:, :M].double().clamp_min(1e-12)
            sc0 = torch.where(m0 >= 0, 1.0 - torch.sqrt(d1f / d2f), torch.zeros_like(d1f)).float()
        sc1 = torch.zeros((1, N), dtype=torch.float32, device=m0.device)
        valid1 = m1[0] >= 0
        sc1[0, valid1] = sc0[0, m1[0, valid1]]
        valid = m0[0] >= 0
        idx0 = torch.nonzero(valid).flatten()
        matches = torch.stack([idx0, m0[0, idx0]], -1)
        pred = {
            "matches0": m0.to(out_dev),
            "matches1": m1.to(out_dev),
            "matching_scores0": sc0.to(out_dev),
            "matching_scores1": sc1.to(out_dev),
            "stop": 1,
            "matches": [matches.to(out_dev)],
            "scores": [sc0[0, idx0].to(out_dev)],
        }
        return pred


def vq(obs, code_book, check_finite: bool = True):
    """``scipy.cluster.vq.vq`` on the GPU: (codes int32 (K,), dist f64 (K,)).

    Exact (bit-identical codes and distances) for integer-valued inputs; for
    general floats the k-ordered f64 sum can differ from scipy's BLAS-based
    distance in the last bits ("vq parity").
    """
    o = np.asarray(obs, dtype=np.float64)
    c = np.asarray(code_book, dtype=np.float64)
    if o.ndim == 1:
        o = o[:, None]
    if c.ndim == 1:
        c = c[:, None]
    if o.shape[1] != c.shape[1]:
        raise ValueError("Observation and code_book should have the same rank")
    if check_finite and (not np.isfinite(o).all() or not np.isfinite(c).all()):
        raise ValueError("array must not contain infs or NaNs")
    ot, ct = dev(o, torch.float64), dev(c, torch.float64)
    K = ot.shape[0]
    codes = torch.empty(K, dtype=torch.int32, device=ot.device)
    dist = torch.empty(K, dtype=torch.float64, device=ot.device)
    call("sfmhip_vq", ptr(ot), K, ptr(ct), ct.shape[0], ct.shape[1], ptr(codes), ptr(dist), stream_ptr())
    torch.cuda.synchronize()
    return codes.cpu().numpy(), dist.cpu().numpy()
