// ransac.hip — SURVEY.md §8f row 2: batched geometric verification, f64.
//
// Reference call sites:
//   cv2.findEssentialMat(pts0, pts1, K, method=cv2.RANSAC, prob=0.999, threshold=1)
//        matching.py:134, sfm.py:108
//   cv2.recoverPose(E, pts0, pts1, K)                 matching.py:139, sfm.py:117,119
// Restated from OpenCV 4.x (calib3d: ptsetreg.cpp RANSACPointSetRegistrator,
// five-point.cpp EMEstimatorCallback, decomposeEssentialMat, recoverPose);
// the CPU restatement is oracle/ransac.py.  Parity at the OpenCV boundary is
// unpinned (cv2 absent).
//
// One workgroup (8 waves) per image pair.  Hypotheses are processed kRH = 32
// at a time:
//   1. lane 0 draws the 32 five-point samples from cv::RNG(-1) (sequential by
//      definition — a sample depends only on the draw order, never on the
//      models, so the draws can run ahead of the scoring);
//   2. each sample is solved by a 16-lane group (Nister's method): the 10x20
//      constraint matrix is held column-per-lane in registers and reduced by
//      Gauss-Jordan with shuffles; the real roots of the degree-10 polynomial
//      are isolated level by level between the roots of its derivatives, one
//      interval per lane; one lane per root back-substitutes;
//   3. all 512 lanes score every model of the chunk (points in registers,
//      Sampson error as float with an exact division only near the
//      threshold): the chunk's models are listed once, then scored two at a
//      time (independent chains for latency hiding at 2 waves/SIMD), each
//      wave's ballot counts stored per (model, wave) in LDS without atomics;
//   4. lane 0 replays the chunk in OpenCV's sequential order: a model
//      replaces the best iff count > max(best, 4), niters shrinks by
//      RANSACUpdateNumIters — so the chosen model and the iteration count are
//      exactly those of the sequential loop over the same models.
#include <algorithm>
#include <climits>
#include <cstdlib>
#include <mutex>

#include "common.h"
#include "geom_dev.h"

namespace sfmhip {
namespace {

constexpr int kRThreads = 512;          // essential kernel: 8 waves
constexpr int kGL = 16;                 // lanes per hypothesis group
constexpr int kRH = kRThreads / kGL;    // hypotheses per chunk (32)
constexpr int kMaxModels = 10;
constexpr int kGS = 224;                // LDS doubles per group
constexpr int kPB = 4;                  // points per lane per scoring block
constexpr int kRWaves = kRThreads / 64;
constexpr int kPThreads = 768;          // recover_pose kernel: 3 waves per SIMD (156 VGPRs), one workgroup per CU
constexpr double kDblEps = 2.220446049250313e-16;
constexpr double kDblMin = 2.2250738585072014e-308;
#ifndef SFMHIP_ABERTH_FAST
#define SFMHIP_ABERTH_FAST 1
#endif
constexpr bool kAberthFast = SFMHIP_ABERTH_FAST != 0;   // Aberth steps on rcp_nr (A/B: -DSFMHIP_ABERTH_FAST=0)

// cv::RNG: multiply-with-carry, uniform(a, b) = a + next() % (b - a).
struct CvRng {
    uint64_t s;
    __device__ unsigned next() {
        s = (uint64_t)(unsigned)s * 4164903690ULL + (unsigned)(s >> 32);
        return (unsigned)s;
    }
    __device__ int uniform(int a, int b) { return a == b ? a : (int)(next() % (unsigned)(b - a) + (unsigned)a); }
    // uniform(0, n) with x % n computed from a double reciprocal (exact after
    // one correction: x < 2^32, so the quotient estimate is off by at most 1)
    __device__ int uniform0(unsigned n, double inv_n) {
        const unsigned x = next();
        unsigned qd = (unsigned)((double)x * inv_n);
        long long r = (long long)x - (long long)qd * n;
        if (r < 0) r += n;
        else if (r >= (long long)n) r -= n;
        return (int)r;
    }
};

// RANSACUpdateNumIters (ptsetreg.cpp).
__device__ int update_num_iters(double p, double ep, int m, int max_iters) {
    p = fmax(p, 0.0);
    p = fmin(p, 1.0);
    ep = fmax(ep, 0.0);
    ep = fmin(ep, 1.0);
    double num = fmax(1.0 - p, kDblMin);
    double denom = 1.0 - pow(1.0 - ep, (double)m);
    if (denom < kDblMin) return 0;
    num = log(num);
    denom = log(denom);
    return (denom >= 0 || -num >= max_iters * (-denom)) ? max_iters : (int)rint(num / denom);
}

// Monomial tables.  Linear: x y z 1.  Quadratic: x2 xy xz x y2 yz y z2 z 1.
// Cubic (Nister / OpenCV order): x3 y3 x2y xy2 x2z x2 y2z y2 xyz xy | xz2 xz x yz2 yz y z3 z2 z 1.
constexpr int kLL[4][4] = {{0, 1, 2, 3}, {1, 4, 5, 6}, {2, 5, 7, 8}, {3, 6, 8, 9}};
constexpr int kQL[10][4] = {{0, 2, 4, 5},    {2, 3, 8, 9},     {4, 8, 10, 11},   {5, 9, 11, 12},
                            {3, 1, 6, 7},    {8, 6, 13, 14},   {9, 7, 14, 15},   {10, 13, 16, 17},
                            {11, 14, 17, 18}, {12, 15, 18, 19}};
__device__ __forceinline__ void mul_ll(const double* a, const double* b, double sgn, double* q) {
#pragma clang fp contract(fast)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) q[kLL[i][j]] += sgn * (a[i] * b[j]);
}
__device__ __forceinline__ void mul_ql(const double* q, const double* l, double sgn, double* c) {
#pragma clang fp contract(fast)
#pragma unroll
    for (int i = 0; i < 10; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) c[kQL[i][j]] += sgn * (q[i] * l[j]);
}

template <int NA, int NB>
__device__ __forceinline__ void pmul(const double* a, const double* b, double* o) {
#pragma clang fp contract(fast)
#pragma unroll
    for (int i = 0; i < NA + NB - 1; ++i) o[i] = 0.0;
#pragma unroll
    for (int i = 0; i < NA; ++i)
#pragma unroll
        for (int j = 0; j < NB; ++j) o[i + j] += a[i] * b[j];
}

__device__ __forceinline__ void wave_sync_lds() { __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront"); }

// Phase timers for tools/prof_ransac.py: build with -DSFMHIP_RANSAC_PROF
// (make EXTRA=-DSFMHIP_RANSAC_PROF); compiled out otherwise.
#ifdef SFMHIP_RANSAC_PROF
__device__ unsigned long long g_rprof[16];
#define SPROF(i) do { if (threadIdx.x == 0) { const unsigned long long t1 = wall_clock64(); atomicAdd(&g_rprof[i], t1 - st); st = t1; } } while (0)
#define SPROF_INIT unsigned long long st = wall_clock64()
#define RPROF(i, t0) do { if (tid == 0) { const unsigned long long t1 = wall_clock64(); atomicAdd(&g_rprof[i], t1 - t0); t0 = t1; } } while (0)
#define RPROF_INIT unsigned long long tp = wall_clock64()
#define PROF_COUNT(i, v) do { if (threadIdx.x == 0) atomicAdd(&g_rprof[i], (unsigned long long)(v)); } while (0)
#else
#define SPROF(i) do {} while (0)
#define SPROF_INIT do {} while (0)
#define RPROF(i, t0) do {} while (0)
#define RPROF_INIT do {} while (0)
#define PROF_COUNT(i, v) do {} while (0)
#endif

// EMEstimatorCallback::runKernel for one sample, by a 16-lane group (gl =
// lane in group, gsh = bit offset of the group in the wave's ballot).  G is
// the group's LDS area; up to 10 unit-norm E (row-major) go to models.
__device__ int five_point_group(const double (&q)[5][4], int gl, int gsh, double* G, double* models) {
#pragma clang fp contract(fast)
    SPROF_INIT;
    // 1. orthonormal null-space basis of the 5x9 system (Householder QR of
    //    Q^T, reflectors stored in place; every lane computes it in registers).
    double A[9][5], beta[5];
#pragma unroll
    for (int j = 0; j < 5; ++j) {
        const double x1 = q[j][0], y1 = q[j][1], x2 = q[j][2], y2 = q[j][3];
        A[0][j] = x1 * x2; A[1][j] = y1 * x2; A[2][j] = x2;
        A[3][j] = x1 * y2; A[4][j] = y1 * y2; A[5][j] = y2;
        A[6][j] = x1;      A[7][j] = y1;      A[8][j] = 1.0;
    }
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        double nrm2 = 0;
#pragma unroll
        for (int r = k; r < 9; ++r) nrm2 += A[r][k] * A[r][k];
        const double nrm = sqrt_nr(nrm2);
        const double alpha = (A[k][k] >= 0) ? -nrm : nrm;
        A[k][k] -= alpha;  // column k below the diagonal is now the reflector v_k
        double vn2 = 0;
#pragma unroll
        for (int r = k; r < 9; ++r) vn2 += A[r][k] * A[r][k];
        beta[k] = (vn2 > 0) ? 2.0 * rcp_nr(vn2) : 0.0;
#pragma unroll
        for (int c = k + 1; c < 5; ++c) {
            double s = 0;
#pragma unroll
            for (int r = k; r < 9; ++r) s += A[r][k] * A[r][c];
            s *= beta[k];
#pragma unroll
            for (int r = k; r < 9; ++r) A[r][c] -= s * A[r][k];
        }
    }
    double basis[4][9];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
#pragma unroll
        for (int r = 0; r < 9; ++r) basis[j][r] = (r == 5 + j) ? 1.0 : 0.0;
#pragma unroll
        for (int k = 4; k >= 0; --k) {
            double s = 0;
#pragma unroll
            for (int r = k; r < 9; ++r) s += A[r][k] * basis[j][r];
            s *= beta[k];
#pragma unroll
            for (int r = k; r < 9; ++r) basis[j][r] -= s * A[r][k];
        }
    }
    SPROF(3);
    // E entries as linear polys in (x, y, z, 1): E = x b0 + y b1 + z b2 + b3.
    double E[9][4];
#pragma unroll
    for (int e = 0; e < 9; ++e)
#pragma unroll
        for (int j = 0; j < 4; ++j) E[e][j] = basis[j][e];

    // 2. constraint rows: lane 0 -> det E, lane r = 1..9 -> (2 E E^T E - tr(E E^T) E)_{ij}
    //    with i = (r-1)/3, j = (r-1)%3.  Rows go through LDS to become columns.
    if (gl < 10) {
        double c[20];
#pragma unroll
        for (int m = 0; m < 20; ++m) c[m] = 0.0;
        if (gl == 0) {
            double t1[10], t2[10], t3[10];
#pragma unroll
            for (int m = 0; m < 10; ++m) t1[m] = t2[m] = t3[m] = 0.0;
            mul_ll(E[4], E[8], 1.0, t1); mul_ll(E[5], E[7], -1.0, t1);
            mul_ll(E[3], E[8], 1.0, t2); mul_ll(E[5], E[6], -1.0, t2);
            mul_ll(E[3], E[7], 1.0, t3); mul_ll(E[4], E[6], -1.0, t3);
            mul_ql(t1, E[0], 1.0, c);
            mul_ql(t2, E[1], -1.0, c);
            mul_ql(t3, E[2], 1.0, c);
        } else {
            const int i = (gl - 1) / 3, j = (gl - 1) % 3;
            double Ei[3][4], Ej[3][4], Eij[4];
#pragma unroll
            for (int k = 0; k < 3; ++k)
#pragma unroll
                for (int m = 0; m < 4; ++m) {
                    Ei[k][m] = (i == 0) ? E[k][m] : (i == 1) ? E[3 + k][m] : E[6 + k][m];
                    Ej[k][m] = (j == 0) ? E[3 * k][m] : (j == 1) ? E[3 * k + 1][m] : E[3 * k + 2][m];
                }
#pragma unroll
            for (int m = 0; m < 4; ++m) Eij[m] = (j == 0) ? Ei[0][m] : (j == 1) ? Ei[1][m] : Ei[2][m];
            double tr[10];
#pragma unroll
            for (int m = 0; m < 10; ++m) tr[m] = 0.0;
#pragma unroll
            for (int e = 0; e < 9; ++e) mul_ll(E[e], E[e], 1.0, tr);
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                double eet[10];
#pragma unroll
                for (int m = 0; m < 10; ++m) eet[m] = 0.0;
#pragma unroll
                for (int l = 0; l < 3; ++l) mul_ll(Ei[l], E[3 * k + l], 1.0, eet);
                mul_ql(eet, Ej[k], 2.0, c);
            }
            mul_ql(tr, Eij, -1.0, c);
        }
#pragma unroll
        for (int m = 0; m < 20; ++m) G[gl * 20 + m] = c[m];
    }
    wave_sync_lds();
    double col[10], col2[10];
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        col[r] = G[r * 20 + gl];
        col2[r] = (gl < 4) ? G[r * 20 + 16 + gl] : 0.0;
    }
    wave_sync_lds();
    double* GE = G + 128;   // E polys, kept for the back-substitution
    double* GB = G + 64;    // B(z) polys
    if (gl == 0)
#pragma unroll
        for (int e = 0; e < 9; ++e)
#pragma unroll
            for (int j = 0; j < 4; ++j) GE[e * 4 + j] = E[e][j];
    SPROF(4);
    // 3. Gauss-Jordan on the left 10x10 block (partial pivoting; OpenCV's LU
    //    calls a pivot below 100*DBL_EPSILON singular).  Column k lives in lane k.
#pragma unroll
    for (int k = 0; k < 10; ++k) {
        int pl = k;
        double pv = fabs(col[k]);
#pragma unroll
        for (int r = k + 1; r < 10; ++r)
            if (fabs(col[r]) > pv) { pv = fabs(col[r]); pl = r; }
        const int p = __shfl(pl, k, kGL);
#pragma unroll
        for (int r = k + 1; r < 10; ++r)
            if (r == p) {
                double t = col[k]; col[k] = col[r]; col[r] = t;
                t = col2[k]; col2[k] = col2[r]; col2[r] = t;
            }
        double f[10];
#pragma unroll
        for (int r = 0; r < 10; ++r) f[r] = __shfl(col[r], k, kGL);
        if (fabs(f[k]) < 100 * kDblEps) return 0;
        const double inv = rcp_nr(f[k]);
        const double xk = col[k] * inv, xk2 = col2[k] * inv;
#pragma unroll
        for (int r = 0; r < 10; ++r) {
            if (r == k) continue;
            col[r] -= f[r] * xk;
            col2[r] -= f[r] * xk2;
        }
        col[k] = xk;
        col2[k] = xk2;
    }
    SPROF(5);
    // 4. rows 4..9 of A[:, :10]^-1 A[:, 10:] -> B(z) = e_row - z f_row (ascending in z).
    if (gl >= 10) {
#pragma unroll
        for (int r = 0; r < 6; ++r) G[r * 10 + gl - 10] = col[4 + r];
    } else if (gl < 4) {
#pragma unroll
        for (int r = 0; r < 6; ++r) G[r * 10 + 6 + gl] = col2[4 + r];
    }
    wave_sync_lds();
    double bx[3][4], by[3][4], bc[3][5];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        double e[10], f[10];
#pragma unroll
        for (int c = 0; c < 10; ++c) {
            e[c] = G[(2 * r) * 10 + c];
            f[c] = G[(2 * r + 1) * 10 + c];
        }
        bx[r][0] = e[2]; bx[r][1] = e[1] - f[2]; bx[r][2] = e[0] - f[1]; bx[r][3] = -f[0];
        by[r][0] = e[5]; by[r][1] = e[4] - f[5]; by[r][2] = e[3] - f[4]; by[r][3] = -f[3];
        bc[r][0] = e[9]; bc[r][1] = e[8] - f[9]; bc[r][2] = e[7] - f[8]; bc[r][3] = e[6] - f[7]; bc[r][4] = -f[6];
    }
    wave_sync_lds();
    if (gl == 0)
#pragma unroll
        for (int r = 0; r < 3; ++r) {
#pragma unroll
            for (int m = 0; m < 4; ++m) { GB[r * 13 + m] = bx[r][m]; GB[r * 13 + 4 + m] = by[r][m]; }
#pragma unroll
            for (int m = 0; m < 5; ++m) GB[r * 13 + 8 + m] = bc[r][m];
        }
    // 5. det B(z), degree 10 (every lane).
    double c[11];
    {
        double a7[8], b7[8], m7[8], a6[7], b6[7], m6[7], t[11];
        pmul<4, 5>(by[1], bc[2], a7); pmul<4, 5>(by[2], bc[1], b7);
#pragma unroll
        for (int i = 0; i < 8; ++i) m7[i] = a7[i] - b7[i];
        pmul<4, 8>(bx[0], m7, t);
#pragma unroll
        for (int i = 0; i < 11; ++i) c[i] = t[i];
        pmul<4, 5>(bx[1], bc[2], a7); pmul<4, 5>(bx[2], bc[1], b7);
#pragma unroll
        for (int i = 0; i < 8; ++i) m7[i] = a7[i] - b7[i];
        pmul<4, 8>(by[0], m7, t);
#pragma unroll
        for (int i = 0; i < 11; ++i) c[i] -= t[i];
        pmul<4, 4>(bx[1], by[2], a6); pmul<4, 4>(bx[2], by[1], b6);
#pragma unroll
        for (int i = 0; i < 7; ++i) m6[i] = a6[i] - b6[i];
        pmul<5, 7>(bc[0], m6, t);
#pragma unroll
        for (int i = 0; i < 11; ++i) c[i] += t[i];
    }
    SPROF(6);
    // 6. roots of det B(z) by Aberth-Ehrlich simultaneous iteration, one root
    //    per lane (OpenCV's solvePoly iterates all roots simultaneously too,
    //    Durand-Kerner); real roots = |imag| <= 1e-10 (five-point.cpp's
    //    test), polished by two real Newton steps, visited in ascending order.
    double cmax = 0;
#pragma unroll
    for (int i = 0; i < 11; ++i) cmax = fmax(cmax, fabs(c[i]));
    if (cmax == 0.0) return 0;
    int n = 10;
#pragma unroll
    for (int i = 10; i >= 1; --i)
        if (n == i && fabs(c[i]) <= kDblEps * cmax) n = i - 1;
    if (n == 0) return 0;
    double lead = 0;
#pragma unroll
    for (int i = 0; i < 11; ++i)
        if (i == n) lead = c[i];
    double a[10];  // monic: z^n + a[n-1] z^(n-1) + ... + a[0]
#pragma unroll
    for (int i = 0; i < 10; ++i) a[i] = (i < n) ? c[i] / lead : 0.0;
    const bool act = gl < n;
    double zr = 0, zi = 0;
    {
        const double R = fmax(exp(log(fmax(fabs(a[0]), 1e-300)) / n), 1e-8);
        const double ang = 6.283185307179586 * gl / n + 0.4;
        zr = R * cos(ang);
        zi = R * sin(ang);
    }
    double* Z = G;
    bool conv = !act;
    for (int it = 0; it < 80; ++it) {
        if (act) { Z[2 * gl] = zr; Z[2 * gl + 1] = zi; }
        wave_sync_lds();
        if (!conv) {
            double pr = 1.0, pim = 0.0, dr = 0.0, di = 0.0, pabs = 1.0;
            const double az = sqrt(zr * zr + zi * zi);
#pragma unroll
            for (int j = 9; j >= 0; --j)
                if (j < n) {
                    pabs = __builtin_fma(pabs, az, fabs(a[j]));
                    const double ndr = __builtin_fma(dr, zr, __builtin_fma(-di, zi, pr));
                    const double ndi = __builtin_fma(dr, zi, __builtin_fma(di, zr, pim));
                    const double npr = __builtin_fma(pr, zr, __builtin_fma(-pim, zi, a[j]));
                    const double npi = __builtin_fma(pr, zi, pim * zr);
                    dr = ndr; di = ndi; pr = npr; pim = npi;
                }
            // N = p / p'.  The iteration's quotients use Newton-refined reciprocals (rcp_nr, within
            // an ulp): the roots are fixed points of the iteration whatever the rounding of its
            // steps, and real roots are polished below with IEEE Newton steps.
            const double dd = dr * dr + di * di;
            double nr_ = 0, ni_ = 0;
            if (dd > 0) {
                const double idd = kAberthFast ? rcp_nr(dd) : 1.0 / dd;
                nr_ = (pr * dr + pim * di) * idd;
                ni_ = (pim * dr - pr * di) * idd;
            }
            double sr = 0, si = 0;  // S = sum_{j != i} 1 / (z - z_j)
#pragma unroll
            for (int j = 0; j < 10; ++j)
                if (j < n && j != gl) {
                    const double xr = zr - Z[2 * j], xi = zi - Z[2 * j + 1];
                    const double m = xr * xr + xi * xi;
                    if (m > 0) {
                        if (kAberthFast) {
                            const double im = rcp_nr(m);
                            sr += xr * im;
                            si -= xi * im;
                        } else {
                            sr += xr / m;
                            si -= xi / m;
                        }
                    }
                }
            // w = N / (1 - N S)
            const double qr = 1.0 - (nr_ * sr - ni_ * si), qi = -(nr_ * si + ni_ * sr);
            const double qq = qr * qr + qi * qi;
            double wr = nr_, wi = ni_;
            if (qq > 0) {
                const double iqq = kAberthFast ? rcp_nr(qq) : 1.0 / qq;
                wr = (nr_ * qr + ni_ * qi) * iqq;
                wi = (ni_ * qr - nr_ * qi) * iqq;
            }
            zr -= wr;
            zi -= wi;
            // converged: step at rounding level, or |p(z)| within the rounding noise of Horner
            // (compared squared: no square roots on the chain).  Magnitudes >= 2^500 are scaled
            // by 2^-600 first (exact), so no square overflows into a trivially true test.
            const double sc = (pabs >= 0x1p500 || az >= 0x1p500 || fabs(wr) + fabs(wi) >= 0x1p500) ? 0x1p-600 : 1.0;
            const double wrs = wr * sc, wis = wi * sc, zrs = zr * sc, zis = zi * sc;
            const double prs = pr * sc, pis = pim * sc, pas = pabs * sc;
            conv = (wrs * wrs + wis * wis) <= (16 * kDblEps * kDblEps) * (zrs * zrs + zis * zis) ||
                   (prs * prs + pis * pis) <= (256 * kDblEps * kDblEps) * (pas * pas);
        }
        wave_sync_lds();
        if ((((unsigned)(__ballot(!conv) >> gsh)) & 0xFFFFu) == 0u) {
            PROF_COUNT(12, it);
            PROF_COUNT(13, 1);
            break;
        }
    }
    bool real = act && fabs(zi) <= 1e-10;
    double xr = zr;
    if (real) {
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
            double f = 1.0, df = 0.0;
#pragma unroll
            for (int j = 9; j >= 0; --j)
                if (j < n) {
                    df = __builtin_fma(df, xr, f);
                    f = __builtin_fma(f, xr, a[j]);
                }
            if (df != 0.0 && f != 0.0) xr -= f / df;
        }
    }
    if (act) { Z[2 * gl] = real ? xr : 0.0; Z[2 * gl + 1] = real ? 1.0 : 0.0; }
    wave_sync_lds();
    const unsigned rm = ((unsigned)(__ballot(real) >> gsh)) & 0xFFFFu;
    int rank = 0;
#pragma unroll
    for (int j = 0; j < 10; ++j)
        if (j < n && j != gl && Z[2 * j + 1] != 0.0) {
            const double xj = Z[2 * j];
            rank += (xj < xr || (xj == xr && j < gl)) ? 1 : 0;
        }
    wave_sync_lds();
    double* prev = G + 32;
    if (real) prev[rank] = xr;
    wave_sync_lds();
    const int np = __popc(rm);
    const int nr = np;
    SPROF(7);
    // 7. back-substitution, one root per lane: null vector of B(z) -> (x, y),
    //    E = x E0 + y E1 + z E2 + E3, normalised.
    bool ok = false;
    double ev[9];
    if (gl < nr) {
        const double z = prev[gl];
        double row[3][3];
#pragma unroll
        for (int r = 0; r < 3; ++r) {
            const double* b = GB + r * 13;
            row[r][0] = ((b[3] * z + b[2]) * z + b[1]) * z + b[0];
            row[r][1] = ((b[7] * z + b[6]) * z + b[5]) * z + b[4];
            row[r][2] = (((b[12] * z + b[11]) * z + b[10]) * z + b[9]) * z + b[8];
        }
        double best[3] = {0, 0, 0}, bn = -1;
#pragma unroll
        for (int pi = 0; pi < 3; ++pi) {
            const int a = (pi == 2) ? 1 : 0, b = (pi == 0) ? 1 : 2;
            const double cx = row[a][1] * row[b][2] - row[a][2] * row[b][1];
            const double cy = row[a][2] * row[b][0] - row[a][0] * row[b][2];
            const double cz = row[a][0] * row[b][1] - row[a][1] * row[b][0];
            const double n2 = cx * cx + cy * cy + cz * cz;
            if (n2 > bn) { bn = n2; best[0] = cx; best[1] = cy; best[2] = cz; }
        }
        if (bn > 0) {
            const double inv = 1.0 / sqrt(bn);
            const double v0 = best[0] * inv, v1 = best[1] * inv, v2 = best[2] * inv;
            if (fabs(v2) >= 1e-10) {
                const double x = v0 / v2, y = v1 / v2;
                double n2 = 0;
#pragma unroll
                for (int e = 0; e < 9; ++e) {
                    ev[e] = GE[4 * e] * x + GE[4 * e + 1] * y + GE[4 * e + 2] * z + GE[4 * e + 3];
                    n2 += ev[e] * ev[e];
                }
                const double s = 1.0 / sqrt(n2);
#pragma unroll
                for (int e = 0; e < 9; ++e) ev[e] *= s;
                ok = true;
            }
        }
    }
    const unsigned gm = (unsigned)(__ballot(ok) >> gsh) & 0xFFFFu;
    if (ok) {
        const int slot = __popc(gm & ((1u << gl) - 1u));
#pragma unroll
        for (int e = 0; e < 9; ++e) models[slot * 9 + e] = ev[e];
    }
    SPROF(8);
    return __popc(gm);
}

// EMEstimatorCallback::computeError (Matx op order) <= t, where the stored
// error is (float)(num / den).  T = the largest double that rounds to a float
// <= t; num/den is compared against T with a 2^-40 relative margin and only
// the undecided points take the exact division.
__device__ __forceinline__ bool sampson_in(const double* E, double x1, double y1, double x2, double y2, float tf,
                                           double tlo, double thi) {
    const double ex0 = (E[0] * x1 + E[1] * y1) + E[2];
    const double ex1 = (E[3] * x1 + E[4] * y1) + E[5];
    const double ex2 = (E[6] * x1 + E[7] * y1) + E[8];
    const double et0 = (E[0] * x2 + E[3] * y2) + E[6];
    const double et1 = (E[1] * x2 + E[4] * y2) + E[7];
    const double d = (x2 * ex0 + y2 * ex1) + ex2;
    const double num = d * d;
    const double den = ((ex0 * ex0 + ex1 * ex1) + et0 * et0) + et1 * et1;
    if (den > 0) {
        if (num <= den * tlo) return true;
        if (num > den * thi) return false;
    }
    return (float)(num / den) <= tf;
}

// Sampson numerator and denominator (cv::EMEstimatorCallback::computeError's
// double arithmetic); inlier iff (float)(num / den) <= t^2 as a float.
__device__ __forceinline__ void sampson_nd(const double* E, double x1, double y1, double x2, double y2, double& num,
                                           double& den) {
    const double ex0 = (E[0] * x1 + E[1] * y1) + E[2];
    const double ex1 = (E[3] * x1 + E[4] * y1) + E[5];
    const double ex2 = (E[6] * x1 + E[7] * y1) + E[8];
    const double et0 = (E[0] * x2 + E[3] * y2) + E[6];
    const double et1 = (E[1] * x2 + E[4] * y2) + E[7];
    const double d = (x2 * ex0 + y2 * ex1) + ex2;
    num = d * d;
    den = ((ex0 * ex0 + ex1 * ex1) + et0 * et0) + et1 * et1;
}

__device__ __forceinline__ float sampson(const double* E, double x1, double y1, double x2, double y2) {
    const double ex0 = (E[0] * x1 + E[1] * y1) + E[2];
    const double ex1 = (E[3] * x1 + E[4] * y1) + E[5];
    const double ex2 = (E[6] * x1 + E[7] * y1) + E[8];
    const double et0 = (E[0] * x2 + E[3] * y2) + E[6];
    const double et1 = (E[1] * x2 + E[4] * y2) + E[7];
    const double d = (x2 * ex0 + y2 * ex1) + ex2;
    return (float)(d * d / (((ex0 * ex0 + ex1 * ex1) + et0 * et0) + et1 * et1));
}

__device__ __forceinline__ int wave_count(bool pred) { return __popcll(__ballot(pred)); }
__device__ __forceinline__ int wave_sum(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}


// Scores every listed model of a chunk on all n points: each wave's ballot counts go to
// s_cnt[model][wave] (no atomics).  Branch-free margin tests for two models x kPB points at a
// time, so the chains interleave; the exact division only where a test is ambiguous.
template <int NT = kRThreads>
__device__ __forceinline__ void score_chunk(const double* __restrict__ q, int n, const int* s_list, int nlist,
                                            const double* s_models, int (*s_cnt)[NT / 64], float tf, double tlo,
                                            double thi, int tid, int p_lo = 0, int p_hi = INT_MAX) {
    const int lane = tid & 63, wave = tid >> 6;
    n = min(n, p_hi);   // points [p_lo, p_hi): p_lo a multiple of NT * kPB
    for (int b0 = p_lo; b0 < n; b0 += NT * kPB) {
        double pt[kPB][4];
        bool val[kPB];
#pragma unroll
        for (int u = 0; u < kPB; ++u) {
            const int i = b0 + u * NT + tid;
            val[u] = i < n;
#pragma unroll
            for (int c = 0; c < 4; ++c) pt[u][c] = val[u] ? q[4 * i + c] : 0.0;
        }
        for (int j = 0; j < nlist; j += 2) {   // two models per step: independent chains
            const int ma = s_list[j], mb = s_list[min(j + 1, nlist - 1)];
            double Ea[9], Eb[9];
#pragma unroll
            for (int e = 0; e < 9; ++e) {
                Ea[e] = s_models[ma * 9 + e];
                Eb[e] = s_models[mb * 9 + e];
            }
            // branch-free margin tests for all 2 x kPB (model, point) pairs, so the
            // chains interleave; the exact division only where a test is ambiguous
            double nm[2][kPB], dn[2][kPB];
            bool in[2][kPB], amb = false;
#pragma unroll
            for (int u = 0; u < kPB; ++u) {
                sampson_nd(Ea, pt[u][0], pt[u][1], pt[u][2], pt[u][3], nm[0][u], dn[0][u]);
                sampson_nd(Eb, pt[u][0], pt[u][1], pt[u][2], pt[u][3], nm[1][u], dn[1][u]);
            }
#pragma unroll
            for (int k = 0; k < 2; ++k)
#pragma unroll
                for (int u = 0; u < kPB; ++u) {
                    in[k][u] = nm[k][u] <= dn[k][u] * tlo;
                    amb = amb || !(in[k][u] || nm[k][u] > dn[k][u] * thi) || !(dn[k][u] > 0);
                }
            if (amb) {   // rare: near the threshold (2^-40 relative) or a degenerate denominator
#pragma unroll
                for (int k = 0; k < 2; ++k)
#pragma unroll
                    for (int u = 0; u < kPB; ++u) {
                        const double n_ = nm[k][u], d_ = dn[k][u];
                        const bool sure = d_ > 0 && (n_ <= d_ * tlo || n_ > d_ * thi);
                        if (!sure) in[k][u] = (float)(n_ / d_) <= tf;
                    }
            }
            int ca = 0, cb = 0;  // wave-uniform: ballots + scalar popcounts
#pragma unroll
            for (int u = 0; u < kPB; ++u) {
                ca += wave_count(val[u] && in[0][u]);
                cb += wave_count(val[u] && in[1][u]);
            }
            if (lane == 0) {
                s_cnt[ma][wave] += ca;
                if (j + 1 < nlist) s_cnt[mb][wave] += cb;
            }
        }
    }
}

// The f64 decision of one (model, point) pair: essential_ransac_kernel's margin tests around the
// largest double that rounds to a float <= t, and the exact division where they cannot decide.
__device__ __forceinline__ bool sampson_in_f64(const double* E, const double (&pt)[4], float tf, double tlo,
                                               double thi) {
    double nm, dn;
    sampson_nd(E, pt[0], pt[1], pt[2], pt[3], nm, dn);
    if (dn > 0 && nm <= dn * tlo) return true;
    if (dn > 0 && nm > dn * thi) return false;
    return (float)(nm / dn) <= tf;
}

typedef float f2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2v f2b(float a) { return f2v{a, a}; }
__device__ __forceinline__ f2v fma2v(f2v a, f2v b, f2v c) { return __builtin_elementwise_fma(a, b, c); }

// score_chunk with a packed-f32 pre-test (the load-balanced chunk kernel).  Two points per
// instruction: Ex1, E^T x2, d = x2^T E x1 and den in f32 FMA arithmetic from the f32-rounded
// points and model (|E_ij| <= 1: unit Frobenius norm).  With a = 1 + |x1| + |y1|, b = 1 + |x2| + |y2|
// (u = 2^-24) every f32 ex/et is within 4.01 u a (b) of its exact value, d within 7.1 u a b and
// den within 24.2 u (a^2 + b^2); the bounds used are 12 u a b and 32 u (a^2 + b^2).  A point is
// surely in when (|d| + dd)^2 <= T (1 - 2^-20) (den - dden) and surely out when
// (|d| - dd)^2 > T (1 + 2^-20) (den + dden), T the largest double rounding to a float <= t: the
// margins cover the test's own f32 rounding (< 2^-22) and the f64 path's (~1e-15), so a sure
// decision is the f64 decision.  Every other pair takes sampson_in_f64 (its own lanes only).
template <int NT>
__device__ __forceinline__ void score_chunk_f32(const double* __restrict__ q, int n, const int* s_list, int nlist,
                                                const double* s_models, const float* s_models32,
                                                int (*s_cnt)[NT / 64], float tf, double Tmax, double tlo,
                                                double thi, int tid, int p_lo = 0, int p_hi = INT_MAX) {
    static_assert(kPB % 2 == 0, "points are processed in pairs");
    constexpr int NP = kPB / 2;
    constexpr float u24 = 0x1p-24f;
    const float Tl = (float)(Tmax * (1.0 - 0x1p-20)), Th = (float)(Tmax * (1.0 + 0x1p-20));
    const int lane = tid & 63, wave = tid >> 6;
    n = min(n, p_hi);
    for (int b0 = p_lo; b0 < n; b0 += NT * kPB) {
        double pt[kPB][4];
        bool val[kPB];
#pragma unroll
        for (int u = 0; u < kPB; ++u) {
            const int i = b0 + u * NT + tid;
            val[u] = i < n;
#pragma unroll
            for (int c = 0; c < 4; ++c) pt[u][c] = val[u] ? q[4 * i + c] : 0.0;
        }
        f2v X1[NP], Y1[NP], X2[NP], Y2[NP], DD[NP], DN[NP];
#pragma unroll
        for (int v = 0; v < NP; ++v) {
            X1[v] = f2v{(float)pt[2 * v][0], (float)pt[2 * v + 1][0]};
            Y1[v] = f2v{(float)pt[2 * v][1], (float)pt[2 * v + 1][1]};
            X2[v] = f2v{(float)pt[2 * v][2], (float)pt[2 * v + 1][2]};
            Y2[v] = f2v{(float)pt[2 * v][3], (float)pt[2 * v + 1][3]};
            const f2v a = f2b(1.0f) + __builtin_elementwise_abs(X1[v]) + __builtin_elementwise_abs(Y1[v]);
            const f2v b = f2b(1.0f) + __builtin_elementwise_abs(X2[v]) + __builtin_elementwise_abs(Y2[v]);
            DD[v] = f2b(12.0f * u24) * (a * b);
            DN[v] = f2b(32.0f * u24) * fma2v(a, a, b * b);
        }
        for (int j = 0; j < nlist; j += 2) {   // two models per step: independent chains
            const int mm[2] = {s_list[j], s_list[min(j + 1, nlist - 1)]};
            bool in[2][kPB], amb[2][kPB];
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                float E[9];
#pragma unroll
                for (int e = 0; e < 9; ++e) E[e] = s_models32[mm[k] * 9 + e];
#pragma unroll
                for (int v = 0; v < NP; ++v) {
                    const f2v ex0 = fma2v(f2b(E[0]), X1[v], fma2v(f2b(E[1]), Y1[v], f2b(E[2])));
                    const f2v ex1 = fma2v(f2b(E[3]), X1[v], fma2v(f2b(E[4]), Y1[v], f2b(E[5])));
                    const f2v ex2 = fma2v(f2b(E[6]), X1[v], fma2v(f2b(E[7]), Y1[v], f2b(E[8])));
                    const f2v et0 = fma2v(f2b(E[0]), X2[v], fma2v(f2b(E[3]), Y2[v], f2b(E[6])));
                    const f2v et1 = fma2v(f2b(E[1]), X2[v], fma2v(f2b(E[4]), Y2[v], f2b(E[7])));
                    const f2v d = fma2v(X2[v], ex0, fma2v(Y2[v], ex1, ex2));
                    const f2v den = fma2v(ex0, ex0, fma2v(ex1, ex1, fma2v(et0, et0, et1 * et1)));
                    const f2v ad = __builtin_elementwise_abs(d);
                    const f2v up = ad + DD[v], lo = ad - DD[v];
                    const f2v dl = den - DN[v], dh = den + DN[v];
                    const f2v lhs_in = up * up, rhs_in = f2b(Tl) * dl;
                    const f2v lhs_out = lo * lo, rhs_out = f2b(Th) * dh;
#pragma unroll
                    for (int w = 0; w < 2; ++w) {
                        const bool sin = dl[w] > 0.0f && lhs_in[w] <= rhs_in[w];
                        const bool sout = lo[w] > 0.0f && lhs_out[w] > rhs_out[w];
                        in[k][2 * v + w] = sin;
                        amb[k][2 * v + w] = !(sin || sout);
                    }
                }
            }
#pragma unroll
            for (int k = 0; k < 2; ++k)
#pragma unroll
                for (int u = 0; u < kPB; ++u)
                    if (amb[k][u]) in[k][u] = sampson_in_f64(s_models + mm[k] * 9, pt[u], tf, tlo, thi);
            int ca = 0, cb = 0;  // wave-uniform: ballots + scalar popcounts
#pragma unroll
            for (int u = 0; u < kPB; ++u) {
                ca += wave_count(val[u] && in[0][u]);
                cb += wave_count(val[u] && in[1][u]);
            }
            if (lane == 0) {
                s_cnt[mm[0]][wave] += ca;
                if (j + 1 < nlist) s_cnt[mm[1]][wave] += cb;
            }
        }
    }
}

__global__ __launch_bounds__(kRThreads) void essential_ransac_kernel(
    const double* __restrict__ pts0, const double* __restrict__ pts1, const int64_t* __restrict__ offs,
    const double* __restrict__ cam, double prob, double threshold, int max_iters, double* __restrict__ qn,
    double* __restrict__ E_out, int32_t* __restrict__ nmodels_out, uint8_t* __restrict__ mask,
    int32_t* __restrict__ ninl_out, int32_t* __restrict__ iters_out) {
    __shared__ double s_grp[kRH * kGS];
    __shared__ double s_models[kRH * kMaxModels * 9];
    __shared__ int s_nmod[kRH];
    __shared__ int s_cnt[kRH * kMaxModels][kRWaves];   // per-wave inlier counts
    __shared__ int s_list[kRH * kMaxModels];           // the chunk's models, in replay order
    __shared__ int s_nlist;
    __shared__ int s_sub[kRH * 5];
    __shared__ double s_best[9];
    __shared__ int s_niters, s_maxgood, s_k0, s_last;

    const int p = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
    const int h = tid / kGL, gl = tid % kGL, gsh = (lane / kGL) * kGL;
    const int64_t off = offs[p];
    const int n = (int)(offs[p + 1] - off);
    const double fx = cam[4 * p], fy = cam[4 * p + 1], cx = cam[4 * p + 2], cy = cam[4 * p + 3];
    const double thresh = threshold / ((fx + fy) / 2);
    const float tf = (float)(thresh * thresh);
    // largest double that rounds to a float <= tf (round to nearest even)
    const float tfu = nextafterf(tf, INFINITY);
    const double mid = 0.5 * ((double)tf + (double)tfu);
    const double Tmax = ((__float_as_uint(tf) & 1u) == 0u) ? mid : nextafter(mid, 0.0);
    const double tlo = Tmax * (1.0 - 0x1p-40), thi = Tmax * (1.0 + 0x1p-40);
    double* q = qn + off * 4;
    for (int i = tid; i < n; i += kRThreads) {
        q[4 * i + 0] = (pts0[2 * (off + i)] - cx) / fx;
        q[4 * i + 1] = (pts0[2 * (off + i) + 1] - cy) / fy;
        q[4 * i + 2] = (pts1[2 * (off + i)] - cx) / fx;
        q[4 * i + 3] = (pts1[2 * (off + i) + 1] - cy) / fy;
        mask[off + i] = 0;
    }
    if (tid == 0) {
        s_niters = max(max_iters, 1);
        s_maxgood = 0;
        s_k0 = 0;
        s_last = -1;
    }
    __syncthreads();
    double* Eo = E_out + (int64_t)p * kMaxModels * 9;
    if (n < 5) {
        if (tid == 0) { nmodels_out[p] = 0; ninl_out[p] = 0; iters_out[p] = 0; }
        return;
    }
    if (n == 5) {  // count == modelPoints: one kernel call on all points, mask all ones
        if (h == 0) {
            double qq[5][4];
#pragma unroll
            for (int j = 0; j < 5; ++j)
#pragma unroll
                for (int c = 0; c < 4; ++c) qq[j][c] = q[4 * j + c];
            const int nm = five_point_group(qq, gl, gsh, s_grp, s_models);
            if (gl == 0) {
                for (int e = 0; e < nm * 9; ++e) Eo[e] = s_models[e];
                nmodels_out[p] = nm;
                ninl_out[p] = nm > 0 ? 5 : 0;
                iters_out[p] = 1;
                for (int i = 0; i < 5; ++i) mask[off + i] = nm > 0 ? 1 : 0;
            }
        }
        return;
    }
    CvRng rng{~0ULL};
    const double inv_n = 1.0 / (double)n;
    RPROF_INIT;
    for (;;) {
        const int k0 = s_k0, niters = s_niters;
        if (tid == 0) {
            const int nh = min(kRH, niters - k0);
            for (int hh = 0; hh < nh; ++hh)
                for (int i = 0; i < 5; ++i) {
                    int idx;
                    for (;;) {
                        idx = rng.uniform0((unsigned)n, inv_n);
                        int j = 0;
                        while (j < i && s_sub[hh * 5 + j] != idx) ++j;
                        if (j == i) break;
                    }
                    s_sub[hh * 5 + i] = idx;
                }
        }
        for (int i = tid; i < kRH * kMaxModels * kRWaves; i += kRThreads) (&s_cnt[0][0])[i] = 0;
        __syncthreads();
        RPROF(0, tp);
        {
            int nm = 0;
            if (k0 + h < niters) {
                double qq[5][4];
#pragma unroll
                for (int j = 0; j < 5; ++j) {
                    const int idx = s_sub[h * 5 + j];
#pragma unroll
                    for (int c = 0; c < 4; ++c) qq[j][c] = q[4 * idx + c];
                }
                nm = five_point_group(qq, gl, gsh, s_grp + h * kGS, s_models + h * kMaxModels * 9);
            }
            if (gl == 0) s_nmod[h] = nm;
        }
        __syncthreads();
        if (tid == 0) {
            int c = 0;
            for (int hh = 0; hh < kRH; ++hh)
                for (int m = 0; m < s_nmod[hh]; ++m) s_list[c++] = hh * kMaxModels + m;
            s_nlist = c;
        }
        __syncthreads();
        RPROF(1, tp);
        score_chunk(q, n, s_list, s_nlist, s_models, s_cnt, tf, tlo, thi, tid);
        __syncthreads();
        RPROF(2, tp);
        if (tid == 0) {
            int nit = niters, maxgood = s_maxgood, last = s_last;
            for (int hh = 0; hh < kRH; ++hh) {
                const int k = k0 + hh;
                if (k >= nit) break;
                for (int m = 0; m < s_nmod[hh]; ++m) {
                    int good = 0;
                    for (int w = 0; w < kRWaves; ++w) good += s_cnt[hh * kMaxModels + m][w];
                    if (good > max(maxgood, 4)) {
                        for (int e = 0; e < 9; ++e) s_best[e] = s_models[(hh * kMaxModels + m) * 9 + e];
                        maxgood = good;
                        nit = update_num_iters(prob, (double)(n - good) / n, 5, nit);
                    }
                }
                last = k;
            }
            s_niters = nit;
            s_maxgood = maxgood;
            s_last = last;
            s_k0 = k0 + kRH;
        }
        __syncthreads();
        if (s_k0 >= s_niters) break;
    }
    const int maxgood = s_maxgood;
    if (tid == 0) {
        nmodels_out[p] = maxgood > 0 ? 1 : 0;
        ninl_out[p] = maxgood;
        iters_out[p] = s_last + 1;
        if (maxgood > 0)
            for (int e = 0; e < 9; ++e) Eo[e] = s_best[e];
    }
    if (maxgood > 0)
        for (int i = tid; i < n; i += kRThreads)
            mask[off + i] = sampson(s_best, q[4 * i], q[4 * i + 1], q[4 * i + 2], q[4 * i + 3]) <= tf ? 1 : 0;
}

// ---------------------------------------------------------------------------
// Load-balanced form (default).  essential_ransac_kernel runs a pair's chunks one after another on
// one CU, so a call lasts as long as its pair with the most chunks: on the bench scene (256 pairs
// x 2048 matches) 2-8 chunks of 32 hypotheses, mean 2.9, and the call ~2.6x the mean pair.  Here a
// chunk is a work item that any CU may take, and the sequential parts are separate passes:
//   ess_init_kernel    normalised points, per-pair state (EssState), outputs of n < 5 pairs;
//   ess_gen            one lane per pair draws the pair's samples from cv::RNG(-1) in draw order up
//                      to a target hypothesis count (below) and appends the chunks that cover them to a work list;
//   ess_chunk_kernel   persistent workgroups (256 threads by default, SFMHIP_ESS_CT=512) take
//                      (pair, chunk) items from the list: the chunk's 16 (32) samples solved by
//                      16-lane groups and its models scored on every point (essential_ransac_kernel's
//                      own solver and scoring, with the packed-f32 Sampson pre-test), then its
//                      records: the models whose count exceeds max(4, every earlier count of the
//                      chunk), in replay order;
//   ess_replay_kernel  one lane per pair replays the records in OpenCV's order (a model replaces
//                      the best iff count > max(best, 4); RANSACUpdateNumIters shrinks niters),
//                      then runs ess_gen for the next round (round 0: ess_init_kernel).
// Only a record can ever replace the best (a model at or below an earlier count of its chunk was
// either beaten by that model's acceptance or is <= max(best, 4) already), and niters never grows,
// so the last round — every chunk below the niters the previous replay left, an upper bound of the
// final one — completes every pair; rounds 0 and 1 list hypotheses up to cap0 (default 64) and cap1 (default
// 256, as far as the side stream draws ahead) per pair (bounded speculation: a chunk a later replay
// finds unneeded is wasted work, never a different result).
// The same best model, inlier count and iteration count as the sequential loop over the same
// models.  ess_final_kernel writes E (kept with the record, or re-solved from its sample) and the
// mask.
constexpr int kSpecHyps = 64;      // round 0 lists hypotheses up to cap0 (default kSpecHyps; round 1: cap1; last: all)
constexpr int kEssRounds = 3;
constexpr int kRecE = 16;          // records per chunk whose E is kept (later ones: re-solved)
constexpr int kEssFive = 1, kEssDone = 2;

struct EssState {
    uint64_t rng;
    int n, flags, niters, maxgood;
    int gen_upto, eval_upto, rc, cur_k;   // samples drawn, hypotheses listed, replay cursor (chunk, hyp)
    int kp, best_c, best_i, best_k, best_m, last;
    int solve_upto;   // hypotheses below this are solved (the listing target; samples may run ahead)
};

struct EssBufs {
    EssState* st;
    int* samp;       // [P][hcap][5]
    int2* rec;       // [P][cmax][ch * kMaxModels]: {count, h * 16 + m}
    int* nrec;       // [P][cmax]
    double* recE;    // [P][cmax][kRecE][9]
    int2* list;      // [kEssRounds][P * cmax]: {pair, chunk (-1: the n == 5 call)}
    int* ctr;        // [2 kEssRounds]: (count, head) per round
    int cmax, hcap, rece;
    int ch;          // hypotheses per chunk (16-lane groups of the chunk kernel)
    int cap0, cap1;  // rounds 0 and 1 list hypotheses up to min(niters, cap)
    uint64_t* spec_rng;   // [P]: the side stream's pre-drawn samples run to spec_upto with this state
    int* spec_upto;       // [P]
};

// One lane per pair: draws samples [gen_upto, target) exactly as essential_ransac_kernel's lane 0
// does (5 distinct indices per sample, redrawing duplicates), then lists the chunks covering them.
__device__ void ess_gen(EssState& s, int p, int P, int round, const EssBufs& B) {
    int2* list = B.list + (size_t)round * P * B.cmax;
    int* cnt = B.ctr + 2 * round;
    const int target = round == 0 ? min(s.niters, B.cap0) : round + 1 < kEssRounds ? min(s.niters, B.cap1) : s.niters;
    if (round > 0 && B.spec_upto && B.spec_upto[p] > s.gen_upto) {   // samples drawn ahead (ess_pregen_kernel)
        s.gen_upto = B.spec_upto[p];
        s.rng = B.spec_rng[p];
    }
    s.solve_upto = target;
    const unsigned n = (unsigned)s.n;
    uint64_t rs = s.rng;
    int* smp = B.samp + (size_t)p * B.hcap * 5;
    const unsigned mg = (unsigned)((1ULL << 32) / n);   // n > 5
    for (int k = s.gen_upto; k < target; ++k) {
        int d[5];
        cv_rng_sample5(rs, n, mg, d);
#pragma unroll
        for (int i = 0; i < 5; ++i) smp[5 * k + i] = d[i];
    }
    if (target > s.gen_upto) {
        s.gen_upto = target;
        s.rng = rs;
    }
    const int c0 = s.eval_upto / B.ch, c1 = (target + B.ch - 1) / B.ch;
    if (c1 > c0) {
        const int base = atomicAdd(cnt, c1 - c0);
        for (int c = c0; c < c1; ++c) list[base + c - c0] = make_int2(p, c);
        s.eval_upto = c1 * B.ch;
    }
}

// Side stream, beside round 0's chunk kernel: each pair's samples drawn ahead from where round 0's
// stopped up to min(niters, kPreHyps), into the sample table past what round 0 solves, with the
// state they leave in spec_rng / spec_upto (the pair state itself is left alone: round 0 reads
// it).  The draws do not depend on any model, so round 1's replay only adopts them (ess_gen).
constexpr int kPreHyps = 256;
__global__ __launch_bounds__(64) void ess_pregen_kernel(int P, EssBufs B) {
    const int p = blockIdx.x * 64 + threadIdx.x;
    if (p >= P) return;
    const EssState s = B.st[p];
    int upto = s.gen_upto;
    uint64_t rng = s.rng;
    if (!(s.flags & (kEssFive | kEssDone))) {
        const unsigned n = (unsigned)s.n;
        const unsigned mg = (unsigned)((1ULL << 32) / n);   // n > 5
        int* smp = B.samp + (size_t)p * B.hcap * 5;
        const int target = min(min(s.niters, kPreHyps), B.hcap);
        for (; upto < target; ++upto) {
            int d[5];
            cv_rng_sample5(rng, n, mg, d);
#pragma unroll
            for (int i = 0; i < 5; ++i) smp[5 * upto + i] = d[i];
        }
    }
    B.spec_rng[p] = rng;
    B.spec_upto[p] = upto;
}

__global__ __launch_bounds__(256) void ess_init_kernel(const double* __restrict__ pts0, const double* __restrict__ pts1,
                                                       const int64_t* __restrict__ offs, const double* __restrict__ cam,
                                                       int max_iters, double* __restrict__ qn, uint8_t* __restrict__ mask,
                                                       int32_t* __restrict__ nmodels_out,
                                                       int32_t* __restrict__ ninl_out, int32_t* __restrict__ iters_out,
                                                       int P, EssBufs B) {
    const int p = blockIdx.x, tid = threadIdx.x;
    const int64_t off = offs[p];
    const int n = (int)(offs[p + 1] - off);
    const double fx = cam[4 * p], fy = cam[4 * p + 1], cx = cam[4 * p + 2], cy = cam[4 * p + 3];
    double* q = qn + off * 4;
    for (int i = tid; i < n; i += 256) {
        q[4 * i + 0] = (pts0[2 * (off + i)] - cx) / fx;
        q[4 * i + 1] = (pts0[2 * (off + i) + 1] - cy) / fy;
        q[4 * i + 2] = (pts1[2 * (off + i)] - cx) / fx;
        q[4 * i + 3] = (pts1[2 * (off + i) + 1] - cy) / fy;
        mask[off + i] = 0;
    }
    if (tid == 0) {
        EssState s;
        s.rng = ~0ULL;
        s.n = n;
        s.flags = n < 5 ? kEssDone : n == 5 ? kEssFive : 0;
        s.niters = max(max_iters, 1);
        s.maxgood = 0;
        s.gen_upto = s.eval_upto = s.rc = 0;
        s.cur_k = s.kp = -1;
        s.best_c = s.best_i = s.best_k = s.best_m = -1;
        s.last = -1;
        s.solve_upto = 0;
        if (n < 5) { nmodels_out[p] = 0; ninl_out[p] = 0; iters_out[p] = 0; }
        if (n == 5) B.list[atomicAdd(B.ctr, 1)] = make_int2(p, -1);   // the one kernel call on all points
        if (n > 5) ess_gen(s, p, P, 0, B);                               // round 0's samples and items
        B.st[p] = s;
    }
}

// Persistent: each workgroup takes items until the list is exhausted (the count is final: the
// list was written by the previous launch), so every wave reaches the exit.
template <int NT>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(2))) void ess_chunk_kernel(int P, int round, const int64_t* __restrict__ offs,
                                                              const double* __restrict__ cam, double threshold,
                                                              const double* __restrict__ qn,
                                                              double* __restrict__ E_out,
                                                              int32_t* __restrict__ nmodels_out,
                                                              uint8_t* __restrict__ mask,
                                                              int32_t* __restrict__ ninl_out,
                                                              int32_t* __restrict__ iters_out, EssBufs B) {
    constexpr int CH = NT / kGL, NW = NT / 64;
    __shared__ double s_grp[CH * kGS];
    __shared__ double s_models[CH * kMaxModels * 9];
    __shared__ float s_models32[CH * kMaxModels * 9];   // f32 copies for the packed pre-test
    __shared__ int s_nmod[CH];
    __shared__ int s_cnt[CH * kMaxModels][NW];
    __shared__ int s_list[CH * kMaxModels];
    __shared__ int s_good[CH * kMaxModels];
    __shared__ int s_act[CH * kMaxModels];
    __shared__ int s_nlist, s_item, s_nact;
    const int tid = threadIdx.x, lane = tid & 63;
    const int h = tid / kGL, gl = tid % kGL, gsh = (lane / kGL) * kGL;
    const int2* list = B.list + (size_t)round * P * B.cmax;
    const int count = B.ctr[2 * round];
    for (;;) {
        if (tid == 0) s_item = atomicAdd(B.ctr + 2 * round + 1, 1);
        __syncthreads();
        const int it = s_item;
        if (it >= count) break;
        const int2 item = list[it];
        const int p = item.x, c = item.y;
        const int64_t off = offs[p];
        const int n = (int)(offs[p + 1] - off);
        const double* q = qn + off * 4;
        if (c < 0) {   // count == modelPoints: one kernel call on all points, mask all ones
            if (h == 0) {
                double qq[5][4];
#pragma unroll
                for (int j = 0; j < 5; ++j)
#pragma unroll
                    for (int cc = 0; cc < 4; ++cc) qq[j][cc] = q[4 * j + cc];
                const int nm = five_point_group(qq, gl, gsh, s_grp, s_models);
                if (gl == 0) {
                    double* Eo = E_out + (int64_t)p * kMaxModels * 9;
                    for (int e = 0; e < nm * 9; ++e) Eo[e] = s_models[e];
                    nmodels_out[p] = nm;
                    ninl_out[p] = nm > 0 ? 5 : 0;
                    iters_out[p] = 1;
                    for (int i = 0; i < 5; ++i) mask[off + i] = nm > 0 ? 1 : 0;
                }
            }
            __syncthreads();
            continue;
        }
        const double fx = cam[4 * p], fy = cam[4 * p + 1];
        const double thresh = threshold / ((fx + fy) / 2);
        const float tf = (float)(thresh * thresh);
        const float tfu = nextafterf(tf, INFINITY);
        const double mid = 0.5 * ((double)tf + (double)tfu);
        const double Tmax = ((__float_as_uint(tf) & 1u) == 0u) ? mid : nextafter(mid, 0.0);
        const double tlo = Tmax * (1.0 - 0x1p-40), thi = Tmax * (1.0 + 0x1p-40);
        const int gen = B.st[p].solve_upto;
        const int k = c * CH + h;
        RPROF_INIT;
        PROF_COUNT(14, 1);
        for (int i = tid; i < CH * kMaxModels * NW; i += NT) (&s_cnt[0][0])[i] = 0;
        {
            int nm = 0;
            if (k < gen) {
                const int* smp = B.samp + ((size_t)p * B.hcap + k) * 5;
                double qq[5][4];
#pragma unroll
                for (int j = 0; j < 5; ++j) {
                    const int idx = smp[j];
#pragma unroll
                    for (int cc = 0; cc < 4; ++cc) qq[j][cc] = q[4 * idx + cc];
                }
                nm = five_point_group(qq, gl, gsh, s_grp + h * kGS, s_models + h * kMaxModels * 9);
            }
            if (gl == 0) s_nmod[h] = nm;
        }
        __syncthreads();
        if (tid == 0) {
            int cn = 0;
            for (int hh = 0; hh < CH; ++hh)
                for (int m = 0; m < s_nmod[hh]; ++m) s_list[cn++] = hh * kMaxModels + m;
            s_nlist = cn;
        }
        for (int e = tid; e < CH * kMaxModels * 9; e += NT) s_models32[e] = (float)s_models[e];
        __syncthreads();
        const int nlist = s_nlist;
        RPROF(9, tp);
        auto score = [&](const int* lst, int nl, int lo, int hi) {
            score_chunk_f32<NT>(q, n, lst, nl, s_models, s_models32, s_cnt, tf, Tmax, tlo, thi, tid, lo, hi);
        };
        // Rounds >= 1: every model of this chunk is replayed after the previous rounds' replays, so
        // one whose count cannot exceed max(their best, 4) never replaces the best and need not be
        // counted exactly: after the first block of points, models whose count plus the points left
        // is at most that bound drop out (s_good = -1: never a record; a later model it would have
        // shadowed is recorded instead and rejected by the replay's own test).
        const int bound = round > 0 ? max(B.st[p].maxgood, 4) : 4;
        constexpr int blk = NT * kPB;
        if (bound > 4 && n > blk && n - blk < bound) {
            score(s_list, nlist, 0, blk);
            __syncthreads();
            if (tid < 64) {   // wave 0: compact the live models (order kept) into s_act
                int na = 0;
                for (int b0 = 0; b0 < nlist; b0 += 64) {
                    const int e = b0 + tid;
                    bool live = false;
                    if (e < nlist) {
                        int g = 0;
#pragma unroll
                        for (int w = 0; w < NW; ++w) g += s_cnt[s_list[e]][w];
                        live = g + (n - blk) > bound;
                        s_good[e] = live ? 0 : -1;
                    }
                    const unsigned long long bm = __ballot(live);
                    if (live) s_act[na + __popcll(bm & ((1ULL << tid) - 1ULL))] = s_list[e];
                    na += __popcll(bm);
                }
                if (tid == 0) s_nact = na;
            }
            __syncthreads();
            score(s_act, s_nact, blk, INT_MAX);
            __syncthreads();
            for (int e = tid; e < nlist; e += NT) {
                if (s_good[e] < 0) continue;
                int g = 0;
#pragma unroll
                for (int w = 0; w < NW; ++w) g += s_cnt[s_list[e]][w];
                s_good[e] = g;
            }
        } else {
            score(s_list, nlist, 0, INT_MAX);
            __syncthreads();
            for (int e = tid; e < nlist; e += NT) {
                int g = 0;
#pragma unroll
                for (int w = 0; w < NW; ++w) g += s_cnt[s_list[e]][w];
                s_good[e] = g;
            }
        }
        __syncthreads();
        RPROF(10, tp);
        if (tid < 64) {   // records: strict prefix maxima above 4, by a running max over 64-entry blocks
            int2* rec = B.rec + ((size_t)p * B.cmax + c) * (CH * kMaxModels);
            double* recE = B.recE + ((size_t)p * B.cmax + c) * kRecE * 9;
            int carry = 4, nr = 0;
            for (int b0 = 0; b0 < nlist; b0 += 64) {
                const int e = b0 + lane;
                const int g = e < nlist ? s_good[e] : -1;
                int pm = g;   // inclusive prefix max
#pragma unroll
                for (int o = 1; o < 64; o <<= 1) {
                    const int t = __shfl_up(pm, o);
                    if (lane >= o) pm = max(pm, t);
                }
                int ex = __shfl_up(pm, 1);
                ex = lane == 0 ? carry : max(carry, ex);
                const bool isr = e < nlist && g > ex;
                const unsigned long long bm = __ballot(isr);
                if (isr) {
                    const int r = nr + __popcll(bm & ((1ULL << lane) - 1ULL));
                    const int code = s_list[e];
                    const int hh = code / kMaxModels, m = code % kMaxModels;
                    rec[r] = make_int2(g, hh * 16 + m);
                    if (r < B.rece)
                        for (int q9 = 0; q9 < 9; ++q9) recE[r * 9 + q9] = s_models[code * 9 + q9];
                }
                nr += __popcll(bm);
                carry = max(carry, __shfl(pm, 63));
            }
            if (lane == 0) B.nrec[(size_t)p * B.cmax + c] = nr;
        }
        __syncthreads();
    }
}

// One wave per pair: the records of the listed chunks in order (essential_ransac_kernel's replay),
// then, unless the pair is complete, the next round's samples and work items (lane 0).  The lanes
// first stage a window of chunks' records in LDS — lane t loads chunk t's count and then its
// records, all loads independent — so lane 0's replay waits on memory once per window, not once
// per record.
constexpr int kRpCap = 2048;   // records staged per window
__global__ __launch_bounds__(64) void ess_replay_kernel(int P, int round, double prob, EssBufs B) {
    __shared__ int2 s_rec[kRpCap];
    __shared__ int s_off[65], s_cnt[64];
    const int p = blockIdx.x, lane = threadIdx.x;
    EssState s = B.st[p];
    if (s.flags & (kEssFive | kEssDone)) return;   // uniform
    const int recmax = B.ch * kMaxModels;
    int nit = s.niters;
    bool done = false;
    int c = s.rc;
    const int cend = s.eval_upto / B.ch;
    while (c < cend && !done) {   // uniform: done is broadcast below
        const int t_n = c + lane < cend ? B.nrec[(size_t)p * B.cmax + c + lane] : 0;
        int pre = t_n;   // inclusive scan
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int t = __shfl_up(pre, d);
            if (lane >= d) pre += t;
        }
        // window: the leading chunks whose records fit (a chunk holds at most recmax <= kRpCap)
        const unsigned long long fit = __ballot(c + lane < cend && pre <= kRpCap);
        const int nwin = __popcll(fit);   // fit is a prefix of the lanes (pre grows with lane)
        if (lane < nwin) {
            const int2* rec = B.rec + ((size_t)p * B.cmax + c + lane) * recmax;
            for (int i = 0; i < t_n; ++i) s_rec[pre - t_n + i] = rec[i];
            s_off[lane] = pre - t_n;
            s_cnt[lane] = t_n;
        }
        __syncthreads();
        if (lane == 0) {
            int w = 0;
            for (; w < nwin && !done; ++w) {
                const int cc = c + w;
                for (int i = 0; i < s_cnt[w]; ++i) {
                    const int2 r = s_rec[s_off[w] + i];
                    const int k = cc * B.ch + (r.y >> 4), m = r.y & 15;
                    if (k != s.cur_k) {
                        if (k >= nit) { done = true; break; }
                        s.cur_k = k;
                    }
                    s.kp = k;
                    if (r.x > max(s.maxgood, 4)) {
                        s.maxgood = r.x;
                        s.best_c = cc;
                        s.best_i = i;
                        s.best_k = k;
                        s.best_m = m;
                        nit = update_num_iters(prob, (double)(s.n - r.x) / s.n, 5, nit);
                    }
                }
            }
            s_off[64] = (done ? 1 : 0) | (w << 1);
        }
        __syncthreads();
        done = s_off[64] & 1;
        c += done ? (s_off[64] >> 1) : nwin;
        __syncthreads();
    }
    if (lane != 0) return;
    s.rc = c;
    s.niters = nit;
    if (done || nit <= s.eval_upto) {
        s.flags |= kEssDone;
        s.last = max(nit, s.kp + 1) - 1;
    } else if (round + 1 < kEssRounds) {
        ess_gen(s, p, P, round + 1, B);
    }
    B.st[p] = s;
}

__global__ __launch_bounds__(256) void ess_final_kernel(const int64_t* __restrict__ offs,
                                                        const double* __restrict__ cam, double threshold,
                                                        const double* __restrict__ qn, double* __restrict__ E_out,
                                                        int32_t* __restrict__ nmodels_out,
                                                        uint8_t* __restrict__ mask, int32_t* __restrict__ ninl_out,
                                                        int32_t* __restrict__ iters_out, EssBufs B) {
    __shared__ double s_grp[kGS];
    __shared__ double s_models[kMaxModels * 9];
    __shared__ double s_E[9];
    const int p = blockIdx.x, tid = threadIdx.x;
    const EssState s = B.st[p];
    if (s.n <= 5) return;   // n < 5: written by ess_init_kernel; n == 5: by ess_chunk_kernel
    const int64_t off = offs[p];
    const int n = s.n;
    const double* q = qn + off * 4;
    const int maxgood = s.maxgood;
    if (maxgood > 0) {
        if (s.best_i < B.rece) {
            if (tid < 9) s_E[tid] = B.recE[(((size_t)p * B.cmax + s.best_c) * kRecE + s.best_i) * 9 + tid];
        } else if (tid < kGL) {   // the record's E was not kept: re-solve its sample (the same bits)
            const int* smp = B.samp + ((size_t)p * B.hcap + s.best_k) * 5;
            double qq[5][4];
#pragma unroll
            for (int j = 0; j < 5; ++j) {
                const int idx = smp[j];
#pragma unroll
                for (int cc = 0; cc < 4; ++cc) qq[j][cc] = q[4 * idx + cc];
            }
            five_point_group(qq, tid, 0, s_grp, s_models);
            wave_sync_lds();
            if (tid < 9) s_E[tid] = s_models[s.best_m * 9 + tid];
        }
    }
    __syncthreads();
    if (tid == 0) {
        nmodels_out[p] = maxgood > 0 ? 1 : 0;
        ninl_out[p] = maxgood;
        iters_out[p] = s.last + 1;
        if (maxgood > 0)
            for (int e = 0; e < 9; ++e) E_out[(int64_t)p * kMaxModels * 9 + e] = s_E[e];
    }
    if (maxgood > 0) {
        const double fx = cam[4 * p], fy = cam[4 * p + 1];
        const double thresh = threshold / ((fx + fy) / 2);
        const float tf = (float)(thresh * thresh);
        for (int i = tid; i < n; i += 256)
            mask[off + i] = sampson(s_E, q[4 * i], q[4 * i + 1], q[4 * i + 2], q[4 * i + 3]) <= tf ? 1 : 0;
    }
}

// cv::decomposeEssentialMat: SVD by one-sided Jacobi on E's columns, U's third
// column = u1 x u2 (det U = +1); Vt negated when det(Vt) < 0.
__device__ void decompose_essential(const double* E, double* R1, double* R2, double* t) {
    double A[3][3], V[3][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}};  // A[col][row], V[col][row]
    for (int c = 0; c < 3; ++c)
        for (int r = 0; r < 3; ++r) A[c][r] = E[3 * r + c];
    for (int sweep = 0; sweep < 40; ++sweep) {
        bool rotated = false;
        for (int pc = 0; pc < 2; ++pc)
            for (int qc = pc + 1; qc < 3; ++qc) {
                double al = 0, be = 0, ga = 0;
                for (int r = 0; r < 3; ++r) {
                    al += A[pc][r] * A[pc][r];
                    be += A[qc][r] * A[qc][r];
                    ga += A[pc][r] * A[qc][r];
                }
                if (ga == 0.0 || fabs(ga) <= 1e-15 * sqrt(al * be)) continue;
                rotated = true;
                const double zeta = (be - al) / (2.0 * ga);
                const double tt = (zeta >= 0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
                const double c = 1.0 / sqrt(1.0 + tt * tt), s = c * tt;
                for (int r = 0; r < 3; ++r) {
                    const double ap = A[pc][r], aq = A[qc][r];
                    A[pc][r] = c * ap - s * aq;
                    A[qc][r] = s * ap + c * aq;
                    const double vp = V[pc][r], vq = V[qc][r];
                    V[pc][r] = c * vp - s * vq;
                    V[qc][r] = s * vp + c * vq;
                }
            }
        if (!rotated) break;
    }
    double sg[3];
    int ord[3] = {0, 1, 2};
    for (int c = 0; c < 3; ++c) sg[c] = sqrt(A[c][0] * A[c][0] + A[c][1] * A[c][1] + A[c][2] * A[c][2]);
    for (int i = 0; i < 2; ++i)
        for (int j = 0; j < 2 - i; ++j)
            if (sg[ord[j]] < sg[ord[j + 1]]) { const int t2 = ord[j]; ord[j] = ord[j + 1]; ord[j + 1] = t2; }
    double U[3][3], Vs[3][3];  // [col][row]
    for (int c = 0; c < 2; ++c)
        for (int r = 0; r < 3; ++r) U[c][r] = A[ord[c]][r] / sg[ord[c]];
    U[2][0] = U[0][1] * U[1][2] - U[0][2] * U[1][1];
    U[2][1] = U[0][2] * U[1][0] - U[0][0] * U[1][2];
    U[2][2] = U[0][0] * U[1][1] - U[0][1] * U[1][0];
    const double un = sqrt(U[2][0] * U[2][0] + U[2][1] * U[2][1] + U[2][2] * U[2][2]);
    for (int r = 0; r < 3; ++r) U[2][r] /= un;
    for (int c = 0; c < 3; ++c)
        for (int r = 0; r < 3; ++r) Vs[c][r] = V[ord[c]][r];
    const double detV = Vs[0][0] * (Vs[1][1] * Vs[2][2] - Vs[1][2] * Vs[2][1]) -
                        Vs[1][0] * (Vs[0][1] * Vs[2][2] - Vs[0][2] * Vs[2][1]) +
                        Vs[2][0] * (Vs[0][1] * Vs[1][2] - Vs[0][2] * Vs[1][1]);
    if (detV < 0)
        for (int c = 0; c < 3; ++c)
            for (int r = 0; r < 3; ++r) Vs[c][r] = -Vs[c][r];
    // R1 = U W Vt, R2 = U W^T Vt with W = [[0,1,0],[-1,0,0],[0,0,1]]:
    // U W = [-u2, u1, u3], U W^T = [u2, -u1, u3]; (X Vt)[r][c] = sum_k X[k][r] * V[k][c]
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) {
            R1[3 * r + c] = (-U[1][r] * Vs[0][c] + U[0][r] * Vs[1][c]) + U[2][r] * Vs[2][c];
            R2[3 * r + c] = (U[1][r] * Vs[0][c] - U[0][r] * Vs[1][c]) + U[2][r] * Vs[2][c];
        }
    for (int r = 0; r < 3; ++r) t[r] = U[2][r];
}

// cv::recoverPose (distanceThresh variant): cheirality of the DLT
// triangulation for the 4 candidate poses; best count wins, ties in the
// order (R1,t), (R2,t), (R1,-t), (R2,-t).
__global__ __launch_bounds__(kPThreads) void recover_pose_kernel(
    const double* __restrict__ Ein, int64_t e_stride, const double* __restrict__ pts0,
    const double* __restrict__ pts1, const int64_t* __restrict__ offs, const double* __restrict__ cam,
    const uint8_t* __restrict__ mask_in, double dist, double* __restrict__ R_out, double* __restrict__ t_out,
    uint8_t* __restrict__ mask_out, int32_t* __restrict__ good_out) {
    __shared__ double sP[4][12];
    __shared__ double sPP[4][24];   // [P0 | P_k] contiguous, for dlt_point_normal
    __shared__ int s_cnt[4];
    __shared__ int s_sel;
    const int p = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
    const int64_t off = offs[p];
    const int n = (int)(offs[p + 1] - off);
    if (tid == 0) {
        double R1[9], R2[9], t[3];
        decompose_essential(Ein + (int64_t)p * e_stride, R1, R2, t);
        for (int k = 0; k < 4; ++k) {
            const double* R = (k & 1) ? R2 : R1;
            const double sg = (k & 2) ? -1.0 : 1.0;
            for (int r = 0; r < 3; ++r) {
                for (int c = 0; c < 3; ++c) sP[k][4 * r + c] = R[3 * r + c];
                sP[k][4 * r + 3] = sg * t[r];
            }
            for (int e = 0; e < 12; ++e) {
                sPP[k][e] = (e % 5 == 0) ? 1.0 : 0.0;   // [I | 0]
                sPP[k][12 + e] = sP[k][e];
            }
            s_cnt[k] = 0;
        }
    }
    __syncthreads();
    const double fx = cam[4 * p], fy = cam[4 * p + 1], cx = cam[4 * p + 2], cy = cam[4 * p + 3];
    const double P0[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0};
    for (int i0 = 0; i0 < n; i0 += kPThreads) {
        const int i = i0 + tid;
        int code = 0;
        if (i < n && (!mask_in || mask_in[off + i])) {
            const double x1 = (pts0[2 * (off + i)] - cx) / fx, y1 = (pts0[2 * (off + i) + 1] - cy) / fy;
            const double x2 = (pts1[2 * (off + i)] - cx) / fx, y2 = (pts1[2 * (off + i) + 1] - cy) / fy;
            for (int k = 0; k < 4; ++k) {
                const double* P = sP[k];
                auto test = [&](const double* Q, bool& ok, double& scale) {
                    ok = Q[2] * Q[3] > 0;
                    const double X = Q[0] / Q[3], Y = Q[1] / Q[3], Z = Q[2] / Q[3], W = Q[3] / Q[3];
                    ok = ok && Z < dist;
                    const double z2 = ((P[8] * X + P[9] * Y) + P[10] * Z) + P[11] * W;
                    ok = ok && z2 > 0 && z2 < dist;
                    // distance of every tested quantity from its decision boundary, relative to
                    // what a 1e-6 change of the unit null vector could move it
                    const double aq3 = fabs(Q[3]);
                    const double m = 4e-6 * (1.0 + fabs(X) + fabs(Y) + fabs(Z)) / fmax(aq3, 1e-300) *
                                     (1.0 + fabs(P[8]) + fabs(P[9]) + fabs(P[10]) + fabs(P[11]));
                    scale = fmin(fmin(fmin(fabs(Q[2]), aq3) * 1e6, fmin(fabs(Z), fabs(Z - dist)) / m),
                                 fmin(fabs(z2), fabs(z2 - dist)) / m);
                };
                // the normal-equation fast path (geom_dev.h dlt_point_normal: null vector within
                // ~1e-9 of the SVD's when it decides); dlt_point where it cannot decide or where a
                // cheirality test lies within the fast path's error bound of its boundary, so the
                // decisions are dlt_point's
                double Q[4];
                bool ok = false, sure = false;
                if (dlt_point_normal(sPP[k], x1, y1, x2, y2, Q) == 0) {
                    double sc;
                    test(Q, ok, sc);
                    sure = sc > 1.0;
                }
                if (!sure) {
                    double sc;
                    dlt_point(P0, P, x1, y1, x2, y2, Q);
                    test(Q, ok, sc);
                }
                code |= ok ? (1 << k) : 0;
            }
        }
        for (int k = 0; k < 4; ++k) {
            const int c = wave_count((code >> k) & 1);
            if (lane == 0 && c) atomicAdd(&s_cnt[k], c);
        }
        if (i < n) mask_out[off + i] = (uint8_t)code;
    }
    __syncthreads();
    if (tid == 0) {
        int sel = 3;
        for (int k = 0; k < 4; ++k) {
            bool best = true;
            for (int o = 0; o < 4; ++o) best = best && s_cnt[k] >= s_cnt[o];
            if (best) { sel = k; break; }
        }
        s_sel = sel;
        good_out[p] = s_cnt[sel];
        for (int r = 0; r < 3; ++r) {
            for (int c = 0; c < 3; ++c) R_out[9 * p + 3 * r + c] = sP[sel][4 * r + c];
            t_out[3 * p + r] = sP[sel][4 * r + 3];
        }
    }
    __syncthreads();
    const int sel = s_sel;
    for (int i = tid; i < n; i += kPThreads) mask_out[off + i] = ((mask_out[off + i] >> sel) & 1) ? 255 : 0;
}

}  // namespace
}  // namespace sfmhip

using namespace sfmhip;

#ifdef SFMHIP_RANSAC_PROF
// Phase timers of essential_ransac_kernel for tools/prof_ransac.py: exported only
// by a profiling build (make EXTRA=-DSFMHIP_RANSAC_PROF), not part of the ABI.
extern "C" int sfmhip_debug_ransac_prof(unsigned long long* out) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_rprof), sizeof(unsigned long long) * 16) != hipSuccess) return -2;
    unsigned long long z[16] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_rprof), z, sizeof(z)) != hipSuccess) return -2;
    return 0;
}
#endif

// Library-owned side stream per device for ess_pregen_kernel (created once; events fork it from
// and join it to the caller's stream, so the call stays ordered on that stream).  The mutex keeps
// one fork/join sequence at a time per device.
struct EssSide {
    hipStream_t s = nullptr;
    hipEvent_t fork = nullptr, join = nullptr;
    std::mutex mu;
};
static EssSide g_ess_side[64];
static std::once_flag g_ess_side_once[64];
static EssSide* ess_side(int dev) {
    if (dev < 0 || dev >= 64) return nullptr;
    std::call_once(g_ess_side_once[dev], [dev] {
        EssSide& e = g_ess_side[dev];
        if (hipStreamCreateWithFlags(&e.s, hipStreamNonBlocking) != hipSuccess ||
            hipEventCreateWithFlags(&e.fork, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&e.join, hipEventDisableTiming) != hipSuccess)
            e.s = nullptr;
        (void)hipGetLastError();
    });
    return g_ess_side[dev].s ? &g_ess_side[dev] : nullptr;
}

extern "C" int sfmhip_find_essential(const double* pts0, const double* pts1, const int64_t* offsets,
                                     int n_pairs, const double* cam, double prob, double threshold,
                                     int max_iters, double* work, double* E, int32_t* n_models,
                                     uint8_t* mask, int32_t* n_inliers, int32_t* iters, void* stream) {
    SFMHIP_REQUIRE(n_pairs >= 0, "find_essential: n_pairs < 0");
    if (n_pairs == 0) return SFMHIP_OK;
    SFMHIP_REQUIRE(pts0 && pts1 && offsets && cam && work && E && n_models && mask && n_inliers && iters,
                   "find_essential: null pointer");
    SFMHIP_REQUIRE(prob >= 0 && prob <= 1 && threshold > 0, "find_essential: prob in [0,1], threshold > 0");
    hipStream_t st = as_stream(stream);
    if (knobs().ess_mono) {   // the one-workgroup-per-pair kernel (tests: the balanced form's reference)
        hipLaunchKernelGGL(essential_ransac_kernel, dim3(n_pairs), dim3(kRThreads), 0, st, pts0, pts1, offsets, cam,
                           prob, threshold, max_iters, work, E, n_models, mask, n_inliers, iters);
        return check_launch("essential_ransac_kernel");
    }
    // load-balanced form: per-pair scratch, pairs in batches of at most ~192 MB of it.  Chunk
    // kernel: 256 threads (16 hypotheses per item, two workgroups per CU so one's scoring overlaps
    // the other's solve; 512 threads, 32 per item, measured slower), packed-f32 Sampson pre-test
    // with certified bounds (f64 throughout measured slower: 1.065 vs 0.98 ms)
    constexpr int ct = 256;
    const int ch = ct / kGL, recmax = ch * kMaxModels;
    const int cmax = ceil_div(std::max(max_iters, 1), ch), hcap = cmax * ch;
    auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
    const size_t per_pair = sizeof(EssState) + (size_t)hcap * 5 * sizeof(int) + (size_t)cmax * recmax * sizeof(int2) +
                            (size_t)cmax * sizeof(int) + (size_t)cmax * kRecE * 9 * sizeof(double) +
                            kEssRounds * (size_t)cmax * sizeof(int2);
    const int batch = (int)std::max<int64_t>(1, std::min<int64_t>(n_pairs, ((size_t)192 << 20) / per_pair));
    const size_t bytes = al(batch * sizeof(EssState)) + al((size_t)batch * hcap * 5 * sizeof(int)) +
                         al((size_t)batch * cmax * recmax * sizeof(int2)) + al((size_t)batch * cmax * sizeof(int)) +
                         al((size_t)batch * cmax * kRecE * 9 * sizeof(double)) +
                         al(kEssRounds * (size_t)batch * cmax * sizeof(int2)) + al(2 * kEssRounds * sizeof(int)) +
                         al(batch * sizeof(uint64_t)) + al(batch * sizeof(int));
    char* base = nullptr;
    if (scratch_alloc((void**)&base, bytes, st) != hipSuccess) {
        (void)hipGetLastError();
        set_error("find_essential: scratch allocation of %zu bytes failed", bytes);
        return SFMHIP_E_HIP;
    }
    EssBufs B;
    char* cur = base;
    auto carve = [&](size_t b) { char* r = cur; cur += al(b); return r; };
    B.st = (EssState*)carve(batch * sizeof(EssState));
    B.samp = (int*)carve((size_t)batch * hcap * 5 * sizeof(int));
    B.rec = (int2*)carve((size_t)batch * cmax * recmax * sizeof(int2));
    B.nrec = (int*)carve((size_t)batch * cmax * sizeof(int));
    B.recE = (double*)carve((size_t)batch * cmax * kRecE * 9 * sizeof(double));
    B.list = (int2*)carve(kEssRounds * (size_t)batch * cmax * sizeof(int2));
    B.ctr = (int*)carve(2 * kEssRounds * sizeof(int));
    B.spec_rng = (uint64_t*)carve(batch * sizeof(uint64_t));
    B.spec_upto = (int*)carve(batch * sizeof(int));
    B.cmax = cmax;
    B.hcap = hcap;
    B.ch = ch;
    // samples drawn ahead on a side stream while round 0 runs
    int dev = -1;
    EssSide* side = hipGetDevice(&dev) == hipSuccess ? ess_side(dev) : nullptr;
    (void)hipGetLastError();
    std::unique_lock<std::mutex> side_lock;
    if (side) side_lock = std::unique_lock<std::mutex>(side->mu);
    else B.spec_upto = nullptr;
    // records whose E is kept (SFMHIP_ESS_RECE, tests: 0 re-solves every chosen model from its sample)
    B.rece = std::min(kRecE, std::max(0, knobs().ess_rece));
    // speculation caps: round 0 (kSpecHyps; 32/48/96 measured no faster) and round 1 (the pre-drawn
    // samples' reach), so round 1 is the last round a pair needs unless its niters exceeds kPreHyps.
    // Whole chunks: a listed chunk counts as evaluated, and the chunk kernel solves only below the
    // listing target, so a target short of niters must end a chunk
    B.cap0 = ceil_div(kSpecHyps, ch) * ch;
    B.cap1 = std::max(B.cap0, ceil_div(kPreHyps, ch) * ch);
    int rc = SFMHIP_OK;
    for (int p0 = 0; p0 < n_pairs && rc == SFMHIP_OK; p0 += batch) {
        const int PB = std::min(batch, n_pairs - p0);
        const int64_t* of = offsets + p0;
        const double* cm = cam + 4 * (size_t)p0;
        double* Eb = E + (size_t)p0 * kMaxModels * 9;
        int32_t *nmb = n_models + p0, *nib = n_inliers + p0, *itb = iters + p0;
        (void)hipMemsetAsync(B.ctr, 0, 2 * kEssRounds * sizeof(int), st);
        hipLaunchKernelGGL(ess_init_kernel, dim3(PB), dim3(256), 0, st, pts0, pts1, of, cm, max_iters, work, mask, nmb,
                           nib, itb, PB, B);
        if (side) {   // fork: the side stream draws ahead once the init kernel has run
            (void)hipEventRecord(side->fork, st);
            (void)hipStreamWaitEvent(side->s, side->fork, 0);
            hipLaunchKernelGGL(ess_pregen_kernel, dim3(ceil_div(PB, 64)), dim3(64), 0, side->s, PB, B);
            (void)hipEventRecord(side->join, side->s);
        }
        for (int round = 0; round < kEssRounds; ++round) {
            const int items = round == 0 ? ceil_div(B.cap0, ch) : round + 1 < kEssRounds ? ceil_div(B.cap1, ch) : cmax;
            const int g = (int)std::min<int64_t>(1024, (int64_t)PB * std::min(cmax, items));
            hipLaunchKernelGGL(ess_chunk_kernel<ct>, dim3(g), dim3(ct), 0, st, PB, round, of, cm, threshold, work, Eb,
                               nmb, mask, nib, itb, B);
            if (side && round == 0) (void)hipStreamWaitEvent(st, side->join, 0);   // join before round 1's draws
            hipLaunchKernelGGL(ess_replay_kernel, dim3(PB), dim3(64), 0, st, PB, round, prob, B);
        }
        hipLaunchKernelGGL(ess_final_kernel, dim3(PB), dim3(256), 0, st, of, cm, threshold, work, Eb, nmb, mask, nib,
                           itb, B);
        rc = check_launch("ess_*_kernel");
    }
    scratch_free(base, st);
    return rc;
}

extern "C" int sfmhip_recover_pose(const double* E, int64_t e_stride, const double* pts0, const double* pts1,
                                   const int64_t* offsets, int n_pairs, const double* cam, const uint8_t* mask_in,
                                   double distance_thresh, double* R, double* t, uint8_t* mask_out,
                                   int32_t* n_good, void* stream) {
    SFMHIP_REQUIRE(n_pairs >= 0, "recover_pose: n_pairs < 0");
    if (n_pairs == 0) return SFMHIP_OK;
    SFMHIP_REQUIRE(E && pts0 && pts1 && offsets && cam && R && t && mask_out && n_good,
                   "recover_pose: null pointer");
    SFMHIP_REQUIRE(e_stride >= 9, "recover_pose: e_stride >= 9");
    hipLaunchKernelGGL(recover_pose_kernel, dim3(n_pairs), dim3(kPThreads), 0, as_stream(stream), E, e_stride,
                       pts0, pts1, offsets, cam, mask_in, distance_thresh, R, t, mask_out, n_good);
    return check_launch("recover_pose_kernel");
}
