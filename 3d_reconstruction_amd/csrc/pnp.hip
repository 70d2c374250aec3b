// pnp.hip — SURVEY.md §8f row 2 (last part): cv2.solvePnPRansac at sfm.py:116
//     cv2.solvePnPRansac(X, pts1, K, np.zeros((5, 1)), cv2.SOLVEPNP_ITERATIVE)
// i.e. iterationsCount 100, reprojectionError 8, confidence 0.99, flags
// ITERATIVE (the 5th positional argument is rvec), restated from OpenCV 4.x
// (solvepnp.cpp, epnp.cpp, ptsetreg.cpp, calibration.cpp
// cvFindExtrinsicCameraParams2 + CvLevMarq); CPU restatement oracle/pnp.py.
// Parity with OpenCV is unpinned (cv2 absent).
//
// One workgroup (4 waves) per registration problem:
//   * points are converted to float (solvePnPRansac's CV_32F conversion);
//   * RANSAC: lane 0 draws 32 five-point samples per chunk from cv::RNG(-1)
//     (OpenCV's ~25 iterations at 30 % outliers fit one chunk);
//     each sample is solved by EPnP in an 8-lane group (M^T M eigenvectors by
//     a parallel-ordered two-sided Jacobi in LDS, the three beta
//     approximations + Gauss-Newton in lanes 0..2, Procrustes), scored by all
//     lanes (float squared reprojection error <= 64, wave ballots) and
//     replayed in OpenCV's sequential order;
//   * the RANSAC pose is refined on the inliers by Levenberg-Marquardt with
//     CvLevMarq's control flow; J^T J / J^T e are block reductions in a fixed
//     order, the 6x6 damped system is solved by thread 0.
#include <algorithm>
#include <cstdlib>

#include "common.h"
#include "geom_dev.h"

namespace sfmhip {
namespace {

constexpr int kPnThreads = 256;
constexpr int kPnGL = 8;                   // lanes per EPnP group
constexpr int kPnH = kPnThreads / kPnGL;  // hypotheses per chunk
constexpr int kJcN = 144 / kPnGL;          // convergence-check elements per lane
constexpr int kJbN = (36 + kPnGL - 1) / kPnGL;  // 2x2 rotation blocks per lane
static_assert(144 % kPnGL == 0 && kPnGL >= 6, "EPnP group width");
constexpr int kPnGS = 448;                // LDS doubles per group
constexpr int kPnStageCap = kPnH * kPnGS * 8 / 21;   // LM points staged in the group scratch (5 floats + a flag)
#ifndef SFMHIP_PNP_FAST_ROT   // 1: measured 0.705 vs 0.713 ms (noise level, profiles/r4/ab_pnp_verify_heavyprobe_r4j.log)
#define SFMHIP_PNP_FAST_ROT 0
#endif
constexpr bool kPnFastRot = SFMHIP_PNP_FAST_ROT != 0;   // EPnP Jacobi rotations without IEEE div / sqrt
constexpr double kEps64 = 2.220446049250313e-16;
constexpr double kDblMin64 = 2.2250738585072014e-308;

// group scratch map (doubles)
constexpr int gA = 0, gV = 144, gRot = 288 /* 6 x (c, s) */, gL = 300, gRho = 360, gSol = 366 /* 3 x 13 */,
              gCws = 405 /* 12 */, gAl = 417 /* 5 x 4 alphas */, gUd = 437 /* 5 x (uc - u, vc - v) */;
static_assert(gUd + 10 <= kPnGS, "group scratch map");

struct CvRng {
    uint64_t s;
    __device__ unsigned next() {
        s = (uint64_t)(unsigned)s * 4164903690ULL + (unsigned)(s >> 32);
        return (unsigned)s;
    }
    __device__ int uniform0(unsigned n, double inv_n) {
        const unsigned x = next();
        unsigned qd = (unsigned)((double)x * inv_n);
        long long r = (long long)x - (long long)qd * n;
        if (r < 0) r += n;
        else if (r >= (long long)n) r -= n;
        return (int)r;
    }
};

__device__ int update_num_iters(double p, double ep, int m, int max_iters) {
    p = fmin(fmax(p, 0.0), 1.0);
    ep = fmin(fmax(ep, 0.0), 1.0);
    double num = fmax(1.0 - p, kDblMin64);
    double denom = 1.0 - pow(1.0 - ep, (double)m);
    if (denom < kDblMin64) return 0;
    num = log(num);
    denom = log(denom);
    return (denom >= 0 || -num >= max_iters * (-denom)) ? max_iters : (int)rint(num / denom);
}

__device__ __forceinline__ void lds_fence() { __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "workgroup"); }

// Symmetric 3x3 eigen-decomposition by cyclic Jacobi: eigenvalues descending,
// rows of E = eigenvectors with the largest-|.| component positive.
__device__ void eig3_desc(double A[3][3], double w[3], double E[3][3]) {
    double V[3][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
    for (int sweep = 0; sweep < 30; ++sweep) {
        const double off = A[0][1] * A[0][1] + A[0][2] * A[0][2] + A[1][2] * A[1][2];
        const double dg = A[0][0] * A[0][0] + A[1][1] * A[1][1] + A[2][2] * A[2][2];
        if (off <= 1e-32 * dg || off == 0.0) break;
        for (int p = 0; p < 2; ++p)
            for (int q = p + 1; q < 3; ++q) {
                if (A[p][q] == 0.0) continue;
                const double tau = (A[q][q] - A[p][p]) / (2.0 * A[p][q]);
                const double t = (tau >= 0 ? 1.0 : -1.0) / (fabs(tau) + sqrt(1.0 + tau * tau));
                const double c = 1.0 / sqrt(1.0 + t * t), s = t * c;
                for (int k = 0; k < 3; ++k) {  // A <- A J (columns p, q)
                    const double ap = A[k][p], aq = A[k][q];
                    A[k][p] = c * ap - s * aq;
                    A[k][q] = s * ap + c * aq;
                }
                for (int k = 0; k < 3; ++k) {  // A <- J^T A (rows p, q)
                    const double ap = A[p][k], aq = A[q][k];
                    A[p][k] = c * ap - s * aq;
                    A[q][k] = s * ap + c * aq;
                }
                for (int k = 0; k < 3; ++k) {
                    const double vp = V[k][p], vq = V[k][q];
                    V[k][p] = c * vp - s * vq;
                    V[k][q] = s * vp + c * vq;
                }
            }
    }
    // bubble sort (descending) of (diagonal, eigenvector column) pairs; static indices only
    double d[3] = {A[0][0], A[1][1], A[2][2]};
    double C[3][3];  // C[c] = column c of V
    for (int c = 0; c < 3; ++c)
        for (int k = 0; k < 3; ++k) C[c][k] = V[k][c];
    auto cswap = [&](int j) {
        if (d[j] < d[j + 1]) {
            const double t = d[j]; d[j] = d[j + 1]; d[j + 1] = t;
            for (int k = 0; k < 3; ++k) { const double u = C[j][k]; C[j][k] = C[j + 1][k]; C[j + 1][k] = u; }
        }
    };
    cswap(0); cswap(1); cswap(0);
    for (int i = 0; i < 3; ++i) {
        w[i] = d[i];
        double big = C[i][0];
        for (int k = 1; k < 3; ++k)
            if (fabs(C[i][k]) > fabs(big)) big = C[i][k];
        const double sg = big >= 0 ? 1.0 : -1.0;
        for (int k = 0; k < 3; ++k) E[i][k] = sg * C[i][k];
    }
}

// SVD of a 3x3 (row-major A) by one-sided Jacobi: A = U diag(s) V^T, s descending.
__device__ __forceinline__ void svd3(const double* A, double U[3][3], double s[3], double V[3][3]) {
    double B[3][3];  // B[col][row]
    double W[3][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}};  // W[col][row]
    for (int c = 0; c < 3; ++c)
        for (int r = 0; r < 3; ++r) B[c][r] = A[3 * r + c];
    for (int sweep = 0; sweep < 40; ++sweep) {
        bool rot = false;
        for (int p = 0; p < 2; ++p)
            for (int q = p + 1; q < 3; ++q) {
                double al = 0, be = 0, ga = 0;
                for (int r = 0; r < 3; ++r) {
                    al += B[p][r] * B[p][r];
                    be += B[q][r] * B[q][r];
                    ga += B[p][r] * B[q][r];
                }
                if (ga == 0.0 || fabs(ga) <= 1e-15 * sqrt(al * be)) continue;
                rot = true;
                const double zeta = (be - al) / (2.0 * ga);
                const double t = (zeta >= 0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
                const double c = 1.0 / sqrt(1.0 + t * t), sn = c * t;
                for (int r = 0; r < 3; ++r) {
                    const double bp = B[p][r], bq = B[q][r];
                    B[p][r] = c * bp - sn * bq;
                    B[q][r] = sn * bp + c * bq;
                    const double wp = W[p][r], wq = W[q][r];
                    W[p][r] = c * wp - sn * wq;
                    W[q][r] = sn * wp + c * wq;
                }
            }
        if (!rot) break;
    }
    double sg[3];
    for (int c = 0; c < 3; ++c) sg[c] = sqrt(B[c][0] * B[c][0] + B[c][1] * B[c][1] + B[c][2] * B[c][2]);
    // bubble sort (descending) of (sigma, B column, W column); static indices only
    auto cswap = [&](int j) {
        if (sg[j] < sg[j + 1]) {
            const double t = sg[j]; sg[j] = sg[j + 1]; sg[j + 1] = t;
            for (int r = 0; r < 3; ++r) {
                const double b = B[j][r]; B[j][r] = B[j + 1][r]; B[j + 1][r] = b;
                const double w = W[j][r]; W[j][r] = W[j + 1][r]; W[j + 1][r] = w;
            }
        }
    };
    cswap(0); cswap(1); cswap(0);
    for (int i = 0; i < 3; ++i) {
        s[i] = sg[i];
        for (int r = 0; r < 3; ++r) V[r][i] = W[i][r];
    }
    for (int i = 0; i < 2; ++i)
        for (int r = 0; r < 3; ++r) U[r][i] = s[i] > 0 ? B[i][r] / s[i] : (r == i ? 1.0 : 0.0);
    if (s[2] > 1e-300 * s[0] && s[2] > 0) {
        for (int r = 0; r < 3; ++r) U[r][2] = B[2][r] / s[2];
    } else {  // rank-deficient: complete the basis
        U[0][2] = U[1][0] * U[2][1] - U[2][0] * U[1][1];
        U[1][2] = U[2][0] * U[0][1] - U[0][0] * U[2][1];
        U[2][2] = U[0][0] * U[1][1] - U[1][0] * U[0][1];
    }
}

// cv::Rodrigues matrix -> vector (calibration.cpp): R projected on SO(3) by
// SVD, then the axis-angle with OpenCV's small-s branch.
__device__ void rodrigues_inv(const double* Rin, double* rv) {
    double U[3][3], s[3], V[3][3], R[3][3];
    svd3(Rin, U, s, V);
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) R[i][j] = U[i][0] * V[j][0] + U[i][1] * V[j][1] + U[i][2] * V[j][2];
    double rx = R[2][1] - R[1][2], ry = R[0][2] - R[2][0], rz = R[1][0] - R[0][1];
    const double sn = sqrt((rx * rx + ry * ry + rz * rz) * 0.25);
    double c = (R[0][0] + R[1][1] + R[2][2] - 1) * 0.5;
    c = c > 1. ? 1. : c < -1. ? -1. : c;
    double theta = acos(c);
    if (sn < 1e-5) {
        if (c > 0) { rv[0] = rv[1] = rv[2] = 0; return; }
        double t = (R[0][0] + 1) * 0.5;
        rx = sqrt(fmax(t, 0.));
        t = (R[1][1] + 1) * 0.5;
        ry = sqrt(fmax(t, 0.)) * (R[0][1] < 0 ? -1. : 1.);
        t = (R[2][2] + 1) * 0.5;
        rz = sqrt(fmax(t, 0.)) * (R[0][2] < 0 ? -1. : 1.);
        if (fabs(rx) < fabs(ry) && fabs(rx) < fabs(rz) && (R[1][2] > 0) != (ry * rz > 0)) rz = -rz;
        theta /= sqrt(rx * rx + ry * ry + rz * rz);
        rv[0] = rx * theta; rv[1] = ry * theta; rv[2] = rz * theta;
        return;
    }
    const double vth = 1 / (2 * sn) * theta;
    rv[0] = rx * vth; rv[1] = ry * vth; rv[2] = rz * vth;
}

// cv::Rodrigues vector -> matrix Jacobian, J[i*9+k] = dR_k / dr_i.
__device__ void rodrigues_jac(const double* rvec, double* J) {
    const double theta = sqrt(rvec[0] * rvec[0] + rvec[1] * rvec[1] + rvec[2] * rvec[2]);
    if (theta < kEps64) {
        for (int k = 0; k < 27; ++k) J[k] = 0;
        J[5] = -1; J[7] = 1; J[9 + 2] = 1; J[9 + 6] = -1; J[18 + 1] = -1; J[18 + 3] = 1;
        return;
    }
    const double c = cos(theta), s = sin(theta), c1 = 1. - c, it = 1. / theta;
    const double rx = rvec[0] * it, ry = rvec[1] * it, rz = rvec[2] * it;
    const double I[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    const double rrt[9] = {rx * rx, rx * ry, rx * rz, rx * ry, ry * ry, ry * rz, rx * rz, ry * rz, rz * rz};
    const double rxm[9] = {0, -rz, ry, rz, 0, -rx, -ry, rx, 0};
    const double drrt[27] = {rx + rx, ry, rz, ry, 0, 0, rz, 0, 0, 0, rx, 0, rx, ry + ry, rz, 0, rz, 0,
                             0, 0, rx, 0, 0, ry, rx, ry, rz + rz};
    const double drx[27] = {0, 0, 0, 0, 0, -1, 0, 1, 0, 0, 0, 1, 0, 0, 0, -1, 0, 0,
                            0, -1, 0, 1, 0, 0, 0, 0, 0};
    for (int i = 0; i < 3; ++i) {
        const double ri = i == 0 ? rx : i == 1 ? ry : rz;
        const double a0 = -s * ri, a1 = (s - 2 * c1 * it) * ri, a2 = c1 * it, a3 = (c - s * it) * ri, a4 = s * it;
        for (int k = 0; k < 9; ++k)
            J[i * 9 + k] = a0 * I[k] + a1 * rrt[k] + a2 * drrt[i * 9 + k] + a3 * rxm[k] + a4 * drx[i * 9 + k];
    }
}

// Least squares min ||A x - b|| for a 6 x nc (nc <= 5) full-column-rank A by
// Householder QR (row-major A, modified in place).
template <int NC>
__device__ void lsq6(double (&A)[6][NC], double (&b)[6], double (&x)[NC]) {
    for (int k = 0; k < NC; ++k) {
        double nrm = 0;
        for (int r = k; r < 6; ++r) nrm += A[r][k] * A[r][k];
        nrm = sqrt(nrm);
        if (nrm == 0.0) continue;
        const double alpha = A[k][k] >= 0 ? -nrm : nrm;
        double v[6];
        for (int r = 0; r < 6; ++r) v[r] = r < k ? 0.0 : A[r][k];
        v[k] -= alpha;
        double vn = 0;
        for (int r = k; r < 6; ++r) vn += v[r] * v[r];
        if (vn == 0.0) continue;
        const double beta = 2.0 / vn;
        for (int c = k; c < NC; ++c) {
            double s = 0;
            for (int r = k; r < 6; ++r) s += v[r] * A[r][c];
            s *= beta;
            for (int r = k; r < 6; ++r) A[r][c] -= s * v[r];
        }
        double s = 0;
        for (int r = k; r < 6; ++r) s += v[r] * b[r];
        s *= beta;
        for (int r = k; r < 6; ++r) b[r] -= s * v[r];
    }
    for (int k = NC - 1; k >= 0; --k) {
        double s = b[k];
        for (int c = k + 1; c < NC; ++c) s -= A[k][c] * x[c];
        x[k] = A[k][k] != 0.0 ? s / A[k][k] : 0.0;
    }
}

struct EpnpData {
    double pw[5][3], us[5][2], al[5][4];
    double fu, fv, uc, vc;
};

// compute_R_and_t for one beta vector (epnp.cpp); returns the mean reprojection error.
__device__ __forceinline__ double epnp_R_t(const EpnpData& D, const double* G, const int* vi, const double* betas, double* R,
                           double* t) {
    double ccs[4][3] = {};
    for (int i = 0; i < 4; ++i) {
        const double* v = G + gV;  // eigenvector vi[i] = column vi[i] of V
        for (int j = 0; j < 4; ++j)
            for (int k = 0; k < 3; ++k) ccs[j][k] += betas[i] * v[(3 * j + k) * 12 + vi[i]];
    }
    double pcs[5][3];
    for (int p = 0; p < 5; ++p)
        for (int j = 0; j < 3; ++j)
            pcs[p][j] = D.al[p][0] * ccs[0][j] + D.al[p][1] * ccs[1][j] + D.al[p][2] * ccs[2][j] + D.al[p][3] * ccs[3][j];
    if (pcs[0][2] < 0)
        for (int p = 0; p < 5; ++p)
            for (int j = 0; j < 3; ++j) pcs[p][j] = -pcs[p][j];
    double pc0[3] = {0, 0, 0}, pw0[3] = {0, 0, 0};
    for (int p = 0; p < 5; ++p)
        for (int j = 0; j < 3; ++j) { pc0[j] += pcs[p][j]; pw0[j] += D.pw[p][j]; }
    for (int j = 0; j < 3; ++j) { pc0[j] /= 5; pw0[j] /= 5; }
    double abt[9] = {};
    for (int p = 0; p < 5; ++p)
        for (int j = 0; j < 3; ++j)
            for (int k = 0; k < 3; ++k) abt[3 * j + k] += (pcs[p][j] - pc0[j]) * (D.pw[p][k] - pw0[k]);
    double U[3][3], s[3], V[3][3];
    svd3(abt, U, s, V);
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) R[3 * i + j] = U[i][0] * V[j][0] + U[i][1] * V[j][1] + U[i][2] * V[j][2];
    const double det = R[0] * R[4] * R[8] + R[1] * R[5] * R[6] + R[2] * R[3] * R[7] - R[2] * R[4] * R[6] -
                       R[1] * R[3] * R[8] - R[0] * R[5] * R[7];
    if (det < 0) { R[6] = -R[6]; R[7] = -R[7]; R[8] = -R[8]; }
    for (int i = 0; i < 3; ++i) t[i] = pc0[i] - (R[3 * i] * pw0[0] + R[3 * i + 1] * pw0[1] + R[3 * i + 2] * pw0[2]);
    double sum = 0;
    for (int p = 0; p < 5; ++p) {
        const double* pw = D.pw[p];
        const double Xc = R[0] * pw[0] + R[1] * pw[1] + R[2] * pw[2] + t[0];
        const double Yc = R[3] * pw[0] + R[4] * pw[1] + R[5] * pw[2] + t[1];
        const double iz = 1.0 / (R[6] * pw[0] + R[7] * pw[1] + R[8] * pw[2] + t[2]);
        const double ue = D.uc + D.fu * Xc * iz, ve = D.vc + D.fv * Yc * iz;
        sum += sqrt((D.us[p][0] - ue) * (D.us[p][0] - ue) + (D.us[p][1] - ve) * (D.us[p][1] - ve));
    }
    return sum / 5;
}

// Phase timers for tools/prof_pnp.py: build with -DSFMHIP_PNP_PROF (make EXTRA=-DSFMHIP_PNP_PROF);
// compiled out otherwise.
#ifdef SFMHIP_PNP_PROF
__device__ unsigned long long g_pprof[16];
__device__ unsigned long long g_wgt[2 * 1024];  // per-workgroup start / end
#define PPROF(i) do { if (threadIdx.x == 0) { const unsigned long long t1_ = wall_clock64(); atomicAdd(&g_pprof[i], t1_ - pp_t); pp_t = t1_; } } while (0)
#define PPROF_INIT unsigned long long pp_t = wall_clock64()
#define PPROF_ADD(i, v) do { if (threadIdx.x == 0) atomicAdd(&g_pprof[i], (unsigned long long)(v)); } while (0)
#define PPROF_WG(k) do { if (threadIdx.x == 0 && blockIdx.x < 1024) g_wgt[2 * blockIdx.x + (k)] = wall_clock64(); } while (0)
#else
#define PPROF(i) do {} while (0)
#define PPROF_INIT do {} while (0)
#define PPROF_WG(k) do {} while (0)
#define PPROF_ADD(i, v) do {} while (0)
#endif

// Round-robin pair schedule of the 12x12 parallel Jacobi: round r pairs (11, r) and
// ((r + k) mod 11, (r - k) mod 11), k = 1..5, each ordered p < q; entry r * 6 + k = p | q << 8.
__device__ __forceinline__ void pnp_pair_table(unsigned short* pq, int tid) {
    if (tid < 66) {
        const int r = tid / 6, k = tid % 6;
        int p, q;
        if (k == 0) { p = 11; q = r; } else { p = (r + k) % 11; q = (r - k + 11) % 11; }
        if (p > q) { const int t = p; p = q; q = t; }
        pq[tid] = (unsigned short)(p | (q << 8));
    }
}

// EPnP eigen-decomposition of M^T M (12x12, symmetric) by Householder tridiagonalisation and
// the implicit QL iteration (EISPACK tred2 / tql2 form), on a kPnGL-lane group.  A (G[gA]) is
// reduced in LDS, each lane owning rows gl and gl + 8; the reflector v and the update vector q
// go through LDS (G[gRot], G[gL]); Q = H_0 ... H_9 is kept in registers (the lane's two rows).
// The QL iteration runs on every lane of the group (d, e in registers, the same operations on
// the same values) and each lane rotates its own rows of Q, so no rotation is broadcast.
// Result as the Jacobi's: eigenvalues on A's diagonal, eigenvectors as the columns of V (G[gV]).
__device__ __forceinline__ void epnp_eig_ql(int gl, double* G) {
    double* A = G + gA;
    double* vv = G + gRot;   // 12 doubles
    double* qv = G + gL;     // 12 doubles
    const int r0 = gl, r1 = gl + kPnGL;
    const bool h1 = r1 < 12;
    double z0[12], z1[12];   // rows r0 and r1 of Q
#pragma unroll
    for (int j = 0; j < 12; ++j) {
        z0[j] = j == r0 ? 1.0 : 0.0;
        z1[j] = j == r1 ? 1.0 : 0.0;
    }
    double d[12], e[12];
#pragma unroll
    for (int k = 0; k < 10; ++k) {
        // x = A[k+1..11][k]; |x|^2 over the group
        const double a0 = r0 > k ? A[r0 * 12 + k] : 0.0;
        const double a1 = h1 && r1 > k ? A[r1 * 12 + k] : 0.0;
        double n2 = fma(a0, a0, a1 * a1);
#pragma unroll
        for (int o = kPnGL / 2; o > 0; o >>= 1) n2 += __shfl_xor(n2, o, kPnGL);
        const double x0 = A[(k + 1) * 12 + k];
        const double s2 = n2 - x0 * x0;
        if (!(s2 > 1e-300 * n2) || !(n2 > 0.0)) {   // column already reduced (uniform in the group)
            e[k] = x0;
            continue;
        }
        const double alpha = x0 >= 0.0 ? -sqrt_nr(n2) : sqrt_nr(n2);
        const double vk = x0 - alpha;
        const double beta = 2.0 * rcp_nr(fma(vk, vk, s2));
        e[k] = alpha;
        const double v0 = r0 == k + 1 ? vk : a0;   // rows <= k: 0 (a0 = 0 there)
        const double v1 = r1 == k + 1 ? vk : a1;
        vv[r0] = v0;
        if (h1) vv[r1] = v1;
        lds_fence();
        // p = beta A v on the trailing block; K = beta / 2 v.p
        double p0 = 0.0, p1 = 0.0;
#pragma unroll
        for (int j = k + 1; j < 12; ++j) {
            const double vj = vv[j];
            p0 = fma(A[r0 * 12 + j], vj, p0);
            if (h1) p1 = fma(A[r1 * 12 + j], vj, p1);
        }
        p0 = r0 > k ? beta * p0 : 0.0;
        p1 = h1 && r1 > k ? beta * p1 : 0.0;
        double kk = fma(v0, p0, v1 * p1);
#pragma unroll
        for (int o = kPnGL / 2; o > 0; o >>= 1) kk += __shfl_xor(kk, o, kPnGL);
        kk *= 0.5 * beta;
        const double q0 = fma(-kk, v0, p0), q1 = fma(-kk, v1, p1);
        qv[r0] = q0;
        if (h1) qv[r1] = q1;
        lds_fence();
        // A <- A - v q^T - q v^T on the trailing block (own rows); Q <- Q H (own rows)
        double w0 = 0.0, w1 = 0.0;
#pragma unroll
        for (int j = k + 1; j < 12; ++j) {
            const double vj = vv[j], qj = qv[j];
            if (r0 > k) A[r0 * 12 + j] = A[r0 * 12 + j] - fma(v0, qj, q0 * vj);
            if (h1 && r1 > k) A[r1 * 12 + j] = A[r1 * 12 + j] - fma(v1, qj, q1 * vj);
            w0 = fma(z0[j], vj, w0);
            w1 = fma(z1[j], vj, w1);
        }
        w0 *= beta;
        w1 *= beta;
#pragma unroll
        for (int j = k + 1; j < 12; ++j) {
            const double vj = vv[j];
            z0[j] = fma(-w0, vj, z0[j]);
            z1[j] = fma(-w1, vj, z1[j]);
        }
        lds_fence();
    }
    e[10] = A[11 * 12 + 10];
    e[11] = 0.0;
#pragma unroll
    for (int i = 0; i < 12; ++i) d[i] = A[i * 13];
    // implicit QL (tql2): e[i] couples d[i] and d[i + 1]
    for (int l = 0; l < 12; ++l) {
        for (int iter = 0; iter < 40; ++iter) {
            int m = 11;
#pragma unroll
            for (int j = 10; j >= 0; --j) {
                const double dd = fabs(d[j]) + fabs(d[j + 1]);
                if (j >= l && fabs(e[j]) + dd == dd) m = j;
            }
            if (m <= l) break;
            double dl = 0.0, dl1 = 0.0, el = 0.0, dm = 0.0;
#pragma unroll
            for (int j = 0; j < 12; ++j) {
                if (j == l) { dl = d[j]; el = e[j]; }
                if (j == l + 1) dl1 = d[j];
                if (j == m) dm = d[j];
            }
            double g = (dl1 - dl) * (0.5 * rcp_nr(el));
            double r = sqrt_nr(fma(g, g, 1.0));
            g = dm - dl + el * rcp_nr(g + (g >= 0.0 ? r : -r));
            double s = 1.0, c = 1.0, p = 0.0;
            bool live = true;
#pragma unroll
            for (int i = 10; i >= 0; --i) {
                if (!(live && i >= l && i < m)) continue;
                const double f = s * e[i], b = c * e[i];
                r = sqrt_nr(fma(f, f, g * g));
                e[i + 1] = r;
                if (r == 0.0) {   // underflow: deflate and restart this l
                    d[i + 1] -= p;
#pragma unroll
                    for (int j = 0; j < 12; ++j)
                        if (j == m) e[j] = 0.0;
                    live = false;
                    continue;
                }
                const double ir = rcp_nr(r);
                s = f * ir;
                c = g * ir;
                g = d[i + 1] - p;
                r = fma(d[i] - g, s, 2.0 * c * b);
                p = s * r;
                d[i + 1] = g + p;
                g = fma(c, r, -b);
                const double f0 = z0[i + 1], f1 = z1[i + 1];
                z0[i + 1] = fma(s, z0[i], c * f0);
                z0[i] = fma(c, z0[i], -s * f0);
                z1[i + 1] = fma(s, z1[i], c * f1);
                z1[i] = fma(c, z1[i], -s * f1);
            }
            if (live) {
#pragma unroll
                for (int j = 0; j < 12; ++j) {
                    if (j == l) { d[j] -= p; e[j] = g; }
                    if (j == m) e[j] = 0.0;
                }
            }
        }
    }
    lds_fence();
    if (gl == 0) {
#pragma unroll
        for (int i = 0; i < 12; ++i) A[i * 13] = d[i];
    }
#pragma unroll
    for (int j = 0; j < 12; ++j) {
        G[gV + r0 * 12 + j] = z0[j];
        if (h1) G[gV + r1 * 12 + j] = z1[j];
    }
    lds_fence();
}

// EPnP on 5 correspondences by a kPnGL-lane group; writes (rvec, tvec) to out[6].
__device__ __forceinline__ void epnp_group(const EpnpData& D, int gl, double* G, double* out,
                                           const unsigned short* __restrict__ pq, bool ql) {
    PPROF_INIT;
    // M^T M (12x12) into A, V = I
    // (alphas and uc - u, vc - v were staged in G by prepare: a dynamic index into D would put
    // it in scratch memory)
    for (int e = gl; e < 144; e += kPnGL) {
        const int i = e / 12, j = e % 12;
        double acc = 0;
#pragma unroll
        for (int p = 0; p < 5; ++p) {
            // M rows 2p (u) and 2p+1 (v): col 3c -> a*fu / 0, col 3c+1 -> 0 / a*fv, col 3c+2 -> a*(uc-u) / a*(vc-v)
            const int ci = i / 3, ki = i % 3, cj = j / 3, kj = j % 3;
            const double ai = G[gAl + 4 * p + ci], aj = G[gAl + 4 * p + cj];
            const double du = G[gUd + 2 * p], dv = G[gUd + 2 * p + 1];
            const double mu_i = ki == 0 ? ai * D.fu : ki == 1 ? 0.0 : ai * du;
            const double mu_j = kj == 0 ? aj * D.fu : kj == 1 ? 0.0 : aj * du;
            const double mv_i = ki == 0 ? 0.0 : ki == 1 ? ai * D.fv : ai * dv;
            const double mv_j = kj == 0 ? 0.0 : kj == 1 ? aj * D.fv : aj * dv;
            acc += mu_i * mu_j + mv_i * mv_j;
        }
        G[gA + e] = acc;
        G[gV + e] = (i == j) ? 1.0 : 0.0;
    }
    lds_fence();
    PPROF(7);
    // parallel-ordered two-sided Jacobi: 11 rounds of 6 disjoint pairs per sweep
    // the round's pairs from the workgroup's LDS table (pnp_pair_table: p | q << 8), not two
    // modulo-11 divisions per block and round
    auto pair_of = [&](int rnd, int k, int& p, int& q) {
        const unsigned e = pq[rnd * 6 + k];
        p = (int)(e & 255u);
        q = (int)(e >> 8);
    };
    double* A = G + gA;
    double* V = G + gV;
    if (ql) epnp_eig_ql(gl, G);   // default (SFMHIP_PNP_EIG=0: the Jacobi below)
    for (int sweep = 0; sweep < (ql ? 0 : 15); ++sweep) {
        // convergence: off-diagonal vs diagonal mass (group reduction; kJcN (18) elements per lane,
        // all loads issued before the sums)
        double av[kJcN];
#pragma unroll
        for (int it = 0; it < kJcN; ++it) av[it] = A[gl + kPnGL * it];
        double off = 0, dg = 0;
#pragma unroll
        for (int it = 0; it < kJcN; ++it) {
            const int e = gl + kPnGL * it;
            if (e / 12 == e % 12) dg += av[it] * av[it]; else off += av[it] * av[it];
        }
        for (int o = kPnGL / 2; o > 0; o >>= 1) { off += __shfl_xor(off, o, kPnGL); dg += __shfl_xor(dg, o, kPnGL); }
        if (off <= 1e-30 * dg) break;
        PPROF_ADD(15, 1);
        for (int rnd = 0; rnd < 11; ++rnd) {
            PPROF(8);
            if (gl < 6) {
                int p, q;
                pair_of(rnd, gl, p, q);
                const double apq = A[p * 12 + q], aqq = A[q * 12 + q], app = A[p * 12 + p];
                const bool rot = apq != 0.0;
                double t, c;
                if (kPnFastRot) {   // Newton-refined v_rcp / v_rsq (a few ulps): any rotation this close keeps
                                    // the sweep convergent, and the chain has no IEEE division / sqrt
                    const double tau = (aqq - app) * (0.5 * rcp_nr(rot ? apq : 1.0));
                    t = (tau >= 0 ? 1.0 : -1.0) * rcp_nr(fabs(tau) + sqrt_nr(fma(tau, tau, 1.0)));
                    c = rsq_nr(fma(t, t, 1.0));
                } else {
                    const double tau = (aqq - app) / (2.0 * apq);
                    t = (tau >= 0 ? 1.0 : -1.0) / (fabs(tau) + sqrt(1.0 + tau * tau));
                    c = 1.0 / sqrt(1.0 + t * t);
                }
                G[gRot + 2 * gl] = rot ? c : 1.0;
                G[gRot + 2 * gl + 1] = rot ? t * c : 0.0;
            }
            lds_fence();
            PPROF(13);
            // A <- J^T A J and V <- V J fused per 2x2 block: block (bi, bj) of A is rows
            // pair bi x columns pair bj, rotated by rows then by columns (the same operations,
            // in the same order, as two separate passes); V block = rows 2bi, 2bi+1 x pair bj.
            // The 36 blocks are disjoint: a lane loads its kJbN blocks, then rotates and stores them.
            int ia[kJbN][4], iv[kJbN][4];
            double ld[kJbN][12];
#pragma unroll
            for (int it = 0; it < kJbN; ++it) {
                const int b = min(gl + kPnGL * it, 35);
                const int bi = b / 6, bj = b - 6 * bi;
                int pi, qi, pj, qj;
                pair_of(rnd, bi, pi, qi);
                pair_of(rnd, bj, pj, qj);
                ia[it][0] = pi * 12 + pj; ia[it][1] = pi * 12 + qj; ia[it][2] = qi * 12 + pj; ia[it][3] = qi * 12 + qj;
                iv[it][0] = 24 * bi + pj; iv[it][1] = 24 * bi + qj; iv[it][2] = 24 * bi + 12 + pj; iv[it][3] = 24 * bi + 12 + qj;
                ld[it][0] = G[gRot + 2 * bi]; ld[it][1] = G[gRot + 2 * bi + 1];
                ld[it][2] = G[gRot + 2 * bj]; ld[it][3] = G[gRot + 2 * bj + 1];
#pragma unroll
                for (int k = 0; k < 4; ++k) { ld[it][4 + k] = A[ia[it][k]]; ld[it][8 + k] = V[iv[it][k]]; }
            }
#pragma unroll
            for (int it = 0; it < kJbN; ++it) {
                if (gl + kPnGL * it >= 36) break;
                const double ci = ld[it][0], si = ld[it][1], cj = ld[it][2], sj = ld[it][3];
                const double a00 = ld[it][4], a01 = ld[it][5], a10 = ld[it][6], a11 = ld[it][7];
                const double v0p = ld[it][8], v0q = ld[it][9], v1p = ld[it][10], v1q = ld[it][11];
                const double r00 = ci * a00 - si * a10, r10 = si * a00 + ci * a10;
                const double r01 = ci * a01 - si * a11, r11 = si * a01 + ci * a11;
                A[ia[it][0]] = cj * r00 - sj * r01;
                A[ia[it][1]] = sj * r00 + cj * r01;
                A[ia[it][2]] = cj * r10 - sj * r11;
                A[ia[it][3]] = sj * r10 + cj * r11;
                V[iv[it][0]] = cj * v0p - sj * v0q;
                V[iv[it][1]] = sj * v0p + cj * v0q;
                V[iv[it][2]] = cj * v1p - sj * v1q;
                V[iv[it][3]] = sj * v1p + cj * v1q;
            }
            lds_fence();
            PPROF(14);
        }
    }
    PPROF(8);
    // the 4 smallest eigenvalues (ascending), canonical signs
    int vi[4];
    {
        double ev[12];
#pragma unroll
        for (int i = 0; i < 12; ++i) ev[i] = G[gA + i * 13];
        unsigned used = 0;  // bit mask: no dynamically indexed arrays
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            int b = -1;
            double eb = 0.0;
#pragma unroll
            for (int i = 0; i < 12; ++i)
                if (!((used >> i) & 1u) && (b < 0 || ev[i] < eb)) { b = i; eb = ev[i]; }
            used |= 1u << b;
            vi[k] = b;
        }
    }
    lds_fence();
    if (gl < 4) {
        const int col = gl == 0 ? vi[0] : gl == 1 ? vi[1] : gl == 2 ? vi[2] : vi[3];
        int im = 0;
        for (int r = 1; r < 12; ++r)
            if (fabs(G[gV + r * 12 + col]) > fabs(G[gV + im * 12 + col])) im = r;
        if (G[gV + im * 12 + col] < 0)
            for (int r = 0; r < 12; ++r) G[gV + r * 12 + col] = -G[gV + r * 12 + col];
    }
    lds_fence();
    // L_6x10 and rho: lane r < 6 builds row r
    if (gl < 6) {
        const int pa[6] = {0, 0, 0, 1, 1, 2}, pb[6] = {1, 2, 3, 2, 3, 3};
        const int a = pa[gl], b = pb[gl];
        double dv[4][3];
        for (int i = 0; i < 4; ++i)
            for (int k = 0; k < 3; ++k)
                dv[i][k] = G[gV + (3 * a + k) * 12 + vi[i]] - G[gV + (3 * b + k) * 12 + vi[i]];
        auto dot = [&](int i, int j) { return dv[i][0] * dv[j][0] + dv[i][1] * dv[j][1] + dv[i][2] * dv[j][2]; };
        double* row = G + gL + 10 * gl;
        row[0] = dot(0, 0); row[1] = 2.0 * dot(0, 1); row[2] = dot(1, 1); row[3] = 2.0 * dot(0, 2);
        row[4] = 2.0 * dot(1, 2); row[5] = dot(2, 2); row[6] = 2.0 * dot(0, 3); row[7] = 2.0 * dot(1, 3);
        row[8] = 2.0 * dot(2, 3); row[9] = dot(3, 3);
        const double* ca = G + gCws + 3 * a;
        const double* cb = G + gCws + 3 * b;
        G[gRho + gl] = (ca[0] - cb[0]) * (ca[0] - cb[0]) + (ca[1] - cb[1]) * (ca[1] - cb[1]) +
                       (ca[2] - cb[2]) * (ca[2] - cb[2]);
    }
    lds_fence();
    PPROF(9);
    // three beta approximations (lane 0: B11 B12 B13 B14, 1: B11 B12 B22, 2: B11 B12 B22 B13 B23)
    if (gl < 3) {
        double L[6][10], rho[6];
        for (int r = 0; r < 6; ++r) {
            for (int c = 0; c < 10; ++c) L[r][c] = G[gL + 10 * r + c];
            rho[r] = G[gRho + r];
        }
        double be[4] = {0, 0, 0, 0};
        if (gl == 0) {
            double A[6][4], b[6], x[4];
            const int cs[4] = {0, 1, 3, 6};
            for (int r = 0; r < 6; ++r) { for (int c = 0; c < 4; ++c) A[r][c] = L[r][cs[c]]; b[r] = rho[r]; }
            lsq6<4>(A, b, x);
            if (x[0] < 0) { be[0] = sqrt(-x[0]); be[1] = -x[1] / be[0]; be[2] = -x[2] / be[0]; be[3] = -x[3] / be[0]; }
            else { be[0] = sqrt(x[0]); be[1] = x[1] / be[0]; be[2] = x[2] / be[0]; be[3] = x[3] / be[0]; }
        } else if (gl == 1) {
            double A[6][3], b[6], x[3];
            for (int r = 0; r < 6; ++r) { for (int c = 0; c < 3; ++c) A[r][c] = L[r][c]; b[r] = rho[r]; }
            lsq6<3>(A, b, x);
            if (x[0] < 0) { be[0] = sqrt(-x[0]); be[1] = x[2] < 0 ? sqrt(-x[2]) : 0.0; }
            else { be[0] = sqrt(x[0]); be[1] = x[2] > 0 ? sqrt(x[2]) : 0.0; }
            if (x[1] < 0) be[0] = -be[0];
        } else {
            double A[6][5], b[6], x[5];
            for (int r = 0; r < 6; ++r) { for (int c = 0; c < 5; ++c) A[r][c] = L[r][c]; b[r] = rho[r]; }
            lsq6<5>(A, b, x);
            if (x[0] < 0) { be[0] = sqrt(-x[0]); be[1] = x[2] < 0 ? sqrt(-x[2]) : 0.0; }
            else { be[0] = sqrt(x[0]); be[1] = x[2] > 0 ? sqrt(x[2]) : 0.0; }
            if (x[1] < 0) be[0] = -be[0];
            be[2] = x[3] / be[0];
        }
        for (int it = 0; it < 5; ++it) {  // gauss_newton
            double A[6][4], b[6], x[4];
            for (int i = 0; i < 6; ++i) {
                const double* l = L[i];
                A[i][0] = 2 * l[0] * be[0] + l[1] * be[1] + l[3] * be[2] + l[6] * be[3];
                A[i][1] = l[1] * be[0] + 2 * l[2] * be[1] + l[4] * be[2] + l[7] * be[3];
                A[i][2] = l[3] * be[0] + l[4] * be[1] + 2 * l[5] * be[2] + l[8] * be[3];
                A[i][3] = l[6] * be[0] + l[7] * be[1] + l[8] * be[2] + 2 * l[9] * be[3];
                b[i] = rho[i] - (l[0] * be[0] * be[0] + l[1] * be[0] * be[1] + l[2] * be[1] * be[1] +
                                 l[3] * be[0] * be[2] + l[4] * be[1] * be[2] + l[5] * be[2] * be[2] +
                                 l[6] * be[0] * be[3] + l[7] * be[1] * be[3] + l[8] * be[2] * be[3] +
                                 l[9] * be[3] * be[3]);
            }
            lsq6<4>(A, b, x);
            for (int i = 0; i < 4; ++i) be[i] += x[i];
        }
        double R[9], t[3];
        const double err = epnp_R_t(D, G, vi, be, R, t);
        double* sol = G + gSol + 13 * gl;
        for (int k = 0; k < 9; ++k) sol[k] = R[k];
        for (int k = 0; k < 3; ++k) sol[9 + k] = t[k];
        sol[12] = err;
    }
    lds_fence();
    PPROF(10);
    if (gl == 0) {
        int N = 0;
        if (G[gSol + 13 + 12] < G[gSol + 12]) N = 1;
        if (G[gSol + 26 + 12] < G[gSol + 13 * N + 12]) N = 2;
        const double* sol = G + gSol + 13 * N;
        rodrigues_inv(sol, out);
        out[3] = sol[9]; out[4] = sol[10]; out[5] = sol[11];
    }
    lds_fence();
    PPROF(11);
}

// projection of a float object point (converted to double) with R, t, K;
// the result rounded to float as cvProjectPoints2 stores into a CV_32F array.
__device__ __forceinline__ void project_f(const double* R, const double* t, double fx, double fy, double cx,
                                          double cy, float X, float Y, float Z, float& u, float& v) {
    const double x = R[0] * X + R[1] * Y + R[2] * Z + t[0];
    const double y = R[3] * X + R[4] * Y + R[5] * Z + t[1];
    double z = R[6] * X + R[7] * Y + R[8] * Z + t[2];
    z = z ? 1.0 / z : 1.0;
    u = (float)(x * z * fx + cx);
    v = (float)(y * z * fy + cy);
}

// K sums at once: the same per-value wave reduction and cross-wave order as block_sum
// (the same bits), one barrier pair instead of K
template <int K>
__device__ __forceinline__ void block_sum_n(double (&v)[K], double* red /* [K * 4] */) {
#pragma unroll
    for (int k = 0; k < K; ++k)
        for (int o = 32; o > 0; o >>= 1) v[k] += __shfl_xor(v[k], o);
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    __syncthreads();
    if ((threadIdx.x & 63) == 0)
#pragma unroll
        for (int k = 0; k < K; ++k) red[k * 4 + w] = v[k];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] = ((red[k * 4] + red[k * 4 + 1]) + red[k * 4 + 2]) + red[k * 4 + 3];
}

__device__ __forceinline__ double block_sum(double v, double* red) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    const int w = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[w] = v;
    __syncthreads();
    return ((red[0] + red[1]) + red[2]) + red[3];
}

// One sample's correspondences (the float copies, as solvePnPRansac casts them) and intrinsics.
__device__ __forceinline__ void pnp_load_sample(const float* __restrict__ f, const int* idx, double fx, double fy,
                                                double cx, double cy, EpnpData& D) {
    D.fu = fx; D.fv = fy; D.uc = cx; D.vc = cy;
    for (int j = 0; j < 5; ++j) {
        for (int k = 0; k < 3; ++k) D.pw[j][k] = (double)f[5 * idx[j] + k];
        for (int k = 0; k < 2; ++k) D.us[j][k] = (double)f[5 * idx[j] + 3 + k];
    }
}

// EPnP control points and barycentric alphas (every lane of the group; lane 0 stages them in G).
__device__ __forceinline__ void pnp_prepare(EpnpData& D, double* G, int gl) {
    double c0[3] = {0, 0, 0};
    for (int j = 0; j < 5; ++j)
        for (int k = 0; k < 3; ++k) c0[k] += D.pw[j][k];
    for (int k = 0; k < 3; ++k) c0[k] /= 5;
    double A[3][3] = {}, w[3], E[3][3];
    for (int j = 0; j < 5; ++j)
        for (int a = 0; a < 3; ++a)
            for (int b = 0; b < 3; ++b) A[a][b] += (D.pw[j][a] - c0[a]) * (D.pw[j][b] - c0[b]);
    eig3_desc(A, w, E);
    double cws[4][3];
    for (int k = 0; k < 3; ++k) cws[0][k] = c0[k];
    for (int i = 1; i < 4; ++i) {
        const double kk = sqrt(fmax(w[i - 1], 0.0) / 5);
        for (int k = 0; k < 3; ++k) cws[i][k] = c0[k] + kk * E[i - 1][k];
    }
    if (gl == 0)
        for (int i = 0; i < 4; ++i)
            for (int k = 0; k < 3; ++k) G[gCws + 3 * i + k] = cws[i][k];
    double CC[3][3];
    for (int i = 0; i < 3; ++i)
        for (int j = 1; j < 4; ++j) CC[i][j - 1] = cws[j][i] - cws[0][i];
    const double det = CC[0][0] * (CC[1][1] * CC[2][2] - CC[1][2] * CC[2][1]) -
                       CC[0][1] * (CC[1][0] * CC[2][2] - CC[1][2] * CC[2][0]) +
                       CC[0][2] * (CC[1][0] * CC[2][1] - CC[1][1] * CC[2][0]);
    const double id = det != 0.0 ? 1.0 / det : 0.0;
    double ci[3][3];
    ci[0][0] = (CC[1][1] * CC[2][2] - CC[1][2] * CC[2][1]) * id;
    ci[0][1] = (CC[0][2] * CC[2][1] - CC[0][1] * CC[2][2]) * id;
    ci[0][2] = (CC[0][1] * CC[1][2] - CC[0][2] * CC[1][1]) * id;
    ci[1][0] = (CC[1][2] * CC[2][0] - CC[1][0] * CC[2][2]) * id;
    ci[1][1] = (CC[0][0] * CC[2][2] - CC[0][2] * CC[2][0]) * id;
    ci[1][2] = (CC[0][2] * CC[1][0] - CC[0][0] * CC[1][2]) * id;
    ci[2][0] = (CC[1][0] * CC[2][1] - CC[1][1] * CC[2][0]) * id;
    ci[2][1] = (CC[0][1] * CC[2][0] - CC[0][0] * CC[2][1]) * id;
    ci[2][2] = (CC[0][0] * CC[1][1] - CC[0][1] * CC[1][0]) * id;
    for (int j = 0; j < 5; ++j) {
        const double d0 = D.pw[j][0] - cws[0][0], d1 = D.pw[j][1] - cws[0][1], d2 = D.pw[j][2] - cws[0][2];
        for (int a = 0; a < 3; ++a) D.al[j][1 + a] = ci[a][0] * d0 + ci[a][1] * d1 + ci[a][2] * d2;
        D.al[j][0] = 1.0 - D.al[j][1] - D.al[j][2] - D.al[j][3];
    }
    if (gl == 0)
        for (int j = 0; j < 5; ++j) {
            for (int a = 0; a < 4; ++a) G[gAl + 4 * j + a] = D.al[j][a];
            G[gUd + 2 * j] = D.uc - D.us[j][0];
            G[gUd + 2 * j + 1] = D.vc - D.us[j][1];
        }
    lds_fence();
}

// After the RANSAC loop (best model s_best, maxgood inliers, last hypothesis run): the inlier mask
// of the best model, CvLevMarq on the inliers (cvProjectPoints2's analytic Jacobian, J^T J / J^T e
// as fixed-order block reductions), the outputs.  Every thread of the kPnThreads workgroup.
// stage (LDS the caller no longer needs, cap points): the problem's points and inlier flags are
// copied there when they fit, so the LM passes read LDS instead of global memory (the same values
// and per-thread order: the same bits); null or n > cap reads global memory.
__device__ __forceinline__ void pnp_refine(int p, int n, int64_t off, const float* __restrict__ fg, double fx,
                                           double fy, double cx, double cy, float thr, int maxgood, int last,
                                           const double* s_best, double* s_lm, double* s_red,
                                           uint8_t* __restrict__ mask, double* __restrict__ rvec_out,
                                           double* __restrict__ tvec_out, int32_t* __restrict__ ninl_out,
                                           int32_t* __restrict__ iters_out, int32_t* __restrict__ ok_out,
                                           float* stage = nullptr, int cap = 0) {
    const int tid = threadIdx.x;
#ifdef SFMHIP_PNP_PROF
    unsigned long long pp_t = wall_clock64();
#endif
    if (maxgood <= 0) {
        if (tid == 0) { ok_out[p] = 0; ninl_out[p] = 0; iters_out[p] = last + 1; }
        return;
    }
    const bool staged = stage && n <= cap;
    uint8_t* inl = staged ? reinterpret_cast<uint8_t*>(stage + 5 * cap) : mask + off;
    if (staged)
        for (int t = tid; t < 5 * n; t += kPnThreads) stage[t] = fg[t];
    const float* f = staged ? stage : fg;
    // inlier mask of the best model
    if (tid == 0) rodrigues(s_best, s_lm + 39);
    __syncthreads();
    for (int i = tid; i < n; i += kPnThreads) {
        float pu, pv;
        project_f(s_lm + 39, s_best + 3, fx, fy, cx, cy, f[5 * i], f[5 * i + 1], f[5 * i + 2], pu, pv);
        const float du = f[5 * i + 3] - pu, dv = f[5 * i + 4] - pv;
        const uint8_t m = (du * du + dv * dv <= thr) ? 1 : 0;
        mask[off + i] = m;
        if (staged) inl[i] = m;
    }
    // Levenberg-Marquardt refinement on the inliers (CvLevMarq control flow)
    double* prm = s_lm;       // param[6]
    double* prev = s_lm + 6;  // prevParam[6]
    double* dR = s_lm + 12;   // dR/dr (27)
    double* Rm = s_lm + 39;   // R (9)
    if (tid < 6) prm[tid] = s_best[tid];
    __syncthreads();
    PPROF(4);
    auto eval = [&](bool with_j, double* jtj, double* jte) -> double {
        if (tid == 0) {
            rodrigues(prm, Rm);
            rodrigues_jac(prm, dR);
        }
        __syncthreads();
        double acc[28];
        for (int k = 0; k < 28; ++k) acc[k] = 0;
        for (int i = tid; i < n; i += kPnThreads) {
            if (!inl[i]) continue;
            const double X = f[5 * i], Y = f[5 * i + 1], Z = f[5 * i + 2];
            const double xc = Rm[0] * X + Rm[1] * Y + Rm[2] * Z + prm[3];
            const double yc = Rm[3] * X + Rm[4] * Y + Rm[5] * Z + prm[4];
            double z = Rm[6] * X + Rm[7] * Y + Rm[8] * Z + prm[5];
            z = z ? 1.0 / z : 1.0;
            const double x = xc * z, y = yc * z;
            const double eu = (x * fx + cx) - (double)f[5 * i + 3], ev = (y * fy + cy) - (double)f[5 * i + 4];
            acc[27] += eu * eu + ev * ev;
            if (with_j) {
                double ju[6], jv[6];
                for (int j = 0; j < 3; ++j) {
                    const double dx0 = X * dR[j * 9 + 0] + Y * dR[j * 9 + 1] + Z * dR[j * 9 + 2];
                    const double dy0 = X * dR[j * 9 + 3] + Y * dR[j * 9 + 4] + Z * dR[j * 9 + 5];
                    const double dz0 = X * dR[j * 9 + 6] + Y * dR[j * 9 + 7] + Z * dR[j * 9 + 8];
                    ju[j] = fx * (z * (dx0 - x * dz0));
                    jv[j] = fy * (z * (dy0 - y * dz0));
                }
                ju[3] = fx * z; ju[4] = 0; ju[5] = fx * (-x * z);
                jv[3] = 0; jv[4] = fy * z; jv[5] = fy * (-y * z);
                int k = 0;
                for (int a = 0; a < 6; ++a)
                    for (int b = a; b < 6; ++b) acc[k++] += ju[a] * ju[b] + jv[a] * jv[b];
                for (int a = 0; a < 6; ++a) acc[21 + a] += ju[a] * eu + jv[a] * ev;
            }
        }
        double e2 = 0;
        if (with_j) {   // all 28 sums behind one barrier pair
            block_sum_n<28>(acc, s_red);
            for (int k = 0; k < 21; ++k) jtj[k] = acc[k];
            for (int k = 21; k < 27; ++k) jte[k - 21] = acc[k];
            e2 = acc[27];
        } else {
            e2 = block_sum(acc[27], s_red);
        }
        return sqrt(e2);
    };
    // thread 0 solves (JtJ + lambda diag) x = JtErr; param = prev - x
    auto step = [&](const double* jtj, const double* jte, int lam) {
        if (tid == 0) {
            double A[6][7];
            int k = 0;
            for (int a = 0; a < 6; ++a)
                for (int b = a; b < 6; ++b) { A[a][b] = jtj[k]; A[b][a] = jtj[k]; ++k; }
            const double l = exp(lam * log(10.0));
            for (int a = 0; a < 6; ++a) { A[a][a] *= 1.0 + l; A[a][6] = jte[a]; }
#pragma unroll
            for (int c = 0; c < 6; ++c) {  // Gaussian elimination, partial pivoting (static indices)
                int pv = c;
                double best = fabs(A[c][c]);
#pragma unroll
                for (int r = c + 1; r < 6; ++r)
                    if (fabs(A[r][c]) > best) { pv = r; best = fabs(A[r][c]); }
#pragma unroll
                for (int r = c + 1; r < 6; ++r)
                    if (pv == r)
#pragma unroll
                        for (int j = 0; j < 7; ++j) { const double t = A[c][j]; A[c][j] = A[r][j]; A[r][j] = t; }
                if (A[c][c] == 0.0) continue;
#pragma unroll
                for (int r = c + 1; r < 6; ++r) {
                    const double fct = A[r][c] / A[c][c];
#pragma unroll
                    for (int j = c; j < 7; ++j) A[r][j] -= fct * A[c][j];
                }
            }
            double x[6];
            for (int r = 5; r >= 0; --r) {
                double s = A[r][6];
                for (int j = r + 1; j < 6; ++j) s -= A[r][j] * x[j];
                x[r] = A[r][r] != 0.0 ? s / A[r][r] : 0.0;
            }
            for (int a = 0; a < 6; ++a) prm[a] = prev[a] - x[a];
        }
        __syncthreads();
    };
    double jtj[21], jte[6];
    int lam = -3, iters = 0;
    double prev_err = 0;
    double err = eval(true, jtj, jte);
    for (;;) {
        if (tid < 6) prev[tid] = prm[tid];
        __syncthreads();
        step(jtj, jte, lam);
        if (iters == 0) prev_err = err;
        double err_norm;
        for (;;) {
            err_norm = eval(false, nullptr, nullptr);
            if (err_norm > prev_err) {
                ++lam;
                if (lam <= 16) { step(jtj, jte, lam); continue; }
            }
            break;
        }
        lam = max(lam - 1, -16);
        ++iters;
        double dn = 0, pn = 0;
        for (int a = 0; a < 6; ++a) { dn += (prm[a] - prev[a]) * (prm[a] - prev[a]); pn += prev[a] * prev[a]; }
        if (iters >= 20 || sqrt(dn) < 1.1920928955078125e-07 * sqrt(pn)) break;
        prev_err = err_norm;
        err = eval(true, jtj, jte);
    }
    PPROF(5);
    PPROF_WG(1);
    if (tid == 0) {
        for (int k = 0; k < 3; ++k) { rvec_out[3 * p + k] = prm[k]; tvec_out[3 * p + k] = prm[3 + k]; }
        ok_out[p] = 1; ninl_out[p] = maxgood; iters_out[p] = last + 1;
    }
}

__global__ __launch_bounds__(kPnThreads) void pnp_ransac_kernel(
    const double* __restrict__ obj, const double* __restrict__ img, const int64_t* __restrict__ offs,
    const double* __restrict__ cam, int max_iters, double reproj, double confidence, float* __restrict__ wf,
    double* __restrict__ rvec_out, double* __restrict__ tvec_out, uint8_t* __restrict__ mask,
    int32_t* __restrict__ ninl_out, int32_t* __restrict__ iters_out, int32_t* __restrict__ ok_out, int eig_ql) {
    __shared__ double s_grp[kPnH * kPnGS];
    __shared__ double s_models[kPnH][6 + 9];  // rvec, tvec, R
    __shared__ int s_cnt[kPnH];
    __shared__ int s_sub[kPnH * 5];
    __shared__ double s_best[6];
    __shared__ double s_red[4 * 28];
    __shared__ double s_lm[6 + 6 + 27 + 9];   // param, prev, dRdr, R
    __shared__ int s_niters, s_maxgood, s_k0, s_last, s_flag;
    __shared__ unsigned short s_pq[66];

    const int p = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
    const int h = tid / kPnGL, gl = tid % kPnGL;
    PPROF_WG(0);
    const int64_t off = offs[p];
    const int n = (int)(offs[p + 1] - off);
    const double fx = cam[4 * p], fy = cam[4 * p + 1], cx = cam[4 * p + 2], cy = cam[4 * p + 3];
    const float thr = (float)(reproj * reproj);
    float* f = wf + off * 5;  // float copies: X, Y, Z, u, v
    for (int i = tid; i < n; i += kPnThreads) {
        for (int k = 0; k < 3; ++k) f[5 * i + k] = (float)obj[3 * (off + i) + k];
        for (int k = 0; k < 2; ++k) f[5 * i + 3 + k] = (float)img[2 * (off + i) + k];
        mask[off + i] = 0;
    }
    if (tid == 0) { s_niters = max(max_iters, 1); s_maxgood = 0; s_k0 = 0; s_last = -1; }
    pnp_pair_table(s_pq, tid);
    __syncthreads();
    if (n < 5) {
        if (tid == 0) { ok_out[p] = 0; ninl_out[p] = 0; iters_out[p] = 0; }
        return;
    }
    auto load_sample = [&](const int* idx, EpnpData& D) { pnp_load_sample(f, idx, fx, fy, cx, cy, D); };
    auto prepare = [&](EpnpData& D, double* G) { pnp_prepare(D, G, gl); };
    if (n == 5) {  // model_points == npoints: solvePnP(EPnP) on all points, no refinement
        if (h == 0) {
            const int idx[5] = {0, 1, 2, 3, 4};
            EpnpData D;
            load_sample(idx, D);
            prepare(D, s_grp);
            epnp_group(D, gl, s_grp, s_best, s_pq, eig_ql != 0);
        }
        __syncthreads();
        if (tid == 0) {
            for (int k = 0; k < 3; ++k) { rvec_out[3 * p + k] = s_best[k]; tvec_out[3 * p + k] = s_best[3 + k]; }
            ok_out[p] = 1; ninl_out[p] = 5; iters_out[p] = 1;
        }
        if (tid < 5) mask[off + tid] = 1;
        return;
    }
    CvRng rng{~0ULL};
    const unsigned mg = (unsigned)((1ULL << 32) / (unsigned)n);   // n > 5 here
    PPROF_INIT;
    for (;;) {
        const int k0 = s_k0, niters = s_niters;
        if (tid == 0) {   // samples in registers (geom_dev.h cv_rng_sample5), then to LDS
            const int nh = min(kPnH, niters - k0);
            for (int hh = 0; hh < nh; ++hh) {
                int d[5];
                cv_rng_sample5(rng.s, (unsigned)n, mg, d);
#pragma unroll
                for (int i = 0; i < 5; ++i) s_sub[hh * 5 + i] = d[i];
            }
        }
        if (tid < kPnH) s_cnt[tid] = 0;
        __syncthreads();
        PPROF(0);
        const bool live = k0 + h < niters;
        if (live) {
            EpnpData D;
            PPROF_INIT;
            load_sample(s_sub + h * 5, D);
            double* G = s_grp + h * kPnGS;
            prepare(D, G);
            PPROF(6);
            epnp_group(D, gl, G, s_models[h], s_pq, eig_ql != 0);
            if (gl == 0) rodrigues(s_models[h], s_models[h] + 6);
        }
        __syncthreads();
        PPROF(1);
        const int nh = min(kPnH, niters - k0);   // uniform
        for (int i0 = 0; i0 < n; i0 += kPnThreads) {
            const int i = i0 + tid;
            const bool valid = i < n;
            float X = 0, Y = 0, Z = 0, u = 0, v = 0;
            if (valid) { X = f[5 * i]; Y = f[5 * i + 1]; Z = f[5 * i + 2]; u = f[5 * i + 3]; v = f[5 * i + 4]; }
            // four models per step: independent projection chains (each with its IEEE division)
            for (int h0 = 0; h0 < nh; h0 += 4) {
                float e4[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int hh = min(h0 + q, nh - 1);
                    float pu, pv;
                    project_f(s_models[hh] + 6, s_models[hh] + 3, fx, fy, cx, cy, X, Y, Z, pu, pv);
                    const float du = u - pu, dv = v - pv;
                    e4[q] = du * du + dv * dv;
                }
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int c = __popcll(__ballot(valid && e4[q] <= thr));
                    if (lane == 0 && c && h0 + q < nh) atomicAdd(&s_cnt[h0 + q], c);
                }
            }
        }
        __syncthreads();
        PPROF(2);
        if (tid == 0) {
            int nit = niters, maxgood = s_maxgood, last = s_last;
            for (int hh = 0; hh < kPnH; ++hh) {
                const int k = k0 + hh;
                if (k >= nit) break;
                const int good = s_cnt[hh];
                if (good > max(maxgood, 4)) {
                    for (int e = 0; e < 6; ++e) s_best[e] = s_models[hh][e];
                    maxgood = good;
                    nit = update_num_iters(confidence, (double)(n - good) / n, 5, nit);
                }
                last = k;
            }
            s_niters = nit; s_maxgood = maxgood; s_last = last; s_k0 = k0 + kPnH;
        }
        __syncthreads();
        if (s_k0 >= s_niters) break;
    }
    PPROF(3);
    // the EPnP group scratch is free now: the LM stages the points there
    pnp_refine(p, n, off, f, fx, fy, cx, cy, thr, s_maxgood, s_last, s_best, s_lm, s_red, mask, rvec_out,
               tvec_out, ninl_out, iters_out, ok_out, reinterpret_cast<float*>(s_grp), kPnStageCap);
    (void)s_flag;
}


// ---------------------------------------------------------------------------
// Phase-split form (SFMHIP_PNP_MONO=0; the default is pnp_ransac_kernel).  With one workgroup per
// problem the call lasts as long as its slowest problem: one that needs a second 32-hypothesis
// chunk (33-37 iterations on the bench scene) runs the EPnP solves twice in a row, at one wave per
// SIMD (the whole kernel's 454 VGPRs), scoring included.  Here the phases are separate kernels:
//   pnp_init_kernel    float copies, per-problem state, outputs of n < 5, round 0's samples
//                      (hypotheses up to min(niters, 32): one chunk);
//   pnp_solve_kernel   persistent workgroups take (problem, chunk) items: the chunk's EPnP solves
//                      (one workgroup per CU: 454 VGPRs and 115 KB of LDS per 32 hypotheses, so a
//                      second chunk cannot run beside the first without halving both);
//   pnp_score_kernel   each item's hypotheses scored on every correspondence (96 VGPRs: full
//                      occupancy, where the one-workgroup kernel scored at one wave per SIMD);
//   pnp_replay_kernel  one wave per problem replays the counts in OpenCV's order (a model
//                      replaces the best iff count > max(best, 4); niters shrinks) and, unless the
//                      problem is complete, draws round 1's samples up to the niters it left;
//   pnp_final_kernel   the best model's inlier mask, CvLevMarq and the outputs (pnp_refine).
// The same samples, solver, counts and replay as pnp_ransac_kernel: the same outputs; a
// hypothesis past the final niters costs work, never a different result.
constexpr int kPnSpecHyps = 32;   // round 0: one chunk per problem (the solve kernel holds one workgroup per CU)
constexpr int kPnRounds = 2;
constexpr int kPnFive = 1, kPnDone = 2;

struct PnpState {
    uint64_t rng;
    int n, flags, niters, maxgood, gen_upto, eval_upto, rk, last, best_k;
};

struct PnpBufs {
    PnpState* st;
    int* samp;        // [P][hcap][5]
    double* models;   // [P][hcap][15]: rvec, tvec, R
    int* cnt;         // [P][hcap]
    int2* list;       // [kPnRounds][P * cmax]: {problem, chunk (-1: the n == 5 call)}
    int* ctr;         // [2 kPnRounds]: (count, head) per round
    int cmax, hcap;
};

// One lane per problem: samples [gen_upto, target) in cv::RNG order, then the chunks covering them.
__device__ void pnp_gen(PnpState& s, int p, int P, int round, const PnpBufs& B) {
    const int target = round + 1 < kPnRounds ? min(s.niters, kPnSpecHyps) : s.niters;
    const unsigned n = (unsigned)s.n;
    const unsigned mg = (unsigned)((1ULL << 32) / n);   // n > 5
    int* smp = B.samp + (size_t)p * B.hcap * 5;
    for (int k = s.gen_upto; k < target; ++k) {
        int d[5];
        cv_rng_sample5(s.rng, n, mg, d);
#pragma unroll
        for (int i = 0; i < 5; ++i) smp[5 * k + i] = d[i];
    }
    s.gen_upto = max(s.gen_upto, target);
    const int c0 = s.eval_upto / kPnH, c1 = (target + kPnH - 1) / kPnH;
    if (c1 > c0) {
        int2* list = B.list + (size_t)round * P * B.cmax;
        const int base = atomicAdd(B.ctr + 2 * round, c1 - c0);
        for (int c = c0; c < c1; ++c) list[base + c - c0] = make_int2(p, c);
        s.eval_upto = c1 * kPnH;
    }
}

__global__ __launch_bounds__(kPnThreads) void pnp_init_kernel(const double* __restrict__ obj,
                                                              const double* __restrict__ img,
                                                              const int64_t* __restrict__ offs, int max_iters,
                                                              float* __restrict__ wf, uint8_t* __restrict__ mask,
                                                              int32_t* __restrict__ ninl_out,
                                                              int32_t* __restrict__ iters_out,
                                                              int32_t* __restrict__ ok_out, int P, PnpBufs B) {
    const int p = blockIdx.x, tid = threadIdx.x;
    const int64_t off = offs[p];
    const int n = (int)(offs[p + 1] - off);
    float* f = wf + off * 5;
    for (int i = tid; i < n; i += kPnThreads) {
        for (int k = 0; k < 3; ++k) f[5 * i + k] = (float)obj[3 * (off + i) + k];
        for (int k = 0; k < 2; ++k) f[5 * i + 3 + k] = (float)img[2 * (off + i) + k];
        mask[off + i] = 0;
    }
    if (tid == 0) {
        PnpState s;
        s.rng = ~0ULL;
        s.n = n;
        s.flags = n < 5 ? kPnDone : n == 5 ? kPnFive : 0;
        s.niters = max(max_iters, 1);
        s.maxgood = 0;
        s.gen_upto = s.eval_upto = s.rk = 0;
        s.last = s.best_k = -1;
        if (n < 5) { ok_out[p] = 0; ninl_out[p] = 0; iters_out[p] = 0; }
        if (n == 5) B.list[atomicAdd(B.ctr, 1)] = make_int2(p, -1);
        if (n > 5) pnp_gen(s, p, P, 0, B);
        B.st[p] = s;
    }
}

__global__ __launch_bounds__(kPnThreads) void pnp_solve_kernel(
    int P, int round, const int64_t* __restrict__ offs, const double* __restrict__ cam,
    const float* __restrict__ wf, double* __restrict__ rvec_out, double* __restrict__ tvec_out,
    uint8_t* __restrict__ mask, int32_t* __restrict__ ninl_out, int32_t* __restrict__ iters_out,
    int32_t* __restrict__ ok_out, int eig_ql, PnpBufs B) {
    __shared__ double s_grp[kPnH * kPnGS];
    __shared__ double s_models[kPnH][6 + 9];
    __shared__ unsigned short s_pq[66];
    __shared__ int s_item, s_five[5];
    const int tid = threadIdx.x, h = tid / kPnGL, gl = tid % kPnGL;
    pnp_pair_table(s_pq, tid);
    if (tid < 5) s_five[tid] = tid;
    const int2* list = B.list + (size_t)round * P * B.cmax;
    const int count = B.ctr[2 * round];
    for (;;) {
        if (tid == 0) s_item = atomicAdd(B.ctr + 2 * round + 1, 1);
        __syncthreads();
        const int it = s_item;
        if (it >= count) break;
        const int p = list[it].x, c = list[it].y;
        const int64_t off = offs[p];
        const double fx = cam[4 * p], fy = cam[4 * p + 1], cx = cam[4 * p + 2], cy = cam[4 * p + 3];
        const float* f = wf + off * 5;
        // c < 0: model_points == npoints, solvePnP(EPnP) on all points (group 0), no refinement.
        // One call site of the solver for both kinds of item (one inlined copy of it).
        const bool five = c < 0;
        const int k = five ? 0 : c * kPnH + h;
        if (five ? h == 0 : k < B.st[p].gen_upto) {
            EpnpData D;
            pnp_load_sample(f, five ? s_five : B.samp + ((size_t)p * B.hcap + k) * 5, fx, fy, cx, cy, D);
            double* G = s_grp + h * kPnGS;
            pnp_prepare(D, G, gl);
            epnp_group(D, gl, G, s_models[h], s_pq, eig_ql != 0);
            if (gl == 0 && !five) rodrigues(s_models[h], s_models[h] + 6);
            lds_fence();
            if (!five) {
                double* mo = B.models + ((size_t)p * B.hcap + k) * 15;
                mo[gl] = s_models[h][gl];
                if (gl + kPnGL < 15) mo[gl + kPnGL] = s_models[h][gl + kPnGL];
            }
        }
        __syncthreads();
        if (five) {
            if (tid == 0) {
                for (int q = 0; q < 3; ++q) { rvec_out[3 * p + q] = s_models[0][q]; tvec_out[3 * p + q] = s_models[0][3 + q]; }
                ok_out[p] = 1; ninl_out[p] = 5; iters_out[p] = 1;
            }
            if (tid < 5) mask[off + tid] = 1;
            __syncthreads();
        }
    }
}

// One item per workgroup pass: the chunk's models against every correspondence, four per step.
__global__ __launch_bounds__(kPnThreads) void pnp_score_kernel(int P, int round, const int64_t* __restrict__ offs,
                                                               const double* __restrict__ cam, double reproj,
                                                               const float* __restrict__ wf, PnpBufs B) {
    __shared__ double s_m[kPnH][15];
    __shared__ int s_cnt[kPnH];
    const int tid = threadIdx.x, lane = tid & 63;
    const int2* list = B.list + (size_t)round * P * B.cmax;
    const int count = B.ctr[2 * round];
    const float thr = (float)(reproj * reproj);
    for (int it = blockIdx.x; it < count; it += gridDim.x) {
        const int p = list[it].x, c = list[it].y;
        if (c < 0) continue;   // uniform
        const int64_t off = offs[p];
        const int n = B.st[p].n;
        const int nh = min(kPnH, B.st[p].gen_upto - c * kPnH);
        const double fx = cam[4 * p], fy = cam[4 * p + 1], cx = cam[4 * p + 2], cy = cam[4 * p + 3];
        const float* f = wf + off * 5;
        const double* mo = B.models + ((size_t)p * B.hcap + c * kPnH) * 15;
        for (int e = tid; e < nh * 15; e += kPnThreads) s_m[e / 15][e % 15] = mo[e];
        if (tid < kPnH) s_cnt[tid] = 0;
        __syncthreads();
        for (int i0 = 0; i0 < n; i0 += kPnThreads) {
            const int i = i0 + tid;
            const bool valid = i < n;
            float X = 0, Y = 0, Z = 0, u = 0, v = 0;
            if (valid) { X = f[5 * i]; Y = f[5 * i + 1]; Z = f[5 * i + 2]; u = f[5 * i + 3]; v = f[5 * i + 4]; }
            for (int h0 = 0; h0 < nh; h0 += 4) {
                float e4[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int hh = min(h0 + q, nh - 1);
                    float pu, pv;
                    project_f(s_m[hh] + 6, s_m[hh] + 3, fx, fy, cx, cy, X, Y, Z, pu, pv);
                    const float du = u - pu, dv = v - pv;
                    e4[q] = du * du + dv * dv;
                }
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int cq = __popcll(__ballot(valid && e4[q] <= thr));
                    if (lane == 0 && cq && h0 + q < nh) atomicAdd(&s_cnt[h0 + q], cq);
                }
            }
        }
        __syncthreads();
        if (tid < nh) B.cnt[(size_t)p * B.hcap + c * kPnH + tid] = s_cnt[tid];
        __syncthreads();
    }
}

// One wave per problem: the counts of the listed hypotheses staged in LDS, lane 0 replays them.
__global__ __launch_bounds__(64) void pnp_replay_kernel(int P, int round, double confidence, PnpBufs B) {
    __shared__ int s_c[256];
    const int p = blockIdx.x, lane = threadIdx.x;
    PnpState s = B.st[p];
    if (s.flags & (kPnFive | kPnDone)) return;   // uniform
    int nit = s.niters, k = s.rk;
    bool done = false;
    while (k < s.eval_upto && k < nit && !done) {   // windows of 256 hypotheses
        const int w = min(256, s.eval_upto - k);
        for (int t = lane; t < w; t += 64) s_c[t] = B.cnt[(size_t)p * B.hcap + k + t];
        __syncthreads();
        if (lane == 0) {
            int t = 0;
            for (; t < w; ++t) {
                if (k + t >= nit) { done = true; break; }
                const int good = s_c[t];
                if (good > max(s.maxgood, 4)) {
                    s.best_k = k + t;
                    s.maxgood = good;
                    nit = update_num_iters(confidence, (double)(s.n - good) / s.n, 5, nit);
                }
                s.last = k + t;
            }
            s_c[0] = t | (done ? 1 << 30 : 0);
        }
        __syncthreads();
        const int r = s_c[0];
        done = (r >> 30) & 1;
        k += r & ((1 << 30) - 1);
        nit = __shfl(nit, 0);
        __syncthreads();
    }
    if (lane != 0) return;
    s.rk = k;
    s.niters = nit;
    if (done || k >= nit) s.flags |= kPnDone;
    else if (round + 1 < kPnRounds) pnp_gen(s, p, P, round + 1, B);
    B.st[p] = s;
}

__global__ __launch_bounds__(kPnThreads) void pnp_final_kernel(const int64_t* __restrict__ offs,
                                                               const double* __restrict__ cam, double reproj,
                                                               const float* __restrict__ wf,
                                                               double* __restrict__ rvec_out,
                                                               double* __restrict__ tvec_out,
                                                               uint8_t* __restrict__ mask,
                                                               int32_t* __restrict__ ninl_out,
                                                               int32_t* __restrict__ iters_out,
                                                               int32_t* __restrict__ ok_out, PnpBufs B) {
    __shared__ double s_best[6];
    __shared__ double s_red[4 * 28];
    __shared__ double s_lm[6 + 6 + 27 + 9];
    const int p = blockIdx.x, tid = threadIdx.x;
    const PnpState s = B.st[p];
    if (s.n <= 5) return;   // n < 5: ess_init; n == 5: the solve kernel
    if (s.maxgood > 0 && tid < 6) s_best[tid] = B.models[((size_t)p * B.hcap + s.best_k) * 15 + tid];
    __syncthreads();
    const int64_t off = offs[p];
    const double fx = cam[4 * p], fy = cam[4 * p + 1], cx = cam[4 * p + 2], cy = cam[4 * p + 3];
    pnp_refine(p, s.n, off, wf + off * 5, fx, fy, cx, cy, (float)(reproj * reproj), s.maxgood, s.last, s_best,
               s_lm, s_red, mask, rvec_out, tvec_out, ninl_out, iters_out, ok_out);
}

}  // namespace
}  // namespace sfmhip

using namespace sfmhip;

#ifdef SFMHIP_PNP_PROF
// Phase timers of pnp_ransac_kernel for tools/prof_pnp.py: exported only by a profiling build
// (make EXTRA=-DSFMHIP_PNP_PROF), not part of the ABI.
extern "C" int sfmhip_debug_pnp_prof(unsigned long long* out) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(sfmhip::g_pprof), sizeof(unsigned long long) * 16) != hipSuccess) return -2;
    unsigned long long z[16] = {0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(sfmhip::g_pprof), z, sizeof(z)) != hipSuccess) return -2;
    return 0;
}
extern "C" int sfmhip_debug_pnp_wg(unsigned long long* out /* [2 * 1024] */) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(sfmhip::g_wgt), sizeof(unsigned long long) * 2048) == hipSuccess ? 0 : -2;
}
#endif

extern "C" int sfmhip_pnp_ransac(const double* obj, const double* img, const int64_t* offsets, int n_problems,
                                 const double* cam, int iterations, double reprojection_error, double confidence,
                                 float* work, double* rvec, double* tvec, uint8_t* inlier_mask, int32_t* n_inliers,
                                 int32_t* iters, int32_t* ok, void* stream) {
    SFMHIP_REQUIRE(n_problems >= 0, "pnp_ransac: n_problems < 0");
    if (n_problems == 0) return SFMHIP_OK;
    SFMHIP_REQUIRE(obj && img && offsets && cam && work && rvec && tvec && inlier_mask && n_inliers && iters && ok,
                   "pnp_ransac: null pointer");
    SFMHIP_REQUIRE(reprojection_error > 0 && confidence >= 0 && confidence <= 1,
                   "pnp_ransac: reprojection_error > 0, confidence in [0, 1]");
    // EPnP's 12x12 eigen-decomposition: tridiagonal QL (default) or the parallel Jacobi (A/B)
    const char* eg = getenv("SFMHIP_PNP_EIG");
    const int eig_ql = eg && *eg ? atoi(eg) : 1;
    hipStream_t st = as_stream(stream);
    const char* mo = getenv("SFMHIP_PNP_MONO");   // 1 (default): one workgroup per problem; 0: phase-split
    if (!(mo && *mo && atoi(mo) == 0)) {
        hipLaunchKernelGGL(pnp_ransac_kernel, dim3(n_problems), dim3(kPnThreads), 0, st, obj, img, offsets, cam,
                           iterations, reprojection_error, confidence, work, rvec, tvec, inlier_mask, n_inliers, iters,
                           ok, eig_ql);
        return check_launch("pnp_ransac_kernel");
    }
    const int cmax = ceil_div(std::max(iterations, 1), kPnH), hcap = cmax * kPnH;
    auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
    const size_t per = sizeof(PnpState) + (size_t)hcap * (5 * sizeof(int) + 15 * sizeof(double) + sizeof(int)) +
                       kPnRounds * (size_t)cmax * sizeof(int2);
    const int batch = (int)std::max<int64_t>(1, std::min<int64_t>(n_problems, ((size_t)192 << 20) / per));
    const size_t bytes = al(batch * sizeof(PnpState)) + al((size_t)batch * hcap * 5 * sizeof(int)) +
                         al((size_t)batch * hcap * 15 * sizeof(double)) + al((size_t)batch * hcap * sizeof(int)) +
                         al(kPnRounds * (size_t)batch * cmax * sizeof(int2)) + al(2 * kPnRounds * sizeof(int));
    char* base = nullptr;
    if (scratch_alloc((void**)&base, bytes, st) != hipSuccess) {
        (void)hipGetLastError();
        set_error("pnp_ransac: scratch allocation of %zu bytes failed", bytes);
        return SFMHIP_E_HIP;
    }
    PnpBufs B;
    char* cur = base;
    auto carve = [&](size_t b) { char* r = cur; cur += al(b); return r; };
    B.st = (PnpState*)carve(batch * sizeof(PnpState));
    B.samp = (int*)carve((size_t)batch * hcap * 5 * sizeof(int));
    B.models = (double*)carve((size_t)batch * hcap * 15 * sizeof(double));
    B.cnt = (int*)carve((size_t)batch * hcap * sizeof(int));
    B.list = (int2*)carve(kPnRounds * (size_t)batch * cmax * sizeof(int2));
    B.ctr = (int*)carve(2 * kPnRounds * sizeof(int));
    B.cmax = cmax;
    B.hcap = hcap;
    int rc = SFMHIP_OK;
    for (int p0 = 0; p0 < n_problems && rc == SFMHIP_OK; p0 += batch) {
        const int PB = std::min(batch, n_problems - p0);
        const int64_t* of = offsets + p0;
        const double* cm = cam + 4 * (size_t)p0;
        double *rv = rvec + 3 * (size_t)p0, *tv = tvec + 3 * (size_t)p0;
        int32_t *nib = n_inliers + p0, *itb = iters + p0, *okb = ok + p0;
        (void)hipMemsetAsync(B.ctr, 0, 2 * kPnRounds * sizeof(int), st);
        hipLaunchKernelGGL(pnp_init_kernel, dim3(PB), dim3(kPnThreads), 0, st, obj, img, of, iterations, work,
                           inlier_mask, nib, itb, okb, PB, B);
        for (int round = 0; round < kPnRounds; ++round) {
            const int items = (int)std::min<int64_t>((int64_t)PB * (round == 0 ? std::min(cmax, ceil_div(kPnSpecHyps, kPnH)) : cmax), 1 << 30);
            hipLaunchKernelGGL(pnp_solve_kernel, dim3(std::min(items, 512)), dim3(kPnThreads), 0, st, PB, round, of,
                               cm, work, rv, tv, inlier_mask, nib, itb, okb, eig_ql, B);
            hipLaunchKernelGGL(pnp_score_kernel, dim3(std::min(items, 2048)), dim3(kPnThreads), 0, st, PB, round, of,
                               cm, reprojection_error, work, B);
            hipLaunchKernelGGL(pnp_replay_kernel, dim3(PB), dim3(64), 0, st, PB, round, confidence, B);
        }
        hipLaunchKernelGGL(pnp_final_kernel, dim3(PB), dim3(kPnThreads), 0, st, of, cm, reprojection_error, work, rv,
                           tv, inlier_mask, nib, itb, okb, B);
        rc = check_launch("pnp_*_kernel");
    }
    scratch_free(base, st);
    return rc;
}
