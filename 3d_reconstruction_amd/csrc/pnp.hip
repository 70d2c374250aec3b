// pnp.hip — SURVEY.md §8f row 2 (last part): cv2.solvePnPRansac at sfm.py:116
//     cv2.solvePnPRansac(X, pts1, K, np.zeros((5, 1)), cv2.SOLVEPNP_ITERATIVE)
// i.e. iterationsCount 100, reprojectionError 8, confidence 0.99, flags
// ITERATIVE (the 5th positional argument is rvec), restated from OpenCV 4.x
// (solvepnp.cpp, epnp.cpp, ptsetreg.cpp, calibration.cpp
// cvFindExtrinsicCameraParams2 + CvLevMarq); CPU restatement oracle/pnp.py.
// Parity with OpenCV is unpinned (cv2 absent).
//
// One workgroup (8 waves, two per SIMD) per registration problem:
//   * points are converted to float (solvePnPRansac's CV_32F conversion);
//   * RANSAC: lane 0 draws 64 five-point samples per chunk from cv::RNG(-1)
//     (OpenCV's ~25-40 iterations at 30 % outliers fit one chunk: round 4's
//     32-hypothesis chunks sent the 33-37-iteration problems through a second
//     chunk, which bounded the call); each sample is solved by EPnP in an
//     8-lane group (M^T M reduced to tridiagonal form, its four smallest
//     eigenpairs by bisection + inverse iteration, the three beta approximations + Gauss-Newton
//     in lanes 0..2, Procrustes; the sample, alphas, L and V live in the
//     group's LDS scratch so that the kernel fits 256 VGPRs), scored by all
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

constexpr int kPnThreads = 512;           // 8 waves: two per SIMD (<= 256 VGPRs)
constexpr int kPnNW = kPnThreads / 64;
constexpr int kPnGL = 8;                   // lanes per EPnP group
constexpr int kPnH = kPnThreads / kPnGL;  // hypotheses per chunk: 64 (OpenCV's ~25-40 iterations at 30 % outliers)
static_assert(144 % kPnGL == 0 && kPnGL >= 6, "EPnP group width");
constexpr int kPnGS = 280;                // LDS doubles per group
constexpr int kPnStageCap = kPnH * kPnGS * 8 / 21;   // LM points staged in the group scratch (5 floats + a flag)
constexpr double kEps64 = 2.220446049250313e-16;
constexpr double kDblMin64 = 2.2250738585072014e-308;

// group scratch map (doubles): M^T M, reduced in place, then the eigenvectors (columns of V) over it;
// the eigenvalues; L_6x10 (the tridiagonalisation's reflector and update vectors before it); rho; the
// control points; the alphas; the sample's object points and image points
constexpr int gA = 0, gV = 0, gEv = 144, gL = 156, gRho = 216, gCws = 222 /* 12 */, gAl = 234 /* 5 x 4 */,
              gPw = 254 /* 5 x 3 */, gUs = 269 /* 5 x 2 */;
static_assert(gUs + 10 <= kPnGS, "group scratch map");

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

// The Jacobi rotation's tangent t = sign(x) / (|x| + sqrt(1 + x^2)) by the Newton reciprocal and
// square root; 0 for |x| > 1e150 (|t| < 1e-150, where 1 + x^2 overflows and the Newton forms
// would give inf * 0) and for a NaN x (0 * rcp of an off-diagonal below the normal range: that
// rotation is skipped)
__device__ __forceinline__ double jacobi_tan(double x) {
    const double t = (x >= 0 ? 1.0 : -1.0) * rcp_nr(fabs(x) + sqrt_nr(1.0 + x * x));
    return fabs(x) <= 1e150 ? t : 0.0;
}

// Symmetric 3x3 eigen-decomposition by cyclic Jacobi: eigenvalues descending,
// rows of E = eigenvectors with the largest-|.| component positive.
__device__ void eig3_desc(double A[3][3], double w[3], double E[3][3]) {
#pragma clang fp contract(fast)
    double V[3][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
    for (int sweep = 0; sweep < 30; ++sweep) {
        const double off = A[0][1] * A[0][1] + A[0][2] * A[0][2] + A[1][2] * A[1][2];
        const double dg = A[0][0] * A[0][0] + A[1][1] * A[1][1] + A[2][2] * A[2][2];
        if (off <= 1e-32 * dg || off == 0.0) break;
        for (int p = 0; p < 2; ++p)
            for (int q = p + 1; q < 3; ++q) {
                if (A[p][q] == 0.0) continue;
                const double tau = (A[q][q] - A[p][p]) * rcp_nr(2.0 * A[p][q]);
                const double t = jacobi_tan(tau);
                const double c = rsq_nr(1.0 + t * t), s = t * c;
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
#pragma clang fp contract(fast)
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
                if (ga == 0.0 || fabs(ga) <= 1e-15 * sqrt_nr(al * be)) continue;
                rot = true;
                const double zeta = (be - al) * rcp_nr(2.0 * ga);
                const double t = jacobi_tan(zeta);
                const double c = rsq_nr(1.0 + t * t), sn = c * t;
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
    for (int c = 0; c < 3; ++c) sg[c] = sqrt_nr(B[c][0] * B[c][0] + B[c][1] * B[c][1] + B[c][2] * B[c][2]);
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
        for (int r = 0; r < 3; ++r) U[r][i] = s[i] > 0 ? B[i][r] * rcp_nr(s[i]) : (r == i ? 1.0 : 0.0);
    if (s[2] > 1e-300 * s[0] && s[2] > 0) {
        const double i2 = rcp_nr(s[2]);
        for (int r = 0; r < 3; ++r) U[r][2] = B[2][r] * i2;
    } else {  // rank-deficient: complete the basis
        U[0][2] = U[1][0] * U[2][1] - U[2][0] * U[1][1];
        U[1][2] = U[2][0] * U[0][1] - U[0][0] * U[2][1];
        U[2][2] = U[0][0] * U[1][1] - U[1][0] * U[0][1];
    }
}

// cv::Rodrigues matrix -> vector (calibration.cpp): R projected on SO(3) by
// SVD, then the axis-angle with OpenCV's small-s branch.
__device__ void rodrigues_inv(const double* Rin, double* rv) {
#pragma clang fp contract(fast)
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

// The LM's R(r) (geom_dev.h rodrigues, the same formula) with one sincos, the Newton reciprocal
// and FMAs: one thread forms it between two barriers every evaluation, so its instruction count is
// on the refinement's critical path.  The inlier masks keep the IEEE rodrigues.
__device__ __forceinline__ void rodrigues_lm(const double* rv, double* R) {
#pragma clang fp contract(fast)
    double rx = rv[0], ry = rv[1], rz = rv[2];
    const double theta = sqrt_nr(rx * rx + ry * ry + rz * rz);
    if (theta < 2.220446049250313e-16) {
        R[0] = 1; R[1] = 0; R[2] = 0; R[3] = 0; R[4] = 1; R[5] = 0; R[6] = 0; R[7] = 0; R[8] = 1;
        return;
    }
    double s, c;
    sincos(theta, &s, &c);
    const double c1 = 1.0 - c;
    const double itheta = rcp_nr(theta);
    rx = rx * itheta; ry = ry * itheta; rz = rz * itheta;
    const double rrt[9] = {rx * rx, rx * ry, rx * rz, rx * ry, ry * ry, ry * rz, rx * rz, ry * rz, rz * rz};
    const double rxm[9] = {0, -rz, ry, rz, 0, -rx, -ry, rx, 0};
    const double I[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
#pragma unroll
    for (int k = 0; k < 9; ++k) R[k] = (c * I[k] + c1 * rrt[k]) + s * rxm[k];
}

// cv::Rodrigues vector -> matrix Jacobian, J[i*9+k] = dR_k / dr_i (one sincos, FMAs).
__device__ void rodrigues_jac(const double* rvec, double* J) {
#pragma clang fp contract(fast)
    const double theta = sqrt(rvec[0] * rvec[0] + rvec[1] * rvec[1] + rvec[2] * rvec[2]);
    if (theta < kEps64) {
        for (int k = 0; k < 27; ++k) J[k] = 0;
        J[5] = -1; J[7] = 1; J[9 + 2] = 1; J[9 + 6] = -1; J[18 + 1] = -1; J[18 + 3] = 1;
        return;
    }
    double s, c;
    sincos(theta, &s, &c);
    const double c1 = 1. - c, it = rcp_nr(theta);
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

// EPnP (the sample solve: control points, M^T M, its eigenpairs, the betas, R and t) and the
// 3x3 SVD / Rodrigues inverse contract a * b + c into FMAs (#pragma clang fp contract(fast)):
// the library builds with -ffp-contract=off for the kernels whose operation order follows the
// oracle bit for bit; EPnP agrees with it to a tolerance (its eigen-solver is its own), and the
// scoring, the inlier masks and the LM keep the uncontracted order.
//
// Least squares min ||A x - b|| for a 6 x nc (nc <= 5) full-column-rank A by
// Householder QR (row-major A, modified in place); Newton reciprocals / square roots (the IEEE
// division and square-root sequences were most of the EPnP beta phase's instructions).
template <int NC>
__device__ void lsq6(double (&A)[6][NC], double (&b)[6], double (&x)[NC]) {
#pragma clang fp contract(fast)
    for (int k = 0; k < NC; ++k) {
        double nrm = 0;
        for (int r = k; r < 6; ++r) nrm += A[r][k] * A[r][k];
        nrm = sqrt_nr(nrm);
        if (nrm == 0.0) continue;
        const double alpha = A[k][k] >= 0 ? -nrm : nrm;
        double v[6];
        for (int r = 0; r < 6; ++r) v[r] = r < k ? 0.0 : A[r][k];
        v[k] -= alpha;
        double vn = 0;
        for (int r = k; r < 6; ++r) vn += v[r] * v[r];
        if (vn == 0.0) continue;
        const double beta = 2.0 * rcp_nr(vn);
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
        x[k] = A[k][k] != 0.0 ? s * rcp_nr(A[k][k]) : 0.0;
    }
}

struct EpnpData {   // the sample's points and alphas live in the group scratch (gPw, gUs, gAl)
    double fu, fv, uc, vc;
};

// compute_R_and_t for one beta vector (epnp.cpp); returns the mean reprojection error.
__device__ __forceinline__ double epnp_R_t(const EpnpData& D, const double* G, const int* vi, const double* betas, double* R,
                           double* t) {
#pragma clang fp contract(fast)
    double ccs[4][3] = {};
    for (int i = 0; i < 4; ++i) {
        const double* v = G + gV;  // eigenvector vi[i] = column vi[i] of V
        for (int j = 0; j < 4; ++j)
            for (int k = 0; k < 3; ++k) ccs[j][k] += betas[i] * v[(3 * j + k) * 12 + vi[i]];
    }
    double pcs[5][3];
    for (int p = 0; p < 5; ++p)
        for (int j = 0; j < 3; ++j)
            pcs[p][j] = G[gAl + 4 * p] * ccs[0][j] + G[gAl + 4 * p + 1] * ccs[1][j] + G[gAl + 4 * p + 2] * ccs[2][j] +
                        G[gAl + 4 * p + 3] * ccs[3][j];
    if (pcs[0][2] < 0)
        for (int p = 0; p < 5; ++p)
            for (int j = 0; j < 3; ++j) pcs[p][j] = -pcs[p][j];
    double pc0[3] = {0, 0, 0}, pw0[3] = {0, 0, 0};
    for (int p = 0; p < 5; ++p)
        for (int j = 0; j < 3; ++j) { pc0[j] += pcs[p][j]; pw0[j] += G[gPw + 3 * p + j]; }
    for (int j = 0; j < 3; ++j) { pc0[j] /= 5; pw0[j] /= 5; }
    double abt[9] = {};
    for (int p = 0; p < 5; ++p)
        for (int j = 0; j < 3; ++j)
            for (int k = 0; k < 3; ++k) abt[3 * j + k] += (pcs[p][j] - pc0[j]) * (G[gPw + 3 * p + k] - pw0[k]);
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
        const double* pw = G + gPw + 3 * p;
        const double Xc = R[0] * pw[0] + R[1] * pw[1] + R[2] * pw[2] + t[0];
        const double Yc = R[3] * pw[0] + R[4] * pw[1] + R[5] * pw[2] + t[1];
        const double iz = rcp_nr(R[6] * pw[0] + R[7] * pw[1] + R[8] * pw[2] + t[2]);
        const double ue = D.uc + D.fu * Xc * iz, ve = D.vc + D.fv * Yc * iz;
        const double u0 = G[gUs + 2 * p], u1 = G[gUs + 2 * p + 1];
        sum += sqrt_nr((u0 - ue) * (u0 - ue) + (u1 - ve) * (u1 - ve));
    }
    return sum / 5;
}

// Phase timers for tools/prof_pnp.py: build with -DSFMHIP_PNP_PROF (make EXTRA=-DSFMHIP_PNP_PROF);
// compiled out otherwise.
#ifdef SFMHIP_PNP_PROF
__device__ unsigned long long g_pprof[16];
__device__ unsigned long long g_wgt[4 * 1024];  // per workgroup: start, end, first chunk's EPnP end, RANSAC end
#define PPROF(i) do { if (threadIdx.x == 0) { const unsigned long long t1_ = wall_clock64(); atomicAdd(&g_pprof[i], t1_ - pp_t); pp_t = t1_; } } while (0)
#define PPROF_INIT unsigned long long pp_t = wall_clock64()
#define PPROF_ADD(i, v) do { if (threadIdx.x == 0) atomicAdd(&g_pprof[i], (unsigned long long)(v)); } while (0)
#define PPROF_WG(k) do { if (threadIdx.x == 0 && blockIdx.x < 1024) g_wgt[4 * blockIdx.x + (k)] = wall_clock64(); } while (0)
#else
#define PPROF(i) do {} while (0)
#define PPROF_INIT do {} while (0)
#define PPROF_WG(k) do {} while (0)
#define PPROF_ADD(i, v) do {} while (0)
#endif

// The 4 smallest eigenpairs of the tridiagonal T (d, e: e[i] couples i and i + 1) that the
// Householder reduction left, back-transformed by Q (rows z0, z1 of this lane): EPnP needs only
// the four eigenvectors of the smallest eigenvalues of M^T M.  Lane k = gl & 3 bisects the Sturm
// counts for the k-th smallest eigenvalue (LAPACK dstebz form; lanes k and k + 4 trisect the
// Gershgorin interval together, 30 steps); then, in order k = 0..3, every lane of the group runs three steps
// of inverse iteration on T - lambda_k I (Gaussian elimination with partial pivoting, dlagtf /
// dlagts form, tiny pivots perturbed), each step reorthogonalised against the earlier vectors
// (the two exact null vectors of M^T M form a cluster).  Output as the QL's: the eigenvalues in
// G[gEv] (slots 4..11 = +inf, so the selection below takes 0..3 ascending), the eigenvectors in
// columns 0..3 of V.
template <int NB, int NI>
__device__ __forceinline__ void epnp_eig4_tri(int gl, double* G, const double (&d)[12], const double (&e)[12],
                                              const double (&z0)[12], const double (&z1)[12], int r0, int r1,
                                              bool h1) {
#pragma clang fp contract(fast)
    PPROF_INIT;
    // Q's rows wait in the reduced matrix's slots (A is consumed: d, e are in registers)
    const int r1s = h1 ? r1 : 12;
#pragma unroll
    for (int j = 0; j < 12; ++j) {
        G[gA + r0 * 12 + j] = z0[j];
        G[gA + r1s * 12 + j] = z1[j];
    }
    double lo = d[0], hi = d[0], emax2 = 0.0, tn = 0.0;
#pragma unroll
    for (int i = 0; i < 12; ++i) {
        const double r = (i > 0 ? fabs(e[i - 1]) : 0.0) + fabs(e[i]);
        lo = fmin(lo, d[i] - r);
        hi = fmax(hi, d[i] + r);
        emax2 = fmax(emax2, e[i] * e[i]);
        tn = fmax(tn, fabs(d[i]) + r);
    }
    // the counts run on T scaled by a power of two to |T| <= 1 (exact), where the leading minors
    // p_i of T - x I (three-term recurrence, one FMA per step on the chain) cannot overflow:
    // |p_i| <= 3^12; a cluster at x (the null pair) leaves |p_12| ~ 1e-32, far from underflow
    (void)emax2;
    const double sc = tn > 0.0 ? ldexp(1.0, -ilogb(tn) - 1) : 1.0;
    double ds[12], es2[11];
#pragma unroll
    for (int i = 0; i < 12; ++i) ds[i] = d[i] * sc;
#pragma unroll
    for (int i = 0; i < 11; ++i) es2[i] = (e[i] * sc) * (e[i] * sc);
    const double margin = 0x1p-50;
    auto count = [&](double x) -> int {   // eigenvalues < x: sign changes of 1, p_1, ..., p_12
        double p0 = 1.0, p1 = ds[0] - x;
        int c = p1 < 0.0 ? 1 : 0;
#pragma unroll
        for (int i = 1; i < 12; ++i) {
            const double p2 = fma(ds[i] - x, p1, -es2[i - 1] * p0);
            c += (p2 < 0.0) != (p1 < 0.0) ? 1 : 0;
            p0 = p1;
            p1 = p2;
        }
        return c;
    };
    // lanes k and k + 4 trisect together: counts at a + w and a + 2w, exchanged (3^30 ~ 2^47.5)
    const int kk = gl & 3;
    double a = lo * sc - margin, b = hi * sc + margin;
    for (int it = 0; it < NB; ++it) {
        const double w = (b - a) * (1.0 / 3.0);
        const double m1 = a + w, m2 = a + 2.0 * w;
        const int c = count(gl < 4 ? m1 : m2);
        const int c1 = __shfl(c, kk, kPnGL), c2 = __shfl(c, kk + 4, kPnGL);
        if (c1 > kk) {
            b = m1;
        } else if (c2 > kk) {
            a = m1;
            b = m2;
        } else {
            a = m2;
        }
    }
    a /= sc;
    b /= sc;
    const double lam_own = 0.5 * (a + b);
    PPROF(13);
    double* Y = G + gL;   // the four vectors of T (the reduction's scratch is free)
    const double tol = 0x1p-52 * fmax(tn, 0x1p-1000);
    // lane k (and k + 4) iterates eigenvector k; the four run in lockstep and every step ends
    // with modified Gram-Schmidt in order 0..3 through LDS (lane j publishes its normalised
    // vector, the lanes after it remove that direction): the null pair of M^T M is a cluster
    const double lk = lam_own;
    // T - lambda I = P L U (U: diagonal u0 and two superdiagonals u1, u2)
    double u0[12], u1[12], u2[12], lm[11];
    bool sw[11];
    double pd = d[0] - lk, p1 = e[0], p2 = 0.0;
#pragma unroll
    for (int i = 0; i < 11; ++i) {
        const double nd = e[i], n1 = d[i + 1] - lk, n2 = i + 1 < 11 ? e[i + 1] : 0.0;
        sw[i] = fabs(nd) > fabs(pd);
        const double piv = sw[i] ? nd : (fabs(pd) < tol ? (pd < 0.0 ? -tol : tol) : pd);
        const double num = sw[i] ? pd : nd;
        const double m = num * rcp_nr(piv);
        const double a1 = sw[i] ? n1 : p1, a2 = sw[i] ? n2 : p2;   // the pivot row's superdiagonals
        const double b1 = sw[i] ? p1 : n1, b2 = sw[i] ? p2 : n2;   // the other row's
        u0[i] = piv; u1[i] = a1; u2[i] = a2; lm[i] = m;
        pd = b1 - m * a1; p1 = b2 - m * a2; p2 = 0.0;
    }
    u0[11] = fabs(pd) < tol ? (pd < 0.0 ? -tol : tol) : pd;
    u1[11] = 0.0; u2[11] = 0.0; u2[10] = 0.0;
#pragma unroll
    for (int i = 0; i < 12; ++i) u0[i] = rcp_nr(u0[i]);   // the solves multiply by 1 / u0
    double y[12];
#pragma unroll
    for (int i = 0; i < 12; ++i) y[i] = 1.0 / (1.0 + (double)((i * 7 + kk * 5) % 12));   // a generic start
#pragma unroll 1
    for (int step = 0; step < NI; ++step) {
        // solve (T - lambda I) x = y: the row operations, then U back-substitution
#pragma unroll
        for (int i = 0; i < 11; ++i) {
            const double t0 = y[i], t1 = y[i + 1];
            y[i] = sw[i] ? t1 : t0;
            y[i + 1] = (sw[i] ? t0 : t1) - lm[i] * y[i];
        }
        y[11] = y[11] * u0[11];
        y[10] = (y[10] - u1[10] * y[11]) * u0[10];
#pragma unroll
        for (int i = 9; i >= 0; --i) y[i] = (y[i] - u1[i] * y[i + 1] - u2[i] * y[i + 2]) * u0[i];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            if (kk == j) {   // publish vector j, normalised
                double n2 = 0.0;
#pragma unroll
                for (int i = 0; i < 12; ++i) n2 = fma(y[i], y[i], n2);
                const double inv = n2 > 0.0 ? rsq_nr(n2) : 0.0;
#pragma unroll
                for (int i = 0; i < 12; ++i) {
                    y[i] *= inv;
                    Y[12 * j + i] = y[i];
                }
            }
            lds_fence();
            if (kk > j) {   // remove direction j
                double dt = 0.0;
#pragma unroll
                for (int i = 0; i < 12; ++i) dt = fma(y[i], Y[12 * j + i], dt);
#pragma unroll
                for (int i = 0; i < 12; ++i) y[i] = fma(-dt, Y[12 * j + i], y[i]);
            }
        }
    }
    double lam[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) lam[k] = __shfl(lam_own, k, kPnGL);
    PPROF(14);
    // V[:, k] = Q y_k (this lane's rows: read back, then overwritten by V's), the eigenvalues
    double q0[12], q1[12];
#pragma unroll
    for (int j = 0; j < 12; ++j) {
        q0[j] = G[gA + r0 * 12 + j];
        q1[j] = G[gA + r1s * 12 + j];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        double v0 = 0.0, v1 = 0.0;
#pragma unroll
        for (int j = 0; j < 12; ++j) {
            const double yj = Y[12 * k + j];
            v0 = fma(q0[j], yj, v0);
            v1 = fma(q1[j], yj, v1);
        }
        G[gV + r0 * 12 + k] = v0;
        if (h1) G[gV + r1 * 12 + k] = v1;
    }
    if (gl == 0) {
#pragma unroll
        for (int i = 0; i < 12; ++i) G[gEv + i] = i < 4 ? lam[i] : INFINITY;
    }
    lds_fence();
    PPROF(15);
}

// EPnP eigen-decomposition of M^T M (12x12, symmetric): Householder tridiagonalisation (EISPACK
// tred2 form) on a kPnGL-lane group, then the four smallest eigenpairs of the tridiagonal
// (epnp_eig4_tri).  A (G[gA]) is reduced in LDS, each lane owning rows gl and gl + 8; the
// reflector v and the update vector q go through LDS (G[gL], before L is built); Q = H_0 ... H_9
// is kept in registers (the lane's two rows).  Round 4-5 ran the implicit QL iteration (tql2) for
// all twelve eigenpairs instead: 96-100 us of a 150 us EPnP; bisection + inverse iteration took
// the bench's PnP call from 0.414 to 0.353 ms (profiles/r5/ab/pnp_512_ab_r5.txt).
// Result: the eigenvalues in G[gEv], the eigenvectors as the columns of V (G[gV], over A).
template <int NB, int NI>
__device__ __forceinline__ void epnp_eig(int gl, double* G) {
#pragma clang fp contract(fast)
    double* A = G + gA;
    double* vv = G + gL;        // 13 doubles (L is built later)
    double* qv = G + gL + 13;   // 13 doubles
    const int r0 = gl, r1 = gl + kPnGL;
    const bool h1 = r1 < 12;
    // lanes without a second row read and write a sink row 12 (A[144..155] = the eigenvalue slots,
    // written after the QL): every load is unconditional (no branch and wait per element) and the
    // results of the sink row are masked by selects
    const int r1s = h1 ? r1 : 12;
    PPROF_INIT;
    double z0[12], z1[12];   // rows r0 and r1 of Q
#pragma unroll
    for (int j = 0; j < 12; ++j) {
        z0[j] = j == r0 ? 1.0 : 0.0;
        z1[j] = j == r1 ? 1.0 : 0.0;
    }
    // the lane's rows of A in registers (A is symmetric: the trailing block's columns are rows);
    // only v and q go through LDS
    double a0[12], a1[12];
#pragma unroll
    for (int j = 0; j < 12; ++j) {
        a0[j] = A[r0 * 12 + j];
        a1[j] = h1 ? A[r1s * 12 + j] : 0.0;
    }
    double d[12], e[12];
#pragma unroll
    for (int k = 0; k < 10; ++k) {
        // x = A[k+1..11][k]; |x|^2 over the group; x0 = A[k+1][k] from the owner of row k+1
        const double t0 = a0[k], t1 = a1[k];
        const double a0k = r0 > k ? t0 : 0.0;
        const double a1k = h1 && r1 > k ? t1 : 0.0;
        double n2 = fma(a0k, a0k, a1k * a1k);
        const double x0 = __shfl(k + 1 < kPnGL ? t0 : t1, (k + 1) % kPnGL, kPnGL);
#pragma unroll
        for (int o = kPnGL / 2; o > 0; o >>= 1) n2 += __shfl_xor(n2, o, kPnGL);
        const double s2 = n2 - x0 * x0;
        if (!(s2 > 1e-300 * n2) || !(n2 > 0.0)) {   // column already reduced (uniform in the group)
            e[k] = x0;
            continue;
        }
        const double alpha = x0 >= 0.0 ? -sqrt_nr(n2) : sqrt_nr(n2);
        const double vk = x0 - alpha;
        const double beta = 2.0 * rcp_nr(fma(vk, vk, s2));
        e[k] = alpha;
        const double v0 = r0 == k + 1 ? vk : a0k;   // rows <= k: 0 (a0k = 0 there)
        const double v1 = r1 == k + 1 ? vk : a1k;
        vv[r0] = v0;
        vv[r1s] = v1;
        lds_fence();
        // p = beta A v on the trailing block; K = beta / 2 v.p
        double p0 = 0.0, p1 = 0.0;
#pragma unroll
        for (int j = k + 1; j < 12; ++j) {
            const double vj = vv[j];
            p0 = fma(a0[j], vj, p0);
            p1 = fma(a1[j], vj, p1);
        }
        p0 = r0 > k ? beta * p0 : 0.0;
        p1 = h1 && r1 > k ? beta * p1 : 0.0;
        double kk = fma(v0, p0, v1 * p1);
#pragma unroll
        for (int o = kPnGL / 2; o > 0; o >>= 1) kk += __shfl_xor(kk, o, kPnGL);
        kk *= 0.5 * beta;
        const double q0 = fma(-kk, v0, p0), q1 = fma(-kk, v1, p1);
        qv[r0] = q0;
        qv[r1s] = q1;
        lds_fence();
        // A <- A - v q^T - q v^T on the trailing block (own rows); Q <- Q H (own rows)
        double w0 = 0.0, w1 = 0.0;
#pragma unroll
        for (int j = k + 1; j < 12; ++j) {
            const double vj = vv[j], qj = qv[j];
            if (r0 > k) a0[j] = a0[j] - fma(v0, qj, q0 * vj);
            if (r1 > k) a1[j] = a1[j] - fma(v1, qj, q1 * vj);
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
    // the diagonal and the last subdiagonal element through the v slots
    double dg0 = 0.0, dg1 = 0.0;
#pragma unroll
    for (int j = 0; j < 12; ++j) {
        if (j == r0) dg0 = a0[j];
        if (j == r1) dg1 = a1[j];
    }
    e[10] = __shfl(a1[10], 11 - kPnGL, kPnGL);
    e[11] = 0.0;
    vv[r0] = dg0;
    vv[r1s] = dg1;
    lds_fence();
#pragma unroll
    for (int i = 0; i < 12; ++i) d[i] = vv[i];
    PPROF(12);
    epnp_eig4_tri<NB, NI>(gl, G, d, e, z0, z1, r0, r1, h1);
}

// EPnP on 5 correspondences by a kPnGL-lane group; writes (rvec, tvec) to out[6].
template <int NB, int NI>
__device__ __forceinline__ void epnp_group(const EpnpData& D, int gl, double* G, double* out) {
#pragma clang fp contract(fast)
    PPROF_INIT;
    // M^T M (12x12) into A
    // (alphas and uc - u, vc - v were staged in G by prepare: a dynamic index into D would put
    // it in scratch memory)
    double al[5][4], dup[5], dvp[5];   // the alphas and (uc - u, vc - v) in registers: static indices below
#pragma unroll
    for (int p = 0; p < 5; ++p) {
#pragma unroll
        for (int c = 0; c < 4; ++c) al[p][c] = G[gAl + 4 * p + c];
        dup[p] = D.uc - G[gUs + 2 * p];
        dvp[p] = D.vc - G[gUs + 2 * p + 1];
    }
    // M^T M = sum_p (a_p a_p^T) (x) S_p with S_p = [[fu^2, 0, fu du], [0, fv^2, fv dv],
    // [fu du, fv dv, du^2 + dv^2]]: block (ci, cj) needs four sums over the points; lane gl forms
    // blocks gl and gl + 8 of the ten with ci <= cj and writes them and their mirror images
    double nn[5];
#pragma unroll
    for (int p = 0; p < 5; ++p) nn[p] = dup[p] * dup[p] + dvp[p] * dvp[p];
    const double fu2 = D.fu * D.fu, fv2 = D.fv * D.fv;
#pragma unroll
    for (int rep = 0; rep < 2; ++rep) {
        const int bk = gl + kPnGL * rep;
        if (bk < 10) {
            const int ci = bk < 4 ? 0 : bk < 7 ? 1 : bk < 9 ? 2 : 3;
            const int cj = bk < 4 ? bk : bk < 7 ? bk - 3 : bk < 9 ? bk - 5 : 3;
            double W = 0.0, Wu = 0.0, Wv = 0.0, Wn = 0.0;
#pragma unroll
            for (int p = 0; p < 5; ++p) {
                const double ai = ci == 0 ? al[p][0] : ci == 1 ? al[p][1] : ci == 2 ? al[p][2] : al[p][3];
                const double aj = cj == 0 ? al[p][0] : cj == 1 ? al[p][1] : cj == 2 ? al[p][2] : al[p][3];
                const double w = ai * aj;
                W += w;
                Wu += w * dup[p];
                Wv += w * dvp[p];
                Wn += w * nn[p];
            }
            const double blk[9] = {fu2 * W, 0.0, D.fu * Wu, 0.0, fv2 * W, D.fv * Wv, D.fu * Wu, D.fv * Wv, Wn};
#pragma unroll
            for (int r = 0; r < 3; ++r)
#pragma unroll
                for (int c = 0; c < 3; ++c) {
                    G[gA + (3 * ci + r) * 12 + 3 * cj + c] = blk[3 * r + c];
                    G[gA + (3 * cj + c) * 12 + 3 * ci + r] = blk[3 * r + c];
                }
        }
    }
    lds_fence();
    PPROF(7);
    // the four smallest eigenpairs of the 12x12 M^T M: Householder tridiagonalisation + bisection +
    // inverse iteration (the implicit QL for all twelve, round 4-5, and a parallel-ordered two-sided
    // Jacobi before it measured slower)
    epnp_eig<NB, NI>(gl, G);
    PPROF(8);
    // the 4 smallest eigenvalues (ascending), canonical signs
    int vi[4];
    {
        double ev[12];
#pragma unroll
        for (int i = 0; i < 12; ++i) ev[i] = G[gEv + i];
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
    // three beta approximations (lane 0: B11 B12 B13 B14, 1: B11 B12 B22, 2: B11 B12 B22 B13 B23);
    // L and rho are read from the group scratch where they are used (registers for 3 lanes of 8)
    double R[9], t[3], err = INFINITY;
    if (gl < 3) {
        const double* L = G + gL;   // row r: L[10 r + c]
        const double* rho = G + gRho;
        double be[4] = {0, 0, 0, 0};
        {   // one least-squares solve on all three lanes: each lane's columns of L, zero-padded to
            // five (a zero column leaves the Householder steps of the others and x unchanged, so
            // x is lsq6<4> / <3> / <5> of the lane's own system bit for bit)
            double A[6][5], bb[6], x[5];
            for (int r = 0; r < 6; ++r) {
#pragma unroll
                for (int c = 0; c < 5; ++c) {
                    const int col = gl == 0 ? (c == 0 ? 0 : c == 1 ? 1 : c == 2 ? 3 : 6) : c;
                    const bool use = gl == 0 ? c < 4 : gl == 1 ? c < 3 : true;
                    A[r][c] = use ? L[10 * r + col] : 0.0;
                }
                bb[r] = rho[r];
            }
            lsq6<5>(A, bb, x);
            if (gl == 0) {
                be[0] = sqrt_nr(fabs(x[0]));
                const double ib = (x[0] < 0 ? -1.0 : 1.0) * rcp_nr(be[0]);
                be[1] = x[1] * ib; be[2] = x[2] * ib; be[3] = x[3] * ib;
            } else {
                be[0] = sqrt_nr(fabs(x[0]));
                be[1] = (x[0] < 0 ? x[2] < 0 : x[2] > 0) ? sqrt_nr(fabs(x[2])) : 0.0;
                if (x[1] < 0) be[0] = -be[0];
                if (gl == 2) be[2] = x[3] * rcp_nr(be[0]);
            }
        }
        for (int it = 0; it < 5; ++it) {  // gauss_newton
            __asm__ volatile("" ::: "memory");   // L is re-read from LDS each step, not held in registers
            double A[6][4], b[6], x[4];
            for (int i = 0; i < 6; ++i) {
                const double* l = L + 10 * i;
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
        err = epnp_R_t(D, G, vi, be, R, t);
        if (!(err <= INFINITY)) err = INFINITY;   // a degenerate sample (NaN from the Newton forms) loses
    }
    PPROF(10);
    // the solution with the least mean reprojection error (the first on ties), chosen within the group
    const double e0 = __shfl(err, 0, kPnGL), e1 = __shfl(err, 1, kPnGL), e2 = __shfl(err, 2, kPnGL);
    int N = 0;
    if (e1 < e0) N = 1;
    if (e2 < (N == 1 ? e1 : e0)) N = 2;
    if (gl == N) {
        rodrigues_inv(R, out);
        out[3] = t[0]; out[4] = t[1]; out[5] = t[2];
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
// (the same bits), one barrier pair instead of K.  LAST_ONLY: waves other than wave 0 form only
// the last sum (the LM's cost; J^T J and J^T e go to thread 0 alone)
template <int K, bool LAST_ONLY = false>
__device__ __forceinline__ void block_sum_n(double (&v)[K], double* red /* [K * kPnNW] */) {
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    int idx;
    bool wr;
    const double x = wave_reduce_scatter<K>(v, lane, idx, wr);   // geom_dev.h: the same sums, fewer shuffles
    __syncthreads();
    if (wr) red[idx * kPnNW + w] = x;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < K; ++k) {   // the waves in order
        if (LAST_ONLY && k < K - 1 && w != 0) continue;
        double a = red[k * kPnNW];
#pragma unroll
        for (int u = 1; u < kPnNW; ++u) a += red[k * kPnNW + u];
        v[k] = a;
    }
}

__device__ __forceinline__ double block_sum(double v, double* red) {
    double a[1] = {v};
    block_sum_n<1>(a, red);
    return a[0];
}

// One sample's correspondences (the float copies, as solvePnPRansac casts them) into the group
// scratch (lane j < 5: point j), and the intrinsics.
__device__ __forceinline__ void pnp_load_sample(const float* __restrict__ f, const int* idx, double fx, double fy,
                                                double cx, double cy, EpnpData& D, double* G, int gl) {
    D.fu = fx; D.fv = fy; D.uc = cx; D.vc = cy;
    if (gl < 5) {
        const int j = idx[gl == 0 ? 0 : gl == 1 ? 1 : gl == 2 ? 2 : gl == 3 ? 3 : 4];
        for (int k = 0; k < 3; ++k) G[gPw + 3 * gl + k] = (double)f[5 * j + k];
        for (int k = 0; k < 2; ++k) G[gUs + 2 * gl + k] = (double)f[5 * j + 3 + k];
    }
    lds_fence();
}

// EPnP control points and barycentric alphas (every lane of the group; lane 0 stages them in G).
__device__ __forceinline__ void pnp_prepare(double* G, int gl) {
#pragma clang fp contract(fast)
    const double* pw = G + gPw;
    double c0[3] = {0, 0, 0};
    for (int j = 0; j < 5; ++j)
        for (int k = 0; k < 3; ++k) c0[k] += pw[3 * j + k];
    for (int k = 0; k < 3; ++k) c0[k] /= 5;
    double A[3][3] = {}, w[3], E[3][3];
    for (int j = 0; j < 5; ++j)
        for (int a = 0; a < 3; ++a)
            for (int b = 0; b < 3; ++b) A[a][b] += (pw[3 * j + a] - c0[a]) * (pw[3 * j + b] - c0[b]);
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
    if (gl == 0)
        for (int j = 0; j < 5; ++j) {
            const double d0 = pw[3 * j] - cws[0][0], d1 = pw[3 * j + 1] - cws[0][1], d2 = pw[3 * j + 2] - cws[0][2];
            double al[4];
            for (int a = 0; a < 3; ++a) al[1 + a] = ci[a][0] * d0 + ci[a][1] * d1 + ci[a][2] * d2;
            al[0] = 1.0 - al[1] - al[2] - al[3];
            for (int a = 0; a < 4; ++a) G[gAl + 4 * j + a] = al[a];
        }
    lds_fence();
}

// 10^k, k = -16..16 (the LM's damping factors)
__constant__ double kPow10[33] = {1e-16, 1e-15, 1e-14, 1e-13, 1e-12, 1e-11, 1e-10, 1e-9, 1e-8, 1e-7, 1e-6,
                                  1e-5,  1e-4,  1e-3,  1e-2,  1e-1,  1e0,   1e1,   1e2,  1e3,  1e4,  1e5,
                                  1e6,   1e7,   1e8,   1e9,   1e10,  1e11,  1e12,  1e13, 1e14, 1e15, 1e16};

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
        if (tid == 0) rodrigues_lm(prm, Rm);
        if (with_j && tid == 64) rodrigues_jac(prm, dR);   // another wave: the two run side by side
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
            block_sum_n<28, true>(acc, s_red);
            for (int k = 0; k < 21; ++k) jtj[k] = acc[k];
            for (int k = 21; k < 27; ++k) jte[k - 21] = acc[k];
            e2 = acc[27];
        } else {
            e2 = block_sum(acc[27], s_red);
        }
        return sqrt(e2);
    };
    // thread 0 solves (JtJ + lambda diag) x = JtErr; param = prev - x
    // (one thread: FMAs, one Newton reciprocal per pivot, 10^lambda from a table)
    auto step = [&](const double* jtj, const double* jte, int lam) {
#pragma clang fp contract(fast)
        if (tid == 0) {
            double A[6][7];
            int k = 0;
            for (int a = 0; a < 6; ++a)
                for (int b = a; b < 6; ++b) { A[a][b] = jtj[k]; A[b][a] = jtj[k]; ++k; }
            const double l = kPow10[lam + 16];
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
                const double ip = rcp_nr(A[c][c]);
#pragma unroll
                for (int r = c + 1; r < 6; ++r) {
                    const double fct = A[r][c] * ip;
#pragma unroll
                    for (int j = c; j < 7; ++j) A[r][j] -= fct * A[c][j];
                }
            }
            double x[6];
            for (int r = 5; r >= 0; --r) {
                double s = A[r][6];
                for (int j = r + 1; j < 6; ++j) s -= A[r][j] * x[j];
                x[r] = A[r][r] != 0.0 ? s * rcp_nr(A[r][r]) : 0.0;
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

template <int NB, int NI>
__global__ __launch_bounds__(kPnThreads) void pnp_ransac_kernel(
    const double* __restrict__ obj, const double* __restrict__ img, const int64_t* __restrict__ offs,
    const double* __restrict__ cam, int max_iters, double reproj, double confidence, float* __restrict__ wf,
    double* __restrict__ rvec_out, double* __restrict__ tvec_out, uint8_t* __restrict__ mask,
    int32_t* __restrict__ ninl_out, int32_t* __restrict__ iters_out, int32_t* __restrict__ ok_out) {
    __shared__ double s_grp[kPnH * kPnGS];
    __shared__ double s_models[kPnH][6 + 9];  // rvec, tvec, R
    __shared__ int s_cnt[kPnH];
    __shared__ int s_sub[kPnH * 5];
    __shared__ double s_best[6];
    __shared__ double s_red[kPnNW * 28];
    __shared__ double s_lm[6 + 6 + 27 + 9];   // param, prev, dRdr, R
    __shared__ int s_niters, s_maxgood, s_k0, s_last, s_flag;

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
    __syncthreads();
    if (n < 5) {
        if (tid == 0) { ok_out[p] = 0; ninl_out[p] = 0; iters_out[p] = 0; }
        return;
    }
    auto load_sample = [&](const int* idx, EpnpData& D, double* G) { pnp_load_sample(f, idx, fx, fy, cx, cy, D, G, gl); };
    if (n == 5) {  // model_points == npoints: solvePnP(EPnP) on all points, no refinement
        if (h == 0) {
            const int idx[5] = {0, 1, 2, 3, 4};
            EpnpData D;
            load_sample(idx, D, s_grp);
            pnp_prepare(s_grp, gl);
            epnp_group<NB, NI>(D, gl, s_grp, s_best);
        }
        __syncthreads();
        if (tid == 0) {
            for (int k = 0; k < 3; ++k) { rvec_out[3 * p + k] = s_best[k]; tvec_out[3 * p + k] = s_best[3 + k]; }
            ok_out[p] = 1; ninl_out[p] = 5; iters_out[p] = 1;
        }
        if (tid < 5) mask[off + tid] = 1;
        return;
    }
    uint64_t rs = ~0ULL;   // cv::RNG's state (wave 0)
    const unsigned mg = (unsigned)((1ULL << 32) / (unsigned)n);   // n > 5 here
    PPROF_INIT;
    for (;;) {
        const int k0 = s_k0, niters = s_niters;
        if (tid < 64)   // the chunk's samples by wave 0 (jump-ahead, one sample per lane)
            cv_rng_sample_wave(rs, (unsigned)n, mg, min(kPnH, niters - k0), s_sub, lane);
        if (tid < kPnH) s_cnt[tid] = 0;
        __syncthreads();
        PPROF(0);
        const bool live = k0 + h < niters;
        if (live) {
            EpnpData D;
            PPROF_INIT;
            double* G = s_grp + h * kPnGS;
            load_sample(s_sub + h * 5, D, G);
            pnp_prepare(G, gl);
            PPROF(6);
            epnp_group<NB, NI>(D, gl, G, s_models[h]);
            if (gl == 0) rodrigues(s_models[h], s_models[h] + 6);
        }
        __syncthreads();
        PPROF(1);
        if (k0 == 0) PPROF_WG(2);
        // scoring and replay in two halves of the chunk: the replay of the first half usually
        // lowers niters below the second (OpenCV's ~25 iterations), whose scoring is then skipped
        for (int hb = 0; hb < kPnH; hb += kPnH / 2) {
            const int nh = min(hb + kPnH / 2, s_niters - k0);   // uniform: the models [hb, nh) are live
            if (nh <= hb) break;
            for (int i0 = 0; i0 < n; i0 += kPnThreads) {
                const int i = i0 + tid;
                const bool valid = i < n;
                float X = 0, Y = 0, Z = 0, u = 0, v = 0;
                if (valid) { X = f[5 * i]; Y = f[5 * i + 1]; Z = f[5 * i + 2]; u = f[5 * i + 3]; v = f[5 * i + 4]; }
                // four models per step: independent projection chains (each with its IEEE division)
                for (int h0 = hb; h0 < nh; h0 += 4) {
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
                int nit = s_niters, maxgood = s_maxgood, last = s_last;
                for (int hh = hb; hh < hb + kPnH / 2; ++hh) {
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
                s_niters = nit; s_maxgood = maxgood; s_last = last;
            }
            __syncthreads();
        }
        if (tid == 0) s_k0 = k0 + kPnH;
        __syncthreads();
        if (s_k0 >= s_niters) break;
    }
    PPROF(3);
    PPROF_WG(3);
    // the EPnP group scratch is free now: the LM stages the points there
    pnp_refine(p, n, off, f, fx, fy, cx, cy, thr, s_maxgood, s_last, s_best, s_lm, s_red, mask, rvec_out,
               tvec_out, ninl_out, iters_out, ok_out, reinterpret_cast<float*>(s_grp), kPnStageCap);
    (void)s_flag;
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
extern "C" int sfmhip_debug_pnp_wg(unsigned long long* out /* [4 * 1024] */) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(sfmhip::g_wgt), sizeof(unsigned long long) * 4096) == hipSuccess ? 0 : -2;
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
    // one 512-thread workgroup per problem (a phase-split form -- EPnP solves, scoring and the RANSAC
    // replay as separate kernels over (problem, chunk) items -- measured slower: 0.694 vs 0.555 ms,
    // round 4; 256 threads with 32-hypothesis chunks and 432 registers: 0.517 vs 0.467 ms, round 5)
    // 30 trisection steps (bisection: 40 / 48 / 56 steps within 2 %), 3 inverse-iteration steps
    hipLaunchKernelGGL((pnp_ransac_kernel<30, 3>), dim3(n_problems), dim3(kPnThreads), 0, as_stream(stream), obj, img, offsets,
                       cam, iterations, reprojection_error, confidence, work, rvec, tvec, inlier_mask, n_inliers, iters,
                       ok);
    return check_launch("pnp_ransac_kernel");
}
