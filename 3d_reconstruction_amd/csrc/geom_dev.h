// geom_dev.h — f64 device helpers shared by geometry.hip and ransac.hip:
// cv::Rodrigues (vector -> matrix), cv::projectPoints without distortion and
// the cvTriangulatePoints DLT for one correspondence.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sfmhip {

// Wave sum of K doubles per lane as a reduce-scatter: at the step with offset o (32, 16, ...)
// each lane keeps the half of its values that its lane bit o selects and adds the partner's copy
// of that half, then the last value is summed over the remaining offsets.  Each value is summed
// by the same pairwise tree as the plain xor butterfly (offset 32 first), so the sums are the same
// bits, with 2^P - 1 + (6 - P) shuffles (P = ceil(log2 K)) instead of 6 K.  Returns the sum of
// value `idx` = lane >> (6 - P); the lanes whose low 6 - P bits are zero hold distinct indices.
template <int K>
__device__ __forceinline__ double wave_reduce_scatter(const double (&v)[K], int lane, int& idx, bool& writer) {
    constexpr int P = K <= 1 ? 0 : K <= 2 ? 1 : K <= 4 ? 2 : K <= 8 ? 3 : K <= 16 ? 4 : 5;
    static_assert(K <= 32, "reduce-scatter width");
    constexpr int NP = 1 << P;
    double x[NP];
#pragma unroll
    for (int k = 0; k < NP; ++k) x[k] = k < K ? v[k] : 0.0;
#pragma unroll
    for (int st = 0; st < P; ++st) {
        const int o = 32 >> st, half = NP >> (st + 1);
        const bool hi = (lane & o) != 0;
#pragma unroll
        for (int j = 0; j < half; ++j) {
            const double keep = hi ? x[j + half] : x[j], send = hi ? x[j] : x[j + half];
            x[j] = keep + __shfl_xor(send, o);
        }
    }
#pragma unroll
    for (int o = 32 >> P; o >= 1; o >>= 1) x[0] += __shfl_xor(x[0], o);
    idx = lane >> (6 - P);
    writer = (lane & ((64 >> P) - 1)) == 0 && idx < K;
    return x[0];
}

// OpenCV Rodrigues (vector -> matrix), op order of cv::Rodrigues:
//   theta = sqrt(rx^2+ry^2+rz^2); theta < DBL_EPSILON -> I;
//   R = (c*I + c1*r r^T) + s*[r]_x  with r normalised by itheta = 1/theta.
__device__ __forceinline__ void rodrigues(const double* rv, double* R) {
    double rx = rv[0], ry = rv[1], rz = rv[2];
    const double theta = sqrt(rx * rx + ry * ry + rz * rz);
    if (theta < 2.220446049250313e-16) {
        R[0] = 1; R[1] = 0; R[2] = 0; R[3] = 0; R[4] = 1; R[5] = 0; R[6] = 0; R[7] = 0; R[8] = 1;
        return;
    }
    const double c = cos(theta), s = sin(theta), c1 = 1.0 - c;
    const double itheta = 1.0 / theta;
    rx = rx * itheta; ry = ry * itheta; rz = rz * itheta;
    const double rrt[9] = {rx * rx, rx * ry, rx * rz, rx * ry, ry * ry, ry * rz, rx * rz, ry * rz, rz * rz};
    const double rxm[9] = {0, -rz, ry, rz, 0, -rx, -ry, rx, 0};
    const double I[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
#pragma unroll
    for (int k = 0; k < 9; ++k) R[k] = (c * I[k] + c1 * rrt[k]) + s * rxm[k];
}

// cv::projectPoints without distortion: x = R X + t; z = z ? 1/z : 1; u = x*z*fx + cx.
__device__ __forceinline__ void project(const double* R, const double* t, const double* X,
                                        double fx, double fy, double cx, double cy,
                                        double& u, double& v) {
    double x = R[0] * X[0] + R[1] * X[1] + R[2] * X[2] + t[0];
    double y = R[3] * X[0] + R[4] * X[1] + R[5] * X[2] + t[1];
    double z = R[6] * X[0] + R[7] * X[1] + R[8] * X[2] + t[2];
    z = (z != 0.0) ? 1.0 / z : 1.0;
    x = x * z;
    y = y * z;
    u = x * fx + cx;
    v = y * fy + cy;
}

// scipy _compute_absolute_step for '2-point': EPS**0.5 * sign0(x) * max(1, |x|)
__device__ __forceinline__ double fd_step(double x) {
    const double rstep = 1.4901161193847656e-08;  // np.finfo(float64).eps ** 0.5
    const double sgn = (x >= 0.0) ? 1.0 : -1.0;
    return rstep * sgn * fmax(1.0, fabs(x));
}

// Residual and the 18 scipy 2-point FD values of one observation (geometry.hip
// fdjac_kernel explains the op order): R = {R(rvec), R(rvec + h_k e_k), k < 3}
// (9 each), c = [rvec, t], k = K (3x3 row-major), X = the point; f0 = the base
// residual if given (else the one computed here); r (2, optional) gets the
// base residual, row[0..8] / row[9..17] the u / v rows (rvec, t, X columns).
__device__ inline void fd_obs(const double* R, const double* c, const double* k, const double* X, double obs_u,
                              double obs_v, const double* f0, double* r, double* row) {
    const double fx = k[0], fy = k[4], cx = k[2], cy = k[5];
    const double t[3] = {c[3], c[4], c[5]};
    const double Xp[3] = {X[0], X[1], X[2]};
    // base projection, keeping the partial sums R X
    const double sx = R[0] * Xp[0] + R[1] * Xp[1] + R[2] * Xp[2];
    const double sy = R[3] * Xp[0] + R[4] * Xp[1] + R[5] * Xp[2];
    const double sz = R[6] * Xp[0] + R[7] * Xp[1] + R[8] * Xp[2];
    const double zb = sz + t[2];
    const double izb = (zb != 0.0) ? 1.0 / zb : 1.0;
    const double xb = (sx + t[0]) * izb, yb = (sy + t[1]) * izb;
    const double base_u = obs_u - (xb * fx + cx), base_v = obs_v - (yb * fy + cy);
    if (r) { r[0] = base_u; r[1] = base_v; }
    const double f0u = f0 ? f0[0] : base_u;
    const double f0v = f0 ? f0[1] : base_v;
    auto put = [&](int q, double u, double v, double dx) {
        row[q] = ((obs_u - u) - f0u) / dx;
        row[9 + q] = ((obs_v - v) - f0v) / dx;
    };
    // rvec: the pair's perturbed rotations
#pragma unroll
    for (int q = 0; q < 3; ++q) {
        const double hx = c[q] + fd_step(c[q]);
        double u, v;
        project(R + 9 * (q + 1), t, Xp, fx, fy, cx, cy, u, v);
        put(q, u, v, hx - c[q]);
    }
    // t: only the last addition of coordinate q changes
    {
        const double h0 = t[0] + fd_step(t[0]), h1 = t[1] + fd_step(t[1]), h2 = t[2] + fd_step(t[2]);
        put(3, ((sx + h0) * izb) * fx + cx, yb * fy + cy, h0 - t[0]);
        put(4, xb * fx + cx, ((sy + h1) * izb) * fy + cy, h1 - t[1]);
        const double z2 = sz + h2;
        const double iz2 = (z2 != 0.0) ? 1.0 / z2 : 1.0;
        put(5, ((sx + t[0]) * iz2) * fx + cx, ((sy + t[1]) * iz2) * fy + cy, h2 - t[2]);
    }
    // X: full re-projection (the perturbed term sits inside the sums)
#pragma unroll
    for (int q = 0; q < 3; ++q) {
        double Xq[3] = {Xp[0], Xp[1], Xp[2]};
        const double hx = Xp[q] + fd_step(Xp[q]);
        Xq[q] = hx;
        double u, v;
        project(R, t, Xq, fx, fy, cx, cy, u, v);
        put(6 + q, u, v, hx - Xp[q]);
    }
}

// DLT: A (6x4) rows per view v: x*P[2]-P[0], y*P[2]-P[1], x*P[1]-y*P[0];
// one-sided (Hestenes) Jacobi on the 4 columns, V accumulates the rotations;
// the right singular vector of the smallest singular value is V's column with
// the smallest resulting column norm.  Output: unit norm, X[3] >= 0.
__device__ inline void dlt_point_jacobi(const double* P0, const double* P1, double x0, double y0, double x1,
                                 double y1, double* Xout) {
    const double* Pv[2] = {P0, P1};
    const double px[2] = {x0, x1};
    const double py[2] = {y0, y1};
    double A[4][6];  // column-major: A[col][row]
#pragma unroll
    for (int v = 0; v < 2; ++v) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const double p0 = Pv[v][k], p1 = Pv[v][4 + k], p2 = Pv[v][8 + k];
            A[k][3 * v + 0] = px[v] * p2 - p0;
            A[k][3 * v + 1] = py[v] * p2 - p1;
            A[k][3 * v + 2] = px[v] * p1 - py[v] * p0;
        }
    }
    double V[4][4] = {{1, 0, 0, 0}, {0, 1, 0, 0}, {0, 0, 1, 0}, {0, 0, 0, 1}};
    for (int sweep = 0; sweep < 30; ++sweep) {
        bool rotated = false;
#pragma unroll
        for (int p = 0; p < 3; ++p) {
#pragma unroll
            for (int q = p + 1; q < 4; ++q) {
                double alpha = 0, beta = 0, gamma = 0;
#pragma unroll
                for (int r = 0; r < 6; ++r) {
                    alpha += A[p][r] * A[p][r];
                    beta += A[q][r] * A[q][r];
                    gamma += A[p][r] * A[q][r];
                }
                if (fabs(gamma) <= 1e-15 * sqrt(alpha * beta) || gamma == 0.0) continue;
                rotated = true;
                const double zeta = (beta - alpha) / (2.0 * gamma);
                const double t = (zeta >= 0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
                const double c = 1.0 / sqrt(1.0 + t * t), s = c * t;
#pragma unroll
                for (int r = 0; r < 6; ++r) {
                    const double ap = A[p][r], aq = A[q][r];
                    A[p][r] = c * ap - s * aq;
                    A[q][r] = s * ap + c * aq;
                }
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const double vp = V[p][r], vq = V[q][r];
                    V[p][r] = c * vp - s * vq;
                    V[q][r] = s * vp + c * vq;
                }
            }
        }
        if (!rotated) break;
    }
    int best = 0;
    double bn = 0;
#pragma unroll
    for (int r = 0; r < 6; ++r) bn += A[0][r] * A[0][r];
#pragma unroll
    for (int k = 1; k < 4; ++k) {
        double nk = 0;
#pragma unroll
        for (int r = 0; r < 6; ++r) nk += A[k][r] * A[k][r];
        if (nk < bn) { bn = nk; best = k; }
    }
    double X[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) X[r] = V[0][r];
#pragma unroll
    for (int k = 1; k < 4; ++k)
        if (k == best) {
#pragma unroll
            for (int r = 0; r < 4; ++r) X[r] = V[k][r];
        }
    const double nrm = sqrt(X[0] * X[0] + X[1] * X[1] + X[2] * X[2] + X[3] * X[3]);
    const double sc = (X[3] < 0 ? -1.0 : 1.0) / nrm;
#pragma unroll
    for (int r = 0; r < 4; ++r) Xout[r] = X[r] * sc;
}

// The same null vector, cheaper: Householder QR of A (6x4 -> R 4x4, backward
// stable, no squaring of A); an exactly singular R (noise-free data) gives the
// null vector by back-substitution; otherwise inverse iteration with R's
// triangular solves (factor (sigma4/sigma3)^2 per step), started from
// R^-1 e4, for at most kDltInvIters steps until the normalised iterate stops
// moving (|dy| <= 1e-15); small-baseline points whose sigma3 ~ sigma4 make it
// crawl finish with one-sided Jacobi on the 4 columns of R (A^T A = R^T R, so
// the right singular vectors are A's).
constexpr int kDltInvIters = 6;

__device__ inline void null_vector_jacobi4(double (&R)[4][4], double* y) {
    double C[4][4], V[4][4];  // C[col][row]
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int r = 0; r < 4; ++r) { C[c][r] = R[r][c]; V[c][r] = (r == c) ? 1.0 : 0.0; }
    for (int sweep = 0; sweep < 30; ++sweep) {
        bool rotated = false;
#pragma unroll
        for (int p = 0; p < 3; ++p) {
#pragma unroll
            for (int q = p + 1; q < 4; ++q) {
                double alpha = 0, beta = 0, gamma = 0;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    alpha += C[p][r] * C[p][r];
                    beta += C[q][r] * C[q][r];
                    gamma += C[p][r] * C[q][r];
                }
                if (gamma == 0.0 || gamma * gamma <= 1e-30 * (alpha * beta)) continue;
                rotated = true;
                const double zeta = (beta - alpha) / (2.0 * gamma);
                const double t = (zeta >= 0 ? 1.0 : -1.0) / (fabs(zeta) + sqrt(1.0 + zeta * zeta));
                const double c = 1.0 / sqrt(1.0 + t * t), s = c * t;
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const double ap = C[p][r], aq = C[q][r];
                    C[p][r] = c * ap - s * aq;
                    C[q][r] = s * ap + c * aq;
                    const double vp = V[p][r], vq = V[q][r];
                    V[p][r] = c * vp - s * vq;
                    V[q][r] = s * vp + c * vq;
                }
            }
        }
        if (!rotated) break;
    }
    int best = 0;
    double bn = C[0][0] * C[0][0] + C[0][1] * C[0][1] + C[0][2] * C[0][2] + C[0][3] * C[0][3];
#pragma unroll
    for (int k = 1; k < 4; ++k) {
        const double nk = C[k][0] * C[k][0] + C[k][1] * C[k][1] + C[k][2] * C[k][2] + C[k][3] * C[k][3];
        if (nk < bn) { bn = nk; best = k; }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) y[r] = V[0][r];
#pragma unroll
    for (int k = 1; k < 4; ++k)
        if (k == best)
#pragma unroll
            for (int r = 0; r < 4; ++r) y[r] = V[k][r];
}

// 1/x and sqrt(x) on v_rcp_f64 / v_rsq_f64 with two Newton steps (within an ulp;
// the IEEE sequences cost ~3x the latency): the FAST paths of the DLT list pass
__device__ __forceinline__ double rcp_nr(double x) {
    double r = __builtin_amdgcn_rcp(x);
    r = fma(fma(-x, r, 1.0), r, r);
    return fma(fma(-x, r, 1.0), r, r);
}
__device__ __forceinline__ double rsq_nr(double x) {
    double r = __builtin_amdgcn_rsq(x);
    r = r * fma(-0.5 * x * r, r, 1.5);
    return r * fma(-0.5 * x * r, r, 1.5);
}
__device__ __forceinline__ double sqrt_nr(double x) { return x > 0.0 ? x * rsq_nr(x) : 0.0; }

// Householder QR of the 6x4 DLT system: R (upper 4x4; A^T A = R^T R), rmax = max |R_kk|.
// FAST: Newton reciprocal / square root instead of the IEEE sequences (dlt_point,
// which recoverPose also uses, keeps the IEEE ones).
template <bool FAST = false>
__device__ inline void dlt_qr(const double* P0, const double* P1, double x0, double y0, double x1, double y1,
                              double (&R)[4][4], double& rmax) {
    const double* Pv[2] = {P0, P1};
    const double px[2] = {x0, x1};
    const double py[2] = {y0, y1};
    double A[6][4];
#pragma unroll
    for (int v = 0; v < 2; ++v)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const double p0 = Pv[v][k], p1 = Pv[v][4 + k], p2 = Pv[v][8 + k];
            A[3 * v + 0][k] = px[v] * p2 - p0;
            A[3 * v + 1][k] = py[v] * p2 - p1;
            A[3 * v + 2][k] = px[v] * p1 - py[v] * p0;
        }
    rmax = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        double nrm2 = 0;
#pragma unroll
        for (int r = k; r < 6; ++r) nrm2 += A[r][k] * A[r][k];
        const double nrm = FAST ? sqrt_nr(nrm2) : sqrt(nrm2);
        const double alpha = (A[k][k] >= 0) ? -nrm : nrm;
        double v[6];
#pragma unroll
        for (int r = 0; r < 6; ++r) v[r] = (r < k) ? 0.0 : A[r][k];
        v[k] -= alpha;
        double vn2 = 0;
#pragma unroll
        for (int r = k; r < 6; ++r) vn2 += v[r] * v[r];
        const double beta = (vn2 > 0) ? (FAST ? 2.0 * rcp_nr(vn2) : 2.0 / vn2) : 0.0;
#pragma unroll
        for (int c = k; c < 4; ++c) {
            double sdot = 0;
#pragma unroll
            for (int r = k; r < 6; ++r) sdot += v[r] * A[r][c];
            sdot *= beta;
#pragma unroll
            for (int r = k; r < 6; ++r) A[r][c] -= sdot * v[r];
        }
        rmax = fmax(rmax, fabs(A[k][k]));
    }
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c) R[r][c] = (c >= r) ? A[r][c] : 0.0;
}

__device__ inline void dlt_point(const double* P0, const double* P1, double x0, double y0, double x1, double y1,
                                 double* Xout) {
    double R[4][4], rmax;
    dlt_qr(P0, P1, x0, y0, x1, y1, R, rmax);
    double y[4];
    bool done = false;
    if (fabs(R[3][3]) <= 1e-15 * rmax && fabs(R[2][2]) > 1e-15 * rmax) {  // exact null vector
        y[3] = 1.0;
#pragma unroll
        for (int r = 2; r >= 0; --r) {
            double sacc = -R[r][3];
#pragma unroll
            for (int c = r + 1; c < 3; ++c) sacc -= R[r][c] * y[c];
            y[r] = sacc / R[r][r];
        }
        done = true;
    } else if (fabs(R[3][3]) > 1e-15 * rmax && fabs(R[2][2]) > 1e-15 * rmax && fabs(R[1][1]) > 1e-15 * rmax &&
               fabs(R[0][0]) > 1e-15 * rmax) {
        double id[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) id[r] = 1.0 / R[r][r];
        y[3] = id[3];
#pragma unroll
        for (int r = 2; r >= 0; --r) {
            double sacc = 0;
#pragma unroll
            for (int c = r + 1; c < 4; ++c) sacc -= R[r][c] * y[c];
            y[r] = sacc * id[r];
        }
        for (int it = 0; it < kDltInvIters && !done; ++it) {
            // normalisation by one reciprocal (the iterate's scale is arbitrary)
            const double inn = 1.0 / sqrt(y[0] * y[0] + y[1] * y[1] + y[2] * y[2] + y[3] * y[3]);
            double yo[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) { y[r] *= inn; yo[r] = y[r]; }
            double z[4];  // R^T z = y (forward)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                double sacc = y[r];
#pragma unroll
                for (int c = 0; c < r; ++c) sacc -= R[c][r] * z[c];
                z[r] = sacc * id[r];
            }
#pragma unroll
            for (int r = 3; r >= 0; --r) {  // R y = z (backward)
                double sacc = z[r];
#pragma unroll
                for (int c = r + 1; c < 4; ++c) sacc -= R[r][c] * y[c];
                y[r] = sacc * id[r];
            }
            const double inn2 = 1.0 / sqrt(y[0] * y[0] + y[1] * y[1] + y[2] * y[2] + y[3] * y[3]);
            double dd = 0;
#pragma unroll
            for (int r = 0; r < 4; ++r) dd += (y[r] * inn2 - yo[r]) * (y[r] * inn2 - yo[r]);
            done = dd <= 1e-30;
        }
    }
    if (!done) null_vector_jacobi4(R, y);
    const double nrm = sqrt(y[0] * y[0] + y[1] * y[1] + y[2] * y[2] + y[3] * y[3]);
    if (!(nrm > 0) || !isfinite(nrm)) {
        dlt_point_jacobi(P0, P1, x0, y0, x1, y1, Xout);
        return;
    }
    const double sc = (y[3] < 0 ? -1.0 : 1.0) / nrm;
#pragma unroll
    for (int r = 0; r < 4; ++r) Xout[r] = y[r] * sc;
}

// ---------------------------------------------------------------------------
// DLT fast path on the normal equations (geometry.hip's dlt_normal_kernel; recoverPose's
// cheirality triangulations): M = A^T A, M = L D L^T, inverse iteration.  PT: the two
// cameras' 24 doubles, contiguous (a constant-space pointer for scalar loads, or plain).
constexpr int kDltNormalIters = 6;
constexpr double kDltLam3Floor = 1e-7;

// M = A^T A: m = {00, 01, 02, 03, 11, 12, 13, 22, 23, 33}
template <class PT>
__device__ __forceinline__ void dlt_normal_matrix(PT Pa, double xa, double ya, double xb, double yb, double (&m)[10]) {
#pragma unroll
    for (int k = 0; k < 10; ++k) m[k] = 0.0;
    auto acc = [&](double r0, double r1, double r2, double r3) {
        m[0] = fma(r0, r0, m[0]); m[1] = fma(r0, r1, m[1]); m[2] = fma(r0, r2, m[2]); m[3] = fma(r0, r3, m[3]);
        m[4] = fma(r1, r1, m[4]); m[5] = fma(r1, r2, m[5]); m[6] = fma(r1, r3, m[6]);
        m[7] = fma(r2, r2, m[7]); m[8] = fma(r2, r3, m[8]); m[9] = fma(r3, r3, m[9]);
    };
#pragma unroll
    for (int v = 0; v < 2; ++v) {
        const PT Q = Pa + 12 * v;
        const double x = v ? xb : xa, y = v ? yb : ya;
        // rows x p2 - p0, y p2 - p1, x p1 - y p0 (cvTriangulatePoints matrA)
        acc(fma(x, Q[8], -Q[0]), fma(x, Q[9], -Q[1]), fma(x, Q[10], -Q[2]), fma(x, Q[11], -Q[3]));
        acc(fma(y, Q[8], -Q[4]), fma(y, Q[9], -Q[5]), fma(y, Q[10], -Q[6]), fma(y, Q[11], -Q[7]));
        acc(fma(x, Q[4], -y * Q[0]), fma(x, Q[5], -y * Q[1]), fma(x, Q[6], -y * Q[2]), fma(x, Q[7], -y * Q[3]));
        // the sums are complete here: without this the compiler sinks the off-diagonal
        // sums to their first use and keeps all 24 row entries live (110 VGPRs)
        asm volatile("" : "+v"(m[0]), "+v"(m[1]), "+v"(m[2]), "+v"(m[3]), "+v"(m[4]), "+v"(m[5]), "+v"(m[6]),
                     "+v"(m[7]), "+v"(m[8]), "+v"(m[9]));
    }
}

// L D L^T of M - shift I (unit lower L: l10 l20 l30 l21 l31 l32; inverse pivots i0..i3)
struct Ldl {
    double l10, l20, l30, l21, l31, l32, i0, i1, i2, i3;
    bool pd3;      // the leading 3x3 pivots are positive
    double t3;     // trace of the leading 3x3 block's inverse (bounds its smallest eigenvalue)
};

__device__ __forceinline__ Ldl dlt_ldl(const double (&m)[10], double shift, double floor3) {
    Ldl f;
    const double d0 = m[0] - shift;
    f.i0 = rcp_nr(d0);
    f.l10 = m[1] * f.i0; f.l20 = m[2] * f.i0; f.l30 = m[3] * f.i0;
    const double d1 = fma(-f.l10, m[1], m[4] - shift);
    f.i1 = rcp_nr(d1);
    const double a21 = fma(-f.l20, m[1], m[5]), a31 = fma(-f.l30, m[1], m[6]);
    f.l21 = a21 * f.i1; f.l31 = a31 * f.i1;
    const double d2 = fma(-f.l21, a21, fma(-f.l20, m[2], m[7] - shift));
    f.i2 = rcp_nr(d2);
    const double a32 = fma(-f.l31, a21, fma(-f.l30, m[2], m[8]));
    f.l32 = a32 * f.i2;
    const double d3 = fma(-f.l32, a32, fma(-f.l31, a31, fma(-f.l30, m[3], m[9] - shift)));
    // d3 ~ lambda4 - shift may round to ~0: keep its sign, floor its size at the rounding level of M
    f.i3 = rcp_nr(d3 < 0.0 ? fmin(d3, -floor3) : fmax(d3, floor3));
    f.pd3 = d0 > 0.0 && d1 > 0.0 && d2 > 0.0;
    const double g = fma(f.l10, f.l21, -f.l20);
    f.t3 = fma(fma(g, g, fma(f.l21, f.l21, 1.0)), f.i2, fma(fma(f.l10, f.l10, 1.0), f.i1, f.i0));
    return f;
}

// One inverse-iteration step on a unit iterate: y <- (M - shift I)^-1 y, renormalised
// (sign aligned with the old y: an indefinite shifted matrix may flip it);
// returns |y_new - y_old|^2.
__device__ __forceinline__ double dlt_inv_step(const Ldl& f, double& y0, double& y1, double& y2, double& y3) {
    const double o0 = y0, o1 = y1, o2 = y2, o3 = y3;
    // L w = o, w /= d, L^T z = w
    const double w0 = o0 * f.i0;
    const double u1 = fma(-f.l10, o0, o1);
    const double w1 = u1 * f.i1;
    const double v2 = fma(-f.l21, u1, fma(-f.l20, o0, o2));
    const double w2 = v2 * f.i2;
    const double z3 = fma(-f.l32, v2, fma(-f.l31, u1, fma(-f.l30, o0, o3))) * f.i3;
    const double z2 = fma(-f.l32, z3, w2);
    const double z1 = fma(-f.l31, z3, fma(-f.l21, z2, w1));
    const double z0 = fma(-f.l30, z3, fma(-f.l20, z2, fma(-f.l10, z1, w0)));
    double s2 = rsq_nr(fma(z0, z0, fma(z1, z1, fma(z2, z2, z3 * z3))));
    if (fma(z0, o0, fma(z1, o1, fma(z2, o2, z3 * o3))) < 0.0) s2 = -s2;
    y0 = z0 * s2;
    y1 = z1 * s2;
    y2 = z2 * s2;
    y3 = z3 * s2;
    const double e0 = y0 - o0, e1 = y1 - o1, e2 = y2 - o2, e3 = y3 - o3;
    return fma(e0, e0, fma(e1, e1, fma(e2, e2, e3 * e3)));
}

__device__ __forceinline__ bool dlt_store_unit(double y0, double y1, double y2, double y3, double* Xout) {
    const double nn = fma(y0, y0, fma(y1, y1, fma(y2, y2, y3 * y3)));
    if (!(nn > 0.0) || !(nn < 1e300)) return false;
    const double sc = (y3 < 0 ? -1.0 : 1.0) / sqrt(nn);
    Xout[0] = y0 * sc;
    Xout[1] = y1 * sc;
    Xout[2] = y2 * sc;
    Xout[3] = y3 * sc;
    return true;
}

// 0: decided (Xout written); 1: lambda3 bound met but not converged; 2: the QR path decides
template <class PT>
__device__ __forceinline__ int dlt_point_normal(PT Pa, double xa, double ya, double xb, double yb, double* Xout) {
    double m[10];
    dlt_normal_matrix(Pa, xa, ya, xb, yb, m);
    // branch-free up to the iteration (an early exit lets the compiler sink the
    // off-diagonal sums past it and keep all 24 row entries live)
    const double tr = (m[0] + m[4]) + (m[7] + m[9]);
    const Ldl f = dlt_ldl(m, 0.0, 1e-30 * tr);
    const bool good = f.pd3 && tr < 1e300 && f.t3 * (kDltLam3Floor * tr) <= 1.0;
    double y0, y1, y2, y3 = 1.0;                        // L^T y = e4, normalised
    y2 = -f.l32;
    y1 = fma(-f.l21, y2, -f.l31);
    y0 = fma(-f.l10, y1, fma(-f.l20, y2, -f.l30));
    const double s0 = rsq_nr(fma(y0, y0, fma(y1, y1, fma(y2, y2, 1.0))));
    y0 *= s0; y1 *= s0; y2 *= s0; y3 = s0;
    bool done = false;
#pragma unroll 1
    for (int it = 0; it < kDltNormalIters && good && !done; ++it) done = dlt_inv_step(f, y0, y1, y2, y3) <= 1e-26;
    if (!good) return 2;
    if (!done) return 1;
    return dlt_store_unit(y0, y1, y2, y3, Xout) ? 0 : 2;
}


// ---------------------------------------------------------------------------
// One RANSAC sample of 5 distinct indices in [0, n) from cv::RNG (multiply-with-carry
// state s; uniform(0, n) = next() % n; a repeated index is redrawn), exactly as the
// one-draw-at-a-time loop (ptsetreg.cpp getSubset) gives it.  The five draws are taken at
// once — the state chain is one v_mad_u64_u32 per draw, x mod n is umulhi(x, mg) * n off by
// at most one n (mg = floor(2^32 / n), n >= 2) — and only a duplicate (~0.5 % of samples at
// n = 2048) falls back to drawing one at a time from the state after it.
__device__ __forceinline__ unsigned cv_rng_mod(unsigned x, unsigned n, unsigned mg) {
    const unsigned r = x - __umulhi(x, mg) * n;
    return r >= n ? r - n : r;
}
__device__ __forceinline__ void cv_rng_sample5(uint64_t& s, unsigned n, unsigned mg, int (&d)[5]) {
    constexpr uint64_t A = 4164903690ULL;
    uint64_t st[5];
    uint64_t sv = s;
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        sv = (uint64_t)(unsigned)sv * A + (unsigned)(sv >> 32);
        st[i] = sv;
        d[i] = (int)cv_rng_mod((unsigned)sv, n, mg);
    }
    int j = 5;   // first draw that repeats an earlier one
#pragma unroll
    for (int i = 4; i >= 1; --i) {
        bool dup = false;
#pragma unroll
        for (int t = 0; t < i; ++t) dup = dup || d[t] == d[i];
        if (dup) j = i;
    }
    if (j == 5) {
        s = st[4];
        return;
    }
    sv = st[j];   // the duplicate draw is consumed; slot j onward one draw at a time
    for (int i = j; i < 5; ++i) {
        int idx;
        for (;;) {
            sv = (uint64_t)(unsigned)sv * A + (unsigned)(sv >> 32);
            idx = (int)cv_rng_mod((unsigned)sv, n, mg);
            bool dup = false;
            for (int t = 0; t < i; ++t) dup = dup || d[t] == idx;
            if (!dup) break;
        }
        d[i] = idx;
    }
    s = sv;
}

// cv::RNG jump-ahead.  The multiply-with-carry step s' = A lo(s) + hi(s) is s' = s b^-1 mod m
// (b = 2^32, m = A b - 1, b^-1 = A mod m) for every state, so the state 5 L draws ahead of s is
// s A^(5 L) mod m: mwc_jump5 forms it as red^3(s C_L) with C_L = A^(5 L - 3) mod m and
// red(T) = (T >> 32) + lo32(T) A = T b^-1 mod m (T < 2^128 -> < 2^96 + 2^64 -> < 2^65 + 2^32 ->
// < 2^64 + 2^33 < 2 m: one conditional subtraction).  Every state after the first draw is below
// m (only the seed ~0 is not, and its lane draws from it directly), so the reduced state is the
// state itself.  C_L: tests/test_device_algorithms_model.py checks the table and the sampler.
static __constant__ uint64_t kMwcJump5[64] = {
    0x0000000000000000ULL, 0xf0badf95453cbc64ULL, 0x5ba03b6718928580ULL, 0xd1d2d0db8d934886ULL,
    0xe69a527185f4f056ULL, 0xc02e3eee453a4663ULL, 0x636eb442dcc2d6eaULL, 0x6cbe3044aad17ec3ULL,
    0x0b3deacb73698228ULL, 0x4ed646868fe1c5fbULL, 0x67b91866a3348f12ULL, 0xbdfe19229db55884ULL,
    0x8b1de00fc853e701ULL, 0x964bfc7907213ec9ULL, 0xa18b02d7c6b8c7a8ULL, 0x119ceafee6ad2026ULL,
    0x851e0ae42a79a01fULL, 0x4d75d441ef06651aULL, 0xca305cd8b6735d9dULL, 0xa0cead46256802d9ULL,
    0xcc0331836d720255ULL, 0x5293772ecb76750aULL, 0x7f9c531a780ed630ULL, 0x16a4383076ab1eb7ULL,
    0xb41cae51c1ab3a46ULL, 0x580309f14acbf443ULL, 0xd3c43315504a7b0eULL, 0xd6cd8ebac60bc726ULL,
    0x21de78f80dc167b5ULL, 0xc16d99fec2c1006fULL, 0x813367d18a1eba79ULL, 0xb9e3b30d5bbc6228ULL,
    0xce86181c1400891eULL, 0x6c2f5101981cd491ULL, 0x0b755f939d9236b7ULL, 0x2bc5b67e95aa60afULL,
    0x769dc25a88e6402eULL, 0xf026697513cafd28ULL, 0x8f57614bbe869ac9ULL, 0x2f555dd061a0c749ULL,
    0x0bb03d0077fce7f4ULL, 0x02694ae2e0277ea6ULL, 0x8f7d57288669d5fdULL, 0x5381a6d920d7393fULL,
    0xb6f3db5ccd8e3480ULL, 0xde07aa5052fe5699ULL, 0xc0ea448bd283eddeULL, 0xbd0f6b5121d2d374ULL,
    0xedfc3be01d06cf79ULL, 0xa25415f2113258adULL, 0x9fc0ea9d68d631acULL, 0x022b45e69f54b3d6ULL,
    0x9c4841ea5e5d86b3ULL, 0x0d0baff2178ada20ULL, 0xb4da0dedd6f4c6e9ULL, 0x6c4cd03af7e06ecdULL,
    0xe8da77b922d167ffULL, 0x295e9ee377d09aa1ULL, 0x4b01b846854dde13ULL, 0x79e0e2751095f676ULL,
    0x15befe6ca57026bbULL, 0x2a400035a330630aULL, 0x3db0c72c02ec828eULL, 0xa043e4b51f7bb93dULL
};

__device__ __forceinline__ uint64_t mwc_jump5(uint64_t s, int L) {
    constexpr uint64_t A = 4164903690ULL;
    constexpr unsigned __int128 M = (((unsigned __int128)A) << 32) - 1;
    unsigned __int128 t = (unsigned __int128)s * kMwcJump5[L];
#pragma unroll
    for (int i = 0; i < 3; ++i) t = (t >> 32) + (unsigned __int128)(uint32_t)t * A;
    return (uint64_t)(t >= M ? t - M : t);
}

// nh <= 64 consecutive samples (5 distinct indices each, cv_rng_sample5's sequence) on the 64
// lanes of a wave: lane h draws sample h from the state 5 (h - b0) draws past the base; the first
// lane whose draws repeat an index redraws one at a time and the lanes after it restart from its
// final state.  rs: the state before the chunk (uniform), the state after it on return; sample h
// goes to out[5 h .. 5 h + 4].  (pnp.hip: a RANSAC chunk into LDS; ransac.hip: ess_pregen_kernel.)
__device__ __forceinline__ void cv_rng_sample_wave(uint64_t& rs, unsigned n, unsigned mg, int nh, int* out,
                                                   int lane) {
    constexpr uint64_t A = 4164903690ULL;
    uint64_t base = rs;
    int b0 = 0;
    for (;;) {
        const int L = lane - b0;
        const bool act = L >= 0 && lane < nh;
        const uint64_t st = L <= 0 ? base : mwc_jump5(base, min(L, 63));
        uint64_t sv = st;
        int d[5];
#pragma unroll
        for (int i = 0; i < 5; ++i) {
            sv = (uint64_t)(unsigned)sv * A + (unsigned)(sv >> 32);
            d[i] = (int)cv_rng_mod((unsigned)sv, n, mg);
        }
        bool dup = false;
#pragma unroll
        for (int i = 1; i < 5; ++i)
#pragma unroll
            for (int t = 0; t < i; ++t) dup = dup || d[t] == d[i];
        const uint64_t dm = __ballot(act && dup);
        const int hs = dm ? __ffsll((unsigned long long)dm) - 1 : nh;
        if (act && lane < hs) {
#pragma unroll
            for (int i = 0; i < 5; ++i) out[lane * 5 + i] = d[i];
        }
        if (hs >= nh) {
            rs = __shfl(sv, nh - 1);
            return;
        }
        uint64_t s2 = st;
        if (lane == hs) {
            cv_rng_sample5(s2, n, mg, d);
#pragma unroll
            for (int i = 0; i < 5; ++i) out[lane * 5 + i] = d[i];
        }
        base = __shfl(s2, hs);
        b0 = hs + 1;
        if (b0 >= nh) {
            rs = base;
            return;
        }
    }
}

}  // namespace sfmhip
