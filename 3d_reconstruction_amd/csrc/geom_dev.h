// geom_dev.h — f64 device helpers shared by geometry.hip and ransac.hip:
// cv::Rodrigues (vector -> matrix), cv::projectPoints without distortion and
// the cvTriangulatePoints DLT for one correspondence.
#pragma once
#include <hip/hip_runtime.h>

namespace sfmhip {

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

// DLT: A (6x4) rows per view v: x*P[2]-P[0], y*P[2]-P[1], x*P[1]-y*P[0];
// one-sided (Hestenes) Jacobi on the 4 columns, V accumulates the rotations;
// the right singular vector of the smallest singular value is V's column with
// the smallest resulting column norm.  Output: unit norm, X[3] >= 0.
__device__ inline void dlt_point(const double* P0, const double* P1, double x0, double y0, double x1,
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

}  // namespace sfmhip
