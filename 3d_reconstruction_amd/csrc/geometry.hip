// geometry.hip — S2 DLT triangulation, S3 reprojection residual, S5 scipy
// 2-point grouped finite-difference Jacobian; all f64, one thread per
// observation, contract off (the Makefile builds with -ffp-contract=off).
//
// Reference boundary:
//   cv2.triangulatePoints            sfm.py:27   (OpenCV calib3d DLT + cvSVD)
//   calculate_reprojection_error     sfm.py:87-91 -> cv2.projectPoints (no distortion)
//   least_squares(jac_sparsity=ba_sparse(...))   sfm.py:37-38, 79-85
//     -> scipy/optimize/_numdiff.py _compute_absolute_step / _sparse_difference
// Restated in oracle/geometry.py; the kernels follow the same op order.
#include "common.h"
#include "geom_dev.h"
#include <climits>

namespace sfmhip {

// scipy _compute_absolute_step for '2-point': EPS**0.5 * sign0(x) * max(1, |x|)
__device__ __forceinline__ double fd_step(double x) {
    const double rstep = 1.4901161193847656e-08;  // np.finfo(float64).eps ** 0.5
    const double sgn = (x >= 0.0) ? 1.0 : -1.0;
    return rstep * sgn * fmax(1.0, fabs(x));
}

// ---------------------------------------------------------------------------
__global__ void dlt_kernel(const double* __restrict__ P, const int32_t* __restrict__ pair_of_obs,
                           const double* __restrict__ x0, const double* __restrict__ x1, int64_t n,
                           double* __restrict__ X4) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int pr = pair_of_obs ? pair_of_obs[i] : 0;
    double X[4];
    dlt_point(P + (size_t)pr * 24, P + (size_t)pr * 24 + 12, x0[i], x0[n + i], x1[i], x1[n + i], X);
#pragma unroll
    for (int r = 0; r < 4; ++r) X4[(int64_t)r * n + i] = X[r];
}

// ---------------------------------------------------------------------------
// Rotation(s) of the block's camera: when every observation of the block
// belongs to one pair (sorted pair_of_obs, or a single pair), the first
// `nrot` threads build them once in LDS (R0 = R(rvec), R1..3 = R(rvec + h e_k)
// for the FD columns) instead of every thread re-evaluating sin/cos; values
// are identical either way.  Returns true if the LDS copy is valid.
__device__ __forceinline__ bool block_rotations(const double* __restrict__ cam,
                                                const int32_t* __restrict__ pair_of_obs, int64_t n, int nrot,
                                                double (*sR)[9]) {
    const int64_t i0 = (int64_t)blockIdx.x * blockDim.x;
    const int64_t i = min(i0 + (int64_t)threadIdx.x, n - 1);
    const int pr = pair_of_obs ? pair_of_obs[i] : 0;
    const int pr0 = pair_of_obs ? pair_of_obs[i0] : 0;
    const bool uniform = __syncthreads_and(pr == pr0);
    if (uniform && threadIdx.x < nrot) {
        const double* c = cam + (size_t)pr0 * 6;
        double p[3] = {c[0], c[1], c[2]};
        const int q = threadIdx.x - 1;
        if (q >= 0) p[q] = p[q] + fd_step(p[q]);
        rodrigues(p, sR[threadIdx.x]);
    }
    __syncthreads();
    return uniform;
}

__global__ void residual_kernel(const double* __restrict__ cam, const double* __restrict__ K,
                                const double* __restrict__ X, const double* __restrict__ pts2d,
                                const int32_t* __restrict__ pair_of_obs, int64_t n,
                                double* __restrict__ r) {
    __shared__ double sR[1][9];
    const bool shared_R = block_rotations(cam, pair_of_obs, n, 1, sR);
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int pr = pair_of_obs ? pair_of_obs[i] : 0;
    const double* c = cam + (size_t)pr * 6;
    const double* k = K + (size_t)pr * 9;
    double R[9];
    if (shared_R) {
#pragma unroll
        for (int e = 0; e < 9; ++e) R[e] = sR[0][e];
    } else {
        rodrigues(c, R);
    }
    const double Xp[3] = {X[3 * i], X[3 * i + 1], X[3 * i + 2]};
    double u, v;
    project(R, c + 3, Xp, k[0], k[4], k[2], k[5], u, v);
    r[2 * i] = pts2d[2 * i] - u;
    r[2 * i + 1] = pts2d[2 * i + 1] - v;
}

// Rotations of every pair for the FD Jacobian: Rt[pair][0] = R(rvec),
// Rt[pair][1 + k] = R(rvec + h_k e_k) (scipy's step h_k), one thread each —
// the sin/cos work is per pair, not per observation.
__global__ void fd_rotations_kernel(const double* __restrict__ cam, int n_pairs, double* __restrict__ Rt) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= 4 * n_pairs) return;
    const double* c = cam + (size_t)(t >> 2) * 6;
    double p[3] = {c[0], c[1], c[2]};
    const int q = (t & 3) - 1;
    if (q >= 0) p[q] = p[q] + fd_step(p[q]);
    rodrigues(p, Rt + (size_t)t * 9);
}

// 2-point FD: for each of the 9 parameters touching observation i, perturb it
// by h (scipy step), re-project, J = (f(x+h) - f0) / ((x+h) - x).  Groups of
// structurally orthogonal columns are perturbed together by scipy, but only
// one column of each group touches row i, so each value depends only on that
// column's perturbation (DESIGN.md "FD Jacobian").  Every projection is the
// op sequence of `project`; a perturbed t_k only changes the last addition of
// camera coordinate k, so those three re-use the base partial sums (the same
// operations, hence the same values).  The 18 values per observation are staged
// in LDS and written as one contiguous, coalesced block per workgroup.
constexpr int kFdThreads = 256;
__global__ __launch_bounds__(kFdThreads) void fdjac_kernel(const double* __restrict__ Rt,
                                                           const double* __restrict__ cam,
                                                           const double* __restrict__ K,
                                                           const double* __restrict__ X,
                                                           const double* __restrict__ pts2d,
                                                           const int32_t* __restrict__ pair_of_obs, int64_t n,
                                                           const double* __restrict__ f0, double* __restrict__ r,
                                                           double* __restrict__ jv) {
    __shared__ double sj[kFdThreads * 18];
    const int64_t i0 = (int64_t)blockIdx.x * kFdThreads;
    const int64_t i = i0 + threadIdx.x;
    if (i < n) {
        const int pr = pair_of_obs ? pair_of_obs[i] : 0;
        const double* c = cam + (size_t)pr * 6;
        const double* k = K + (size_t)pr * 9;
        const double* R = Rt + (size_t)pr * 36;
        const double fx = k[0], fy = k[4], cx = k[2], cy = k[5];
        const double obs_u = pts2d[2 * i], obs_v = pts2d[2 * i + 1];
        const double t[3] = {c[3], c[4], c[5]};
        const double Xp[3] = {X[3 * i], X[3 * i + 1], X[3 * i + 2]};
        // base projection, keeping the partial sums R X
        const double sx = R[0] * Xp[0] + R[1] * Xp[1] + R[2] * Xp[2];
        const double sy = R[3] * Xp[0] + R[4] * Xp[1] + R[5] * Xp[2];
        const double sz = R[6] * Xp[0] + R[7] * Xp[1] + R[8] * Xp[2];
        const double zb = sz + t[2];
        const double izb = (zb != 0.0) ? 1.0 / zb : 1.0;
        const double xb = (sx + t[0]) * izb, yb = (sy + t[1]) * izb;
        const double base_u = obs_u - (xb * fx + cx), base_v = obs_v - (yb * fy + cy);
        if (r) { r[2 * i] = base_u; r[2 * i + 1] = base_v; }
        const double f0u = f0 ? f0[2 * i] : base_u;
        const double f0v = f0 ? f0[2 * i + 1] : base_v;
        double* row = sj + threadIdx.x * 18;
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
    __syncthreads();
    // coalesced write-out of the workgroup's rows [i0, min(n, i0 + 256)) x 18 doubles
    const int64_t nv = (min(n, i0 + kFdThreads) - i0) * 18;
    double* out = jv + i0 * 18;
    for (int64_t e = threadIdx.x; e < nv; e += kFdThreads) out[e] = sj[e];
}

}  // namespace sfmhip

using namespace sfmhip;

extern "C" int sfmhip_triangulate_dlt(const double* P, const int32_t* pair_of_obs, const double* x0,
                                      const double* x1, int64_t n, double* X4, void* stream) {
    SFMHIP_REQUIRE(P && x0 && x1 && X4, "sfmhip_triangulate_dlt: null pointer");
    SFMHIP_REQUIRE(n >= 0, "sfmhip_triangulate_dlt: negative n");
    if (n == 0) return SFMHIP_OK;
    hipLaunchKernelGGL(dlt_kernel, dim3(ceil_div(n, 128)), dim3(128), 0, as_stream(stream), P,
                       pair_of_obs, x0, x1, n, X4);
    return check_launch("dlt_kernel");
}

extern "C" int sfmhip_reproj_residual(const double* cam, const double* K, const double* X,
                                      const double* pts2d, const int32_t* pair_of_obs, int64_t n,
                                      double* r, void* stream) {
    SFMHIP_REQUIRE(cam && K && X && pts2d && r, "sfmhip_reproj_residual: null pointer");
    SFMHIP_REQUIRE(n >= 0, "sfmhip_reproj_residual: negative n");
    if (n == 0) return SFMHIP_OK;
    hipLaunchKernelGGL(residual_kernel, dim3(ceil_div(n, 256)), dim3(256), 0, as_stream(stream), cam,
                       K, X, pts2d, pair_of_obs, n, r);
    return check_launch("residual_kernel");
}

extern "C" int sfmhip_reproj_fd_jacobian(const double* cam, const double* K, const double* X,
                                         const double* pts2d, const int32_t* pair_of_obs, int n_pairs,
                                         int64_t n, const double* f0, double* r, double* jvals,
                                         void* stream) {
    SFMHIP_REQUIRE(cam && K && X && pts2d && jvals, "sfmhip_reproj_fd_jacobian: null pointer");
    SFMHIP_REQUIRE(n >= 0 && n_pairs >= 1, "sfmhip_reproj_fd_jacobian: bad counts");
    if (n == 0) return SFMHIP_OK;
    hipStream_t st = as_stream(stream);
    double* Rt = nullptr;
    if (scratch_alloc((void**)&Rt, (size_t)n_pairs * 36 * sizeof(double), st) != hipSuccess) {
        (void)hipGetLastError();
        set_error("sfmhip_reproj_fd_jacobian: rotation table allocation failed");
        return SFMHIP_E_HIP;
    }
    hipLaunchKernelGGL(fd_rotations_kernel, dim3(ceil_div(4 * n_pairs, 64)), dim3(64), 0, st, cam, n_pairs, Rt);
    hipLaunchKernelGGL(fdjac_kernel, dim3(ceil_div(n, kFdThreads)), dim3(kFdThreads), 0, st, Rt, cam, K, X,
                       pts2d, pair_of_obs, n, f0, r, jvals);
    const int rc = check_launch("fdjac_kernel");
    (void)hipFreeAsync(Rt, st);
    return rc;
}
