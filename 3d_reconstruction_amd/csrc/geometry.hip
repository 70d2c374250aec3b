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
#include <cstring>
#include <mutex>
#include "geom_dev.h"
#include <climits>

namespace sfmhip {

// ---------------------------------------------------------------------------
// DLT, two passes (sfm.py:27, cv2.triangulatePoints).
//
// Fast pass (dlt_normal_kernel, one lane per observation, 72 VGPRs): the
// null vector of A (6x4) is the eigenvector of the smallest eigenvalue of the
// normal matrix M = A^T A (10 distinct sums of the 6 rank-1 row products).
// M = L D L^T (no pivoting; M is positive semi-definite), then inverse
// iteration started from L^-T e4 (= M^-1 applied to L e4), normalising each
// iterate, until two iterates agree to 1e-13 (factor lambda4/lambda3 per step:
// median 2e-7 on the C3 scene, so 2-3 steps).  Forming M squares A's
// condition, so a lane is kept only if a lower bound on lambda3 (the leading
// 3x3 block's smallest eigenvalue >= 1 / trace(M3^-1), by interlacing) is at
// least 1e-7 trace(M): the eigenvector's perturbation is then below ~1e-9.
// Lanes that fail either test (~1.2 % of C3 observations: small-baseline
// points whose lambda3 is tiny or close to lambda4) go to their wave's slot
// list, and the list pass decides them with the backward-stable Householder QR
// and a three-vector block inverse iteration (dlt_point_qr3; tried and dropped:
// a Rayleigh-quotient iteration on M for the slow-converging ones, 1.7e-8 off
// the SVD where lambda4/lambda3 -> 1 from M's rounding, and a two-vector block,
// 2e-7 off where sigma2 ~ sigma3), and with geom_dev.h's dlt_point (inverse
// iteration + 4x4 Jacobi) what that cannot decide.
typedef const double __attribute__((address_space(4))) const_f64;   // constant space: uniform -> s_load

// Listed observations: Householder QR of A (backward stable: no squaring of the
// condition), then a three-vector block inverse iteration with R's triangular
// solves and a 3x3 Rayleigh-Ritz.  On the C3 scene sigma1 (the x p2 - y p1
// rows, ~x f) exceeds sigma2..sigma4 (~f) by ~1e3, so the block {v2, v3, v4}
// converges at (sigma2/sigma1)^2 ~ 1e-5 per step whatever the sigma3/sigma4 gap
// (a two-vector block converges at (sigma3/sigma2)^2, ~0.5 on the listed
// points), and B^T B for B = R Z holds only lambda2..lambda4, so forming it
// costs no accuracy; cyclic Jacobi on that 3x3 finishes in a few sweeps.
// Fixed cost, no 4x4 Jacobi.  false: dlt_point decides.
__device__ inline bool dlt_point_qr3(const double* P0, const double* P1, double xa, double ya, double xb, double yb,
                                     double* Xout) {
    double R[4][4], rmax;
    dlt_qr<true>(P0, P1, xa, ya, xb, yb, R, rmax);
    double id[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        if (!(fabs(R[k][k]) > 1e-15 * rmax) || !(rmax < 1e300)) return false;
        id[k] = rcp_nr(R[k][k]);
    }
    auto bsolve = [&](double (&z)[4]) {   // R z = z
#pragma unroll
        for (int r = 3; r >= 0; --r) {
            double a = z[r];
#pragma unroll
            for (int c = r + 1; c < 4; ++c) a = fma(-R[r][c], z[c], a);
            z[r] = a * id[r];
        }
    };
    auto fsolve = [&](double (&z)[4]) {   // R^T z = z
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            double a = z[r];
#pragma unroll
            for (int c = 0; c < r; ++c) a = fma(-R[c][r], z[c], a);
            z[r] = a * id[r];
        }
    };
    auto dot = [](const double (&u)[4], const double (&v)[4]) {
        return fma(u[0], v[0], fma(u[1], v[1], fma(u[2], v[2], u[3] * v[3])));
    };
    auto unit = [&](double (&u)[4]) {
        const double sc = rsq_nr(dot(u, u));
#pragma unroll
        for (int k = 0; k < 4; ++k) u[k] *= sc;
    };
    auto drop = [&](const double (&u)[4], double (&v)[4]) {   // v -= (u.v) u, twice
#pragma unroll
        for (int pass = 0; pass < 2; ++pass) {
            const double c = dot(u, v);
#pragma unroll
            for (int k = 0; k < 4; ++k) v[k] = fma(-c, u[k], v[k]);
        }
    };
    double Z[3][4] = {{0, 0, 0, 1}, {0, 0, 1, 0}, {0, 1, 0, 0}};   // R^-1 [e4 e3 e2]
    auto orth = [&]() {
        unit(Z[0]);
        drop(Z[0], Z[1]);
        unit(Z[1]);
        drop(Z[0], Z[2]);
        drop(Z[1], Z[2]);
        unit(Z[2]);
    };
#pragma unroll
    for (int k = 0; k < 3; ++k) bsolve(Z[k]);
#pragma unroll 1
    for (int it = 0; it < 2; ++it) {   // 2 steps: 1e-13 on the C3 and test scenes (1 step: 8e-10)
        orth();
#pragma unroll
        for (int k = 0; k < 3; ++k) { fsolve(Z[k]); bsolve(Z[k]); }
    }
    orth();
    double B[3][4];   // B = R Z
#pragma unroll
    for (int k = 0; k < 3; ++k)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            double a = 0.0;
#pragma unroll
            for (int c = r; c < 4; ++c) a = fma(R[r][c], Z[k][c], a);
            B[k][r] = a;
        }
    double G[3][3], V[3][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = i; j < 3; ++j) G[i][j] = G[j][i] = dot(B[i], B[j]);
    for (int sweep = 0; sweep < 12; ++sweep) {
        bool rotated = false;
#pragma unroll
        for (int p = 0; p < 2; ++p)
#pragma unroll
            for (int q = p + 1; q < 3; ++q) {
                const double gpq = G[p][q];
                // |g_pq| <= 1e-18 sqrt(|g_pp g_qq|), squared: no square root on the rotation chain
                if (gpq * gpq <= 1e-36 * fabs(G[p][p] * G[q][q])) continue;
                rotated = true;
                const double zeta = (G[q][q] - G[p][p]) * (0.5 * rcp_nr(gpq));
                const double t = (zeta >= 0.0 ? 1.0 : -1.0) * rcp_nr(fabs(zeta) + sqrt_nr(fma(zeta, zeta, 1.0)));
                const double c = rsq_nr(fma(t, t, 1.0)), sn = t * c;
                // G <- J^T G J with J = [[c, sn], [-sn, c]] on (p, q)
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    const double gkp = G[k][p], gkq = G[k][q];
                    G[k][p] = c * gkp - sn * gkq;
                    G[k][q] = sn * gkp + c * gkq;
                }
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    const double gpk = G[p][k], gqk = G[q][k];
                    G[p][k] = c * gpk - sn * gqk;
                    G[q][k] = sn * gpk + c * gqk;
                }
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    const double vkp = V[k][p], vkq = V[k][q];
                    V[k][p] = c * vkp - sn * vkq;
                    V[k][q] = sn * vkp + c * vkq;
                }
            }
        if (!rotated) break;
    }
    int best = 0;
#pragma unroll
    for (int k = 1; k < 3; ++k)
        if (G[k][k] < G[best][best]) best = k;
    double u[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) u[k] = best == 0 ? V[k][0] : (best == 1 ? V[k][1] : V[k][2]);
    double y[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) y[r] = fma(u[0], Z[0][r], fma(u[1], Z[1][r], u[2] * Z[2][r]));
    return dlt_store_unit(y[0], y[1], y[2], y[3], Xout);
}

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8))) void dlt_normal_kernel(const double* __restrict__ P,
                                                         const int32_t* __restrict__ pair_of_obs,
                                                         const double* __restrict__ x0, const double* __restrict__ x1,
                                                         int64_t n, double* __restrict__ X4,
                                                         unsigned* __restrict__ slots, unsigned* __restrict__ counts,
                                                         double4* __restrict__ recx, int* __restrict__ recpr) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t wave = i >> 6;   // global wave index (n_waves = ceil(n / 64) slots of 64)
    if (i >= n) return;
    const int pr = pair_of_obs ? pair_of_obs[i] : 0;
    const double xa = x0[i], ya = x0[n + i], xb = x1[i], yb = x1[n + i];
    double X[4];
    int st = 2;
    // waterfall over the wave's pairs (sorted observations: one or two per wave),
    // so each pair's projection matrices are wave-uniform scalar loads
    while (true) {
        const int cur = __builtin_amdgcn_readfirstlane(pr);
        int cs = cur;
        asm volatile("" : "+s"(cs));   // an opaque SGPR copy: under pr == cur the compiler would address with pr
        if (pr == cur) {
            st = dlt_point_normal((const const_f64*)(P + (size_t)cs * 24), xa, ya, xb, yb, X);
            break;
        }
    }
    if (st == 0) {
#pragma unroll
        for (int r = 0; r < 4; ++r) X4[(int64_t)r * n + i] = X[r];
    }
    // the undecided lanes go to this wave's own 64-entry slot, the count to counts[wave]: no atomics (one returning
    // atomic per wave on a shared counter serialised the kernel: 101 us, 71 % of
    // wave cycles waiting)
    const unsigned long long m = __ballot(st != 0);
    const int lane = threadIdx.x & 63;
    if (st != 0) {   // the slot carries the observation (index, pair, both image points): the list pass
                     // then needs one dependent load level less
        const int64_t pos = (wave << 6) + __popcll(m & ((1ull << lane) - 1ull));
        slots[pos] = (unsigned)i;
        recx[pos] = make_double4(xa, ya, xb, yb);
        recpr[pos] = pr;
    }
    if (lane == __ffsll((long long)__ballot(true)) - 1) counts[wave] = (unsigned)__popcll(m);
}

// List pass: one 64-lane workgroup per 64 source waves gathers their slots
// densely into LDS (prefix sum of the counts across lanes); each lane then
// decides one gathered observation at a time.
__global__ __launch_bounds__(64) void dlt_list_kernel(const double* __restrict__ P,
                                                      const int32_t* __restrict__ pair_of_obs,
                                                      const double* __restrict__ x0, const double* __restrict__ x1,
                                                      int64_t n, double* __restrict__ X4,
                                                      const unsigned* __restrict__ slots,
                                                      const unsigned* __restrict__ counts,
                                                      const double4* __restrict__ recx, const int* __restrict__ recpr,
                                                      int64_t n_waves) {
    __shared__ unsigned items[64 * 64];
    const int lane = threadIdx.x;
    const int64_t w = (int64_t)blockIdx.x * 64 + lane;
    const unsigned c = w < n_waves ? counts[w] : 0u;
    unsigned pre = c;   // inclusive scan over the 64 lanes
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const unsigned t = __shfl_up(pre, d);
        if (lane >= d) pre += t;
    }
    const unsigned total = __shfl(pre, 63);
    if (total == 0) return;
    for (unsigned t = 0; t < c; ++t) items[pre - c + t] = (unsigned)((w << 6) + t);   // slot positions
    __syncthreads();
    for (unsigned k = lane; k < total; k += 64) {
        const unsigned pos = items[k];
        const int64_t i = slots[pos];
        const int pr = recpr[pos];
        const double4 xr = recx[pos];
        double X[4];
        const double *Pa = P + (size_t)pr * 24, xa = xr.x, ya = xr.y, xb = xr.z, yb = xr.w;
        if (!dlt_point_qr3(Pa, Pa + 12, xa, ya, xb, yb, X)) dlt_point(Pa, Pa + 12, xa, ya, xb, yb, X);
#pragma unroll
        for (int r = 0; r < 4; ++r) X4[(int64_t)r * n + i] = X[r];
    }
}

// the QR path for every observation (SFMHIP_DLT_QR=1, tests; scratch failure)
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
        fd_obs(Rt + (size_t)pr * 36, c, k, X + 3 * i, pts2d[2 * i], pts2d[2 * i + 1], f0 ? f0 + 2 * i : nullptr,
               r ? r + 2 * i : nullptr, sj + threadIdx.x * 18);
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
    SFMHIP_REQUIRE(n >= 0, "sfmhip_triangulate_dlt: negative n");
    if (n == 0) return SFMHIP_OK;
    SFMHIP_REQUIRE(P && x0 && x1 && X4, "sfmhip_triangulate_dlt: null pointer");
    hipStream_t st = as_stream(stream);
    unsigned* slots = nullptr;   // [n_waves][64] listed observations + [n_waves] counts
    const int64_t n_waves = ceil_div(n, 64);
    // SFMHIP_DLT_QR=1 (tests): the QR path for every observation, as on a scratch failure
    if (knobs().dlt_qr == 0 && n < ((int64_t)1 << 31) &&
        scratch_alloc((void**)&slots, (size_t)ceil_div(n_waves * 65, (int64_t)8) * 32 + (size_t)n_waves * 64 * 36, st) ==
            hipSuccess) {
        // [n_waves * 64] indices, [n_waves] counts, then (32-B aligned) the listed observations'
        // points (double4) and pairs (int), at the same slot positions
        unsigned* counts = slots + n_waves * 64;
        double4* recx = reinterpret_cast<double4*>(slots + ceil_div(n_waves * 65, (int64_t)8) * 8);
        int* recpr = reinterpret_cast<int*>(recx + n_waves * 64);
        hipLaunchKernelGGL(dlt_normal_kernel, dim3(ceil_div(n, 256)), dim3(256), 0, st, P, pair_of_obs, x0, x1, n,
                           X4, slots, counts, recx, recpr);
        int rc = check_launch("dlt_normal_kernel");
        if (rc == SFMHIP_OK) {
            hipLaunchKernelGGL(dlt_list_kernel, dim3((unsigned)ceil_div(n_waves, 64)), dim3(64), 0, st, P, pair_of_obs,
                               x0, x1, n, X4, slots, counts, recx, recpr, n_waves);
            rc = check_launch("dlt_list_kernel");
        }
        scratch_free(slots, st);
        return rc;
    }
    (void)hipGetLastError();
    hipLaunchKernelGGL(dlt_kernel, dim3(ceil_div(n, 128)), dim3(128), 0, st, P, pair_of_obs, x0, x1, n, X4);
    return check_launch("dlt_kernel");
}

extern "C" int sfmhip_reproj_residual(const double* cam, const double* K, const double* X,
                                      const double* pts2d, const int32_t* pair_of_obs, int64_t n,
                                      double* r, void* stream) {
    SFMHIP_REQUIRE(n >= 0, "sfmhip_reproj_residual: negative n");
    if (n == 0) return SFMHIP_OK;
    SFMHIP_REQUIRE(cam && K && X && pts2d && r, "sfmhip_reproj_residual: null pointer");
    hipLaunchKernelGGL(residual_kernel, dim3(ceil_div(n, 256)), dim3(256), 0, as_stream(stream), cam,
                       K, X, pts2d, pair_of_obs, n, r);
    return check_launch("residual_kernel");
}

// Host-array form of sfmhip_reproj_residual for the cv2/scipy contract (sfm.py:87-91 called by
// least_squares ~60 times per pair at sfm.py:38): the inputs are packed into one pinned staging
// buffer that the kernel reads over PCIe and writes the residual back into (zero-copy, ~224 B per
// observation), then one stream synchronisation — no copies, no per-call device allocation.  The
// staging buffer is library-owned per device and grows on demand.
namespace {
struct HostStage {
    std::mutex mu;
    double* h = nullptr;   // pinned, device-accessible: [cam 6 | K 9 | pad 1 | X 3n | pts 2n | r 2n]
    size_t cap = 0;        // doubles
};
HostStage g_stage[64];
}  // namespace

extern "C" int sfmhip_reproj_residual_host(const double* cam, const double* K, const double* X,
                                           const double* pts2d, int64_t n, double* r, void* stream) {
    SFMHIP_REQUIRE(n >= 0 && n < ((int64_t)1 << 40), "sfmhip_reproj_residual_host: bad n");
    if (n == 0) return SFMHIP_OK;
    SFMHIP_REQUIRE(cam && K && X && r, "sfmhip_reproj_residual_host: null pointer");
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) {
        (void)hipGetLastError();
        set_error("sfmhip_reproj_residual_host: no current HIP device");
        return SFMHIP_E_HIP;
    }
    HostStage& st = g_stage[dev];
    std::lock_guard<std::mutex> lk(st.mu);
    const size_t need = 16 + 7 * (size_t)n;
    if (st.cap < need) {
        if (st.h) (void)hipHostFree(st.h);
        st.h = nullptr;
        st.cap = 0;
        const size_t cap = need + need / 2;
        if (hipHostMalloc((void**)&st.h, cap * sizeof(double), hipHostMallocMapped) != hipSuccess) {
            (void)hipGetLastError();
            st.h = nullptr;
            set_error("sfmhip_reproj_residual_host: staging allocation failed");
            return SFMHIP_E_HIP;
        }
        st.cap = cap;
    }
    double* h = st.h;
    std::memcpy(h, cam, 6 * sizeof(double));
    std::memcpy(h + 6, K, 9 * sizeof(double));
    h[15] = 0.0;
    std::memcpy(h + 16, X, 3 * (size_t)n * sizeof(double));
    if (pts2d) std::memcpy(h + 16 + 3 * n, pts2d, 2 * (size_t)n * sizeof(double));
    else std::memset(h + 16 + 3 * n, 0, 2 * (size_t)n * sizeof(double));
    hipStream_t s = as_stream(stream);
    double* d = nullptr;
    hipError_t e = hipHostGetDevicePointer((void**)&d, h, 0);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(residual_kernel, dim3(ceil_div(n, 256)), dim3(256), 0, s, d, d + 6, d + 16,
                           d + 16 + 3 * n, nullptr, n, d + 16 + 5 * n);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        set_error("sfmhip_reproj_residual_host: %s", hipGetErrorString(e));
        return SFMHIP_E_HIP;
    }
    std::memcpy(r, h + 16 + 5 * n, 2 * (size_t)n * sizeof(double));
    return SFMHIP_OK;
}

extern "C" int sfmhip_reproj_fd_jacobian(const double* cam, const double* K, const double* X,
                                         const double* pts2d, const int32_t* pair_of_obs, int n_pairs,
                                         int64_t n, const double* f0, double* r, double* jvals,
                                         void* stream) {
    SFMHIP_REQUIRE(n >= 0 && n_pairs >= 1, "sfmhip_reproj_fd_jacobian: bad counts");
    if (n == 0) return SFMHIP_OK;
    SFMHIP_REQUIRE(cam && K && X && pts2d && jvals, "sfmhip_reproj_fd_jacobian: null pointer");
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
    scratch_free(Rt, st);
    return rc;
}
