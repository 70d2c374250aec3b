// ba.hip — the BA solve of sfm.py:37-38 on the GPU, all pairs at once:
//   least_squares(calculate_reprojection_error, [rvec, t, X...], jac_sparsity=
//                 ba_sparse(...), x_scale='jac', ftol=1e-8, args=(K, pts1))
// i.e. scipy's 'trf' with tr_solver 'lsmr' and the grouped 2-point FD
// Jacobian, restated on the BA structure (oracle/ba.py is the same algorithm
// in numpy, pinned against scipy itself by tests/test_oracle_ba.py):
//   * J: scipy's FD values per observation (geom_dev.h fd_obs), 2x6 camera +
//     2x3 point block, scale = 1 / column norms (max with the previous ones);
//   * the Gauss-Newton direction lsmr(J_h, f, damp = sqrt(reg)) (scipy stops
//     LSMR at atol = btol = 1e-6) is the EXACT damped solution
//     J_h^T (J_h J_h^T + mu I)^-1 f by Woodbury over the 2x2 point blocks
//     (one 6x6 Cholesky per iteration);
//   * the 2-D subspace {g_h, gn_h}, its trust-region solve, the radius update
//     and the ftol / xtol / gtol tests as scipy's trf_no_bounds.
// One workgroup per pair (the pair's observations are a contiguous range), the
// per-observation J / f / column scales in a scratch record, every scalar of
// the iteration reduced across the workgroup and held in LDS; thread 0 does the
// 6x6 and 2x2 algebra.
#include "common.h"
#include <mutex>
#include "geom_dev.h"
#include <climits>
#include <cstdlib>

namespace sfmhip {
namespace {

#ifdef SFMHIP_BA_PROF
// phase timing of the solve kernel (thread 0, wall clock at 100 MHz), a tool-only build
// (make EXTRA=-DSFMHIP_BA_PROF; tools/ba_phase_prof.py): never in the product library
constexpr int kProfPhases = 10;
__device__ unsigned long long g_ba_prof[4096 * kProfPhases];
#define BA_MARK(k)                                                   \
    do {                                                             \
        if (threadIdx.x == 0) {                                      \
            const unsigned long long t_ = wall_clock64();            \
            prof_acc[k] += t_ - prof_t;                              \
            prof_t = t_;                                             \
        }                                                            \
    } while (0)
#else
#define BA_MARK(k) \
    do {           \
    } while (0)
#endif

// Tool-only audit builds (tools/ba_audit.sh; never the product library): SFMHIP_BA_AUDIT puts a full
// wait + workgroup barrier at every phase boundary and around every pass over the records (a missing
// barrier or an LDS / global ordering race in the shipped kernel would change its bits); SFMHIP_BA_PRINTF
// adds an inert printf inside every pass (never executed: p < 0), which changes register allocation,
// spills and scheduling — the symptom round 5's fused prototype showed.  Both must give the product
// build's bits on the bench batch.
#if defined(SFMHIP_BA_AUDIT)
#define BA_AUDIT()                          \
    do {                                    \
        __builtin_amdgcn_s_waitcnt(0);      \
        __threadfence_block();              \
        __syncthreads();                    \
    } while (0)
#else
#define BA_AUDIT() \
    do {           \
    } while (0)
#endif
#if defined(SFMHIP_BA_PRINTF)
#define BA_PRINTF(i)                                                         \
    do {                                                                     \
        if (p < 0) printf("ba pair %d obs %d nfev %d\n", p, (int)(i), S.nfev); \
    } while (0)
#else
#define BA_PRINTF(i) \
    do {             \
    } while (0)
#endif

// per observation: J (18: u row, v row; the point block stored scaled, J_p d with the point's
// column scales d = 1 / scale_inv), f (2), X_new (3), scale_inv (3: the column norms, max'ed
// across Jacobian evaluations).  d itself is not stored: the trial pass, the one pass that needs
// it alone, forms the same IEEE quotient 1 / scale_inv again (round 5: 29 -> 26 fields, the
// records of all 256 C3 pairs 243 -> 218 MB)
constexpr int kRec = 26;
constexpr int kFX = 20, kFS = 23;   // X_new, scale_inv
constexpr int kBaLdsObs = 768;       // observations per pair whose records stay in LDS (156 KB)

// sum of K doubles over the workgroup (NW waves); every thread receives the totals in out[]
template <int NW, int K>
__device__ void block_sum(double (&v)[K], double* red /* [NW][K] */, double* out /* [K] */) {
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
#pragma unroll
    for (int k = 0; k < K; ++k) {
        double x = v[k];
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) x += __shfl_xor(x, off);
        v[k] = x;
    }
    if (lane == 0)
#pragma unroll
        for (int k = 0; k < K; ++k) red[wave * K + k] = v[k];
    __syncthreads();
    if (threadIdx.x < K) {   // pairwise over the waves, a fixed order
        double t[NW];
#pragma unroll
        for (int w = 0; w < NW; ++w) t[w] = red[w * K + threadIdx.x];
#pragma unroll
        for (int h = NW / 2; h >= 1; h >>= 1)
#pragma unroll
            for (int w = 0; w < h; ++w) t[w] = t[w] + t[w + h];
        out[threadIdx.x] = t[0];
    }
    __syncthreads();
}

template <int NW>
__device__ double block_max(double v, double* red) {
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v = fmax(v, __shfl_xor(v, off));
    if (lane == 0) red[wave] = v;
    __syncthreads();
    double m = red[0];
#pragma unroll
    for (int w = 1; w < NW; ++w) m = fmax(m, red[w]);
    __syncthreads();
    return m;
}

// 6x6 SPD solve (lower Cholesky), in place on b; false if not positive definite
__device__ bool chol6_solve(double (&A)[6][6], double (&b)[6]) {
    for (int j = 0; j < 6; ++j) {
        double s = A[j][j];
        for (int k = 0; k < j; ++k) s -= A[j][k] * A[j][k];
        if (!(s > 0.0)) return false;
        const double d = sqrt(s);
        A[j][j] = d;
        for (int i = j + 1; i < 6; ++i) {
            double t = A[i][j];
            for (int k = 0; k < j; ++k) t -= A[i][k] * A[j][k];
            A[i][j] = t / d;
        }
    }
    for (int i = 0; i < 6; ++i) {
        double t = b[i];
        for (int k = 0; k < i; ++k) t -= A[i][k] * b[k];
        b[i] = t / A[i][i];
    }
    for (int i = 5; i >= 0; --i) {
        double t = b[i];
        for (int k = i + 1; k < 6; ++k) t -= A[k][i] * b[k];
        b[i] = t / A[i][i];
    }
    return true;
}

// scipy solve_trust_region_2d on a whole wave (every lane returns the same p): the
// interior Newton point if B is positive definite and it fits, else the minimiser of
// the quadratic on the circle |p| = Delta (scipy takes the best real root of its
// quartic; here the same point from a 64-angle scan, lane l at 2 pi l / 64, lowest
// index on ties, refined by Newton on the angle).  On one thread the scan's 128
// sin/cos took up to 150 us of a pair's solve (tools/ba_phase_prof.py).
__device__ void tr_solve_2d_wave(const double B[3], const double g[2], double Delta, double p[2]) {
    const double b00 = B[0], b01 = B[1], b11 = B[2];
    if (b00 > 0.0) {
        const double l00 = sqrt(b00), l10 = b01 / l00, s = b11 - l10 * l10;
        if (s > 0.0) {
            const double l11 = sqrt(s);
            const double y0 = g[0] / l00, y1 = (g[1] - l10 * y0) / l11;
            const double x1 = y1 / l11, x0 = (y0 - l10 * x1) / l00;
            if (x0 * x0 + x1 * x1 <= Delta * Delta) { p[0] = -x0; p[1] = -x1; return; }
        }
    }
    auto val = [&](double ph) {
        const double c = cos(ph), s = sin(ph);
        return 0.5 * Delta * Delta * (b00 * c * c + 2.0 * b01 * c * s + b11 * s * s) + Delta * (g[0] * c + g[1] * s);
    };
    const int lane = threadIdx.x & 63;
    constexpr int kScan = 64;
    double bv = val(lane == 0 ? 0.0 : 6.283185307179586 * lane / kScan);
    int bi = lane;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {   // (value, index) min, lowest index on ties
        const double ov = __shfl_xor(bv, off);
        const int oi = __shfl_xor(bi, off);
        if (ov < bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
    }
    double best = bi == 0 ? 0.0 : 6.283185307179586 * bi / kScan;
    for (int it = 0; it < 40; ++it) {   // Newton on dq/dphi
        const double c = cos(best), s = sin(best);
        const double d1 = Delta * Delta * ((b11 - b00) * c * s + b01 * (c * c - s * s)) + Delta * (g[1] * c - g[0] * s);
        const double d2 = Delta * Delta * ((b11 - b00) * (c * c - s * s) - 4.0 * b01 * c * s) - Delta * (g[0] * c + g[1] * s);
        if (!(d2 > 0.0)) break;
        const double step = d1 / d2;
        best -= step;
        if (fabs(step) < 1e-16) break;
    }
    p[0] = Delta * cos(best);
    p[1] = Delta * sin(best);
}

template <int NW>
struct BaState {   // LDS: the iteration's scalars, written by thread 0 or by block_sum
    double cam[6], cam_new[6], R[4][9], Rn[9];
    double gc[6], sic[6], dc[6], ghc[6], gnc[6], s1c[6], s2c[6], shc[6];
    double G[6][6], z[6];
    double red[NW * 27], tot[27];
    double Delta, mu, cost, cost_new, pS[2];
    double gmax, gh2, ghn, c12, s2n, BS[3], gS[2];
    int status, nfev, njev, done, accept;
};

// A pair's observation records in the scratch block of kRec doubles per
// observation, field-major within the pair (field f of record i at f * n + i: a
// wave's load of one field is 64 consecutive doubles; AoS records measured slower,
// profiles/r3/ba_variants_r3m.txt).  Passes copy the fields they use into registers.
// The records of the first L observations live in LDS instead (field f of record i < L at
// lds[f L + i]); i = tid + k NT with L a multiple of the wave size keeps the choice uniform per
// wave.  kLdsF < kRec would keep only the pass fields there (more observations per byte): it
// spilled 76 VGPRs instead of 36 and measured slower (1.26 vs 1.15 ms).
constexpr int kLdsF = kRec;
template <bool USE_LDS>
struct RecsT {
    double* base;
    int n;
    __attribute__((address_space(3))) double* lds;   // dynamic LDS, L * kLdsF doubles (L = 0: none)
    int L;
    __device__ __forceinline__ double* at(int i, int f) const {   // (scratch fields only)
        return base + (size_t)f * n + i;
    }
    template <int LO, int HI>
    __device__ __forceinline__ void load(int i, double* r) const {
        constexpr int M = HI < kLdsF ? HI : kLdsF, G0 = LO > kLdsF ? LO : kLdsF;
        if (USE_LDS && LO < kLdsF && i < L) {
#pragma unroll
            for (int f = LO; f < M; ++f) r[f] = lds[f * L + i];
#pragma unroll
            for (int f = G0; f < HI; ++f) r[f] = base[(size_t)f * n + i];
        } else {
#pragma unroll
            for (int f = LO; f < HI; ++f) r[f] = base[(size_t)f * n + i];
        }
    }
    template <int LO, int HI>
    __device__ __forceinline__ void store(int i, const double* r) const {
        constexpr int M = HI < kLdsF ? HI : kLdsF, G0 = LO > kLdsF ? LO : kLdsF;
        if (USE_LDS && LO < kLdsF && i < L) {
#pragma unroll
            for (int f = LO; f < M; ++f) lds[f * L + i] = r[f];
#pragma unroll
            for (int f = G0; f < HI; ++f) base[(size_t)f * n + i] = r[f];
        } else {
#pragma unroll
            for (int f = LO; f < HI; ++f) base[(size_t)f * n + i] = r[f];
        }
    }
};

// for i = tid, tid + NT, ... < n: body(i, r) with r[LO, HI) = record i, the next
// record's loads issued before the current one's arithmetic (one record ahead)
template <int NT, int LO, int HI, typename R, typename F>
__device__ __forceinline__ void stream_recs(const R& rec, int n, F&& body) {
    double nx[kRec];
    int i = threadIdx.x;
    if (i < n) rec.template load<LO, HI>(i, nx);
    for (; i < n; i += NT) {
        double r[kRec];
#pragma unroll
        for (int f = LO; f < HI; ++f) r[f] = nx[f];
        if (i + NT < n) rec.template load<LO, HI>(i + NT, nx);
        body(i, r);
    }
}

// residual of one observation at (camera rotation R, c = [rvec, t], X)
__device__ __forceinline__ void resid(const double* R, const double* c, const double* k, const double* X,
                                      const double* pts, double& ru, double& rv) {
    double u, v;
    project(R, c + 3, X, k[0], k[4], k[2], k[5], u, v);
    ru = pts[0] - u;
    rv = pts[1] - v;
}

// FUSED: the Jacobian at the trial point is formed inside the trial pass into a second record set
// (taken, with the trial's sums, when the step is accepted: nfev ~ njev on the bench scenes), so an
// accepted step costs no separate Jacobian sweep; the records then carry the point of their
// Jacobian (fields kFX) and X is written once at the end.  The same arithmetic in the same order
// as the two-pass form (the trial's residual IS fd_obs's base residual), so the same bits.
template <int NT, bool FUSED = false>
__global__ __launch_bounds__(NT) void ba_trf_kernel(double* __restrict__ cam_io, const double* __restrict__ Kall,
                                                    double* __restrict__ X, const double* __restrict__ pts2d,
                                                    const int64_t* __restrict__ off, int64_t n_obs, double ftol,
                                                    double xtol, double gtol, int max_nfev_arg,
                                                    double* __restrict__ scratch, double* __restrict__ cost_out,
                                                    int32_t* __restrict__ nfev_out, int32_t* __restrict__ njev_out,
                                                    int32_t* __restrict__ status_out, int lds_obs) {
    constexpr int NW = NT / 64;
    __shared__ BaState<NW> S;
    extern __shared__ __attribute__((aligned(16))) double lrec[];   // lds_obs * kLdsF (not FUSED)
    const int p = blockIdx.x, tid = threadIdx.x;
    const int64_t o0 = off[p], o1 = off[p + 1];
    if (!(0 <= o0 && o0 <= o1 && o1 <= n_obs && o1 - o0 <= INT_MAX)) {   // malformed offsets: touch nothing
        if (tid == 0) { cost_out[p] = 0.0; nfev_out[p] = 0; njev_out[p] = 0; status_out[p] = -1; }
        return;
    }
    const int n = (int)(o1 - o0);
    const double* k = Kall + (size_t)p * 9;
    double* Xp = X + 3 * o0;
    const double* pts = pts2d + 2 * o0;
    // FUSED: two record sets (the current one and the trial point's), scratch holds 2 n_obs records
    const int L = FUSED ? 0 : min(lds_obs, n);
    using Recs = RecsT<!FUSED>;
    auto* lr = (__attribute__((address_space(3))) double*)lrec;
    const Recs recs[2] = {{scratch + (size_t)o0 * kRec, n, lr, L}, {scratch + (size_t)(n_obs + o0) * kRec, n, lr, 0}};
    int cur = 0;   // every thread flips it at the same point (after a barrier): uniform
    // the pass view of observation i: r[0..17] J, r[18..19] f; the records hold the point block
    // of J already scaled, Pp = J_p d (fields 6-8, 15-17), so the passes read 20 fields
    // (round 5: 1.33 -> 1.27 ms); the trial pass adds scale_inv (its d = 1 / scale_inv)
    auto pass_rec = [&](int i, double* r) { recs[cur].template load<0, 20>(i, r); };
    auto pass_rec_d = [&](int i, double* r) {
        recs[cur].template load<0, 20>(i, r);
        recs[cur].template load<kFS, kFS + 3>(i, r);
    };
    if (tid < 6) S.cam[tid] = cam_io[(size_t)p * 6 + tid];
    __syncthreads();
    if (n == 0) {
        if (tid == 0) { cost_out[p] = 0.0; nfev_out[p] = 0; njev_out[p] = 0; status_out[p] = 1; }
        return;
    }
    const int max_nfev = max_nfev_arg > 0 ? max_nfev_arg : (int)min((int64_t)INT_MAX, 100 * (6 + 3 * (int64_t)n));
#ifdef SFMHIP_BA_PROF
    unsigned long long prof_acc[kProfPhases] = {}, prof_t = wall_clock64();
    const unsigned long long prof_t0 = prof_t;   // slots 8, 9: the pair's start and end
#endif

    // J, f at the current point; scale_inv (max with the old unless first); gc, cost, |g|_inf.
    // moved: the point is the accepted trial point, read from the records (X_new fields)
    // and written to X here (no separate pass to move X)
    auto jacobian = [&](bool first, bool moved) {
        if (tid < 4) {   // R(rvec) and the three perturbed rotations of the FD
            double q[3] = {S.cam[0], S.cam[1], S.cam[2]};
            if (tid > 0) q[tid - 1] = q[tid - 1] + fd_step(q[tid - 1]);
            rodrigues(q, S.R[tid]);
        }
        __syncthreads();
        double acc[13] = {0};   // gc (6), column sums of squares (6), cost
        double gmax = 0.0;
        BA_AUDIT();
        for (int i = tid; i < n; i += NT) {
            BA_PRINTF(i);
            double r[kRec];
            double f[2], Xi[3];
            if (moved) {
                recs[cur].template load<kFX, kFX + 3>(i, r);
                for (int c = 0; c < 3; ++c) { Xi[c] = r[kFX + c]; Xp[3 * i + c] = Xi[c]; }
            } else {
                for (int c = 0; c < 3; ++c) Xi[c] = Xp[3 * i + c];
            }
            if (!first) recs[cur].template load<kFS, kFS + 3>(i, r);
            fd_obs(&S.R[0][0], S.cam, k, Xi, pts[2 * i], pts[2 * i + 1], nullptr, f, r);
            r[18] = f[0];
            r[19] = f[1];
            acc[12] += f[0] * f[0] + f[1] * f[1];
#pragma unroll
            for (int c = 0; c < 6; ++c) {
                acc[c] += r[c] * f[0] + r[9 + c] * f[1];
                acc[6 + c] += r[c] * r[c] + r[9 + c] * r[9 + c];
            }
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                const double gp = r[6 + c] * f[0] + r[15 + c] * f[1];
                gmax = fmax(gmax, fabs(gp));
                double si = sqrt(r[6 + c] * r[6 + c] + r[15 + c] * r[15 + c]);
                if (first) si = si == 0.0 ? 1.0 : si;
                else si = fmax(si, r[kFS + c]);
                r[kFS + c] = si;
                const double d = 1.0 / si;
                r[6 + c] = r[6 + c] * d;   // Pp
                r[15 + c] = r[15 + c] * d;
            }
            recs[cur].template store<0, 20>(i, r);
            recs[cur].template store<kFS, kFS + 3>(i, r);
            if (FUSED) {   // the point of this Jacobian (X is read from the records from now on)
                for (int c = 0; c < 3; ++c) r[kFX + c] = Xi[c];
                recs[cur].template store<kFX, kFX + 3>(i, r);
            }
        }
        gmax = block_max<NW>(gmax, S.red);
        BA_AUDIT();
        block_sum<NW, 13>(acc, S.red, S.tot);
        BA_AUDIT();
        if (tid == 0) {
            double gm = gmax;
            for (int c = 0; c < 6; ++c) {
                S.gc[c] = S.tot[c];
                gm = fmax(gm, fabs(S.gc[c]));
                const double si = sqrt(S.tot[6 + c]);
                S.sic[c] = first ? (si == 0.0 ? 1.0 : si) : fmax(si, S.sic[c]);
            }
            S.gmax = gm;
            S.cost = 0.5 * S.tot[12];
        }
        __syncthreads();
    };

    jacobian(true, false);
    BA_MARK(0);
    // Delta = |x0 * scale_inv|
    {
        double acc[1] = {0.0};
        BA_AUDIT();
        for (int i = tid; i < n; i += NT) {
            BA_PRINTF(i);
            double r[kRec];
            recs[cur].template load<kFS, kFS + 3>(i, r);
            for (int c = 0; c < 3; ++c) { const double t = Xp[3 * i + c] * r[kFS + c]; acc[0] += t * t; }
        }
        block_sum<NW, 1>(acc, S.red, S.tot);
        BA_AUDIT();
        if (tid == 0) {
            double d2 = S.tot[0];
            for (int c = 0; c < 6; ++c) d2 += (S.cam[c] * S.sic[c]) * (S.cam[c] * S.sic[c]);
            S.Delta = sqrt(d2);
            if (S.Delta == 0.0) S.Delta = 1.0;
            S.nfev = 1; S.njev = 1; S.status = -1; S.done = 0;
        }
        __syncthreads();
    }

    while (true) {
        __syncthreads();   // every wave has read the previous iteration's S.status / S.done
        if (tid == 0) {
            if (S.gmax < gtol) S.status = 1;
            S.done = S.status >= 0 || S.nfev == max_nfev;
            for (int c = 0; c < 6; ++c) { S.dc[c] = 1.0 / S.sic[c]; S.ghc[c] = S.dc[c] * S.gc[c]; }
        }
        __syncthreads();
        if (S.done) break;
        // regularize: a = 0.5 |J_h (-g_h)|^2, |g_h|^2 (build_quadratic_1d along -g_h)
        {
            double acc[2] = {0.0, 0.0};
            BA_AUDIT();
            for (int i = tid; i < n; i += NT) {
                BA_PRINTF(i);
                double r[kRec];
                pass_rec(i, r);
                double vu = 0.0, vv = 0.0;
                for (int c = 0; c < 6; ++c) { vu -= r[c] * S.dc[c] * S.ghc[c]; vv -= r[9 + c] * S.dc[c] * S.ghc[c]; }
                for (int c = 0; c < 3; ++c) {
                    const double gh = r[6 + c] * r[18] + r[15 + c] * r[19];   // Pp^T f
                    vu -= r[6 + c] * gh;
                    vv -= r[15 + c] * gh;
                    acc[1] += gh * gh;
                }
                acc[0] += vu * vu + vv * vv;
            }
            block_sum<NW, 2>(acc, S.red, S.tot);
            BA_AUDIT();
            if (tid == 0) {
                double gh2 = S.tot[1];
                for (int c = 0; c < 6; ++c) gh2 += S.ghc[c] * S.ghc[c];
                const double a = 0.5 * S.tot[0], b = -gh2, to_tr = S.Delta / sqrt(gh2);
                double ag = 0.0;                                  // t = 0
                ag = fmin(ag, to_tr * (a * to_tr + b));           // t = to_tr (argmin keeps the first on ties)
                if (a != 0.0) {
                    const double ext = -0.5 * b / a;
                    if (0.0 < ext && ext < to_tr) ag = fmin(ag, ext * (a * ext + b));
                }
                S.mu = -ag / (S.Delta * S.Delta);
                S.gh2 = gh2;
            }
            __syncthreads();
            BA_MARK(1);
        }
        const double mu = S.mu;
        // ridge: G = I + sum C^T B^-1 C, h = sum C^T B^-1 f  (C = J_h camera block, B = Jp_h Jp_h^T + mu I)
        {
            double acc[27];
#pragma unroll
            for (int e = 0; e < 27; ++e) acc[e] = 0.0;
            BA_AUDIT();
            for (int i = tid; i < n; i += NT) {
                BA_PRINTF(i);
                double r[kRec];
                pass_rec(i, r);
                double C[2][6], Pp[2][3];
                for (int c = 0; c < 6; ++c) { C[0][c] = r[c] * S.dc[c]; C[1][c] = r[9 + c] * S.dc[c]; }
                for (int c = 0; c < 3; ++c) {
                    Pp[0][c] = r[6 + c];
                    Pp[1][c] = r[15 + c];
                }
                const double b00 = Pp[0][0] * Pp[0][0] + Pp[0][1] * Pp[0][1] + Pp[0][2] * Pp[0][2] + mu;
                const double b01 = Pp[0][0] * Pp[1][0] + Pp[0][1] * Pp[1][1] + Pp[0][2] * Pp[1][2];
                const double b11 = Pp[1][0] * Pp[1][0] + Pp[1][1] * Pp[1][1] + Pp[1][2] * Pp[1][2] + mu;
                const double idet = 1.0 / (b00 * b11 - b01 * b01);
                const double i00 = b11 * idet, i01 = -b01 * idet, i11 = b00 * idet;
                const double u0 = i00 * r[18] + i01 * r[19], u1 = i01 * r[18] + i11 * r[19];
                double Y[2][6];
                for (int c = 0; c < 6; ++c) { Y[0][c] = i00 * C[0][c] + i01 * C[1][c]; Y[1][c] = i01 * C[0][c] + i11 * C[1][c]; }
                int e = 0;
                for (int a = 0; a < 6; ++a)
                    for (int b = a; b < 6; ++b) acc[e++] += C[0][a] * Y[0][b] + C[1][a] * Y[1][b];
                for (int a = 0; a < 6; ++a) acc[21 + a] += C[0][a] * u0 + C[1][a] * u1;
            }
            block_sum<NW, 27>(acc, S.red, S.tot);
            BA_AUDIT();
            if (tid == 0) {
                double G[6][6], h[6];
                int e = 0;
                for (int a = 0; a < 6; ++a)
                    for (int b = a; b < 6; ++b) { G[a][b] = G[b][a] = S.tot[e++] + (a == b ? 1.0 : 0.0); }
                for (int a = 0; a < 6; ++a) h[a] = S.tot[21 + a];
                if (!chol6_solve(G, h)) S.status = -2;   // not expected: G = I + PSD
                for (int a = 0; a < 6; ++a) S.z[a] = h[a];
            }
            __syncthreads();
            BA_MARK(2);
        }
        // gn_h = J_h^T y, y = B^-1 f - B^-1 C z; g_h . gn_h and |gn_h|^2 (Gram-Schmidt of [g_h, gn_h])
        {
            double acc[7] = {0};   // gnc (6), point part of g_h . gn_h
            BA_AUDIT();
            for (int i = tid; i < n; i += NT) {
                BA_PRINTF(i);
                double r[kRec];
                pass_rec(i, r);
                double C[2][6], Pp[2][3];
                for (int c = 0; c < 6; ++c) { C[0][c] = r[c] * S.dc[c]; C[1][c] = r[9 + c] * S.dc[c]; }
                for (int c = 0; c < 3; ++c) {
                    Pp[0][c] = r[6 + c];
                    Pp[1][c] = r[15 + c];
                }
                const double b00 = Pp[0][0] * Pp[0][0] + Pp[0][1] * Pp[0][1] + Pp[0][2] * Pp[0][2] + mu;
                const double b01 = Pp[0][0] * Pp[1][0] + Pp[0][1] * Pp[1][1] + Pp[0][2] * Pp[1][2];
                const double b11 = Pp[1][0] * Pp[1][0] + Pp[1][1] * Pp[1][1] + Pp[1][2] * Pp[1][2] + mu;
                const double idet = 1.0 / (b00 * b11 - b01 * b01);
                const double i00 = b11 * idet, i01 = -b01 * idet, i11 = b00 * idet;
                double w0 = r[18], w1 = r[19];
                for (int c = 0; c < 6; ++c) { w0 -= C[0][c] * S.z[c]; w1 -= C[1][c] * S.z[c]; }
                const double y0 = i00 * w0 + i01 * w1, y1 = i01 * w0 + i11 * w1;
                for (int c = 0; c < 6; ++c) acc[c] += C[0][c] * y0 + C[1][c] * y1;
                for (int c = 0; c < 3; ++c) {
                    const double gn = Pp[0][c] * y0 + Pp[1][c] * y1;
                    const double gh = Pp[0][c] * r[18] + Pp[1][c] * r[19];   // d * (J^T f) = g_h
                    acc[6] += gh * gn;
                }
            }
            block_sum<NW, 7>(acc, S.red, S.tot);
            BA_AUDIT();
            if (tid == 0) {
                const double ghn = sqrt(S.gh2);
                double dot = S.tot[6];
                for (int c = 0; c < 6; ++c) {
                    S.gnc[c] = S.tot[c];
                    dot += S.ghc[c] * S.gnc[c];
                    S.s1c[c] = S.ghc[c] / ghn;
                }
                S.c12 = dot / ghn;   // s2 = gn_h - (s1 . gn_h) s1, normalised by the next pass
                for (int c = 0; c < 6; ++c) S.s2c[c] = S.gnc[c] - S.c12 * S.s1c[c];
                S.ghn = ghn;
            }
            __syncthreads();
            BA_MARK(3);
        }
        // |s2|^2 exactly; then JS (2 columns) -> B_S, g_S
        const double ghn = S.ghn, c12 = S.c12;
        auto point_vecs = [&](const double* r, double (&s1)[3], double (&s2)[3]) {
            double C[2][6], Pp[2][3];
            for (int c = 0; c < 6; ++c) { C[0][c] = r[c] * S.dc[c]; C[1][c] = r[9 + c] * S.dc[c]; }
            for (int c = 0; c < 3; ++c) {
                Pp[0][c] = r[6 + c];
                Pp[1][c] = r[15 + c];
            }
            const double b00 = Pp[0][0] * Pp[0][0] + Pp[0][1] * Pp[0][1] + Pp[0][2] * Pp[0][2] + mu;
            const double b01 = Pp[0][0] * Pp[1][0] + Pp[0][1] * Pp[1][1] + Pp[0][2] * Pp[1][2];
            const double b11 = Pp[1][0] * Pp[1][0] + Pp[1][1] * Pp[1][1] + Pp[1][2] * Pp[1][2] + mu;
            const double idet = 1.0 / (b00 * b11 - b01 * b01);
            const double i00 = b11 * idet, i01 = -b01 * idet, i11 = b00 * idet;
            double w0 = r[18], w1 = r[19];
            for (int c = 0; c < 6; ++c) { w0 -= C[0][c] * S.z[c]; w1 -= C[1][c] * S.z[c]; }
            const double y0 = i00 * w0 + i01 * w1, y1 = i01 * w0 + i11 * w1;
            for (int c = 0; c < 3; ++c) {
                const double gn = Pp[0][c] * y0 + Pp[1][c] * y1;
                const double gh = Pp[0][c] * r[18] + Pp[1][c] * r[19];
                s1[c] = gh / ghn;
                s2[c] = gn - c12 * s1[c];
            }
        };
        // one pass for |s2|^2 and the products of JS = J_h [s1, s2]: with the unnormalised s2
        // (camera part S.s2c, point part from point_vecs) every product that involves s2 is
        // divided by |s2| (or |s2|^2) once afterwards
        {
            double acc[6] = {0};   // JS1.JS1, JS1.JS2u, JS2u.JS2u, s2u . g_h and s1 . g_h (point parts), |s2u pts|^2
            BA_AUDIT();
            for (int i = tid; i < n; i += NT) {
                BA_PRINTF(i);
                double r[kRec];
                pass_rec(i, r);
                double s1[3], s2[3];
                point_vecs(r, s1, s2);
                double a0 = 0, a1 = 0, b0 = 0, b1 = 0;
                for (int c = 0; c < 6; ++c) {
                    a0 += r[c] * S.dc[c] * S.s1c[c];
                    a1 += r[9 + c] * S.dc[c] * S.s1c[c];
                    b0 += r[c] * S.dc[c] * S.s2c[c];
                    b1 += r[9 + c] * S.dc[c] * S.s2c[c];
                }
                for (int c = 0; c < 3; ++c) {
                    const double p0 = r[6 + c], p1 = r[15 + c];
                    a0 += p0 * s1[c];
                    a1 += p1 * s1[c];
                    b0 += p0 * s2[c];
                    b1 += p1 * s2[c];
                    const double gh = p0 * r[18] + p1 * r[19];
                    acc[3] += s2[c] * gh;
                    acc[4] += s1[c] * gh;
                    acc[5] += s2[c] * s2[c];
                }
                acc[0] += a0 * a0 + a1 * a1;
                acc[1] += a0 * b0 + a1 * b1;
                acc[2] += b0 * b0 + b1 * b1;
            }
            block_sum<NW, 6>(acc, S.red, S.tot);
            BA_AUDIT();
            if (tid == 0) {
                double n2 = S.tot[5];
                for (int c = 0; c < 6; ++c) n2 += S.s2c[c] * S.s2c[c];
                const double s2n = sqrt(n2);
                double g0 = S.tot[4], g1 = S.tot[3];
                for (int c = 0; c < 6; ++c) { g0 += S.s1c[c] * S.ghc[c]; g1 += S.s2c[c] * S.ghc[c]; }
                for (int c = 0; c < 6; ++c) S.s2c[c] /= s2n;
                S.s2n = s2n;
                S.BS[0] = S.tot[0];
                S.BS[1] = S.tot[1] / s2n;
                S.BS[2] = S.tot[2] / s2n / s2n;
                S.gS[0] = g0;
                S.gS[1] = g1 / s2n;
            }
            __syncthreads();
            BA_MARK(4);
        }
        const double s2n = S.s2n;
        // inner loop: trial steps until the cost decreases
        if (tid == 0) S.accept = 0;
        __syncthreads();
        while (true) {
            if (tid < 64) {   // wave 0: the 2-D subproblem (the circle scan's 64 angles one per lane)
                if (!(S.nfev < max_nfev)) {
                    if (tid == 0) S.done = 1;
                } else {
                    double pS[2];
                    tr_solve_2d_wave(S.BS, S.gS, S.Delta, pS);
                    if (tid == 0) {
                        S.done = 0;
                        S.pS[0] = pS[0];
                        S.pS[1] = pS[1];
                        for (int c = 0; c < 6; ++c) {
                            S.shc[c] = S.pS[0] * S.s1c[c] + S.pS[1] * S.s2c[c];
                            S.cam_new[c] = S.cam[c] + S.dc[c] * S.shc[c];
                        }
                        rodrigues(S.cam_new, S.Rn);
                    }
                }
            }
            __syncthreads();
            BA_MARK(5);
            if (S.done) break;
            if (FUSED) {   // R(rvec_new) and the three perturbed rotations of the FD at the trial point
                if (tid < 4) {
                    double q[3] = {S.cam_new[0], S.cam_new[1], S.cam_new[2]};
                    if (tid > 0) q[tid - 1] = q[tid - 1] + fd_step(q[tid - 1]);
                    rodrigues(q, S.R[tid]);
                }
                __syncthreads();
            }
            // step, J_h step, f(x_new): predicted reduction, cost_new, |step_h|, |step|, |x|, finiteness
            // (FUSED also: J at x_new into the other record set, gc (6), column sums of squares (6), |g|_inf)
            constexpr int KT = FUSED ? 19 : 7;
            double acc[KT] = {0};   // |J_h s|^2, s.g_h (points), cost_new*2, |step_h|^2 pts, |step|^2 pts, |x|^2 pts, nonfinite
            double gmax_n = 0.0;
            if constexpr (FUSED) {
                BA_AUDIT();
                for (int i = tid; i < n; i += NT) {
                    BA_PRINTF(i);
                    double r[kRec];
                    pass_rec_d(i, r);
                    recs[cur].template load<kFX, kFX + 3>(i, r);   // the current point
                    double s1[3], s2[3];
                    point_vecs(r, s1, s2);
                    double ju = 0, jv = 0;
                    for (int c = 0; c < 6; ++c) { ju += r[c] * S.dc[c] * S.shc[c]; jv += r[9 + c] * S.dc[c] * S.shc[c]; }
                    double Xn[3];
                    for (int c = 0; c < 3; ++c) {
                        const double d = 1.0 / r[kFS + c];   // the Jacobian pass's quotient
                        const double sh = S.pS[0] * s1[c] + S.pS[1] * (s2[c] / s2n);
                        ju += r[6 + c] * sh;
                        jv += r[15 + c] * sh;
                        acc[1] += sh * (r[6 + c] * r[18] + r[15 + c] * r[19]);
                        acc[3] += sh * sh;
                        const double st = d * sh;
                        acc[4] += st * st;
                        const double x = r[kFX + c];
                        acc[5] += x * x;
                        Xn[c] = x + st;
                    }
                    acc[0] += ju * ju + jv * jv;
                    // J at x_new (jacobian(false, true)'s record: the base residual is the trial's)
                    double o[kRec], f[2];
                    for (int c = 0; c < 3; ++c) o[kFS + c] = r[kFS + c];
                    fd_obs(&S.R[0][0], S.cam_new, k, Xn, pts[2 * i], pts[2 * i + 1], nullptr, f, o);
                    acc[2] += f[0] * f[0] + f[1] * f[1];
                    if (!isfinite(f[0]) || !isfinite(f[1])) acc[6] += 1.0;
                    o[18] = f[0];
                    o[19] = f[1];
#pragma unroll
                    for (int c = 0; c < 6; ++c) {
                        acc[7 + c] += o[c] * f[0] + o[9 + c] * f[1];
                        acc[13 + c] += o[c] * o[c] + o[9 + c] * o[9 + c];
                    }
#pragma unroll
                    for (int c = 0; c < 3; ++c) {
                        const double gp = o[6 + c] * f[0] + o[15 + c] * f[1];
                        gmax_n = fmax(gmax_n, fabs(gp));
                        const double si = fmax(sqrt(o[6 + c] * o[6 + c] + o[15 + c] * o[15 + c]), o[kFS + c]);
                        o[kFS + c] = si;
                        const double d = 1.0 / si;
                        o[6 + c] = o[6 + c] * d;   // Pp
                        o[15 + c] = o[15 + c] * d;
                        o[kFX + c] = Xn[c];
                    }
                    recs[cur ^ 1].template store<0, 20>(i, o);
                    recs[cur ^ 1].template store<kFX, kRec>(i, o);
                }
                gmax_n = block_max<NW>(gmax_n, S.red);
                BA_AUDIT();
                block_sum<NW, KT>(acc, S.red, S.tot);
                BA_AUDIT();
                BA_MARK(6);
            } else {
                for (int i = tid; i < n; i += NT) {
                    BA_PRINTF(i);
                    double r[kRec];
                    pass_rec_d(i, r);
                    double s1[3], s2[3];
                    point_vecs(r, s1, s2);
                    double ju = 0, jv = 0;
                    for (int c = 0; c < 6; ++c) { ju += r[c] * S.dc[c] * S.shc[c]; jv += r[9 + c] * S.dc[c] * S.shc[c]; }
                    double Xn[3];
                    for (int c = 0; c < 3; ++c) {
                        const double d = 1.0 / r[kFS + c];   // the Jacobian pass's quotient
                        const double sh = S.pS[0] * s1[c] + S.pS[1] * (s2[c] / s2n);
                        ju += r[6 + c] * sh;
                        jv += r[15 + c] * sh;
                        acc[1] += sh * (r[6 + c] * r[18] + r[15 + c] * r[19]);
                        acc[3] += sh * sh;
                        const double st = d * sh;
                        acc[4] += st * st;
                        const double x = Xp[3 * i + c];
                        acc[5] += x * x;
                        Xn[c] = x + st;
                        r[kFX + c] = Xn[c];
                    }
                    recs[cur].template store<kFX, kFX + 3>(i, r);
                    acc[0] += ju * ju + jv * jv;
                    double ru, rv;
                    resid(S.Rn, S.cam_new, k, Xn, pts + 2 * i, ru, rv);
                    acc[2] += ru * ru + rv * rv;
                    if (!isfinite(ru) || !isfinite(rv)) acc[6] += 1.0;
                }
                block_sum<NW, 7>(acc, S.red, S.tot);
                BA_AUDIT();
                BA_MARK(6);
            }
            if (tid == 0) {
                double sg = S.tot[1], sh2 = S.tot[3], st2 = S.tot[4], x2 = S.tot[5];
                for (int c = 0; c < 6; ++c) {
                    sg += S.shc[c] * S.ghc[c];
                    sh2 += S.shc[c] * S.shc[c];
                    st2 += (S.dc[c] * S.shc[c]) * (S.dc[c] * S.shc[c]);
                    x2 += S.cam[c] * S.cam[c];
                }
                const double predicted = -(0.5 * S.tot[0] + sg);
                S.nfev += 1;
                const double sh_norm = sqrt(sh2);
                if (S.tot[6] > 0.0) {   // non-finite residuals: shrink and retry
                    S.Delta = 0.25 * sh_norm;
                    S.accept = -1;
                } else {
                    S.cost_new = 0.5 * S.tot[2];
                    const double actual = S.cost - S.cost_new;
                    double ratio;
                    if (predicted > 0.0) ratio = actual / predicted;
                    else if (predicted == 0.0 && actual == 0.0) ratio = 1.0;
                    else ratio = 0.0;
                    double Dn = S.Delta;
                    if (ratio < 0.25) Dn = 0.25 * sh_norm;
                    else if (ratio > 0.75 && sh_norm > 0.95 * S.Delta) Dn = S.Delta * 2.0;
                    const double step_norm = sqrt(st2), x_norm = sqrt(x2);
                    const bool fok = actual < ftol * S.cost && ratio > 0.25;
                    const bool xok = step_norm < xtol * (xtol + x_norm);
                    S.status = (fok && xok) ? 4 : fok ? 2 : xok ? 3 : -1;
                    S.accept = actual > 0.0 ? 1 : 0;
                    if (S.status < 0) S.Delta = Dn;
                    if (FUSED && S.accept == 1) {   // jacobian(false, true)'s scalars, from the same sums
                        double gm = gmax_n;
                        for (int c = 0; c < 6; ++c) {
                            S.gc[c] = S.tot[7 + c];
                            gm = fmax(gm, fabs(S.gc[c]));
                            S.sic[c] = fmax(sqrt(S.tot[13 + c]), S.sic[c]);
                        }
                        S.gmax = gm;
                        S.cost = 0.5 * S.tot[2];
                    }
                }
            }
            __syncthreads();
            BA_MARK(7);
            if (S.status >= 0 || S.accept == 1) break;
        }
        if (S.accept == 1) {   // x = x_new (moved by the Jacobian pass); J at the new point
            if (tid < 6) S.cam[tid] = S.cam_new[tid];
            __syncthreads();
            if (FUSED) cur ^= 1;   // the trial pass formed J at x_new already
            else jacobian(false, true);
            if (tid == 0) { S.njev += 1; }
            __syncthreads();
            BA_MARK(0);
        }
        if (S.done) break;
    }
#ifdef SFMHIP_BA_PROF
    prof_acc[8] = prof_t0;
    prof_acc[9] = wall_clock64();
    if (tid == 0 && p < 4096)
        for (int kk = 0; kk < kProfPhases; ++kk) g_ba_prof[p * kProfPhases + kk] = prof_acc[kk];
#endif
    if (FUSED)   // X = the current records' point
        for (int i = tid; i < n; i += NT)
            for (int c = 0; c < 3; ++c) Xp[3 * i + c] = *recs[cur].at(i, kFX + c);
    if (tid < 6) cam_io[(size_t)p * 6 + tid] = S.cam[tid];
    if (tid == 0) {
        cost_out[p] = S.cost;
        nfev_out[p] = S.nfev;
        njev_out[p] = S.njev;
        status_out[p] = S.status < 0 ? 0 : S.status;
    }
}

}  // namespace
}  // namespace sfmhip

using namespace sfmhip;

extern "C" int sfmhip_ba_solve(double* cam, const double* K, double* X, const double* pts2d, const int64_t* pair_off,
                               int n_pairs, int64_t n_obs, double ftol, double xtol, double gtol, int max_nfev,
                               double* cost, int32_t* nfev, int32_t* njev, int32_t* status, void* stream) {
    SFMHIP_REQUIRE(n_pairs >= 0, "sfmhip_ba_solve: negative n_pairs");
    SFMHIP_REQUIRE(n_obs >= 0, "sfmhip_ba_solve: negative n_obs");
    if (n_pairs == 0) return SFMHIP_OK;
    SFMHIP_REQUIRE(cam && K && X && pts2d && pair_off && cost && nfev && njev && status,
                   "sfmhip_ba_solve: null pointer");
    hipStream_t st = as_stream(stream);
    double* scratch = nullptr;
    const bool fused = knobs().ab == 9;   // A/B (temporary): the fused trial + Jacobian form
    if (scratch_alloc((void**)&scratch, (size_t)std::max<int64_t>(n_obs, 1) * kRec * sizeof(double) * (fused ? 2 : 1),
                      st) != hipSuccess) {
        (void)hipGetLastError();
        set_error("sfmhip_ba_solve: scratch allocation failed");
        return SFMHIP_E_HIP;
    }
    // one 512-thread workgroup per pair, field-major records (256 threads, AoS records and the
    // recompute form measured slower: profiles/r3/ba_variants_r3m.txt, DESIGN.md K3'')
    // the first 768 observations' records of each pair in LDS (156 KB): the kernel's 256 VGPRs per
    // lane already hold a CU to one workgroup, so the LDS costs no residency
    const int lds_obs = (!fused && knobs().ab != 7) ? kBaLdsObs : 0;
    const size_t lds_bytes = (size_t)lds_obs * kLdsF * sizeof(double);
    if (lds_bytes > 0) {
        static std::once_flag attr_once;
        static hipError_t attr_rc = hipSuccess;
        std::call_once(attr_once, [&] {
            attr_rc = hipFuncSetAttribute(reinterpret_cast<const void*>(&ba_trf_kernel<512>),
                                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)(kLdsF * kBaLdsObs * 8));
        });
        if (attr_rc != hipSuccess) {
            scratch_free(scratch, st);
            set_error("sfmhip_ba_solve: LDS attribute: %s", hipGetErrorString(attr_rc));
            return SFMHIP_E_HIP;
        }
    }
    if (fused)
        hipLaunchKernelGGL((ba_trf_kernel<512, true>), dim3(n_pairs), dim3(512), 0, st, cam, K, X, pts2d, pair_off, n_obs,
                           ftol, xtol, gtol, max_nfev, scratch, cost, nfev, njev, status, 0);
    else
        hipLaunchKernelGGL((ba_trf_kernel<512>), dim3(n_pairs), dim3(512), lds_bytes, st, cam, K, X, pts2d, pair_off,
                           n_obs, ftol, xtol, gtol, max_nfev, scratch, cost, nfev, njev, status, lds_obs);
    const int rc = check_launch("ba_trf_kernel");
    scratch_free(scratch, st);
    return rc;
}

#ifdef SFMHIP_BA_PROF
// tool-only build: the per-pair phase times of the last solve launch (wall-clock ticks)
extern "C" int sfmhip_ba_prof_read(unsigned long long* host, int n_pairs) {
    const int n = std::min(n_pairs, 4096) * kProfPhases;
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_ba_prof), (size_t)n * sizeof(unsigned long long)) == hipSuccess
               ? 0 : -1;
}
#endif
