// tsdf.hip — V5 TSDF integration (build-defined), laid out
// like the sdf.py grid (sdf.py:284-304: (D,H,W), x -> W, align_corners).
//
// Definition (oracle/voxel.py tsdf_integrate, every f32 op one IEEE RN step in
// the order written): per voxel and frame the projection, the skip rules and
// tsdf = min(1, sdf * (1/mu)) of the running-average TSDF; the frames of one
// integration step (a call, split into steps of at most kTsdfMaxFrames) are
// then fused ORDER-FREE:
//     q_f = rint(tsdf_f * 2^21)   (an exact integer, |q| <= 2^21 + 1)
//     S = sum q_f, n = #updates   (integer sums: any order, any split)
//     W' = W + n                  (one f32 add)
//     T' = f32( (f64(T) f64(W) + f64(S) 2^-21) / (f64(W) + n) )
// which telescopes the sequential T <- (T W + tsdf)/(W + 1), W <- W + 1 (within
// 2^-22 per update of the exact average; tests/test_gpu_voxel.py checks it against
// the sequential restatement too): no per-voxel update chain, no per-frame division,
// and any split of the frames (tiles, waves, ranks) gives the same bits.
//
// Pipeline per step (one launch of each kernel):
//   tsdf_setup_kernel     validated camera records (f32 for the fusion, f64 CullCam
//                         for the culling passes), the slab's block range per frame
//   depth_blockmax_kernel {min, max} per 16x16 depth block: the step's one
//                         compulsory streaming read of the depth maps
//   coarse_table_kernel + tsdf_brick_kernel   (whole-grid mode) brick pre-pass
//   (SFMHIP_AB=3: the block pass and the culling in one persistent tsdf_prepass_kernel +
//   tsdf_pack_kernel instead; measured slower)
//   tsdf_cull_kernel      exact (tile, frame) culling / free-space proofs -> masks
//   tsdf_refine_kernel    (whole-grid mode) the projected pairs again per wave sub-tile
//   tsdf_order_kernel     longest-first workgroup order per XCD class
//   tsdf_fuse_kernel      one wave per 8x2x8 sub-tile: integer (S, n) in registers over
//                         the step's frames, then the voxels finished in place
// All fp32/fp64 with -ffp-contract=off so the op order matches the oracle.
#include "common.h"
#include <climits>
#include <cstdlib>
#include <algorithm>
#include <vector>

namespace sfmhip {

constexpr int kTsdfMaxFrames = 512;   // frames per integration step (host splits longer calls)
constexpr int kTsdfQBits = 21;        // tsdf fixed point: |S| <= 512 (2^21 + 1) < 2^31
static_assert(kTsdfMaxFrames * ((1 << kTsdfQBits) + 1) < INT_MAX, "S must fit an int32");
constexpr double kTsdfLatencyRounds = 1.0;   // below: latency mode (tsdf_run)
constexpr double kTsdfDeepRounds = 6.0;      // below: four projected frames per fusion stage
constexpr int kTsdfTX = 8, kTsdfTY = 8, kTsdfTZ = 8;    // workgroup tile: 4 waves x (8 x, 2 y, 8 z)
constexpr int kCullSub = 4;           // wave sub-tiles per tile

struct GridBox { float mn[3], mx[3]; };

typedef float f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2 f2s(float a) { return f2{a, a}; }
__device__ __forceinline__ f2 fma2(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ f2 rcp2(f2 a) { return f2{__builtin_amdgcn_rcpf(a.x), __builtin_amdgcn_rcpf(a.y)}; }

// RN(1/z) for z in [2^-60, 2^60): Fma0..Fma4 + div_fmas of the f32 IEEE
// division with numerator 1 (v_div_scale / v_div_fixup are identities there).
__device__ __forceinline__ f2 recip_rn(f2 z) {
    const f2 one = f2s(1.f), nz = -z;
    f2 r = rcp2(z);
    r = fma2(fma2(nz, r, one), r, r);
    const f2 q = fma2(fma2(nz, r, one), r, r);
    return fma2(fma2(nz, q, one), r, q);
}
__device__ __forceinline__ int cvt_flr(float x) {
    int r;
    asm("v_cvt_flr_i32_f32 %0, %1" : "=v"(r) : "v"(x));
    return r;
}
// Zc in [2^-60, 2^60) (false for <= 0, NaN, inf): one subtract + one compare
__device__ __forceinline__ bool z_ok(float z) {
    return __builtin_bit_cast(unsigned, z) - 0x21800000u < 0x3C000000u;
}

// ---------------------------------------------------------------------------
// Culling (exact: it only drops (tile, frame) pairs in which provably no voxel
// of the box would update, and marks "free space" pairs in which every voxel
// updates with tsdf = 1).
constexpr int kCullBlock = 16;
constexpr int kCullMaxBlocks = 256;   // larger footprints are simply kept

// The culling passes' f64 view of the grid (host-computed once per call) and of
// a frame (CullCam, built once per frame by tsdf_setup_kernel and read with
// scalar loads where the frame is wave-uniform).
struct CullGeom { double mn[3], s[3], as[3]; };
struct CullCam { double P[12], aP[12], k[4], good, pad[3]; };   // 256 B

__device__ __forceinline__ void cull_cam(const float* __restrict__ poses, const float* __restrict__ Kf, int f,
                                         CullCam& c) {
    bool good = true;
#pragma unroll
    for (int q = 0; q < 12; ++q) {
        const float x = poses[f * 12 + q];
        c.P[q] = x;
        c.aP[q] = fabs((double)x);
        good = good && fabsf(x) < 0x1p60f;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const float x = Kf[f * 4 + q];
        c.k[q] = x;
        good = good && fabsf(x) < 0x1p60f;
    }
    c.good = good ? 1.0 : 0.0;
}

// Newton-refined v_rcp_f64 (a few ulps of 1/z; the bounds below carry margins of
// ~2^-21 relative, so the footprint stays conservative).
__device__ __forceinline__ double cull_rcp(double z) {
    double r = __builtin_amdgcn_rcp(z);
    r = fma(fma(-z, r, 1.0), r, r);
    return fma(fma(-z, r, 1.0), r, r);
}

// Conservative pixel footprint of the voxel box [xa,xb] x [ya,yb] x [za,zb] in
// frame c: interval bounds on the affine camera coordinates (centre +- sum |P_rj|
// h_j) widened by a bound on the fusion kernel's f32 rounding, and the X/Z, Y/Z
// interval quotients.  Returns 0 (no bound: box not safely in front of the
// camera), 1 (every voxel's pixel is off-image) or 2 (pixel range [u0,u1] x
// [v0,v1], clipped to the image, and zlo <= every f32 Zc <= zhi).
__device__ __forceinline__ int box_footprint(const CullCam& cc, const CullGeom& G, int xa, int xb, int ya, int yb,
                                             int za, int zb, int Hd, int Wd, int& u0, int& u1, int& v0, int& v1,
                                             double& zlo, double& zhi, bool& inside) {
    const double cxw = G.mn[0] + 0.5 * (xa + xb) * G.s[0], hx = 0.5 * (xb - xa) * G.as[0];
    const double cyw = G.mn[1] + 0.5 * (ya + yb) * G.s[1], hy = 0.5 * (yb - ya) * G.as[1];
    const double czw = G.mn[2] + 0.5 * (za + zb) * G.s[2], hz = 0.5 * (zb - za) * G.as[2];
    const double mxw = fabs(cxw) + hx, myw = fabs(cyw) + hy, mzw = fabs(czw) + hz;   // |coord| bounds
    double c[3], e[3], mag[3], magm[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        const double* p = cc.P + 4 * r;
        const double* a = cc.aP + 4 * r;
        c[r] = p[0] * cxw + p[1] * cyw + p[2] * czw + p[3];
        e[r] = a[0] * hx + a[1] * hy + a[2] * hz;
        mag[r] = a[0] * mxw + a[1] * myw + a[2] * mzw + a[3];
        magm[r] = a[0] * fabs(G.mn[0]) + a[1] * fabs(G.mn[1]) + a[2] * fabs(G.mn[2]);
    }
    // f32 error of the kernel's Zc / Xc / Yc (unit roundoff u = 2^-24).  The kernel's voxel
    // coordinate v' = fl(mn + fl(i fl(fl(mx - mn) / (R - 1)))) is within u (4.01 |v| + 3.01 |mn|)
    // of this f64 model's v — a term in |mn| that does not shrink with |v| (a camera inside a
    // grid with a large |bmin|) — and the row's four products and three sums add at most
    // 4 u (sum |P_rj| |v_j| + |P_r3|): so 10 u mag + 4 u sum_j |P_rj| |mn_j| covers both.
    const double eps = 0x1p-24;
    double dr[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) dr[r] = 10 * eps * mag[r] + 4 * eps * magm[r];
    zlo = c[2] - e[2] - dr[2];
    zhi = c[2] + e[2] + dr[2];
    inside = false;
    if (!(zlo > 1e-3 && zhi < 1e30 && c[0] == c[0] && c[1] == c[1])) return 0;
    const double izl = cull_rcp(zlo), izh = cull_rcp(zhi);
    const double xl = c[0] - e[0] - dr[0], xh = c[0] + e[0] + dr[0];
    const double yl = c[1] - e[1] - dr[1], yh = c[1] + e[1] + dr[1];
    const double qx0 = fmin(fmin(xl * izl, xl * izh), fmin(xh * izl, xh * izh));
    const double qx1 = fmax(fmax(xl * izl, xl * izh), fmax(xh * izl, xh * izh));
    const double qy0 = fmin(fmin(yl * izl, yl * izh), fmin(yh * izl, yh * izh));
    const double qy1 = fmax(fmax(yl * izl, yl * izh), fmax(yh * izl, yh * izh));
    const double ua = cc.k[0] * qx0, ub = cc.k[0] * qx1, va = cc.k[1] * qy0, vb = cc.k[1] * qy1;
    const double um0 = fmin(ua, ub) + cc.k[2] + 0.5, um1 = fmax(ua, ub) + cc.k[2] + 0.5;
    const double vm0 = fmin(va, vb) + cc.k[3] + 0.5, vm1 = fmax(va, vb) + cc.k[3] + 0.5;
    if (!(um0 > -1e9 && um1 < 1e9 && vm0 > -1e9 && vm1 < 1e9)) return 0;
    // rounding of (f X) iz + c: a few ulps of the magnitudes involved
    const double du = 8 * eps * (fmax(fabs(um0), fabs(um1)) + fabs(cc.k[2]) + 1) + 1e-3;
    const double dv = 8 * eps * (fmax(fabs(vm0), fabs(vm1)) + fabs(cc.k[3]) + 1) + 1e-3;
    u0 = (int)floor(um0 - du);
    u1 = (int)floor(um1 + du);
    v0 = (int)floor(vm0 - dv);
    v1 = (int)floor(vm1 + dv);
    if (u1 < 0 || v1 < 0 || u0 >= Wd || v0 >= Hd) return 1;
    inside = u0 >= 0 && v0 >= 0 && u1 < Wd && v1 < Hd;
    u0 = max(u0, 0); u1 = min(u1, Wd - 1); v0 = max(v0, 0); v1 = min(v1, Hd - 1);
    return 2;
}

__global__ void full_range_kernel(int F, int nbu, int nbv, int4* __restrict__ range) {
    const int f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f < F) range[f] = make_int4(0, nbu - 1, 0, nbv - 1);
}

// {min, max} of every 16x16 depth block inside the slab's block range of the frame
// (int4 {bu0, bu1, bv0, bv1}, tsdf_setup_kernel): max ignores NaN (a NaN depth never
// updates), min is poisoned by NaN (-inf: such a block never proves free space).
// VEC: Wd % 4 == 0, one float4 (4 pixels) per lane, 4 lanes per block column, all 16
// rows' loads in flight.  Otherwise one pixel per lane, 16 lanes per block.
__device__ __forceinline__ float nan_low(float x) { return x == x ? x : -__builtin_inff(); }
template <bool VEC>
__global__ __launch_bounds__(256) void depth_blockmax_kernel(const float* __restrict__ depth, int F, int Hd, int Wd,
                                                             int nbu, int nbv, const int4* __restrict__ range,
                                                             float2* __restrict__ bmm) {
    const int f = blockIdx.z, bv = blockIdx.y;
    const int4 rg = range[f];                       // blocks the slab can touch in this frame
    if (bv < rg.z || bv > rg.w) return;
    const int ucol0 = blockIdx.x * (VEC ? 1024 : 256);
    if (ucol0 / kCullBlock > rg.y || (ucol0 + (VEC ? 1024 : 256) - 1) / kCullBlock < rg.x) return;
    const float* dp = depth + (size_t)f * Hd * Wd;
    const int r0 = bv * kCullBlock, nr = min(kCullBlock, Hd - r0);
    float m = -__builtin_inff(), mn = __builtin_inff();
    const size_t slot = (size_t)f * nbv + bv;
    if (VEC) {
        const int u = (blockIdx.x * 256 + threadIdx.x) * 4;
        if (u < Wd) {
            typedef float f4v __attribute__((ext_vector_type(4)));
            float4 q[kCullBlock];
#pragma unroll
            for (int r = 0; r < kCullBlock; ++r) {   // streamed once here: non-temporal
                q[r] = make_float4(-__builtin_inff(), -__builtin_inff(), -__builtin_inff(), -__builtin_inff());
                if (r < nr) {
                    const f4v t = __builtin_nontemporal_load(reinterpret_cast<const f4v*>(dp + (size_t)(r0 + r) * Wd + u));
                    q[r] = make_float4(t.x, t.y, t.z, t.w);
                }
            }
#pragma unroll
            for (int r = 0; r < kCullBlock; ++r) m = fmaxf(m, fmaxf(fmaxf(q[r].x, q[r].y), fmaxf(q[r].z, q[r].w)));
#pragma unroll
            for (int r = 0; r < kCullBlock; ++r)
                if (r < nr)
                    mn = fminf(mn, fminf(fminf(nan_low(q[r].x), nan_low(q[r].y)), fminf(nan_low(q[r].z), nan_low(q[r].w))));
        }
        m = fmaxf(m, __shfl_xor(m, 1, 4));
        m = fmaxf(m, __shfl_xor(m, 2, 4));
        mn = fminf(mn, __shfl_xor(mn, 1, 4));
        mn = fminf(mn, __shfl_xor(mn, 2, 4));
        const int bu = u / kCullBlock;
        if ((threadIdx.x & 3) == 0 && bu < nbu) bmm[slot * nbu + bu] = make_float2(mn, m);
    } else {
        const int u = blockIdx.x * 256 + threadIdx.x;
        if (u < Wd)
            for (int r = 0; r < nr; ++r) {
                const float x = dp[(size_t)(r0 + r) * Wd + u];
                m = fmaxf(m, x);
                mn = fminf(mn, nan_low(x));
            }
#pragma unroll
        for (int off = 8; off >= 1; off >>= 1) {
            m = fmaxf(m, __shfl_xor(m, off, 16));
            mn = fminf(mn, __shfl_xor(mn, off, 16));
        }
        const int bu = u / kCullBlock;
        if ((threadIdx.x & 15) == 0 && bu < nbu) bmm[slot * nbu + bu] = make_float2(mn, m);
    }
}

// The decision from a box's footprint (box_footprint == 2) and the {min, max} depth
// over the table blocks that cover it.
__device__ __forceinline__ void cull_decide(const CullCam& cc, float trunc, float m, float mn, double zlo, double zhi,
                                            bool inside, bool& skip, bool& fre) {
    // every depth <= m and every f32 Zc >= zlo: sdf < -trunc with room for the
    // rounding of (depth - Zc), so the kernel's !(sdf < -trunc) test fails everywhere
    skip = m <= 0.f || ((double)m + (double)trunc * (1 + 4 * 0x1p-24) + 1e-30 < zlo);
    // free space: for every voxel fl(depth - Zc) >= mu (1 + 2^-21) and
    // fl(fl(depth - Zc) fl(1/mu)) >= 1, i.e. tsdf = 1 exactly (mu in [2^-100, 2^100]);
    // needs a frame record the fusion kernel fuses (every parameter < 2^60)
    fre = false;
    if (!skip && inside && zlo >= 0x1p-59 && zhi <= 0x1p59 && cc.good != 0.0)
        fre = (double)mn - zhi >= (double)trunc * (1 + 0x1p-20);
}

// The (box, frame) test: skip = provably no voxel of the box updates; fre = every
// voxel of the box updates with tsdf = 1 (free space).
// BLK: pixel edge of the table's blocks; CAP: larger footprints are kept; range null:
// every entry of the table is valid.
template <int BLK = kCullBlock, int CAP = kCullMaxBlocks>
__device__ __forceinline__ void cull_test(const CullCam& cc, const CullGeom& G, int xa, int xb, int ya, int yb,
                                          int za, int zb, int Hd, int Wd, float trunc, int f,
                                          const float2* __restrict__ bmm, int nbu, int nbv,
                                          const int4* __restrict__ range, bool& skip, bool& fre) {
    skip = fre = false;
    int u0, u1, v0, v1;
    double zlo, zhi;
    bool inside = false;
    const int st = ya <= yb ? box_footprint(cc, G, xa, xb, ya, yb, za, zb, Hd, Wd, u0, u1, v0, v1, zlo, zhi, inside)
                            : 0;
    if (st == 1) {
        skip = true;
    } else if (st == 2) {
        const int bu0 = u0 / BLK, bu1 = u1 / BLK, bv0 = v0 / BLK, bv1 = v1 / BLK;
        // only blocks inside the slab's range were computed
        const int4 rg = range ? range[f] : make_int4(0, nbu - 1, 0, nbv - 1);
        const int nu = bu1 - bu0 + 1, nb = nu * (bv1 - bv0 + 1);
        if (nb <= CAP && bu0 >= rg.x && bu1 <= rg.y && bv0 >= rg.z && bv1 <= rg.w) {
            const float2* bp = bmm + ((size_t)f * nbv + bv0) * nbu + bu0;
            float m = -__builtin_inff(), mn = __builtin_inff();
            // rows in pairs, 8 predicated loads per row: up to 16 loads in flight per round
            // (min / max are exact in any order; mins are never NaN, poisoned to -inf)
            for (int bv = bv0; bv <= bv1; bv += 2, bp += 2 * nbu) {
                const bool two_rows = bv + 1 <= bv1;
                for (int i = 0; i < nu; i += 8) {
                    float2 e[16];
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        e[j] = i + j < nu ? bp[i + j] : make_float2(__builtin_inff(), -__builtin_inff());
                        e[8 + j] = two_rows && i + j < nu ? bp[nbu + i + j]
                                                          : make_float2(__builtin_inff(), -__builtin_inff());
                    }
#pragma unroll
                    for (int j = 0; j < 16; ++j) {
                        m = fmaxf(m, e[j].y);
                        mn = fminf(mn, e[j].x);
                    }
                }
            }
            cull_decide(cc, trunc, m, mn, zlo, zhi, inside, skip, fre);
        }
    }
}

// The frame record of frame f from the per-call table: f is wave-uniform at every
// call site that uses it, so these are scalar loads.
__device__ __forceinline__ void load_cull_cam(const CullCam* __restrict__ tab, int f, CullCam& c) {
    const CullCam* p = tab + __builtin_amdgcn_readfirstlane(f);
#pragma unroll
    for (int q = 0; q < 12; ++q) { c.P[q] = p->P[q]; c.aP[q] = p->aP[q]; }
#pragma unroll
    for (int q = 0; q < 4; ++q) c.k[q] = p->k[q];
    c.good = p->good;
}

// Brick pre-pass (whole-grid mode).  The cull pass's workgroups are 4x4x4 bricks of
// tiles (32^3 voxels); a brick-level test decides ~40 % of the (brick, frame) pairs of
// C5 outright (culled or free space; tools/sim_brick_cull.py), and the cull pass's wave
// for such a pair writes the decision without its 64 tile tests.  The brick test reads
// a 4x coarser table (64x64-pixel blocks), so a brick footprint of up to 512 px square
// costs at most 64 loads.  Every decision is the same proof as the tile test's, on a
// box that contains the tile's voxels.
constexpr int kCoarse = 4;
constexpr int kCoarseBlock = kCullBlock * kCoarse;
constexpr int kCoarseMaxBlocks = 64;

// Coarse {min, max} of kCoarse x kCoarse fine blocks; an entry with a fine block the
// slab's range did not compute is (-inf, +inf), which never decides anything.
__global__ void coarse_table_kernel(const float2* __restrict__ bmm, int nf, int nbu, int nbv, int ncu, int ncv,
                                    const int4* __restrict__ range, float2* __restrict__ cmm) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)nf * ncu * ncv) return;
    const int cu = (int)(i % ncu), cv = (int)((i / ncu) % ncv), f = (int)(i / ((int64_t)ncu * ncv));
    const int4 rg = range ? range[f] : make_int4(0, nbu - 1, 0, nbv - 1);
    const int bu0 = cu * kCoarse, bu1 = min(nbu, bu0 + kCoarse) - 1;
    const int bv0 = cv * kCoarse, bv1 = min(nbv, bv0 + kCoarse) - 1;
    float mn = __builtin_inff(), m = -__builtin_inff();
    if (bu0 >= rg.x && bu1 <= rg.y && bv0 >= rg.z && bv1 <= rg.w) {
        for (int bv = bv0; bv <= bv1; ++bv)
            for (int bu = bu0; bu <= bu1; ++bu) {
                const float2 e = bmm[((size_t)f * nbv + bv) * nbu + bu];
                mn = fminf(mn, e.x);
                m = fmaxf(m, e.y);
            }
    } else {
        mn = -__builtin_inff();
        m = __builtin_inff();
    }
    cmm[i] = make_float2(mn, m);
}

// One lane per (cull brick, frame): byte 0 undecided, 1 culled, 2 free space.
// Lanes are (frame, brick) with the brick count padded to whole waves, so the
// frame, and its record, is wave-uniform.
__global__ __launch_bounds__(256) void tsdf_brick_kernel(int H, int W, int z0, int z1, int F, int Hd, int Wd,
                                                         const CullCam* __restrict__ cams, CullGeom G, float trunc,
                                                         const float2* __restrict__ cmm, int ncu, int ncv,
                                                         int nbricks, unsigned char* __restrict__ bdec) {
    const int npad = (nbricks + 63) & ~63;
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int f = (int)(g / npad), brick = (int)(g % npad);
    if (f >= F) return;   // wave-uniform
    CullCam cc;
    load_cull_cam(cams, f, cc);
    if (brick >= nbricks) return;
    const int ntx = (W + kTsdfTX - 1) / kTsdfTX, nty = (H + kTsdfTY - 1) / kTsdfTY;
    const int ntz = (z1 - z0 + kTsdfTZ - 1) / kTsdfTZ;
    const int nqx = (ntx + 3) >> 2, nqy = (nty + 3) >> 2;
    const int qx = brick % nqx, qy = (brick / nqx) % nqy, qz = brick / (nqx * nqy);
    const int xa = qx * 4 * kTsdfTX, xb = min(W, (qx * 4 + 4) * kTsdfTX) - 1;
    const int ya = qy * 4 * kTsdfTY, yb = min(H, (qy * 4 + 4) * kTsdfTY) - 1;
    const int za = z0 + qz * 4 * kTsdfTZ, zb = min(z1, z0 + min(ntz, qz * 4 + 4) * kTsdfTZ) - 1;
    bool skip, fre;
    cull_test<kCoarseBlock, kCoarseMaxBlocks>(cc, G, xa, xb, ya, yb, za, zb, Hd, Wd, trunc, f, cmm, ncu, ncv, nullptr,
                                              skip, fre);
    bdec[(size_t)f * nbricks + brick] = (unsigned char)(skip ? 1 : fre ? 2 : 0);
}

// One workgroup per (4x4x4 brick of tiles, 16 frames): wave j tests frame 16 h + j for
// the brick's 64 tiles (one per lane), so the camera loads are scalar and the
// block-table reads of neighbouring footprints share cache lines; the 16 bits of each
// tile are packed through LDS and stored as the low or high half of its mask word in
// each of the tile's 4 wave slots.  Masks are [wave slot][nw] words, bit j of word w =
// frame 32 w + j.  With `plist`, every (tile, frame) that is neither culled nor free
// space is appended to a list for tsdf_refine_kernel; `tcost` sums each tile's cost
// (4 x projected + free-space frames per wave slot, before refinement) for the
// fusion's longest-first order.
constexpr int kCullFrames = 16;
// waves_per_eu(8): two 16-wave workgroups per CU (the f64 frame record lives in SGPRs)
__global__ __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(8))) void tsdf_cull_kernel(
    int H, int W, int z0, int z1, int F, int Hd, int Wd, const CullCam* __restrict__ cams, CullGeom G, float trunc,
    const float2* __restrict__ bmm, int nbu, int nbv, const int4* __restrict__ range, int nw,
    const unsigned char* __restrict__ bdec, unsigned short* __restrict__ cull, unsigned short* __restrict__ freem,
    unsigned* __restrict__ plist, unsigned* __restrict__ pcount, unsigned* __restrict__ tcost) {
    __shared__ unsigned char bits[kCullFrames][64];
    __shared__ unsigned wcnt[kCullFrames + 1];
    const int ntx = (W + kTsdfTX - 1) / kTsdfTX, nty = (H + kTsdfTY - 1) / kTsdfTY;
    const int ntz = (z1 - z0 + kTsdfTZ - 1) / kTsdfTZ;
    const int nqx = (ntx + 3) >> 2, nqy = (nty + 3) >> 2;  // 4x4x4 bricks of tiles
    const int nh = 2 * nw;                                  // 16-frame halves
    const int hf = (int)(blockIdx.x % nh), brick = (int)(blockIdx.x / nh);
    const int l = threadIdx.x & 63, j = threadIdx.x >> 6;
    const int f = hf * kCullFrames + j;
    const int tx = (brick % nqx) * 4 + (l & 3);
    const int ty = ((brick / nqx) % nqy) * 4 + ((l >> 2) & 3);
    const int tz = (brick / (nqx * nqy)) * 4 + (l >> 4);
    const bool tile_ok = tx < ntx && ty < nty && tz < ntz;
    const int64_t tile = ((int64_t)tz * nty + ty) * ntx + tx;
    bool skip = false, fre = false;
    // the brick pre-pass's decision for (brick, frame f): wave-uniform
    const int dec = bdec && f < F ? bdec[(size_t)__builtin_amdgcn_readfirstlane(f) * (gridDim.x / nh) + brick] : 0;
    if (tile_ok && f < F && dec) {
        skip = dec == 1;
        fre = dec == 2;
    } else if (tile_ok && f < F) {
        const int xa = tx * kTsdfTX, xb = min(W, xa + kTsdfTX) - 1;
        const int ya = ty * kTsdfTY, yb = min(H, ya + kTsdfTY) - 1;
        const int za = z0 + tz * kTsdfTZ, zb = min(z1, za + kTsdfTZ) - 1;
        CullCam cc;
        load_cull_cam(cams, f, cc);
        cull_test(cc, G, xa, xb, ya, yb, za, zb, Hd, Wd, trunc, f, bmm, nbu, nbv, range, skip, fre);
    }
    // compact list of the projected (tile, frame) pairs: one atomic per workgroup
    const bool proj = plist && tile_ok && f < F && !skip && !fre;
    const unsigned long long bal = __ballot(proj);
    if (l == 0) wcnt[j] = (unsigned)__popcll(bal);
    bits[j][l] = (unsigned char)(skip | (fre << 1));
    __syncthreads();
    if (plist) {
        if (threadIdx.x == 0) {
            unsigned tot = 0u;
            for (int q = 0; q < kCullFrames; ++q) {
                const unsigned c = wcnt[q];
                wcnt[q] = tot;
                tot += c;
            }
            wcnt[kCullFrames] = tot ? atomicAdd(pcount, tot) : 0u;
        }
        __syncthreads();
        if (proj)
            plist[wcnt[kCullFrames] + wcnt[j] + __popcll(bal & ((1ull << l) - 1ull))] =
                ((unsigned)tile << 9) | (unsigned)f;
    }
    if (j == 0 && tile_ok) {
        unsigned cw = 0u, fw = 0u;
#pragma unroll
        for (int q = 0; q < kCullFrames; ++q) {
            const unsigned b = bits[q][l];
            cw |= (b & 1u) << q;
            fw |= (b >> 1) << q;
        }
        if (tcost) {   // the fusion's workgroup order: 4 x projected + free-space frames per wave sub-tile
            const int nlive = min(kCullFrames, F - hf * kCullFrames);
            const unsigned live = nlive >= kCullFrames ? 0xFFFFu : (nlive > 0 ? (1u << nlive) - 1u : 0u);
            const unsigned c = 4u * __popc(live & ~cw & ~fw) + __popc(live & fw & ~cw);
            if (c) atomicAdd(tcost + tile, 4u * c);
        }
        for (int q = 0; q < kCullSub; ++q) {
            const int64_t h = ((tile * kCullSub + q) * nw) * 2 + hf;   // half hf of word hf / 2
            cull[h] = (unsigned short)cw;
            freem[h] = (unsigned short)fw;
        }
    }
}

// Second, finer pass over the projected (tile, frame) pairs only: one lane per
// (pair, wave sub-tile of 8x2x8 voxels); a sub-tile proven culled or free space
// gets its bit set in its own wave slot's mask (the tile-level bits of a
// projected pair are 0, so OR-ing refines them).  Grid-stride over the device-side
// count, so the host never waits for it.
__global__ __launch_bounds__(256) void tsdf_refine_kernel(int H, int W, int z0, int z1, int F, int Hd,
                                                          int Wd, const float* __restrict__ poses,
                                                          const float* __restrict__ Kf, CullGeom G, float trunc,
                                                          const float2* __restrict__ bmm, int nbu,
                                                          int nbv, const int4* __restrict__ range, int nw,
                                                          unsigned* __restrict__ cull, unsigned* __restrict__ freem,
                                                          const unsigned* __restrict__ plist,
                                                          const unsigned* __restrict__ pcount) {
    const int ntx = (W + kTsdfTX - 1) / kTsdfTX, nty = (H + kTsdfTY - 1) / kTsdfTY;
    const int64_t n = (int64_t)(*pcount) * kCullSub;
    for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < n; g += (int64_t)gridDim.x * blockDim.x) {
        const unsigned e = plist[g >> 2];
        const int q = (int)(g & 3), f = (int)(e & 511u);
        const int64_t tile = e >> 9;
        const int tx = (int)(tile % ntx), ty = (int)((tile / ntx) % nty), tz = (int)(tile / ((int64_t)ntx * nty));
        const int xa = tx * kTsdfTX, xb = min(W, xa + kTsdfTX) - 1;
        const int ya = ty * kTsdfTY + (kTsdfTY / kCullSub) * q, yb = min(H, ya + kTsdfTY / kCullSub) - 1;
        const int za = z0 + tz * kTsdfTZ, zb = min(z1, za + kTsdfTZ) - 1;
        bool skip, fre;
        CullCam cc;   // f differs per lane here: the record from the f32 inputs
        cull_cam(poses, Kf, f, cc);
        cull_test(cc, G, xa, xb, ya, yb, za, zb, Hd, Wd, trunc, f, bmm, nbu, nbv, range, skip, fre);
        const int64_t word = (tile * kCullSub + q) * nw + (f >> 5);
        if (skip) atomicOr(cull + word, 1u << (f & 31));
        else if (fre) atomicOr(freem + word, 1u << (f & 31));
    }
}

// ---------------------------------------------------------------------------
// Whole-grid pre-pass in ONE persistent launch (round 6): the block pass streams the
// depth maps (HBM-bound, ~0.4 ms for C5) while the culling of frames whose table is
// complete runs beside it in the same workgroups, instead of after it (as separate
// brick / cull / refine launches the culling added ~0.3 ms of latency-bound work behind
// the stream; on separate streams the kernels starved each other: profiles/r6).
//   Tasks: per frame, ceil(nbv / kPreRows) stream tasks (kPreRows block rows of the
//   table each) and ceil(bricks / (8 kPreBpw)) culling tasks (kPreBpw 4x4x4 bricks of
//   tiles per wave).  Frames are dealt to 8 shards (f % 8, with the workgroups
//   blockIdx % 8); each shard hands its tasks out in ticket order, the culling tasks of
//   a frame kPreLag shard frames behind its stream tasks, so a culling task normally
//   finds its table complete.  A task's frame and the waits are shard-local, and a ticket
//   is only taken by a running workgroup, so the waits cannot cycle.
//   Hand-off (cdna_hip_programming.md §6 Guideline 16, R1): the table entries are stored
//   write-through (8-B agent-scope atomic stores), every storing wave drains, a barrier,
//   one lane adds to the frame's counter; the culling task's wave 0 polls that counter
//   relaxed (bounded, s_sleep), ONE agent acquire, a barrier, then plain vector loads.
//   A poll that gives up leaves the frame undecided (byte 0: every pair projected),
//   which the fusion evaluates in full: slower, never wrong.
//   The culling per (frame, brick), one wave: the brick's box against the full-resolution
//   table, its footprint's blocks read by all 64 lanes (culled / free space decides the
//   brick's 64 tiles); otherwise one tile per lane (cull_test), and the projected tiles'
//   4 wave sub-tiles again, 4 per projected tile spread over the wave's lanes.  One byte
//   per (frame, tile): bit 2q culled, bit 2q + 1 free space, for wave sub-tile q.
//   tsdf_pack_kernel turns the bytes into the fusion's mask words and per-tile costs.
// Every decision is the same proof as the separate passes' (cull_decide on a box that
// contains the voxels); the masks may differ from theirs, the fused grids do not.
// Measured (C5, profiles/r6/tsdf_fused_prepass_r6.txt): 0.71-0.73 ms for the launch vs 0.75 ms
// for the separate passes, but the call is 2 % slower (1.75 vs 1.71 ms): the stream tasks
// alone take 0.48 ms here (vs 0.40 in depth_blockmax_kernel, which runs at twice the waves per
// SIMD), the culling tasks alone 0.42 (vs 0.33: 4 vs 8 waves per SIMD for latency-bound tests),
// and the fusion after it runs ~25 us slower.  Selected by SFMHIP_AB=3 (tests keep it exact).
// The ticket loop's branches are on readfirstlane'd values: with the task index left in a VGPR
// the compiler restructured the loop per lane and the barriers deadlocked (first build, r6).
constexpr int kPreThreads = 512, kPreWaves = kPreThreads / 64;
constexpr int kPreRows = 4;            // table block rows per stream task
constexpr int kPreHalf = 16;           // depth rows per load batch of a stream task
constexpr int kPreBpw = 4;             // bricks per culling task per wave (dealt to the waves one by one)
constexpr int kPreLag = 4;             // shard frames between a frame's stream and culling tasks
constexpr int kPreShards = kNumXcd;
constexpr int kPreTicketStride = 32;   // words between the shards' tickets (own 128-B lines)
constexpr int kPreBrickLoads = 64;     // brick footprints of up to 64 x 64 table blocks
constexpr unsigned kPreSpinMax = 1u << 16;   // x (sc1 load + s_sleep) ~ 0.1 s
typedef __attribute__((address_space(1))) unsigned gu32;
typedef __attribute__((address_space(1))) unsigned long long gu64;

// LDS written by some lanes of a wave, then read by other lanes of the same wave
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ unsigned long long f2bits(float lo, float hi) {
    return (unsigned long long)__float_as_uint(lo) | ((unsigned long long)__float_as_uint(hi) << 32);
}

// One wave: the brick box's decision from the full-resolution table (0 undecided, 1
// culled, 2 free space); every lane computes the same footprint.
__device__ __forceinline__ int brick_decide_wave(const CullCam& cc, const CullGeom& G, int xa, int xb, int ya, int yb,
                                                 int za, int zb, int Hd, int Wd, float trunc, int f,
                                                 const float2* __restrict__ bmm, int nbu, int nbv, int4 rg, int lane) {
    int u0, u1, v0, v1;
    double zlo, zhi;
    bool inside = false;
    const int st = box_footprint(cc, G, xa, xb, ya, yb, za, zb, Hd, Wd, u0, u1, v0, v1, zlo, zhi, inside);
    if (st == 1) return 1;
    if (st != 2) return 0;
    const int bu0 = u0 / kCullBlock, bu1 = u1 / kCullBlock, bv0 = v0 / kCullBlock, bv1 = v1 / kCullBlock;
    const int nu = bu1 - bu0 + 1, nb = nu * (bv1 - bv0 + 1);
    if (nb > 64 * kPreBrickLoads || bu0 < rg.x || bu1 > rg.y || bv0 < rg.z || bv1 > rg.w) return 0;
    const float2* bp = bmm + ((size_t)f * nbv + bv0) * nbu + bu0;
    float m = -__builtin_inff(), mn = __builtin_inff();
    for (int k = lane; k < nb; k += 64) {
        const int r = k / nu;
        const float2 e = bp[(size_t)r * nbu + (k - r * nu)];
        m = fmaxf(m, e.y);
        mn = fminf(mn, e.x);
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        m = fmaxf(m, __shfl_xor(m, off, 64));
        mn = fminf(mn, __shfl_xor(mn, off, 64));
    }
    bool skip, fre;
    cull_decide(cc, trunc, m, mn, zlo, zhi, inside, skip, fre);
    return skip ? 1 : fre ? 2 : 0;
}

__global__ __launch_bounds__(kPreThreads, 4) void tsdf_prepass_kernel(
    const float* __restrict__ depth, int F, int Hd, int Wd, int nbu, int nbv, const int4* __restrict__ range,
    float2* bmm, int H, int W, int z0, int z1, const CullCam* __restrict__ cams, CullGeom G, float trunc,
    unsigned* tickets, unsigned* fdone, unsigned char* __restrict__ dec, unsigned* gaveup, int lag,
    unsigned spin_max) {
    __shared__ int s_task, s_ok, s_next;
    __shared__ int plist[kPreWaves][64];
    __shared__ unsigned char sub[kPreWaves][64][kCullSub];
    // every branch around a barrier is on a readfirstlane'd (scalar) value: the compiler must see
    // the control flow as uniform, or it may restructure the ticket loop per lane
    const int tid = threadIdx.x, lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int shard = (int)(blockIdx.x % kPreShards);
    const int ntx = (W + kTsdfTX - 1) / kTsdfTX, nty = (H + kTsdfTY - 1) / kTsdfTY;
    const int ntz = (z1 - z0 + kTsdfTZ - 1) / kTsdfTZ;
    const int nqx = (ntx + 3) >> 2, nqy = (nty + 3) >> 2, nqz = (ntz + 3) >> 2;
    const int nbricks = nqx * nqy * nqz;
    const int64_t ntiles = (int64_t)ntx * nty * ntz;
    const int rows = kPreRows, bpw = kPreBpw;
    const int ns = (nbv + rows - 1) / rows;
    const int nc = (nbricks + kPreWaves * bpw - 1) / (kPreWaves * bpw);
    const int nfs = F > shard ? (F - shard + kPreShards - 1) / kPreShards : 0;   // this shard's frames
    const int per = ns + nc;
    const int total = nfs ? (nfs + lag) * per : 0;
    gu32* tk = (gu32*)(tickets + shard * kPreTicketStride);
    for (;;) {
        if (tid == 0) s_task = (int)__hip_atomic_fetch_add(tk, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __syncthreads();
        const int t = __builtin_amdgcn_readfirstlane(s_task);
        __syncthreads();
        if (t >= total) break;
        const int blk = t / per, j = t - blk * per;
        if (j < ns && blk < nfs) {
            // ---- stream task: block rows [rows j, rows (j + 1)) of frame shard + 8 blk
            const int f = shard + kPreShards * blk;
            const int4 rg = range[f];
            const float* dp = depth + (size_t)f * Hd * Wd;
            for (int bv = j * rows; bv < min(nbv, (j + 1) * rows); ++bv) {
                if (bv < rg.z || bv > rg.w) continue;
                const int r0 = bv * kCullBlock, nr = min(kCullBlock, Hd - r0);
                for (int c0 = 0; c0 < Wd; c0 += 4 * kPreThreads) {
                    const int u = c0 + 4 * tid, bu = u / kCullBlock;
                    const bool act = u < Wd && bu >= rg.x && bu <= rg.y;
                    typedef float f4v __attribute__((ext_vector_type(4)));
                    float m = -__builtin_inff(), mn = __builtin_inff();
                    for (int h = 0; h < kCullBlock; h += kPreHalf) {   // kPreHalf rows' loads in flight
                        f4v q[kPreHalf];
#pragma unroll
                        for (int r = 0; r < kPreHalf; ++r) {   // streamed once here: non-temporal
                            q[r] = f4v{-__builtin_inff(), -__builtin_inff(), -__builtin_inff(), -__builtin_inff()};
                            if (act && h + r < nr)
                                q[r] = __builtin_nontemporal_load(
                                    reinterpret_cast<const f4v*>(dp + (size_t)(r0 + h + r) * Wd + u));
                        }
#pragma unroll
                        for (int r = 0; r < kPreHalf; ++r)
                            m = fmaxf(m, fmaxf(fmaxf(q[r].x, q[r].y), fmaxf(q[r].z, q[r].w)));
#pragma unroll
                        for (int r = 0; r < kPreHalf; ++r)
                            if (h + r < nr)
                                mn = fminf(mn, fminf(fminf(nan_low(q[r].x), nan_low(q[r].y)),
                                                     fminf(nan_low(q[r].z), nan_low(q[r].w))));
                    }
                    m = fmaxf(m, __shfl_xor(m, 1, 4));
                    m = fmaxf(m, __shfl_xor(m, 2, 4));
                    mn = fminf(mn, __shfl_xor(mn, 1, 4));
                    mn = fminf(mn, __shfl_xor(mn, 2, 4));
                    if ((tid & 3) == 0 && act && bu < nbu)   // write-through: the culling tasks read it in this launch
                        __hip_atomic_store((gu64*)(bmm + ((size_t)f * nbv + bv) * nbu + bu), f2bits(mn, m),
                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every storing wave drains
            __syncthreads();
            if (tid == 0) __hip_atomic_fetch_add((gu32*)(fdone + f), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (j < ns || blk < lag) continue;   // (scalar branch)
        // ---- culling task: bricks of part j - ns of frame shard + 8 (blk - lag)
        const int f = shard + kPreShards * (blk - lag), part = j - ns;
        if (tid == 0) {
            int ok = 1;
            unsigned spins = 0;
            while (__hip_atomic_load((gu32*)(fdone + f), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (unsigned)ns) {
                if (++spins > spin_max) { ok = 0; break; }
                __builtin_amdgcn_s_sleep(4);
            }
            if (!ok) atomicAdd(gaveup, 1u);
            s_ok = ok;
            s_next = 0;
        }
        if (wv == 0) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __syncthreads();
        const bool ok = __builtin_amdgcn_readfirstlane(s_ok) != 0;
        CullCam cc;
        load_cull_cam(cams, f, cc);
        const int4 rg = range[f];
        // the task's bricks, dealt to its waves one at a time (bricks differ in cost)
        const int b0 = part * kPreWaves * bpw, nbt = min(kPreWaves * bpw, nbricks - b0);
        for (;;) {
            int bi = 0;
            if (lane == 0) bi = atomicAdd(&s_next, 1);
            bi = __builtin_amdgcn_readfirstlane(bi);
            if (bi >= nbt) break;
            const int brick = b0 + bi;
            const int qx = brick % nqx, qy = (brick / nqx) % nqy, qz = brick / (nqx * nqy);
            const int tx = qx * 4 + (lane & 3), ty = qy * 4 + ((lane >> 2) & 3), tz = qz * 4 + (lane >> 4);
            const bool tile_ok = tx < ntx && ty < nty && tz < ntz;
            const int64_t tile = ((int64_t)tz * nty + ty) * ntx + tx;
            int bd = 0;
            if (ok) {
                const int xa = qx * 4 * kTsdfTX, xb = min(W, (qx * 4 + 4) * kTsdfTX) - 1;
                const int ya = qy * 4 * kTsdfTY, yb = min(H, (qy * 4 + 4) * kTsdfTY) - 1;
                const int za = z0 + qz * 4 * kTsdfTZ, zb = min(z1, z0 + min(ntz, qz * 4 + 4) * kTsdfTZ) - 1;
                bd = brick_decide_wave(cc, G, xa, xb, ya, yb, za, zb, Hd, Wd, trunc, f, bmm, nbu, nbv, rg, lane);
            }
            // one cull_test call site (register pressure): the lane's tile, then the projected
            // tiles' wave sub-tiles, 64 per round over the wave's lanes
            bool skip = bd == 1, fre = bd == 2, proj = false;
            int n = -1;   // -1: the tile round; then the number of projected tiles
            for (int base = 0;;) {
                int sx = tx, sy = ty, sz = tz, q = 0, l = lane, yh = kTsdfTY;
                bool valid;
                if (n < 0) {
                    valid = tile_ok && ok && bd == 0;
                } else {
                    const int it = base + lane;
                    valid = it < kCullSub * n;
                    l = plist[wv][valid ? it / kCullSub : 0];
                    q = it % kCullSub;
                    sx = qx * 4 + (l & 3), sy = qy * 4 + ((l >> 2) & 3), sz = qz * 4 + (l >> 4);
                    yh = kTsdfTY / kCullSub;
                }
                const int xa = sx * kTsdfTX, xb = min(W, xa + kTsdfTX) - 1;
                const int ya = sy * kTsdfTY + yh * q, yb = min(H, ya + yh) - 1;
                const int za = z0 + sz * kTsdfTZ, zb = min(z1, za + kTsdfTZ) - 1;
                bool s2 = false, f2v = false;
                if (valid) cull_test(cc, G, xa, xb, ya, yb, za, zb, Hd, Wd, trunc, f, bmm, nbu, nbv, range, s2, f2v);
                if (n < 0) {
                    if (valid) {
                        skip = s2;
                        fre = f2v;
                    }
                    proj = tile_ok && ok && !skip && !fre;
                    const unsigned long long bal = __ballot(proj);
                    if (proj) plist[wv][__popcll(bal & ((1ull << lane) - 1ull))] = lane;
                    wave_lds_sync();   // the lists are per wave: no workgroup barrier (bricks differ in cost)
                    n = __popcll(bal);
                } else {
                    if (valid) sub[wv][l][q] = (unsigned char)(s2 ? 1 : f2v ? 2 : 0);
                    base += 64;
                }
                if (n >= 0 && base >= kCullSub * n) break;
            }
            wave_lds_sync();
            if (tile_ok) {
                unsigned b = skip ? 0x55u : fre ? 0xAAu : 0u;
                if (proj)
                    for (int q = 0; q < kCullSub; ++q) b |= (unsigned)sub[wv][lane][q] << (2 * q);
                dec[(size_t)f * ntiles + tile] = (unsigned char)b;
            }
        }
    }
}

// Mask words and per-tile costs from the pre-pass bytes: one thread per (tile, word).
__global__ __launch_bounds__(256) void tsdf_pack_kernel(int F, int64_t ntiles, int nw,
                                                        const unsigned char* __restrict__ dec,
                                                        unsigned* __restrict__ cull, unsigned* __restrict__ freem,
                                                        unsigned* __restrict__ tcost) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= ntiles * nw) return;
    const int64_t tile = i % ntiles;
    const int w = (int)(i / ntiles);
    const int nb = min(32, F - 32 * w);
    unsigned cw[kCullSub] = {0u, 0u, 0u, 0u}, fw[kCullSub] = {0u, 0u, 0u, 0u};
    const unsigned char* dp = dec + (size_t)32 * w * ntiles + tile;
#pragma unroll 8
    for (int j = 0; j < nb; ++j) {
        const unsigned b = dp[(size_t)j * ntiles];
#pragma unroll
        for (int q = 0; q < kCullSub; ++q) {
            cw[q] |= ((b >> (2 * q)) & 1u) << j;
            fw[q] |= ((b >> (2 * q + 1)) & 1u) << j;
        }
    }
    const unsigned live = nb >= 32 ? ~0u : (1u << nb) - 1u;
    unsigned c = 0u;
#pragma unroll
    for (int q = 0; q < kCullSub; ++q) {
        const int64_t word = (tile * kCullSub + q) * nw + w;
        cull[word] = cw[q];
        freem[word] = fw[q];
        c += 4u * __popc(live & ~cw[q] & ~fw[q]) + __popc(live & fw[q] & ~cw[q]);
    }
    if (tcost && c) atomicAdd(tcost + tile, c);
}

// Validated camera records, 16 floats per frame (non-finite or >= 2^60 anywhere:
// all zero, so Zc = 0 and the frame is skipped):
//   P0 P4 | P2 P6 | P3 P7 | P8 P10 P11 | P1 P5 P9 | fx fy | cx+.5 cy+.5
__device__ __forceinline__ void tsdf_cam_record(const float* __restrict__ poses, const float* __restrict__ Kf, int f,
                                                float* __restrict__ rec) {
    float p[12], k[4];
    bool good = true;
#pragma unroll
    for (int q = 0; q < 12; ++q) { p[q] = poses[f * 12 + q]; good = good && fabsf(p[q]) < 0x1p60f; }
#pragma unroll
    for (int q = 0; q < 4; ++q) { k[q] = Kf[f * 4 + q]; good = good && fabsf(k[q]) < 0x1p60f; }
    const float r[16] = {p[0], p[4], p[2], p[6], p[3], p[7], p[8], p[10], p[11], p[1], p[5], p[9],
                         k[0], k[1], k[2] + 0.5f, k[3] + 0.5f};
#pragma unroll
    for (int q = 0; q < 16; ++q) rec[f * 16 + q] = good ? r[q] : 0.f;
}

// Per-step setup in one launch: per frame the fusion's f32 record, the culling
// passes' CullCam and the slab's block range (range_mode 1: every block, an external
// table; 2: the slab's footprint); the workgroups past the frames zero the step's
// counters (nzero words: the refinement-list counter and the per-tile costs).
__global__ __launch_bounds__(64) void tsdf_setup_kernel(const float* __restrict__ poses, const float* __restrict__ Kf,
                                                        int F, float* __restrict__ rec, CullCam* __restrict__ ccam,
                                                        int range_mode, int H, int W, int z0, int z1, int Hd, int Wd,
                                                        CullGeom G, int nbu, int nbv, int4* __restrict__ range,
                                                        unsigned* __restrict__ zero, int nzero) {
    const int fb = (F + 63) / 64;
    if ((int)blockIdx.x >= fb) {
        const int nb = gridDim.x - fb, b = blockIdx.x - fb;
        for (int i = b * 64 + threadIdx.x; i < nzero; i += nb * 64) zero[i] = 0u;
        return;
    }
    const int f = blockIdx.x * 64 + threadIdx.x;
    if (f >= F) return;
    tsdf_cam_record(poses, Kf, f, rec);
    CullCam c;
    cull_cam(poses, Kf, f, c);
    c.pad[0] = c.pad[1] = c.pad[2] = 0.0;
    ccam[f] = c;
    if (range_mode == 1) {
        range[f] = make_int4(0, nbu - 1, 0, nbv - 1);
    } else {
        int u0, u1, v0, v1;
        double zlo, zhi;
        bool inside;
        const int st = box_footprint(c, G, 0, W - 1, 0, H - 1, z0, z1 - 1, Hd, Wd, u0, u1, v0, v1, zlo, zhi, inside);
        range[f] = st == 2   ? make_int4(u0 / kCullBlock, u1 / kCullBlock, v0 / kCullBlock, v1 / kCullBlock)
                   : st == 1 ? make_int4(1, 0, 1, 0)
                             : make_int4(0, nbu - 1, 0, nbv - 1);
    }
}

// ---------------------------------------------------------------------------
// Fusion workgroup order.  One 8x8x8 tile per workgroup (4 waves = its 4 wave
// sub-tiles).  Spatially compact "super-bricks" of SB_X x SB_Y x SB_Z tiles, dealt
// round-robin over the 8 XCDs (the 1-D grid's slot % 8 is its XCD): workgroups resident
// on one XCD at the same time project onto one compact image region per frame, so the
// depth lines they gather meet in that XCD's L2, and the round-robin spreads the uneven
// culled work (the floor plane, the spheres) over the XCDs (speed only, never
// correctness).  A y-band per XCD instead (every ray of the nearly horizontal orbit
// cameras in one XCD) measured 1.97 vs 1.17 ms: the floor's band holds most of the work.
//   tsdf_slot_tile: (slot) -> tile, false for padding slots
//   tsdf_order_kernel: longest-first order within each XCD class (the cull pass sums each
//     tile's cost): the surface tiles, up to ~10x the work of a free-space tile, would
//     otherwise land in the last round of a short call (a z-slab of an N-way split).
struct SlotMap { int ntx, nty, ntz, sbx, sby, sbz, nsx, nsy, per; };   // per: slots per XCD class

static SlotMap make_slot_map(int ntx, int nty, int ntz) {
    SlotMap m;
    m.ntx = ntx;
    m.nty = nty;
    m.ntz = ntz;
    // 1 x 2 x 8 tiles (8 x 16 x 64 voxels): round-6 sweep of the shipped fusion over 23 shapes
    // (profiles/r6/tsdf_superbrick_sweep_r6.txt): C5 call 1.68 vs 1.73 ms for round 2's 3 x 2 x 8,
    // the N = 8 slabs 3-4 % faster; the small super-bricks deal the costly surface columns over the
    // XCDs more evenly
    m.sbx = 1;
    m.sby = 2;
    m.sbz = std::min(8, ntz);
    m.nsx = ceil_div(ntx, m.sbx);
    m.nsy = ceil_div(nty, m.sby);
    const int nsb = m.nsx * m.nsy * ceil_div(ntz, m.sbz);
    m.per = ceil_div(nsb, kNumXcd) * m.sbx * m.sby * m.sbz;   // padding super-bricks exit at once
    return m;
}

__device__ __forceinline__ bool tsdf_slot_tile(int slot, const SlotMap& m, int& tx, int& ty, int& tz) {
    const int j = slot / kNumXcd, sbn = m.sbx * m.sby * m.sbz;
    const int sb = (j / sbn) * kNumXcd + slot % kNumXcd, in = j % sbn;
    tx = (sb % m.nsx) * m.sbx + in % m.sbx;
    ty = ((sb / m.nsx) % m.nsy) * m.sby + (in / m.sbx) % m.sby;
    tz = (sb / (m.nsx * m.nsy)) * m.sbz + in / (m.sbx * m.sby);
    return tx < m.ntx && ty < m.nty && tz < m.ntz;
}

constexpr int kOrderBuckets = 64;
__device__ __forceinline__ unsigned slot_bucket(int s, const SlotMap& m, int F, const unsigned* __restrict__ tcost) {
    int tx, ty, tz;
    const bool ok = tsdf_slot_tile(s, m, tx, ty, tz);
    const unsigned cost = ok ? tcost[((size_t)tz * m.nty + ty) * m.ntx + tx] : 0u;
    return min((unsigned)(kOrderBuckets - 1), cost * kOrderBuckets / (16u * F + 1u));
}

// One workgroup per XCD class, stable counting sort of the class's slots by cost
// bucket, heaviest first: order[x + 8 k] = k-th slot.  Dynamic LDS: one bucket byte per
// slot of the class (m <= 30000, host-checked).
__global__ __launch_bounds__(256) void tsdf_order_kernel(SlotMap SM, int F, const unsigned* __restrict__ tcost,
                                                         unsigned* __restrict__ order) {
    __shared__ unsigned short hist[kOrderBuckets][256];
    __shared__ unsigned wsum[4];
    extern __shared__ unsigned char bk[];
    const int x = blockIdx.x, t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const int m = SM.per;   // slots x, x+8, ... of this class
    const int per = (m + 255) / 256, j0 = min(m, t * per), j1 = min(m, j0 + per);
    for (int b = 0; b < kOrderBuckets; ++b) hist[b][t] = 0;
    for (int j = t; j < m; j += 256)   // coalesced over the class: every cost load in flight
        bk[j] = (unsigned char)slot_bucket(x + kNumXcd * j, SM, F, tcost);
    __syncthreads();
    for (int j = j0; j < j1; ++j) ++hist[bk[j]][t];
    __syncthreads();
    // exclusive scan over (bucket descending, thread): thread u owns entries [64u, 64u + 64)
    unsigned run = 0;
    for (int e = 64 * t; e < 64 * t + 64; ++e) run += hist[kOrderBuckets - 1 - e / 256][e % 256];
    unsigned incl = run;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const unsigned up = __shfl_up(incl, off, 64);
        if (lane >= off) incl += up;
    }
    if (lane == 63) wsum[wv] = incl;
    __syncthreads();
    unsigned base = 0;
    for (int w = 0; w < wv; ++w) base += wsum[w];
    run = base + incl - run;
    for (int e = 64 * t; e < 64 * t + 64; ++e) {
        unsigned short& h = hist[kOrderBuckets - 1 - e / 256][e % 256];
        const unsigned v = h;
        h = (unsigned short)run;   // positions < m <= 65535
        run += v;
    }
    __syncthreads();
    for (int j = j0; j < j1; ++j) {
        const unsigned pos = hist[bk[j]][t]++;
        order[x + kNumXcd * pos] = (unsigned)(x + kNumXcd * j);
    }
}

constexpr int kCntPl = 0, kNCnt = 4;   // counters: the refinement list

// Voxel of lane l in wave sub-tile q of tile (bx, by, bz): each 16-lane quarter-wave
// is a 4x4 (x, z) patch at one y (the orbiting cameras map y to image rows: a compact
// x-z patch has the fewest distinct depth rows), each lane two y-adjacent voxels run
// as one packed-f32 pair (v_pk_* ops).
__device__ __forceinline__ void sub_voxel(int64_t sub, int ntx, int nty, int z0, int l, int& x, int& y, int& z) {
    const int64_t tile = sub / kCullSub;
    const int q = (int)(sub % kCullSub);
    const int bx = (int)(tile % ntx), by = (int)((tile / ntx) % nty), bz = (int)(tile / ((int64_t)ntx * nty));
    x = bx * kTsdfTX + (l & 3) + 4 * ((l >> 4) & 1);
    z = z0 + bz * kTsdfTZ + ((l >> 2) & 3) + 4 * (l >> 5);
    y = by * kTsdfTY + 2 * q;
}

// The step's finish of one voxel: n updates with fixed-point sum S.
__device__ __forceinline__ void tsdf_finish_voxel(float& t, float& w, int S, int n) {
    const double num = (double)t * (double)w + (double)S * 0x1p-21;
    const double den = (double)w + (double)n;
    t = (float)(num / den);
    w = w + (float)n;
}

struct FrameCtx {
    const float* rec;
    const float* depth;
    const float2* bmm;
    size_t frame;
    int nbytes, Wd4, Hd, Wd, nbu, nbv;
    float trunc, inv_trunc;
};

// The same evaluation for NF frames at once, in stages, so that every stage's loads
// of all NF frames are in flight together (one basic block: the boolean logic is
// bitwise, loads a lane does not need get the out-of-range offset, which the buffer
// load drops without a cache access): projections -> block-table loads -> block
// tests and depth loads -> tsdf.  The second voxel of a lane reads the table only
// when its block differs from the first voxel's.
template <bool VT, int NF>
__device__ __forceinline__ void frames_eval(const FrameCtx& c, const int* f, float vx, f2 vy, float vz, bool two,
                                            int* q0, int* q1, bool* g0, bool* g1) {
    f2 Zc[NF];
    int iu0[NF], iv0[NF], iu1[NF], iv1[NF];
    bool ok0[NF], ok1[NF];
#pragma unroll
    for (int k = 0; k < NF; ++k) {
        const float* r = c.rec + f[k] * 16;   // uniform: scalar loads
        const f2 Q = (f2{r[0], r[1]} * f2s(vx) + f2{r[2], r[3]} * f2s(vz)) + f2{r[4], r[5]};
        const float Qz = (r[6] * vx + r[7] * vz) + r[8];
        const f2 Xc = f2s(r[9]) * vy + f2s(Q.x);
        const f2 Yc = f2s(r[10]) * vy + f2s(Q.y);
        Zc[k] = f2s(r[11]) * vy + f2s(Qz);
        const f2 iz = recip_rn(Zc[k]);
        const f2 uu = (f2s(r[12]) * Xc) * iz + f2s(r[14]);
        const f2 vv = (f2s(r[13]) * Yc) * iz + f2s(r[15]);
        iu0[k] = cvt_flr(uu.x);
        iv0[k] = cvt_flr(vv.x);
        iu1[k] = cvt_flr(uu.y);
        iv1[k] = cvt_flr(vv.y);
        ok0[k] = z_ok(Zc[k].x) & ((unsigned)iu0[k] < (unsigned)c.Wd) & ((unsigned)iv0[k] < (unsigned)c.Hd);
        ok1[k] = two & z_ok(Zc[k].y) & ((unsigned)iu1[k] < (unsigned)c.Wd) & ((unsigned)iv1[k] < (unsigned)c.Hd);
    }
    bool fr0[NF], fr1[NF], need0[NF], need1[NF];
    if constexpr (VT) {
        unsigned b0[NF], b1[NF];
        uint64_t e0[NF], e1[NF];
        const unsigned tb = (unsigned)(c.nbv * c.nbu * 8);
#pragma unroll
        for (int k = 0; k < NF; ++k) {
            // 24-bit multiplies (v_mad_u32_u24, full rate): block indices are < 2^20 in range
            b0[k] = __umul24((unsigned)(iv0[k] >> 4) & 0xFFFFFFu, (unsigned)c.nbu) + ((unsigned)iu0[k] >> 4);
            b1[k] = __umul24((unsigned)(iv1[k] >> 4) & 0xFFFFFFu, (unsigned)c.nbu) + ((unsigned)iu1[k] >> 4);
            const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(
                (void*)(c.bmm + (size_t)f[k] * c.nbv * c.nbu), (short)0, (int)tb, 0x00020000);
            const auto x0 = __builtin_amdgcn_raw_buffer_load_b64(rb, (int)(ok0[k] ? b0[k] << 3 : tb), 0, 0);
            const auto x1 = __builtin_amdgcn_raw_buffer_load_b64(rb, (int)((ok1[k] & (b1[k] != b0[k])) ? b1[k] << 3 : tb),
                                                                 0, 0);
            e0[k] = ((uint64_t)(unsigned)x0[1] << 32) | (unsigned)x0[0];
            e1[k] = ((uint64_t)(unsigned)x1[1] << 32) | (unsigned)x1[0];
        }
#pragma unroll
        for (int k = 0; k < NF; ++k) {
            const uint64_t e1k = b1[k] == b0[k] ? e0[k] : e1[k];
            const f2 bmn = {__builtin_bit_cast(float, (unsigned)e0[k]), __builtin_bit_cast(float, (unsigned)e1k)};
            const f2 bmx = {__builtin_bit_cast(float, (unsigned)(e0[k] >> 32)),
                            __builtin_bit_cast(float, (unsigned)(e1k >> 32))};
            const f2 scm = (bmn - Zc[k]) * f2s(c.inv_trunc);
            const f2 smx = bmx - Zc[k];
            fr0[k] = ok0[k] & (bmn.x > 0.f) & (scm.x >= 1.f);
            fr1[k] = ok1[k] & (bmn.y > 0.f) & (scm.y >= 1.f);
            need0[k] = ok0[k] & !fr0[k] & (bmx.x > 0.f) & !(smx.x < -c.trunc);
            need1[k] = ok1[k] & !fr1[k] & (bmx.y > 0.f) & !(smx.y < -c.trunc);
        }
    } else {
#pragma unroll
        for (int k = 0; k < NF; ++k) {
            fr0[k] = fr1[k] = false;
            need0[k] = ok0[k];
            need1[k] = ok1[k];
        }
    }
    f2 dep[NF];
    const unsigned oob = (unsigned)c.nbytes;
#pragma unroll
    for (int k = 0; k < NF; ++k) {
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(c.depth + (size_t)f[k] * c.frame), (short)0, c.nbytes, 0x00020000);
        dep[k] = f2{__builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                         rs, (int)(need0[k] ? __umul24(iv0[k], c.Wd4) + ((unsigned)iu0[k] << 2) : oob), 0, 0)),
                     __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                         rs, (int)(need1[k] ? __umul24(iv1[k], c.Wd4) + ((unsigned)iu1[k] << 2) : oob), 0, 0))};
    }
#pragma unroll
    for (int k = 0; k < NF; ++k) {
        const f2 sdf = dep[k] - Zc[k];
        g0[k] = fr0[k] | (need0[k] & (dep[k].x > 0.f) & !(sdf.x < -c.trunc));
        g1[k] = fr1[k] | (need1[k] & (dep[k].y > 0.f) & !(sdf.y < -c.trunc));
        const f2 sc = sdf * f2s(c.inv_trunc);
        const f2 qs = f2{fminf(1.0f, sc.x), fminf(1.0f, sc.y)} * f2s(0x1p21f);   // exact (power-of-two scale)
        q0[k] = fr0[k] ? (1 << kTsdfQBits) : (int)__builtin_rintf(qs.x);
        q1[k] = fr1[k] ? (1 << kTsdfQBits) : (int)__builtin_rintf(qs.y);
    }
}

// One wave = one wave sub-tile (8 x 2 x 8 voxels, two per lane): a sub-tile with every
// frame culled returns before touching the grid.  Walks the sub-tile's mask words
// (scalar): culled frames are skipped, free-space frames add 2^21 and 1 per voxel, the
// projected frames are evaluated two at a time (three or four in flight measured the
// same: 1.13 / 1.16 ms, profiles/r5).  The voxels are finished in place (grid read and
// written once, only where a voxel updated).
// Splitting a surface sub-tile's frames over several waves (integer sums make any split
// exact; partial sums + a finish pass) measured slower in both modes: whole grid 1.19 vs
// 1.13 ms, an N = 8 slab 0.33 vs 0.28 ms (profiles/r5): the fusion is bound by the gather
// traffic, not by its longest sub-tiles.  Walking each wave's frames from a wall-clock
// phase (so that resident waves gather from the same frames at the same time) and
// frame-window-major work lists (32-frame windows over the whole grid, partial sums)
// did not raise the L2 hit rate (23 -> 26 %) and measured slower too.
// NFS: projected frames evaluated per stage (their loads in flight together): 2 when the grid
// is many rounds of resident waves (throughput: three or four measured no faster), 4 for a thin
// z-slab (an N-way split: a couple of rounds, the call is its heaviest waves' frame chains).
template <bool VT, int NFS = 2>
__global__ __launch_bounds__(256) void tsdf_fuse_kernel(float* __restrict__ T, float* __restrict__ Wt, int D,
                                                        int H, int W, int z0, int z1, FrameCtx c, GridBox B, int F,
                                                        SlotMap SM, const unsigned* __restrict__ cull,
                                                        const unsigned* __restrict__ freem, int nw,
                                                        const unsigned* __restrict__ order) {
    const int l = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    int tx, ty, tz;
    if (!tsdf_slot_tile(order ? (int)order[blockIdx.x] : (int)blockIdx.x, SM, tx, ty, tz)) return;
    const int64_t sub = (((int64_t)tz * SM.nty + ty) * SM.ntx + tx) * kCullSub + wave;
    const size_t slot = (size_t)sub * nw;
    {   // every frame culled for this wave: the grid is not even read
        unsigned any = 0u;
        for (int w = 0; w < nw; ++w) {
            const int w0 = w << 5;
            any |= ~cull[slot + w] & (F - w0 >= 32 ? ~0u : ((1u << (F - w0)) - 1u));
        }
        if (__builtin_amdgcn_readfirstlane((int)any) == 0) return;
    }
    int x, y, z;
    sub_voxel(sub, SM.ntx, SM.nty, z0, l, x, y, z);
    if (y >= H) return;                      // wave-uniform (a ragged last tile row)
    const bool in0 = x < W && z < z1;
    const bool two = in0 && y + 1 < H;
    const float sx = (B.mx[0] - B.mn[0]) / (float)(W - 1);
    const float sy = (B.mx[1] - B.mn[1]) / (float)(H - 1);
    const float sz = (B.mx[2] - B.mn[2]) / (float)(D - 1);
    const float vx = B.mn[0] + (float)x * sx;
    const f2 vy = {B.mn[1] + (float)y * sy, B.mn[1] + (float)(y + 1) * sy};
    const float vz = B.mn[2] + (float)z * sz;
    int S0 = 0, S1 = 0, n0 = 0, n1 = 0;
    int kfree = 0;                           // free-space frames
    int pend[NFS], np = 0;                   // projected frames waiting for a full stage
    auto add = [&](int q0, int q1, bool g0, bool g1) {
        S0 += g0 ? q0 : 0;
        n0 += g0 ? 1 : 0;
        S1 += g1 ? q1 : 0;
        n1 += g1 ? 1 : 0;
    };
    for (int w = 0; w < nw; ++w) {
        const int w0 = w << 5;
        const unsigned live = F - w0 >= 32 ? ~0u : ((1u << (F - w0)) - 1u);
        const unsigned todo = (unsigned)__builtin_amdgcn_readfirstlane((int)(live & ~cull[slot + w]));
        const unsigned fre = (unsigned)__builtin_amdgcn_readfirstlane((int)freem[slot + w]) & todo;
        unsigned proj = todo & ~fre;
        kfree += __builtin_popcount(fre);
        while (proj) {
            pend[np++] = w0 + __builtin_ctz(proj);
            proj &= proj - 1u;
            if (np < NFS) continue;
            int qa[NFS], qb[NFS];
            bool ga[NFS], gb[NFS];
            frames_eval<VT, NFS>(c, pend, vx, vy, vz, two, qa, qb, ga, gb);
#pragma unroll
            for (int k = 0; k < NFS; ++k) add(qa[k], qb[k], ga[k], gb[k]);
            np = 0;
        }
    }
    for (int k = 0; k < np; ++k) {   // the last stage's remainder, one frame at a time
        int qa[1], qb[1];
        bool ga[1], gb[1];
        frames_eval<VT, 1>(c, pend + k, vx, vy, vz, two, qa, qb, ga, gb);
        add(qa[0], qb[0], ga[0], gb[0]);
    }
    S0 += kfree << kTsdfQBits;   // free space: tsdf = 1 for every voxel of the sub-tile
    S1 += kfree << kTsdfQBits;
    n0 += kfree;
    n1 += kfree;
    if (!in0) return;
    const size_t idx = ((size_t)z * H + y) * W + x;
    if (n0 > 0) {
        float t = T[idx], wt = Wt[idx];
        tsdf_finish_voxel(t, wt, S0, n0);
        T[idx] = t;
        Wt[idx] = wt;
    }
    if (two && n1 > 0) {
        float t = T[idx + W], wt = Wt[idx + W];
        tsdf_finish_voxel(t, wt, S1, n1);
        T[idx + W] = t;
        Wt[idx + W] = wt;
    }
}

// ---------------------------------------------------------------------------
// Host.  Knob (read once, sfmhip_knobs_reload re-reads it: lib.hip):
//   SFMHIP_TSDF_LATENCY  -1 auto (default), 0 whole-grid mode, 1 latency mode
// Latency mode (less than one resident round of fusion waves): no brick pre-pass, no
// refinement pass, no per-voxel block test.  Round 3's sequential fusion put an N = 8 z-slab
// (two rounds) in it (0.39 vs 0.44 ms); with the order-free fusion the whole-grid mode is
// faster there: slowest N = 8 slab 0.29-0.30 vs 0.31-0.35 ms (profiles/r5/tsdf_slabs_r5.txt).
// stats != nullptr: run only the culling pre-passes and count (wave sub-tile, frame)
// pairs: stats[0] tested, [1] culled, [2] free space (layer_stats: per 8-voxel z layer).
// ext_table != nullptr: the caller's {min, max} block table of every frame over the
// whole image ([F][nbv][nbu] float2, sfmhip_tsdf_block_table); the block pass is skipped.
static int tsdf_run(float* T, float* Wt, int D, int H, int W, int z0, int z1, const float* depth, int F, int Hd,
                    int Wd, const float* poses, const float* Kf, const float* bmin, const float* bmax, float trunc,
                    void* stream, int64_t* stats, const float2* ext_table, int64_t* layer_stats = nullptr) {
    // F = 0: nothing to fuse, the frame arrays may be null (an empty tensor's pointer)
    SFMHIP_REQUIRE(D > 1 && H > 1 && W > 1 && F >= 0 && Hd > 0 && Wd > 0, "sfmhip_tsdf_integrate: bad shape");
    SFMHIP_REQUIRE(0 <= z0 && z0 <= z1 && z1 <= D, "sfmhip_tsdf_integrate: bad z range");
    SFMHIP_REQUIRE(trunc > 0.f, "sfmhip_tsdf_integrate: trunc must be > 0");
    if (F == 0 || z0 == z1) return SFMHIP_OK;
    SFMHIP_REQUIRE(T && Wt && bmin && bmax && (F == 0 || (depth && poses && Kf)), "sfmhip_tsdf_integrate: null pointer");
    SFMHIP_REQUIRE((int64_t)Hd * Wd * 4 < (int64_t)INT_MAX && Wd < (1 << 22) && Hd < (1 << 22),
                   "sfmhip_tsdf_integrate: depth map too large (4*Hd*Wd must be < 2^31)");
    for (int a = 0; a < 3; ++a)
        SFMHIP_REQUIRE(std::fabs(bmin[a]) < 0x1p60f && std::fabs(bmax[a]) < 0x1p60f,
                       "sfmhip_tsdf_integrate: bounds must be finite and below 2^60 in magnitude");
    const int nbx = ceil_div(W, kTsdfTX), nby = ceil_div(H, kTsdfTY), nbz = ceil_div(z1 - z0, kTsdfTZ);
    const int64_t ntiles = (int64_t)nbx * nby * nbz, nsub = ntiles * kCullSub;
    SFMHIP_REQUIRE(nsub < (1 << 27) && ntiles < (1 << 23), "sfmhip_tsdf_integrate: grid too large");
    const SlotMap sm = make_slot_map(nbx, nby, nbz);
    const int64_t main_slots = (int64_t)sm.per * kNumXcd;
    SFMHIP_REQUIRE(main_slots < INT_MAX / 2, "sfmhip_tsdf_integrate: grid too large");
    const Knobs kn = knobs();
    int ncu = 256;
    {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
            ncu = 256;
        (void)hipGetLastError();
    }
    const double rounds = (double)nsub / (ncu * 32.0);   // 8 waves per SIMD
    const bool latency_mode = kn.tsdf_latency >= 0 ? kn.tsdf_latency != 0 : rounds < kTsdfLatencyRounds;
    // a thin slab (fewer than kTsdfDeepRounds rounds of resident fusion waves: a z-slab of an N >= 4
    // split): four projected frames per fusion stage and no brick / refinement pre-passes (their
    // fixed cost outweighs the fusion work they save there); SFMHIP_AB=1 (2) keeps the whole-grid
    // form with the separate (fused) pre-passes
    const bool deep = rounds < kTsdfDeepRounds && kn.ab != 1 && kn.ab != 3 && kn.ab != 31;
    const bool refine = !latency_mode && !deep;
    const bool brick = !latency_mode && !deep;
    const bool vox_test = !latency_mode;
    // SFMHIP_AB=3: the whole-grid pre-passes as one persistent launch (tsdf_prepass_kernel) instead
    // of the separate block / brick / cull / refine launches: bit-identical grids, measured 2 %
    // slower on C5 (1.75 vs 1.71 ms: profiles/r6/tsdf_fused_prepass_r6.txt), so not the default
    const bool fusedpre = brick && !ext_table && !stats && Wd % 4 == 0 && (kn.ab == 3 || kn.ab == 31);
    // SFMHIP_AB=31 (tests): the fused pre-pass with no lag and no patience, so culling tasks give up
    // on frames whose table is not complete yet: the undecided fallback must give the same grid
    const bool pre_stress = kn.ab == 31;
    GridBox gb;
    CullGeom cg;
    {
        const int n[3] = {W, H, D};
        for (int a = 0; a < 3; ++a) {
            gb.mn[a] = bmin[a];
            gb.mx[a] = bmax[a];
            cg.mn[a] = gb.mn[a];
            cg.s[a] = ((double)gb.mx[a] - gb.mn[a]) / (n[a] - 1);
            cg.as[a] = std::fabs(cg.s[a]);
        }
    }
    hipStream_t st = as_stream(stream);
    const int nbu = ceil_div(Wd, kCullBlock), nbv = ceil_div(Hd, kCullBlock);
    const int cf = std::min(kTsdfMaxFrames, F);
    const int nwmax = ceil_div(cf, 32);
    const int64_t cull_bricks = (int64_t)ceil_div(nbx, 4) * ceil_div(nby, 4) * ceil_div(nbz, 4);
    SFMHIP_REQUIRE(cull_bricks * 2 * nwmax < INT_MAX, "sfmhip_tsdf_integrate: grid too large");
    const int ncbu = ceil_div(nbu, kCoarse), ncbv = ceil_div(nbv, kCoarse);
    // refinement list capacity: one entry per (tile, frame)
    const int64_t plist_cap = ntiles * 32 * nwmax;
    const bool order = !stats && sm.per <= 30000;
    // scratch (stream-ordered, one block): counters + per-tile costs first (zeroed by the setup kernel)
    size_t off = 0;
    auto take = [&](size_t bytes) { const size_t o = off; off += (bytes + 255) & ~(size_t)255; return o; };
    // zeroed words: [pre-pass tickets, one 128-B line per shard] [counters] [per-tile costs] [frame counters]
    const int n_tk = fusedpre ? kPreShards * kPreTicketStride : 0;
    const int nzero = n_tk + kNCnt + (order ? (int)ntiles : 0) + (fusedpre ? cf : 0);
    const size_t o_cnt = take((size_t)nzero * sizeof(unsigned));
    const size_t o_rec = take((size_t)cf * 16 * sizeof(float));
    const size_t o_cam = take((size_t)cf * sizeof(CullCam));
    const size_t o_rng = take((size_t)cf * sizeof(int4));
    const size_t o_bmm = ext_table ? 0 : take((size_t)cf * nbu * nbv * sizeof(float2));
    const size_t o_msk = take((size_t)nsub * nwmax * sizeof(unsigned));
    const size_t o_fre = take((size_t)nsub * nwmax * sizeof(unsigned));
    const bool sep = brick && !fusedpre;
    const size_t o_ctab = sep ? take((size_t)cf * ncbu * ncbv * sizeof(float2)) : 0;
    const size_t o_bdec = sep ? take((size_t)cull_bricks * cf) : 0;
    const size_t o_pl = refine && !fusedpre ? take((size_t)plist_cap * sizeof(unsigned)) : 0;
    const size_t o_dec = fusedpre ? take((size_t)cf * ntiles) : 0;
    const size_t o_ord = order ? take((size_t)main_slots * sizeof(unsigned)) : 0;
    char* sc = nullptr;
    if (scratch_alloc((void**)&sc, off, st) != hipSuccess) {
        (void)hipGetLastError();
        set_error("sfmhip_tsdf_integrate: scratch allocation of %zu bytes failed", off);
        return SFMHIP_E_HIP;
    }
    unsigned* zbase = reinterpret_cast<unsigned*>(sc + o_cnt);
    unsigned* tickets = zbase;
    unsigned* cnt = zbase + n_tk;
    unsigned* tcost = order ? cnt + kNCnt : nullptr;
    unsigned* fdone = cnt + kNCnt + (order ? ntiles : 0);
    unsigned char* pdec = fusedpre ? reinterpret_cast<unsigned char*>(sc + o_dec) : nullptr;
    float* rec = reinterpret_cast<float*>(sc + o_rec);
    CullCam* ccam = reinterpret_cast<CullCam*>(sc + o_cam);
    int4* crange = reinterpret_cast<int4*>(sc + o_rng);
    float2* cbmm = ext_table ? nullptr : reinterpret_cast<float2*>(sc + o_bmm);
    unsigned* cmask = reinterpret_cast<unsigned*>(sc + o_msk);
    unsigned* cfree = reinterpret_cast<unsigned*>(sc + o_fre);
    float2* ctab = sep ? reinterpret_cast<float2*>(sc + o_ctab) : nullptr;
    unsigned char* bdec = sep ? reinterpret_cast<unsigned char*>(sc + o_bdec) : nullptr;
    unsigned* plist = refine && !fusedpre ? reinterpret_cast<unsigned*>(sc + o_pl) : nullptr;
    int pre_grid = 0;
    if (fusedpre) {   // the persistent grid: every resident workgroup, a multiple of the shard count
        int nb = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, tsdf_prepass_kernel, kPreThreads, 0) != hipSuccess ||
            nb <= 0)
            nb = 1;
        (void)hipGetLastError();
        pre_grid = std::max(kPreShards, nb * ncu / kPreShards * kPreShards);
    }
    unsigned* ord = order ? reinterpret_cast<unsigned*>(sc + o_ord) : nullptr;
    int rc = SFMHIP_OK;
    // integration steps of at most kTsdfMaxFrames frames, in order on the stream
    for (int f0 = 0; f0 < F; f0 += kTsdfMaxFrames) {
        const int nf = std::min(kTsdfMaxFrames, F - f0);
        const int nw = ceil_div(nf, 32);
        const float* dp = depth + (size_t)f0 * Hd * Wd;
        const float* pp = poses + (size_t)f0 * 12;
        const float* kp = Kf + (size_t)f0 * 4;
        hipLaunchKernelGGL(tsdf_setup_kernel, dim3(ceil_div(nf, 64) + std::min(64, ceil_div(nzero, 1024) + 1)),
                           dim3(64), 0, st, pp, kp, nf, rec, ccam, ext_table ? 1 : 2, H, W, z0, z1, Hd, Wd, cg, nbu,
                           nbv, crange, zbase, nzero);
        const float2* tab = ext_table ? ext_table + (size_t)f0 * nbv * nbu : cbmm;
        if (fusedpre) {
            hipLaunchKernelGGL(tsdf_prepass_kernel, dim3(pre_grid), dim3(kPreThreads), 0, st, dp, nf, Hd, Wd, nbu, nbv,
                               crange, cbmm, H, W, z0, z1, ccam, cg, trunc, tickets, fdone, pdec, cnt + 1,
                               pre_stress ? 0 : kPreLag, pre_stress ? 0u : kPreSpinMax);
            hipLaunchKernelGGL(tsdf_pack_kernel, dim3((unsigned)ceil_div(ntiles * nw, (int64_t)256)), dim3(256), 0, st,
                               nf, ntiles, nw, pdec, cmask, cfree, tcost);
        } else if (!ext_table) {
            if (Wd % 4 == 0)
                hipLaunchKernelGGL(depth_blockmax_kernel<true>, dim3(ceil_div(Wd, 1024), nbv, nf), dim3(256), 0, st,
                                   dp, nf, Hd, Wd, nbu, nbv, crange, cbmm);
            else
                hipLaunchKernelGGL(depth_blockmax_kernel<false>, dim3(ceil_div(Wd, 256), nbv, nf), dim3(256), 0, st,
                                   dp, nf, Hd, Wd, nbu, nbv, crange, cbmm);
        }
        if (sep) {
            const int64_t nc = (int64_t)nf * ncbu * ncbv, nd = (cull_bricks + 63) / 64 * 64 * nf;
            hipLaunchKernelGGL(coarse_table_kernel, dim3((unsigned)ceil_div(nc, (int64_t)256)), dim3(256), 0, st, tab,
                               nf, nbu, nbv, ncbu, ncbv, ext_table ? nullptr : crange, ctab);
            hipLaunchKernelGGL(tsdf_brick_kernel, dim3((unsigned)ceil_div(nd, (int64_t)256)), dim3(256), 0, st, H, W,
                               z0, z1, nf, Hd, Wd, ccam, cg, trunc, ctab, ncbu, ncbv, (int)cull_bricks, bdec);
        }
        if (!fusedpre)
            hipLaunchKernelGGL(tsdf_cull_kernel, dim3((unsigned)(cull_bricks * nw * 2)), dim3(1024), 0, st, H, W, z0,
                               z1, nf, Hd, Wd, ccam, cg, trunc, tab, nbu, nbv, crange, nw, bdec,
                               (unsigned short*)cmask, (unsigned short*)cfree, plist, cnt + kCntPl, tcost);
        // refinement: grid-stride over the device-side count (atomic ORs: any grid gives the
        // same masks); 8192 x 256 threads fill the 6 waves per SIMD its VGPRs allow
        if (plist)
            hipLaunchKernelGGL(tsdf_refine_kernel, dim3(8192), dim3(256), 0, st, H, W, z0, z1, nf, Hd, Wd, pp, kp, cg,
                               trunc, tab, nbu, nbv, crange, nw, cmask, cfree, plist, cnt + kCntPl);
        if (stats) {
            std::vector<unsigned> mc((size_t)nsub * nw), mf((size_t)nsub * nw);
            hipError_t e = hipMemcpyAsync(mc.data(), cmask, mc.size() * sizeof(unsigned), hipMemcpyDeviceToHost, st);
            if (e == hipSuccess)
                e = hipMemcpyAsync(mf.data(), cfree, mf.size() * sizeof(unsigned), hipMemcpyDeviceToHost, st);
            if (e == hipSuccess) e = hipStreamSynchronize(st);
            if (e != hipSuccess) {
                set_error("sfmhip_tsdf_cull_stats: %s", hipGetErrorString(e));
                rc = SFMHIP_E_HIP;
                break;
            }
            for (size_t i = 0; i < mc.size(); ++i) {
                const int nb = std::min(32, nf - 32 * (int)(i % nw));
                const unsigned live = nb >= 32 ? ~0u : ((1u << nb) - 1u);
                const int tested = nb, culled = __builtin_popcount(mc[i] & live);
                const int fre = __builtin_popcount(mf[i] & live & ~mc[i]);
                stats[0] += tested;
                stats[1] += culled;
                stats[2] += fre;
                if (layer_stats) {   // slot = tile * kCullSub + wave, tile = (tz * nby + ty) * nbx + tx
                    const int64_t tile = (int64_t)(i / nw) / kCullSub;
                    int64_t* ls = layer_stats + 3 * (tile / ((int64_t)nbx * nby));
                    ls[0] += tested;
                    ls[1] += culled;
                    ls[2] += fre;
                }
            }
            continue;
        }
        if (ord)   // longest-first workgroup order within each XCD class (same results)
            hipLaunchKernelGGL(tsdf_order_kernel, dim3(kNumXcd), dim3(256), (size_t)sm.per, st, sm, nf, tcost, ord);
        FrameCtx fc;
        fc.rec = rec;
        fc.depth = dp;
        fc.bmm = tab;
        fc.frame = (size_t)Hd * Wd;
        fc.nbytes = (int)(fc.frame * 4);
        fc.Wd4 = Wd * 4;
        fc.Hd = Hd;
        fc.Wd = Wd;
        fc.nbu = nbu;
        fc.nbv = nbv;
        fc.trunc = trunc;
        fc.inv_trunc = 1.0f / trunc;
        if (deep)
            hipLaunchKernelGGL((vox_test ? tsdf_fuse_kernel<true, 4> : tsdf_fuse_kernel<false, 4>),
                               dim3((unsigned)main_slots), dim3(256), 0, st, T, Wt, D, H, W, z0, z1, fc, gb, nf, sm,
                               cmask, cfree, nw, ord);
        else
            hipLaunchKernelGGL((vox_test ? tsdf_fuse_kernel<true, 2> : tsdf_fuse_kernel<false, 2>),
                               dim3((unsigned)main_slots), dim3(256), 0, st, T, Wt, D, H, W, z0, z1, fc, gb, nf, sm,
                               cmask, cfree, nw, ord);
        rc = check_launch("tsdf_fuse_kernel");
        if (rc != SFMHIP_OK) break;
    }
    scratch_free(sc, st);
    return rc;
}

}  // namespace sfmhip

using namespace sfmhip;

extern "C" int sfmhip_tsdf_integrate(float* T, float* Wt, int D, int H, int W, int z0, int z1,
                                     const float* depth, int F, int Hd, int Wd, const float* poses,
                                     const float* Kf, const float* bmin, const float* bmax, float trunc,
                                     void* stream) {
    return tsdf_run(T, Wt, D, H, W, z0, z1, depth, F, Hd, Wd, poses, Kf, bmin, bmax, trunc, stream, nullptr,
                    nullptr);
}

extern "C" int sfmhip_tsdf_integrate_tab(float* T, float* Wt, int D, int H, int W, int z0, int z1,
                                         const float* depth, int F, int Hd, int Wd, const float* poses,
                                         const float* Kf, const float* bmin, const float* bmax, float trunc,
                                         const float* table, void* stream) {
    SFMHIP_REQUIRE(table || F == 0, "sfmhip_tsdf_integrate_tab: null pointer");
    return tsdf_run(T, Wt, D, H, W, z0, z1, depth, F, Hd, Wd, poses, Kf, bmin, bmax, trunc, stream, nullptr,
                    reinterpret_cast<const float2*>(table));
}

extern "C" int sfmhip_tsdf_block_table(const float* depth, int F, int Hd, int Wd, int f0, int f1, float* table,
                                       void* stream) {
    SFMHIP_REQUIRE(F >= 0 && Hd > 0 && Wd > 0 && 0 <= f0 && f0 <= f1 && f1 <= F,
                   "sfmhip_tsdf_block_table: bad shape or frame range");
    if (f0 == f1) return SFMHIP_OK;
    SFMHIP_REQUIRE(depth && table, "sfmhip_tsdf_block_table: null pointer");
    SFMHIP_REQUIRE((int64_t)Hd * Wd * 4 < (int64_t)INT_MAX, "sfmhip_tsdf_block_table: depth map too large");
    const int nbu = ceil_div(Wd, kCullBlock), nbv = ceil_div(Hd, kCullBlock), nf = f1 - f0;
    hipStream_t st = as_stream(stream);
    int4* rg = nullptr;
    if (scratch_alloc((void**)&rg, (size_t)nf * sizeof(int4), st) != hipSuccess) {
        (void)hipGetLastError();
        set_error("sfmhip_tsdf_block_table: scratch allocation failed");
        return SFMHIP_E_HIP;
    }
    hipLaunchKernelGGL(full_range_kernel, dim3(ceil_div(nf, 64)), dim3(64), 0, st, nf, nbu, nbv, rg);
    const float* dp = depth + (size_t)f0 * Hd * Wd;
    float2* tp = reinterpret_cast<float2*>(table) + (size_t)f0 * nbv * nbu;
    if (Wd % 4 == 0)
        hipLaunchKernelGGL(depth_blockmax_kernel<true>, dim3(ceil_div(Wd, 1024), nbv, nf), dim3(256), 0, st, dp, nf,
                           Hd, Wd, nbu, nbv, rg, tp);
    else
        hipLaunchKernelGGL(depth_blockmax_kernel<false>, dim3(ceil_div(Wd, 256), nbv, nf), dim3(256), 0, st, dp, nf,
                           Hd, Wd, nbu, nbv, rg, tp);
    const int rc = check_launch("depth_blockmax_kernel");
    scratch_free(rg, st);
    return rc;
}

extern "C" int sfmhip_tsdf_cull_stats(int D, int H, int W, int z0, int z1, const float* depth, int F, int Hd,
                                      int Wd, const float* poses, const float* Kf, const float* bmin,
                                      const float* bmax, float trunc, int64_t* stats, void* stream) {
    SFMHIP_REQUIRE(stats, "sfmhip_tsdf_cull_stats: null pointer");
    stats[0] = stats[1] = stats[2] = 0;
    float dummy = 0.f;   // the grids are not touched
    return tsdf_run(&dummy, &dummy, D, H, W, z0, z1, depth, F, Hd, Wd, poses, Kf, bmin, bmax, trunc, stream, stats,
                    nullptr);
}

extern "C" int sfmhip_tsdf_layer_stats(int D, int H, int W, const float* depth, int F, int Hd, int Wd,
                                       const float* poses, const float* Kf, const float* bmin, const float* bmax,
                                       float trunc, int64_t* layer_stats, void* stream) {
    SFMHIP_REQUIRE(layer_stats, "sfmhip_tsdf_layer_stats: null pointer");
    const int nl = ceil_div(std::max(D, 0), kTsdfTZ);
    for (int i = 0; i < 3 * nl; ++i) layer_stats[i] = 0;
    int64_t tot[3] = {0, 0, 0};
    float dummy = 0.f;   // the grids are not touched
    return tsdf_run(&dummy, &dummy, D, H, W, 0, D, depth, F, Hd, Wd, poses, Kf, bmin, bmax, trunc, stream, tot,
                    nullptr, layer_stats);
}
