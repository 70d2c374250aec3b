// voxel.hip — voxel-grid kernels: V1 DDA traversal (voxel_travesal.py), V2
// trilinear grid sample (sdf.py get_sdf/get_sdf_sh, plenoxel NerfModel), V4
// fused sample + SH-2 colour + alpha composite (sdf.py forward, plenoxel
// render_rays) and the grid training step.  V5 TSDF integration: tsdf.hip.
// All fp32 with -ffp-contract=off so the op order matches oracle/voxel.py.
#include "common.h"
#include <mutex>
#include <climits>
#include <cstdlib>
#include <algorithm>
#include <vector>

namespace sfmhip {

// ---------------------------------------------------------------------------
// V1: torch.floor_divide on floats (c10::div_floor_floating): Python floor
// division via fmod, with the same fix-ups.
__device__ __forceinline__ float floor_div(float a, float b) {
    if (b == 0.f) return a / b;
    const float mod = fmodf(a, b);
    float div = (a - mod) / b;
    if (mod != 0.f && ((b < 0.f) != (mod < 0.f))) div -= 1.f;
    float fl;
    if (div != 0.f) {
        fl = floorf(div);
        if (div - fl > 0.5f) fl += 1.f;
    } else {
        fl = copysignf(0.f, a / b);
    }
    return fl;
}

struct Ray {
    float cur[3], last[3], step[3], tmax[3], tdelta[3];
};

__device__ __forceinline__ void ray_setup(const float* rr, float bin, Ray& R) {
    const float near = rr[6], far = rr[7];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const float o = rr[a], d = rr[3 + a];
        const float start = o + d * near;
        const float end = o + d * far;
        R.cur[a] = floor_div(start, bin);
        R.last[a] = floor_div(end, bin);
        R.step[a] = (d < 0.f) ? -1.f : 1.f;
        const float nvb = (R.cur[a] + R.step[a]) * bin;
        R.tmax[a] = (d == 0.f) ? __builtin_inff() : (nvb - start) / d;
        R.tdelta[a] = (d == 0.f) ? __builtin_inff() : (R.step[a] * bin) / d;
    }
}

// voxel_travesal.py:32-37 get_maskt: any axis with cur==cur and step*cur < step*last
// (bitwise, not short-circuit: no exec-mask branches on the walk's critical path)
__device__ __forceinline__ bool ray_active(const Ray& R) {
    bool m = false;
#pragma unroll
    for (int a = 0; a < 3; ++a)
        m = m | ((R.cur[a] == R.cur[a]) & (R.step[a] * R.cur[a] < R.step[a] * R.last[a]));
    return m;
}

// voxel_travesal.py:43-64: one step; axis masks are mutually exclusive.
__device__ __forceinline__ void ray_step(Ray& R) {
    const float tx = R.tmax[0], ty = R.tmax[1], tz = R.tmax[2];
    const bool mx = (tx < ty) && (tx < tz);
    const bool my = (ty <= tx) && (ty < tz);
    const bool mz = ((tx >= ty) && (ty >= tz)) || ((tx >= tz) && (ty > tx));
    // selects, not branches: the walk is one long dependent chain per ray
    R.cur[0] = mx ? R.cur[0] + R.step[0] : R.cur[0];
    R.tmax[0] = mx ? R.tmax[0] + R.tdelta[0] : R.tmax[0];
    R.cur[1] = my ? R.cur[1] + R.step[1] : R.cur[1];
    R.tmax[1] = my ? R.tmax[1] + R.tdelta[1] : R.tmax[1];
    R.cur[2] = mz ? R.cur[2] + R.step[2] : R.cur[2];
    R.tmax[2] = mz ? R.tmax[2] + R.tdelta[2] : R.tmax[2];
}

__global__ void dda_count_kernel(const float* __restrict__ rays, int64_t N, float bin, int max_steps,
                                 int32_t* __restrict__ n_steps) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    Ray R;
    ray_setup(rays + 8 * i, bin, R);
    int k = 0;
    bool act = ray_active(R);
    while (act && k < max_steps) {
        ray_step(R);
        ++k;
        act = ray_active(R);
    }
    n_steps[i] = act ? max_steps + 1 : k;   // max_steps + 1 = still active at the cap
}

// Pass 2: every lane walks its ray; rows are produced kDdaCh steps at a time
// into an LDS tile [64 rays][kDdaCh*3] and written back cooperatively by the
// wave (consecutive lanes -> consecutive floats of one ray's row), instead of
// 64 lanes each storing to its own far-apart row.
constexpr int kDdaCh = 16;

__global__ __launch_bounds__(256) void dda_fill_kernel(const float* __restrict__ rays, int64_t N, float bin, int S,
                                                       float* __restrict__ out) {
    __shared__ float tile[4][64 * kDdaCh * 3];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t ray0 = ((int64_t)blockIdx.x * 4 + w) * 64;   // first ray of this wave
    if (ray0 >= N) return;                                     // wave-uniform
    const int64_t i = ray0 + lane;
    const float nan = __builtin_nanf("");
    Ray R;
    bool act = false, dup = false;
    if (i < N) {
        ray_setup(rays + 8 * i, bin, R);
        act = ray_active(R);
        dup = !act;   // inactive from the start: the reference's first loop pass re-appends it
    }
    float* t = tile[w];
    const int nrows = (int)min((int64_t)64, N - ray0);
    for (int s0 = 0; s0 < S; s0 += kDdaCh) {
        if (s0 >= 2 && !__any(act)) {
            // Every ray of the wave has ended (S is the longest ray of the whole
            // batch): the rest of these rows is NaN padding, stored row by row in
            // 64-lane contiguous runs without walking the remaining steps.
            const int rest = (S - s0) * 3;
            for (int r = 0; r < nrows; ++r) {
                float* o = out + ((size_t)(ray0 + r) * S + s0) * 3;
                for (int f = lane; f < rest; f += 64) o[f] = nan;
            }
            return;
        }
        const int cnt = min(kDdaCh, S - s0);
        for (int q = 0; q < cnt; ++q) {
            const int s = s0 + q;
            float v0 = nan, v1 = nan, v2 = nan;
            if (i < N) {
                if (s == 0 || (s == 1 && dup)) {
                    v0 = R.cur[0]; v1 = R.cur[1]; v2 = R.cur[2];
                } else if (act) {
                    ray_step(R);
                    v0 = R.cur[0]; v1 = R.cur[1]; v2 = R.cur[2];
                    act = ray_active(R);
                }
            }
            t[(lane * kDdaCh + q) * 3 + 0] = v0;
            t[(lane * kDdaCh + q) * 3 + 1] = v1;
            t[(lane * kDdaCh + q) * 3 + 2] = v2;
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        if (cnt == kDdaCh) {   // full chunk: constant row length (division by a constant)
            constexpr int per_row = kDdaCh * 3;
            for (int f = lane; f < nrows * per_row; f += 64) {
                const int r = f / per_row, c = f - r * per_row;
                out[((size_t)(ray0 + r) * S + s0) * 3 + c] = t[r * kDdaCh * 3 + c];
            }
        } else {
            const int per_row = cnt * 3;
            for (int f = lane; f < nrows * per_row; f += 64) {
                const int r = f / per_row, c = f - r * per_row;
                out[((size_t)(ray0 + r) * S + s0) * 3 + c] = t[r * kDdaCh * 3 + c];
            }
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    }
}

// Pass 2, few rays (latency-bound: the launch lasts as long as its longest ray):
// each lane stores its own row directly, one 12-B store per step, no LDS
// staging; lanes whose rays have ended store NaN rows, and a wave whose rays
// have all ended stores the remaining padding in 64-lane runs and exits.
// n_steps (optional, the capped one-walk form): each lane's step count, S when its ray is
// still active after the row is full.
__global__ __launch_bounds__(64) void dda_fill_direct_kernel(const float* __restrict__ rays, int64_t N, float bin,
                                                             int S, float* __restrict__ out,
                                                             int32_t* __restrict__ n_steps) {
    const int lane = threadIdx.x;
    const int64_t ray0 = (int64_t)blockIdx.x * 64, i = ray0 + lane;
    const float nan = __builtin_nanf("");
    Ray R;
    bool act = false, dup = false;
    if (i < N) {
        ray_setup(rays + 8 * i, bin, R);
        act = ray_active(R);
        dup = !act;
    }
    const int nrows = (int)min((int64_t)64, N - ray0);
    float* row = out + (size_t)min(i, N - 1) * S * 3;
    int k = 0;   // steps walked
    for (int s = 0; s < S; ++s) {
        if (s >= 2 && !__any(act)) {
            if (n_steps && i < N) n_steps[i] = k;
            if (n_steps) return;   // capped form: dda_rows_kernel pads each row from its step count
            const int rest = (S - s) * 3;
            for (int r = 0; r < nrows; ++r) {
                float* o = out + ((size_t)(ray0 + r) * S + s) * 3;
                for (int f = lane; f < rest; f += 64) o[f] = nan;
            }
            return;
        }
        float v0 = nan, v1 = nan, v2 = nan;
        if (s == 0 || (s == 1 && dup)) {
            v0 = R.cur[0]; v1 = R.cur[1]; v2 = R.cur[2];
        } else if (act) {
            ray_step(R);
            ++k;
            v0 = R.cur[0]; v1 = R.cur[1]; v2 = R.cur[2];
            act = ray_active(R);
        }
        if (i < N) {
            row[3 * s] = v0;
            row[3 * s + 1] = v1;
            row[3 * s + 2] = v2;
        }
    }
    if (n_steps && i < N) n_steps[i] = act ? S : k;
}

// ---------------------------------------------------------------------------
// V2: sdf.py:287-291 / plenoxel.py:34-37 normalisation, then ATen
// grid_sampler_3d (bilinear, zeros, align_corners=True) weight formulas.
struct Bounds { float mn[3], mx[3]; };

__device__ __forceinline__ bool normalise(const float* p, const Bounds& B, int mode, float* g) {
    if (mode == 0) {
        const bool in = (p[0] >= B.mn[0]) && (p[1] >= B.mn[1]) && (p[2] >= B.mn[2]) &&
                        (p[0] <= B.mx[0]) && (p[1] <= B.mx[1]) && (p[2] <= B.mx[2]);
        if (!in) return false;
#pragma unroll
        for (int a = 0; a < 3; ++a) g[a] = ((p[a] - B.mn[a]) / (B.mx[a] - B.mn[a])) * 2.f - 1.f;
        return true;
    }
    const float s = B.mx[0];
    const bool in = (fabsf(p[0]) < s) && (fabsf(p[1]) < s) && (fabsf(p[2]) < s);
    if (!in) return false;
#pragma unroll
    for (int a = 0; a < 3; ++a) g[a] = fminf(fmaxf(p[a] / s, -1.f), 1.f);
    return true;
}

struct Corners {
    int ix, iy, iz;     // tnw corner
    float w[8];         // tnw tne tsw tse bnw bne bsw bse
};

__device__ __forceinline__ void corners(const float* g, int D, int H, int W, Corners& c) {
    const float ix = ((g[0] + 1.f) / 2.f) * (float)(W - 1);
    const float iy = ((g[1] + 1.f) / 2.f) * (float)(H - 1);
    const float iz = ((g[2] + 1.f) / 2.f) * (float)(D - 1);
    const float fx = floorf(ix), fy = floorf(iy), fz = floorf(iz);
    c.ix = (int)fx; c.iy = (int)fy; c.iz = (int)fz;
    const float x1 = fx + 1.f, y1 = fy + 1.f, z1 = fz + 1.f;
    c.w[0] = (x1 - ix) * (y1 - iy) * (z1 - iz);  // tnw
    c.w[1] = (ix - fx) * (y1 - iy) * (z1 - iz);  // tne
    c.w[2] = (x1 - ix) * (iy - fy) * (z1 - iz);  // tsw
    c.w[3] = (ix - fx) * (iy - fy) * (z1 - iz);  // tse
    c.w[4] = (x1 - ix) * (y1 - iy) * (iz - fz);  // bnw
    c.w[5] = (ix - fx) * (y1 - iy) * (iz - fz);  // bne
    c.w[6] = (x1 - ix) * (iy - fy) * (iz - fz);  // bsw
    c.w[7] = (ix - fx) * (iy - fy) * (iz - fz);  // bse
}

__device__ __forceinline__ bool corner_in(const Corners& c, int k, int D, int H, int W, int& x, int& y, int& z) {
    x = c.ix + (k & 1);
    y = c.iy + ((k >> 1) & 1);
    z = c.iz + ((k >> 2) & 1);
    return x >= 0 && x < W && y >= 0 && y < H && z >= 0 && z < D;
}

__global__ void grid_sample_kernel(const float* __restrict__ grid, int C, int D, int H, int W, Bounds B,
                                   int mode, const float* __restrict__ pts, int64_t P, float* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P) return;
    const float p[3] = {pts[3 * i], pts[3 * i + 1], pts[3 * i + 2]};
    float g[3];
    float* o = out + (size_t)i * C;
    if (!normalise(p, B, mode, g)) {
        for (int c = 0; c < C; ++c) o[c] = 0.f;
        return;
    }
    Corners cn;
    corners(g, D, H, W, cn);
    int64_t off[8];
    bool in[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        int x, y, z;
        in[k] = corner_in(cn, k, D, H, W, x, y, z);
        off[k] = ((int64_t)z * H + y) * W + x;
    }
    const int64_t plane = (int64_t)D * H * W;
    for (int c = 0; c < C; ++c) {
        const float* gc = grid + (size_t)c * plane;
        float acc = 0.f;
#pragma unroll
        for (int k = 0; k < 8; ++k)
            if (in[k]) acc = acc + gc[off[k]] * cn.w[k];
        o[c] = acc;
    }
}

// (C,D,H,W) -> (D,H,W,32), zero padded channels.
__global__ void to_vm_kernel(const float* __restrict__ grid, int C, int64_t nvox, float* __restrict__ vm) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= nvox * 32) return;
    const int64_t v = e >> 5;
    const int c = (int)(e & 31);
    vm[e] = (c < C) ? grid[(size_t)c * nvox + v] : 0.f;
}

// ---------------------------------------------------------------------------
// V4: one wave per ray, one lane per sample (chunks of 64 samples).
__device__ __forceinline__ void sh_colour(const float* k, float x, float y, float z, float* col) {
    // sdf.py:361-369 / plenoxel.py:9-16, Python operator order, fp32 constants.
    const float C0 = 0.282095f, C1 = 0.488603f, C2 = 1.092548f, C3 = 0.315392f, C4 = 0.546274f;
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) {
        const float* kk = k + 9 * ch;
        const float inner = ((((C2 * x) * y) * kk[4] - ((C2 * y) * z) * kk[5]) +
                             (C3 * (((2.0f * z) * z - x * x) - y * y)) * kk[6]) +
                            ((-C2) * x) * z * kk[7];
        const float inner2 = inner + (C4 * (x * x - y * y)) * kk[8];
        col[ch] = (((C0 * kk[0] + ((-C1) * y) * kk[1]) + (C1 * z) * kk[2]) - (C1 * x) * kk[3]) + inner2;
    }
}

// order (optional): wave w renders ray order[w] (rays sorted by where they cross the
// grid, render_order below); rgb stays indexed by the caller's ray, so the result
// is the same bits in any order.
// SIG (sdfp = the reference layout's channel-0 plane (D,H,W), the caller guarantees a finite
// grid): the sample's sdf is interpolated from that compact plane first (same corners, weights
// and order: the same value), and the 28-channel voxel lines are fetched only for samples whose
// alpha is non-zero.  Where alpha = 0, w = T alpha = 0 and the finite colour adds +-0 to sums that
// end in + 1: the same bits.  Rays with a non-finite direction take the full path.
template <bool SIG>
__device__ __forceinline__ void render_body(const float* __restrict__ gvm, int D, int H, int W,
                                                     Bounds B, int mode, const float* __restrict__ ro,
                                                     const float* __restrict__ rd, const float* __restrict__ zv,
                                                     int64_t nrays, int S, float* __restrict__ rgb,
                                                     const unsigned* __restrict__ order,
                                                     const float* __restrict__ sdfp) {
    const int lane = threadIdx.x & 63;
    const int64_t w = (int64_t)blockIdx.x * (blockDim.x >> 6) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (w >= nrays) return;  // wave-uniform
    const int64_t ray = order ? (int64_t)order[w] : w;
    const float o[3] = {ro[3 * ray], ro[3 * ray + 1], ro[3 * ray + 2]};
    const float d[3] = {rd[3 * ray], rd[3 * ray + 1], rd[3 * ray + 2]};
    const float* z = zv + (size_t)ray * S;
    const bool sig = SIG && isfinite(d[0]) && isfinite(d[1]) && isfinite(d[2]);
    float carry = 1.f;  // transmittance entering this chunk
    float cr = 0.f, cg = 0.f, cb = 0.f, ws = 0.f;
    for (int s0 = 0; s0 < S; s0 += 64) {
        const int s = s0 + lane;
        float alpha = 0.f, col[3] = {0.f, 0.f, 0.f};
        if (s < S) {
            const float zs = z[s];
            const float p[3] = {o[0] + d[0] * zs, o[1] + d[1] * zs, o[2] + d[2] * zs};
            float g[3];
            float sdf = 0.f;
            float k[27];
#pragma unroll
            for (int c = 0; c < 27; ++c) k[c] = 0.f;
            const float delta = (s + 1 < S) ? (z[s + 1] - zs) : 1e10f;
            if (normalise(p, B, mode, g)) {
                Corners cn;
                corners(g, D, H, W, cn);
                bool lines = true;
                if (sig) {   // sdf from the compact plane; the voxel lines only where alpha != 0
                    // the 8 plane gathers in flight together: an out-of-range corner reads its clamped
                    // neighbour with weight 0 (finite grid: v * 0 = +-0 leaves a sum that starts at +0
                    // unchanged, the same bits as skipping it)
                    float pv[8], wq[8];
#pragma unroll
                    for (int q = 0; q < 8; ++q) {
                        int x, y, zz;
                        const bool in = corner_in(cn, q, D, H, W, x, y, zz);
                        x = min(max(x, 0), W - 1);
                        y = min(max(y, 0), H - 1);
                        zz = min(max(zz, 0), D - 1);
                        wq[q] = in ? cn.w[q] : 0.f;
                        pv[q] = sdfp[((size_t)zz * H + y) * W + x];
                    }
#pragma unroll
                    for (int q = 0; q < 8; ++q) sdf = sdf + pv[q] * wq[q];
                    lines = 1.f - expf((-fmaxf(sdf, 0.f)) * delta) != 0.f;
                }
                if (lines) {
#pragma unroll
                    for (int q = 0; q < 8; ++q) {
                        int x, y, zz;
                        if (!corner_in(cn, q, D, H, W, x, y, zz)) continue;
                        const float w = cn.w[q];
                        const float4* v = reinterpret_cast<const float4*>(gvm + ((((size_t)zz * H + y) * W + x) << 5));
                        float vv[28];
#pragma unroll
                        for (int t = 0; t < 7; ++t) {
                            const float4 f = v[t];
                            vv[4 * t] = f.x; vv[4 * t + 1] = f.y; vv[4 * t + 2] = f.z; vv[4 * t + 3] = f.w;
                        }
                        if (!sig) sdf = sdf + vv[0] * w;
#pragma unroll
                        for (int c = 0; c < 27; ++c) k[c] = k[c] + vv[1 + c] * w;
                    }
                }
            }
            sh_colour(k, d[0], d[1], d[2], col);
            const float sigma = fmaxf(sdf, 0.f);
            alpha = 1.f - expf((-sigma) * delta);
        }
        // exclusive multiplicative scan of (1 - alpha) across the wave
        float incl = 1.f - alpha;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const float up = __shfl_up(incl, off, 64);
            if (lane >= off) incl = incl * up;
        }
        float excl = __shfl_up(incl, 1, 64);
        if (lane == 0) excl = 1.f;
        const float T = carry * excl;
        const float w = T * alpha;
        float pr = w * col[0], pg = w * col[1], pb = w * col[2], pw = w;
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            pr += __shfl_xor(pr, off, 64);
            pg += __shfl_xor(pg, off, 64);
            pb += __shfl_xor(pb, off, 64);
            pw += __shfl_xor(pw, off, 64);
        }
        cr += pr; cg += pg; cb += pb; ws += pw;
        carry = carry * __shfl(incl, 63, 64);
    }
    if (lane == 0) {
        rgb[3 * ray] = (cr + 1.f) - ws;
        rgb[3 * ray + 1] = (cg + 1.f) - ws;
        rgb[3 * ray + 2] = (cb + 1.f) - ws;
    }
}

// OCC: amdgpu_waves_per_eu floor (register budget); 0 = the compiler's choice (130 VGPRs: 3
// waves per SIMD).  The sdf-plane form runs at 4 waves per SIMD (128 VGPRs): 0.524 vs 0.538 ms
// on the bench workload; 5, 6 and 8 spill (0.69 / 0.84 / 3.8 ms,
// profiles/r4/ab_render_occ_heavy_trace_r4g.log).  A two-phase sdf-plane form (every chunk's
// plane gathers in flight at once, colour lines after) measured no faster (round 4) and left.
template <bool SIG, int OCC>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(OCC > 0 ? OCC : 1)))
void render_kernel(const float* __restrict__ gvm, int D, int H, int W, Bounds B, int mode,
                   const float* __restrict__ ro, const float* __restrict__ rd, const float* __restrict__ zv,
                   int64_t nrays, int S, float* __restrict__ rgb, const unsigned* __restrict__ order,
                   const float* __restrict__ sdfp) {
    render_body<SIG>(gvm, D, H, W, B, mode, ro, rd, zv, nrays, S, rgb, order, sdfp);
}

// NerfModel.forward (plenoxel.py:31-43): the 28 channels at each point
// (grid_sample arithmetic of grid_sample_kernel, reference layout), sigma =
// ReLU(channel 0), colour = eval_spherical_function(channels 1..27, d); both
// zero outside the mask.  One thread per point.
__global__ void nerf_forward_kernel(const float* __restrict__ grid, int D, int H, int W, Bounds B, int mode,
                                    const float* __restrict__ pts, const float* __restrict__ dirs, int64_t P,
                                    float* __restrict__ color, float* __restrict__ sigma) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P) return;
    const float p[3] = {pts[3 * i], pts[3 * i + 1], pts[3 * i + 2]};
    float g[3];
    if (!normalise(p, B, mode, g)) {
        color[3 * i] = color[3 * i + 1] = color[3 * i + 2] = 0.f;
        sigma[i] = 0.f;
        return;
    }
    Corners cn;
    corners(g, D, H, W, cn);
    int64_t off[8];
    bool in[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        int x, y, z;
        in[k] = corner_in(cn, k, D, H, W, x, y, z);
        off[k] = ((int64_t)z * H + y) * W + x;
    }
    const int64_t plane = (int64_t)D * H * W;
    float v[28];
#pragma unroll
    for (int c = 0; c < 28; ++c) {
        const float* gc = grid + (size_t)c * plane;
        float acc = 0.f;
#pragma unroll
        for (int k = 0; k < 8; ++k)
            if (in[k]) acc = acc + gc[off[k]] * cn.w[k];
        v[c] = acc;
    }
    float col[3];
    sh_colour(v + 1, dirs[3 * i], dirs[3 * i + 1], dirs[3 * i + 2], col);
    sigma[i] = fmaxf(v[0], 0.f);
    color[3 * i] = col[0];
    color[3 * i + 1] = col[1];
    color[3 * i + 2] = col[2];
}


// ---------------------------------------------------------------------------
// §8f row 4: one training step of the grid (plenoxel.py:100-111, sdf.py:427-438):
// fused render forward + mse gradient + analytic backward + trilinear scatter
// (ATen grid_sampler_3d backward) into a voxel-major gradient, then Adam.
// One wave per ray, one lane per sample, up to kTrainChunks x 64 samples kept
// in registers between the forward and the reverse (suffix) pass.
constexpr int kTrainChunks = 4;

// coefficient of k[ch*9 + m] in eval_spherical_function (oracle/train.py sh_basis)
__device__ __forceinline__ void sh_basis(float x, float y, float z, float* b) {
    const float C0 = 0.282095f, C1 = 0.488603f, C2 = 1.092548f, C3 = 0.315392f, C4 = 0.546274f;
    b[0] = C0;
    b[1] = (-C1) * y;
    b[2] = C1 * z;
    b[3] = -(C1 * x);
    b[4] = (C2 * x) * y;
    b[5] = -((C2 * y) * z);
    b[6] = C3 * (((2.0f * z) * z - x * x) - y * y);
    b[7] = ((-C2) * x) * z;
    b[8] = C4 * (x * x - y * y);
}

__global__ __launch_bounds__(256) void render_train_kernel(
    const float* __restrict__ gvm, int D, int H, int W, Bounds B, int mode, const float* __restrict__ ro,
    const float* __restrict__ rd, const float* __restrict__ zv, const float* __restrict__ gt, int64_t nrays, int S,
    float gscale, float* __restrict__ rgb, float* __restrict__ sqerr, float* __restrict__ grad,
    unsigned char* __restrict__ touched) {
    // per-wave LDS staging of the scatter: sample -> (28 channel grads, 8 corners)
    __shared__ float s_dt[4][64 * 29];
    __shared__ int s_cv[4][64 * 8];
    __shared__ float s_cw[4][64 * 8];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t ray = (int64_t)blockIdx.x * (blockDim.x >> 6) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (ray >= nrays) return;  // wave-uniform
    const float o[3] = {ro[3 * ray], ro[3 * ray + 1], ro[3 * ray + 2]};
    const float d[3] = {rd[3 * ray], rd[3 * ray + 1], rd[3 * ray + 2]};
    const float* z = zv + (size_t)ray * S;
    float* dt = s_dt[wv];
    int* cvx = s_cv[wv];
    float* cwt = s_cw[wv];
    float sA[kTrainChunks], sE[kTrainChunks], sDel[kTrainChunks], sT[kTrainChunks], sC[kTrainChunks][3];
    bool sRelu[kTrainChunks];
    float carry = 1.f;
    float cr = 0.f, cg = 0.f, cb = 0.f, ws = 0.f;
#pragma unroll
    for (int c = 0; c < kTrainChunks; ++c) {
        sA[c] = 0.f; sE[c] = 1.f; sDel[c] = 0.f; sT[c] = 0.f; sC[c][0] = sC[c][1] = sC[c][2] = 0.f; sRelu[c] = false;
        if (c * 64 >= S) continue;  // wave-uniform
        const int s = c * 64 + lane;
        float alpha = 0.f;
        if (s < S) {
            const float zs = z[s];
            const float p[3] = {o[0] + d[0] * zs, o[1] + d[1] * zs, o[2] + d[2] * zs};
            float g[3], sdf = 0.f, k[27];
#pragma unroll
            for (int q = 0; q < 27; ++q) k[q] = 0.f;
            if (normalise(p, B, mode, g)) {
                Corners cn;
                corners(g, D, H, W, cn);
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    int x, y, zz;
                    if (!corner_in(cn, q, D, H, W, x, y, zz)) continue;
                    const float w = cn.w[q];
                    const float4* v = reinterpret_cast<const float4*>(gvm + ((((size_t)zz * H + y) * W + x) << 5));
                    float vv[28];
#pragma unroll
                    for (int t = 0; t < 7; ++t) {
                        const float4 f = v[t];
                        vv[4 * t] = f.x; vv[4 * t + 1] = f.y; vv[4 * t + 2] = f.z; vv[4 * t + 3] = f.w;
                    }
                    sdf = sdf + vv[0] * w;
#pragma unroll
                    for (int q2 = 0; q2 < 27; ++q2) k[q2] = k[q2] + vv[1 + q2] * w;
                }
            }
            sh_colour(k, d[0], d[1], d[2], sC[c]);
            const float sigma = fmaxf(sdf, 0.f);
            sRelu[c] = sdf > 0.f;
            sDel[c] = (s + 1 < S) ? (z[s + 1] - zs) : 1e10f;
            sE[c] = expf((-sigma) * sDel[c]);
            alpha = 1.f - sE[c];
        }
        sA[c] = alpha;
        float incl = 1.f - alpha;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const float up = __shfl_up(incl, off, 64);
            if (lane >= off) incl = incl * up;
        }
        float excl = __shfl_up(incl, 1, 64);
        if (lane == 0) excl = 1.f;
        sT[c] = carry * excl;
        const float w = sT[c] * alpha;
        float pr = w * sC[c][0], pg = w * sC[c][1], pb = w * sC[c][2], pw = w;
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            pr += __shfl_xor(pr, off, 64);
            pg += __shfl_xor(pg, off, 64);
            pb += __shfl_xor(pb, off, 64);
            pw += __shfl_xor(pw, off, 64);
        }
        cr += pr; cg += pg; cb += pb; ws += pw;
        carry = carry * __shfl(incl, 63, 64);
    }
    const float out[3] = {(cr + 1.f) - ws, (cg + 1.f) - ws, (cb + 1.f) - ws};
    float gch[3], se = 0.f;
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) {
        const float df = out[ch] - gt[3 * ray + ch];
        se += df * df;
        gch[ch] = gscale * df;  // d mse / d rgb
    }
    if (lane == 0) {
        rgb[3 * ray] = out[0]; rgb[3 * ray + 1] = out[1]; rgb[3 * ray + 2] = out[2];
        sqerr[ray] = se;
    }
    float bas[9];
    sh_basis(d[0], d[1], d[2], bas);
    float vcarry = 0.f;  // V after the last sample
#pragma unroll
    for (int c = kTrainChunks - 1; c >= 0; --c) {
        if (c * 64 >= S) continue;  // wave-uniform
        const int s = c * 64 + lane;
        const bool live = s < S;
        const float e = live ? ((gch[0] * (sC[c][0] - 1.f) + gch[1] * (sC[c][1] - 1.f)) + gch[2] * (sC[c][2] - 1.f))
                             : 0.f;
        // f_k(V) = a_k e_k + (1 - a_k) V ; suffix composition F_k = f_k o ... o f_63
        float fa = live ? 1.f - sA[c] : 1.f, fb = live ? sA[c] * e : 0.f;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const float na = __shfl_down(fa, off, 64), nb = __shfl_down(fb, off, 64);
            if (lane + off < 64) { fb = fb + fa * nb; fa = fa * na; }
        }
        float nxa = __shfl_down(fa, 1, 64), nxb = __shfl_down(fb, 1, 64);
        if (lane == 63) { nxa = 1.f; nxb = 0.f; }
        const float V = nxb + nxa * vcarry;
        vcarry = __shfl(fb, 0, 64) + __shfl(fa, 0, 64) * vcarry;
        bool has = false;
        if (live) {
            const float zs = z[s];
            const float p[3] = {o[0] + d[0] * zs, o[1] + d[1] * zs, o[2] + d[2] * zs};
            float g[3];
            if (normalise(p, B, mode, g)) {
                has = true;
                const float dalpha = sT[c] * (e - V);
                const float dsig = (dalpha * sE[c]) * sDel[c];
                dt[lane * 29] = sRelu[c] ? dsig : 0.f;
                const float w = sT[c] * sA[c];
#pragma unroll
                for (int ch = 0; ch < 3; ++ch) {
                    const float dc = w * gch[ch];
#pragma unroll
                    for (int m = 0; m < 9; ++m) dt[lane * 29 + 1 + 9 * ch + m] = dc * bas[m];
                }
                Corners cn;
                corners(g, D, H, W, cn);
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    int x, y, zz;
                    cvx[lane * 8 + q] = corner_in(cn, q, D, H, W, x, y, zz) ? (zz * H + y) * W + x : -1;
                    cwt[lane * 8 + q] = cn.w[q];
                }
            }
        }
        if (!has)
#pragma unroll
            for (int q = 0; q < 8; ++q) cvx[lane * 8 + q] = -1;
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        // scatter: each wave-instruction adds the 28 channels of two (sample, corner)
        // pairs, lanes 0..27 and 32..59 -> two contiguous 112-B runs (full-rate
        // atomics; one voxel per lane would be ~17x slower, MI355X_MICROARCH.md)
        const unsigned long long any = __ballot(has);
        if (any) {
            const int ch = lane & 31, half = lane >> 5;
            const int first = __ffsll((long long)any) - 1, last = 63 - __clzll((long long)any);
            for (int pr = first * 4; pr < (last + 1) * 4; ++pr) {
                const int idx = 2 * pr + half, smp = idx >> 3;
                const int vox = cvx[idx];
                if (ch < 28 && vox >= 0)
                    unsafeAtomicAdd(grad + ((size_t)vox << 5) + ch, cwt[idx] * dt[smp * 29 + ch]);
                if (touched && ch == 0 && vox >= 0) touched[vox] = 1;   // every writer stores 1: no atomic
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    }
}

// torch.optim.Adam single-tensor step (torch/optim/adam.py, CPU kernels):
//   m = fma(1-b1, g - m, m)            (vectorised lerp_)
//   v = fma((1-b2) * g, g, v * b2)      (vectorised addcmul_)
//   p = p + (step * m) / (sqrt(v) / bc2s + eps)   (addcdiv_, step = -lr / (1 - b1^t))
// and zero_grad: g = 0.  float4 streams: 32 algorithmic bytes per parameter.
typedef float v4f __attribute__((ext_vector_type(4)));

__device__ __forceinline__ v4f adam4(v4f pp, v4f gg, v4f& mm, v4f& vv, float w1, float b2, float s2, float bc2s,
                                     float eps, float step) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        mm[j] = fmaf(w1, gg[j] - mm[j], mm[j]);
        vv[j] = fmaf(s2 * gg[j], gg[j], vv[j] * b2);
        const float den = sqrtf(vv[j]) / bc2s + eps;
        pp[j] = pp[j] + (step * mm[j]) / den;
    }
    return pp;
}

// Streams are touched once per step: non-temporal loads/stores.  Workgroup b owns the
// contiguous float4 range [b * chunk, (b + 1) * chunk) of every stream, two float4 per
// thread in flight (512 per round), so the resident workgroups sweep each buffer in a
// compact front; a grid-stride assignment (the resident workgroups spread over 8-16
// regions 134 MB apart in all four buffers) ran 4-8 % slower on the same box
// (tools/adam_layout_micro.hip, profiles/r3/ab/adam_access_micro_r3l.txt).
constexpr int64_t kAdamChunk4 = 16384;   // float4 per workgroup and stream (256 KB)

__global__ __launch_bounds__(256) void adam_kernel(v4f* __restrict__ p, v4f* __restrict__ g, v4f* __restrict__ m,
                                                   v4f* __restrict__ v, int64_t n4, float w1, float b2, float s2,
                                                   float bc2s, float eps, float step, int zero_grad) {
    const int64_t b0 = (int64_t)blockIdx.x * kAdamChunk4, b1 = min(n4, b0 + kAdamChunk4);
    const v4f z4 = {0.f, 0.f, 0.f, 0.f};
    int64_t i = b0 + threadIdx.x;
    for (; i + 256 < b1; i += 512) {
        const int64_t j = i + 256;
        const v4f g0 = __builtin_nontemporal_load(g + i), g1 = __builtin_nontemporal_load(g + j);
        v4f m0 = __builtin_nontemporal_load(m + i), m1 = __builtin_nontemporal_load(m + j);
        v4f v0 = __builtin_nontemporal_load(v + i), v1 = __builtin_nontemporal_load(v + j);
        const v4f p0 = __builtin_nontemporal_load(p + i), p1 = __builtin_nontemporal_load(p + j);
        const v4f q0 = adam4(p0, g0, m0, v0, w1, b2, s2, bc2s, eps, step);
        const v4f q1 = adam4(p1, g1, m1, v1, w1, b2, s2, bc2s, eps, step);
        __builtin_nontemporal_store(m0, m + i); __builtin_nontemporal_store(m1, m + j);
        __builtin_nontemporal_store(v0, v + i); __builtin_nontemporal_store(v1, v + j);
        __builtin_nontemporal_store(q0, p + i); __builtin_nontemporal_store(q1, p + j);
        if (zero_grad) { __builtin_nontemporal_store(z4, g + i); __builtin_nontemporal_store(z4, g + j); }
    }
    for (; i < b1; i += 256) {
        v4f m0 = m[i], v0 = v[i];
        p[i] = adam4(p[i], g[i], m0, v0, w1, b2, s2, bc2s, eps, step);
        m[i] = m0;
        v[i] = v0;
        if (zero_grad) g[i] = z4;
    }
}

// The same step where a flag byte per 2^fshift parameters marks the ones whose
// gradient can be non-zero (the trainer's scatter sets it per touched voxel):
// elsewhere the gradient is known to be 0 and is neither read nor re-zeroed, so a
// step touching ~1/12 of the voxel lines moves ~24.7 instead of 32 bytes per parameter.
// Results are those of adam_kernel (g = 0 exactly where the flag is 0).
__global__ __launch_bounds__(256) void adam_flagged_kernel(v4f* __restrict__ p, v4f* __restrict__ g,
                                                           v4f* __restrict__ m, v4f* __restrict__ v, int64_t n4,
                                                           float w1, float b2, float s2, float bc2s, float eps,
                                                           float step, int zero_grad,
                                                           const unsigned char* __restrict__ flags, int fshift4) {
    const int64_t b0 = (int64_t)blockIdx.x * kAdamChunk4, b1 = min(n4, b0 + kAdamChunk4);
    const v4f z4 = {0.f, 0.f, 0.f, 0.f};
    int64_t i = b0 + threadIdx.x;
    for (; i + 256 < b1; i += 512) {
        const int64_t j = i + 256;
        const bool t0 = flags[i >> fshift4] != 0, t1 = flags[j >> fshift4] != 0;
        v4f m0 = __builtin_nontemporal_load(m + i), m1 = __builtin_nontemporal_load(m + j);
        v4f v0 = __builtin_nontemporal_load(v + i), v1 = __builtin_nontemporal_load(v + j);
        const v4f p0 = __builtin_nontemporal_load(p + i), p1 = __builtin_nontemporal_load(p + j);
        v4f g0 = z4, g1 = z4;
        if (t0) g0 = __builtin_nontemporal_load(g + i);
        if (t1) g1 = __builtin_nontemporal_load(g + j);
        const v4f q0 = adam4(p0, g0, m0, v0, w1, b2, s2, bc2s, eps, step);
        const v4f q1 = adam4(p1, g1, m1, v1, w1, b2, s2, bc2s, eps, step);
        __builtin_nontemporal_store(m0, m + i); __builtin_nontemporal_store(m1, m + j);
        __builtin_nontemporal_store(v0, v + i); __builtin_nontemporal_store(v1, v + j);
        __builtin_nontemporal_store(q0, p + i); __builtin_nontemporal_store(q1, p + j);
        if (zero_grad && t0) __builtin_nontemporal_store(z4, g + i);
        if (zero_grad && t1) __builtin_nontemporal_store(z4, g + j);
    }
    for (; i < b1; i += 256) {
        const bool t0 = flags[i >> fshift4] != 0;
        v4f m0 = m[i], v0 = v[i];
        p[i] = adam4(p[i], t0 ? g[i] : z4, m0, v0, w1, b2, s2, bc2s, eps, step);
        m[i] = m0;
        v[i] = v0;
        if (zero_grad && t0) g[i] = z4;
    }
}

// (D,H,W,32) -> (C,D,H,W): the parameter export of the trainer.
__global__ void from_vm_kernel(const float* __restrict__ vm, int C, int64_t nvox, float* __restrict__ grid) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= nvox * C) return;
    const int c = (int)(e / nvox);
    const int64_t vx = e - (int64_t)c * nvox;
    grid[e] = vm[(vx << 5) + c];
}

// ---------------------------------------------------------------------------
// V3: GradientBasedSampler's effective output (sdf.py:154-180, 220-256): the
// slab ray/AABB test and the stratified uniform samples (its importance
// samples are computed and then discarded at sdf.py:251-252).  torch
// semantics: NaN from 0 * inf propagates through min/max and makes the ray
// invalid; linspace(0, 1, S) in f32 with torch's two-sided formula.
__global__ void ray_aabb_kernel(const float* __restrict__ ro, const float* __restrict__ rd, int64_t B, Bounds bb,
                                float* __restrict__ t_near, float* __restrict__ t_far, uint8_t* __restrict__ valid) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= B) return;
    float tn = 0.f, tf = 0.f;
    bool nan = false;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const float inv = 1.0f / rd[3 * i + a];
        const float t0 = (bb.mn[a] - ro[3 * i + a]) * inv;
        const float t1 = (bb.mx[a] - ro[3 * i + a]) * inv;
        nan = nan || (t0 != t0) || (t1 != t1);
        const float lo = fminf(t0, t1), hi = fmaxf(t0, t1);
        tn = (a == 0) ? lo : fmaxf(tn, lo);
        tf = (a == 0) ? hi : fminf(tf, hi);
    }
    if (nan) { tn = __int_as_float(0x7fc00000); tf = tn; }
    tn = (tn != tn) ? tn : fmaxf(tn, 0.f);
    t_near[i] = tn;
    t_far[i] = tf;
    valid[i] = (tf > tn) ? 1 : 0;
}

__device__ __forceinline__ float torch_linspace01(int k, int S) {
    // start + step*k / end - step*(S-k-1), each a fused multiply-add as in the
    // compiled torch kernel (bit-exact with torch.linspace(0, 1, S), f32)
    const float step = (1.0f - 0.0f) / (float)(S - 1);
    return (k < S / 2) ? fmaf(step, (float)k, 0.0f) : fmaf(-step, (float)(S - k - 1), 1.0f);
}

__global__ void stratified_kernel(const float* __restrict__ tn, const float* __restrict__ tf,
                                  const float* __restrict__ t_rand, int64_t B, int S, int perturb,
                                  float* __restrict__ z) {
    const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= B * S) return;
    const int64_t r = e / S;
    const int k = (int)(e - r * S);
    auto zk = [&](int j) {
        const float t = torch_linspace01(j, S);
        return tn[r] * (1.0f - t) + tf[r] * t;
    };
    const float zc = zk(k);
    if (!perturb) { z[e] = zc; return; }
    const float lower = (k == 0) ? zc : 0.5f * (zc + zk(k - 1));
    const float upper = (k == S - 1) ? zc : 0.5f * (zk(k + 1) + zc);
    z[e] = lower + (upper - lower) * t_rand[e];
}

}  // namespace sfmhip

using namespace sfmhip;

extern "C" int sfmhip_voxel_traversal_count(const float* rays, int64_t N, float bin, int32_t max_steps,
                                            int32_t* n_steps, void* stream) {
    SFMHIP_REQUIRE(N >= 0 && max_steps > 0 && max_steps < INT_MAX, "sfmhip_voxel_traversal_count: bad args");
    if (N == 0) return SFMHIP_OK;
    SFMHIP_REQUIRE(rays && n_steps, "sfmhip_voxel_traversal_count: null pointer");
    hipLaunchKernelGGL(dda_count_kernel, dim3(ceil_div(N, 64)), dim3(64), 0, as_stream(stream), rays, N, bin,
                       max_steps, n_steps);   // one wave per workgroup: the waves spread over the CUs
    return check_launch("dda_count_kernel");
}

extern "C" int sfmhip_voxel_traversal(const float* rays, int64_t N, float bin, int32_t S, float* out,
                                      void* stream) {
    SFMHIP_REQUIRE(N >= 0 && S >= 1, "sfmhip_voxel_traversal: bad args");
    if (N == 0) return SFMHIP_OK;
    SFMHIP_REQUIRE(rays && out, "sfmhip_voxel_traversal: null pointer");
    // SFMHIP_DDA_DIRECT (tests): 1 per-lane row stores, 0 LDS-staged coalesced
    // chunks; default: direct below 64k rays (latency-bound), staged above.
    const int dk = knobs().dda_direct;
    const bool direct = dk >= 0 ? dk != 0 : N < 65536;
    if (direct) {
        hipLaunchKernelGGL(dda_fill_direct_kernel, dim3(ceil_div(N, 64)), dim3(64), 0, as_stream(stream), rays, N,
                           bin, S, out, nullptr);
        return check_launch("dda_fill_direct_kernel");
    }
    hipLaunchKernelGGL(dda_fill_kernel, dim3(ceil_div(N, 256)), dim3(256), 0, as_stream(stream), rays, N, bin, S,
                       out);  // 4 waves x 64 rays per workgroup
    return check_launch("dda_fill_kernel");
}

// The capped form's rows -> out [N][S][3]: entries past a row's own length are NaN (length
// k + 1, or 2 for a ray inactive from the start — k == 0 — whose start voxel is emitted twice).
__global__ __launch_bounds__(256) void dda_rows_kernel(const float* __restrict__ buf, int cap,
                                                       const int32_t* __restrict__ n_steps, int64_t N, int S,
                                                       float* __restrict__ out) {
    const int64_t total = N * (int64_t)S * 3;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = e / (3 * (int64_t)S);
        const int rem = (int)(e - i * 3 * (int64_t)S), s = rem / 3, c = rem - 3 * s;
        const int k = n_steps[i], len = k == 0 ? 2 : k + 1;
        out[e] = s < len ? buf[(i * cap + s) * 3 + c] : __builtin_nanf("");
    }
}

extern "C" int sfmhip_voxel_traversal_rows(const float* buf, int32_t cap, const int32_t* n_steps, int64_t N,
                                           int32_t S, float* out, void* stream) {
    SFMHIP_REQUIRE(N >= 0 && S >= 1 && S <= cap, "sfmhip_voxel_traversal_rows: bad args (1 <= S <= cap)");
    if (N == 0) return SFMHIP_OK;
    SFMHIP_REQUIRE(buf && n_steps && out, "sfmhip_voxel_traversal_rows: null pointer");
    const int64_t total = N * (int64_t)S * 3;
    hipLaunchKernelGGL(dda_rows_kernel, dim3((unsigned)std::min<int64_t>(ceil_div(total, 256), 8192)), dim3(256), 0,
                       as_stream(stream), buf, cap, n_steps, N, S, out);
    return check_launch("dda_rows_kernel");
}

extern "C" int sfmhip_voxel_traversal_capped(const float* rays, int64_t N, float bin, int32_t cap, float* out,
                                             int32_t* n_steps, void* stream) {
    SFMHIP_REQUIRE(N >= 0 && cap >= 2, "sfmhip_voxel_traversal_capped: bad args (cap >= 2)");
    if (N == 0) return SFMHIP_OK;
    SFMHIP_REQUIRE(rays && out && n_steps, "sfmhip_voxel_traversal_capped: null pointer");
    hipLaunchKernelGGL(dda_fill_direct_kernel, dim3(ceil_div(N, 64)), dim3(64), 0, as_stream(stream), rays, N, bin,
                       cap, out, n_steps);
    return check_launch("dda_fill_direct_kernel");
}

static Bounds make_bounds(const float* bmin, const float* bmax) {
    Bounds B;
    for (int a = 0; a < 3; ++a) { B.mn[a] = bmin[a]; B.mx[a] = bmax[a]; }
    return B;
}

extern "C" int sfmhip_grid_sample(const float* grid, int C, int D, int H, int W, const float* bmin,
                                  const float* bmax, int mask_mode, const float* pts, int64_t P, float* out,
                                  void* stream) {
    SFMHIP_REQUIRE(C > 0 && D > 1 && H > 1 && W > 1 && P >= 0, "sfmhip_grid_sample: bad shape");
    SFMHIP_REQUIRE(mask_mode == 0 || mask_mode == 1, "sfmhip_grid_sample: mask_mode must be 0 or 1");
    if (P == 0) return SFMHIP_OK;
    SFMHIP_REQUIRE(grid && bmin && bmax && pts && out, "sfmhip_grid_sample: null pointer");
    hipLaunchKernelGGL(grid_sample_kernel, dim3(ceil_div(P, 256)), dim3(256), 0, as_stream(stream), grid, C, D,
                       H, W, make_bounds(bmin, bmax), mask_mode, pts, P, out);
    return check_launch("grid_sample_kernel");
}

extern "C" int sfmhip_nerf_forward(const float* grid, int D, int H, int W, const float* bmin, const float* bmax,
                                   int mask_mode, const float* pts, const float* dirs, int64_t P, float* color,
                                   float* sigma, void* stream) {
    SFMHIP_REQUIRE(D > 0 && H > 0 && W > 0 && P >= 0, "sfmhip_nerf_forward: bad shape");
    SFMHIP_REQUIRE(mask_mode == 0 || mask_mode == 1, "sfmhip_nerf_forward: mask_mode must be 0 or 1");
    if (P == 0) return SFMHIP_OK;
    SFMHIP_REQUIRE(grid && bmin && bmax && pts && dirs && color && sigma, "sfmhip_nerf_forward: null pointer");
    const Bounds bb = make_bounds(bmin, bmax);
    hipLaunchKernelGGL(nerf_forward_kernel, dim3(ceil_div(P, 256)), dim3(256), 0, as_stream(stream), grid, D, H, W, bb,
                       mask_mode, pts, dirs, P, color, sigma);
    return check_launch("nerf_forward_kernel");
}

extern "C" int sfmhip_grid_to_voxel_major(const float* grid, int C, int D, int H, int W, float* grid_vm,
                                          void* stream) {
    SFMHIP_REQUIRE(grid && grid_vm, "sfmhip_grid_to_voxel_major: null pointer");
    SFMHIP_REQUIRE(C > 0 && C <= 32 && D > 0 && H > 0 && W > 0, "sfmhip_grid_to_voxel_major: bad shape");
    const int64_t nvox = (int64_t)D * H * W;
    hipLaunchKernelGGL(to_vm_kernel, dim3(ceil_div(nvox * 32, 256)), dim3(256), 0, as_stream(stream), grid, C,
                       nvox, grid_vm);
    return check_launch("to_vm_kernel");
}

// ---------------------------------------------------------------------------
// Ray order for the renderer: rays whose samples touch the same voxel lines should
// run close together in time (and on one XCD), so a line fetched for one ray is
// still in L2 for the next.  Key = Morton code of the cell (2^bits per axis of
// the bounds) holding the ray's sample sidx; a counting sort over the 2^(3 bits)
// keys (histogram with ranks, then the scatter, which prefixes the bucket counts itself).
// Order inside a bucket follows the atomics (arbitrary), which cannot change any ray's
// colour.
__device__ __forceinline__ unsigned morton_spread(unsigned v) {   // 10 bits -> every third bit
    v &= 0x3FFu;
    v = (v | (v << 16)) & 0x30000FFu;
    v = (v | (v << 8)) & 0x300F00Fu;
    v = (v | (v << 4)) & 0x30C30C3u;
    v = (v | (v << 2)) & 0x9249249u;
    return v;
}

// Key of ray i: Morton code of the cell holding its sample sidx.  Ranks inside a bucket
// come from an LDS histogram per workgroup plus one global atomic per (workgroup,
// non-empty bucket) that reserves the workgroup's run: the hot buckets of a ray bundle
// see one global atomic per workgroup instead of one per ray.
constexpr int kRenderSortMaxBuckets = 4096;   // bits <= 4
__global__ __launch_bounds__(256) void render_key_kernel(const float* __restrict__ ro, const float* __restrict__ rd,
                                                         const float* __restrict__ zv, int64_t nrays, int S, int sidx,
                                                         Bounds B, int bits, unsigned* __restrict__ hist,
                                                         unsigned* __restrict__ key, unsigned* __restrict__ rank) {
    __shared__ unsigned cnt[kRenderSortMaxBuckets];
    const int nb = 1 << (3 * bits);
    for (int b = threadIdx.x; b < nb; b += 256) cnt[b] = 0u;
    __syncthreads();
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    unsigned k = 0u, r = 0u;
    if (i < nrays) {
        const float zs = zv[(size_t)i * S + sidx];
        const float n = (float)(1 << bits);
        unsigned q[3];
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            const float p = ro[3 * i + a] + rd[3 * i + a] * zs;
            const float c = (p - B.mn[a]) / (B.mx[a] - B.mn[a]) * n;   // NaN -> cell 0
            q[a] = c >= n ? (1u << bits) - 1u : (c > 0.f ? (unsigned)c : 0u);
        }
        k = morton_spread(q[0]) | (morton_spread(q[1]) << 1) | (morton_spread(q[2]) << 2);
        r = atomicAdd(&cnt[k], 1u);
    }
    __syncthreads();
    for (int b = threadIdx.x; b < nb; b += 256) {
        const unsigned c = cnt[b];
        cnt[b] = c ? atomicAdd(&hist[b], c) : 0u;   // this workgroup's run inside bucket b
    }
    __syncthreads();
    if (i < nrays) {
        key[i] = k;
        rank[i] = cnt[k] + r;
    }
}

// order[pos] = ray, pos = (exclusive prefix of the bucket counts, recomputed per
// workgroup from the L2-resident histogram) + rank
__global__ __launch_bounds__(256) void render_scatter_kernel(const unsigned* __restrict__ hist, int nb,
                                                             const unsigned* __restrict__ key,
                                                             const unsigned* __restrict__ rank, int64_t nrays,
                                                             unsigned* __restrict__ order) {
    __shared__ unsigned base[kRenderSortMaxBuckets];
    __shared__ unsigned part[256];
    const int t = threadIdx.x, per = (nb + 255) / 256, a = t * per, e = min(nb, a + per);
    unsigned sum = 0;
    for (int j = a; j < e; ++j) sum += hist[j];
    part[t] = sum;
    __syncthreads();
    for (int d = 1; d < 256; d <<= 1) {   // Hillis-Steele over the 256 partial sums
        const unsigned v = t >= d ? part[t - d] : 0u;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    unsigned run = part[t] - sum;
    for (int j = a; j < e; ++j) {
        base[j] = run;
        run += hist[j];
    }
    __syncthreads();
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nrays) return;
    order[(int64_t)base[key[i]] + rank[i]] = (unsigned)i;
}

static void launch_render(const float* sdfp, dim3 grid, hipStream_t st, const float* gvm, int D, int H, int W,
                          const Bounds& bb, int mode, const float* ro, const float* rd, const float* z, int64_t B, int S,
                          float* rgb, const unsigned* order) {
    if (sdfp)
        hipLaunchKernelGGL((render_kernel<true, 4>), grid, dim3(256), 0, st, gvm, D, H, W, bb, mode, ro, rd, z, B, S,
                           rgb, order, sdfp);
    else
        hipLaunchKernelGGL((render_kernel<false, 0>), grid, dim3(256), 0, st, gvm, D, H, W, bb, mode, ro, rd, z, B, S,
                           rgb, order, nullptr);
}

static int render_run(const float* grid_vm, const float* sdfp, int D, int H, int W, const float* bmin,
                      const float* bmax, int mask_mode, const float* rays_o, const float* rays_d, const float* z,
                      int64_t B, int S, float* rgb, void* stream) {
    SFMHIP_REQUIRE(D > 1 && H > 1 && W > 1 && B >= 0 && S >= 1, "sfmhip_render_rays: bad shape");
    SFMHIP_REQUIRE(mask_mode == 0 || mask_mode == 1, "sfmhip_render_rays: mask_mode must be 0 or 1");
    SFMHIP_REQUIRE(B < ((int64_t)1 << 32), "sfmhip_render_rays: more than 2^32 rays");
    if (B == 0) return SFMHIP_OK;
    SFMHIP_REQUIRE(grid_vm && bmin && bmax && rays_o && rays_d && z && rgb, "sfmhip_render_rays: null pointer");
    hipStream_t st = as_stream(stream);
    const Bounds bb = make_bounds(bmin, bmax);
    // ray ordering (SFMHIP_RENDER_SORT=0 off, tests): Morton cells of 2^3 per axis holding each
    // ray's last sample; batches below 8192 rays fill only a fraction of the chip's waves at
    // once and are rendered as given.  Bench workload (tools/bench_render_order.py,
    // profiles/r3/ab/render_order_r3j.txt): 0.627-0.648 ms as given, 0.598 ms with this
    // ordering (sort kernels included); keys and cell sizes from 2^2 to 2^8 per axis,
    // host-sorted, and XCD-run layouts all give the same ~0.58 ms kernel
    const int sort = knobs().render_sort;
    constexpr int bits = 3;
    const int sidx = S - 1;
    unsigned* scratch = nullptr;
    const int nb = 1 << (3 * bits);
    if (sort && B >= 8192) {
        if (scratch_alloc((void**)&scratch, (size_t)(nb + 3 * B) * sizeof(unsigned), st) != hipSuccess) {
            (void)hipGetLastError();
            scratch = nullptr;   // render in the given order
        }
    }
    if (scratch) {
        unsigned *hist = scratch, *key = hist + nb, *rank = key + B, *order = rank + B;
        int rc = hipMemsetAsync(hist, 0, (size_t)nb * sizeof(unsigned), st) == hipSuccess ? SFMHIP_OK : SFMHIP_E_HIP;
        if (rc == SFMHIP_OK) {
            hipLaunchKernelGGL(render_key_kernel, dim3(ceil_div(B, 256)), dim3(256), 0, st, rays_o, rays_d, z, B, S,
                               sidx, bb, bits, hist, key, rank);
            rc = check_launch("render_key_kernel");
        }
        if (rc == SFMHIP_OK) {
            hipLaunchKernelGGL(render_scatter_kernel, dim3(ceil_div(B, 256)), dim3(256), 0, st, hist, nb, key, rank, B,
                               order);
            rc = check_launch("render_scatter_kernel");
        }
        if (rc == SFMHIP_OK) {
            launch_render(sdfp, dim3(ceil_div(B, 4)), st, grid_vm, D, H, W, bb, mask_mode, rays_o, rays_d, z, B, S,
                          rgb, order);
            rc = check_launch("render_kernel");
        }
        scratch_free(scratch, st);
        return rc;
    }
    launch_render(sdfp, dim3(ceil_div(B, 4)), st, grid_vm, D, H, W, bb, mask_mode, rays_o, rays_d, z, B, S, rgb,
                  nullptr);
    return check_launch("render_kernel");
}

extern "C" int sfmhip_render_rays(const float* grid_vm, int D, int H, int W, const float* bmin,
                                  const float* bmax, int mask_mode, const float* rays_o, const float* rays_d,
                                  const float* z, int64_t B, int S, float* rgb, void* stream) {
    return render_run(grid_vm, nullptr, D, H, W, bmin, bmax, mask_mode, rays_o, rays_d, z, B, S, rgb, stream);
}

extern "C" int sfmhip_render_rays_sdf(const float* grid_vm, const float* sdf_plane, int D, int H, int W,
                                      const float* bmin, const float* bmax, int mask_mode, const float* rays_o,
                                      const float* rays_d, const float* z, int64_t B, int S, float* rgb,
                                      void* stream) {
    SFMHIP_REQUIRE(sdf_plane, "sfmhip_render_rays_sdf: null sdf plane");
    return render_run(grid_vm, sdf_plane, D, H, W, bmin, bmax, mask_mode, rays_o, rays_d, z, B, S, rgb, stream);
}

// stats != nullptr: run only the culling pre-passes (forced on) and count
// (wave sub-tile, frame) pairs: stats[0] tested, [1] culled, [2] free space.

extern "C" int sfmhip_grid_from_voxel_major(const float* grid_vm, int C, int D, int H, int W, float* grid,
                                            void* stream) {
    SFMHIP_REQUIRE(grid && grid_vm, "sfmhip_grid_from_voxel_major: null pointer");
    SFMHIP_REQUIRE(C > 0 && C <= 32 && D > 0 && H > 0 && W > 0, "sfmhip_grid_from_voxel_major: bad shape");
    const int64_t nvox = (int64_t)D * H * W;
    hipLaunchKernelGGL(from_vm_kernel, dim3(ceil_div(nvox * C, 256)), dim3(256), 0, as_stream(stream), grid_vm, C,
                       nvox, grid);
    return check_launch("from_vm_kernel");
}

extern "C" int sfmhip_render_train(const float* grid_vm, int D, int H, int W, const float* bmin, const float* bmax,
                                   int mask_mode, const float* rays_o, const float* rays_d, const float* z,
                                   const float* gt, int64_t B, int S, float* rgb, float* sqerr, float* grad_vm,
                                   uint8_t* touched, void* stream) {
    SFMHIP_REQUIRE(D > 1 && H > 1 && W > 1 && B >= 0 && S >= 1, "sfmhip_render_train: bad shape");
    SFMHIP_REQUIRE(S <= 64 * kTrainChunks, "sfmhip_render_train: S must be <= %d", 64 * kTrainChunks);
    SFMHIP_REQUIRE(mask_mode == 0 || mask_mode == 1, "sfmhip_render_train: mask_mode must be 0 or 1");
    if (B == 0) return SFMHIP_OK;
    SFMHIP_REQUIRE(grid_vm && bmin && bmax && rays_o && rays_d && z && gt && rgb && sqerr && grad_vm,
                   "sfmhip_render_train: null pointer");
    const float gscale = (float)(2.0 / (3.0 * (double)B));  // mse_loss mean over B x 3
    hipLaunchKernelGGL(render_train_kernel, dim3(ceil_div(B, 4)), dim3(256), 0, as_stream(stream), grid_vm, D, H,
                       W, make_bounds(bmin, bmax), mask_mode, rays_o, rays_d, z, gt, B, S, gscale, rgb, sqerr,
                       grad_vm, touched);
    return check_launch("render_train_kernel");
}

extern "C" int sfmhip_adam_step(float* param, float* grad, float* exp_avg, float* exp_avg_sq, int64_t n,
                                double lr, double beta1, double beta2, double eps, int64_t step, int zero_grad,
                                void* stream) {
    SFMHIP_REQUIRE(n >= 0 && n % 4 == 0, "sfmhip_adam_step: n must be a multiple of 4");
    SFMHIP_REQUIRE(step >= 1, "sfmhip_adam_step: step counts from 1");
    if (n == 0) return SFMHIP_OK;
    SFMHIP_REQUIRE(param && grad && exp_avg && exp_avg_sq, "sfmhip_adam_step: null pointer");
    // torch computes these in Python floats (double) and casts to the tensor dtype
    const float w1 = (float)(1.0 - beta1), b2 = (float)beta2, s2 = (float)(1.0 - beta2);
    const float bc2s = (float)std::sqrt(1.0 - std::pow(beta2, (double)step));
    const float stp = (float)(-lr / (1.0 - std::pow(beta1, (double)step)));
    const int64_t n4 = n / 4;
    const int blocks = ceil_div(n4, kAdamChunk4);
    hipLaunchKernelGGL(adam_kernel, dim3(blocks), dim3(256), 0, as_stream(stream), reinterpret_cast<v4f*>(param),
                       reinterpret_cast<v4f*>(grad), reinterpret_cast<v4f*>(exp_avg),
                       reinterpret_cast<v4f*>(exp_avg_sq), n4, w1, b2, s2, bc2s, (float)eps, stp, zero_grad);
    return check_launch("adam_kernel");
}

extern "C" int sfmhip_adam_step_flagged(float* param, float* grad, float* exp_avg, float* exp_avg_sq, int64_t n,
                                        double lr, double beta1, double beta2, double eps, int64_t step,
                                        int zero_grad, uint8_t* flags, int flag_shift, void* stream) {
    SFMHIP_REQUIRE(n >= 0 && n % 4 == 0, "sfmhip_adam_step_flagged: n must be a multiple of 4");
    SFMHIP_REQUIRE(flag_shift >= 2 && flag_shift <= 30, "sfmhip_adam_step_flagged: flag_shift must be in [2, 30]");
    SFMHIP_REQUIRE(step >= 1, "sfmhip_adam_step_flagged: step counts from 1");
    if (n == 0) return SFMHIP_OK;
    SFMHIP_REQUIRE(param && grad && exp_avg && exp_avg_sq && flags, "sfmhip_adam_step_flagged: null pointer");
    const float w1 = (float)(1.0 - beta1), b2 = (float)beta2, s2 = (float)(1.0 - beta2);
    const float bc2s = (float)std::sqrt(1.0 - std::pow(beta2, (double)step));
    const float stp = (float)(-lr / (1.0 - std::pow(beta1, (double)step)));
    const int64_t n4 = n / 4;
    const int blocks = ceil_div(n4, kAdamChunk4);
    hipStream_t st = as_stream(stream);
    hipLaunchKernelGGL(adam_flagged_kernel, dim3(blocks), dim3(256), 0, st, reinterpret_cast<v4f*>(param),
                       reinterpret_cast<v4f*>(grad), reinterpret_cast<v4f*>(exp_avg),
                       reinterpret_cast<v4f*>(exp_avg_sq), n4, w1, b2, s2, bc2s, (float)eps, stp, zero_grad, flags,
                       flag_shift - 2);
    int rc = check_launch("adam_flagged_kernel");
    if (rc == SFMHIP_OK && zero_grad) {   // every gradient is 0 again: so is every flag
        const hipError_t e = hipMemsetAsync(flags, 0, (size_t)((n - 1) >> flag_shift) + 1, st);
        if (e != hipSuccess) {
            set_error("sfmhip_adam_step_flagged: %s", hipGetErrorString(e));
            rc = SFMHIP_E_HIP;
        }
    }
    return rc;
}

extern "C" int sfmhip_ray_aabb(const float* rays_o, const float* rays_d, int64_t B, const float* bmin,
                               const float* bmax, float* t_near, float* t_far, uint8_t* valid, void* stream) {
    SFMHIP_REQUIRE(B >= 0, "sfmhip_ray_aabb: B < 0");
    if (B == 0) return SFMHIP_OK;
    SFMHIP_REQUIRE(rays_o && rays_d && bmin && bmax && t_near && t_far && valid, "sfmhip_ray_aabb: null pointer");
    hipLaunchKernelGGL(ray_aabb_kernel, dim3(ceil_div(B, 256)), dim3(256), 0, as_stream(stream), rays_o, rays_d, B,
                       make_bounds(bmin, bmax), t_near, t_far, valid);
    return check_launch("ray_aabb_kernel");
}

extern "C" int sfmhip_stratified_samples(const float* t_near, const float* t_far, const float* t_rand, int64_t B,
                                         int S, int perturb, float* z, void* stream) {
    SFMHIP_REQUIRE(B >= 0 && S >= 2, "sfmhip_stratified_samples: bad shape");
    if (B == 0) return SFMHIP_OK;
    SFMHIP_REQUIRE(t_near && t_far && z && (t_rand || !perturb), "sfmhip_stratified_samples: null pointer");
    hipLaunchKernelGGL(stratified_kernel, dim3(ceil_div(B * S, 256)), dim3(256), 0, as_stream(stream), t_near, t_far,
                       t_rand, B, S, perturb, z);
    return check_launch("stratified_kernel");
}
