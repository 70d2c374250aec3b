// voxel.hip — voxel-grid kernels: V1 DDA traversal (voxel_travesal.py), V2
// trilinear grid sample (sdf.py get_sdf/get_sdf_sh, plenoxel NerfModel), V4
// fused sample + SH-2 colour + alpha composite (sdf.py forward, plenoxel
// render_rays) and V5 TSDF integration (build-defined).
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

// Two-phase form of render_body<true> (SFMHIP_RENDER_2PH): per group of NCH chunks of 64 samples,
// phase 1 issues every chunk's depth and sdf-plane gathers together and composites the alphas
// (the transmittance scan in chunk order), phase 2 fetches the colour lines of the alpha != 0
// samples chunk by chunk.  Each chunk's scan, weights and sums are the same operations in the same
// order as render_body's, so the colours are the same bits; the plane gathers of all chunks are in
// flight at once instead of one chunk's per round trip.
template <int NCH>
__device__ __forceinline__ void render_body_2ph(const float* __restrict__ gvm, int D, int H, int W, Bounds B, int mode,
                                                const float* __restrict__ ro, const float* __restrict__ rd,
                                                const float* __restrict__ zv, int64_t nrays, int S,
                                                float* __restrict__ rgb, const unsigned* __restrict__ order,
                                                const float* __restrict__ sdfp) {
    const int lane = threadIdx.x & 63;
    const int64_t w = (int64_t)blockIdx.x * (blockDim.x >> 6) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (w >= nrays) return;  // wave-uniform
    const int64_t ray = order ? (int64_t)order[w] : w;
    const float o[3] = {ro[3 * ray], ro[3 * ray + 1], ro[3 * ray + 2]};
    const float d[3] = {rd[3 * ray], rd[3 * ray + 1], rd[3 * ray + 2]};
    if (!(isfinite(d[0]) && isfinite(d[1]) && isfinite(d[2]))) {   // the full path (wave-uniform)
        render_body<true>(gvm, D, H, W, B, mode, ro, rd, zv, nrays, S, rgb, order, sdfp);
        return;
    }
    const float* z = zv + (size_t)ray * S;
    float carry = 1.f;
    float cr = 0.f, cg = 0.f, cb = 0.f, ws = 0.f;
    for (int g0 = 0; g0 < S; g0 += 64 * NCH) {
        float alpha[NCH], wgt[NCH], zsv[NCH];
        bool lines[NCH];
#pragma unroll
        for (int c = 0; c < NCH; ++c) {   // phase 1: depths, plane sdf, alpha
            const int s = g0 + 64 * c + lane;
            alpha[c] = 0.f;
            lines[c] = false;
            zsv[c] = 0.f;
            if (s < S) {
                const float zs = z[s];
                zsv[c] = zs;
                const float p[3] = {o[0] + d[0] * zs, o[1] + d[1] * zs, o[2] + d[2] * zs};
                const float delta = (s + 1 < S) ? (z[s + 1] - zs) : 1e10f;
                float g[3], sdf = 0.f;
                if (normalise(p, B, mode, g)) {
                    Corners cn;
                    corners(g, D, H, W, cn);
#pragma unroll
                    for (int q = 0; q < 8; ++q) {
                        int x, y, zz;
                        if (!corner_in(cn, q, D, H, W, x, y, zz)) continue;
                        sdf = sdf + sdfp[((size_t)zz * H + y) * W + x] * cn.w[q];
                    }
                }
                alpha[c] = 1.f - expf((-fmaxf(sdf, 0.f)) * delta);
                lines[c] = alpha[c] != 0.f;
            }
        }
#pragma unroll
        for (int c = 0; c < NCH; ++c) {   // transmittance in chunk order (render_body's scan)
            wgt[c] = 0.f;
            if (g0 + 64 * c >= S) continue;   // wave-uniform
            float incl = 1.f - alpha[c];
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
                const float up = __shfl_up(incl, off, 64);
                if (lane >= off) incl = incl * up;
            }
            float excl = __shfl_up(incl, 1, 64);
            if (lane == 0) excl = 1.f;
            wgt[c] = (carry * excl) * alpha[c];
            carry = carry * __shfl(incl, 63, 64);
        }
#pragma unroll
        for (int c = 0; c < NCH; ++c) {   // phase 2: colour lines where alpha != 0, sums in chunk order
            if (g0 + 64 * c >= S) continue;   // wave-uniform
            float k[27];
#pragma unroll
            for (int q = 0; q < 27; ++q) k[q] = 0.f;
            if (lines[c]) {
                const float zs = zsv[c];
                const float p[3] = {o[0] + d[0] * zs, o[1] + d[1] * zs, o[2] + d[2] * zs};
                float g[3];
                normalise(p, B, mode, g);   // true: alpha != 0 needs a sample inside the mask
                Corners cn;
                corners(g, D, H, W, cn);
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    int x, y, zz;
                    if (!corner_in(cn, q, D, H, W, x, y, zz)) continue;
                    const float cw = cn.w[q];
                    const float4* v = reinterpret_cast<const float4*>(gvm + ((((size_t)zz * H + y) * W + x) << 5));
                    float vv[28];
#pragma unroll
                    for (int t = 0; t < 7; ++t) {
                        const float4 f = v[t];
                        vv[4 * t] = f.x; vv[4 * t + 1] = f.y; vv[4 * t + 2] = f.z; vv[4 * t + 3] = f.w;
                    }
#pragma unroll
                    for (int q2 = 0; q2 < 27; ++q2) k[q2] = k[q2] + vv[1 + q2] * cw;
                }
            }
            float col[3];
            sh_colour(k, d[0], d[1], d[2], col);
            const float wc = wgt[c];
            float pr = wc * col[0], pg = wc * col[1], pb = wc * col[2], pw = wc;
#pragma unroll
            for (int off = 32; off >= 1; off >>= 1) {
                pr += __shfl_xor(pr, off, 64);
                pg += __shfl_xor(pg, off, 64);
                pb += __shfl_xor(pb, off, 64);
                pw += __shfl_xor(pw, off, 64);
            }
            cr += pr; cg += pg; cb += pb; ws += pw;
        }
    }
    if (lane == 0) {
        rgb[3 * ray] = (cr + 1.f) - ws;
        rgb[3 * ray + 1] = (cg + 1.f) - ws;
        rgb[3 * ray + 2] = (cb + 1.f) - ws;
    }
}

// OCC: amdgpu_waves_per_eu floor (register budget) for the occupancy A/B (SFMHIP_RENDER_OCC);
// 0 = the compiler's choice (130 VGPRs: 3 waves per SIMD)
template <bool SIG, int OCC, int NCH = 0>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(OCC > 0 ? OCC : 1)))
void render_kernel(const float* __restrict__ gvm, int D, int H, int W, Bounds B, int mode,
                   const float* __restrict__ ro, const float* __restrict__ rd, const float* __restrict__ zv,
                   int64_t nrays, int S, float* __restrict__ rgb, const unsigned* __restrict__ order,
                   const float* __restrict__ sdfp) {
    if constexpr (SIG && NCH > 0)
        render_body_2ph<NCH>(gvm, D, H, W, B, mode, ro, rd, zv, nrays, S, rgb, order, sdfp);
    else
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
// V5: TSDF integration (arithmetic defined op for op in oracle/voxel.py
// tsdf_integrate).  Bound by the per-CU texture pipeline (TA/TD ~87 % busy,
// profiles/r1): every depth gather costs one L1 tag lookup per distinct
// cache line per 16-lane quarter-wave, and neighbouring voxels land ~5.6 px
// apart, so the lane->voxel layout decides the cost:
//   * each 16-lane quarter-wave covers a 4 x 4 (x, z) patch at one y (the
//     orbiting cameras map y to image rows, and a compact x-z patch has the
//     smallest depth spread, i.e. the fewest distinct rows); a wave covers
//     8 x 8 (x, z).  Simulated over the C5 orbit: 0.44 line lookups per
//     voxel-frame vs 0.60 for a 16 x 4 strip and 0.79 for x-pairs;
//   * each lane owns TWO voxels adjacent in y, run as one packed-f32 pair
//     (v_pk_mul/add/fma_f32: two results per instruction); their (T, W) stay
//     in registers across all frames of the launch (grid read and written
//     once per launch);
//   * the x/z part of each camera row, Q = (P0 vx + P2 vz) + P3, is per lane and
//     shared by the pair, so a voxel pays one multiply-add per camera row;
//   * 1/Zc and the running-average division use the IEEE f32 division
//     sequence without v_div_scale / v_div_fixup, which are identities on the
//     ranges the algorithm admits (2^-60 <= Zc < 2^60; weights 0..2^24, |T| <=
//     2^30, numerators |n| >= 2^-100); lanes outside those ranges take the
//     full IEEE division (rare, divergent), so every result is the oracle's;
//   * pixel = v_cvt_flr_i32_f32 of (f X) iz + (c + 0.5) and one unsigned
//     compare per axis; the depth gather is a bounds-checked buffer load, so
//     off-image lanes need no address select;
//   * poses/intrinsics are validated once per frame while being staged in LDS
//     (non-finite or >= 2^60 anywhere: Z row zeroed, so the frame is skipped).
// U frames' projections + gathers are issued before their (ordered) updates.
constexpr int kTsdfMaxFrames = 512;   // frames per launch (host splits longer runs)
constexpr double kTsdfLatencyRounds = 4.0;   // below: latency mode (tsdf_run)
constexpr int kTsdfTX = 8, kTsdfTY = 8, kTsdfTZ = 8;    // workgroup tile: 4 waves x (8 x, 2 y, 8 z)

// Spatially compact brick order: the 1-D grid is dealt round-robin over the 8
// XCDs, so xcd_remap gives each XCD a contiguous range of logical bricks, and
// logical bricks are ordered by "super-bricks" of SB_X x SB_Y x SB_Z bricks.
// Workgroups resident on one XCD at the same time then project onto one
// compact image region per frame, so the depth lines they gather stay in that
// XCD's L2 (speed only, never correctness).
struct SuperBrick { int x, y, z, il; };   // il: super-bricks dealt round-robin over the XCDs

typedef float f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2 f2s(float a) { return f2{a, a}; }
__device__ __forceinline__ f2 fma2(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ f2 rcp2(f2 a) { return f2{__builtin_amdgcn_rcpf(a.x), __builtin_amdgcn_rcpf(a.y)}; }

// RN(1/z) for z in [2^-60, 2^60): Fma0..Fma4 + div_fmas of the f32 IEEE
// division with numerator 1 (Mul = 1 * Fma1 = Fma1).
__device__ __forceinline__ f2 recip_rn(f2 z) {
    const f2 one = f2s(1.f), nz = -z;
    f2 r = rcp2(z);
    r = fma2(fma2(nz, r, one), r, r);
    const f2 q = fma2(fma2(nz, r, one), r, r);
    return fma2(fma2(nz, q, one), r, q);
}
// RN(n/d) for d in [1, 2^25] and |n| in [2^-100, 2^60] (or any d, n of those
// exponent ranges: no scaling, no fixup case).
__device__ __forceinline__ f2 div_rn(f2 n, f2 d) {
    const f2 one = f2s(1.f), nd = -d;
    f2 r = rcp2(d);
    r = fma2(fma2(nd, r, one), r, r);
    f2 q = n * r;
    q = fma2(fma2(nd, q, n), r, q);
    return fma2(fma2(nd, q, n), r, q);
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
__device__ __forceinline__ bool tame(float t, float w) {
    return fabsf(t) <= 0x1p30f && w >= 0.f && w <= 0x1p24f;
}

// ---------------------------------------------------------------------------
// TSDF culling (exact: it only drops (tile, frame) pairs in which provably no
// voxel of the 8x8x8 workgroup tile would update).  Two small pre-passes per
// launch chunk:
//   depth_blockmax_kernel: max depth of every 16x16 pixel block (NaN ignored:
//     a NaN depth never updates), one coalesced pass over the chunk's maps;
//   tsdf_cull_kernel: one lane per (tile, frame), 32 frames per ballot word.
//     The tile's 8 corner voxels are projected in f64; if any corner is not
//     comfortably in front of the camera the pair is kept.  Otherwise the
//     pixel bbox of the corners (the projection of a box in front of the
//     camera is the hull of its corner projections), widened by a margin far
//     above the kernel's f32 rounding, bounds every voxel's pixel, and the
//     tile's min corner depth (Zc is affine in the voxel position) bounds every
//     voxel's Zc from below.  Culled: bbox off-image, or every block under it
//     has max depth <= 0, or max depth + mu < min Zc (sdf < -mu everywhere).
constexpr int kCullBlock = 16;
constexpr int kCullMaxBlocks = 256;   // larger footprints are simply kept

// Conservative pixel footprint of the voxel box [xa,xb] x [ya,yb] x [za,zb] in
// frame (P, k): interval bounds on the affine camera coordinates (centre +-
// sum |P_rj| h_j) widened by a bound on the fusion kernel's f32 rounding, and
// the X/Z, Y/Z interval quotients.  Returns 0 (no bound: box not safely in
// front of the camera), 1 (every voxel's pixel is off-image) or 2 (pixel range
// [u0,u1] x [v0,v1], clipped to the image, and zlo <= every f32 Zc).
// The culling passes' f64 view of the grid (host-computed: the same IEEE divisions
// as before, once per call) and of a frame (CullCam, built once per frame by
// tsdf_setup_kernel and read with scalar loads where the frame is wave-uniform).
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
// [v0,v1], clipped to the image, and zlo <= every f32 Zc).
__device__ __forceinline__ int box_footprint(const CullCam& cc, const CullGeom& G, int xa, int xb, int ya, int yb,
                                             int za, int zb, int Hd, int Wd, int& u0, int& u1, int& v0, int& v1,
                                             double& zlo, double& zhi, bool& inside) {
    const double cxw = G.mn[0] + 0.5 * (xa + xb) * G.s[0], hx = 0.5 * (xb - xa) * G.as[0];
    const double cyw = G.mn[1] + 0.5 * (ya + yb) * G.s[1], hy = 0.5 * (yb - ya) * G.as[1];
    const double czw = G.mn[2] + 0.5 * (za + zb) * G.s[2], hz = 0.5 * (zb - za) * G.as[2];
    const double mxw = fabs(cxw) + hx, myw = fabs(cyw) + hy, mzw = fabs(czw) + hz;   // |coord| bounds
    double c[3], e[3], mag[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        const double* p = cc.P + 4 * r;
        const double* a = cc.aP + 4 * r;
        c[r] = p[0] * cxw + p[1] * cyw + p[2] * czw + p[3];
        e[r] = a[0] * hx + a[1] * hy + a[2] * hz;
        mag[r] = a[0] * mxw + a[1] * myw + a[2] * mzw + a[3];
    }
    // f32 error of the kernel's Zc / Xc / Yc (unit roundoff 2^-24, generous op counts)
    const double eps = 0x1p-24;
    const double dz = 8 * eps * mag[2];
    zlo = c[2] - e[2] - dz;
    zhi = c[2] + e[2] + dz;
    inside = false;
    if (!(zlo > 1e-3 && zhi < 1e30 && c[0] == c[0] && c[1] == c[1])) return 0;
    const double izl = cull_rcp(zlo), izh = cull_rcp(zhi);
    const double xl = c[0] - e[0] - 8 * eps * mag[0], xh = c[0] + e[0] + 8 * eps * mag[0];
    const double yl = c[1] - e[1] - 8 * eps * mag[1], yh = c[1] + e[1] + 8 * eps * mag[1];
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

// The depth blocks the slab [z0, z1) can touch in a frame (tsdf_setup_kernel,
// int4 {bu0, bu1, bv0, bv1}): an empty range when the whole slab is off-image,
// every block when the footprint cannot be bounded.  The block-max pass fills only
// these blocks and the tile test reads only inside them.

// VEC: Wd % 4 == 0, one float4 (4 pixels) per lane, 4 lanes per block column,
// all 16 rows' loads in flight.  Otherwise one pixel per lane, 16 lanes per block.
// Table entry {min, max} per 16x16 block: max ignores NaN (a NaN depth never
// updates), min is poisoned by NaN (-inf: such a block never proves free space).
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

constexpr int kCullSub = 4;   // waves per workgroup tile

// The (box, frame) test: skip = provably no voxel of the box updates; fre = every
// voxel of the box updates with tsdf = 1 (free space).
// BLK: pixel edge of the table's blocks; CAP: larger footprints are kept; range null:
// every entry of the table is valid.
template <int BLK = kCullBlock, int CAP = kCullMaxBlocks>
__device__ __forceinline__ void cull_test(const CullCam& cc, const CullGeom& G, int xa, int xb, int ya, int yb,
                                          int za, int zb, int Hd, int Wd, float trunc, int f,
                                          const float2* __restrict__ bmm, int use_free, int nbu, int nbv,
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
            // every depth <= m and every f32 Zc >= zlo: sdf < -trunc with room for the
            // rounding of (depth - Zc), so the kernel's !(sdf < -trunc) test fails everywhere
            skip = m <= 0.f || ((double)m + (double)trunc * (1 + 4 * 0x1p-24) + 1e-30 < zlo);
            // free space needs a frame record the fusion kernel fuses (every parameter < 2^60)
            if (!skip && use_free && inside && zlo >= 0x1p-59 && zhi <= 0x1p59 && cc.good != 0.0)
                fre = (double)mn - zhi >= (double)trunc * (1 + 0x1p-20);
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

// Brick pre-pass (SFMHIP_TSDF_BRICK=0 off).  The cull pass's workgroups are 4x4x4
// bricks of tiles (32^3 voxels); a brick-level test decides ~40 % of the (brick,
// frame) pairs of C5 outright (culled or free space; tools/sim_brick_cull.py), and
// the cull pass's wave for such a pair writes the decision without its 64 tile tests.
// The brick test reads a 4x coarser table (64x64-pixel blocks), so a brick footprint
// of up to 512 px square costs at most 64 loads.  Every decision is the same proof
// as the tile test's, on a box that contains the tile's voxels.
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
                                                         const float2* __restrict__ cmm, int use_free, int ncu,
                                                         int ncv, int per_tile, int nbricks,
                                                         unsigned char* __restrict__ bdec) {
    const int npad = (nbricks + 63) & ~63;
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int f = (int)(g / npad), brick = (int)(g % npad);
    if (f >= F) return;   // wave-uniform
    CullCam cc;
    load_cull_cam(cams, f, cc);
    if (brick >= nbricks) return;
    const int ntx = (W + kTsdfTX - 1) / kTsdfTX, nty = (H + kTsdfTY - 1) / kTsdfTY;
    const int ntz = (z1 - z0 + kTsdfTZ - 1) / kTsdfTZ;
    const int nsy = nty * per_tile;
    const int nqx = (ntx + 3) >> 2, nqy = (nsy + 3) >> 2;
    const int qx = brick % nqx, qy = (brick / nqx) % nqy, qz = brick / (nqx * nqy);
    const int sub = kTsdfTY / per_tile;   // voxel rows per sub-tile
    const int sy0 = qy * 4, sy1 = min(nsy, sy0 + 4) - 1;
    const int xa = qx * 4 * kTsdfTX, xb = min(W, (qx * 4 + 4) * kTsdfTX) - 1;
    const int ya = (sy0 / per_tile) * kTsdfTY + sub * (sy0 % per_tile);
    const int yb = min(H, (sy1 / per_tile) * kTsdfTY + sub * (sy1 % per_tile + 1)) - 1;
    const int za = z0 + qz * 4 * kTsdfTZ, zb = min(z1, z0 + min(ntz, qz * 4 + 4) * kTsdfTZ) - 1;
    bool skip, fre;
    cull_test<kCoarseBlock, kCoarseMaxBlocks>(cc, G, xa, xb, ya, yb, za, zb, Hd, Wd, trunc, f, cmm, use_free, ncu,
                                              ncv, nullptr, skip, fre);
    bdec[(size_t)f * nbricks + brick] = (unsigned char)(skip ? 1 : fre ? 2 : 0);
}

// One workgroup per (4x4x4 brick of tiles or sub-tiles, 16 frames): wave j tests
// frame 16 h + j for the brick's 64 boxes (one per lane), so the camera loads are
// scalar and the block-table reads of neighbouring footprints share cache lines;
// the 16 bits of each box are packed through LDS and stored as the low or high
// half of its mask word.  Masks are [wave slot][nw] words, bit j of word w =
// frame 32 w + j.  With `plist` (per_tile = 1), every (tile, frame) that is
// neither culled nor free space is appended to a list for tsdf_refine_kernel.
constexpr int kCullFrames = 16;
// waves_per_eu(8): two 16-wave workgroups per CU (the f64 frame record lives in SGPRs)
__global__ __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(8))) void tsdf_cull_kernel(int H, int W, int z0, int z1, int F, int Hd, int Wd,
                                                         const CullCam* __restrict__ cams, CullGeom G, float trunc,
                                                         const float2* __restrict__ bmm,
                                                         int use_free, int nbu, int nbv,
                                                         const int4* __restrict__ range, int per_tile, int nw,
                                                         const unsigned char* __restrict__ bdec,
                                                         unsigned short* __restrict__ cull,
                                                         unsigned short* __restrict__ freem,
                                                         unsigned* __restrict__ plist, unsigned* __restrict__ pcount,
                                                         unsigned* __restrict__ tcost, int h_off, int nhs) {
    __shared__ unsigned char bits[kCullFrames][64];
    const int ntx = (W + kTsdfTX - 1) / kTsdfTX, nty = (H + kTsdfTY - 1) / kTsdfTY;
    const int ntz = (z1 - z0 + kTsdfTZ - 1) / kTsdfTZ;
    const int nsy = nty * per_tile;                        // sub-tile rows in y
    const int nqx = (ntx + 3) >> 2, nqy = (nsy + 3) >> 2;  // 4x4x4 bricks of boxes
    // 16-frame halves [h_off, h_off + nhs) of the launch's 2 nw (the pre-pass pipeline runs the
    // pass per group of frames; mask halves are addressed by the absolute half index)
    const int hf = h_off + (int)(blockIdx.x % nhs), brick = (int)(blockIdx.x / nhs);
    const int nh = nhs;
    const int l = threadIdx.x & 63, j = threadIdx.x >> 6;
    const int f = hf * kCullFrames + j;
    const int tx = (brick % nqx) * 4 + (l & 3);
    const int sy = ((brick / nqx) % nqy) * 4 + ((l >> 2) & 3);
    const int tz = (brick / (nqx * nqy)) * 4 + (l >> 4);
    const bool tile_ok = tx < ntx && sy < nsy && tz < ntz;
    const int ty = sy / per_tile, w = sy % per_tile;
    const int64_t tile = ((int64_t)tz * nty + ty) * ntx + tx;
    bool skip = false, fre = false;
    // the brick pre-pass's decision for (brick, frame f): wave-uniform
    const int dec = bdec && f < F ? bdec[(size_t)__builtin_amdgcn_readfirstlane(f) * (gridDim.x / nh) + brick] : 0;
    if (tile_ok && f < F && dec) {
        skip = dec == 1;
        fre = dec == 2;
    } else if (tile_ok && f < F) {
        const int xa = tx * kTsdfTX, xb = min(W, xa + kTsdfTX) - 1;
        const int ya = ty * kTsdfTY + (kTsdfTY / per_tile) * w, yb = min(H, ya + kTsdfTY / per_tile) - 1;
        const int za = z0 + tz * kTsdfTZ, zb = min(z1, za + kTsdfTZ) - 1;
        CullCam cc;
        load_cull_cam(cams, f, cc);
        cull_test(cc, G, xa, xb, ya, yb, za, zb, Hd, Wd, trunc, f, bmm, use_free, nbu, nbv, range, skip, fre);
    }
    // compact list of the projected (tile, frame) pairs: one atomic per workgroup
    __shared__ unsigned wcnt[kCullFrames + 1];
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
            if (c) atomicAdd(tcost + tile, per_tile == kCullSub ? c : 4u * c);
        }
        const int q0 = per_tile == kCullSub ? w : 0, q1 = per_tile == kCullSub ? w + 1 : kCullSub;
        for (int q = q0; q < q1; ++q) {
            const int64_t h = ((tile * kCullSub + q) * nw) * 2 + hf;   // half hf of word hf / 2
            cull[h] = (unsigned short)cw;
            if (freem) freem[h] = (unsigned short)fw;
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
                                                          const float2* __restrict__ bmm, int use_free, int nbu,
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
        cull_test(cc, G, xa, xb, ya, yb, za, zb, Hd, Wd, trunc, f, bmm, use_free, nbu, nbv, range, skip, fre);
        const int64_t word = (tile * kCullSub + q) * nw + (f >> 5);
        if (skip) atomicOr(cull + word, 1u << (f & 31));
        else if (fre && freem) atomicOr(freem + word, 1u << (f & 31));
    }
}

// Timing probes only (SFMHIP_TSDF_FREE=3: free-space frames dropped instead of fused;
// =4: every frame dropped): results are wrong by design, never the default.
__global__ void tsdf_probe_mask_kernel(unsigned* __restrict__ cull, const unsigned* __restrict__ freem, int64_t n,
                                       int all) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) cull[i] = all ? ~0u : (cull[i] | freem[i]);
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

// Per-call setup in one launch: per frame the fusion's f32 record, the culling
// passes' CullCam (ccam non-null) and the slab's block range (range_mode 1: every
// block, an external table; 2: the slab's footprint); the workgroups past the
// frames zero the per-tile cost counters (nzero words) and the refinement list count.
__global__ __launch_bounds__(64) void tsdf_setup_kernel(const float* __restrict__ poses, const float* __restrict__ Kf,
                                                        int F, float* __restrict__ rec, CullCam* __restrict__ ccam,
                                                        int range_mode, int H, int W, int z0, int z1, int Hd, int Wd,
                                                        CullGeom G, int nbu, int nbv, int4* __restrict__ range,
                                                        unsigned* __restrict__ zero, int nzero,
                                                        unsigned* __restrict__ pcount) {
    const int fb = (F + 63) / 64;
    if ((int)blockIdx.x >= fb) {
        const int nb = gridDim.x - fb, b = blockIdx.x - fb;
        if (b == 0 && threadIdx.x == 0 && pcount) *pcount = 0u;
        for (int i = b * 64 + threadIdx.x; i < nzero; i += nb * 64) zero[i] = 0u;
        return;
    }
    const int f = blockIdx.x * 64 + threadIdx.x;
    if (f >= F) return;
    tsdf_cam_record(poses, Kf, f, rec);
    if (!ccam) return;
    CullCam c;
    cull_cam(poses, Kf, f, c);
    c.pad[0] = c.pad[1] = c.pad[2] = 0.0;
    ccam[f] = c;
    if (range_mode == 1) {
        range[f] = make_int4(0, nbu - 1, 0, nbv - 1);
    } else if (range_mode == 2) {
        int u0, u1, v0, v1;
        double zlo, zhi;
        bool inside;
        const int st = box_footprint(c, G, 0, W - 1, 0, H - 1, z0, z1 - 1, Hd, Wd, u0, u1, v0, v1, zlo, zhi, inside);
        range[f] = st == 2   ? make_int4(u0 / kCullBlock, u1 / kCullBlock, v0 / kCullBlock, v1 / kCullBlock)
                   : st == 1 ? make_int4(1, 0, 1, 0)
                             : make_int4(0, nbu - 1, 0, nbv - 1);
    }
}

// Workgroup slot -> tile of the super-brick order: the 1-D grid is dealt
// round-robin over the 8 XCDs (slot % 8), so XCD x fuses super-bricks x, x+8,
// ... (il; spreads uneven culled work) or one contiguous range of them.
__device__ __forceinline__ void tsdf_slot_tile(int slot, int nslots, int W, int H, const SuperBrick& SB, int& bx,
                                               int& by, int& bz) {
    const int nbx = (W + kTsdfTX - 1) / kTsdfTX, nby = (H + kTsdfTY - 1) / kTsdfTY;
    const int nsx = (nbx + SB.x - 1) / SB.x, nsy = (nby + SB.y - 1) / SB.y;
    const int sbn = SB.x * SB.y * SB.z;
    int sb, in;
    if (SB.il) {
        const int j = slot / kNumXcd;
        sb = (j / sbn) * kNumXcd + slot % kNumXcd;
        in = j % sbn;
    } else {
        const int L = xcd_remap(slot, nslots);
        sb = L / sbn;
        in = L % sbn;
    }
    const int sx = sb % nsx, sy = (sb / nsx) % nsy, sz = sb / (nsx * nsy);
    bx = sx * SB.x + in % SB.x;
    by = sy * SB.y + (in / SB.x) % SB.y;
    bz = sz * SB.z + in / (SB.x * SB.y);
}

// Longest-first order of the fusion's workgroups (per XCD class, so each slot
// stays on the XCD its super-brick was dealt to): with few workgroups per CU
// (a z-slab of an N-way split: ~2 rounds) the surface tiles, up to ~10x the
// work of a free-space tile, otherwise land in the last round.
//   tsdf_cull_kernel adds each tile's cost (4 x projected frames + free-space
//     frames, over the 4 wave sub-tiles, before refinement) into a counter;
//   tsdf_order_kernel: one workgroup per XCD class, stable counting sort of the
//     class's slots by cost bucket 0..63, heaviest first: order[x + 8 k] = k-th slot.
constexpr int kOrderBuckets = 64;
__device__ __forceinline__ unsigned slot_bucket(int s, int nslots, int W, int H, int z0, int z1,
                                                const SuperBrick& SB, int F, const unsigned* __restrict__ tcost) {
    const int ntx = (W + kTsdfTX - 1) / kTsdfTX, nty = (H + kTsdfTY - 1) / kTsdfTY;
    const int ntz = (z1 - z0 + kTsdfTZ - 1) / kTsdfTZ;
    int bx, by, bz;
    tsdf_slot_tile(s, nslots, W, H, SB, bx, by, bz);
    const unsigned cost = bx < ntx && by < nty && bz < ntz ? tcost[((size_t)bz * nty + by) * ntx + bx] : 0u;
    return min((unsigned)(kOrderBuckets - 1), cost * kOrderBuckets / (16u * F + 1u));
}

// Dynamic LDS: one bucket byte per slot of the class (m <= 65535, host-checked).
__global__ __launch_bounds__(256) void tsdf_order_kernel(int nslots, int W, int H, int z0, int z1, SuperBrick SB,
                                                         int F, const unsigned* __restrict__ tcost,
                                                         unsigned* __restrict__ order) {
    __shared__ unsigned short hist[kOrderBuckets][256];
    __shared__ unsigned wsum[4];
    extern __shared__ unsigned char bk[];
    const int x = blockIdx.x, t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const int m = nslots > x ? (nslots - x + kNumXcd - 1) / kNumXcd : 0;   // slots x, x+8, ... of this class
    const int per = (m + 255) / 256, j0 = min(m, t * per), j1 = min(m, j0 + per);
    for (int b = 0; b < kOrderBuckets; ++b) hist[b][t] = 0;
    for (int j = t; j < m; j += 256)   // coalesced over the class: every cost load in flight
        bk[j] = (unsigned char)slot_bucket(x + kNumXcd * j, nslots, W, H, z0, z1, SB, F, tcost);
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

#ifdef SFMHIP_TSDF_PROF
// tool-only build (tools/tsdf_wave_prof.py): per fusion wave {start, end} wall clock (100 MHz)
// and its projected-frame count; never in the product library
constexpr int kTsdfProfWaves = 1 << 18;
__device__ unsigned long long g_tsdf_prof[kTsdfProfWaves * 3];
#endif

// One projected frame of one lane's voxel pair (tsdf_kernel's non-PIPE loop and the heavy-tile
// producers): projection, the per-voxel block test against the pixel's 16x16 {min, max} (exact, with
// this kernel's own f32 Zc: every depth d of the block has fl(d - Zc) between fl(min - Zc) and
// fl(max - Zc)) when bmm is given, the bounds-checked depth gather where the test did not decide,
// and the update inputs: ts and whether each voxel updates (g0, g1).
__device__ __forceinline__ void tsdf_frame_eval(const float* __restrict__ rec, int f, float vx, f2 vy, float vz,
                                                bool two, const float* __restrict__ depth, size_t frame, int nbytes,
                                                int Wd4, int Hd, int Wd, float trunc, float inv_trunc, float free_ts,
                                                const float2* __restrict__ bmm, int nbu, int nbv, f2& ts, bool& g0,
                                                bool& g1) {
    const float* r = rec + f * 16;   // uniform: scalar loads
    const f2 Q = (f2{r[0], r[1]} * f2s(vx) + f2{r[2], r[3]} * f2s(vz)) + f2{r[4], r[5]};
    const float Qz = (r[6] * vx + r[7] * vz) + r[8];
    const f2 Xc = f2s(r[9]) * vy + f2s(Q.x);
    const f2 Yc = f2s(r[10]) * vy + f2s(Q.y);
    const f2 Zc = f2s(r[11]) * vy + f2s(Qz);
    const f2 iz = recip_rn(Zc);
    const f2 uu = (f2s(r[12]) * Xc) * iz + f2s(r[14]);
    const f2 vv = (f2s(r[13]) * Yc) * iz + f2s(r[15]);
    const int iu0 = cvt_flr(uu.x), iv0 = cvt_flr(vv.x);
    const int iu1 = cvt_flr(uu.y), iv1 = cvt_flr(vv.y);
    const bool ok0 = z_ok(Zc.x) && (unsigned)iu0 < (unsigned)Wd && (unsigned)iv0 < (unsigned)Hd;
    const bool ok1 = two && z_ok(Zc.y) && (unsigned)iu1 < (unsigned)Wd && (unsigned)iv1 < (unsigned)Hd;
    // Per-voxel test against the pixel's 16x16 block {min, max} (exact, with this
    // kernel's own f32 Zc: every depth d of the block has fl(d - Zc) between
    // fl(min - Zc) and fl(max - Zc)): free (tsdf = 1) or no update without the depth.
    bool fr0 = false, fr1 = false, need0 = ok0, need1 = ok1;
    if (bmm) {
        const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(bmm + (size_t)f * nbv * nbu), (short)0, nbv * nbu * 8, 0x00020000);
        // 24-bit multiplies (v_mad_u32_u24, full rate; v_mul_lo_u32 is quarter rate): the
        // block indices are < 2^20 when the pixel is in range, and out-of-range lanes'
        // offsets only have to stay bounds-checked
        const auto e0 = __builtin_amdgcn_raw_buffer_load_b64(
            rb, (int)((__umul24((unsigned)(iv0 >> 4) & 0xFFFFFFu, (unsigned)nbu) + ((unsigned)iu0 >> 4)) << 3), 0, 0);
        const auto e1 = __builtin_amdgcn_raw_buffer_load_b64(
            rb, (int)((__umul24((unsigned)(iv1 >> 4) & 0xFFFFFFu, (unsigned)nbu) + ((unsigned)iu1 >> 4)) << 3), 0, 0);
        const f2 bmn = {__builtin_bit_cast(float, (unsigned)e0[0]), __builtin_bit_cast(float, (unsigned)e1[0])};
        const f2 bmx = {__builtin_bit_cast(float, (unsigned)e0[1]), __builtin_bit_cast(float, (unsigned)e1[1])};
        const f2 scm = (bmn - Zc) * f2s(inv_trunc);
        const f2 smx = bmx - Zc;
        fr0 = ok0 && bmn.x > 0.f && scm.x >= 1.f;
        fr1 = ok1 && bmn.y > 0.f && scm.y >= 1.f;
        need0 = ok0 && !fr0 && bmx.x > 0.f && !(smx.x < -trunc);
        need1 = ok1 && !fr1 && bmx.y > 0.f && !(smx.y < -trunc);
    }
    // bounds-checked gather, only where the block test did not decide
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void*)(depth + (size_t)f * frame), (short)0, nbytes, 0x00020000);
    f2 dep = {0.f, 0.f};
    if (need0)
        dep.x = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                             rs, (int)(__umul24(iv0, Wd4) + ((unsigned)iu0 << 2)), 0, 0));
    if (need1)
        dep.y = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                             rs, (int)(__umul24(iv1, Wd4) + ((unsigned)iu1 << 2)), 0, 0));
    const f2 sdf = dep - Zc;
    g0 = fr0 || (need0 && dep.x > 0.f && !(sdf.x < -trunc));
    g1 = fr1 || (need1 && dep.y > 0.f && !(sdf.y < -trunc));
    const f2 sc = sdf * f2s(inv_trunc);
    ts = f2{fr0 ? free_ts : fminf(1.0f, sc.x), fr1 ? free_ts : fminf(1.0f, sc.y)};
}

// W may take k more exact +1 steps with T = 1 fixed when it is an integer in [0, 2^24 - 512].
// Updates only add 1 to W (general or division-free; W + 1 is exact below 2^24), at most
// kTsdfMaxFrames = 512 per launch, so a W that starts the launch an integer in
// [0, 2^24 - 1024] stays in that range for every frame: tested once per voxel instead of
// per projected frame.  (A lane outside the range takes the general update, which gives
// the same bits.)
static_assert(kTsdfMaxFrames <= 512, "w_runs_launch assumes at most 512 updates per launch");
__device__ __forceinline__ bool w_runs_launch(float w) { return w >= 0.f && w <= 0x1p24f - 1024.f && w == truncf(w); }

// One workgroup = one 8x8x8 tile; every frame of the launch is fused with the
// tile's (T, W) in registers.  The (tile, frame) masks of the cull pass drive a
// scalar walk over the frames: culled frames are skipped, a run of k free-space
// frames is applied as k updates with tsdf = 1 — or, when every voxel of the
// wave holds T = 1 and an integer weight, as W += k (each of the k updates would
// compute (1 W + 1)/(W + 1) = 1 exactly and W + 1 exactly) — and every other
// frame is projected and gathered.
// PIPE (latency mode only, no block table): the gather of the next projected frame
// is issued before the current one's update and the free-space run between them,
// so a thin slab's longest waves overlap one depth load with the previous frame's
// arithmetic instead of waiting out each load in turn.  The order of the updates
// per voxel is unchanged.
template <bool SWZ, bool PIPE = false>
__global__ __launch_bounds__(256) void tsdf_kernel(float* __restrict__ T, float* __restrict__ Wt, int D, int H,
                                                   int W, int z0, int z1, const float* __restrict__ depth, int F,
                                                   int Hd, int Wd, const float* __restrict__ rec, Bounds B,
                                                   float trunc, SuperBrick SB, const unsigned* __restrict__ cull,
                                                   const unsigned* __restrict__ freem, int nw, float free_ts,
                                                   const float2* __restrict__ bmm, int nbu, int nbv,
                                                   const unsigned* __restrict__ order, int easy,
                                                   const unsigned char* __restrict__ skip) {
#ifdef SFMHIP_TSDF_PROF
    const unsigned long long prof_t0 = wall_clock64();
    int prof_nproj = 0;
    const int prof_w = (int)(((size_t)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x) * 4 +
                       (int)(threadIdx.x >> 6);
#endif
    int bx = blockIdx.x, by = blockIdx.y, bz = blockIdx.z;
    if (SWZ) tsdf_slot_tile(order ? (int)order[blockIdx.x] : (int)blockIdx.x, gridDim.x, W, H, SB, bx, by, bz);
    const int l = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int x = bx * kTsdfTX + (l & 3) + 4 * ((l >> 4) & 1);
    const int z = z0 + bz * kTsdfTZ + ((l >> 2) & 3) + 4 * (l >> 5);
    const int y = by * kTsdfTY + 2 * wave;
    if (x >= W || y >= H || z >= z1) return;  // no barrier in this kernel
    const bool two = y + 1 < H;
    const float sx = (B.mx[0] - B.mn[0]) / (float)(W - 1);
    const float sy = (B.mx[1] - B.mn[1]) / (float)(H - 1);
    const float sz = (B.mx[2] - B.mn[2]) / (float)(D - 1);
    const float vx = B.mn[0] + (float)x * sx;
    const f2 vy = {B.mn[1] + (float)y * sy, B.mn[1] + (float)(y + 1) * sy};
    const float vz = B.mn[2] + (float)z * sz;
    const float inv_trunc = 1.0f / trunc;
    const int ntx = (W + kTsdfTX - 1) / kTsdfTX, nty = (H + kTsdfTY - 1) / kTsdfTY;
    const size_t sub = (((size_t)bz * nty + by) * ntx + bx) * kCullSub + wave;
    const size_t slot = sub * (size_t)nw;
    if (skip && skip[sub]) return;   // a heavy sub-tile: tsdf_heavy_kernel fuses it
    if (cull) {   // every frame of the launch culled for this wave: the grid is not even read
        unsigned any = 0u;
        for (int w0 = 0; w0 < F; w0 += 32)
            any |= ~cull[slot + (w0 >> 5)] & (F - w0 >= 32 ? ~0u : ((1u << (F - w0)) - 1u));
        if (__builtin_amdgcn_readfirstlane((int)any) == 0) return;
    }
    const size_t idx = ((size_t)z * H + y) * W + x;
    f2 tv = {T[idx], two ? T[idx + W] : 1.f};   // the absent voxel reads as T = 1, W = 0 (never stored)
    f2 wv = {Wt[idx], two ? Wt[idx + W] : 0.f};
    // lanes whose stored (T, W) lie outside the fast division's range divide exactly throughout
    const bool wild = !(tame(tv.x, wv.x) && tame(tv.y, wv.y));
    const bool wi0 = w_runs_launch(wv.x), wi1 = w_runs_launch(wv.y);
    const size_t frame = (size_t)Hd * Wd;
    const int nbytes = (int)(frame * 4);   // host-checked < 2^31
    const int Wd4 = Wd * 4;                 // < 2^24: exact in v_mul_u32_u24

    auto update = [&](f2 ts, bool g0, bool g1) {
        const f2 n = tv * wv + ts;
        const f2 d = wv + f2s(1.0f);
        f2 q = div_rn(n, d);
        if (wild || !(fabsf(n.x) >= 0x1p-100f)) q.x = n.x / d.x;
        if (wild || !(fabsf(n.y) >= 0x1p-100f)) q.y = n.y / d.y;
        tv.x = g0 ? q.x : tv.x;
        wv.x = g0 ? d.x : wv.x;
        tv.y = g1 ? q.y : tv.y;
        wv.y = g1 ? d.y : wv.y;
    };

    if constexpr (PIPE) {
        // frame cursor over the masks: events are free-space runs (k frames) and
        // projected frames, in frame order
        int cw = -1;
        unsigned ctodo = 0u, cfre = 0u;
        auto next = [&](int& val) -> int {   // 0 end, 1 free run of val frames, 2 projected frame val
            while (ctodo == 0u) {
                if (++cw >= nw) return 0;
                const int w0 = cw << 5;
                unsigned t = F - w0 >= 32 ? ~0u : ((1u << (F - w0)) - 1u), fr = 0u;
                if (cull) {
                    t &= ~cull[slot + cw];
                    if (freem) fr = freem[slot + cw] & t;
                }
                ctodo = (unsigned)__builtin_amdgcn_readfirstlane((int)t);
                cfre = (unsigned)__builtin_amdgcn_readfirstlane((int)fr);
            }
            if (cfre & ctodo & (0u - ctodo)) {
                const unsigned full = ctodo & ~cfre;
                const unsigned run = ctodo & (full ? (full & (0u - full)) - 1u : ~0u);
                ctodo &= ~run;
                val = __builtin_popcount(run);
                return 1;
            }
            val = (cw << 5) + __builtin_ctz(ctodo);
            ctodo &= ctodo - 1u;
            return 2;
        };
        struct Proj { f2 Zc, dep; bool ok0, ok1; };
        auto project = [&](int f) -> Proj {   // projection + the (issued) depth gather
#ifdef SFMHIP_TSDF_PROF
            ++prof_nproj;
#endif
            const float* r = rec + f * 16;
            const f2 Q = (f2{r[0], r[1]} * f2s(vx) + f2{r[2], r[3]} * f2s(vz)) + f2{r[4], r[5]};
            const float Qz = (r[6] * vx + r[7] * vz) + r[8];
            const f2 Xc = f2s(r[9]) * vy + f2s(Q.x);
            const f2 Yc = f2s(r[10]) * vy + f2s(Q.y);
            Proj p;
            p.Zc = f2s(r[11]) * vy + f2s(Qz);
            const f2 iz = recip_rn(p.Zc);
            const f2 uu = (f2s(r[12]) * Xc) * iz + f2s(r[14]);
            const f2 vv = (f2s(r[13]) * Yc) * iz + f2s(r[15]);
            const int iu0 = cvt_flr(uu.x), iv0 = cvt_flr(vv.x);
            const int iu1 = cvt_flr(uu.y), iv1 = cvt_flr(vv.y);
            p.ok0 = z_ok(p.Zc.x) && (unsigned)iu0 < (unsigned)Wd && (unsigned)iv0 < (unsigned)Hd;
            p.ok1 = two && z_ok(p.Zc.y) && (unsigned)iu1 < (unsigned)Wd && (unsigned)iv1 < (unsigned)Hd;
            const __amdgpu_buffer_rsrc_t rs =
                __builtin_amdgcn_make_buffer_rsrc((void*)(depth + (size_t)f * frame), (short)0, nbytes, 0x00020000);
            p.dep = f2{0.f, 0.f};
            if (p.ok0)
                p.dep.x = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                        rs, (int)(__umul24(iv0, Wd4) + ((unsigned)iu0 << 2)), 0, 0));
            if (p.ok1)
                p.dep.y = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                        rs, (int)(__umul24(iv1, Wd4) + ((unsigned)iu1 << 2)), 0, 0));
            return p;
        };
        auto finish = [&](const Proj& p) {
            const f2 sdf = p.dep - p.Zc;
            const bool g0 = p.ok0 && p.dep.x > 0.f && !(sdf.x < -trunc);
            const bool g1 = p.ok1 && p.dep.y > 0.f && !(sdf.y < -trunc);
            const f2 sc = sdf * f2s(inv_trunc);
            const f2 ts = {fminf(1.0f, sc.x), fminf(1.0f, sc.y)};
            const bool easy0 = !g0 || (ts.x == 1.f && tv.x == 1.f && wi0);
            const bool easy1 = !g1 || (ts.y == 1.f && tv.y == 1.f && wi1);
            if (easy && __builtin_amdgcn_ballot_w64(!(easy0 && easy1)) == 0) {
                wv.x = g0 ? wv.x + 1.f : wv.x;
                wv.y = g1 ? wv.y + 1.f : wv.y;
            } else {
                update(ts, g0, g1);
            }
        };
        auto free_run = [&](int k) {
            const bool ones = tv.x == 1.f && tv.y == 1.f && wi0 && wi1;
            if (free_ts == 1.f && __builtin_amdgcn_ballot_w64(!ones) == 0) {
                wv = wv + f2s((float)k);
            } else {
                for (int i = 0; i < k; ++i) update(f2s(free_ts), true, two);
            }
        };
        int val = 0, kind = next(val);
        Proj pend;
        bool have = false;
        int run = 0;   // free frames between the pending projected frame and the next event
        while (kind != 0) {
            if (kind == 1) {
                if (have) run += val;
                else free_run(val);
                kind = next(val);
                continue;
            }
            const Proj p = project(val);   // its gather is in flight from here
            if (have) {
                finish(pend);
                if (run) free_run(run);
            }
            pend = p;
            have = true;
            run = 0;
            kind = next(val);
        }
        if (have) {
            finish(pend);
            if (run) free_run(run);
        }
    } else
    for (int w0 = 0; w0 < F; w0 += 32) {
        const int wd = w0 >> 5;
        unsigned todo = F - w0 >= 32 ? ~0u : ((1u << (F - w0)) - 1u), fre = 0u;
        if (cull) {   // wave-uniform address: scalar loads
            todo &= ~cull[slot + wd];
            if (freem) fre = freem[slot + wd] & todo;
        }
        todo = (unsigned)__builtin_amdgcn_readfirstlane((int)todo);
        fre = (unsigned)__builtin_amdgcn_readfirstlane((int)fre);
        while (todo) {
            if (fre & todo & (0u - todo)) {   // lowest pending frame is free space: take its run
                const unsigned full = todo & ~fre;
                const unsigned run = todo & (full ? (full & (0u - full)) - 1u : ~0u);
                todo &= ~run;
                const int k = __builtin_popcount(run);
                const bool ones = tv.x == 1.f && tv.y == 1.f && wi0 && wi1;
                if (free_ts == 1.f && __builtin_amdgcn_ballot_w64(!ones) == 0) {
                    wv = wv + f2s((float)k);
                } else {
                    for (int i = 0; i < k; ++i) update(f2s(free_ts), true, two);
                }
                continue;
            }
            const int f = w0 + __builtin_ctz(todo);
            todo &= todo - 1u;
#ifdef SFMHIP_TSDF_PROF
            ++prof_nproj;
#endif
            f2 ts;
            bool g0, g1;
            tsdf_frame_eval(rec, f, vx, vy, vz, two, depth, frame, nbytes, Wd4, Hd, Wd, trunc, inv_trunc, free_ts,
                            bmm, nbu, nbv, ts, g0, g1);
            // every updating voxel of the wave has tsdf = 1, T = 1 and an integer W: each
            // update is (1 W + 1)/(W + 1) = 1 and W + 1, exactly (no division)
            const bool easy0 = !g0 || (ts.x == 1.f && tv.x == 1.f && wi0);
            const bool easy1 = !g1 || (ts.y == 1.f && tv.y == 1.f && wi1);
            if (easy && __builtin_amdgcn_ballot_w64(!(easy0 && easy1)) == 0) {
                wv.x = g0 ? wv.x + 1.f : wv.x;
                wv.y = g1 ? wv.y + 1.f : wv.y;
            } else {
                update(ts, g0, g1);
            }
        }
    }
    T[idx] = tv.x;
    Wt[idx] = wv.x;
    if (two) {
        T[idx + W] = tv.y;
        Wt[idx + W] = wv.y;
    }
#ifdef SFMHIP_TSDF_PROF
    if ((threadIdx.x & 63) == __builtin_amdgcn_readfirstlane((int)(threadIdx.x & 63)) && prof_w < kTsdfProfWaves) {
        g_tsdf_prof[3 * prof_w] = prof_t0;
        g_tsdf_prof[3 * prof_w + 1] = wall_clock64();
        g_tsdf_prof[3 * prof_w + 2] = (unsigned long long)prof_nproj;
    }
#endif
}

// ---------------------------------------------------------------------------
// Heavy sub-tiles (surface bands: up to ~225 projected frames of one 8x2x8 sub-tile): the
// per-voxel update T <- (T W + ts)/(W + 1) must run in frame order (bit-exact with the oracle), but
// the projection, block test, gather and ts of a frame do not depend on T or W.  tsdf_kernel keeps
// all of it on the sub-tile's one wave, ~1 us per projected frame of dependent work, which bounds a
// thin z-slab.  Here one 512-thread workgroup owns one heavy sub-tile: waves 1..7
// (producers) evaluate the projected frames, interleaved, kHvyK per wave per round, into an LDS
// round buffer (ts per voxel, NaN = no update); wave 0 (the consumer) holds (T, W) and applies the
// rounds in frame order — free-space runs from the masks and the projected frames from the buffer,
// with tsdf_kernel's own update and division-free paths — while the producers fill the next round
// (double buffer, one barrier per round).  Same updates in the same order: the same bits.
//   tsdf_heavy_list_kernel: per sub-tile projected-frame count from the final masks; sub-tiles at
//     or above the threshold are listed (wave-aggregated append) and flagged so tsdf_kernel skips
//     them; the heavy kernel runs concurrently with tsdf_kernel on a side stream (tsdf_run).
constexpr int kHvyWaves = 8, kHvyProd = kHvyWaves - 1, kHvyK = 4;   // K: frames per producer per round

__global__ __launch_bounds__(256) void tsdf_heavy_list_kernel(const unsigned* __restrict__ cull,
                                                              const unsigned* __restrict__ freem, int nw, int F,
                                                              int64_t nsub, unsigned thr,
                                                              unsigned char* __restrict__ skip,
                                                              unsigned* __restrict__ hlist,
                                                              unsigned* __restrict__ hcount) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    unsigned cnt = 0u;
    if (i < nsub) {
        for (int w = 0; w < nw; ++w) {
            const int w0 = w << 5;
            const unsigned live = F - w0 >= 32 ? ~0u : ((1u << (F - w0)) - 1u);
            const unsigned c = cull[i * nw + w], fr = freem ? freem[i * nw + w] : 0u;
            cnt += __builtin_popcount(live & ~c & ~fr);
        }
        skip[i] = cnt >= thr ? 1 : 0;
    }
    const bool heavy = i < nsub && cnt >= thr;
    const uint64_t b = __builtin_amdgcn_ballot_w64(heavy);
    if (b == 0) return;
    const int lane = threadIdx.x & 63;
    const int first = __builtin_ctzll(b);
    unsigned base = 0;
    if (lane == first) base = atomicAdd(hcount, (unsigned)__builtin_popcountll(b));
    base = __shfl(base, first, 64);
    if (heavy) hlist[base + __builtin_popcountll(b & ((1ull << lane) - 1ull))] = (unsigned)i;
}

template <int K>
__global__ __launch_bounds__(kHvyWaves * 64) void tsdf_heavy_kernel(
    float* __restrict__ T, float* __restrict__ Wt, int D, int H, int W, int z0, int z1, const float* __restrict__ depth,
    int F, int Hd, int Wd, const float* __restrict__ rec, Bounds B, float trunc, const unsigned* __restrict__ cull,
    const unsigned* __restrict__ freem, int nw, float free_ts, const float2* __restrict__ bmm, int nbu, int nbv,
    int easy, const unsigned* __restrict__ hlist, const unsigned* __restrict__ hcount, int hprobe) {
    constexpr int R = kHvyProd * K;   // projected frames per round
    __shared__ f2 buf[2][R][64];
    __shared__ unsigned short plist[kTsdfMaxFrames];
    __shared__ int s_np;
    const int l = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const unsigned count = *hcount;
    const int ntx = (W + kTsdfTX - 1) / kTsdfTX, nty = (H + kTsdfTY - 1) / kTsdfTY;
    const float sx = (B.mx[0] - B.mn[0]) / (float)(W - 1);
    const float sy = (B.mx[1] - B.mn[1]) / (float)(H - 1);
    const float sz = (B.mx[2] - B.mn[2]) / (float)(D - 1);
    const float inv_trunc = 1.0f / trunc;
    const size_t frame = (size_t)Hd * Wd;
    const int nbytes = (int)(frame * 4);
    const int Wd4 = Wd * 4;
    const float no_upd = __builtin_bit_cast(float, 0x7FC00000u);
    for (unsigned item = blockIdx.x; item < count; item += gridDim.x) {
        const unsigned sub = __builtin_amdgcn_readfirstlane((int)hlist[item]);
        const unsigned tile = sub / kCullSub;
        const int ws = (int)(sub % kCullSub);
        const int bx = (int)(tile % ntx), by = (int)((tile / ntx) % nty), bz = (int)(tile / ((unsigned)ntx * nty));
        const int x = bx * kTsdfTX + (l & 3) + 4 * ((l >> 4) & 1);
        const int z = z0 + bz * kTsdfTZ + ((l >> 2) & 3) + 4 * (l >> 5);
        const int y = by * kTsdfTY + 2 * ws;
        const bool inb = x < W && y < H && z < z1;
        const bool two = inb && y + 1 < H;
        const float vx = B.mn[0] + (float)x * sx;
        const f2 vy = {B.mn[1] + (float)y * sy, B.mn[1] + (float)(y + 1) * sy};
        const float vz = B.mn[2] + (float)z * sz;
        const size_t slot = (size_t)sub * nw;
        if (wave == 0) {   // the projected frames in order: lane w < nw takes mask word w
            unsigned pw = 0u;
            if (l < nw) {
                const int w0 = l << 5;
                pw = (F - w0 >= 32 ? ~0u : ((1u << (F - w0)) - 1u)) & ~cull[slot + l];
                if (freem) pw &= ~freem[slot + l];
            }
            const int c = __builtin_popcount(pw);
            int incl = c;
#pragma unroll
            for (int off = 1; off < 16; off <<= 1) {
                const int up = __shfl_up(incl, off, 64);
                if (l >= off) incl += up;
            }
            int pos = incl - c;
            while (pw) {
                plist[pos++] = (unsigned short)((l << 5) + __builtin_ctz(pw));
                pw &= pw - 1u;
            }
            if (l == 15) s_np = incl;
        }
        __syncthreads();
        const int np = s_np;
        const int nr = (np + R - 1) / R;
        auto produce = [&](int r) {   // producer wave p: projected frames r R + (p - 1) + kHvyProd j
            for (int j = wave - 1; j < R; j += kHvyProd) {
                const int k = r * R + j;
                if (k >= np) break;
                const int f = plist[k];
                f2 ts;
                bool g0, g1;
#ifdef SFMHIP_PROBES   // timing probe 1: no frame evaluation (a constant partial update)
                if (hprobe & 1) {
                    ts = f2{0.5f, 0.5f};
                    g0 = g1 = (f & 1) == 0;
                } else
#endif
                tsdf_frame_eval(rec, f, vx, vy, vz, two, depth, frame, nbytes, Wd4, Hd, Wd, trunc, inv_trunc,
                                free_ts, bmm, nbu, nbv, ts, g0, g1);
                buf[r & 1][j][l] = f2{g0 && inb ? ts.x : no_upd, g1 ? ts.y : no_upd};
            }
        };
        // consumer state (wave 0): (T, W) in registers, tsdf_kernel's update paths, events in frame order
        const size_t idx = ((size_t)z * H + y) * W + x;
        f2 tv = f2{1.f, 1.f}, wv = f2{0.f, 0.f};
        if (wave == 0) {
            tv = f2{inb ? T[idx] : 1.f, two ? T[idx + W] : 1.f};
            wv = f2{inb ? Wt[idx] : 0.f, two ? Wt[idx + W] : 0.f};
        }
        const bool wild = !(tame(tv.x, wv.x) && tame(tv.y, wv.y));
        const bool wi0 = w_runs_launch(wv.x), wi1 = w_runs_launch(wv.y);
        auto update = [&](f2 ts, bool g0, bool g1) {
            const f2 n = tv * wv + ts;
            const f2 d = wv + f2s(1.0f);
            f2 q = div_rn(n, d);
            if (wild || !(fabsf(n.x) >= 0x1p-100f)) q.x = n.x / d.x;
            if (wild || !(fabsf(n.y) >= 0x1p-100f)) q.y = n.y / d.y;
            tv.x = g0 ? q.x : tv.x;
            wv.x = g0 ? d.x : wv.x;
            tv.y = g1 ? q.y : tv.y;
            wv.y = g1 ? d.y : wv.y;
        };
        auto free_run = [&](int k) {
            const bool ones = tv.x == 1.f && tv.y == 1.f && wi0 && wi1;
            if (free_ts == 1.f && __builtin_amdgcn_ballot_w64(!ones) == 0) {
                wv = wv + f2s((float)k);
            } else {
                for (int i = 0; i < k; ++i) update(f2s(free_ts), inb, two);
            }
        };
        int cw = -1;
        unsigned ctodo = 0u, cfre = 0u;
        int done = 0;   // projected frames applied
        // apply every event before projected frame `upto` (its free-space run included)
        auto consume = [&](int upto, int r) {
            while (true) {
                while (ctodo == 0u) {
                    if (++cw >= nw) return;
                    const int w0 = cw << 5;
                    unsigned t = F - w0 >= 32 ? ~0u : ((1u << (F - w0)) - 1u), fr = 0u;
                    t &= ~cull[slot + cw];
                    if (freem) fr = freem[slot + cw] & t;
                    ctodo = (unsigned)__builtin_amdgcn_readfirstlane((int)t);
                    cfre = (unsigned)__builtin_amdgcn_readfirstlane((int)fr);
                }
                if (cfre & ctodo & (0u - ctodo)) {   // lowest pending frame is free space: its run
                    const unsigned full = ctodo & ~cfre;
                    const unsigned run = ctodo & (full ? (full & (0u - full)) - 1u : ~0u);
                    ctodo &= ~run;
                    free_run(__builtin_popcount(run));
                    continue;
                }
                if (done >= upto) return;   // the next projected frame belongs to a later round
                ctodo &= ctodo - 1u;
                const f2 ts = buf[r & 1][done - r * R][l];
                ++done;
                const bool g0 = ts.x == ts.x, g1 = ts.y == ts.y;   // NaN: no update
                const bool easy0 = !g0 || (ts.x == 1.f && tv.x == 1.f && wi0);
                const bool easy1 = !g1 || (ts.y == 1.f && tv.y == 1.f && wi1);
                if (easy && __builtin_amdgcn_ballot_w64(!(easy0 && easy1)) == 0) {
                    wv.x = g0 ? wv.x + 1.f : wv.x;
                    wv.y = g1 ? wv.y + 1.f : wv.y;
                } else {
                    update(ts, g0, g1);
                }
            }
        };
        if (wave != 0) produce(0);
        __syncthreads();   // round 0 produced
        for (int r = 0; r < nr; ++r) {   // the consumer applies round r while the producers fill round r + 1
#ifdef SFMHIP_PROBES   // timing probe 2: the consumer skips the application
            if (wave == 0 && (hprobe & 2)) done = min(np, (r + 1) * R);
            else
#endif
            if (wave == 0) consume(min(np, (r + 1) * R), r);
            else if (r + 1 < nr) produce(r + 1);
            __syncthreads();
        }
        if (wave == 0) {
            consume(np, nr);   // the free-space runs after the last projected frame
            if (inb) {
                T[idx] = tv.x;
                Wt[idx] = wv.x;
            }
            if (two) {
                T[idx + W] = tv.y;
                Wt[idx + W] = wv.y;
            }
        }
        __syncthreads();   // plist / s_np reused by the next item
    }
}

static int env_int(const char* name, int dflt) {
    const char* e = std::getenv(name);
    return e ? std::atoi(e) : dflt;
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
    SFMHIP_REQUIRE(rays && n_steps, "sfmhip_voxel_traversal_count: null pointer");
    SFMHIP_REQUIRE(N >= 0 && max_steps > 0 && max_steps < INT_MAX, "sfmhip_voxel_traversal_count: bad args");
    if (N == 0) return SFMHIP_OK;
    hipLaunchKernelGGL(dda_count_kernel, dim3(ceil_div(N, 64)), dim3(64), 0, as_stream(stream), rays, N, bin,
                       max_steps, n_steps);   // one wave per workgroup: the waves spread over the CUs
    return check_launch("dda_count_kernel");
}

extern "C" int sfmhip_voxel_traversal(const float* rays, int64_t N, float bin, int32_t S, float* out,
                                      void* stream) {
    SFMHIP_REQUIRE(rays && out, "sfmhip_voxel_traversal: null pointer");
    SFMHIP_REQUIRE(N >= 0 && S >= 1, "sfmhip_voxel_traversal: bad args");
    if (N == 0) return SFMHIP_OK;
    // SFMHIP_DDA_DIRECT (A/B): 1 per-lane row stores, 0 LDS-staged coalesced
    // chunks; default: direct below 64k rays (latency-bound), staged above.
    const char* denv = std::getenv("SFMHIP_DDA_DIRECT");
    const bool direct = denv ? std::atoi(denv) != 0 : N < 65536;
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
    SFMHIP_REQUIRE(buf && n_steps && out, "sfmhip_voxel_traversal_rows: null pointer");
    SFMHIP_REQUIRE(N >= 0 && S >= 1 && S <= cap, "sfmhip_voxel_traversal_rows: bad args (1 <= S <= cap)");
    if (N == 0) return SFMHIP_OK;
    const int64_t total = N * (int64_t)S * 3;
    hipLaunchKernelGGL(dda_rows_kernel, dim3((unsigned)std::min<int64_t>(ceil_div(total, 256), 8192)), dim3(256), 0,
                       as_stream(stream), buf, cap, n_steps, N, S, out);
    return check_launch("dda_rows_kernel");
}

extern "C" int sfmhip_voxel_traversal_capped(const float* rays, int64_t N, float bin, int32_t cap, float* out,
                                             int32_t* n_steps, void* stream) {
    SFMHIP_REQUIRE(rays && out && n_steps, "sfmhip_voxel_traversal_capped: null pointer");
    SFMHIP_REQUIRE(N >= 0 && cap >= 2, "sfmhip_voxel_traversal_capped: bad args (cap >= 2)");
    if (N == 0) return SFMHIP_OK;
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
    SFMHIP_REQUIRE(grid && bmin && bmax && pts && out, "sfmhip_grid_sample: null pointer");
    SFMHIP_REQUIRE(C > 0 && D > 1 && H > 1 && W > 1 && P >= 0, "sfmhip_grid_sample: bad shape");
    SFMHIP_REQUIRE(mask_mode == 0 || mask_mode == 1, "sfmhip_grid_sample: mask_mode must be 0 or 1");
    if (P == 0) return SFMHIP_OK;
    hipLaunchKernelGGL(grid_sample_kernel, dim3(ceil_div(P, 256)), dim3(256), 0, as_stream(stream), grid, C, D,
                       H, W, make_bounds(bmin, bmax), mask_mode, pts, P, out);
    return check_launch("grid_sample_kernel");
}

extern "C" int sfmhip_nerf_forward(const float* grid, int D, int H, int W, const float* bmin, const float* bmax,
                                   int mask_mode, const float* pts, const float* dirs, int64_t P, float* color,
                                   float* sigma, void* stream) {
    SFMHIP_REQUIRE(grid && bmin && bmax && pts && dirs && color && sigma, "sfmhip_nerf_forward: null pointer");
    SFMHIP_REQUIRE(D > 0 && H > 0 && W > 0 && P >= 0, "sfmhip_nerf_forward: bad shape");
    SFMHIP_REQUIRE(mask_mode == 0 || mask_mode == 1, "sfmhip_nerf_forward: mask_mode must be 0 or 1");
    if (P == 0) return SFMHIP_OK;
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
// workgroup from the L2-resident histogram) + rank; with xchunk > 0 the sorted positions
// are laid out so that XCD x gets runs of xchunk consecutive 4-ray workgroups (blocks
// are dealt round-robin over the XCDs)
__global__ __launch_bounds__(256) void render_scatter_kernel(const unsigned* __restrict__ hist, int nb,
                                                             const unsigned* __restrict__ key,
                                                             const unsigned* __restrict__ rank, int64_t nrays,
                                                             int xchunk, unsigned* __restrict__ order) {
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
    int64_t pos = (int64_t)base[key[i]] + rank[i];
    if (xchunk > 0) {
        const int64_t grp = (int64_t)4 * kNumXcd * xchunk;   // rays per full round of runs
        const int64_t full = nrays / grp * grp;
        if (pos < full) {   // logical block L -> launch block: L = ((s / c) * 8 + x) * c + s % c
            const int64_t L = pos >> 2, c = xchunk;
            const int64_t rn = L / c, s_in = L % c, x = rn % kNumXcd, sq = (rn / kNumXcd) * c + s_in;
            pos = ((sq * kNumXcd + x) << 2) | (pos & 3);
        }
    }
    order[pos] = (unsigned)i;
}

static void launch_render(const float* sdfp, dim3 grid, hipStream_t st, const float* gvm, int D, int H, int W,
                          const Bounds& bb, int mode, const float* ro, const float* rd, const float* z, int64_t B, int S,
                          float* rgb, const unsigned* order) {
    // 4 waves per SIMD for the sdf-plane form (128 VGPRs): 0.524 vs 0.538 ms on the bench workload; 5, 6
    // and 8 spill (0.69 / 0.84 / 3.8 ms), profiles/r4/ab_render_occ_heavy_trace_r4g.log
    const int occ = env_int("SFMHIP_RENDER_OCC", sdfp ? 4 : 0);
#define SFMHIP_RENDER_LAUNCH(SIG, OCC)                                                                        \
    hipLaunchKernelGGL((render_kernel<SIG, OCC>), grid, dim3(256), 0, st, gvm, D, H, W, bb, mode, ro, rd, z, B, S, \
                       rgb, order, SIG ? sdfp : nullptr)
    const int two = env_int("SFMHIP_RENDER_2PH", 0);   // A/B: two-phase sdf-plane form, chunks per group
    if (sdfp && two > 0) {
        if (two >= 4) {
            if (occ == 4) hipLaunchKernelGGL((render_kernel<true, 4, 4>), grid, dim3(256), 0, st, gvm, D, H, W, bb, mode,
                                             ro, rd, z, B, S, rgb, order, sdfp);
            else hipLaunchKernelGGL((render_kernel<true, 0, 4>), grid, dim3(256), 0, st, gvm, D, H, W, bb, mode, ro, rd,
                                    z, B, S, rgb, order, sdfp);
        } else {
            if (occ == 4) hipLaunchKernelGGL((render_kernel<true, 4, 3>), grid, dim3(256), 0, st, gvm, D, H, W, bb, mode,
                                             ro, rd, z, B, S, rgb, order, sdfp);
            else hipLaunchKernelGGL((render_kernel<true, 0, 3>), grid, dim3(256), 0, st, gvm, D, H, W, bb, mode, ro, rd,
                                    z, B, S, rgb, order, sdfp);
        }
    } else if (sdfp) {
        if (occ == 4) SFMHIP_RENDER_LAUNCH(true, 4);
        else if (occ == 5) SFMHIP_RENDER_LAUNCH(true, 5);
        else if (occ == 6) SFMHIP_RENDER_LAUNCH(true, 6);
        else if (occ == 8) SFMHIP_RENDER_LAUNCH(true, 8);
        else SFMHIP_RENDER_LAUNCH(true, 0);
    } else {
        if (occ == 4) SFMHIP_RENDER_LAUNCH(false, 4);
        else if (occ == 5) SFMHIP_RENDER_LAUNCH(false, 5);
        else if (occ == 6) SFMHIP_RENDER_LAUNCH(false, 6);
        else if (occ == 8) SFMHIP_RENDER_LAUNCH(false, 8);
        else SFMHIP_RENDER_LAUNCH(false, 0);
    }
#undef SFMHIP_RENDER_LAUNCH
}

static int render_run(const float* grid_vm, const float* sdfp, int D, int H, int W, const float* bmin,
                      const float* bmax, int mask_mode, const float* rays_o, const float* rays_d, const float* z,
                      int64_t B, int S, float* rgb, void* stream) {
    SFMHIP_REQUIRE(grid_vm && bmin && bmax && rays_o && rays_d && z && rgb, "sfmhip_render_rays: null pointer");
    SFMHIP_REQUIRE(D > 1 && H > 1 && W > 1 && B >= 0 && S >= 1, "sfmhip_render_rays: bad shape");
    SFMHIP_REQUIRE(mask_mode == 0 || mask_mode == 1, "sfmhip_render_rays: mask_mode must be 0 or 1");
    SFMHIP_REQUIRE(B < ((int64_t)1 << 32), "sfmhip_render_rays: more than 2^32 rays");
    if (B == 0) return SFMHIP_OK;
    hipStream_t st = as_stream(stream);
    const Bounds bb = make_bounds(bmin, bmax);
    // ray ordering (SFMHIP_RENDER_SORT=0 off; _BITS cells per axis as a power of two, _SIDX the
    // sample (default the last), _XCHUNK XCD runs of workgroups): batches below 8192 rays fill
    // only a fraction of the chip's waves at once and are rendered as given.  Bench workload
    // (tools/bench_render_order.py, profiles/r3/ab/render_order_r3j.txt): 0.627-0.648 ms as
    // given, 0.598 ms with this ordering (sort kernels included); keys and cell sizes from
    // 2^2 to 2^8 per axis, host-sorted, all give the same ~0.58 ms kernel
    const int sort = env_int("SFMHIP_RENDER_SORT", 1);
    const int bits = std::min(std::max(env_int("SFMHIP_RENDER_SORT_BITS", 3), 1), 4);
    const int sidx = std::min(std::max(env_int("SFMHIP_RENDER_SORT_SIDX", S - 1), 0), S - 1);
    const int xchunk = std::max(env_int("SFMHIP_RENDER_SORT_XCHUNK", 0), 0);
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
                               xchunk, order);
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
// ext_table != nullptr: the caller's {min, max} block table of every frame over the
// whole image ([F][nbv][nbu] float2, sfmhip_tsdf_block_table); the block pass is skipped.
// Library-owned side stream per device (created once): tsdf_heavy_kernel runs on it beside
// tsdf_kernel on the caller's stream, forked and joined with events, so the call stays ordered on
// the caller's stream.  The mutex keeps one fork/join sequence at a time per device.
constexpr int kPrePipeMax = 8;   // frame groups of the pre-pass pipeline
struct SideStream {
    hipStream_t s = nullptr, hi = nullptr;   // hi: the device's greatest stream priority
    hipEvent_t fork = nullptr, join = nullptr;
    hipEvent_t grp[kPrePipeMax] = {};        // pre-pass pipeline: block tables of frame groups ready
    std::mutex mu;
};
static SideStream g_side[64];
static std::once_flag g_side_once[64];
static SideStream* side_stream(int dev) {
    if (dev < 0 || dev >= 64) return nullptr;
    std::call_once(g_side_once[dev], [dev] {
        SideStream& ss = g_side[dev];
        int lo = 0, hi = 0;
        if (hipDeviceGetStreamPriorityRange(&lo, &hi) != hipSuccess ||
            hipStreamCreateWithPriority(&ss.hi, hipStreamNonBlocking, hi) != hipSuccess)
            ss.hi = nullptr;
        bool ok = hipStreamCreateWithFlags(&ss.s, hipStreamNonBlocking) == hipSuccess &&
                  hipEventCreateWithFlags(&ss.fork, hipEventDisableTiming) == hipSuccess &&
                  hipEventCreateWithFlags(&ss.join, hipEventDisableTiming) == hipSuccess;
        for (int k = 0; ok && k < kPrePipeMax; ++k)
            ok = hipEventCreateWithFlags(&ss.grp[k], hipEventDisableTiming) == hipSuccess;
        if (!ok) ss.s = nullptr;
        (void)hipGetLastError();
    });
    return g_side[dev].s ? &g_side[dev] : nullptr;
}

static int tsdf_run(float* T, float* Wt, int D, int H, int W, int z0, int z1, const float* depth, int F, int Hd,
                    int Wd, const float* poses, const float* Kf, const float* bmin, const float* bmax, float trunc,
                    void* stream, int64_t* stats, const float2* ext_table, int64_t* layer_stats = nullptr) {
    SFMHIP_REQUIRE(T && Wt && depth && poses && Kf && bmin && bmax, "sfmhip_tsdf_integrate: null pointer");
    SFMHIP_REQUIRE(D > 1 && H > 1 && W > 1 && F >= 0 && Hd > 0 && Wd > 0, "sfmhip_tsdf_integrate: bad shape");
    SFMHIP_REQUIRE(0 <= z0 && z0 <= z1 && z1 <= D, "sfmhip_tsdf_integrate: bad z range");
    SFMHIP_REQUIRE(trunc > 0.f, "sfmhip_tsdf_integrate: trunc must be > 0");
    if (F == 0 || z0 == z1) return SFMHIP_OK;
    SFMHIP_REQUIRE((int64_t)Hd * Wd * 4 < (int64_t)INT_MAX && Wd < (1 << 22) && Hd < (1 << 22),
                   "sfmhip_tsdf_integrate: depth map too large (4*Hd*Wd must be < 2^31)");
    for (int a = 0; a < 3; ++a)
        SFMHIP_REQUIRE(std::fabs(bmin[a]) < 0x1p60f && std::fabs(bmax[a]) < 0x1p60f,
                       "sfmhip_tsdf_integrate: bounds must be finite and below 2^60 in magnitude");
    // Tuning knobs (A/B runs only): SFMHIP_TSDF_SWZ (super-brick XCD order),
    // SFMHIP_TSDF_SBX/SBY/SBZ/IL and SFMHIP_TSDF_CHUNK (frames per launch).
    const int swz = env_int("SFMHIP_TSDF_SWZ", 1);
    // default: super-bricks of 3 x 2 x 8 tiles (24 x 16 x 64 voxels) dealt round-robin over the
    // XCDs (sweeps in tools/bench_tsdf_variants.py; with culling the work per tile is uneven, and
    // the interleave plus a width that does not divide the grid spreads it over the XCDs)
    const int nbx = ceil_div(W, kTsdfTX), nby = ceil_div(H, kTsdfTY), nbz = ceil_div(z1 - z0, kTsdfTZ);
    // SFMHIP_TSDF_CULL: 0 off (A/B runs), otherwise on: with the free-space path the
    // pre-passes pay even for the thin z-slabs of an 8-way split (tools/bench_tsdf_slabs.py:
    // N=8 slab 0.92 vs 1.34 ms without them)
    const int cull_env = env_int("SFMHIP_TSDF_CULL", 1);
    const bool want_cull = stats || cull_env != 0;
    // every frame in one launch (<= 512) with culling: the grid is read and written once and
    // there is one dispatch (64-frame launches: 2.65 vs 2.29 ms on C5); without culling every
    // frame gathers, and 64-frame launches keep the resident workgroups' depth set in L2
    const int chunk = std::max(1, std::min(kTsdfMaxFrames, env_int("SFMHIP_TSDF_CHUNK", want_cull ? kTsdfMaxFrames : 64)));
    const int nw = ceil_div(std::min(chunk, F), 32);   // mask words per sub-tile slot
    const SuperBrick sb{std::max(1, env_int("SFMHIP_TSDF_SBX", 3)), std::max(1, env_int("SFMHIP_TSDF_SBY", 2)),
                        std::max(1, env_int("SFMHIP_TSDF_SBZ", std::min(8, nbz))), env_int("SFMHIP_TSDF_IL", 1)};
    dim3 grid(nbx, nby, nbz);
    if (swz) {
        int64_t nsb = (int64_t)ceil_div(nbx, sb.x) * ceil_div(nby, sb.y) * ceil_div(nbz, sb.z);
        if (sb.il) nsb = (nsb + kNumXcd - 1) / kNumXcd * kNumXcd;   // padding super-bricks exit at once
        const int64_t slots = nsb * (sb.x * sb.y * sb.z);
        SFMHIP_REQUIRE(slots < INT_MAX, "sfmhip_tsdf_integrate: grid too large");
        grid = dim3((unsigned)slots, 1, 1);
    }
    const Bounds bb = make_bounds(bmin, bmax);
    CullGeom cg;
    {
        const int n[3] = {W, H, D};
        for (int a = 0; a < 3; ++a) {
            cg.mn[a] = bb.mn[a];
            cg.s[a] = ((double)bb.mx[a] - bb.mn[a]) / (n[a] - 1);
            cg.as[a] = std::fabs(cg.s[a]);
        }
    }
    hipStream_t st = as_stream(stream);
    // Scratch (stream-ordered): validated camera records; culling buffers
    // (SFMHIP_TSDF_CULL=0 disables culling, SFMHIP_TSDF_FREE=0 the free-space path, for A/B
    // runs).  An allocation failure of the culling buffers only disables culling.
    const int nbu = ceil_div(Wd, kCullBlock), nbv = ceil_div(Hd, kCullBlock);
    const int64_t nsub = (int64_t)nbx * nby * nbz * kCullSub;
    const int per_tile = env_int("SFMHIP_TSDF_CULLSUB", 1) == 4 ? kCullSub : 1;
    // SFMHIP_TSDF_REFINE=0: no per-wave second pass over the projected tile-frames (A/B runs)
    // Few fusion workgroups per CU (a z-slab of a multi-GPU split: ~2 waves per SIMD slot
    // at N = 8) make the call latency-bound on its longest waves: then each projected
    // frame's depth is gathered without the block-table lookup in front of it and the
    // per-wave refinement pass is skipped (N = 8 centre slab 0.44 -> 0.39 ms; on the
    // whole grid, 16 rounds, the lookup saves more gathers than it costs: 2.63 vs 2.14 ms).
    // SFMHIP_TSDF_LATENCY: 0 never, 1 always, default by the rounds of resident waves.
    int ncu = 256;
    {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
            ncu = 256;
        (void)hipGetLastError();
    }
    const double rounds = (double)nbx * nby * nbz * kCullSub / (ncu * 32.0);   // 4 waves per tile, 32 per CU
    const int lat_env = env_int("SFMHIP_TSDF_LATENCY", -1);
    const bool latency_mode = lat_env >= 0 ? lat_env != 0 : rounds < kTsdfLatencyRounds;
    const bool want_refine = per_tile == 1 && env_int("SFMHIP_TSDF_REFINE", latency_mode ? 0 : 1) != 0;
    // cull pass: one workgroup per (4x4x4 brick of sub-tiles, 16 frames)
    const int64_t cull_bricks = (int64_t)ceil_div(nbx, 4) * ceil_div(nby * per_tile, 4) * ceil_div(nbz, 4);
    SFMHIP_REQUIRE(cull_bricks * ceil_div(std::min(chunk, F), 16) < INT_MAX, "sfmhip_tsdf_integrate: grid too large");
    // the free-space proof needs a trunc whose f32 reciprocal is a normal number
    const int free_env = env_int("SFMHIP_TSDF_FREE", 1);
    const bool want_free = free_env != 0 && trunc >= 0x1p-100f && trunc <= 0x1p100f;
    const float free_ts = free_env == 2 ? 0.5f : 1.0f;
    const int cf = std::min(chunk, F);
    const size_t nblk = (size_t)cf * nbu * nbv;
    float* rec = nullptr;   // the fusion kernel's f32 records, then the culling passes' CullCam table
    if (scratch_alloc((void**)&rec, (size_t)cf * (16 * sizeof(float) + sizeof(CullCam)), st) != hipSuccess) {
        (void)hipGetLastError();
        set_error("sfmhip_tsdf_integrate: camera table allocation failed");
        return SFMHIP_E_HIP;
    }
    float2* cbmm = nullptr;
    unsigned* cfree = nullptr;
    unsigned* cmask = nullptr;
    unsigned* plist = nullptr;   // projected (tile, frame) list + its count (last element)
    float2* ctab = nullptr;      // coarse table + brick decisions (brick pre-pass)
    unsigned char* bdec = nullptr;
    const int ncbu = ceil_div(nbu, kCoarse), ncbv = ceil_div(nbv, kCoarse);
    int4* crange = nullptr;
    // refinement list capacity: one entry per (tile, frame) of whole 32-frame words (the pre-pass
    // pipeline gives each frame group its own region), then the counters
    const int64_t plist_cap = (int64_t)nbx * nby * nbz * 32 * ceil_div(std::min(chunk, F), 32);
    if (want_cull) {
        if (ext_table) cbmm = const_cast<float2*>(ext_table);
        else if (scratch_alloc((void**)&cbmm, nblk * sizeof(float2), st) != hipSuccess) cbmm = nullptr;
        if (cbmm && (scratch_alloc((void**)&cmask, (size_t)nsub * nw * sizeof(unsigned), st) != hipSuccess ||
                     scratch_alloc((void**)&crange, (size_t)cf * sizeof(int4), st) != hipSuccess)) {
            if (cmask) scratch_free(cmask, st);
            if (!ext_table) scratch_free(cbmm, st);
            cbmm = nullptr;
            cmask = nullptr;
            crange = nullptr;
        }
        if (cmask && want_free && scratch_alloc((void**)&cfree, (size_t)nsub * nw * sizeof(unsigned), st) != hipSuccess)
            cfree = nullptr;   // free-space path off, culling unchanged
        // brick pre-pass (SFMHIP_TSDF_BRICK; default off in latency mode, where a thin slab's
        // cull pass is short and the two extra launches cost more than they save)
        if (cmask && env_int("SFMHIP_TSDF_BRICK", latency_mode ? 0 : 1) != 0) {
            if (scratch_alloc((void**)&ctab, (size_t)cf * ncbu * ncbv * sizeof(float2) + (size_t)cull_bricks * cf, st) ==
                hipSuccess)
                bdec = reinterpret_cast<unsigned char*>(ctab + (size_t)cf * ncbu * ncbv);
            else
                ctab = nullptr;   // no brick pre-pass
        }
        if (cmask && want_refine && plist_cap < (int64_t)1 << 30 && nbx * nby * nbz < (1 << 23) &&
            scratch_alloc((void**)&plist, (size_t)(plist_cap + kPrePipeMax) * sizeof(unsigned), st) != hipSuccess)
            plist = nullptr;   // no second pass
        (void)hipGetLastError();
    }
    // per-voxel block test in the fusion kernel (with the free-space path; SFMHIP_TSDF_VOXTEST=0 off)
    const bool vox_test = cfree && env_int("SFMHIP_TSDF_VOXTEST", latency_mode ? 0 : 1) != 0;
    // division-free update of projected frames whose updates are all tsdf = 1 on T = 1 (SFMHIP_TSDF_EASY=0 off)
    const int easy = env_int("SFMHIP_TSDF_EASY", 1) != 0;
    // latency mode without the block table: gathers one projected frame ahead (SFMHIP_TSDF_PIPE=0 off)
    const bool pipe = !vox_test && latency_mode && env_int("SFMHIP_TSDF_PIPE", 1) != 0;
    // longest-first workgroup order (SFMHIP_TSDF_ORDER=0 off): needs the masks and the 1-D slot grid;
    // at most 30000 slots per XCD class (16-bit sort positions; a bucket byte per slot in LDS
    // next to the 32 KB histogram, within the default 64 KB)
    unsigned* ord = nullptr;
    unsigned* tcost = nullptr;   // per-tile cost counters (after the order)
    const int64_t ntiles = (int64_t)nbx * nby * nbz;
    if (cmask && swz && !stats && env_int("SFMHIP_TSDF_ORDER", 1) != 0 && (int64_t)grid.x <= 30000LL * kNumXcd) {
        if (scratch_alloc((void**)&ord, (size_t)(grid.x + ntiles) * sizeof(unsigned), st) == hipSuccess)
            tcost = ord + grid.x;
        else
            ord = nullptr;
        (void)hipGetLastError();
    }
    // heavy sub-tiles (tsdf_heavy_kernel, frame-split over 7 producer waves): the projected-frame
    // threshold SFMHIP_TSDF_HEAVY (0 = off, the default) and the persistent grid SFMHIP_TSDF_HEAVY_WG.
    // Measured slower at every threshold and launch form (N = 8 centre slab 0.35 ms off,
    // 0.47-0.54 ms on; whole grid 1.93 vs 2.42-2.90 ms): kept as a tested A/B form only
    const int heavy_thr = env_int("SFMHIP_TSDF_HEAVY", 0);
    unsigned* hbuf = nullptr;   // [count][list nsub][skip nsub bytes]
    int dev_id = 0;
    (void)hipGetDevice(&dev_id);
    (void)hipGetLastError();
    SideStream* side = heavy_thr > 0 && cmask && !stats && swz ? side_stream(dev_id) : nullptr;
    if (side && scratch_alloc((void**)&hbuf, (size_t)(nsub + 1) * sizeof(unsigned) + (size_t)nsub, st) != hipSuccess) {
        (void)hipGetLastError();
        hbuf = nullptr;
    }
    const int heavy_wg = std::max(1, std::min<int>((int)std::min<int64_t>(nsub, INT_MAX),
                                                   env_int("SFMHIP_TSDF_HEAVY_WG", 2048)));
    // refine pass grid (grid-stride over the device-side count; atomic ORs, any grid gives the same masks):
    // 8192 x 256 threads fill the 6 waves per SIMD its 79 VGPRs allow, where 2048 gave 2 (C5 call
    // 1.93 -> 1.90 ms, profiles/r3/ab/tsdf_refine_wg_r3bp.txt)
    const int refine_wg = std::max(1, env_int("SFMHIP_TSDF_REFINE_WG", 8192));
    // Pre-pass pipeline (SFMHIP_TSDF_PREPIPE = frame groups, 0/1 off): the block pass of frame group
    // k + 1 (HBM-bound) runs on the library's side stream while the cull and refinement passes of
    // group k (latency-bound f64 tests) run on the caller's stream; every mask word is written by
    // the group that owns its frames, the refinement list has a region per group, and the fusion
    // waits for all of them.  Whole-grid mode with the call's own table; the brick pre-pass runs per
    // group too (coarse table and brick decisions are per frame).
    int pre_groups = 1;
    SideStream* pside = nullptr;
    if (cmask && !ext_table && !stats && !latency_mode) {
        pre_groups = std::min(kPrePipeMax, std::max(1, env_int("SFMHIP_TSDF_PREPIPE", 1)));
        if (pre_groups > 1 && !(pside = side_stream(dev_id))) pre_groups = 1;
    }
    // frame chunks run in order on the stream, so per-voxel update order is kept
    int rc = SFMHIP_OK;
    for (int f0 = 0; f0 < F; f0 += chunk) {
        const int nf = std::min(chunk, F - f0);
        const int nwf = ceil_div(nf, 32);
        const float* dp = depth + (size_t)f0 * Hd * Wd;
        const float* pp = poses + (size_t)f0 * 12;
        const float* kp = Kf + (size_t)f0 * 4;
        CullCam* ccam = cmask ? reinterpret_cast<CullCam*>(rec + (size_t)cf * 16) : nullptr;
        unsigned* pcount = plist ? plist + plist_cap : nullptr;
        const int nzero = tcost ? (int)ntiles : 0;
        hipLaunchKernelGGL(tsdf_setup_kernel, dim3(ceil_div(nf, 64) + (nzero || pcount ? std::min(64, ceil_div(nzero, 1024) + 1) : 0)),
                           dim3(64), 0, st, pp, kp, nf, rec, ccam, !cmask ? 0 : ext_table ? 1 : 2, H, W, z0, z1, Hd,
                           Wd, cg, nbu, nbv, crange, tcost, nzero, pcount);
        const float2* tab = ext_table ? ext_table + (size_t)f0 * nbv * nbu : cbmm;
        const int nh_all = 2 * nwf;
        const int groups = std::min(pre_groups, nh_all);
        if (groups > 1) {   // the pre-pass pipeline (above)
            std::lock_guard<std::mutex> lk(pside->mu);
            if (plist) (void)hipMemsetAsync(plist + plist_cap, 0, kPrePipeMax * sizeof(unsigned), st);
            (void)hipEventRecord(pside->fork, st);
            (void)hipStreamWaitEvent(pside->s, pside->fork, 0);
            for (int k = 0; k < groups; ++k) {
                const int h0 = nh_all * k / groups, h1 = nh_all * (k + 1) / groups;
                const int fa = h0 * kCullFrames, fb = std::min(nf, h1 * kCullFrames);
                if (fb > fa) {
                    if (Wd % 4 == 0)
                        hipLaunchKernelGGL(depth_blockmax_kernel<true>, dim3(ceil_div(Wd, 1024), nbv, fb - fa), dim3(256),
                                           0, pside->s, dp + (size_t)fa * Hd * Wd, fb - fa, Hd, Wd, nbu, nbv,
                                           crange + fa, cbmm + (size_t)fa * nbv * nbu);
                    else
                        hipLaunchKernelGGL(depth_blockmax_kernel<false>, dim3(ceil_div(Wd, 256), nbv, fb - fa), dim3(256),
                                           0, pside->s, dp + (size_t)fa * Hd * Wd, fb - fa, Hd, Wd, nbu, nbv,
                                           crange + fa, cbmm + (size_t)fa * nbv * nbu);
                }
                (void)hipEventRecord(pside->grp[k], pside->s);
            }
            for (int k = 0; k < groups; ++k) {
                const int h0 = nh_all * k / groups, h1 = nh_all * (k + 1) / groups;
                (void)hipStreamWaitEvent(st, pside->grp[k], 0);
                const int fa = h0 * kCullFrames, fb = std::min(nf, h1 * kCullFrames);
                if (bdec && fb > fa) {   // the group's coarse table and brick decisions (per frame)
                    const int gn = fb - fa;
                    const int64_t nc = (int64_t)gn * ncbu * ncbv, nd = (cull_bricks + 63) / 64 * 64 * gn;
                    float2* gtab = ctab + (size_t)fa * ncbu * ncbv;
                    hipLaunchKernelGGL(coarse_table_kernel, dim3((unsigned)ceil_div(nc, (int64_t)256)), dim3(256), 0, st,
                                       tab + (size_t)fa * nbv * nbu, gn, nbu, nbv, ncbu, ncbv, crange + fa, gtab);
                    hipLaunchKernelGGL(tsdf_brick_kernel, dim3((unsigned)ceil_div(nd, (int64_t)256)), dim3(256), 0, st,
                                       H, W, z0, z1, gn, Hd, Wd, ccam + fa, cg, trunc, gtab, cfree ? 1 : 0, ncbu, ncbv,
                                       per_tile, (int)cull_bricks, bdec + (size_t)fa * cull_bricks);
                }
                unsigned* pl = plist ? plist + (int64_t)nbx * nby * nbz * kCullFrames * h0 : nullptr;
                unsigned* pc = plist ? plist + plist_cap + k : nullptr;
                hipLaunchKernelGGL(tsdf_cull_kernel, dim3((unsigned)(cull_bricks * (h1 - h0))), dim3(1024), 0, st, H,
                                   W, z0, z1, nf, Hd, Wd, ccam, cg, trunc, tab, cfree ? 1 : 0, nbu, nbv, crange, per_tile,
                                   nwf, bdec, (unsigned short*)cmask, (unsigned short*)cfree, pl, pc, tcost, h0,
                                   h1 - h0);
                if (plist)
                    hipLaunchKernelGGL(tsdf_refine_kernel, dim3(refine_wg), dim3(256), 0, st, H, W, z0, z1, nf, Hd, Wd,
                                       pp, kp, cg, trunc, tab, cfree ? 1 : 0, nbu, nbv, crange, nwf, cmask, cfree, pl,
                                       pc);
            }
        } else if (cmask && !ext_table) {
            if (Wd % 4 == 0)
                hipLaunchKernelGGL(depth_blockmax_kernel<true>, dim3(ceil_div(Wd, 1024), nbv, nf), dim3(256), 0, st,
                                   dp, nf, Hd, Wd, nbu, nbv, crange, cbmm);
            else
                hipLaunchKernelGGL(depth_blockmax_kernel<false>, dim3(ceil_div(Wd, 256), nbv, nf), dim3(256), 0, st,
                                   dp, nf, Hd, Wd, nbu, nbv, crange, cbmm);
        }
        if (cmask && groups <= 1) {
            if (bdec) {
                const int64_t nc = (int64_t)nf * ncbu * ncbv, nd = (cull_bricks + 63) / 64 * 64 * nf;
                hipLaunchKernelGGL(coarse_table_kernel, dim3((unsigned)ceil_div(nc, (int64_t)256)), dim3(256), 0, st,
                                   tab, nf, nbu, nbv, ncbu, ncbv, ext_table ? nullptr : crange, ctab);
                hipLaunchKernelGGL(tsdf_brick_kernel, dim3((unsigned)ceil_div(nd, (int64_t)256)), dim3(256), 0, st, H,
                                   W, z0, z1, nf, Hd, Wd, ccam, cg, trunc, ctab, cfree ? 1 : 0, ncbu, ncbv, per_tile,
                                   (int)cull_bricks, bdec);
            }
            hipLaunchKernelGGL(tsdf_cull_kernel, dim3((unsigned)(cull_bricks * nwf * 2)), dim3(1024), 0, st, H,
                               W, z0, z1, nf, Hd, Wd, ccam, cg, trunc, tab, cfree ? 1 : 0, nbu, nbv, crange, per_tile,
                               nwf, bdec, (unsigned short*)cmask, (unsigned short*)cfree, plist, pcount, tcost, 0,
                               2 * nwf);
            if (plist)
                hipLaunchKernelGGL(tsdf_refine_kernel, dim3(refine_wg), dim3(256), 0, st, H, W, z0, z1, nf, Hd, Wd, pp,
                                   kp, cg, trunc, tab, cfree ? 1 : 0, nbu, nbv, crange, nwf, cmask, cfree, plist,
                                   pcount);
        }
        if (stats) {
            if (!cmask) {
                set_error("sfmhip_tsdf_cull_stats: scratch allocation failed");
                rc = SFMHIP_E_HIP;
                break;
            }
            std::vector<unsigned> mc((size_t)nsub * nwf), mf((size_t)nsub * nwf, 0u);
            hipError_t e = hipMemcpyAsync(mc.data(), cmask, mc.size() * sizeof(unsigned), hipMemcpyDeviceToHost, st);
            if (e == hipSuccess && cfree)
                e = hipMemcpyAsync(mf.data(), cfree, mf.size() * sizeof(unsigned), hipMemcpyDeviceToHost, st);
            if (e == hipSuccess) e = hipStreamSynchronize(st);
            if (e != hipSuccess) {
                set_error("sfmhip_tsdf_cull_stats: %s", hipGetErrorString(e));
                rc = SFMHIP_E_HIP;
                break;
            }
            for (size_t i = 0; i < mc.size(); ++i) {
                const int nb = std::min(32, nf - 32 * (int)(i % nwf));
                const unsigned live = nb >= 32 ? ~0u : ((1u << nb) - 1u);
                const int tested = nb, culled = __builtin_popcount(mc[i] & live);
                const int fre = __builtin_popcount(mf[i] & live & ~mc[i]);
                stats[0] += tested;
                stats[1] += culled;
                stats[2] += fre;
                if (layer_stats) {   // slot = tile * kCullSub + wave, tile = (tz * nby + ty) * nbx + tx
                    const int64_t tile = (int64_t)(i / nwf) / kCullSub;
                    int64_t* ls = layer_stats + 3 * (tile / ((int64_t)nbx * nby));
                    ls[0] += tested;
                    ls[1] += culled;
                    ls[2] += fre;
                }
            }
            continue;
        }
        const unsigned* fmask = cfree;
        if (cmask && cfree && free_env >= 3) {
            hipLaunchKernelGGL(tsdf_probe_mask_kernel, dim3((unsigned)ceil_div(nsub * nwf, (int64_t)256)), dim3(256),
                               0, st, cmask, cfree, nsub * nwf, free_env == 4 ? 1 : 0);
            fmask = nullptr;
        }
        if (ord) {   // longest-first workgroup order within each XCD class (bit-identical results)
            hipLaunchKernelGGL(tsdf_order_kernel, dim3(kNumXcd), dim3(256), (size_t)ceil_div((int)grid.x, kNumXcd), st,
                               (int)grid.x, W, H, z0, z1, sb, nf, tcost, ord);
        }
#ifdef SFMHIP_TSDF_PROF
        // probe build: dynamic LDS per fusion workgroup to cap the resident waves (occupancy experiments)
        const size_t prof_lds = (size_t)env_int("SFMHIP_TSDF_PROF_LDS", 0);
#else
        constexpr size_t prof_lds = 0;
#endif
        const unsigned char* skip = nullptr;
        bool joined = true;
        std::unique_lock<std::mutex> side_lock;
        if (hbuf) {   // list the heavy sub-tiles, then fork tsdf_heavy_kernel onto the side stream
            unsigned* hcount = hbuf;
            unsigned* hlist = hbuf + 1;
            unsigned char* hskip = reinterpret_cast<unsigned char*>(hbuf + 1 + nsub);
            (void)hipMemsetAsync(hcount, 0, sizeof(unsigned), st);
            hipLaunchKernelGGL(tsdf_heavy_list_kernel, dim3((unsigned)ceil_div(nsub, (int64_t)256)), dim3(256), 0, st,
                               cmask, fmask, nwf, nf, nsub, (unsigned)heavy_thr, hskip, hlist, hcount);
            // SFMHIP_TSDF_HEAVY_MODE (A/B): 0 side stream, 1 high-priority side stream, 2 before
            // tsdf_kernel on the caller's stream
            const int hmode = env_int("SFMHIP_TSDF_HEAVY_MODE", 1);
            hipStream_t hs = hmode == 2 ? st : hmode == 1 && side->hi ? side->hi : side->s;
            if (hs != st) {
                side_lock = std::unique_lock<std::mutex>(side->mu);
                (void)hipEventRecord(side->fork, st);
                (void)hipStreamWaitEvent(hs, side->fork, 0);
            }
            const int hk = env_int("SFMHIP_TSDF_HEAVY_K", kHvyK);   // frames per producer and round (A/B)
#ifdef SFMHIP_PROBES
            const int hprobe = env_int("SFMHIP_TSDF_HEAVY_PROBE", 0);   // tool-only builds: timing probes
#else
            constexpr int hprobe = 0;
#endif
            auto hkern = hk <= 1 ? tsdf_heavy_kernel<1> : hk == 2 ? tsdf_heavy_kernel<2>
                         : hk >= 8 ? tsdf_heavy_kernel<8> : tsdf_heavy_kernel<kHvyK>;
            hipLaunchKernelGGL(hkern, dim3((unsigned)heavy_wg), dim3(kHvyWaves * 64), 0, hs, T,
                               Wt, D, H, W, z0, z1, dp, nf, Hd, Wd, rec, bb, trunc, cmask, fmask, nwf, free_ts,
                               vox_test ? tab : nullptr, nbu, nbv, easy, hlist, hcount, hprobe);
            if (hs != st) (void)hipEventRecord(side->join, hs);
            joined = hs == st;
            skip = hskip;
        }
        if (swz && pipe)
            hipLaunchKernelGGL((tsdf_kernel<true, true>), grid, dim3(256), prof_lds, st, T, Wt, D, H, W, z0, z1, dp, nf, Hd,
                               Wd, rec, bb, trunc, sb, cmask, fmask, nwf, free_ts, nullptr, nbu, nbv, ord, easy, skip);
        else if (swz)
            hipLaunchKernelGGL(tsdf_kernel<true>, grid, dim3(256), 0, st, T, Wt, D, H, W, z0, z1, dp, nf, Hd, Wd, rec,
                               bb, trunc, sb, cmask, fmask, nwf, free_ts, vox_test ? tab : nullptr, nbu, nbv, ord, easy,
                               skip);
        else
            hipLaunchKernelGGL(tsdf_kernel<false>, grid, dim3(256), 0, st, T, Wt, D, H, W, z0, z1, dp, nf, Hd, Wd, rec,
                               bb, trunc, sb, cmask, fmask, nwf, free_ts, vox_test ? tab : nullptr, nbu, nbv, nullptr, easy,
                               nullptr);
        if (!joined) (void)hipStreamWaitEvent(st, side->join, 0);   // join: the call stays ordered on st
        rc = check_launch("tsdf_kernel");
        if (rc != SFMHIP_OK) break;
    }
    scratch_free(rec, st);
    if (hbuf) scratch_free(hbuf, st);
    if (ord) scratch_free(ord, st);
    if (crange) scratch_free(crange, st);
    if (cmask) scratch_free(cmask, st);
    if (plist) scratch_free(plist, st);
    if (ctab) scratch_free(ctab, st);
    if (cbmm && !ext_table) scratch_free(cbmm, st);
    if (cfree) scratch_free(cfree, st);
    return rc;
}

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
    SFMHIP_REQUIRE(table, "sfmhip_tsdf_integrate_tab: null pointer");
    return tsdf_run(T, Wt, D, H, W, z0, z1, depth, F, Hd, Wd, poses, Kf, bmin, bmax, trunc, stream, nullptr,
                    reinterpret_cast<const float2*>(table));
}

extern "C" int sfmhip_tsdf_block_table(const float* depth, int F, int Hd, int Wd, int f0, int f1, float* table,
                                       void* stream) {
    SFMHIP_REQUIRE(depth && table, "sfmhip_tsdf_block_table: null pointer");
    SFMHIP_REQUIRE(F >= 0 && Hd > 0 && Wd > 0 && 0 <= f0 && f0 <= f1 && f1 <= F,
                   "sfmhip_tsdf_block_table: bad shape or frame range");
    if (f0 == f1) return SFMHIP_OK;
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
    SFMHIP_REQUIRE(grid_vm && bmin && bmax && rays_o && rays_d && z && gt && rgb && sqerr && grad_vm,
                   "sfmhip_render_train: null pointer");
    SFMHIP_REQUIRE(D > 1 && H > 1 && W > 1 && B >= 0 && S >= 1, "sfmhip_render_train: bad shape");
    SFMHIP_REQUIRE(S <= 64 * kTrainChunks, "sfmhip_render_train: S must be <= %d", 64 * kTrainChunks);
    SFMHIP_REQUIRE(mask_mode == 0 || mask_mode == 1, "sfmhip_render_train: mask_mode must be 0 or 1");
    if (B == 0) return SFMHIP_OK;
    const float gscale = (float)(2.0 / (3.0 * (double)B));  // mse_loss mean over B x 3
    hipLaunchKernelGGL(render_train_kernel, dim3(ceil_div(B, 4)), dim3(256), 0, as_stream(stream), grid_vm, D, H,
                       W, make_bounds(bmin, bmax), mask_mode, rays_o, rays_d, z, gt, B, S, gscale, rgb, sqerr,
                       grad_vm, touched);
    return check_launch("render_train_kernel");
}

extern "C" int sfmhip_adam_step(float* param, float* grad, float* exp_avg, float* exp_avg_sq, int64_t n,
                                double lr, double beta1, double beta2, double eps, int64_t step, int zero_grad,
                                void* stream) {
    SFMHIP_REQUIRE(param && grad && exp_avg && exp_avg_sq, "sfmhip_adam_step: null pointer");
    SFMHIP_REQUIRE(n >= 0 && n % 4 == 0, "sfmhip_adam_step: n must be a multiple of 4");
    SFMHIP_REQUIRE(step >= 1, "sfmhip_adam_step: step counts from 1");
    if (n == 0) return SFMHIP_OK;
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
    SFMHIP_REQUIRE(param && grad && exp_avg && exp_avg_sq && flags, "sfmhip_adam_step_flagged: null pointer");
    SFMHIP_REQUIRE(n >= 0 && n % 4 == 0, "sfmhip_adam_step_flagged: n must be a multiple of 4");
    SFMHIP_REQUIRE(flag_shift >= 2 && flag_shift <= 30, "sfmhip_adam_step_flagged: flag_shift must be in [2, 30]");
    SFMHIP_REQUIRE(step >= 1, "sfmhip_adam_step_flagged: step counts from 1");
    if (n == 0) return SFMHIP_OK;
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
    SFMHIP_REQUIRE(rays_o && rays_d && bmin && bmax && t_near && t_far && valid, "sfmhip_ray_aabb: null pointer");
    SFMHIP_REQUIRE(B >= 0, "sfmhip_ray_aabb: B < 0");
    if (B == 0) return SFMHIP_OK;
    hipLaunchKernelGGL(ray_aabb_kernel, dim3(ceil_div(B, 256)), dim3(256), 0, as_stream(stream), rays_o, rays_d, B,
                       make_bounds(bmin, bmax), t_near, t_far, valid);
    return check_launch("ray_aabb_kernel");
}

extern "C" int sfmhip_stratified_samples(const float* t_near, const float* t_far, const float* t_rand, int64_t B,
                                         int S, int perturb, float* z, void* stream) {
    SFMHIP_REQUIRE(t_near && t_far && z && (t_rand || !perturb), "sfmhip_stratified_samples: null pointer");
    SFMHIP_REQUIRE(B >= 0 && S >= 2, "sfmhip_stratified_samples: bad shape");
    if (B == 0) return SFMHIP_OK;
    hipLaunchKernelGGL(stratified_kernel, dim3(ceil_div(B * S, 256)), dim3(256), 0, as_stream(stream), t_near, t_far,
                       t_rand, B, S, perturb, z);
    return check_launch("stratified_kernel");
}

#ifdef SFMHIP_TSDF_PROF
extern "C" int sfmhip_tsdf_prof_read(unsigned long long* host, int n_waves, int clear) {
    const int n = std::min(n_waves, kTsdfProfWaves) * 3;
    if (hipMemcpyFromSymbol(host, HIP_SYMBOL(g_tsdf_prof), (size_t)n * sizeof(unsigned long long)) != hipSuccess)
        return -1;
    if (clear) {
        static std::vector<unsigned long long> z((size_t)kTsdfProfWaves * 3, 0ull);
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_tsdf_prof), z.data(), z.size() * sizeof(unsigned long long)) != hipSuccess)
            return -1;
    }
    return 0;
}
#endif
