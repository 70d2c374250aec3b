// match.hip — M1 brute-force L2 matching + Lowe ratio test on MFMA (int8),
// M2 scipy-compatible vq, and the descriptor prep kernels.
//
// Reference boundary: the matcher call site matching.py:20,122-128 (LightGlue)
// and scipy.cluster.vq.vq at matching.py:27.  Semantics: SURVEY.md §8a M1/M2,
// pinned by oracle/match.py.
//
// Design (DESIGN.md "K1"):
//   * descriptors int8 in HBM, [img][m_pad][d]; squared L2 is exact in int32.
//   * one 512-thread workgroup = one pair x 512 rows of image a; each wave keeps
//     its 64 rows of image a as MFMA B-operands in registers for the whole run.
//   * image b streams through LDS in 128-row blocks (XOR-swizzled, double
//     buffered); v_mfma_i32_32x32x32_i8 computes C'[j][i] = <b_j, a_i>, so a
//     lane owns ONE query row i and sixteen candidate rows j per tile.
//   * fused epilogue, <= 2.5 VALU ops per distance: packed key
//        k = (dot << 8) + keys[j],  keys[j] = (-|b_j|^2 << 7) | (127 - j%128)
//     i.e. k = ((2 dot - |b_j|^2) << 7) | (127 - j%128); larger k = smaller
//     distance, lower index on ties.  top-2 per lane via max3 + med3 + max per
//     two candidates; blocks
//     merge into (best key, best index, second key) with explicit index order.
//   * nothing of the M x N distance matrix is ever written.
#include "common.h"
#include <climits>
#include <cstdlib>

namespace sfmhip {

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));

constexpr int kJB = 128;              // candidate rows per staged LDS block (7-bit local index)

// Byte offset of logical 16-byte chunk c of row r inside a [rows][D] int8 LDS
// tile.  XOR swizzle makes the 16 rows a ds_read_b128 lane group touches land
// on 16 distinct 16-byte bank slots (cdna_hip_programming.md §5.5 T2).
template <int D>
__device__ __forceinline__ int swz_off(int r, int c) {
    constexpr int CPR = D / 16;   // chunks per row
    constexpr int RPB = 256 / D;  // rows per 256-byte bank row
    return r * D + ((c ^ ((r / RPB) % CPR)) << 4);
}

__device__ __forceinline__ int max3i(int a, int b, int c) {
    int r;
    asm("v_max3_i32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
// (the min/max pattern instead of the asm selects v_med3_i32 too, but the compiler then reorders the
// C3 loop badly: 434 vs 101 ms, C2 1.32 vs 1.27 ms; profiles/r5/ab/match_med3_ab_r5.txt)
__device__ __forceinline__ int med3i(int a, int b, int c) {
    int r;
    asm("v_med3_i32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

// ---------------------------------------------------------------------------
// Quantisation f32 -> int8 (padded rows zeroed).  4 elements per thread.
__global__ void quantize_kernel(const float* __restrict__ in, int64_t total, int d, int m_pad,
                                const int32_t* __restrict__ nk, int mode, int8_t* __restrict__ out) {
    const int64_t n4 = total >> 2;
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n4;
         q += (int64_t)gridDim.x * blockDim.x) {
        const int64_t e = q << 2;
        const int64_t row = e / d;
        const int img = (int)(row / m_pad);
        const int r = (int)(row % m_pad);
        const float4 x = *reinterpret_cast<const float4*>(in + e);
        char4 o = make_char4(0, 0, 0, 0);
        if (r < nk[img]) {
            float v[4] = {x.x, x.y, x.z, x.w};
            int qv[4];
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                if (mode == 0) {
                    float rr = fminf(fmaxf(__builtin_rintf(v[t]), 0.f), 255.f);
                    qv[t] = (int)rr - 128;
                } else {
                    float rr = __builtin_rintf(127.f * v[t]);
                    rr = fminf(fmaxf(rr, -127.f), 127.f);
                    qv[t] = (int)rr;
                }
            }
            o = make_char4((signed char)qv[0], (signed char)qv[1], (signed char)qv[2], (signed char)qv[3]);
        }
        *reinterpret_cast<char4*>(out + e) = o;
    }
}

// Row norms and packed candidate keys, one thread per row.
__global__ void prepare_kernel(const int8_t* __restrict__ desc, int n_rows, int m_pad, int d,
                               const int32_t* __restrict__ nk, int32_t* __restrict__ norms,
                               int32_t* __restrict__ keys) {
    const int row = blockIdx.x * blockDim.x + threadIdx.x;
    if (row >= n_rows) return;
    const int img = row / m_pad, r = row % m_pad;
    const int8_t* p = desc + (size_t)row * d;
    int s = 0;
    for (int k = 0; k < d; k += 16) {
        const i32x4 v = *reinterpret_cast<const i32x4*>(p + k);
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            const int x = v[w];
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const int q = (int)(signed char)((x >> (8 * t)) & 0xff);
                s += q * q;
            }
        }
    }
    norms[row] = s;
    const int low = 127 - (r & (kJB - 1));
    keys[row] = (r < nk[img]) ? (-s * 128 + low) : (INT_MIN + low);
}

// ---------------------------------------------------------------------------
// Stage candidate block `blk` of image b into LDS buffer `dst` (XOR-swizzled
// rows) and its 128 packed keys into `kdst`.
//   GLDS=true : LDS-DMA (global_load_lds_dwordx4): the LDS image is lane-linear
//               per wave-instruction, so the swizzle moves to the per-lane SOURCE
//               chunk (cdna_hip_programming.md §5.4 rule 21).  No VGPRs.
//   GLDS=false: register staging (load now, ds_write later).
template <int D, int WAVES>
struct Stager {
    static constexpr int CPR = D / 16;                 // 16-B chunks per row
    static constexpr int RPB = 256 / D;                // rows per 256-B bank row
    static constexpr int TILE = kJB * D;               // bytes per block
    static constexpr int NI = TILE / 1024;             // 1-KiB wave-instructions per block
    static constexpr int PER_WAVE = NI / WAVES;        // per wave
    static constexpr int LDT = TILE / 16 / (64 * WAVES);  // 16-B register loads per thread
    static_assert(NI % WAVES == 0 && LDT >= 1, "block / workgroup mismatch");

    __device__ static void dma(const int8_t* src, const int32_t* ksrc, int8_t* dst, int32_t* kdst, int wave,
                               int lane) {
#pragma unroll
        for (int u = 0; u < PER_WAVE; ++u) {
            const int ins = wave * PER_WAVE + u;
            const int rows_per_ins = 1024 / D;
            const int r0 = ins * rows_per_ins;
            const int r = r0 + lane / CPR;
            const int c = (lane % CPR) ^ ((r / RPB) % CPR);
            __builtin_amdgcn_global_load_lds(
                (__attribute__((address_space(1))) void*)(src + (size_t)r * D + c * 16),
                (__attribute__((address_space(3))) void*)(dst + r0 * D), 16, 0, 0);
        }
        if (wave == WAVES - 1) {  // 128 keys = 2 x (64 lanes x 4 B)
#pragma unroll
            for (int u = 0; u < 2; ++u)
                __builtin_amdgcn_global_load_lds(
                    (__attribute__((address_space(1))) void*)(ksrc + u * 64 + lane),
                    (__attribute__((address_space(3))) void*)(kdst + u * 64), 4, 0, 0);
        }
    }
};

// MFMA shape traits.  MF = output tile edge (32: v_mfma_i32_32x32x32_i8,
// 16: v_mfma_i32_16x16x64_i8).  Both give lane l the 16 bytes of tile row
// (l % MF) for k-chunk group (l / MF), and D/C layouts
//   32x32: col = l % 32, row = (q & 3) + 8 (q >> 2) + 4 (l / 32)   (q < 16)
//   16x16: col = l % 16, row = 4 (l / 16) + q                      (q < 4)
// The k order inside an MFMA is irrelevant here: A and B use the same map.
template <int MF> struct Mfma;
template <> struct Mfma<32> {
    using acc_t = i32x16;
    static constexpr int NREG = 16, KB = 32;   // accumulators per lane, k bytes per MFMA
    __device__ static acc_t run(i32x4 a, i32x4 b, acc_t c) {
        return __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c, 0, 0, 0);
    }
    __device__ static int row(int q, int grp) { return (q & 3) + 8 * (q >> 2) + 4 * grp; }
};
template <> struct Mfma<16> {
    using acc_t = i32x4;
    static constexpr int NREG = 4, KB = 64;
    __device__ static acc_t run(i32x4 a, i32x4 b, acc_t c) {
        return __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c, 0, 0, 0);
    }
    __device__ static int row(int q, int grp) { return 4 * grp + q; }
};

// ---------------------------------------------------------------------------
// Exact float mode (SURVEY.md §7 hard part 1: an int8 candidate pass with an
// exact re-score).  Float descriptors x are matched through their int8
// quantisation q with a rigorous bound on the quantisation residual:
//   x = v(q) + delta,  v(q) = q / 127 (MODE_FLOAT) or q + 128 (MODE_SIFT),
//   | |x_a - x_b| - |v_a - v_b| | <= |delta_a| + |delta_b| =: E    (triangle inequality)
// with |v_a - v_b| = sqrt(D) / s (D the matcher's exact integer distance, s =
// 127 or 1).  The order statistics obey the same bound, so from the matcher's
// (D1, D2) a row is decided without the floats when the bound settles it:
//   reject  if  den^2 * lo(d1) >= num^2 * hi(d2)
//   accept  if  hi(d1) < lo(d2)  (unique winner = the int8 winner)  and  den^2 hi(d1) < num^2 lo(d2)
// where lo/hi bound the reference distance d = sum_k (x_ak - x_bk)^2 as the
// oracle evaluates it in f64 (relative error <= (d + 2) 2^-53 < 1e-13 for
// d <= 256, covered by the 1e-12 widening; the sqrt/scale/sum roundings by the
// 2^-50 operand margins).  Undecided rows are marked -(3 + D2) and settled
// exactly by match_resolve_kernel.
struct CertArgs {
    const double* erow;   // [n_img][m_pad] residual bound per row (desc_residual_kernel)
    const double* eimg;   // [n_img] max over the image's rows
    double inv_s;         // 1/127 (MODE_FLOAT) or 1 (MODE_SIFT)
    int force;            // 1: no row is certified (every row takes the exact path; tests)
};
constexpr int kUndecidedBase = -3;   // matches0 = kUndecidedBase - D2 marks an undecided row
// int16 graphs (m_pad <= 32767: dist.graph_dtype) carry an upper bound of sqrt(D2) instead:
// mark = kUndecidedBase - u, u = ceil(8 sqrt(D2)) <= 32640 for d <= 256 (D2 <= 256 * 255^2),
// so the mark stays above -32768 and the resolve's candidate radius only grows (by < 1/8).
__device__ __forceinline__ int sqrt8_ceil(int d2) {
    const long long t = 64LL * d2;
    int u = (int)ceil(sqrt((double)t));
    while (u > 0 && (long long)(u - 1) * (u - 1) >= t) --u;
    while ((long long)u * u < t) ++u;
    return u;
}
template <typename OutT>
__device__ __forceinline__ int undecided_mark(int d2) {
    if constexpr (sizeof(OutT) == 2) return kUndecidedBase - sqrt8_ceil(d2);
    else return kUndecidedBase - d2;
}
// an upper bound of sqrt(D2) from a mark (the resolve widens it by 1e-12 relative)
template <typename OutT>
__device__ __forceinline__ double mark_sqrt_d2(int mark) {
    if constexpr (sizeof(OutT) == 2) return (double)(kUndecidedBase - mark) * 0.125;
    else return sqrt((double)(kUndecidedBase - mark));
}

// 1 accept, 0 reject, -1 undecided
__device__ __forceinline__ int certify(int d1, int d2, double E, double inv_s, double rn2, double rd2) {
    const double up = 1.0 + 0x1p-50, dn = 1.0 - 0x1p-50;
    const double s1 = sqrt((double)d1) * inv_s, s2 = sqrt((double)d2) * inv_s;
    const double a1 = fmax(s1 * dn - E * up, 0.0), b1 = (s1 + E) * up;
    const double a2 = fmax(s2 * dn - E * up, 0.0), b2 = (s2 + E) * up;
    const double wl = 1.0 - 1e-12, wh = 1.0 + 1e-12;
    const double lo1 = a1 * a1 * wl, hi1 = b1 * b1 * wh, lo2 = a2 * a2 * wl, hi2 = b2 * b2 * wh;
    if (rd2 * lo1 >= rn2 * hi2) return 0;
    if (hi1 < lo2 && rd2 * hi1 < rn2 * lo2) return 1;
    return -1;
}

// One workgroup = one pair x (WAVES * NS * MF) query rows of image a.  Each
// wave owns NS column tiles of MF query rows as resident B-operand fragments
// and streams image b's 128-row blocks from the LDS ring (LDS-DMA filled).
template <int D, int MF, int NS, int WAVES, bool CERT = false, typename OutT = int32_t>
__global__ __launch_bounds__(64 * WAVES, 2) void match_kernel(
    const int8_t* __restrict__ desc, const int32_t* __restrict__ norms,
    const int32_t* __restrict__ keys, const int32_t* __restrict__ nk, int m_pad,
    const int32_t* __restrict__ pairs, int n_iblk, int nwg, long long rn2, long long rd2,
    OutT* __restrict__ m0, int32_t* __restrict__ dist1, int32_t* __restrict__ dist2, CertArgs ca) {
    using S = Stager<D, WAVES>;
    using M = Mfma<MF>;
    using acc_t = typename M::acc_t;
    constexpr int KK = D / M::KB;                   // MFMAs per output tile
    constexpr int CPK = M::KB / 16;                 // 16-B chunks per MFMA k-step
    constexpr int NG = 64 / MF;                     // lane groups sharing a query row
    constexpr int TILE = S::TILE;
    constexpr int NT = 64 * WAVES;
    constexpr int IW = MF * NS;                     // query rows per wave
    constexpr int IB = IW * WAVES;                  // query rows per workgroup
    constexpr int JT = kJB / MF;                    // candidate tiles per block
    static_assert(NS % NG == 0 || NG % NS == 0, "output lane mapping");

    __shared__ __attribute__((aligned(16))) int8_t lds[2 * TILE + 2 * kJB * 4];

    const int wg = xcd_remap(blockIdx.x, nwg);
    const int pair = wg / n_iblk, ib = wg % n_iblk;
    const int a = pairs[2 * pair], b = pairs[2 * pair + 1];
    const int na_rows = nk[a], nb_rows = nk[b];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform: the LDS-DMA M0 addresses stay scalar
    const int grp = lane / MF, lr = lane % MF;
    const int ibase = ib * IB + wave * IW;
    OutT* out_m = m0 + (size_t)pair * m_pad;

    if (ib * IB >= na_rows || nb_rows < 2) {  // block-uniform: nothing to match
        const int iend = min(ib * IB + IB, m_pad);
        for (int i = ib * IB + tid; i < iend; i += NT) {
            out_m[i] = -1;
            if (dist1) dist1[(size_t)pair * m_pad + i] = -1;
            if (dist2) dist2[(size_t)pair * m_pad + i] = -1;
        }
        return;
    }

    const int8_t* bdesc = desc + (size_t)b * m_pad * D;
    const int32_t* bkeys = keys + (size_t)b * m_pad;
    const int nblk = (nb_rows + kJB - 1) / kJB;
    int32_t* kbase = reinterpret_cast<int32_t*>(lds + 2 * TILE);

    S::dma(bdesc, bkeys, lds, kbase, wave, lane);  // block 0 in flight

    // Query rows of image a -> MFMA B-operand fragments, resident for the run.
    i32x4 bq[NS][KK];
#pragma unroll
    for (int s = 0; s < NS; ++s) {
        const int i = min(ibase + s * MF + lr, m_pad - 1);
        const int8_t* rp = desc + ((size_t)a * m_pad + i) * D + grp * 16;
#pragma unroll
        for (int kk = 0; kk < KK; ++kk) bq[s][kk] = *reinterpret_cast<const i32x4*>(rp + kk * M::KB);
    }

    int g1k[NS], g1i[NS], g2k[NS], g1w[NS], g1b[NS];   // best key, its packed word and block; second key
#pragma unroll
    for (int s = 0; s < NS; ++s) { g1k[s] = INT_MIN; g1i[s] = 0; g1w[s] = 127; g1b[s] = 0; g2k[s] = INT_MIN; }

    __syncthreads();

    for (int blk = 0; blk < nblk; ++blk) {
        const int cur = blk & 1;
        if (blk + 1 < nblk)  // next block in flight under the MFMAs
            S::dma(bdesc + (size_t)(blk + 1) * TILE, bkeys + (blk + 1) * kJB, lds + (cur ^ 1) * TILE,
                   kbase + (cur ^ 1) * kJB, wave, lane);
        const int8_t* tl = lds + cur * TILE;
        const int32_t* kl = kbase + cur * kJB;
        int t1[NS], t2[NS];
#pragma unroll
        for (int s = 0; s < NS; ++s) { t1[s] = INT_MIN; t2[s] = INT_MIN; }
#pragma unroll
        for (int jt = 0; jt < JT; ++jt) {
            acc_t acc[NS];
#pragma unroll
            for (int s = 0; s < NS; ++s) acc[s] = acc_t{0};
            const int r = jt * MF + lr;
#pragma unroll
            for (int kk = 0; kk < KK; ++kk) {
                const i32x4 av = *reinterpret_cast<const i32x4*>(tl + swz_off<D>(r, kk * CPK + grp));
#pragma unroll
                for (int s = 0; s < NS; ++s) acc[s] = M::run(av, bq[s][kk], acc[s]);
            }
#pragma unroll
            for (int g = 0; g < M::NREG / 4; ++g) {
                const i32x4 kv = *reinterpret_cast<const i32x4*>(kl + jt * MF + M::row(4 * g, grp));
                // two candidates per step: with t1 >= t2 the top two of {t1, t2, ka, kb} (distinct
                // keys) are max3(t1, ka, kb) and max(t2, med3(t1, ka, kb)) — 5 VALU per 2 distances
                // (2 packings + med3 + max3 + max) instead of 6; the same keys, so the same result
#pragma unroll
                for (int e = 0; e < 4; e += 2) {
#pragma unroll
                    for (int s = 0; s < NS; ++s) {
                        const int ka = acc[s][4 * g + e] * 256 + kv[e];
                        const int kb = acc[s][4 * g + e + 1] * 256 + kv[e + 1];
                        const int m = med3i(t1[s], ka, kb);
                        t1[s] = max3i(t1[s], ka, kb);
                        t2[s] = max(t2[s], m);
                    }
                }
            }
        }
        // merge this block's top-2 into the running (key, packed word + block, second key): the
        // second of {g1, g2, k1, k2} is max3(min(g1, k1), g2, k2); an equal key from a later
        // block never replaces the best (lower index on ties); the index is formed once at the end
        // (d <= 128, where a block has half the MFMAs per merge; at d = 256 the branchy form below
        // measured ~1 % faster: profiles/r3/ab/match_merge_ab_r3as.txt)
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            if constexpr (D <= 128) {
                const int k1 = t1[s] >> 7, k2 = t2[s] >> 7;
                const bool up = k1 > g1k[s];
                g2k[s] = max3i(min(g1k[s], k1), g2k[s], k2);
                g1w[s] = up ? t1[s] : g1w[s];
                g1b[s] = up ? blk : g1b[s];
                g1k[s] = max(g1k[s], k1);
            } else {
                const int k1 = t1[s] >> 7, k2 = t2[s] >> 7, ix = blk * kJB + 127 - (t1[s] & 127);
                if (k1 > g1k[s]) { g2k[s] = max(g1k[s], k2); g1k[s] = k1; g1i[s] = ix; }
                else             { g2k[s] = max(g2k[s], k1); }
            }
        }
        __syncthreads();  // drains this wave's DMA; next block visible to all waves
    }

    if constexpr (D <= 128) {
#pragma unroll
        for (int s = 0; s < NS; ++s) g1i[s] = g1b[s] * kJB + 127 - (g1w[s] & 127);
    }
    // lanes of the NG groups hold the same query row, disjoint candidate rows.
#pragma unroll
    for (int s = 0; s < NS; ++s) {
#pragma unroll
        for (int off = MF; off < 64; off <<= 1) {
            const int ok = __shfl_xor(g1k[s], off), oi = __shfl_xor(g1i[s], off), o2 = __shfl_xor(g2k[s], off);
            const bool mine = (g1k[s] > ok) || (g1k[s] == ok && g1i[s] < oi);
            const int n2 = mine ? max(g2k[s], ok) : max(o2, g1k[s]);
            if (!mine) { g1k[s] = ok; g1i[s] = oi; }
            g2k[s] = n2;
        }
    }
#pragma unroll
    for (int s = 0; s < NS; ++s) {
        if (s % NG != grp % NS) continue;   // one lane group writes each tile
        const int i = ibase + s * MF + lr;
        if (i >= m_pad) continue;
        int res = -1, d1 = -1, d2 = -1;
        if (i < na_rows) {
            const int na = norms[(size_t)a * m_pad + i];
            d1 = na - g1k[s];
            d2 = na - g2k[s];
            if (CERT) {
                const int v = ca.force ? -1
                                       : certify(d1, d2, ca.erow[(size_t)a * m_pad + i] + ca.eimg[b], ca.inv_s,
                                                 (double)rn2, (double)rd2);
                res = v > 0 ? g1i[s] : (v == 0 ? -1 : undecided_mark<OutT>(d2));
            } else if (rd2 * (long long)d1 < rn2 * (long long)d2) {
                res = g1i[s];
            }
        }
        out_m[i] = (OutT)res;
        if (dist1) dist1[(size_t)pair * m_pad + i] = d1;
        if (dist2) dist2[(size_t)pair * m_pad + i] = d2;
    }
}

__global__ void mutual_kernel(int32_t* __restrict__ m0, int32_t* __restrict__ m1, int P, int m_pad) {
    // In place is race-free: an entry is cleared only when it is not mutual, and
    // a reader that sees the cleared value (-1) decides the same way.
    const int64_t total = (int64_t)P * m_pad;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
         e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t base = (e / m_pad) * m_pad;
        const int i = (int)(e - base);
        const int j0 = m0[e];
        const int j1 = m1[e];
        const bool keep0 = j0 >= 0 && m1[base + j0] == i;
        const bool keep1 = j1 >= 0 && m0[base + j1] == i;
        if (j0 >= 0 && !keep0) m0[e] = -1;
        if (j1 >= 0 && !keep1) m1[e] = -1;
    }
}

// ---------------------------------------------------------------------------
// vq: 16 lanes per observation (16 observations per workgroup); the code book
// streams through LDS in chunks of 32 codewords (row stride padded by one f64
// so the 16 codewords a wave reads at one k sit in distinct banks); each lane
// accumulates 2 codewords of the chunk (sum of squared differences in k order,
// one fused multiply-add per term: exact for integer-valued data, within
// rounding of scipy's BLAS-form distance otherwise), then a 16-lane argmin
// with lowest-index tie-break.
constexpr int kVqObsPerBlock = 16;
constexpr int kVqCodesPerChunk = 32;

__global__ __launch_bounds__(256) void vq_kernel(const double* __restrict__ obs, int64_t n_obs,
                                                 const double* __restrict__ code, int n_codes, int d,
                                                 int32_t* __restrict__ codes, double* __restrict__ dist) {
    extern __shared__ double smem[];
    double* sobs = smem;                                   // [16][d]
    double* scode = smem + kVqObsPerBlock * d;             // [64][d + 1]
    const int ld = d + 1;
    const int64_t o0 = (int64_t)blockIdx.x * kVqObsPerBlock;
    for (int t = threadIdx.x; t < kVqObsPerBlock * d; t += blockDim.x) {
        const int64_t o = o0 + t / d;
        sobs[t] = (o < n_obs) ? obs[o * d + (t % d)] : 0.0;
    }
    const int lo = threadIdx.x >> 4, l16 = threadIdx.x & 15;
    const double* x = sobs + lo * d;
    double best = __builtin_inf();
    int bidx = INT_MAX;
    for (int c0 = 0; c0 < n_codes; c0 += kVqCodesPerChunk) {
        const int nc = min(kVqCodesPerChunk, n_codes - c0);
        __syncthreads();
        for (int t = threadIdx.x; t < nc * d; t += blockDim.x) {
            const int r = t / d;
            scode[r * ld + (t - r * d)] = code[(size_t)(c0 + r) * d + (t - r * d)];
        }
        __syncthreads();
        double acc[2] = {0.0, 0.0};
        for (int k = 0; k < d; ++k) {
            const double xv = x[k];
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int r = l16 + 16 * j;
                const double df = xv - scode[r * ld + k];
                acc[j] = __builtin_fma(df, df, acc[j]);
            }
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) {   // codewords ascend with j -> strict < keeps the lowest index
            const int r = l16 + 16 * j;
            if (r < nc && acc[j] < best) { best = acc[j]; bidx = c0 + r; }
        }
    }
#pragma unroll
    for (int off = 8; off >= 1; off >>= 1) {
        const double ob = __shfl_xor(best, off, 16);
        const int oi = __shfl_xor(bidx, off, 16);
        if (ob < best || (ob == best && oi < bidx)) { best = ob; bidx = oi; }
    }
    const int64_t o = o0 + lo;
    if (l16 == 0 && o < n_obs) {
        codes[o] = bidx;
        dist[o] = sqrt(best);
    }
}

// ---------------------------------------------------------------------------
// vq on the f64 matrix cores: argmin_j of |c_j|^2 - 2 x.c_j (= d2 - |x|^2; the
// GEMM form scipy's _vq uses, minus the row constant), with x.c from
// v_mfma_f64_16x16x4_f64.  Exact for integer-valued data (every product and
// partial sum is an integer below 2^53), so integer inputs give scipy's codes
// and distances bit for bit; float inputs agree to rounding.
//
// Layout: one workgroup per CU (8 waves), persistent over 256-observation
// tiles.  The code book passes through LDS in at most a few passes of <=144
// codewords (row stride DP+4 f64, i.e. == 4 mod 32, so the 16 rows x 4 k of an
// MFMA B fragment hit distinct bank pairs).  Each wave keeps the A fragments
// of its 32 observations (2 row tiles x DP/4 f64 per lane) in registers for a
// whole pass; every B fragment read from LDS feeds two MFMAs (two code blocks
// per step, four accumulator chains, measured slower once the difference-form
// epilogue raised register pressure: 1.37 vs 1.33 ms).  Each lane
// tracks the best codeword among j == lane (mod 16) for its 4 C rows, then a
// 16-lane (d2, index) argmin with lowest-index tie-break; passes merge through
// the output arrays (strict <: later passes hold higher indices), and the
// last pass writes the winner's distance recomputed in difference form,
// sqrt(sum (x - c)^2): the GEMM form's cancellation noise would otherwise show
// where x equals its codeword (kmeans singletons), which scipy reports as 0.
typedef double v4d __attribute__((ext_vector_type(4)));
constexpr int kVqmWaves = 8;
constexpr int kVqmObsPerWave = 32;
constexpr int kVqmTile = kVqmWaves * kVqmObsPerWave;   // 256 observations

template <int DP, bool FULL>   // FULL: d == DP (no k padding)
__global__ __launch_bounds__(kVqmWaves * 64) void vq_mfma_kernel(
    const double* __restrict__ obs, int64_t n_obs, const double* __restrict__ code, int n_codes, int d,
    int codes_per_pass, int32_t* __restrict__ codes, double* __restrict__ dist) {
    constexpr int LD = DP + 4;
    constexpr int KS = DP / 4;
    extern __shared__ double smem[];
    double* sc = smem;                                  // [codes_per_pass][LD]
    double* sn = smem + (size_t)codes_per_pass * LD;    // [codes_per_pass] squared norms
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int r16 = lane & 15, kq = lane >> 4;
    const int64_t n_tiles = (n_obs + kVqmTile - 1) / kVqmTile;
    for (int c0 = 0; c0 < n_codes; c0 += codes_per_pass) {
        const int nc = min(codes_per_pass, n_codes - c0);
        const int ncb = (nc + 15) >> 4;
        const bool first = c0 == 0, last = c0 + codes_per_pass >= n_codes;
        __syncthreads();
        for (int t = threadIdx.x; t < ncb * 16 * DP; t += blockDim.x) {
            const int r = t / DP, k = t - r * DP;
            sc[r * LD + k] = (r < nc && (FULL || k < d)) ? code[(size_t)(c0 + r) * d + k] : 0.0;
        }
        __syncthreads();
        for (int r = threadIdx.x; r < ncb * 16; r += blockDim.x) {
            double s = 0.0;
            for (int k = 0; k < DP; ++k) s = __builtin_fma(sc[r * LD + k], sc[r * LD + k], s);
            sn[r] = r < nc ? s : __builtin_inf();    // padded codewords never win
        }
        __syncthreads();
        for (int64_t t = blockIdx.x; t < n_tiles; t += gridDim.x) {
            const int64_t ob = t * kVqmTile + wave * kVqmObsPerWave;
            double a[2][KS];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int64_t o = ob + 16 * h + r16;
                const double* xp = obs + o * d;
#pragma unroll
                for (int s = 0; s < KS; ++s) {
                    const int k = 4 * s + kq;
                    a[h][s] = (o < n_obs && (FULL || k < d)) ? __builtin_nontemporal_load(xp + k) : 0.0;
                }
            }
            double best[2][4];
            int bj[2][4];
#pragma unroll
            for (int h = 0; h < 2; ++h)
#pragma unroll
                for (int g = 0; g < 4; ++g) { best[h][g] = __builtin_inf(); bj[h][g] = INT_MAX; }
            auto epilogue = [&](const v4d& acc0, const v4d& acc1, int j) {
                const double cn = sn[j];
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const double d0 = cn - 2.0 * acc0[g];     // d2 - |x|^2: the row constant drops out
                    const double d1 = cn - 2.0 * acc1[g];
                    if (d0 < best[0][g]) { best[0][g] = d0; bj[0][g] = c0 + j; }
                    if (d1 < best[1][g]) { best[1][g] = d1; bj[1][g] = c0 + j; }
                }
            };
            for (int cb = 0; cb < ncb; ++cb) {
                const int j = cb * 16 + r16;
                const double* bp = sc + j * LD + kq;
                v4d acc0 = {0.0, 0.0, 0.0, 0.0}, acc1 = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
                for (int s = 0; s < KS; ++s) {
                    const double b = bp[4 * s];
                    acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a[0][s], b, acc0, 0, 0, 0);
                    acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a[1][s], b, acc1, 0, 0, 0);
                }
                epilogue(acc0, acc1, j);
            }
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                int win = 0;    // the winning codeword of row r16 (for the last pass's distance)
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    double bv = best[h][g];
                    int bi = bj[h][g];
#pragma unroll
                    for (int off = 8; off >= 1; off >>= 1) {
                        const double ov = __shfl_xor(bv, off, 16);
                        const int oi = __shfl_xor(bi, off, 16);
                        if (ov < bv || (ov == bv && oi < bi)) { bv = ov; bi = oi; }
                    }
                    // all 16 lanes of the kq group now hold row kq + 4g's (d2, index)
                    const int64_t o = ob + 16 * h + kq + 4 * g;
                    if (!first && o < n_obs) {
                        const double prev = dist[o];
                        if (!(bv < prev)) { bv = prev; bi = codes[o]; }
                    }
                    if (!last && r16 == 0 && o < n_obs) {
                        codes[o] = bi;
                        dist[o] = bv;
                    }
                    const int w = __shfl(bi, (r16 & 3) * 16);        // row r16 = (r16 & 3) + 4 (r16 >> 2)
                    if ((r16 >> 2) == g) win = w;
                }
                if (last) {
                    // distance of the winner in difference form, sum (x - c)^2: exact 0 for x == c
                    // (the GEMM form leaves cancellation noise there), otherwise within rounding
                    const int64_t o = ob + 16 * h + r16;
                    const double* cp = code + (size_t)win * d;
                    double part = 0.0;
#pragma unroll
                    for (int s = 0; s < KS; ++s) {
                        const int k = 4 * s + kq;
                        const double df = a[h][s] - ((o < n_obs && (FULL || k < d)) ? cp[k] : 0.0);
                        part = __builtin_fma(df, df, part);
                    }
                    part += __shfl_xor(part, 16);
                    part += __shfl_xor(part, 32);
                    if (kq == 0 && o < n_obs) {
                        codes[o] = win;
                        dist[o] = sqrt(part);
                    }
                }
            }
        }
    }
}


// ---------------------------------------------------------------------------
// vq, d = 128, <= 256 codewords: f32 filter + exact decision (default).
// The f32 MFMA (2x the f64 matrix rate) computes the GEMM-form scores
// s_j = fl32(|c_j|^2) - 2 (x_f . c_f)_f32 with a proven bound on |s_j - (|c_j|^2 - 2 x.c_j)|:
//   input rounding of x and c (2^-24 each), the f32 accumulation of d products
//   (gamma_d), the norm's rounding: eps = 1.01 ((2d + 5) 2^-24 |x| cmax + 2^-24 cmax^2).
// An observation whose best two scores are more than 2 eps apart has a unique
// exact argmin, the best one; its distance is then computed in f64 difference form
// (sqrt(sum (x - c)^2)).  The others (near-ties, exact ties) go to a list that
// vq_exact_kernel settles in f64 difference form over every codeword (lowest index
// on ties) — on integer data every value involved is exact, so codes and distances
// are scipy's bit for bit; on floats the decided argmins are the exact ones.
typedef float f32x4 __attribute__((ext_vector_type(4)));
// Absolute part of the f32 filter's error bound: an input, product or norm that
// lands in (or is flushed from) the f32 subnormal range carries an absolute
// error up to 2^-126 times the other factor, whatever the relative bound says
// (data scaled to ~1e-21).  Per product <= 2^-126 (|c_k| + |x_k| + 1); summed
// over DP products, times 2 in the score, plus the norm:
// <= 2^-126 (2 sqrt(DP) (cmax + |x|) + 2 DP + 4).  Scores closer than that go
// to the exact f64 pass.
__device__ __forceinline__ double vq_eps_abs(int DP, double xn, double cmax) {
    return 0x1p-126 * (2.0 * sqrt((double)DP) * (cmax + xn) + 2.0 * DP + 4.0) * 1.01;
}
typedef double f64x2 __attribute__((ext_vector_type(2)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
constexpr int kVqhWaves = 8;
__device__ __forceinline__ double vq_eps16(int DP, double xn, double cmax) {
    const double u = 0x1p-24;
    return 1.01 * (2.0 * xn * cmax * (0x1.8p-21 + 2.02 * DP * u + 4.0 * u) + 4.0 * u * cmax * cmax +
                   0x1p-24 * sqrt((double)DP) * (xn + cmax) + 2.0 * DP * 0x1p-48) +
           vq_eps_abs(DP, xn, cmax);
}
// k of register j (< 16), half e, for lane group q: pair 8 (j & 7) + 2q + (j >> 3)
__device__ __forceinline__ int vqh_k(int j, int e, int q) { return 16 * (j & 7) + 4 * q + 2 * (j >> 3) + e; }
// lanes l and l ^ 8 of each 16-lane row swap a value (row_ror:8)
__device__ __forceinline__ double vqh_xor8(double v) {
    const int lo = __builtin_amdgcn_mov_dpp((int)__double2loint(v), 0x128, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_mov_dpp((int)__double2hiint(v), 0x128, 0xF, 0xF, false);
    return __hiloint2double(hi, lo);
}
template <int PROBE>   // timing ablations only, never the product: 1 no HBM loads, 2 no winner codeword
                       // loads, 4 no matrix-core pass (every row takes codeword r % n_codes)
__global__ __launch_bounds__(kVqhWaves * 64) void vq_f16s_kernel(const double* __restrict__ obs, int64_t n_obs,
                                                                  const double* __restrict__ code, int n_codes,
                                                                  int32_t* __restrict__ codes,
                                                                  double* __restrict__ dist,
                                                                  unsigned* __restrict__ amb,
                                                                  unsigned* __restrict__ namb) {
    constexpr int DP = 128, KB = 4, KS = 32;
    extern __shared__ f32x4 smh[];
    const int ncb = (n_codes + 15) >> 4;           // codeword blocks of 16
    const int ncp = (ncb + 1) & ~1;                // LDS blocks (even count)
    f16x8* sc = reinterpret_cast<f16x8*>(smh);     // [ncp][KB][2 (hi, lo)][64]
    float* sn = reinterpret_cast<float*>(smh + ncp * KB * 2 * 64);   // [ncp * 16] squared norms
    __shared__ unsigned s_cmax, s_big;
    const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int r16 = lane & 15, kq = lane >> 4;
    const bool b3 = (lane >> 3) & 1;
    if (threadIdx.x == 0) { s_cmax = 0u; s_big = 0u; }
    __syncthreads();
    for (int t = threadIdx.x; t < ncp * KB * 64; t += blockDim.x) {
        const int ln = t & 63, kb = (t >> 6) % KB, cb = t / (KB * 64);
        const int j = cb * 16 + (ln & 15);
        f16x8 hi, lo;
        bool big = false;
#pragma unroll
        for (int e = 0; e < 8; ++e) {   // fragment element e of k-block kb = register 4 kb + e / 2, half e % 2
            const double v = j < n_codes ? code[(size_t)j * DP + vqh_k(4 * kb + (e >> 1), e & 1, ln >> 4)] : 0.0;
            big |= !(fabs(v) < 32768.0);
            const _Float16 h = (_Float16)(float)v;
            hi[e] = h;
            lo[e] = (_Float16)(float)(v - (double)h);
        }
        if (big) s_big = 1u;
        sc[((cb * KB + kb) * 2 + 0) * 64 + ln] = hi;
        sc[((cb * KB + kb) * 2 + 1) * 64 + ln] = lo;
    }
    for (int r = threadIdx.x; r < ncp * 16; r += blockDim.x) {
        double q = 0.0;
        if (r < n_codes)
            for (int k = 0; k < DP; ++k) q = __builtin_fma(code[(size_t)r * DP + k], code[(size_t)r * DP + k], q);
        sn[r] = r < n_codes ? (float)q : __builtin_inff();   // padded codewords never win
        if (r < n_codes) atomicMax(&s_cmax, __float_as_uint((float)sqrt(q) * 1.001f));
    }
    __syncthreads();
    const double cmax = (double)__uint_as_float(s_cmax);
    const bool book_big = s_big != 0u;
    const int64_t n_units = (n_obs + 15) >> 4;
    const int64_t ustep = (int64_t)gridDim.x * kVqhWaves;
    f64x2 nx[KS / 2];   // the next unit's observations (load order), in flight while this unit computes
    auto fetch = [&](int64_t un) {
#pragma unroll
        for (int j = 0; j < KS / 2; ++j) {   // rows (l & 7) + 8 (j >> 3), 128 B each
            const f64x2* xp = reinterpret_cast<const f64x2*>(
                                  obs + min(un * 16 + (lane & 7) + 8 * (j >> 3), n_obs - 1) * DP) +
                              8 * (j & 7) + 2 * kq + b3;
            nx[j] = PROBE == 1 ? f64x2{(double)(lane + un) * 0x1p-10, (double)j * 0x1p-10}
                               : __builtin_nontemporal_load(xp);
        }
    };
    fetch(min((int64_t)blockIdx.x * kVqhWaves + wave, n_units - 1));
    for (int64_t un = (int64_t)blockIdx.x * kVqhWaves + wave; un < n_units; un += ustep) {
        const int64_t o = un * 16 + r16;
        double x[KS];   // x[2 j + e] = row r16, k = vqh_k(j, e, kq) (fragment b, element i: x[8 b + i])
#pragma unroll
        for (int m = 0; m < 8; ++m) {   // load order -> row order: swap registers m / 8 + m across lanes l, l ^ 8
            const f64x2 a0 = nx[m], a1 = nx[8 + m];
            const double s0 = vqh_xor8(b3 ? a0.x : a1.x), s1 = vqh_xor8(b3 ? a0.y : a1.y);
            x[2 * m] = b3 ? s0 : a0.x;
            x[2 * m + 1] = b3 ? s1 : a0.y;
            x[16 + 2 * m] = b3 ? a1.x : s0;
            x[16 + 2 * m + 1] = b3 ? a1.y : s1;
        }
        fetch(min(un + ustep, n_units - 1));
        double xn = 0.0;
        bool big = book_big;
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            xn = __builtin_fma(x[s], x[s], xn);
            big |= !(fabs(x[s]) < 32768.0);
        }
        xn += __shfl_xor(xn, 16);
        xn += __shfl_xor(xn, 32);   // |x|^2 of row r16, in every lane group
        f16x8 ah[KB], al[KB];
#pragma unroll
        for (int b = 0; b < KB; ++b)
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const _Float16 h = (_Float16)(float)x[8 * b + e];
                ah[b][e] = h;
                al[b][e] = (_Float16)(float)(x[8 * b + e] - (double)h);
            }
        float b1[4], b2[4];
        int i1[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) { b1[g] = b2[g] = __builtin_inff(); i1[g] = INT_MAX; }
        auto take = [&](int g, float dd, int j) {   // branch-free top-2 (selects)
            const bool l = dd < b1[g];
            b2[g] = l ? b1[g] : fminf(dd, b2[g]);
            i1[g] = l ? j : i1[g];
            b1[g] = l ? dd : b1[g];
        };
        for (int cb = 0; cb < (PROBE == 4 ? 0 : ncb); cb += 2) {   // two blocks per pass (the odd last one's partner is padding)
            const f16x8* bp = sc + cb * KB * 2 * 64 + lane;
            f32x4 m0 = {0.f, 0.f, 0.f, 0.f}, m1 = m0, c0 = m0, c1 = m0;   // main / correction accumulators
#pragma unroll
            for (int b = 0; b < KB; ++b) {
                const f16x8 c0h = bp[(b * 2 + 0) * 64], c0l = bp[(b * 2 + 1) * 64];
                const f16x8 c1h = bp[((KB + b) * 2 + 0) * 64], c1l = bp[((KB + b) * 2 + 1) * 64];
                m0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[b], c0h, m0, 0, 0, 0);
                m1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[b], c1h, m1, 0, 0, 0);
                c0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[b], c0l, c0, 0, 0, 0);
                c1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[b], c1l, c1, 0, 0, 0);
                c0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[b], c0h, c0, 0, 0, 0);
                c1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[b], c1h, c1, 0, 0, 0);
            }
            const int j0 = cb * 16 + r16;
            const float cn0 = sn[j0], cn1 = sn[j0 + 16];
#pragma unroll
            for (int g = 0; g < 4; ++g) {   // C row 4 kq + g (observation), columns j0, j0 + 16
                take(g, cn0 - 2.f * (m0[g] + c0[g]), j0);
                take(g, cn1 - 2.f * (m1[g] + c1[g]), j0 + 16);
            }
        }
        // the filter's bound for row r16 (every lane group holds |x|^2 of its row r16): formed once
        // per lane, then fetched for the lane's four C rows 4 kq + g
        const double eps_row = vq_eps16(DP, sqrt(xn), cmax);
        int win[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            float v1 = b1[g], v2 = b2[g];
            int x1 = i1[g];
#pragma unroll
            for (int off = 8; off >= 1; off >>= 1) {   // top-2 over the 16 codeword lanes
                const float o1 = __shfl_xor(v1, off, 16), o2 = __shfl_xor(v2, off, 16);
                const int ox = __shfl_xor(x1, off, 16);
                const bool t = o1 < v1 || (o1 == v1 && ox < x1);
                v2 = t ? fminf(v1, o2) : fminf(o1, v2);
                v1 = t ? o1 : v1;
                x1 = t ? ox : x1;
            }
            const double eps = __shfl(eps_row, 4 * kq + g);   // lane 4kq+g: row 4kq+g's bound
            win[g] = PROBE == 4 ? (4 * kq + g) % n_codes : ((double)v2 - (double)v1 > 2.0 * eps) ? x1 : -1;
        }
        int w = -1;   // row r16's verdict: group r16 >> 2, entry r16 & 3
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int t = __shfl(win[g], (r16 >> 2) << 4);
            if ((r16 & 3) == g) w = t;
        }
        // an out-of-range input anywhere in the row (any lane group) decides nothing
        const bool rbig = __shfl_xor((int)big, 16) | __shfl_xor((int)big, 32) | __shfl_xor((int)big, 48) | big;
        if (rbig) w = -1;
        const f64x2* cp = reinterpret_cast<const f64x2*>(code + (size_t)max(w, 0) * DP) + 2 * kq;
        double part = 0.0;
#pragma unroll
        for (int b = 0; b < KB; ++b) {
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const int j = 4 * b + t;   // register j: pair 8 (j & 7) + 2 kq + (j >> 3)
                const f64x2 c = PROBE == 2 ? f64x2{x[2 * j + 1], x[2 * j]} : cp[8 * (j & 7) + (j >> 3)];
                const double d0 = x[2 * j] - c.x, d1 = x[2 * j + 1] - c.y;
                part = __builtin_fma(d0, d0, part);
                part = __builtin_fma(d1, d1, part);
            }
            __builtin_amdgcn_sched_barrier(0);   // 4 codeword loads in flight (VGPRs)
        }
        part += __shfl_xor(part, 16);
        part += __shfl_xor(part, 32);
        if (kq == 0 && o < n_obs) {
            if (w >= 0) {
                codes[o] = w;
                dist[o] = sqrt(part);
            } else {
                amb[atomicAdd(namb, 1u)] = (unsigned)o;
            }
        }
    }
}

// The observations vq_f16s_kernel could not decide: one wave each, every codeword
// in f64 difference form, lowest index on ties.
__global__ __launch_bounds__(256) void vq_exact_kernel(const double* __restrict__ obs, const double* __restrict__ code,
                                                       int n_codes, int d, const unsigned* __restrict__ amb,
                                                       const unsigned* __restrict__ namb, int32_t* __restrict__ codes,
                                                       double* __restrict__ dist) {
    // one wave per listed observation: four 16-lane groups take four codewords at a time, lane
    // k16 of a group the dims 8 k16 .. 8 k16 + 7 of each 128-dim chunk (a codeword row is read as
    // contiguous 1 KB pieces); partial sums of squared differences, then a 16-lane sum.  On
    // integer data every partial sum is exact, so any order gives the same q.
    const int lane = threadIdx.x & 63, cg = lane >> 4, k16 = lane & 15;
    const unsigned n = *namb;
    for (unsigned e = blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); e < n; e += gridDim.x * 4) {
        const int64_t o = amb[e];
        const double* xp = obs + o * d;
        double best = __builtin_inf();
        int bi = INT_MAX;
        for (int j0 = 0; j0 < n_codes; j0 += 4) {
            const int j = j0 + cg;
            const double* cp = code + (size_t)min(j, n_codes - 1) * d;
            double q = 0.0;
            for (int k0 = 8 * k16; k0 < d; k0 += 128) {
#pragma unroll
                for (int t = 0; t < 8; ++t) {
                    const int k = k0 + t;
                    if (k < d) {
                        const double df = xp[k] - cp[k];
                        q = __builtin_fma(df, df, q);
                    }
                }
            }
#pragma unroll
            for (int off = 8; off >= 1; off >>= 1) q += __shfl_xor(q, off, 16);
            if (j < n_codes && q < best) { best = q; bi = j; }   // j increasing per group: the lowest kept
        }
#pragma unroll
        for (int off = 32; off >= 16; off >>= 1) {   // across the four groups, lowest index on ties
            const double ob = __shfl_xor(best, off);
            const int oi = __shfl_xor(bi, off);
            if (ob < best || (ob == best && oi < bi)) { best = ob; bi = oi; }
        }
        if (lane == 0) {
            codes[o] = bi;
            dist[o] = sqrt(best);
        }
    }
}


// ---------------------------------------------------------------------------
// Exact float mode, part 1: per-row residual bounds E_row >= |x - v(q)| (f64,
// outward margins: the sum of squares and sqrt carry <= d 2^-53 relative, the
// computed components <= 2^-52 (|x| + |v|) absolute) and E_img = max per image
// (non-negative doubles order as their bit patterns).  A non-finite row gets
// +inf: every match it takes part in goes to the exact path.  One wave per row.
__global__ __launch_bounds__(256) void desc_residual_kernel(const float* __restrict__ x, const int8_t* __restrict__ q,
                                                            int n_rows, int m_pad, int d, const int32_t* __restrict__ nk,
                                                            int mode, double* __restrict__ erow,
                                                            unsigned long long* __restrict__ eimg) {
    const int lane = threadIdx.x & 63;
    const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (row >= n_rows) return;
    const int img = row / m_pad, r = row % m_pad;
    if (r >= nk[img]) {
        if (lane == 0) erow[row] = 0.0;
        return;
    }
    const float* xr = x + (size_t)row * d;
    const int8_t* qr = q + (size_t)row * d;
    double s2 = 0.0, x2 = 0.0, v2 = 0.0;
    bool finite = true;
    for (int k = lane; k < d; k += 64) {
        const float xf = xr[k];
        const double xv = (double)xf;
        const double v = mode == 0 ? (double)((int)qr[k] + 128) : (double)qr[k] / 127.0;
        const double dl = xv - v;
        s2 = __builtin_fma(dl, dl, s2);
        x2 = __builtin_fma(xv, xv, x2);
        v2 = __builtin_fma(v, v, v2);
        finite = finite && __builtin_isfinite(xf);
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        s2 += __shfl_xor(s2, off);
        x2 += __shfl_xor(x2, off);
        v2 += __shfl_xor(v2, off);
    }
    const bool all_finite = __all(finite);
    if (lane == 0) {
        const double e = all_finite ? sqrt(s2) * (1.0 + 0x1p-40) + 0x1p-50 * (sqrt(x2) + sqrt(v2)) * (1.0 + 0x1p-40)
                                    : __builtin_inf();
        erow[row] = e;
        atomicMax(eimg + img, (unsigned long long)__double_as_longlong(e));
    }
}

// Exact float mode, part 2: every row the certificate left undecided
// (matches0 <= kUndecidedBase, carrying the int8 second-best D2) is settled
// against the f32 descriptors, one wave per row, with the oracle's arithmetic:
//   d(i,j) = sum_k (f64(x_ak) - f64(x_bj,k))^2, one IEEE op per step in k order
//   j1 = lowest index attaining min d, d2 = min over j != j1,
//   accept iff den^2 d1 < num^2 d2 exactly (two-product comparison).
// Candidates: only j whose int8 distance D_j can still reach the top two,
//   sqrt(D_j) <= s E + (sqrt(D2) + s E) (1 + 1e-12)  (E = E_row[a,i] + E_img[b]),
// found with v_dot4 over the int8 rows; the f64 distances are evaluated for
// those (at most kResolveCap, else for every j).  A persistent scan over the
// match graph finds the marked rows (grid-stride over 64-row chunks).
constexpr int kResolveCap = 512;
#ifdef SFMHIP_RESOLVE_PROF
// tool-only build (tools/prof_resolve.py): rows, candidates, rows over the cap, max candidates,
// a histogram by 64 — of the batched resolve
__device__ unsigned long long g_rprof[16];
#endif
// One undecided row e (its mark = kUndecidedBase - D2) by one wave; sxa / sqa / scand: the wave's
// LDS rows.
template <int D, typename OutT>
__device__ __forceinline__ void resolve_row(int64_t e, int mark, const int8_t* __restrict__ q,
                                            const float* __restrict__ x, const int32_t* __restrict__ nk, int m_pad,
                                            const int32_t* __restrict__ pairs, const double* __restrict__ erow,
                                            const double* __restrict__ eimg, double s, double rn2, double rd2,
                                            OutT* __restrict__ m0, unsigned* __restrict__ n_resolved, float* sxa,
                                            int* sqa, int* scand, int lane) {
    constexpr int W4 = D / 4;
    const int pair = (int)(e / m_pad), i = (int)(e % m_pad);
    const int a = pairs[2 * pair], b = pairs[2 * pair + 1], nb = nk[b];
    const size_t arow = (size_t)a * m_pad + i;
    for (int k = lane; k < D; k += 64) sxa[k] = x[arow * D + k];
    for (int w = lane; w < W4; w += 64) sqa[w] = reinterpret_cast<const int*>(q + arow * D)[w];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // |q_a|^2
    int na = 0;
    for (int w = lane; w < W4; w += 64) na = __builtin_amdgcn_sdot4(sqa[w], sqa[w], na, false);
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) na += __shfl_xor(na, off);
    const double se = (erow[arow] + eimg[b]) * s * (1.0 + 1e-12);
    const double bq = (se + (mark_sqrt_d2<OutT>(mark) + se) * (1.0 + 1e-12)) * (1.0 + 1e-12);
    const double tq = floor(bq * bq) + 1.0;   // every j with D_j <= tq may reach the top two
    int ncand = 0;
    for (int j0 = 0; j0 < nb; j0 += 64) {
        const int j = j0 + lane;
        bool in = false;
        if (j < nb) {
            const int4* qb = reinterpret_cast<const int4*>(q + ((size_t)b * m_pad + j) * D);
            int dot = 0, nbn = 0;
#pragma unroll 4
            for (int w4 = 0; w4 < W4 / 4; ++w4) {
                const int4 t = qb[w4];
                const int4 u = reinterpret_cast<const int4*>(sqa)[w4];
                dot = __builtin_amdgcn_sdot4(t.x, u.x, dot, false);
                dot = __builtin_amdgcn_sdot4(t.y, u.y, dot, false);
                dot = __builtin_amdgcn_sdot4(t.z, u.z, dot, false);
                dot = __builtin_amdgcn_sdot4(t.w, u.w, dot, false);
                nbn = __builtin_amdgcn_sdot4(t.x, t.x, nbn, false);
                nbn = __builtin_amdgcn_sdot4(t.y, t.y, nbn, false);
                nbn = __builtin_amdgcn_sdot4(t.z, t.z, nbn, false);
                nbn = __builtin_amdgcn_sdot4(t.w, t.w, nbn, false);
            }
            in = (double)((long long)na + nbn - 2LL * dot) <= tq;
        }
        const unsigned long long cb = __ballot(in);
        const int pos = ncand + __popcll(cb & ((1ull << lane) - 1ull));
        if (in && pos < kResolveCap) scand[pos] = j;
        ncand += __popcll(cb);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const bool every = ncand > kResolveCap;
    const int nc = every ? nb : ncand;
    double v1 = __builtin_inf(), v2 = __builtin_inf();
    int j1 = INT_MAX;
    for (int t = lane; t < nc; t += 64) {   // ascending j per lane
        const int j = every ? t : scand[t];
        const float4* xb = reinterpret_cast<const float4*>(x + ((size_t)b * m_pad + j) * D);
        double acc = 0.0;
        for (int k4 = 0; k4 < D / 4; ++k4) {
            const float4 xv = xb[k4];
            double df;
            df = (double)sxa[4 * k4] - (double)xv.x;
            acc = acc + df * df;
            df = (double)sxa[4 * k4 + 1] - (double)xv.y;
            acc = acc + df * df;
            df = (double)sxa[4 * k4 + 2] - (double)xv.z;
            acc = acc + df * df;
            df = (double)sxa[4 * k4 + 3] - (double)xv.w;
            acc = acc + df * df;
        }
        if (acc < v1) { v2 = v1; v1 = acc; j1 = j; }
        else if (acc < v2) v2 = acc;
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const double o1 = __shfl_xor(v1, off), o2 = __shfl_xor(v2, off);
        const int oj = __shfl_xor(j1, off);
        const bool mine = v1 < o1 || (v1 == o1 && j1 < oj);
        const double n2 = mine ? fmin(v2, o1) : fmin(o2, v1);
        if (!mine) { v1 = o1; j1 = oj; }
        v2 = n2;
    }
    // den^2 d1 < num^2 d2, exactly: (p, e) two-products compare lexicographically (RN is monotone)
    const double p1 = rd2 * v1, e1 = __builtin_fma(rd2, v1, -p1);
    const double p2 = rn2 * v2, e2 = __builtin_fma(rn2, v2, -p2);
    const bool acc_ok = p1 < p2 || (p1 == p2 && e1 < e2);
    if (lane == 0) {
        m0[e] = (OutT)(acc_ok ? j1 : -1);
        if (n_resolved) atomicAdd(n_resolved, 1u);
    }
    __builtin_amdgcn_wave_barrier();   // LDS rows reused by the next marked row
}

template <int D, typename OutT>
__global__ __launch_bounds__(256) void match_resolve_kernel(const int8_t* __restrict__ q, const float* __restrict__ x,
                                                            const int32_t* __restrict__ nk, int m_pad,
                                                            const int32_t* __restrict__ pairs, int P,
                                                            const double* __restrict__ erow,
                                                            const double* __restrict__ eimg, double s, double rn2,
                                                            double rd2, OutT* __restrict__ m0,
                                                            unsigned* __restrict__ n_resolved,
                                                            const unsigned* __restrict__ overflow = nullptr) {
    if (overflow && *overflow == 0u) return;   // the bucketed pass below settled every row
    constexpr int W4 = D / 4;
    __shared__ float sxa[4][D];
    __shared__ __attribute__((aligned(16))) int sqa[4][W4];
    __shared__ int scand[4][kResolveCap];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t total = (int64_t)P * m_pad;
    const int64_t nchunk = (total + 63) >> 6;
    for (int64_t c = (int64_t)blockIdx.x * 4 + wave; c < nchunk; c += (int64_t)gridDim.x * 4) {
        const int64_t e0 = c << 6;
        const int v = (e0 + lane < total) ? (int)m0[e0 + lane] : -1;
        unsigned long long bal = __ballot(v <= kUndecidedBase);
        while (bal) {
            const int l = __builtin_ctzll(bal);
            bal &= bal - 1;
            resolve_row<D, OutT>(e0 + l, __shfl(v, l), q, x, nk, m_pad, pairs, erow, eimg, s, rn2, rd2, m0, n_resolved,
                           sxa[wave], sqa[wave], scand[wave], lane);
        }
    }
}

// Default (round 5): the undecided rows are collected per image b (one scan of the match graph
// into buckets of up to kResolveBucket rows), laid out XCD-major (images b = x, x + 8, ... on XCD x)
// and settled kResolveRows at a time per workgroup (match_resolve_batched_kernel), so image b's int8
// rows — the candidate prefilter reads all of them, 1 MB per row at C3 — are read once per batch.
// A bucket overflow sets *overflow and match_resolve_kernel's graph scan settles every row instead.
constexpr int kResolveBucket = 4096;
template <typename OutT>
__global__ __launch_bounds__(256) void resolve_collect_kernel(const OutT* __restrict__ m0, int64_t total, int m_pad,
                                                              const int32_t* __restrict__ pairs,
                                                              unsigned* __restrict__ cnt, int64_t* __restrict__ list,
                                                              unsigned* __restrict__ overflow) {
    auto take = [&](int64_t e) {
        const int b = pairs[2 * (int)(e / m_pad) + 1];
        const unsigned slot = atomicAdd(cnt + b, 1u);
        if (slot < (unsigned)kResolveBucket) list[(size_t)b * kResolveBucket + slot] = e;
        else atomicOr(overflow, 1u);
    };
    constexpr int PER = 16 / sizeof(OutT);   // entries per 16-B load (m_pad % 128 == 0: whole loads)
    const int64_t n4 = total / PER;
    const int4* m4 = reinterpret_cast<const int4*>(m0);
    for (int64_t e4 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e4 < n4; e4 += (int64_t)gridDim.x * blockDim.x) {
        const int4 v = m4[e4];
        if constexpr (sizeof(OutT) == 2) {
            // 8 int16 entries: a mark is <= -3, i.e. in 0x8000..0xFFFD as an unsigned half
            const unsigned w[4] = {(unsigned)v.x, (unsigned)v.y, (unsigned)v.z, (unsigned)v.w};
            bool any = false;
#pragma unroll
            for (int h = 0; h < 4; ++h) {
                any |= (short)(w[h] & 0xFFFFu) <= kUndecidedBase;
                any |= (short)(w[h] >> 16) <= kUndecidedBase;
            }
            if (!any) continue;
#pragma unroll
            for (int h = 0; h < 4; ++h) {
                if ((short)(w[h] & 0xFFFFu) <= kUndecidedBase) take(PER * e4 + 2 * h);
                if ((short)(w[h] >> 16) <= kUndecidedBase) take(PER * e4 + 2 * h + 1);
            }
        } else {
            if (min(min(v.x, v.y), min(v.z, v.w)) > kUndecidedBase) continue;
            if (v.x <= kUndecidedBase) take(4 * e4);
            if (v.y <= kUndecidedBase) take(4 * e4 + 1);
            if (v.z <= kUndecidedBase) take(4 * e4 + 2);
            if (v.w <= kUndecidedBase) take(4 * e4 + 3);
        }
    }
}

// The buckets flattened XCD-major (images b = x, x + 8, ... for x = 0..7, each image's rows
// together), with each XCD's range [xr[x], xr[x] + xr[8 + x]): resolve_offsets_kernel (one
// workgroup: position p of that order holds image b(p); an LDS scan over the positions, 1024 at a
// time, gives each image's first flat row and first item), then resolve_flatten_kernel (one entry
// per thread, its image found by a binary search over the offsets in that order).
constexpr int kResolveRows = 16;   // rows of one image settled together (resolve_batched_kernel)
__global__ __launch_bounds__(1024) void resolve_offsets_kernel(
    const unsigned* __restrict__ cnt, int n_img, unsigned* __restrict__ off,
    unsigned* __restrict__ okey /* [n_img + 1]: offsets in XCD-major order */, int* __restrict__ oimg,
    unsigned* __restrict__ xr, int* __restrict__ items /* [3][n_img * (kResolveBucket / kResolveRows + 1)] */,
    unsigned* __restrict__ ir /* [16]: per XCD item start, count */, const unsigned* __restrict__ overflow) {
    __shared__ unsigned sr[1024], sk[1024];
    __shared__ unsigned sxs[9], sks[9];
    if (*overflow != 0u) return;
    const int tid = threadIdx.x;
    const int cap = n_img * (kResolveBucket / kResolveRows + 1);
    int ps[9];   // first position of XCD x (ps[8] = n_img)
    ps[0] = 0;
#pragma unroll
    for (int x = 0; x < 8; ++x) ps[x + 1] = ps[x] + (x < n_img ? (n_img - x + 7) / 8 : 0);
    unsigned carry_r = 0, carry_k = 0;
    for (int base = 0; base < n_img; base += 1024) {
        const int p = base + tid;
        int b = -1;
        unsigned cb = 0, ni = 0;
        if (p < n_img) {
            int x = 0;
#pragma unroll
            for (int y = 1; y < 8; ++y) x += (p >= ps[y]) ? 1 : 0;
            b = x + 8 * (p - ps[x]);
            cb = min(cnt[b], (unsigned)kResolveBucket);
            ni = (cb + kResolveRows - 1) / kResolveRows;
        }
        sr[tid] = cb;
        sk[tid] = ni;
        __syncthreads();
        for (int d = 1; d < 1024; d <<= 1) {   // inclusive scan
            const unsigned vr = tid >= d ? sr[tid - d] : 0u, vk = tid >= d ? sk[tid - d] : 0u;
            __syncthreads();
            sr[tid] += vr;
            sk[tid] += vk;
            __syncthreads();
        }
        const unsigned run = carry_r + sr[tid] - cb, k0 = carry_k + sk[tid] - ni;
        if (b >= 0) {
            off[b] = run;
            okey[p] = run;
            oimg[p] = b;
#pragma unroll
            for (int x = 0; x < 8; ++x)
                if (p == ps[x]) {
                    sxs[x] = run;
                    sks[x] = k0;
                }
            for (unsigned i = 0; i < ni; ++i) {
                items[k0 + i] = (int)(run + i * kResolveRows);                          // first flat row
                items[cap + k0 + i] = (int)min((unsigned)kResolveRows, cb - i * kResolveRows);   // rows
                items[2 * cap + k0 + i] = b;
            }
        }
        carry_r += sr[1023];
        carry_k += sk[1023];
        __syncthreads();
    }
    if (tid < 9) {   // XCDs without images (n_img < 8) start at the end
        if (tid == 8 || ps[tid] >= n_img) {
            sxs[tid] = carry_r;
            sks[tid] = carry_k;
        }
    }
    __syncthreads();
    if (tid < 8) {
        xr[tid] = sxs[tid];
        xr[8 + tid] = sxs[tid + 1] - sxs[tid];
        ir[tid] = sks[tid];
        ir[8 + tid] = sks[tid + 1] - sks[tid];
    }
    if (tid == 0) okey[n_img] = carry_r;
}
__global__ __launch_bounds__(256) void resolve_flatten_kernel(const unsigned* __restrict__ okey,
                                                              const int* __restrict__ oimg, int n_img,
                                                              const int64_t* __restrict__ list,
                                                              int64_t* __restrict__ flat,
                                                              const unsigned* __restrict__ overflow) {
    if (*overflow != 0u) return;
    const unsigned total = okey[n_img];
    for (unsigned t = blockIdx.x * blockDim.x + threadIdx.x; t < total; t += gridDim.x * blockDim.x) {
        int lo = 0, hi = n_img - 1;   // the last position with okey <= t
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (okey[mid] <= t) lo = mid;
            else hi = mid - 1;
        }
        flat[t] = list[(size_t)oimg[lo] * kResolveBucket + (t - okey[lo])];
    }
}

// Up to kResolveRows undecided rows of one image b per workgroup (the items of the XCD-major
// order above, dealt to the XCD's own workgroups): the query rows staged in LDS, image b's int8
// rows read ONCE for the whole batch by the candidate prefilter (16 candidates x the batch's 16
// rows per MFMA chain, four tiles' loads in flight per wave: 0.41 -> 0.30 ms per C3 call against
// v_dot4 over the candidates, profiles/r5/ab/resolve_mfma_prefilter_ab_r5.txt), then the f64
// distances of each row's candidates by one wave per row (any order: a tie-aware top two, lowest
// index on equal distances) — resolve_row's result.  At C3 a row keeps ~2 candidates, so the
// prefilter (4096 int8 rows of image b per row in the per-row form) is most of the work.
template <int D, typename OutT>
__global__ __launch_bounds__(256) void match_resolve_batched_kernel(
    const int8_t* __restrict__ q /* the matcher's (shifted) int8 operands */, const int32_t* __restrict__ norms,
    const float* __restrict__ x, const int32_t* __restrict__ nk, int m_pad,
    const int32_t* __restrict__ pairs, int n_img, const double* __restrict__ erow, const double* __restrict__ eimg,
    double s, double rn2, double rd2, OutT* __restrict__ m0, unsigned* __restrict__ n_resolved,
    const int64_t* __restrict__ flat, const int* __restrict__ items, const unsigned* __restrict__ ir,
    const unsigned* __restrict__ overflow) {
    constexpr int W4 = D / 4, R = kResolveRows;
    __shared__ __attribute__((aligned(16))) int sqa[R][W4];
    __shared__ float sxa[R][D];
    __shared__ int scand[R][kResolveCap];
    __shared__ int sncand[R], sna[R], sccd[R];
    __shared__ double stq[R];
    __shared__ int64_t se_[R];
    if (*overflow != 0u) return;   // match_resolve_kernel takes every row
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int cap = n_img * (kResolveBucket / kResolveRows + 1);
    const int xcd = blockIdx.x % 8, nx = (gridDim.x + 7 - xcd) / 8;
    const unsigned ib = ir[xcd], in = ir[8 + xcd];
    for (unsigned k = blockIdx.x / 8; k < in; k += nx) {
        const int f0 = items[ib + k], nr = items[cap + ib + k], b = items[2 * cap + ib + k];
        const int nb = nk[b];
        for (int t = tid; t < nr * W4; t += 256) {
            const int r = t / W4, w = t % W4;
            const int64_t e = flat[f0 + r];
            const size_t arow = (size_t)pairs[2 * (int)(e / m_pad)] * m_pad + (int)(e % m_pad);
            sqa[r][w] = reinterpret_cast<const int*>(q + arow * D)[w];
        }
        for (int t = tid; t < nr * D; t += 256) {
            const int r = t / D, kk = t % D;
            const int64_t e = flat[f0 + r];
            const size_t arow = (size_t)pairs[2 * (int)(e / m_pad)] * m_pad + (int)(e % m_pad);
            sxa[r][kk] = x[arow * D + kk];
        }
        if (tid < R) sncand[tid] = 0;
        __syncthreads();
        for (int r = wave; r < nr; r += 4) {
            int na = 0;
            for (int w = lane; w < W4; w += 64) na = __builtin_amdgcn_sdot4(sqa[r][w], sqa[r][w], na, false);
#pragma unroll
            for (int off = 32; off >= 1; off >>= 1) na += __shfl_xor(na, off);
            if (lane == 0) {
                const int64_t e = flat[f0 + r];
                const size_t arow = (size_t)pairs[2 * (int)(e / m_pad)] * m_pad + (int)(e % m_pad);
                const double se = (erow[arow] + eimg[b]) * s * (1.0 + 1e-12);
                const double bq = (se + (mark_sqrt_d2<OutT>((int)m0[e]) + se) * (1.0 + 1e-12)) * (1.0 + 1e-12);
                stq[r] = floor(bq * bq) + 1.0;   // every j with D_j <= tq may reach the top two
                sna[r] = na;
                sccd[r] = norms[arow] - na;   // the matcher's norms carry c^2 d of its operand shift c
                se_[r] = e;
            }
        }
        __syncthreads();
        {   // the prefilter on the matrix cores: <q_j, q_r> for 16 candidates j x the batch's 16 rows r
            // per v_mfma_i32_16x16x64_i8 chain (the matcher's operands, shifted by c: D_j is
            // shift-invariant, |q_j|^2 = norms_j - c^2 d, and the int32 dots are exact, so the
            // candidate set is the one the per-row form tests)
            using M16 = Mfma<16>;
            constexpr int KK = D / M16::KB;
            const int lr = lane & 15, grp = lane >> 4;   // lane: row lr of the batch, candidates 4 grp + e
            i32x4 bqv[KK];
#pragma unroll
            for (int kk = 0; kk < KK; ++kk) bqv[kk] = *reinterpret_cast<const i32x4*>(&sqa[lr][kk * 16 + grp * 4]);
            const bool live = lr < nr;
            const long long na_r = live ? (long long)sna[lr] - sccd[lr] : 0;   // |q_r|^2 - c^2 d
            const double tq_r = live ? stq[lr] : -1.0;
            const size_t bbase = (size_t)b * m_pad;
            constexpr int TG = 4;   // 16-candidate tiles per wave step, their loads issued together
            for (int jg = wave * 16; jg < nb; jg += 64 * TG) {
                i32x4 av[TG][KK], nv[TG];
#pragma unroll
                for (int t = 0; t < TG; ++t) {
                    const int j0 = min(jg + 64 * t, m_pad - 16);   // whole rows (m_pad % 128 == 0)
                    const int8_t* rp = q + (bbase + j0 + lr) * D + grp * 16;
#pragma unroll
                    for (int kk = 0; kk < KK; ++kk) av[t][kk] = *reinterpret_cast<const i32x4*>(rp + kk * M16::KB);
                    nv[t] = *reinterpret_cast<const i32x4*>(norms + bbase + j0 + 4 * grp);   // norms of the 4 candidates
                }
#pragma unroll
                for (int t = 0; t < TG; ++t) {
                    const int j0 = jg + 64 * t;
                    i32x4 acc = {0, 0, 0, 0};
#pragma unroll
                    for (int kk = 0; kk < KK; ++kk) acc = M16::run(av[t][kk], bqv[kk], acc);
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const int j = j0 + 4 * grp + e;
                        if (live && j < nb && (double)(na_r + nv[t][e] - 2LL * acc[e]) <= tq_r) {
                            const int pos = atomicAdd(&sncand[lr], 1);
                            if (pos < kResolveCap) scand[lr][pos] = j;
                        }
                    }
                }
            }
        }
        __syncthreads();
        for (int r = wave; r < nr; r += 4) {   // f64 distances of the row's candidates
            const int ncand = sncand[r];
            const bool every = ncand > kResolveCap;
#ifdef SFMHIP_RESOLVE_PROF
            if (lane == 0) {
                atomicAdd(&g_rprof[0], 1ull);
                atomicAdd(&g_rprof[1], (unsigned long long)ncand);
                if (every) atomicAdd(&g_rprof[2], 1ull);
                atomicMax(&g_rprof[3], (unsigned long long)ncand);
                atomicAdd(&g_rprof[4 + min(ncand / 64, 11)], 1ull);
            }
#endif
            const int nc = every ? nb : ncand;
            double v1 = __builtin_inf(), v2 = __builtin_inf();
            int j1 = INT_MAX;
            for (int t = lane; t < nc; t += 64) {
                const int j = every ? t : scand[r][t];
                const float4* xb = reinterpret_cast<const float4*>(x + ((size_t)b * m_pad + j) * D);
                double acc = 0.0;
                for (int k4 = 0; k4 < D / 4; ++k4) {
                    const float4 xv = xb[k4];
                    double df;
                    df = (double)sxa[r][4 * k4] - (double)xv.x;
                    acc = acc + df * df;
                    df = (double)sxa[r][4 * k4 + 1] - (double)xv.y;
                    acc = acc + df * df;
                    df = (double)sxa[r][4 * k4 + 2] - (double)xv.z;
                    acc = acc + df * df;
                    df = (double)sxa[r][4 * k4 + 3] - (double)xv.w;
                    acc = acc + df * df;
                }
                if (acc < v1 || (acc == v1 && j < j1)) { v2 = v1; v1 = acc; j1 = j; }
                else if (acc < v2) v2 = acc;
            }
#pragma unroll
            for (int off = 32; off >= 1; off >>= 1) {
                const double o1 = __shfl_xor(v1, off), o2 = __shfl_xor(v2, off);
                const int oj = __shfl_xor(j1, off);
                const bool mine = v1 < o1 || (v1 == o1 && j1 < oj);
                const double n2 = mine ? fmin(v2, o1) : fmin(o2, v1);
                if (!mine) { v1 = o1; j1 = oj; }
                v2 = n2;
            }
            const double p1 = rd2 * v1, e1 = __builtin_fma(rd2, v1, -p1);
            const double p2 = rn2 * v2, e2 = __builtin_fma(rn2, v2, -p2);
            const bool acc_ok = p1 < p2 || (p1 == p2 && e1 < e2);
            if (lane == 0) {
                m0[se_[r]] = (OutT)(acc_ok ? j1 : -1);
                if (n_resolved) atomicAdd(n_resolved, 1u);
            }
        }
        __syncthreads();   // the batch's LDS is reused by the next item
    }
}

}  // namespace sfmhip

using namespace sfmhip;

#ifdef SFMHIP_RESOLVE_PROF
extern "C" int sfmhip_debug_resolve_prof(unsigned long long* out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(sfmhip::g_rprof), sizeof(unsigned long long) * 16) == hipSuccess ? 0 : -2;
}
#endif

extern "C" int sfmhip_desc_quantize(const float* in, int n_img, int m_pad, int d,
                                    const int32_t* n_kpts, int mode, int8_t* out, void* stream) {
    SFMHIP_REQUIRE(in && out && n_kpts, "sfmhip_desc_quantize: null pointer");
    SFMHIP_REQUIRE(n_img > 0 && m_pad > 0 && d > 0 && d % 4 == 0, "sfmhip_desc_quantize: bad shape");
    SFMHIP_REQUIRE(mode == 0 || mode == 1, "sfmhip_desc_quantize: mode must be 0 or 1");
    const int64_t total = (int64_t)n_img * m_pad * d;
    const int64_t n4 = total / 4;
    const int grid = (int)std::min<int64_t>((n4 + 255) / 256, 4096);
    hipLaunchKernelGGL(quantize_kernel, dim3(grid), dim3(256), 0, as_stream(stream), in, total, d,
                       m_pad, n_kpts, mode, out);
    return check_launch("quantize_kernel");
}

extern "C" int sfmhip_desc_prepare(const int8_t* desc, int n_img, int m_pad, int d,
                                   const int32_t* n_kpts, int32_t* norms, int32_t* keys, void* stream) {
    SFMHIP_REQUIRE(desc && n_kpts && norms && keys, "sfmhip_desc_prepare: null pointer");
    SFMHIP_REQUIRE(n_img > 0 && m_pad > 0 && d > 0 && d % 16 == 0, "sfmhip_desc_prepare: bad shape");
    const int rows = n_img * m_pad;
    hipLaunchKernelGGL(prepare_kernel, dim3(ceil_div(rows, 256)), dim3(256), 0, as_stream(stream),
                       desc, rows, m_pad, d, n_kpts, norms, keys);
    return check_launch("prepare_kernel");
}

// Shifted copy for the matcher (sfmhip_desc_prepare_shifted): q' = q + c on valid
// rows (zero on padding rows), with norms and keys adjusted so that the matcher,
// unchanged, returns the distances of the UNSHIFTED descriptors, exactly:
//   2 q'_a.q'_b = 2 q_a.q_b + 2c S_a + 2c S_b + 2c^2 d         (S = sum of q)
//   key'_b  = -(|q_b|^2 + 2c S_b)            (packed with the local index as before)
//   norm'_a = |q_a|^2 + 2c S_a + 2c^2 d      so norm'_a - (2 q'_a.q'_b + key'_b) = |q_a - q_b|^2.
// Same argmin, same ties, same ratio test: only the operand bytes change.  With
// c = 64 and |q| <= 64 the operands are non-negative (sign bits constant), which
// lowers the MFMA array's switching power: the clock-limited int8 rate is ~6 %
// higher (tools/mfma_peak: 2,985 -> 3,176 TOPS with the epilogue).
__global__ void prepare_shifted_kernel(const int8_t* __restrict__ desc, int n_rows, int m_pad, int d,
                                       const int32_t* __restrict__ nk, int c, int8_t* __restrict__ out,
                                       int32_t* __restrict__ norms, int32_t* __restrict__ keys) {
    const int row = blockIdx.x * blockDim.x + threadIdx.x;
    if (row >= n_rows) return;
    const int img = row / m_pad, r = row % m_pad;
    const bool valid = r < nk[img];
    const int8_t* p = desc + (size_t)row * d;
    int8_t* o = out + (size_t)row * d;
    int s = 0, sum = 0;
    for (int k = 0; k < d; k += 16) {
        const i32x4 v = *reinterpret_cast<const i32x4*>(p + k);
        i32x4 w;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            const int x = v[e];
            unsigned packed = 0;
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const int q = (int)(signed char)((x >> (8 * t)) & 0xff);
                s += q * q;
                sum += q;
                packed |= (unsigned)((valid ? q + c : 0) & 0xff) << (8 * t);
            }
            w[e] = (int)packed;
        }
        *reinterpret_cast<i32x4*>(o + k) = w;
    }
    norms[row] = s + 2 * c * sum + 2 * c * c * d;
    const int low = 127 - (r & (kJB - 1));
    keys[row] = valid ? (-(s + 2 * c * sum) * 128 + low) : (INT_MIN + low);
}

extern "C" int sfmhip_desc_prepare_shifted(const int8_t* desc, int n_img, int m_pad, int d, const int32_t* n_kpts,
                                           int shift, int8_t* desc_shifted, int32_t* norms, int32_t* keys,
                                           void* stream) {
    SFMHIP_REQUIRE(desc && n_kpts && desc_shifted && norms && keys, "sfmhip_desc_prepare_shifted: null pointer");
    SFMHIP_REQUIRE(n_img > 0 && m_pad > 0 && d > 0 && d % 16 == 0 && d <= 256,
                   "sfmhip_desc_prepare_shifted: bad shape");
    SFMHIP_REQUIRE(shift >= 0 && shift <= 127, "sfmhip_desc_prepare_shifted: shift must be in [0, 127]");
    const int rows = n_img * m_pad;
    hipLaunchKernelGGL(prepare_shifted_kernel, dim3(ceil_div(rows, 256)), dim3(256), 0, as_stream(stream), desc,
                       rows, m_pad, d, n_kpts, shift, desc_shifted, norms, keys);
    return check_launch("prepare_shifted_kernel");
}

template <typename OutT>
static int match_pairs_impl(const int8_t* desc, const int32_t* norms, const int32_t* keys,
                            const int32_t* n_kpts, int n_img, int m_pad, int d,
                            const int32_t* pairs, int P, int ratio_num, int ratio_den,
                            OutT* matches0, int32_t* dist1, int32_t* dist2, void* stream) {
    SFMHIP_REQUIRE(n_img > 0 && P >= 0, "sfmhip_match_pairs: bad counts");
    SFMHIP_REQUIRE(m_pad > 0 && m_pad % kJB == 0, "sfmhip_match_pairs: m_pad must be a positive multiple of 128");
    SFMHIP_REQUIRE(ratio_num > 0 && ratio_den > 0 && ratio_num <= 65535 && ratio_den <= 65535,
                   "sfmhip_match_pairs: ratio must be a positive fraction");
    if (P == 0) return SFMHIP_OK;
    SFMHIP_REQUIRE(desc && norms && keys && n_kpts && pairs && matches0,
                   "sfmhip_match_pairs: null pointer");
    // 16x16x64 int8 MFMA tiles, 4 per wave, 4 waves per workgroup: 256 query rows per workgroup
    // (32x32 tiles, 8 tiles per wave and 8-wave workgroups measured slower: DESIGN.md K1)
    const int n_iblk = ceil_div(m_pad, 256);
    const int64_t nwg64 = (int64_t)P * n_iblk;
    SFMHIP_REQUIRE(nwg64 < INT_MAX, "sfmhip_match_pairs: too many pairs for one launch");
    const int nwg = (int)nwg64;
    const long long rn2 = (long long)ratio_num * ratio_num, rd2 = (long long)ratio_den * ratio_den;
    hipStream_t s = as_stream(stream);
    if constexpr (sizeof(OutT) == 2)
        SFMHIP_REQUIRE(m_pad <= 32767, "sfmhip_match_pairs_i16: m_pad must be <= 32767 for an int16 graph");
#define SFMHIP_LAUNCH_MATCH(DD, MF, NS, WW)                                                              \
    hipLaunchKernelGGL((match_kernel<DD, MF, NS, WW, false, OutT>), dim3(nwg), dim3(64 * WW), 0, s, desc, norms, keys, \
                       n_kpts, m_pad, pairs, n_iblk, nwg, rn2, rd2, matches0, dist1, dist2, CertArgs{})
#define SFMHIP_LAUNCH_D(DD) SFMHIP_LAUNCH_MATCH(DD, 16, 4, 4)
    switch (d) {
        case 64: SFMHIP_LAUNCH_D(64); break;
        case 128: SFMHIP_LAUNCH_D(128); break;
        case 256: SFMHIP_LAUNCH_D(256); break;
        default:
            set_error("sfmhip_match_pairs: descriptor dim %d not in {64,128,256}", d);
            return SFMHIP_E_UNSUPPORTED;
    }
#undef SFMHIP_LAUNCH_D
#undef SFMHIP_LAUNCH_MATCH
    return check_launch("match_kernel");
}

extern "C" int sfmhip_match_pairs(const int8_t* desc, const int32_t* norms, const int32_t* keys,
                                  const int32_t* n_kpts, int n_img, int m_pad, int d,
                                  const int32_t* pairs, int P, int ratio_num, int ratio_den,
                                  int32_t* matches0, int32_t* dist1, int32_t* dist2, void* stream) {
    return match_pairs_impl(desc, norms, keys, n_kpts, n_img, m_pad, d, pairs, P, ratio_num, ratio_den, matches0,
                            dist1, dist2, stream);
}

extern "C" int sfmhip_match_pairs_i16(const int8_t* desc, const int32_t* norms, const int32_t* keys,
                                      const int32_t* n_kpts, int n_img, int m_pad, int d,
                                      const int32_t* pairs, int P, int ratio_num, int ratio_den,
                                      int16_t* matches0, void* stream) {
    return match_pairs_impl(desc, norms, keys, n_kpts, n_img, m_pad, d, pairs, P, ratio_num, ratio_den, matches0,
                            (int32_t*)nullptr, (int32_t*)nullptr, stream);
}

extern "C" int sfmhip_mutual_filter(int32_t* matches0, int32_t* matches1, int P, int m_pad, void* stream) {
    SFMHIP_REQUIRE(P >= 0 && m_pad > 0, "sfmhip_mutual_filter: bad shape");
    if (P == 0) return SFMHIP_OK;
    SFMHIP_REQUIRE(matches0 && matches1, "sfmhip_mutual_filter: null pointer");
    const int64_t total = (int64_t)P * m_pad;
    const int grid = (int)std::min<int64_t>((total + 255) / 256, 8192);
    hipLaunchKernelGGL(mutual_kernel, dim3(grid), dim3(256), 0, as_stream(stream), matches0, matches1, P,
                       m_pad);
    return check_launch("mutual_kernel");
}

extern "C" int sfmhip_vq(const double* obs, int64_t n_obs, const double* code_book, int n_codes, int d,
                         int32_t* codes, double* dist, void* stream) {
    SFMHIP_REQUIRE(n_obs >= 0 && n_codes > 0 && d > 0 && d <= 256, "sfmhip_vq: bad shape (d <= 256)");
    if (n_obs == 0) return SFMHIP_OK;
    SFMHIP_REQUIRE(obs && code_book && codes && dist, "sfmhip_vq: null pointer");
    // d = 128, <= 256 codewords (matching.py:27's 200-word codebook): the f16-split MFMA
    // filter + exact f64 decision (vq_f16s_kernel + vq_exact_kernel); other shapes: the
    // f64-MFMA GEMM-form kernel (d <= 128) or the f64 difference-form kernel.  The f32
    // filter kernels (LDS-staged and register-resident) measured slower.
    if (d == 128 && n_codes <= 256) {
        const int ncp = ceil_div(n_codes, 32) * 2;
        const size_t shm = (size_t)ncp * 4 * 2 * 64 * 16 + (size_t)ncp * 16 * sizeof(float);
        hipStream_t s = as_stream(stream);
        unsigned* amb = nullptr;
        if (scratch_alloc((void**)&amb, (size_t)(n_obs + 1) * sizeof(unsigned), s) == hipSuccess &&
            n_obs < ((int64_t)1 << 32) - 1) {
            unsigned* namb = amb + n_obs;
            (void)hipMemsetAsync(namb, 0, sizeof(unsigned), s);
            int dev = 0, n_cu = 256;
            if (hipGetDevice(&dev) == hipSuccess)
                (void)hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev);
            const int64_t n_wg = ((n_obs + 15) / 16 + kVqhWaves - 1) / kVqhWaves;
            auto kern = vq_f16s_kernel<0>;
            (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
            hipLaunchKernelGGL(kern, dim3((unsigned)std::min<int64_t>(n_wg, n_cu)), dim3(kVqhWaves * 64), shm, s, obs,
                               n_obs, code_book, n_codes, codes, dist, amb, namb);
            int rc = check_launch("vq_f16s_kernel");
            if (rc == SFMHIP_OK) {
                hipLaunchKernelGGL(vq_exact_kernel, dim3(1024), dim3(256), 0, s, obs, code_book, n_codes, 128, amb,
                                   namb, codes, dist);
                rc = check_launch("vq_exact_kernel");
            }
            scratch_free(amb, s);
            return rc;
        }
        (void)hipGetLastError();   // no scratch: the f64 kernels below
    }
    const int dp = d <= 32 ? 32 : d <= 64 ? 64 : d <= 128 ? 128 : 0;
    if (dp) {
        const int ld = dp + 4;
        const int max_cpp = std::min(144, (int)((150 * 1024 / 8) / (ld + 1)) / 16 * 16);
        const int passes = ceil_div(n_codes, max_cpp);
        const int cpp = ceil_div(ceil_div(n_codes, passes), 16) * 16;
        const size_t shm = (size_t)cpp * (ld + 1) * sizeof(double);
        int dev = 0, n_cu = 256;
        if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev);
        const int64_t n_tiles = (n_obs + kVqmTile - 1) / kVqmTile;
        const int grid = (int)std::min<int64_t>(n_tiles, n_cu);
        hipStream_t s = as_stream(stream);
#define SFMHIP_LAUNCH_VQM(DP, FL)                                                                             \
    do {                                                                                                  \
        (void)hipFuncSetAttribute((const void*)vq_mfma_kernel<DP, FL>, hipFuncAttributeMaxDynamicSharedMemorySize, \
                                  (int)shm);                                                               \
        hipLaunchKernelGGL((vq_mfma_kernel<DP, FL>), dim3(grid), dim3(kVqmWaves * 64), shm, s, obs, n_obs,      \
                           code_book, n_codes, d, cpp, codes, dist);                                       \
    } while (0)
        if (dp == 32) SFMHIP_LAUNCH_VQM(32, false);
        else if (dp == 64) SFMHIP_LAUNCH_VQM(64, false);
        else if (d != 128) SFMHIP_LAUNCH_VQM(128, false);
        else SFMHIP_LAUNCH_VQM(128, true);
#undef SFMHIP_LAUNCH_VQM
        return check_launch("vq_mfma_kernel");
    }
    const int64_t blocks = (n_obs + kVqObsPerBlock - 1) / kVqObsPerBlock;
    SFMHIP_REQUIRE(blocks < INT_MAX, "sfmhip_vq: too many observations");
    const size_t shm = (size_t)(kVqObsPerBlock * d + kVqCodesPerChunk * (d + 1)) * sizeof(double);
    SFMHIP_REQUIRE(shm <= 160 * 1024, "sfmhip_vq: descriptor dim too large for the LDS tiles");
    hipLaunchKernelGGL(vq_kernel, dim3((int)blocks), dim3(256), shm, as_stream(stream), obs, n_obs, code_book,
                       n_codes, d, codes, dist);
    return check_launch("vq_kernel");
}

extern "C" int sfmhip_desc_residual(const float* desc_f, const int8_t* desc_q, int n_img, int m_pad, int d,
                                    const int32_t* n_kpts, int mode, double* resid_row, double* resid_img,
                                    void* stream) {
    SFMHIP_REQUIRE(desc_f && desc_q && n_kpts && resid_row && resid_img, "sfmhip_desc_residual: null pointer");
    SFMHIP_REQUIRE(n_img > 0 && m_pad > 0 && d > 0, "sfmhip_desc_residual: bad shape");
    SFMHIP_REQUIRE(mode == 0 || mode == 1, "sfmhip_desc_residual: mode must be 0 or 1");
    const int64_t rows = (int64_t)n_img * m_pad;
    SFMHIP_REQUIRE(rows < INT_MAX, "sfmhip_desc_residual: too many rows");
    hipStream_t s = as_stream(stream);
    if (hipMemsetAsync(resid_img, 0, (size_t)n_img * sizeof(double), s) != hipSuccess) return check_launch("memset");
    hipLaunchKernelGGL(desc_residual_kernel, dim3(ceil_div(rows, 4)), dim3(256), 0, s, desc_f, desc_q, (int)rows, m_pad,
                       d, n_kpts, mode, resid_row, reinterpret_cast<unsigned long long*>(resid_img));
    return check_launch("desc_residual_kernel");
}

template <typename OutT>
static int match_exact_impl(const int8_t* desc, const int32_t* norms, const int32_t* keys,
                            const int8_t* desc_q, const float* desc_f, const double* resid_row,
                            const double* resid_img, int mode, const int32_t* n_kpts, int n_img,
                            int m_pad, int d, const int32_t* pairs, int P, int ratio_num, int ratio_den,
                            OutT* matches0, int32_t* dist1, int32_t* dist2, uint32_t* n_resolved,
                            void* stream) {
    SFMHIP_REQUIRE(n_img > 0 && P >= 0, "sfmhip_match_pairs_exact: bad counts");
    SFMHIP_REQUIRE(m_pad > 0 && m_pad % kJB == 0, "sfmhip_match_pairs_exact: m_pad must be a positive multiple of 128");
    SFMHIP_REQUIRE(mode == 0 || mode == 1, "sfmhip_match_pairs_exact: mode must be 0 or 1");
    SFMHIP_REQUIRE(ratio_num > 0 && ratio_den > 0 && ratio_num <= 65535 && ratio_den <= 65535,
                   "sfmhip_match_pairs_exact: ratio must be a positive fraction");
    if constexpr (sizeof(OutT) == 2)
        SFMHIP_REQUIRE(m_pad <= 32767, "sfmhip_match_pairs_exact_i16: m_pad must be <= 32767 for an int16 graph");
    if (P == 0) return SFMHIP_OK;
    SFMHIP_REQUIRE(desc && norms && keys && desc_q && desc_f && resid_row && resid_img && n_kpts && pairs && matches0,
                   "sfmhip_match_pairs_exact: null pointer");
    constexpr int IB = 256;   // match_kernel's query rows per workgroup (16x16 tiles, 4 per wave, 4 waves)
    const int n_iblk = ceil_div(m_pad, IB);
    const int64_t nwg64 = (int64_t)P * n_iblk;
    SFMHIP_REQUIRE(nwg64 < INT_MAX, "sfmhip_match_pairs_exact: too many pairs for one launch");
    const int nwg = (int)nwg64;
    const long long rn2 = (long long)ratio_num * ratio_num, rd2 = (long long)ratio_den * ratio_den;
    // SFMHIP_MATCH_CERT=0 (tests): every row through the exact pass
    const CertArgs ca{resid_row, resid_img, mode == 0 ? 1.0 : 1.0 / 127.0, knobs().match_cert == 0 ? 1 : 0};
    hipStream_t s = as_stream(stream);
    int dev = 0, n_cu = 256;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev);
    const int64_t nchunk = ((int64_t)P * m_pad + 63) / 64;
    const int rgrid = (int)std::min<int64_t>((nchunk + 3) / 4, (int64_t)n_cu * 8);
    if (n_resolved && hipMemsetAsync(n_resolved, 0, sizeof(uint32_t), s) != hipSuccess) return check_launch("memset");
    // the resolve's buckets: per image a row count and up to kResolveBucket graph entries
    const int64_t total = (int64_t)P * m_pad;
    void* rbuf = nullptr;
    const size_t rlist_bytes = (size_t)n_img * kResolveBucket * sizeof(int64_t);   // buckets, then the flat list
    const size_t rcnt_bytes = ((size_t)n_img + 1) * sizeof(unsigned);
    const size_t roff_bytes = (3 * (size_t)n_img + 33) * sizeof(unsigned);   // off, okey (+1), oimg, xr, ir
    const size_t ritem_bytes = 3 * (size_t)n_img * (kResolveBucket / kResolveRows + 1) * sizeof(int);
    if (scratch_alloc(&rbuf, 2 * rlist_bytes + rcnt_bytes + roff_bytes + ritem_bytes, s) != hipSuccess) {
        (void)hipGetLastError();
        set_error("sfmhip_match_pairs_exact: scratch allocation failed");
        return SFMHIP_E_HIP;
    }
    int64_t* rlist = reinterpret_cast<int64_t*>(rbuf);
    unsigned* rcnt = reinterpret_cast<unsigned*>(static_cast<char*>(rbuf) + rlist_bytes);
    unsigned* rflag = rcnt + n_img;
    int64_t* rflat = reinterpret_cast<int64_t*>(static_cast<char*>(rbuf) + rlist_bytes + rcnt_bytes + roff_bytes);
    unsigned* roff = reinterpret_cast<unsigned*>(static_cast<char*>(rbuf) + rlist_bytes + rcnt_bytes);
    unsigned* rokey = roff + n_img;
    int* roimg = reinterpret_cast<int*>(rokey + n_img + 1);
    unsigned* rxr = reinterpret_cast<unsigned*>(roimg + n_img);
    unsigned* rir = rxr + 16;
    int* ritems = reinterpret_cast<int*>(static_cast<char*>(rbuf) + 2 * rlist_bytes + rcnt_bytes + roff_bytes);
    if (hipMemsetAsync(rcnt, 0, rcnt_bytes, s) != hipSuccess) {
        scratch_free(rbuf, s);
        return check_launch("memset");
    }
    const int rxgrid = n_cu * 2;   // a multiple of 8: every XCD gets the same number of blocks
#define SFMHIP_LAUNCH_EXACT(DD)                                                                                  \
    hipLaunchKernelGGL((match_kernel<DD, 16, 4, 4, true, OutT>), dim3(nwg), dim3(256), 0, s, desc, norms, keys, n_kpts, \
                       m_pad, pairs, n_iblk, nwg, rn2, rd2, matches0, dist1, dist2, ca);                         \
    if (int rc = check_launch("match_kernel<cert>")) {                                                          \
        scratch_free(rbuf, s);                                                                                    \
        return rc;                                                                                                \
    }                                                                                                             \
    hipLaunchKernelGGL(resolve_collect_kernel<OutT>, dim3(rgrid), dim3(256), 0, s, matches0, total, m_pad, pairs, rcnt,  \
                       rlist, rflag);                                                                             \
    hipLaunchKernelGGL(resolve_offsets_kernel, dim3(1), dim3(1024), 0, s, rcnt, n_img, roff, rokey, roimg, rxr,      \
                       ritems, rir, rflag);                                                                       \
    hipLaunchKernelGGL(resolve_flatten_kernel, dim3(n_cu), dim3(256), 0, s, rokey, roimg, n_img, rlist, rflat,     \
                       rflag);                                                                                    \
    hipLaunchKernelGGL((match_resolve_batched_kernel<DD, OutT>), dim3(rxgrid), dim3(256), 0, s, desc, norms, desc_f, n_kpts,  \
                       m_pad, pairs, n_img, resid_row, resid_img, mode == 0 ? 1.0 : 127.0, (double)rn2,          \
                       (double)rd2, matches0, n_resolved, rflat, ritems, rir, rflag);                              \
    hipLaunchKernelGGL((match_resolve_kernel<DD, OutT>), dim3(rgrid), dim3(256), 0, s, desc_q, desc_f, n_kpts, m_pad,   \
                       pairs, P, resid_row, resid_img, mode == 0 ? 1.0 : 127.0, (double)rn2, (double)rd2,        \
                       matches0, n_resolved, rflag)
    switch (d) {
        case 64: SFMHIP_LAUNCH_EXACT(64); break;
        case 128: SFMHIP_LAUNCH_EXACT(128); break;
        case 256: SFMHIP_LAUNCH_EXACT(256); break;
        default:
            set_error("sfmhip_match_pairs_exact: descriptor dim %d not in {64,128,256}", d);
            scratch_free(rbuf, s);
            return SFMHIP_E_UNSUPPORTED;
    }
#undef SFMHIP_LAUNCH_EXACT
    const int rc = check_launch("match_resolve_kernel");
    scratch_free(rbuf, s);
    return rc;
}

extern "C" int sfmhip_match_pairs_exact(const int8_t* desc, const int32_t* norms, const int32_t* keys,
                                        const int8_t* desc_q, const float* desc_f, const double* resid_row,
                                        const double* resid_img, int mode, const int32_t* n_kpts, int n_img,
                                        int m_pad, int d, const int32_t* pairs, int P, int ratio_num, int ratio_den,
                                        int32_t* matches0, int32_t* dist1, int32_t* dist2, uint32_t* n_resolved,
                                        void* stream) {
    return match_exact_impl(desc, norms, keys, desc_q, desc_f, resid_row, resid_img, mode, n_kpts, n_img, m_pad, d,
                            pairs, P, ratio_num, ratio_den, matches0, dist1, dist2, n_resolved, stream);
}

extern "C" int sfmhip_match_pairs_exact_i16(const int8_t* desc, const int32_t* norms, const int32_t* keys,
                                            const int8_t* desc_q, const float* desc_f, const double* resid_row,
                                            const double* resid_img, int mode, const int32_t* n_kpts, int n_img,
                                            int m_pad, int d, const int32_t* pairs, int P, int ratio_num,
                                            int ratio_den, int16_t* matches0, uint32_t* n_resolved, void* stream) {
    return match_exact_impl(desc, norms, keys, desc_q, desc_f, resid_row, resid_img, mode, n_kpts, n_img, m_pad, d,
                            pairs, P, ratio_num, ratio_den, matches0, (int32_t*)nullptr, (int32_t*)nullptr,
                            n_resolved, stream);
}
