// mfma_peak.hip — diagnostic: the int8 MFMA rate this MI355X sustains on
// random register operands, with and without the matcher's 3-op epilogue per
// output element (no LDS, no global traffic in the loop).  Gives the practical
// ceiling (clock under load) the match kernel is compared against.  The 16x16x64
// epilogue is the matcher's current one (two candidates per top-2 step, ~2.5 VALU per
// distance); the 32x32x32 kernel keeps the older 3-op form (max + med3 per candidate).
// KS = MFMA k-steps per epilogue: d = 256 (C3) is 8 steps of 32x32x32 or 4 of
// 16x16x64; d = 128 (C2) half that, so the epilogue weighs twice as much.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/mfma_peak tools/mfma_peak.hip
// Run:   tools/mfma_peak ITERS MODES   (MODES 1: random operands only)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cmath>

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));
typedef int i32x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ int max3i(int a, int b, int c) {
    int r;
    asm("v_max3_i32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
__device__ __forceinline__ int med3i(int a, int b, int c) {
    int r;
    asm("v_med3_i32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

template <bool EPI, int KS>
__global__ __launch_bounds__(256, 2) void kern(const int* __restrict__ seed, int iters, int* out) {
    const int lane = threadIdx.x & 63;
    i32x4 a[8], b[2][8];
    for (int k = 0; k < 8; ++k)
        for (int e = 0; e < 4; ++e) {
            a[k][e] = seed[(blockIdx.x * 97 + lane * 13 + k * 7 + e) & 4095];
            b[0][k][e] = seed[(blockIdx.x * 31 + lane * 5 + k * 11 + e * 3) & 4095];
            b[1][k][e] = seed[(blockIdx.x * 17 + lane * 7 + k * 3 + e * 5) & 4095];
        }
    int t1a = INT_MIN, t2a = INT_MIN, t1b = INT_MIN, t2b = INT_MIN;
    int kv = seed[lane];
    for (int it = 0; it < iters; ++it) {
        i32x16 acc0 = {0}, acc1 = {0};
#pragma unroll
        for (int k = 0; k < KS; ++k) {
            acc0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[k], b[0][k], acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a[k], b[1][k], acc1, 0, 0, 0);
        }
        if (EPI) {
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const int ka = acc0[q] * 256 + kv;
                t2a = med3i(t2a, ka, t1a);
                t1a = max(t1a, ka);
                const int kb = acc1[q] * 256 + kv;
                t2b = med3i(t2b, kb, t1b);
                t1b = max(t1b, kb);
            }
        } else {
            t1a ^= acc0[lane & 15];
            t1b ^= acc1[(lane + 3) & 15];
        }
        kv += 1;
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = t1a + t2a + t1b + t2b;
}

// the matcher's default shape: v_mfma_i32_16x16x64_i8, 4 output tiles per wave
// (4 independent chains), KS k-steps of 64 per epilogue (4: d = 256, 2: d = 128)
template <bool EPI, int KS>
__global__ __launch_bounds__(256, 2) void kern16(const int* __restrict__ seed, int iters, int* out) {
    const int lane = threadIdx.x & 63;
    i32x4 a[4], b[4][4];
    for (int k = 0; k < 4; ++k)
        for (int e = 0; e < 4; ++e) {
            a[k][e] = seed[(blockIdx.x * 97 + lane * 13 + k * 7 + e) & 4095];
            for (int t = 0; t < 4; ++t) b[t][k][e] = seed[(blockIdx.x * 31 + lane * 5 + k * 11 + e * 3 + t * 17) & 4095];
        }
    int t1[4] = {INT_MIN, INT_MIN, INT_MIN, INT_MIN}, t2[4] = {INT_MIN, INT_MIN, INT_MIN, INT_MIN};
    int kv = seed[lane];
    for (int it = 0; it < iters; ++it) {
        i32x4 acc[4] = {{0}, {0}, {0}, {0}};
#pragma unroll
        for (int k = 0; k < KS; ++k)
#pragma unroll
            for (int t = 0; t < 4; ++t) acc[t] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[k], b[t][k], acc[t], 0, 0, 0);
        if (EPI) {   // the matcher's epilogue: two candidates per top-2 step (max3 + med3 + max)
#pragma unroll
            for (int t = 0; t < 4; ++t)
#pragma unroll
                for (int q = 0; q < 4; q += 2) {
                    const int ka = acc[t][q] * 256 + kv, kb = acc[t][q + 1] * 256 + kv + 1;
                    const int m = med3i(t1[t], ka, kb);
                    t1[t] = max3i(t1[t], ka, kb);
                    t2[t] = max(t2[t], m);
                }
        } else {
#pragma unroll
            for (int t = 0; t < 4; ++t) t1[t] ^= acc[t][lane & 3];
        }
        kv += 1;
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = t1[0] + t2[0] + t1[1] + t2[1] + t1[2] + t2[2] + t1[3] + t2[3];
}

int main(int argc, char** argv) {
    const int blocks = 256 * 2 * 8, iters = argc > 1 ? atoi(argv[1]) : 2000;
    int *seed, *out;
    hipMalloc(&seed, 4096 * 4);
    hipMalloc(&out, blocks * 256 * 4);
    int h[4096];
    // operand byte distributions: 0 uniform random bytes, 1 zero, then C3-like small
    // signed values round(N(0, 8)) (two's complement) shifted by 0, 64, 88, 100
    // (round 6) N(0,6): the C3 descriptors quantised at 95 instead of 127 (|q| <= 30, the same
    // certified decisions in tools/sim_mx_certify-style models); +48 the matcher's shift
    const char* names[8] = {"random", "zero", "N(0,8)+0", "N(0,8)+64", "N(0,8)+88", "N(0,8)+100", "N(0,8)+48",
                            "N(0,6)+48"};
    const int shifts[8] = {0, 0, 0, 64, 88, 100, 48, 48};
    const float sigmas[8] = {8.f, 8.f, 8.f, 8.f, 8.f, 8.f, 8.f, 6.f};
    const int modes = argc > 2 ? atoi(argv[2]) : 2;
    for (int zero = 0; zero < modes; ++zero) {
        unsigned x = 12345;
        for (int i = 0; i < 4096; ++i) {
            x = x * 1664525u + 1013904223u;
            if (zero < 2) { h[i] = zero ? 0 : (int)x; continue; }
            unsigned w = 0;
            for (int b = 0; b < 4; ++b) {
                // Irwin-Hall(12) - 6 ~ N(0, 1), times 8, rounded, clamped to [-40, 39]
                float g = -6.f;
                for (int t = 0; t < 12; ++t) { x = x * 1664525u + 1013904223u; g += (float)(x >> 8) / 16777216.f; }
                int v = (int)lrintf(sigmas[zero] * g);
                v = v < -40 ? -40 : (v > 39 ? 39 : v);
                v += shifts[zero];
                w |= (unsigned)(v & 255) << (8 * b);
            }
            h[i] = (int)w;
        }
        hipMemcpy(seed, h, sizeof(h), hipMemcpyHostToDevice);
        // (shape, d): ops per launch = blocks x 4 waves x iters x (MFMAs per iter) x ops per MFMA
        struct Cfg { const char* name; int id; double mfma_per_iter, ops_per_mfma; };
        const Cfg cfgs[4] = {{"32x32x32 d=256", 0, 16, 65536.0}, {"32x32x32 d=128", 1, 8, 65536.0},
                             {"16x16x64 d=256", 2, 16, 32768.0}, {"16x16x64 d=128", 3, 8, 32768.0}};
        for (const Cfg& c : cfgs)
        for (int epi = 0; epi < 2; ++epi) {
            hipEvent_t e0, e1;
            hipEventCreate(&e0);
            hipEventCreate(&e1);
            for (int rep = 0; rep < 3; ++rep) {
                hipEventRecord(e0);
#define L(K) hipLaunchKernelGGL(K, dim3(blocks), dim3(256), 0, 0, seed, iters, out)
                switch (c.id * 2 + epi) {
                    case 0: L((kern<false, 8>)); break;
                    case 1: L((kern<true, 8>)); break;
                    case 2: L((kern<false, 4>)); break;
                    case 3: L((kern<true, 4>)); break;
                    case 4: L((kern16<false, 4>)); break;
                    case 5: L((kern16<true, 4>)); break;
                    case 6: L((kern16<false, 2>)); break;
                    default: L((kern16<true, 2>)); break;
                }
#undef L
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms;
                hipEventElapsedTime(&ms, e0, e1);
                const double ops = (double)blocks * 4 * iters * c.mfma_per_iter * c.ops_per_mfma;
                if (rep == 2)
                    printf("%s operands, %s, %s epilogue: %.2f ms  %.0f TOPS (%.1f%% of 5000)\n", names[zero], c.name,
                           epi ? "with" : "no", ms, ops / ms / 1e9, ops / ms / 1e9 / 50.0);
            }
        }
    }
    return 0;
}
