// mfma_mx_peak.hip — diagnostic: the rate this MI355X sustains for the
// matcher's per-pair work (16x16 output tiles, 4 independent chains per wave, d = 256 per
// distance) on block-scaled FP6 (e2m3) / FP4 (e2m1) MFMAs — v_mfma_scale_f32_16x16x128_f8f6f4,
// two k-steps of 128 per distance — against today's int8 form (v_mfma_i32_16x16x64_i8, four
// k-steps of 64), each with and without the top-2 epilogue per output element.  The MX
// epilogue first converts the f32 dot to an integer key (one v_cvt per distance), then runs
// the int8 form's two-candidate top-2 (max3 + med3 + max).  No LDS, no global traffic in the
// loop: the ceiling the match kernel would be bound by.  The operands pass through an empty
// asm each iteration so that the compiler cannot hoist the (pure) scaled MFMAs out of the loop
// (it did: a first build measured 22-105 POPS).
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/mfma_mx_peak tools/mfma_mx_peak.hip
// Run:   tools/mfma_mx_peak ITERS
#include <hip/hip_runtime.h>
#include <climits>
#include <cstdio>
#include <cstdlib>

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

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

// today's form: 4 chains x 4 k-steps of v_mfma_i32_16x16x64_i8 per distance tile
template <bool EPI>
__global__ __launch_bounds__(256, 2) void kern_i8(const int* __restrict__ seed, int iters, int* out) {
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
        // opaque to the compiler: the operands "change" every iteration (no hoisted MFMAs)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            asm volatile("" : "+v"(a[k]));
#pragma unroll
            for (int t = 0; t < 4; ++t) asm volatile("" : "+v"(b[t][k]));
        }
        i32x4 acc[4] = {{0}, {0}, {0}, {0}};
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
            for (int t = 0; t < 4; ++t) acc[t] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a[k], b[t][k], acc[t], 0, 0, 0);
        if (EPI) {
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

// block-scaled MX: FMT 2 = fp6 e2m3, 4 = fp4 e2m1; 4 chains x 2 k-steps of 128 per distance tile
template <int FMT, bool EPI>
__global__ __launch_bounds__(256, 2) void kern_mx(const int* __restrict__ seed, int iters, int* out) {
    const int lane = threadIdx.x & 63;
    i32x8 a[2], b[4][2];
    for (int k = 0; k < 2; ++k)
        for (int e = 0; e < 8; ++e) {
            a[k][e] = seed[(blockIdx.x * 97 + lane * 13 + k * 7 + e) & 4095];
            for (int t = 0; t < 4; ++t) b[t][k][e] = seed[(blockIdx.x * 31 + lane * 5 + k * 11 + e * 3 + t * 17) & 4095];
        }
    const int sa = 120 + (lane & 7), sb = 121 + (lane & 3);   // E8M0 block scales (2^-7 .. 2^0)
    int t1[4] = {INT_MIN, INT_MIN, INT_MIN, INT_MIN}, t2[4] = {INT_MIN, INT_MIN, INT_MIN, INT_MIN};
    int kv = seed[lane];
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int k = 0; k < 2; ++k) {
            asm volatile("" : "+v"(a[k]));
#pragma unroll
            for (int t = 0; t < 4; ++t) asm volatile("" : "+v"(b[t][k]));
        }
        f32x4 acc[4] = {{0.f}, {0.f}, {0.f}, {0.f}};
#pragma unroll
        for (int k = 0; k < 2; ++k)
#pragma unroll
            for (int t = 0; t < 4; ++t)
                acc[t] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a[k], b[t][k], acc[t], FMT, FMT, 0, sa, 0,
                                                                          sb);
        if (EPI) {
#pragma unroll
            for (int t = 0; t < 4; ++t)
#pragma unroll
                for (int q = 0; q < 4; q += 2) {
                    const int ka = (int)acc[t][q] * 256 + kv, kb = (int)acc[t][q + 1] * 256 + kv + 1;
                    const int m = med3i(t1[t], ka, kb);
                    t1[t] = max3i(t1[t], ka, kb);
                    t2[t] = max(t2[t], m);
                }
        } else {
#pragma unroll
            for (int t = 0; t < 4; ++t) t1[t] ^= __float_as_int(acc[t][lane & 3]);
        }
        kv += 1;
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = t1[0] + t2[0] + t1[1] + t2[1] + t1[2] + t2[2] + t1[3] + t2[3];
}

int main(int argc, char** argv) {
    const int blocks = 256 * 2 * 8, iters = argc > 1 ? atoi(argv[1]) : 2000;
    int *seed, *out;
    hipMalloc(&seed, 4096 * 4);
    hipMalloc(&out, (size_t)blocks * 256 * 4);
    int h[4096];
    unsigned x = 12345;
    for (int i = 0; i < 4096; ++i) {
        x = x * 1664525u + 1013904223u;
        h[i] = (int)x;   // uniform random bits: random int8 values, random fp6 / fp4 codes (no NaN encodings)
    }
    hipMemcpy(seed, h, sizeof(h), hipMemcpyHostToDevice);
    // per wave-iteration: 4 tiles x 16 x 16 outputs x d = 256 x 2 ops
    const double ops_iter = 4.0 * 16 * 16 * 256 * 2;
    const char* names[6] = {"int8 16x16x64 (today)", "int8 16x16x64 (today)", "fp6 e2m3 16x16x128 scaled",
                            "fp6 e2m3 16x16x128 scaled", "fp4 e2m1 16x16x128 scaled", "fp4 e2m1 16x16x128 scaled"};
    for (int c = 0; c < 6; ++c) {
        hipEvent_t e0, e1;
        hipEventCreate(&e0);
        hipEventCreate(&e1);
        for (int rep = 0; rep < 3; ++rep) {
            hipEventRecord(e0);
#define L(K) hipLaunchKernelGGL(K, dim3(blocks), dim3(256), 0, 0, seed, iters, out)
            switch (c) {
                case 0: L((kern_i8<false>)); break;
                case 1: L((kern_i8<true>)); break;
                case 2: L((kern_mx<2, false>)); break;
                case 3: L((kern_mx<2, true>)); break;
                case 4: L((kern_mx<4, false>)); break;
                default: L((kern_mx<4, true>)); break;
            }
#undef L
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            const double ops = (double)blocks * 4 * iters * ops_iter;
            if (rep == 2)
                printf("%-28s %s epilogue: %8.2f ms  %6.0f TOPS (%.1f%% of the 5000 int8 spec)\n", names[c],
                       (c & 1) ? "with" : "no  ", ms, ops / ms / 1e9, ops / ms / 1e9 / 50.0);
        }
    }
    return 0;
}
