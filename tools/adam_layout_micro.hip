// adam_layout_micro.hip — diagnostic: torch-Adam arithmetic over 256^3 voxel lines of
// 32 floats (the plenoxel trainer's state, 4 x 2 GiB) in three layouts, fresh process:
//   sep    four hipMalloc'ed 2 GiB buffers (param, grad, m, v)
//   one    one allocation, the four buffers back to back (stride 2 GiB)
//   aos    one allocation, the four lines of a voxel adjacent: [p | g | m | v] x 128 B
//   churn  'sep' after allocating, touching and freeing 1.08 / 2.58 / 1.88 / 2.15 GB buffers
//          (the allocation history of tools/adam_probe.py's fast 'after' mode)
//   hold   'sep' with a 1 GiB buffer allocated (and kept) first
//   rev    'sep' allocated in the reverse order
// plus a 2 GiB device copy (p -> g) in each state
// Each thread updates one float4 of one voxel line per iteration (grid-stride), non-temporal
// loads/stores, grads read and zeroed densely.  Prints the median kernel time of 10.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/adam_layout_micro tools/adam_layout_micro.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <string>
#include <vector>

typedef float v4f __attribute__((ext_vector_type(4)));

__device__ __forceinline__ v4f adam4(v4f pp, v4f gg, v4f& mm, v4f& vv) {
    const float w1 = 0.1f, b2 = 0.999f, s2 = 0.001f, bc2s = 0.5f, eps = 1e-8f, step = -0.01f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        mm[j] = fmaf(w1, gg[j] - mm[j], mm[j]);
        vv[j] = fmaf(s2 * gg[j], gg[j], vv[j] * b2);
        pp[j] = pp[j] + (step * mm[j]) / (sqrtf(vv[j]) / bc2s + eps);
    }
    return pp;
}

// element e (float4 index within a buffer of n4): buffer k at base + k * kstride4 + e  (sep/one), or
// voxel-line interleaved (aos): line = e / 8, chunk = e % 8 -> base + (line * 4 + k) * 8 + chunk
template <bool AOS>
__global__ __launch_bounds__(256) void adam_k(v4f* p, v4f* g, v4f* m, v4f* v, int64_t n4) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    const v4f z4 = {0.f, 0.f, 0.f, 0.f};
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n4; e += stride) {
        const int64_t o = AOS ? ((e >> 3) * 32 + (e & 7)) : e;
        v4f m0 = __builtin_nontemporal_load(m + o), v0 = __builtin_nontemporal_load(v + o);
        const v4f g0 = __builtin_nontemporal_load(g + o), p0 = __builtin_nontemporal_load(p + o);
        const v4f q = adam4(p0, g0, m0, v0);
        __builtin_nontemporal_store(m0, m + o);
        __builtin_nontemporal_store(v0, v + o);
        __builtin_nontemporal_store(q, p + o);
        __builtin_nontemporal_store(z4, g + o);
    }
}

// contiguous assignment: workgroup b owns float4 [b * chunk, (b + 1) * chunk), two in flight per thread
__global__ __launch_bounds__(256) void adam_contig_k(v4f* p, v4f* g, v4f* m, v4f* v, int64_t n4, int64_t chunk) {
    const v4f z4 = {0.f, 0.f, 0.f, 0.f};
    const int64_t b0 = (int64_t)blockIdx.x * chunk, b1 = min(n4, b0 + chunk);
    for (int64_t e = b0 + threadIdx.x; e < b1; e += 512) {
        const int64_t f = e + 256;
        const bool two = f < b1;
        v4f m0 = __builtin_nontemporal_load(m + e), v0 = __builtin_nontemporal_load(v + e);
        const v4f g0 = __builtin_nontemporal_load(g + e), p0 = __builtin_nontemporal_load(p + e);
        v4f m1 = z4, v1 = z4, g1 = z4, p1 = z4;
        if (two) {
            m1 = __builtin_nontemporal_load(m + f); v1 = __builtin_nontemporal_load(v + f);
            g1 = __builtin_nontemporal_load(g + f); p1 = __builtin_nontemporal_load(p + f);
        }
        const v4f q0 = adam4(p0, g0, m0, v0);
        __builtin_nontemporal_store(m0, m + e);
        __builtin_nontemporal_store(v0, v + e);
        __builtin_nontemporal_store(q0, p + e);
        __builtin_nontemporal_store(z4, g + e);
        if (two) {
            const v4f q1 = adam4(p1, g1, m1, v1);
            __builtin_nontemporal_store(m1, m + f);
            __builtin_nontemporal_store(v1, v + f);
            __builtin_nontemporal_store(q1, p + f);
            __builtin_nontemporal_store(z4, g + f);
        }
    }
}

static float run_contig(v4f* p, v4f* g, v4f* m, v4f* v, int64_t n4, int64_t chunk) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    std::vector<float> ts;
    const int blocks = (int)((n4 + chunk - 1) / chunk);
    for (int r = 0; r < 12; ++r) {
        hipEventRecord(e0);
        hipLaunchKernelGGL(adam_contig_k, dim3(blocks), dim3(256), 0, 0, p, g, m, v, n4, chunk);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (r >= 2) ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    return ts[ts.size() / 2];
}

static int g_blocks = 256 * 32;

static float run(bool aos, v4f* p, v4f* g, v4f* m, v4f* v, int64_t n4) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    std::vector<float> ts;
    for (int r = 0; r < 12; ++r) {
        hipEventRecord(e0);
        if (aos) hipLaunchKernelGGL(adam_k<true>, dim3(g_blocks), dim3(256), 0, 0, p, g, m, v, n4);
        else hipLaunchKernelGGL(adam_k<false>, dim3(g_blocks), dim3(256), 0, 0, p, g, m, v, n4);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (r >= 2) ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    return ts[ts.size() / 2];
}

__global__ __launch_bounds__(256) void copy_k(const v4f* __restrict__ a, v4f* __restrict__ b, int64_t n4) {
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n4; e += stride)
        __builtin_nontemporal_store(__builtin_nontemporal_load(a + e), b + e);
}

static float run_copy(const v4f* a, v4f* b, int64_t n4) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    std::vector<float> ts;
    for (int r = 0; r < 8; ++r) {
        hipEventRecord(e0);
        hipLaunchKernelGGL(copy_k, dim3(256 * 32), dim3(256), 0, 0, a, b, n4);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (r >= 2) ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    return 2.0f * n4 * 16 / ts[ts.size() / 2] / 1e6f;   // GB/s
}

int main(int argc, char** argv) {
    const int64_t n4 = (int64_t)256 * 256 * 256 * 8;   // float4 per buffer (2 GiB)
    const size_t nb = (size_t)n4 * 16;
    const char* mode = argc > 1 ? argv[1] : "all";
    const std::string md(mode);
    if (md == "churn") {
        const size_t sz[4] = {1080000000ull, 2580000000ull, 1880000000ull, 2150000000ull};
        void* t[4];
        for (int k = 0; k < 4; ++k) { hipMalloc(&t[k], sz[k]); hipMemset(t[k], 1, sz[k]); }
        hipDeviceSynchronize();
        for (int k = 0; k < 4; ++k) hipFree(t[k]);
    }
    void* held = nullptr;
    if (md == "hold") { hipMalloc(&held, (size_t)1 << 30); hipMemset(held, 0, (size_t)1 << 30); }
    if (md == "sep" || md == "all" || md == "churn" || md == "hold" || md == "rev") {
        v4f *p, *g, *m, *v;
        if (md == "rev") { hipMalloc(&v, nb); hipMalloc(&m, nb); hipMalloc(&g, nb); hipMalloc(&p, nb); }
        else { hipMalloc(&p, nb); hipMalloc(&g, nb); hipMalloc(&m, nb); hipMalloc(&v, nb); }
        hipMemset(p, 0, nb); hipMemset(g, 0, nb); hipMemset(m, 0, nb); hipMemset(v, 0, nb);
        printf("%-5s %.3f ms  copy %.0f GB/s  (p %p g %p m %p v %p)\n", md == "all" ? "sep" : mode,
               run(false, p, g, m, v, n4), run_copy(p, g, n4), (void*)p, (void*)g, (void*)m, (void*)v);
        for (int bl : {1024, 2048, 4096, 32768}) {
            g_blocks = bl;
            printf("      grid-stride %5d blocks %.3f ms\n", bl, run(false, p, g, m, v, n4));
        }
        g_blocks = 256 * 32;
        for (int64_t ch : {4096, 16384, 65536})
            printf("      contiguous %6lld float4 per block %.3f ms\n", (long long)ch, run_contig(p, g, m, v, n4, ch));
        hipFree(p); hipFree(g); hipFree(m); hipFree(v);
    }
    if (md == "one" || md == "all") {
        v4f* b;
        hipMalloc(&b, 4 * nb);
        hipMemset(b, 0, 4 * nb);
        printf("one   %.3f ms  copy %.0f GB/s\n", run(false, b, b + n4, b + 2 * n4, b + 3 * n4, n4),
               run_copy(b, b + n4, n4));
        printf("aos   %.3f ms\n", run(true, b, b + 8, b + 16, b + 24, n4));
        hipFree(b);
    }
    return 0;
}
