// adam_layout_micro.hip — diagnostic: torch-Adam arithmetic over 256^3 voxel lines of
// 32 floats (the plenoxel trainer's state, 4 x 2 GiB) in three layouts, fresh process:
//   sep    four hipMalloc'ed 2 GiB buffers (param, grad, m, v)
//   one    one allocation, the four buffers back to back (stride 2 GiB)
//   aos    one allocation, the four lines of a voxel adjacent: [p | g | m | v] x 128 B
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

static float run(bool aos, v4f* p, v4f* g, v4f* m, v4f* v, int64_t n4) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    std::vector<float> ts;
    for (int r = 0; r < 12; ++r) {
        hipEventRecord(e0);
        if (aos) hipLaunchKernelGGL(adam_k<true>, dim3(256 * 32), dim3(256), 0, 0, p, g, m, v, n4);
        else hipLaunchKernelGGL(adam_k<false>, dim3(256 * 32), dim3(256), 0, 0, p, g, m, v, n4);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (r >= 2) ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    return ts[ts.size() / 2];
}

int main(int argc, char** argv) {
    const int64_t n4 = (int64_t)256 * 256 * 256 * 8;   // float4 per buffer (2 GiB)
    const size_t nb = (size_t)n4 * 16;
    const char* mode = argc > 1 ? argv[1] : "all";
    const std::string md(mode);
    if (md == "sep" || md == "all") {
        v4f *p, *g, *m, *v;
        hipMalloc(&p, nb); hipMalloc(&g, nb); hipMalloc(&m, nb); hipMalloc(&v, nb);
        hipMemset(p, 0, nb); hipMemset(g, 0, nb); hipMemset(m, 0, nb); hipMemset(v, 0, nb);
        printf("sep  %.3f ms  (p %p g %p m %p v %p)\n", run(false, p, g, m, v, n4), (void*)p, (void*)g, (void*)m, (void*)v);
        hipFree(p); hipFree(g); hipFree(m); hipFree(v);
    }
    if (md == "one" || md == "all") {
        v4f* b;
        hipMalloc(&b, 4 * nb);
        hipMemset(b, 0, 4 * nb);
        printf("one  %.3f ms\n", run(false, b, b + n4, b + 2 * n4, b + 3 * n4, n4));
        printf("aos  %.3f ms\n", run(true, b, b + 8, b + 16, b + 24, n4));
        hipFree(b);
    }
    return 0;
}
