// Does v_mfma_f32_16x16x32_f16 keep f16 subnormal inputs (the vq f16-split filter's error bound
// assumes it)?  A = 2^-20 (f16 subnormal) everywhere, B = 1: every C element must be 32 x 2^-20.
// Also A = 2^-24 (smallest subnormal) x B = 2^-24 products and a mixed normal/subnormal row.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/mfma_f16_denorm tools/mfma_f16_denorm.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
__global__ void k(float* out, float a, float b) {
    f16x8 A, B;
    for (int e = 0; e < 8; ++e) { A[e] = (_Float16)a; B[e] = (_Float16)b; }
    f32x4 c = {0.f, 0.f, 0.f, 0.f};
    c = __builtin_amdgcn_mfma_f32_16x16x32_f16(A, B, c, 0, 0, 0);
    for (int g = 0; g < 4; ++g) out[threadIdx.x * 4 + g] = c[g];
}
int main() {
    float* d;
    hipMalloc(&d, 256 * sizeof(float));
    float h[256];
    const float cases[][2] = {{0x1p-20f, 1.f}, {0x1p-24f, 1.f}, {0x1p-24f, 0x1p-24f}, {0x1p-14f, 0x1p-10f}, {1.f, 1.f}};
    int bad = 0;
    for (auto& cs : cases) {
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, cs[0], cs[1]);
        hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
        const double want = 32.0 * (double)cs[0] * (double)cs[1];
        int ok = 0;
        for (int i = 0; i < 256; ++i) ok += (double)h[i] == want;
        printf("a=%a b=%a: C=%a (want %a) %d/256 exact\n", cs[0], cs[1], h[0], want, ok);
        bad += ok != 256;
    }
    hipFree(d);
    return bad ? 1 : 0;
}
