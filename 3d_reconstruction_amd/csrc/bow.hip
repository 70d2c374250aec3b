// bow.hip — BoW retrieval support: per-image visual-word
// histograms (matching.py:30-35) and the k-means centroid update of
// scipy.cluster.vq.kmeans (bow.py:23 -> scipy _vq.update_cluster_means).
// Word assignment itself is sfmhip_vq (match.hip).
#include "common.h"
#include <climits>

namespace sfmhip {

// One workgroup per image: LDS histogram of its codes, then one store per bin.
__global__ __launch_bounds__(256) void histogram_kernel(const int32_t* __restrict__ codes,
                                                        const int64_t* __restrict__ offsets, int k,
                                                        int32_t* __restrict__ hist) {
    extern __shared__ int32_t h[];
    const int img = blockIdx.x;
    for (int c = threadIdx.x; c < k; c += blockDim.x) h[c] = 0;
    __syncthreads();
    const int64_t a = offsets[img], b = offsets[img + 1];
    for (int64_t i = a + threadIdx.x; i < b; i += blockDim.x) {
        const int c = codes[i];
        if (c >= 0 && c < k) atomicAdd(&h[c], 1);
    }
    __syncthreads();
    for (int c = threadIdx.x; c < k; c += blockDim.x) hist[(size_t)img * k + c] = h[c];
}

// scipy update_cluster_means: sums accumulate observations in index order per
// cluster, mean = sum / count.  One workgroup per cluster, one lane per
// feature, the whole code array scanned in order (codes staged through LDS in
// chunks) so every f64 sum has scipy's exact order -> bit-identical means.
constexpr int kKmChunk = 2048;

__global__ __launch_bounds__(256) void kmeans_update_kernel(const double* __restrict__ obs, int64_t n, int d,
                                                            const int32_t* __restrict__ codes, int k,
                                                            double* __restrict__ book, int32_t* __restrict__ counts) {
    __shared__ int32_t sc[kKmChunk];
    __shared__ int32_t members[kKmChunk];
    __shared__ int nmem;
    const int c = blockIdx.x;
    double acc[4] = {0.0, 0.0, 0.0, 0.0};  // features threadIdx.x + 256 * q
    int count = 0;
    for (int64_t base = 0; base < n; base += kKmChunk) {
        const int len = (int)min((int64_t)kKmChunk, n - base);
        for (int t = threadIdx.x; t < len; t += blockDim.x) sc[t] = codes[base + t];
        __syncthreads();
        if (threadIdx.x < 64) {  // ordered compaction of this chunk's members by wave 0
            const int lane = threadIdx.x;
            const unsigned long long below = (1ull << lane) - 1ull;
            int m = 0;
            for (int t0 = 0; t0 < len; t0 += 64) {
                const bool hit = (t0 + lane < len) && sc[t0 + lane] == c;
                const unsigned long long mask = __ballot(hit);
                if (hit) members[m + __popcll(mask & below)] = t0 + lane;
                m += __popcll(mask);
            }
            if (lane == 0) nmem = m;
        }
        __syncthreads();
        const int m = nmem;
        count += m;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int f = threadIdx.x + 256 * q;
            if (f < d) {
                double s = acc[q];
                for (int t = 0; t < m; ++t) s = s + obs[(size_t)(base + members[t]) * d + f];
                acc[q] = s;
            }
        }
        __syncthreads();
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int f = threadIdx.x + 256 * q;
        if (f < d && count > 0) book[(size_t)c * d + f] = acc[q] / (double)count;
    }
    if (threadIdx.x == 0) counts[c] = count;
}

}  // namespace sfmhip

using namespace sfmhip;

extern "C" int sfmhip_word_histogram(const int32_t* codes, const int64_t* offsets, int n_img, int k,
                                     int32_t* hist, void* stream) {
    SFMHIP_REQUIRE(n_img >= 0 && k > 0 && k <= 16384, "sfmhip_word_histogram: bad shape");
    if (n_img == 0) return SFMHIP_OK;
    SFMHIP_REQUIRE(codes && offsets && hist, "sfmhip_word_histogram: null pointer");
    hipLaunchKernelGGL(histogram_kernel, dim3(n_img), dim3(256), k * sizeof(int32_t), as_stream(stream), codes,
                       offsets, k, hist);
    return check_launch("histogram_kernel");
}

extern "C" int sfmhip_kmeans_update(const double* obs, int64_t n, int d, const int32_t* codes, int k,
                                    double* book, int32_t* counts, void* stream) {
    SFMHIP_REQUIRE(obs && codes && book && counts, "sfmhip_kmeans_update: null pointer");
    SFMHIP_REQUIRE(n >= 0 && d > 0 && d <= 1024 && k > 0, "sfmhip_kmeans_update: bad shape (d <= 1024)");
    hipLaunchKernelGGL(kmeans_update_kernel, dim3(k), dim3(256), 0, as_stream(stream), obs, n, d, codes, k, book,
                       counts);
    return check_launch("kmeans_update_kernel");
}
