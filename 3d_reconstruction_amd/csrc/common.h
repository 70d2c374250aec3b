// common.h — shared plumbing for libsfmhip.so (gfx950 only).
// Error state is thread-local; every extern "C" entry point returns an int
// status and leaves a message for sfmhip_last_error().
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <cstdio>
#include <cstdarg>

#include "../../include/sfmhip.h"

namespace sfmhip {

void set_error(const char* fmt, ...);

// Launch-status helper: HIP kernel launches report failure through
// hipGetLastError(); translate it into SFMHIP_E_HIP with the kernel name.
inline int check_launch(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_error("%s: %s", what, hipGetErrorString(e));
        return SFMHIP_E_HIP;
    }
    return SFMHIP_OK;
}

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

// Number of XCDs on MI355X; blocks are dealt round-robin over them.
constexpr int kNumXcd = 8;

// Bijective XCD-aware remap (cdna_hip_programming.md §5 template): logical
// block ids that are consecutive land on the same XCD (shared L2).  Speed
// only, never correctness.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
    const int q = nwg / kNumXcd, r = nwg % kNumXcd;
    const int xcd = bid % kNumXcd;
    const int base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
    return base + bid / kNumXcd;
}

inline int ceil_div(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }

// Stream-ordered scratch from a library-owned memory pool per device (lib.hip):
// freed scratch (up to 1 GiB) stays mapped between calls instead of going back
// to the driver at every synchronisation (C5 TSDF: 2.32 -> 2.14 ms per call;
// tools/tsdf_call_gap.py), and buffers up to 256 MB are cached per (device, stream)
// so a call re-uses the previous call's scratch without waiting for it;
// sfmhip_scratch_trim releases both.
hipError_t scratch_alloc(void** p, size_t bytes, hipStream_t s);
// Return scratch from scratch_alloc (stream-ordered: the next call on the same stream may
// reuse it at once, its kernels run after this call's).
void scratch_free(void* p, hipStream_t s);

// Runtime knobs (INTEGRATION.md "Runtime knobs"): read from the environment once, at
// the first call; sfmhip_knobs_reload() re-reads them (tests).  Every other choice is
// fixed in the code.  knobs() returns a copy of the current snapshot (thread-safe).
struct Knobs {
    int tsdf_latency;   // SFMHIP_TSDF_LATENCY: -1 auto, 0 whole-grid mode, 1 latency mode
    int match_cert;     // SFMHIP_MATCH_CERT: 0 sends every row of the exact float mode to the f64 pass
    int ess_mono;       // SFMHIP_ESS_MONO: 1 runs the one-workgroup-per-pair essential RANSAC kernel
    int ess_rece;       // SFMHIP_ESS_RECE: essential models whose E is kept per record (0: all re-solved)
    int dlt_qr;         // SFMHIP_DLT_QR: 1 runs the QR DLT for every observation (no normal-equation pass)
    int render_sort;    // SFMHIP_RENDER_SORT: 0 renders rays in input order (no spatial sort)
    int dda_direct;     // SFMHIP_DDA_DIRECT: fill kernel of the two-pass DDA (-1 auto, 0 staged, 1 direct)
    int ab;             // SFMHIP_AB: A/B selector for a form under measurement (0 = the default form)
};
Knobs knobs();

}  // namespace sfmhip

#define SFMHIP_REQUIRE(cond, ...)                                   \
    do {                                                            \
        if (!(cond)) {                                              \
            ::sfmhip::set_error(__VA_ARGS__);                       \
            return SFMHIP_E_ARG;                                    \
        }                                                           \
    } while (0)
