// lib.hip — library-level entry points: version, thread-local error, arch probe.
#include "common.h"
#include <cstring>
#include <cstdlib>
#include <mutex>

namespace sfmhip {
static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

// Library-owned pool per device (created once, std::call_once): the device's
// default pool, which other hipMallocAsync users share, is never touched.  Up to
// kScratchKeep bytes of freed scratch stay mapped between calls (at a zero
// threshold the pool returned it at every synchronisation and re-mapped it on
// the next call: C5 TSDF 2.32 -> 2.14 ms per call, tools/tsdf_call_gap.py);
// sfmhip_scratch_trim releases it.
constexpr int kMaxDev = 64;
constexpr uint64_t kScratchKeep = 1ull << 30;
static hipMemPool_t g_pool[kMaxDev];
static std::once_flag g_pool_once[kMaxDev];

static hipMemPool_t scratch_pool(int dev) {
    if (dev < 0 || dev >= kMaxDev) return nullptr;
    std::call_once(g_pool_once[dev], [dev] {
        hipMemPoolProps props = {};
        props.allocType = hipMemAllocationTypePinned;
        props.handleTypes = hipMemHandleTypeNone;
        props.location.type = hipMemLocationTypeDevice;
        props.location.id = dev;
        hipMemPool_t pool = nullptr;
        if (hipMemPoolCreate(&pool, &props) == hipSuccess) {
            uint64_t thr = kScratchKeep;
            (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &thr);
            g_pool[dev] = pool;
        }
        (void)hipGetLastError();
    });
    return g_pool[dev];
}

static hipError_t pool_alloc(void** p, size_t bytes, hipStream_t s, int dev, bool have_dev) {
    if (have_dev) {
        if (hipMemPool_t pool = scratch_pool(dev)) return hipMallocFromPoolAsync(p, bytes, pool, s);
    }
    (void)hipGetLastError();
    return hipMallocAsync(p, bytes, s);
}

// Per-stream scratch cache: a pool allocation + free per call made the host wait for the
// previous call's kernels (hipMallocFromPoolAsync re-using memory freed on the stream: the
// enqueue cost of the BA-obs step equalled its GPU time, tools/ba_host_overhead.py).  Buffers
// up to kCacheMax bytes are kept per (device, stream) and handed out again to a later call on
// the same stream — stream order makes that safe with no wait; sfmhip_scratch_trim releases
// them.  Larger ones go straight back to the pool.
constexpr int kCacheSlots = 32;
constexpr size_t kCacheMax = 256ull << 20;     // larger buffers are not cached
constexpr size_t kCacheTotal = 1ull << 30;     // bytes held by the cache at most
struct CacheSlot {
    void* p;
    size_t bytes;
    hipStream_t s;
    int dev;
    bool busy;
};
static CacheSlot g_cache[kCacheSlots];
static std::mutex g_cache_mu;

// Return one idle cached buffer to the pool.  The slot's stream may have been destroyed by the
// caller since it was cached (sfmhip_scratch_release_stream is the clean way out): HIP then
// refuses the stream-ordered free, so the buffer is freed after a device synchronisation (all
// work of a destroyed stream has been issued already) and the error is cleared, so that the
// caller's next launch check does not report it.
static void release_slot(CacheSlot& c) {
    if (hipFreeAsync(c.p, c.s) != hipSuccess) {
        (void)hipGetLastError();
        int cur = -1;
        const bool have = hipGetDevice(&cur) == hipSuccess;
        if (!have || cur != c.dev) (void)hipSetDevice(c.dev);   // the buffer's own device
        (void)hipDeviceSynchronize();
        (void)hipFree(c.p);
        if (have && cur != c.dev) (void)hipSetDevice(cur);
    }
    (void)hipGetLastError();
    c = CacheSlot{};
}

hipError_t scratch_alloc(void** p, size_t bytes, hipStream_t s) {
    int dev = 0;
    const bool have_dev = hipGetDevice(&dev) == hipSuccess;
    if (!have_dev) (void)hipGetLastError();
    if (bytes == 0) bytes = 1;
    if (bytes > kCacheMax || !have_dev) return pool_alloc(p, bytes, s, dev, have_dev);
    std::lock_guard<std::mutex> lk(g_cache_mu);
    int best = -1, empty = -1;
    for (int i = 0; i < kCacheSlots; ++i) {
        CacheSlot& c = g_cache[i];
        if (!c.p) {
            if (empty < 0) empty = i;
        } else if (!c.busy && c.s == s && c.dev == dev && c.bytes >= bytes &&
                   (best < 0 || c.bytes < g_cache[best].bytes)) {
            best = i;
        }
    }
    if (best >= 0) {
        g_cache[best].busy = true;
        *p = g_cache[best].p;
        return hipSuccess;
    }
    if (empty < 0) {   // table full: drop the smallest idle buffer of this device, else allocate uncached
        for (int i = 0; i < kCacheSlots; ++i)
            if (!g_cache[i].busy && g_cache[i].dev == dev && (empty < 0 || g_cache[i].bytes < g_cache[empty].bytes))
                empty = i;
        if (empty >= 0) release_slot(g_cache[empty]);
    }
    const hipError_t e = pool_alloc(p, bytes, s, dev, true);
    if (e == hipSuccess && empty >= 0) {
        g_cache[empty] = CacheSlot{*p, bytes, s, dev, true};
        size_t held = 0;   // keep at most kCacheTotal bytes cached: drop idle buffers, largest first
        for (const auto& c : g_cache) held += c.bytes;
        while (held > kCacheTotal) {
            int big = -1;
            for (int i = 0; i < kCacheSlots; ++i)
                if (g_cache[i].p && !g_cache[i].busy && g_cache[i].dev == dev &&
                    (big < 0 || g_cache[i].bytes > g_cache[big].bytes))
                    big = i;
            if (big < 0) break;
            held -= g_cache[big].bytes;
            release_slot(g_cache[big]);
        }
    }
    return e;
}

void scratch_free(void* p, hipStream_t s) {
    if (!p) return;
    {
        std::lock_guard<std::mutex> lk(g_cache_mu);
        for (int i = 0; i < kCacheSlots; ++i)
            if (g_cache[i].p == p) {
                g_cache[i].busy = false;
                return;
            }
    }
    (void)hipFreeAsync(p, s);
}

static int env_knob(const char* name, int dflt) {
    const char* e = std::getenv(name);
    return e && *e ? std::atoi(e) : dflt;
}
static Knobs read_knobs() {
    Knobs k;
    k.tsdf_latency = env_knob("SFMHIP_TSDF_LATENCY", -1);
    k.match_cert = env_knob("SFMHIP_MATCH_CERT", 1);
    k.ess_mono = env_knob("SFMHIP_ESS_MONO", 0);
    k.ess_rece = env_knob("SFMHIP_ESS_RECE", 1 << 20);
    k.dlt_qr = env_knob("SFMHIP_DLT_QR", 0);
    k.render_sort = env_knob("SFMHIP_RENDER_SORT", 1);
    k.dda_direct = env_knob("SFMHIP_DDA_DIRECT", -1);
    k.ab = env_knob("SFMHIP_AB", 0);
    return k;
}
// Immutable snapshots: knobs() copies the current one out under the lock, so a reload while
// another thread is inside a library call never hands that call a torn mix of old and new
// values (superseded snapshots are kept: a reload is a test-time event, a few dozen bytes each).
static std::mutex g_knobs_mu;
static const Knobs* g_knobs = nullptr;
Knobs knobs() {
    std::lock_guard<std::mutex> lk(g_knobs_mu);
    if (!g_knobs) g_knobs = new Knobs(read_knobs());
    return *g_knobs;
}
}  // namespace sfmhip

// Re-read the runtime knobs from the environment (tests that switch a knob between
// calls); calls already running keep the snapshot they took.
extern "C" int sfmhip_knobs_reload(void) {
    const sfmhip::Knobs* k = new sfmhip::Knobs(sfmhip::read_knobs());
    std::lock_guard<std::mutex> lk(sfmhip::g_knobs_mu);
    sfmhip::g_knobs = k;
    return SFMHIP_OK;
}

// 0.3.0: sfmhip_match_pairs_i16 / sfmhip_match_pairs_exact_i16 (the int16 graph written by the kernels)
// 0.2.0: sfmhip_ba_solve takes n_obs (between n_pairs and ftol); sfmhip_scratch_release_stream
extern "C" int sfmhip_version(void) { return (0 << 16) | (3 << 8) | 0; }

extern "C" const char* sfmhip_last_error(void) { return sfmhip::g_err; }

extern "C" int sfmhip_scratch_trim(uint64_t keep) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) {
        (void)hipGetLastError();
        sfmhip::set_error("sfmhip_scratch_trim: no current HIP device");
        return SFMHIP_E_HIP;
    }
    {   // the idle cached buffers of this device go back to the pool first
        std::lock_guard<std::mutex> lk(sfmhip::g_cache_mu);
        for (auto& c : sfmhip::g_cache)
            if (c.p && !c.busy && c.dev == dev) sfmhip::release_slot(c);
    }
    (void)hipDeviceSynchronize();
    hipMemPool_t pool = sfmhip::scratch_pool(dev);
    if (!pool) return SFMHIP_OK;
    const hipError_t e = hipMemPoolTrimTo(pool, (size_t)keep);
    if (e != hipSuccess) {
        sfmhip::set_error("sfmhip_scratch_trim: %s", hipGetErrorString(e));
        return SFMHIP_E_HIP;
    }
    return SFMHIP_OK;
}

extern "C" int sfmhip_device_arch(char* buf, int len) {
    SFMHIP_REQUIRE(buf != nullptr && len > 0, "sfmhip_device_arch: null buffer");
    hipDeviceProp_t prop;
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e == hipSuccess) e = hipGetDeviceProperties(&prop, dev);
    if (e != hipSuccess) {
        sfmhip::set_error("hipGetDeviceProperties: %s", hipGetErrorString(e));
        return SFMHIP_E_HIP;
    }
    std::strncpy(buf, prop.gcnArchName, (size_t)len - 1);
    buf[len - 1] = '\0';
    return SFMHIP_OK;
}

// Release the idle scratch cached for `stream` (call before destroying a stream that was passed
// to the library; buffers of a destroyed stream are otherwise freed at the next eviction or trim).
extern "C" int sfmhip_scratch_release_stream(void* stream) {
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    std::lock_guard<std::mutex> lk(sfmhip::g_cache_mu);
    for (auto& c : sfmhip::g_cache)
        if (c.p && !c.busy && c.s == s) sfmhip::release_slot(c);
    return SFMHIP_OK;
}
