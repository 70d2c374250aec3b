// Host AddressSanitizer driver for the track bookkeeping C-ABI (tracks.hip,
// matching.py:146-176 semantics).  Built by `make -C 3d_reconstruction_amd/csrc
// asan` with -fsanitize=address on the host side only; run by
// tests/test_asan_host.py.  Random tracks / matches, including the reference's
// out-of-range error paths, checked against a plain restatement of the same
// loop.  Exit status 0 and "asan tracks OK" on success.
#include <cstdint>
#include <cstdio>
#include <random>
#include <vector>

#include "../include/sfmhip.h"

namespace {

struct Ref {
    // matching.py:146-158 (p1/p2 quirk: the id image's tracks are read at p1)
    static int interlace(const std::vector<int32_t>& tr, const std::vector<int32_t>& ti,
                         const std::vector<int64_t>& i0, const std::vector<int64_t>& i1, int64_t* out) {
        int64_t c = 0;
        for (size_t m = 0; m < i0.size(); ++m) {
            const int64_t p1 = i0[m], p2 = i1[m];
            if (p1 < 0 || p1 >= (int64_t)tr.size() || p2 < 0 || p2 >= (int64_t)ti.size()) return -1;
            if (tr[p1] == -1 && ti[p2] == -1) continue;
            if (tr[p1] != -1) { ++c; continue; }
            if (p1 >= (int64_t)ti.size()) return -1;
            if (ti[p1] != -1) ++c;
        }
        *out = c;
        return 0;
    }
    // matching.py:161-176 as written (writes the reference image's tracks at p2)
    static int merge(std::vector<int32_t>& tr, std::vector<int32_t>& ti, const std::vector<int64_t>& i0,
                     const std::vector<int64_t>& i1, int64_t* nid, std::vector<int64_t>& ids) {
        for (size_t m = 0; m < i0.size(); ++m) {
            const int64_t p1 = i0[m], p2 = i1[m];
            if (p1 < 0 || p1 >= (int64_t)tr.size() || p2 < 0 || p2 >= (int64_t)ti.size()) return -1;
            if (tr[p1] == -1 && ti[p2] == -1) {
                tr[p1] = (int32_t)*nid;
                ti[p2] = (int32_t)*nid;
                ++*nid;
            } else if (tr[p1] != -1) {
                ti[p2] = tr[p1];
            } else {
                if (p1 >= (int64_t)ti.size()) return -1;
                if (ti[p1] != -1) {
                    if (p2 >= (int64_t)tr.size()) return -1;
                    tr[p2] = ti[p1];
                }
            }
            ids[m] = tr[p1];
        }
        return 0;
    }
};

}  // namespace

int main() {
    std::mt19937_64 rng(12345);
    int failures = 0, errors_seen = 0;
    for (int it = 0; it < 3000; ++it) {
        const int64_t n_ref = 1 + (int64_t)(rng() % 200), n_id = 1 + (int64_t)(rng() % 200);
        const int64_t n = (int64_t)(rng() % 150);
        std::vector<int32_t> tr((size_t)n_ref), ti((size_t)n_id);
        for (auto& v : tr) v = (rng() % 3 == 0) ? (int32_t)(rng() % 50) : -1;
        for (auto& v : ti) v = (rng() % 3 == 0) ? (int32_t)(rng() % 50) : -1;
        const bool bad = rng() % 10 == 0;   // occasionally an out-of-range match (the reference raises)
        std::vector<int64_t> i0((size_t)n), i1((size_t)n);
        for (int64_t m = 0; m < n; ++m) {
            i0[(size_t)m] = (int64_t)(rng() % (uint64_t)n_ref);
            i1[(size_t)m] = (int64_t)(rng() % (uint64_t)n_id);
        }
        if (bad && n > 0) i1[(size_t)(rng() % (uint64_t)n)] = n_id + (int64_t)(rng() % 3);

        int64_t got = -7, exp = -7;
        const int rc = sfmhip_track_interlace(tr.data(), n_ref, ti.data(), n_id, n ? i0.data() : nullptr,
                                              n ? i1.data() : nullptr, n, &got);
        const int rrc = Ref::interlace(tr, ti, i0, i1, &exp);
        if ((rc == 0) != (rrc == 0) || (rc == 0 && got != exp)) {
            std::printf("interlace mismatch it=%d rc=%d ref=%d got=%lld exp=%lld\n", it, rc, rrc, (long long)got,
                        (long long)exp);
            ++failures;
        }
        if (rc != 0) ++errors_seen;

        std::vector<int32_t> tr2 = tr, ti2 = ti, tr3 = tr, ti3 = ti;
        std::vector<int64_t> ids((size_t)n, -9), ids_ref((size_t)n, -9);
        int64_t nid = 1000, nid_ref = 1000;
        const int mc = sfmhip_track_merge(tr2.data(), n_ref, ti2.data(), n_id, n ? i0.data() : nullptr,
                                          n ? i1.data() : nullptr, n, &nid, n ? ids.data() : nullptr);
        const int mrc = Ref::merge(tr3, ti3, i0, i1, &nid_ref, ids_ref);
        if ((mc == 0) != (mrc == 0) || (mc == 0 && (tr2 != tr3 || ti2 != ti3 || ids != ids_ref || nid != nid_ref))) {
            std::printf("merge mismatch it=%d rc=%d ref=%d\n", it, mc, mrc);
            ++failures;
        }
    }
    // null-pointer and zero-length paths
    int64_t out = 0;
    if (sfmhip_track_interlace(nullptr, 0, nullptr, 0, nullptr, nullptr, 0, &out) != SFMHIP_E_ARG) ++failures;
    int32_t one = -1;
    if (sfmhip_track_interlace(&one, 1, &one, 1, nullptr, nullptr, 0, &out) != 0 || out != 0) ++failures;
    std::printf("asan tracks %s (%d error paths exercised)\n", failures ? "FAILED" : "OK", errors_seen);
    return failures ? 1 : 0;
}
