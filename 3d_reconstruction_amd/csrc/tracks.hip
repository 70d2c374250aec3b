// tracks.hip — host-side track bookkeeping of the match-graph consumer
// (matching.py:146-176), run on the all-gathered match
// graph.  Host memory only (no device code): sequential by definition — each
// match reads state the previous one may have written.  The reference's index
// quirks are reproduced for format parity (matching.py:157 and 169-170 index
// the id image's tracks with p1 and write the reference image's tracks at p2).
#include "common.h"

namespace {
inline bool in(int64_t v, int64_t n) { return v >= 0 && v < n; }
}  // namespace

extern "C" int sfmhip_track_interlace(const int32_t* tracks_ref, int64_t n_ref, const int32_t* tracks_id,
                                      int64_t n_id, const int64_t* idx0, const int64_t* idx1, int64_t n,
                                      int64_t* interlaced) {
    SFMHIP_REQUIRE(tracks_ref && tracks_id && interlaced && (n == 0 || (idx0 && idx1)),
                   "sfmhip_track_interlace: null pointer");
    int64_t cnt = 0;
    for (int64_t m = 0; m < n; ++m) {
        const int64_t p1 = idx0[m], p2 = idx1[m];
        SFMHIP_REQUIRE(in(p1, n_ref) && in(p2, n_id), "sfmhip_track_interlace: match %lld out of range",
                       (long long)m);
        if (tracks_ref[p1] == -1 && tracks_id[p2] == -1) continue;
        if (tracks_ref[p1] != -1) { ++cnt; continue; }
        // matching.py:157 reads the id image's tracks at p1 (IndexError there if p1 >= n_id)
        SFMHIP_REQUIRE(in(p1, n_id), "sfmhip_track_interlace: p1=%lld beyond the id image (reference raises)",
                       (long long)p1);
        if (tracks_id[p1] != -1) ++cnt;
    }
    *interlaced = cnt;
    return SFMHIP_OK;
}

extern "C" int sfmhip_track_merge(int32_t* tracks_ref, int64_t n_ref, int32_t* tracks_id, int64_t n_id,
                                  const int64_t* idx0, const int64_t* idx1, int64_t n, int64_t* next_id,
                                  int64_t* point_ids) {
    SFMHIP_REQUIRE(tracks_ref && tracks_id && next_id && (n == 0 || (idx0 && idx1 && point_ids)),
                   "sfmhip_track_merge: null pointer");
    int64_t nid = *next_id;
    for (int64_t m = 0; m < n; ++m) {
        const int64_t p1 = idx0[m], p2 = idx1[m];
        SFMHIP_REQUIRE(in(p1, n_ref) && in(p2, n_id), "sfmhip_track_merge: match %lld out of range", (long long)m);
        if (tracks_ref[p1] == -1 && tracks_id[p2] == -1) {
            tracks_ref[p1] = (int32_t)nid;
            tracks_id[p2] = (int32_t)nid;
            ++nid;
        } else if (tracks_ref[p1] != -1) {
            tracks_id[p2] = tracks_ref[p1];
        } else {
            SFMHIP_REQUIRE(in(p1, n_id), "sfmhip_track_merge: p1 beyond the id image (reference raises)");
            if (tracks_id[p1] != -1) {   // matching.py:169-170 as written
                SFMHIP_REQUIRE(in(p2, n_ref), "sfmhip_track_merge: p2 beyond the reference image (reference raises)");
                tracks_ref[p2] = tracks_id[p1];
            }
        }
        point_ids[m] = tracks_ref[p1];
    }
    *next_id = nid;
    return SFMHIP_OK;
}
