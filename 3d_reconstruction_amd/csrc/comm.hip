// comm.hip — the multi-GPU collective of the match graph (SURVEY.md §8b
// "multi-GPU" row and §8e): a thin C-ABI over RCCL, so any caller of
// libsfmhip.so (not only Python) has the pair-sharded path of dist.py.
//   * one process per GPU: sfmhip_comm_unique_id on one rank, the 128 bytes
//     broadcast by the caller (dist.RcclComm uses the torch.distributed
//     group), sfmhip_comm_init_rank everywhere (ncclCommInitRank);
//   * one process driving several GPUs: sfmhip_comm_init_all (ncclCommInitAll),
//     collectives issued between sfmhip_comm_group_start / _end.
// The match-graph exchange is ONE ncclAllGather over xGMI on the caller's
// stream (sfmhip_allgather): every rank ends with the full graph.
//
// RCCL is resolved at first use with dlopen: the RCCL already mapped into the
// process (e.g. the copy PyTorch loaded) is reused, so a process never carries
// two RCCL instances; otherwise $SFMHIP_RCCL, then the ROCm install's
// librccl.so.1.  libsfmhip.so has no link-time RCCL dependency.
#include "common.h"
#include <dlfcn.h>
#include <link.h>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>
#include <rccl/rccl.h>

namespace sfmhip {
namespace {

struct RcclApi {
    decltype(&ncclGetUniqueId) get_unique_id = nullptr;
    decltype(&ncclCommInitRank) init_rank = nullptr;
    decltype(&ncclCommInitAll) init_all = nullptr;
    decltype(&ncclAllGather) all_gather = nullptr;
    decltype(&ncclCommDestroy) destroy = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    std::string path;
    bool ok = false;
};

int find_loaded_rccl(struct dl_phdr_info* info, size_t, void* data) {
    const char* n = info->dlpi_name;
    if (n && std::strstr(n, "librccl.so")) {
        *static_cast<std::string*>(data) = n;
        return 1;
    }
    return 0;
}

template <class F>
void bind(void* h, const char* name, F& fn) {
    fn = reinterpret_cast<F>(dlsym(h, name));
}

const RcclApi& rccl() {
    static RcclApi api;
    static std::once_flag once;
    std::call_once(once, [] {
        std::string p;
        void* h = nullptr;
        dl_iterate_phdr(find_loaded_rccl, &p);
        if (!p.empty()) h = dlopen(p.c_str(), RTLD_NOW | RTLD_NOLOAD);
        const char* cands[] = {std::getenv("SFMHIP_RCCL"), "/opt/rocm/lib/librccl.so.1", "librccl.so.1", "librccl.so"};
        for (const char* c : cands) {
            if (h) break;
            if (c && *c && (h = dlopen(c, RTLD_NOW | RTLD_LOCAL)) != nullptr) p = c;
        }
        if (!h) return;
        api.path = p;
        bind(h, "ncclGetUniqueId", api.get_unique_id);
        bind(h, "ncclCommInitRank", api.init_rank);
        bind(h, "ncclCommInitAll", api.init_all);
        bind(h, "ncclAllGather", api.all_gather);
        bind(h, "ncclCommDestroy", api.destroy);
        bind(h, "ncclGetErrorString", api.error_string);
        bind(h, "ncclGroupStart", api.group_start);
        bind(h, "ncclGroupEnd", api.group_end);
        api.ok = api.get_unique_id && api.init_rank && api.init_all && api.all_gather && api.destroy &&
                 api.error_string && api.group_start && api.group_end;
    });
    return api;
}

struct Comm {
    ncclComm_t c;
    int nranks, rank, device;
};

int need_rccl(const char* what) {
    if (rccl().ok) return SFMHIP_OK;
    set_error("%s: RCCL could not be loaded (no librccl in the process, $SFMHIP_RCCL unset or invalid, "
              "/opt/rocm/lib/librccl.so.1 missing)", what);
    return SFMHIP_E_UNSUPPORTED;
}

int status(ncclResult_t r, const char* what) {
    if (r == ncclSuccess) return SFMHIP_OK;
    set_error("%s: %s (RCCL %d)", what, rccl().error_string(r), (int)r);
    return SFMHIP_E_COMM;
}

// element type -> (RCCL type, multiplier on the element count); RCCL has no
// 16-bit integer type, so int16 moves as bytes.
bool map_dtype(int dtype, ncclDataType_t* t, size_t* mult) {
    switch (dtype) {
        case SFMHIP_DT_INT8: *t = ncclInt8; *mult = 1; return true;
        case SFMHIP_DT_UINT8: *t = ncclUint8; *mult = 1; return true;
        case SFMHIP_DT_INT16: *t = ncclInt8; *mult = 2; return true;
        case SFMHIP_DT_INT32: *t = ncclInt32; *mult = 1; return true;
        case SFMHIP_DT_INT64: *t = ncclInt64; *mult = 1; return true;
        case SFMHIP_DT_FLOAT32: *t = ncclFloat32; *mult = 1; return true;
        case SFMHIP_DT_FLOAT64: *t = ncclFloat64; *mult = 1; return true;
        default: return false;
    }
}

}  // namespace
}  // namespace sfmhip

using namespace sfmhip;

extern "C" int sfmhip_comm_unique_id(void* id) {
    SFMHIP_REQUIRE(id, "sfmhip_comm_unique_id: null pointer");
    if (int rc = need_rccl("sfmhip_comm_unique_id")) return rc;
    ncclUniqueId uid;
    if (int rc = status(rccl().get_unique_id(&uid), "ncclGetUniqueId")) return rc;
    std::memcpy(id, &uid, sizeof(uid));
    return SFMHIP_OK;
}

extern "C" int sfmhip_comm_init_rank(int nranks, const void* id, int rank, void** comm) {
    SFMHIP_REQUIRE(id && comm, "sfmhip_comm_init_rank: null pointer");
    SFMHIP_REQUIRE(nranks >= 1 && rank >= 0 && rank < nranks, "sfmhip_comm_init_rank: bad rank %d of %d", rank,
                   nranks);
    if (int rc = need_rccl("sfmhip_comm_init_rank")) return rc;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) {
        (void)hipGetLastError();
        set_error("sfmhip_comm_init_rank: no current HIP device");
        return SFMHIP_E_HIP;
    }
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof(uid));
    ncclComm_t c = nullptr;
    if (int rc = status(rccl().init_rank(&c, nranks, uid, rank), "ncclCommInitRank")) return rc;
    *comm = new Comm{c, nranks, rank, dev};
    return SFMHIP_OK;
}

extern "C" int sfmhip_comm_init_all(int ndev, const int* devs, void** comms) {
    SFMHIP_REQUIRE(comms && ndev >= 1, "sfmhip_comm_init_all: bad arguments");
    if (int rc = need_rccl("sfmhip_comm_init_all")) return rc;
    std::vector<ncclComm_t> cs((size_t)ndev, nullptr);
    if (int rc = status(rccl().init_all(cs.data(), ndev, devs), "ncclCommInitAll")) return rc;
    for (int i = 0; i < ndev; ++i) comms[i] = new Comm{cs[(size_t)i], ndev, i, devs ? devs[i] : i};
    return SFMHIP_OK;
}

extern "C" int sfmhip_comm_info(void* comm, int* nranks, int* rank, int* device) {
    SFMHIP_REQUIRE(comm, "sfmhip_comm_info: null communicator");
    const Comm* c = static_cast<const Comm*>(comm);
    if (nranks) *nranks = c->nranks;
    if (rank) *rank = c->rank;
    if (device) *device = c->device;
    return SFMHIP_OK;
}

extern "C" int sfmhip_allgather(void* comm, const void* send, void* recv, size_t count, int dtype, void* stream) {
    SFMHIP_REQUIRE(comm && recv && (send || count == 0), "sfmhip_allgather: null pointer");
    ncclDataType_t t;
    size_t mult = 1;
    SFMHIP_REQUIRE(map_dtype(dtype, &t, &mult), "sfmhip_allgather: unknown dtype %d", dtype);
    if (int rc = need_rccl("sfmhip_allgather")) return rc;
    const Comm* c = static_cast<const Comm*>(comm);
    if (count == 0) return SFMHIP_OK;
    return status(rccl().all_gather(send, recv, count * mult, t, c->c, as_stream(stream)), "ncclAllGather");
}

extern "C" int sfmhip_comm_group_start(void) {
    if (int rc = need_rccl("sfmhip_comm_group_start")) return rc;
    return status(rccl().group_start(), "ncclGroupStart");
}

extern "C" int sfmhip_comm_group_end(void) {
    if (int rc = need_rccl("sfmhip_comm_group_end")) return rc;
    return status(rccl().group_end(), "ncclGroupEnd");
}

extern "C" int sfmhip_comm_destroy(void* comm) {
    if (!comm) return SFMHIP_OK;
    Comm* c = static_cast<Comm*>(comm);
    int rc = SFMHIP_OK;
    if (rccl().ok) rc = status(rccl().destroy(c->c), "ncclCommDestroy");
    delete c;
    return rc;
}
