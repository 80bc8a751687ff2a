// Ulysses SP collectives over RCCL for C-ABI hosts (include/vstyler.h, "Ulysses SP collectives").
//
// Replaces initialize_usp (reference diffsynth/pipelines/wan_video_new.py:313-323) and the
// all-to-all / all_gather of xFuserLongContextAttention (diffsynth/distributed/
// xdit_context_parallel.py:110-131, wan_video_new.py:1459-1462).  Host code only: the layout
// work around the exchange is vs_ulysses_permute(_rows) on the compute stream; here each exchange
// is one RCCL group of per-peer send/recv (RCCL routes peer traffic over xGMI links).
//
// RCCL is resolved at vs_sp_init through dlopen("librccl.so.1"): inside a PyTorch process that is
// the copy torch already loaded (same soname), elsewhere ROCm's.  Nothing else in libvstyler
// needs it, so the kernels load and run on a host without RCCL.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdio>
#include <cstring>
#include <mutex>

#include "../../include/vstyler.h"

struct vs_sp_comm {
    ncclComm_t comm;
    int rank, world, device;
};

namespace {

struct Rccl {
    decltype(&ncclGetUniqueId) get_unique_id = nullptr;
    decltype(&ncclCommInitRank) init_rank = nullptr;
    decltype(&ncclCommDestroy) destroy = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    decltype(&ncclSend) send = nullptr;
    decltype(&ncclRecv) recv = nullptr;
    decltype(&ncclAllGather) all_gather = nullptr;
    bool ok = false;
};

thread_local char g_last_error[256] = "";

void set_error(const char* what, const char* detail) {
    snprintf(g_last_error, sizeof(g_last_error), "%s%s%s", what, detail ? ": " : "", detail ? detail : "");
}

const Rccl& rccl() {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) return;
#define VS_SYM(field, name) r.field = reinterpret_cast<decltype(r.field)>(dlsym(h, name))
        VS_SYM(get_unique_id, "ncclGetUniqueId");
        VS_SYM(init_rank, "ncclCommInitRank");
        VS_SYM(destroy, "ncclCommDestroy");
        VS_SYM(error_string, "ncclGetErrorString");
        VS_SYM(group_start, "ncclGroupStart");
        VS_SYM(group_end, "ncclGroupEnd");
        VS_SYM(send, "ncclSend");
        VS_SYM(recv, "ncclRecv");
        VS_SYM(all_gather, "ncclAllGather");
#undef VS_SYM
        r.ok = r.get_unique_id && r.init_rank && r.destroy && r.error_string && r.group_start && r.group_end &&
               r.send && r.recv && r.all_gather;
    });
    return r;
}

// the loaded RCCL, or nullptr with the error recorded
const Rccl* lib() {
    const Rccl& r = rccl();
    if (!r.ok) {
        set_error("librccl.so.1 could not be loaded or lacks a symbol", dlerror());
        return nullptr;
    }
    return &r;
}

int check(const Rccl& r, ncclResult_t res, const char* what) {
    if (res == ncclSuccess) return VS_OK;
    set_error(what, r.error_string(res));
    return VS_E_COMM;
}

bool valid(const vs_sp_comm* c, const void* send, const void* recv, long long bytes) {
    return c && c->comm && send && recv && bytes > 0;
}

}  // namespace

extern "C" const char* vs_sp_last_error(void) { return g_last_error; }

extern "C" int vs_sp_unique_id(void* out_id) {
    if (!out_id) return VS_E_INVALID;
    const Rccl* r = lib();
    if (!r) return VS_E_COMM;
    ncclUniqueId id;
    const int rc = check(*r, r->get_unique_id(&id), "ncclGetUniqueId");
    if (rc == VS_OK) memcpy(out_id, &id, VS_SP_UNIQUE_ID_BYTES);
    return rc;
}

extern "C" int vs_sp_init(int rank, int world, const void* unique_id, int device, vs_sp_comm** out) {
    static_assert(sizeof(ncclUniqueId) == VS_SP_UNIQUE_ID_BYTES, "RCCL unique id size");
    if (!unique_id || !out || world < 1 || rank < 0 || rank >= world || device < 0) return VS_E_INVALID;
    *out = nullptr;
    const Rccl* r = lib();
    if (!r) return VS_E_COMM;
    // RCCL creates the communicator on the thread's current device: bind `device` for the call and
    // restore the caller's device afterwards (no side effect on the calling thread)
    int prev = -1;
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (hipSetDevice(device) != hipSuccess) {
        set_error("hipSetDevice failed", nullptr);
        return VS_E_INVALID;
    }
    ncclUniqueId id;
    memcpy(&id, unique_id, VS_SP_UNIQUE_ID_BYTES);
    ncclComm_t comm = nullptr;
    const int rc = check(*r, r->init_rank(&comm, world, id, rank), "ncclCommInitRank");
    if (prev >= 0 && prev != device) (void)hipSetDevice(prev);
    if (rc != VS_OK) return rc;
    *out = new vs_sp_comm{comm, rank, world, device};
    return VS_OK;
}

extern "C" int vs_sp_all_to_all(vs_sp_comm* c, const void* send, void* recv, long long bytes_per_rank,
                                void* stream) {
    if (!valid(c, send, recv, bytes_per_rank)) return VS_E_INVALID;
    const Rccl* r = lib();
    if (!r) return VS_E_COMM;
    const char* s = static_cast<const char*>(send);
    char* d = static_cast<char*>(recv);
    const hipStream_t st = static_cast<hipStream_t>(stream);
    int rc = check(*r, r->group_start(), "ncclGroupStart");
    if (rc != VS_OK) return rc;
    for (int j = 0; j < c->world && rc == VS_OK; ++j) {
        rc = check(*r, r->send(s + j * bytes_per_rank, (size_t)bytes_per_rank, ncclUint8, j, c->comm, st), "ncclSend");
        if (rc == VS_OK)
            rc = check(*r, r->recv(d + j * bytes_per_rank, (size_t)bytes_per_rank, ncclUint8, j, c->comm, st),
                       "ncclRecv");
    }
    const int rc_end = check(*r, r->group_end(), "ncclGroupEnd");   // always close the group
    return rc != VS_OK ? rc : rc_end;
}

extern "C" int vs_sp_all_gather(vs_sp_comm* c, const void* send, void* recv, long long bytes_per_rank,
                                void* stream) {
    if (!valid(c, send, recv, bytes_per_rank)) return VS_E_INVALID;
    const Rccl* r = lib();
    if (!r) return VS_E_COMM;
    return check(*r, r->all_gather(send, recv, (size_t)bytes_per_rank, ncclUint8, c->comm,
                                   static_cast<hipStream_t>(stream)), "ncclAllGather");
}

extern "C" int vs_sp_comm_destroy(vs_sp_comm* c) {
    if (!c) return VS_E_INVALID;
    int rc = VS_OK;
    if (c->comm) {
        const Rccl* r = lib();
        rc = r ? check(*r, r->destroy(c->comm), "ncclCommDestroy") : VS_E_COMM;
    }
    delete c;
    return rc;
}
