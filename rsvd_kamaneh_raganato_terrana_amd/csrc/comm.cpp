// comm.cpp -- library-owned RCCL for C / C++ callers (rsvd_comm_unique_id / rsvd_comm_init,
// include/rsvd_c.h ABI 6).
//
// The reference runs rSVD() collectively on the MPI ranks of MPI_COMM_WORLD (src/rSVD.cpp:15,
// 20-23, Gatherv + Bcast of Omega at :49,52).  Here each rank drives one GPU and the handle owns an
// RCCL communicator over xGMI: the engine's exchange points (the l x l Gram all-reduce of the m-side
// CholeskyQR, the reduce-scatter of A^T Q and the all-gathers of the n-side panels, wide.cpp) call
// ncclAllReduce / ncclReduceScatter / ncclAllGather on the handle's stream -- the same entry points
// the Python front end reaches through torch.distributed, without a host round trip or a hook.
//
// librccl is opened on first use (dlopen), so the engine itself has no link-time dependency on it
// and a process that never shards never loads it.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstring>
#include <mutex>
#include <string>

#include "../../include/rsvd_c.h"
#include "handle.hpp"

namespace {

struct Rccl {
    void* so = nullptr;
    decltype(&ncclGetUniqueId) get_unique_id = nullptr;
    decltype(&ncclCommInitRank) comm_init_rank = nullptr;
    decltype(&ncclCommDestroy) comm_destroy = nullptr;
    decltype(&ncclAllReduce) all_reduce = nullptr;
    decltype(&ncclReduceScatter) reduce_scatter = nullptr;
    decltype(&ncclAllGather) all_gather = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
    std::string why;
};

Rccl& rccl_state() {
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        for (const char* name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"}) {
            r.so = dlopen(name, RTLD_NOW | RTLD_LOCAL);
            if (r.so) break;
        }
        if (!r.so) {
            const char* e = dlerror();
            r.why = std::string("cannot load librccl: ") + (e ? e : "?");
            return;
        }
        auto sym = [](const char* s) { return dlsym(r.so, s); };
        r.get_unique_id = reinterpret_cast<decltype(r.get_unique_id)>(sym("ncclGetUniqueId"));
        r.comm_init_rank = reinterpret_cast<decltype(r.comm_init_rank)>(sym("ncclCommInitRank"));
        r.comm_destroy = reinterpret_cast<decltype(r.comm_destroy)>(sym("ncclCommDestroy"));
        r.all_reduce = reinterpret_cast<decltype(r.all_reduce)>(sym("ncclAllReduce"));
        r.reduce_scatter = reinterpret_cast<decltype(r.reduce_scatter)>(sym("ncclReduceScatter"));
        r.all_gather = reinterpret_cast<decltype(r.all_gather)>(sym("ncclAllGather"));
        r.error_string = reinterpret_cast<decltype(r.error_string)>(sym("ncclGetErrorString"));
        if (!r.get_unique_id || !r.comm_init_rank || !r.comm_destroy || !r.all_reduce || !r.reduce_scatter ||
            !r.all_gather || !r.error_string) {
            r.why = "librccl lacks an entry point the engine needs";
            dlclose(r.so);
            r.so = nullptr;
        }
    });
    return r;
}

Rccl* rccl() {
    Rccl& r = rccl_state();
    return r.so ? &r : nullptr;
}

const char* rccl_why() { return rccl_state().why.c_str(); }

bool nccl_type(int32_t dtype, ncclDataType_t* t) {
    switch (dtype) {
        case RSVD_F64: *t = ncclFloat64; return true;
        case RSVD_F32: *t = ncclFloat32; return true;
        case RSVD_BF16: *t = ncclBfloat16; return true;
        default: return false;
    }
}

// rsvd_allreduce_fn over the handle's communicator (user = the handle)
int rccl_allreduce(void* buf, int64_t count, int32_t dtype, void* stream, void* user) {
    auto* h = static_cast<rsvd_handle_t>(user);
    Rccl* r = rccl();
    ncclDataType_t t;
    if (!r || !h || !h->nccl || !nccl_type(dtype, &t) || count < 0) return 1;
    const ncclResult_t e = r->all_reduce(buf, buf, (size_t)count, t, ncclSum, static_cast<ncclComm_t>(h->nccl),
                                         static_cast<hipStream_t>(stream));
    if (e != ncclSuccess) h->err = std::string("ncclAllReduce: ") + r->error_string(e);
    return e == ncclSuccess ? 0 : 1;
}

// rsvd_collective_fn: reduce-scatter (recv may be send + rank count: RCCL's in-place form) and
// all-gather (send may be recv + rank count)
int rccl_collective(int32_t op, void* send, void* recv, int64_t count, int32_t dtype, void* stream, void* user) {
    auto* h = static_cast<rsvd_handle_t>(user);
    Rccl* r = rccl();
    ncclDataType_t t;
    if (!r || !h || !h->nccl || !nccl_type(dtype, &t) || count < 0) return 1;
    auto comm = static_cast<ncclComm_t>(h->nccl);
    auto s = static_cast<hipStream_t>(stream);
    ncclResult_t e;
    if (op == RSVD_COLL_REDUCE_SCATTER) {
        e = r->reduce_scatter(send, recv, (size_t)count, t, ncclSum, comm, s);
    } else if (op == RSVD_COLL_ALL_GATHER) {
        e = r->all_gather(send, recv, (size_t)count, t, comm, s);
    } else {
        return 1;
    }
    if (e != ncclSuccess) h->err = std::string(op == RSVD_COLL_REDUCE_SCATTER ? "ncclReduceScatter: " : "ncclAllGather: ") +
                                   r->error_string(e);
    return e == ncclSuccess ? 0 : 1;
}

}  // namespace

namespace rsvd {
// Release the handle's communicator (rsvd_destroy, a replacement by rsvd_set_comm / rsvd_comm_init).
void release_comm(rsvd_handle_t h) {
    if (!h || !h->nccl) return;
    if (Rccl* r = rccl()) {
        (void)hipSetDevice(h->device);
        if (h->stream) (void)hipStreamSynchronize(h->stream);
        (void)r->comm_destroy(static_cast<ncclComm_t>(h->nccl));
    }
    h->nccl = nullptr;
    if (h->allreduce == rccl_allreduce) h->allreduce = nullptr, h->ar_user = nullptr;
    if (h->coll == rccl_collective) h->coll = nullptr, h->coll_user = nullptr;
}
}  // namespace rsvd

extern "C" {

int rsvd_comm_unique_id(void* id) {
    if (!id) return RSVD_ERR_INVALID_ARG;
    Rccl* r = rccl();
    if (!r) return RSVD_ERR_UNSUPPORTED;
    static_assert(sizeof(ncclUniqueId) == RSVD_COMM_ID_BYTES, "ncclUniqueId size");
    ncclUniqueId u;
    if (r->get_unique_id(&u) != ncclSuccess) return RSVD_ERR_COMM;
    std::memcpy(id, &u, sizeof(u));
    return RSVD_OK;
}

int rsvd_comm_init(rsvd_handle_t h, const void* id, int rank, int world, int shard_n) {
    if (!h || !id || world < 1 || world > 64 || rank < 0 || rank >= world) return RSVD_ERR_INVALID_ARG;
    Rccl* r = rccl();
    if (!r) {
        h->err = rccl_why();
        return RSVD_ERR_UNSUPPORTED;
    }
    rsvd::release_comm(h);
    if (hipSetDevice(h->device) != hipSuccess) return RSVD_ERR_HIP;
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof(u));
    ncclComm_t comm = nullptr;
    const ncclResult_t e = r->comm_init_rank(&comm, world, u, rank);
    if (e != ncclSuccess) {
        h->err = std::string("ncclCommInitRank: ") + r->error_string(e);
        return RSVD_ERR_COMM;
    }
    h->nccl = comm;
    h->rank = rank;
    h->world = world;
    h->allreduce = rccl_allreduce;
    h->ar_user = h;
    h->coll = shard_n ? rccl_collective : nullptr;
    h->coll_user = shard_n ? h : nullptr;
    return RSVD_OK;
}

int rsvd_comm_destroy(rsvd_handle_t h) {
    if (!h) return RSVD_ERR_INVALID_ARG;
    const bool had = h->nccl != nullptr;
    rsvd::release_comm(h);
    if (had) {
        h->rank = 0;
        h->world = 1;
    }
    return RSVD_OK;
}

}  // extern "C"
