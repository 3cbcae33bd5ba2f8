// handle.hpp -- the rsvd handle (one GPU + stream + workspace) shared by the narrow engine
// (driver.cpp) and the wide engine (wide.cpp).  Private to librsvd_hip.so.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <string>
#include <utility>
#include <vector>

#include "../../include/rsvd_c.h"

struct rsvd_handle_s {
    int device = 0;
    hipStream_t stream = nullptr;
    bool own_stream = false;
    std::string err;
    char* ws = nullptr;
    size_t ws_bytes = 0;
    bool ws_external = false;  // workspace supplied by the caller (rsvd_set_workspace)
    // device flags: [1] jacobi sweeps, [4..15] per-orthonormalisation breakdown flags, [16]
    // power-method triplets kept -- reset at the start of every run; and the STICKY error words
    // (kept across queued runs, cleared when rsvd_sync / rsvd_get_info report them):
    // [2] Gram hand-off timeout, [3] block-Jacobi barrier timeout, [20] a rank-deficiency repair
    // pass that broke down again, [21] non-finite singular values, [22] a row-sharded run whose global
    // row count is below l.
    int* dflags = nullptr;
    rsvd_info_t info{};
    int rank = 0, world = 1;
    rsvd_allreduce_fn allreduce = nullptr;
    void* ar_user = nullptr;
    rsvd_collective_fn coll = nullptr;  // n-side sharding (wide engine), rsvd_set_collectives
    void* coll_user = nullptr;
    void* nccl = nullptr;  // library-owned RCCL communicator (rsvd_comm_init, comm.cpp)
    // timing mode: hipEvent pairs around every projection kernel (kind 0 = A*X, 1 = A^T*Q, 2 = the
    // sketch A*Omega, which also counts as kind 0)
    bool timing = false;
    std::vector<hipEvent_t> ev_pool;
    std::vector<std::pair<int, int>> ev_used;  // (kind, first event index)
    size_t ev_next = 0;
    double acc_ms[3] = {0.0, 0.0, 0.0};
    int acc_n[3] = {0, 0, 0};
};

#define RSVD_CK(expr)                                                                         \
    do {                                                                                      \
        hipError_t _e = (expr);                                                               \
        if (_e == hipErrorCooperativeLaunchTooLarge) {                                        \
            /* a persistent grid the device cannot hold at once (launch_coresident) */        \
            h->err = std::string(#expr) + ": persistent grid exceeds the device's co-resident " \
                     "workgroup capacity (size not supported on this device)";                \
            return RSVD_ERR_UNSUPPORTED;                                                      \
        }                                                                                     \
        if (_e != hipSuccess) {                                                               \
            h->err = std::string(#expr) + ": " + hipGetErrorString(_e);                       \
            return RSVD_ERR_HIP;                                                              \
        }                                                                                     \
    } while (0)

#define RSVD_TRY(expr)                   \
    do {                                 \
        int _s = (expr);                 \
        if (_s != RSVD_OK) return _s;    \
    } while (0)

constexpr int kFlagWords = 32;
constexpr int kFlagGramTimeout = 2, kFlagJacobiTimeout = 3, kFlagUnrepaired = 20, kFlagNonFinite = 21,
              kFlagFewRows = 22;
// the split-Gram fallback test (wide.cpp cholqr_pass) and its factor's breakdown count (never read)
constexpr int kFlagSplitIll = 24, kFlagSplitScratch = 25;
// the deferred second pass's G^-1/2 series (wide.cpp orth2_deferred): [0] series applies, [1] the Cholesky runs
constexpr int kFlagIsqrt = 26;

// Per-run reset of the non-sticky flag words ([0..1] and [4..19]; the sticky words stay).
inline hipError_t reset_run_flags(int* dflags, hipStream_t s) {
    hipError_t e = hipMemsetAsync(dflags, 0, 2 * sizeof(int), s);
    if (e != hipSuccess) return e;
    return hipMemsetAsync(dflags + 4, 0, 16 * sizeof(int), s);
}

namespace rsvd {
// comm.cpp: release the library-owned RCCL communicator (no-op without one)
void release_comm(rsvd_handle_t h);
}  // namespace rsvd

inline int lp_of(int l) { return (l + 15) / 16 * 16; }
inline size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

inline int ensure_ws(rsvd_handle_t h, size_t bytes) {
    if (bytes <= h->ws_bytes) return RSVD_OK;
    if (h->ws_external) {
        h->err = "caller workspace too small: need " + std::to_string(bytes) + " bytes";
        return RSVD_ERR_INVALID_ARG;
    }
    if (h->ws) {
        RSVD_CK(hipStreamSynchronize(h->stream));
        RSVD_CK(hipFree(h->ws));
        h->ws = nullptr;
        h->ws_bytes = 0;
    }
    RSVD_CK(hipMalloc(&h->ws, bytes));
    h->ws_bytes = bytes;
    return RSVD_OK;
}

