// driver.cpp -- native host orchestration of the MI355X rSVD and the C ABI (include/rsvd_c.h).
//
// One handle = one GPU + one HIP stream + a lazily grown device workspace.  rsvd_run enqueues
// the whole randomized SVD of src/rSVD.cpp:72-133 on the stream without host synchronisation:
//
//   Omega (Philox, util.hip)                            generateOmega        src/rSVD.cpp:81
//   Y = A Omega (proj_nn) ; Q = orth(Y) (qr.hip)        intermediate_step    src/rSVD.cpp:59-61
//   q x { Z = A^T Q ; Q_n = orth(Z) ; Y = A Q_n ; Q = orth(Y) }                src/rSVD.cpp:62-69
//   B^T = A^T Q (proj_tn) ; B^T = Q_B R                 B = Q^T A + the QR   src/rSVD.cpp:89,
//                                                       preconditioning of   SVD_class.hpp:116-123
//   W = R^T = U_w S V_w^T (jacobi.hip)                  SVD<Jacobi>          SVD_class.hpp:126-178
//   U = Q U_w ; V = Q_B V_w (panel_small)               U = Q * Utilde       src/rSVD.cpp:128
//
// Row-sharded runs (world > 1) go to the wide engine (wide.cpp), which owns the distributed
// orthonormalisation (Gram all-reduce, rank-deficiency repair with disjoint Philox draws per rank)
// for every l and dtype; this narrow engine is the single-GPU fast path for fp32 / fp64, l <= 64.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/rsvd_c.h"
#include "handle.hpp"
#include "kernels.hpp"
#include "dense.hpp"
#include "wide.hpp"

using namespace rsvd;

namespace {

template <typename T>
struct Layout {
    int64_t m, n;
    int l, LP;
    ProjPlan pnn, ptn;
    int gram_m, gram_n;
    size_t off_Xn, off_Zn, off_Ym, off_Qm, off_T1, off_slab, off_gram, off_small, off_ctr, total;

    Layout(int64_t m_, int64_t n_, int l_) : m(m_), n(n_), l(l_), LP(lp_of(l_)) {
        pnn = plan_proj_nn<T>(m, n, LP);
        ptn = plan_proj_tn<T>(m, n, LP);
        gram_m = plan_gram_blocks(m);
        gram_n = plan_gram_blocks(n);
        const int64_t mx = std::max(m, n);
        size_t o = 0;
        off_Xn = o; o = align256(o + sizeof(T) * n * LP);
        off_Zn = o; o = align256(o + sizeof(T) * n * LP);
        off_Ym = o; o = align256(o + sizeof(T) * m * LP);
        off_Qm = o; o = align256(o + sizeof(T) * m * LP);
        off_T1 = o; o = align256(o + sizeof(T) * mx * LP);
        const int64_t slab_elems = std::max<int64_t>(pnn.splits > 1 ? pnn.splits * m : 0,
                                                     ptn.splits > 1 ? ptn.splits * n : 0);
        off_slab = o; o = align256(o + sizeof(T) * std::max<int64_t>(slab_elems, 1) * LP);
        off_gram = o; o = align256(o + sizeof(double) * 33 * LP * LP);  // <= 32 Gram slabs + reduced tiles
        off_small = o; o = align256(o + sizeof(double) * 8 * LP * LP);  // R1, R2, Rinv, Uw, Vw, Gsum
        off_ctr = o; o = align256(o + 64 * sizeof(unsigned));           // arrival counters
        total = o;
    }
};

// A = a_scale * (stored A); 0 means 1 (rsvd_c.h)
double a_scale_of(const rsvd_desc_t* d) { return d->a_scale != 0.0 ? d->a_scale : 1.0; }

// world: the handle's rank count (0 = unknown, e.g. a workspace-size query).  On a row-sharded handle
// d->m is this rank's share, which may hold fewer rows than l (src/rSVD.cpp:20-23 partitions the
// global m): the engines then check l against the global row count themselves.
int check_desc_msg(const rsvd_desc_t* d, const char** err, int world = 1) {
    if (!d) { *err = "null descriptor"; return RSVD_ERR_INVALID_ARG; }
    if (d->m <= 0 || d->n <= 0 || d->l <= 0 || d->q < 0 || d->lda < d->m) {
        *err = "invalid sizes (need m, n, l > 0, q >= 0, lda >= m)";
        return RSVD_ERR_INVALID_ARG;
    }
    if (d->dtype < RSVD_F64 || d->dtype > RSVD_FP8_E4M3) { *err = "unsupported dtype"; return RSVD_ERR_UNSUPPORTED; }
    if (d->qr_mode < RSVD_QR_AUTO || d->qr_mode > RSVD_QR_CHOLQR2) { *err = "bad qr_mode"; return RSVD_ERR_INVALID_ARG; }
    if (d->flags & ~(RSVD_FLAG_LOWP_INTERMEDIATES | RSVD_FLAG_FORCE_NSHARD)) { *err = "unknown flags"; return RSVD_ERR_INVALID_ARG; }
    if (d->method != RSVD_SVD_JACOBI && d->method != RSVD_SVD_PARALLEL_JACOBI && d->method != RSVD_SVD_POWER &&
        d->method != RSVD_SVD_POWER_IC) {
        *err = "Unsupported SVD method";  // src/rSVD.cpp:123 wording
        return RSVD_ERR_UNSUPPORTED;
    }
    if (d->l > kBigLMax) { *err = "l > 4096 not supported"; return RSVD_ERR_UNSUPPORTED; }
    if (d->l > d->n || (world == 1 && d->l > d->m)) { *err = "l > min(m, n) not supported"; return RSVD_ERR_UNSUPPORTED; }
    if (!std::isfinite(d->a_scale)) { *err = "a_scale is not finite"; return RSVD_ERR_INVALID_ARG; }
    return RSVD_OK;
}

int check_desc(rsvd_handle_t h, const rsvd_desc_t* d) {
    const char* err = "";
    const int st = check_desc_msg(d, &err, h->world);
    if (st != RSVD_OK) h->err = err;
    return st;
}

// ---- the pipeline ---------------------------------------------------------------------------
template <typename T>
struct Engine {
    rsvd_handle_t h;
    const Layout<T>& L;
    hipStream_t s;
    T *Xn, *Zn, *Ym, *Qm, *T1, *slab;
    double *gram, *R1, *R2, *Rinv, *Uw, *Vw, *Gsum;
    unsigned* ctr;
    unsigned tgt0 = 0, tgt1 = 0;  // run-cumulative arrival targets of gram_chol (counters zeroed per run)
    // fp32 panels that only carry a subspace (power-iteration intermediates) get one CholeskyQR
    // pass; panels whose basis is an output (final Q, Q_B) and every fp64 panel get two.
    int inter_passes = sizeof(T) == 4 ? 1 : 2;
    int qr_mode = RSVD_QR_AUTO;

    Engine(rsvd_handle_t h_, const Layout<T>& L_) : h(h_), L(L_), s(h_->stream) {
        char* b = h->ws;
        Xn = reinterpret_cast<T*>(b + L.off_Xn);
        Zn = reinterpret_cast<T*>(b + L.off_Zn);
        Ym = reinterpret_cast<T*>(b + L.off_Ym);
        Qm = reinterpret_cast<T*>(b + L.off_Qm);
        T1 = reinterpret_cast<T*>(b + L.off_T1);
        slab = reinterpret_cast<T*>(b + L.off_slab);
        gram = reinterpret_cast<double*>(b + L.off_gram);
        double* sm = reinterpret_cast<double*>(b + L.off_small);
        const int64_t q2 = (int64_t)L.LP * L.LP;
        R1 = sm; R2 = sm + q2; Rinv = sm + 2 * q2; Uw = sm + 3 * q2; Vw = sm + 4 * q2; Gsum = sm + 5 * q2;
        ctr = reinterpret_cast<unsigned*>(b + L.off_ctr);
    }

    // Per-orth breakdown flags live at dflags[4 + k] (k = orth index within the run, < 12).
    int orth_index = 0;
    int* cur_flag = nullptr;

    // One CholeskyQR pass: R = chol(P^T P), Out = P R^-1 (Out may alias P: panel_small stages its
    // rows before writing).  f32: factor in fp32 (the subspace-only intermediates of the fp32 path,
    // see qr.hip) or fp64.  pred: a predicated pass (skipped unless *pred != 0) on counters of its
    // own.  refine: receives the need for a second pass (cond_F(R) too large for one, or a breakdown).
    int npred = 0, nref = 0;
    int cholqr_pass(const T* P, int64_t rows, T* Out, int f32, const int* pred = nullptr, int* refine = nullptr) {
        const int nb = plan_gram_blocks(rows);
        double* tiles = gram + 32 * (size_t)L.LP * L.LP;
        unsigned* c = ctr;
        unsigned t0, t1;
        if (pred) {  // private arrival counters (ctr[8 ..]): skipping this launch leaves the others' targets intact
            c = ctr + 8 + 2 * (npred++ % 26);
            t0 = (unsigned)nb;
            t1 = (unsigned)gram_tiles(L.LP, 0);
        } else {
            tgt0 += nb;
            tgt1 += gram_tiles(L.LP, 0);
            t0 = tgt0;
            t1 = tgt1;
        }
        RSVD_CK(launch_gram_chol<T>(P, rows, L.LP, nb, gram, tiles, c, t0, t1, 1, f32, nullptr, L.l, R1, Rinv,
                                    cur_flag, h->dflags + kFlagGramTimeout, s, pred, refine));
        RSVD_CK(launch_panel_small<T>(P, rows, L.LP, Rinv, Out, 0, 0, 0, s, pred));
        return RSVD_OK;
    }

    // CholeskyQR (passes = 1: the subspace-only intermediates) or an output panel (passes = 2).
    // Output panels of the fp32 path factor in fp64 and run the second CholeskyQR pass only when
    // the first one's R is too ill-conditioned for one pass (device-side predicate); fp64 panels
    // and qr_mode CHOLQR2 always run two.  Output panels keep the predicated fallback that
    // rebuilds Q from P (CGS2 + random completion, util.hip) if any pass flagged a bad pivot.
    int orth(const T* P, int64_t rows, T* Q, int passes) {
        cur_flag = h->dflags + 4 + (orth_index < 12 ? orth_index : 11);
        ++orth_index;
        if (qr_mode == RSVD_QR_GS2) {  // always the Gram-Schmidt path
            RSVD_CK(hipMemsetAsync(cur_flag, 0xFF, sizeof(int), s));
            RSVD_CK(launch_robust_orth<T>(P, rows, L.l, L.LP, Q, cur_flag, 0x5EEDull + orth_index, s));
            return RSVD_OK;
        }
        if (qr_mode == RSVD_QR_CHOLQR2) passes = 2;
        const bool output = passes >= 2;
        const int f32 = sizeof(T) == 4;
        if (!output) {
            RSVD_TRY(cholqr_pass(P, rows, Q, f32));
        } else if (f32 && qr_mode == RSVD_QR_AUTO) {
            int* refine = reinterpret_cast<int*>(ctr + 62 + (nref++ & 1));
            RSVD_TRY(cholqr_pass(P, rows, Q, 0, nullptr, refine));
            RSVD_TRY(cholqr_pass(Q, rows, Q, 0, refine, nullptr));
        } else {
            RSVD_TRY(cholqr_pass(P, rows, T1, f32));
            RSVD_TRY(cholqr_pass(T1, rows, Q, f32));
        }
        if (output) RSVD_CK(launch_robust_orth<T>(P, rows, L.l, L.LP, Q, cur_flag, 0x5EEDull + orth_index, s));
        return RSVD_OK;
    }

    // Gout = P^T P2 (fp64), e.g. R = Q_B^T B^T for the small SVD.
    int cross_gram(const T* P, const T* P2, int64_t rows, double* Gout) {
        const int nb = plan_gram_blocks(rows);
        double* tiles = gram + 32 * (size_t)L.LP * L.LP;
        tgt0 += nb;
        tgt1 += gram_tiles(L.LP, 1);
        RSVD_CK(launch_cross_gram<T>(P, P2, rows, L.LP, nb, gram, tiles, ctr, tgt0, tgt1, Gout, L.l,
                                     h->dflags + kFlagGramTimeout, s));
        return RSVD_OK;
    }

    // Timing mode: bracket the projection GEMM kernel (not its slab reduction) with events.
    int ev_begin(int kind, int& idx) {
        idx = -1;
        if (!h->timing) return RSVD_OK;
        while (h->ev_pool.size() < h->ev_next + 2) {
            hipEvent_t e;
            RSVD_CK(hipEventCreate(&e));
            h->ev_pool.push_back(e);
        }
        idx = (int)h->ev_next;
        h->ev_next += 2;
        h->ev_used.push_back({kind, idx});
        RSVD_CK(hipEventRecord(h->ev_pool[idx], s));
        return RSVD_OK;
    }
    int ev_end(int idx) {
        if (idx >= 0) RSVD_CK(hipEventRecord(h->ev_pool[idx + 1], s));
        return RSVD_OK;
    }

    int proj_nn(const T* A, int64_t lda, const T* X, T* Y, int kind = 0) {
        int ev;
        RSVD_TRY(ev_begin(kind, ev));
        RSVD_CK(launch_proj_nn<T>(A, lda, L.m, L.n, X, L.LP, L.pnn, slab, Y, s, ev >= 0 ? h->ev_pool[ev + 1] : nullptr));
        return RSVD_OK;
    }
    int proj_tn(const T* A, int64_t lda, const T* Q, T* Z) {
        int ev;
        RSVD_TRY(ev_begin(1, ev));
        RSVD_CK(launch_proj_tn<T>(A, lda, L.m, L.n, Q, L.LP, L.ptn, slab, Z, s, ev >= 0 ? h->ev_pool[ev + 1] : nullptr));
        return RSVD_OK;
    }

    int load_omega(const void* omega, int64_t ldo, uint64_t seed) {
        if (omega) {
            RSVD_CK(launch_colmajor_to_panel<T>(reinterpret_cast<const T*>(omega), ldo, L.n, L.l, L.LP, Xn, s));
        } else {
            RSVD_CK(launch_philox_omega<T>(Xn, L.n, L.l, L.LP, seed, s));
        }
        return RSVD_OK;
    }

    // intermediate_step (src/rSVD.cpp:57-70): leaves Q (m x LP panel) in Qm.
    int range_finder(const T* A, int64_t lda, int q) {
        RSVD_TRY(proj_nn(A, lda, Xn, Ym, 2));  // the sketch
        RSVD_TRY(orth(Ym, L.m, Qm, q == 0 ? 2 : inter_passes));
        for (int i = 0; i < q; ++i) {
            RSVD_TRY(proj_tn(A, lda, Qm, Zn));
            RSVD_TRY(orth(Zn, L.n, Xn, inter_passes));
            RSVD_TRY(proj_nn(A, lda, Xn, Ym));
            RSVD_TRY(orth(Ym, L.m, Qm, i == q - 1 ? 2 : inter_passes));
        }
        return RSVD_OK;
    }

    // SVDMethod::Power (src/rSVD.cpp:106-113): the reference's power method on B = Q^T A, run in
    // the coordinates of Q_B (dense.hip power_prep_kernel): start vectors Philox(power_seed(seed)
    // + i) projected on span(Q_B), s(n) iterations (src/PM.cpp:25-28), U = Q Utilde, V = Q_B Y.
    int power_stage(const rsvd_desc_t* d, void* U, int64_t ldu, T* S, void* V, int64_t ldv) {
        const int64_t q2 = (int64_t)L.LP * L.LP;
        double* sm = R1;  // R1 .. sm + 7 q2: the small-matrix area
        double *Y0 = Gsum, *Pp = R2, *X0s = Rinv, *Bpm = sm + 6 * q2, *Up = Uw, *Vc = Vw, *Sd = sm + 7 * q2;
        RSVD_CK(launch_power_start<T>(T1, L.n, L.l, L.LP, power_seed(d->seed), s));
        RSVD_TRY(cross_gram(Xn, T1, L.n, Y0));  // Y0 = Q_B^T X0
        RSVD_CK(launch_power_prep(R1, Y0, L.l, L.LP, Pp, X0s, Bpm, s));
        RSVD_CK(launch_power_svd(Pp, L.l, L.l, L.LP, Bpm, L.l, 0, power_iterations(L.n), Up, Vc, Sd, h->dflags + 16,
                                 s, X0s, d->method == RSVD_SVD_POWER_IC ? 2 : 1));
        RSVD_CK(launch_convert_scale<T>(Sd, S, L.l, std::fabs(a_scale_of(d)), s));
        RSVD_CK(launch_panel_small<T>(Qm, L.m, L.LP, Up, reinterpret_cast<T*>(U), 1, L.l, ldu, s));
        RSVD_CK(launch_panel_small<T>(Xn, L.n, L.LP, Vc, reinterpret_cast<T*>(V), 1, L.l, ldv, s));
        return finish(d, S, V, ldv);
    }

    // A = a_scale * (stored A) = U (|a_scale| S) (sign(a_scale) V)^T; then the finite check of S.
    int finish(const rsvd_desc_t* d, T* S, void* V, int64_t ldv) {
        const double sc = a_scale_of(d);
        if (sc < 0.0) RSVD_CK(launch_scale_cols<T>(reinterpret_cast<T*>(V), L.n, L.l, ldv, -1.0, s));
        RSVD_CK(launch_check_finite<T>(S, L.l, h->dflags + kFlagNonFinite, s));
        return RSVD_OK;
    }

    int run(const rsvd_desc_t* d, const T* A, void* U, int64_t ldu, T* S, void* V, int64_t ldv) {
        RSVD_TRY(range_finder(A, d->lda, d->q));
        // Stage B: B^T = A^T Q, QR-preconditioned as in SVD_class.hpp:116-123.
        RSVD_TRY(proj_tn(A, d->lda, Qm, Zn));
        RSVD_TRY(orth(Zn, L.n, Xn, 2));  // Xn = Q_B
        RSVD_TRY(cross_gram(Xn, Zn, L.n, R1));    // R = Q_B^T B^T exactly (fp64), W = R^T
        // Inf / NaN in A reach R through B^T = A^T Q whatever the orthonormalisations did with them
        RSVD_CK(launch_check_finite<double>(R1, L.LP * L.LP, h->dflags + kFlagNonFinite, s));
        if (d->method == RSVD_SVD_POWER || d->method == RSVD_SVD_POWER_IC) return power_stage(d, U, ldu, S, V, ldv);
        RSVD_CK(launch_small_svd<T>(R1, L.l, L.LP, Uw, Vw, S, h->dflags + 1, s));
        const double sc = std::fabs(a_scale_of(d));
        if (sc != 1.0) RSVD_CK(launch_scale_cols<T>(S, L.l, 1, L.l, sc, s));
        const int dcols = L.l;  // d = min(l, n) = l (l <= n enforced)
        RSVD_CK(launch_panel_small<T>(Qm, L.m, L.LP, Uw, reinterpret_cast<T*>(U), 1, dcols, ldu, s));
        RSVD_CK(launch_panel_small<T>(Xn, L.n, L.LP, Vw, reinterpret_cast<T*>(V), 1, dcols, ldv, s));
        return finish(d, S, V, ldv);
    }
};

template <typename T>
int run_typed(rsvd_handle_t h, const rsvd_desc_t* d, const void* A, const void* omega, int64_t ldo, void* U,
              int64_t ldu, void* S, void* V, int64_t ldv, void* Qout, int64_t ldq) {
    Layout<T> L(d->m, d->n, d->l);
    RSVD_TRY(ensure_ws(h, L.total));
    RSVD_CK(reset_run_flags(h->dflags, h->stream));
    RSVD_CK(hipMemsetAsync(h->ws + L.off_ctr, 0, 64 * sizeof(unsigned), h->stream));
    h->info.splits_nn = L.pnn.splits;
    h->info.splits_tn = L.ptn.splits;
    h->info.n_shard_rows = 0;
    Engine<T> E(h, L);
    E.qr_mode = d->qr_mode;
    RSVD_TRY(E.load_omega(omega, ldo, d->seed));
    if (Qout) {
        RSVD_TRY(E.range_finder(reinterpret_cast<const T*>(A), d->lda, d->q));
        RSVD_CK(launch_panel_to_colmajor<T>(E.Qm, L.m, L.l, L.LP, reinterpret_cast<T*>(Qout), ldq, h->stream));
        return RSVD_OK;
    }
    return E.run(d, reinterpret_cast<const T*>(A), U, ldu, reinterpret_cast<T*>(S), V, ldv);
}

int set_device(rsvd_handle_t h) {
    RSVD_CK(hipSetDevice(h->device));
    return RSVD_OK;
}

}  // namespace

// =============================================================================================
// C ABI
// =============================================================================================
extern "C" {

const char* rsvd_status_string(int status) {
    switch (status) {
        case RSVD_OK: return "ok";
        case RSVD_ERR_INVALID_ARG: return "invalid argument";
        case RSVD_ERR_UNSUPPORTED: return "unsupported";
        case RSVD_ERR_HIP: return "HIP error";
        case RSVD_ERR_NO_DEVICE: return "no HIP device";
        case RSVD_ERR_NUMERICAL: return "numerical failure";
        case RSVD_ERR_COMM: return "communication failure";
        default: return "unknown status";
    }
}

int rsvd_abi_version(void) { return RSVD_ABI_VERSION; }

int64_t rsvd_row_partition(int64_t rows, int world, int rank, int64_t* offset) {
    // src/rSVD.cpp:20-23: rows_per_proc = rows / P, remainder spread over the first ranks.
    if (world <= 0 || rank < 0 || rank >= world || rows < 0) {
        if (offset) *offset = 0;
        return -1;
    }
    const int64_t per = rows / world, rem = rows % world;
    const int64_t local = (rank < rem) ? per + 1 : per;
    if (offset) *offset = rank * per + std::min<int64_t>(rank, rem);
    return local;
}

int rsvd_create(int device, rsvd_handle_t* out) {
    if (!out) return RSVD_ERR_INVALID_ARG;
    *out = nullptr;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return RSVD_ERR_NO_DEVICE;
    if (device < 0 || device >= count) return RSVD_ERR_INVALID_ARG;
    rsvd_handle_t h = new rsvd_handle_s();
    h->device = device;
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&h->stream, hipStreamNonBlocking) != hipSuccess ||
        hipMalloc(&h->dflags, kFlagWords * sizeof(int)) != hipSuccess ||
        hipMemset(h->dflags, 0, kFlagWords * sizeof(int)) != hipSuccess) {
        delete h;
        return RSVD_ERR_HIP;
    }
    h->own_stream = true;
    *out = h;
    return RSVD_OK;
}

int rsvd_destroy(rsvd_handle_t h) {
    if (!h) return RSVD_OK;
    (void)hipSetDevice(h->device);
    if (h->stream) (void)hipStreamSynchronize(h->stream);
    release_comm(h);
    if (h->ws && !h->ws_external) (void)hipFree(h->ws);
    if (h->dflags) (void)hipFree(h->dflags);
    for (auto e : h->ev_pool) (void)hipEventDestroy(e);
    if (h->own_stream && h->stream) (void)hipStreamDestroy(h->stream);
    delete h;
    return RSVD_OK;
}

int rsvd_set_stream(rsvd_handle_t h, void* stream) {
    if (!h) return RSVD_ERR_INVALID_ARG;
    if (h->own_stream && h->stream) {
        (void)hipStreamSynchronize(h->stream);
        (void)hipStreamDestroy(h->stream);
    }
    h->stream = reinterpret_cast<hipStream_t>(stream);
    h->own_stream = false;
    return RSVD_OK;
}

const char* rsvd_last_error(rsvd_handle_t h) { return h ? h->err.c_str() : "null handle"; }

// Synchronise the handle's stream and turn the sticky device error words into a status
// (clearing them): a timed-out in-kernel hand-off, a rank-deficiency repair that broke down again,
// or non-finite singular values.  `flags` receives the whole flag block.
static int sync_flags(rsvd_handle_t h, int* flags) {
    RSVD_TRY(set_device(h));
    RSVD_CK(hipMemcpyAsync(flags, h->dflags, kFlagWords * sizeof(int), hipMemcpyDeviceToHost, h->stream));
    RSVD_CK(hipStreamSynchronize(h->stream));
    const int sticky[5] = {kFlagGramTimeout, kFlagJacobiTimeout, kFlagUnrepaired, kFlagNonFinite, kFlagFewRows};
    bool any = false;
    for (int w : sticky) any = any || flags[w] != 0;
    if (!any) return RSVD_OK;
    for (int w : sticky) RSVD_CK(hipMemsetAsync(h->dflags + w, 0, sizeof(int), h->stream));
    RSVD_CK(hipStreamSynchronize(h->stream));
    if (flags[kFlagGramTimeout]) {
        h->err = "an in-kernel hand-off (Gram reduction / grid barrier) timed out waiting for its producers";
        return RSVD_ERR_HIP;
    }
    if (flags[kFlagJacobiTimeout]) {
        h->err = "a persistent grid's barrier timed out (block Jacobi grid barrier or the tridiagonalisation's "
                 "hand-off: the abort word was raised and every workgroup left)";
        return RSVD_ERR_HIP;
    }
    if (flags[kFlagFewRows]) {  // (wide.cpp: every rank sums the same count, so all of them report it)
        h->err = "l > min(m, n) not supported (m: the global row count of the sharded A)";
        return RSVD_ERR_UNSUPPORTED;
    }
    if (flags[kFlagUnrepaired]) {
        h->err = "a rank-deficient panel could not be re-orthonormalised";
        return RSVD_ERR_NUMERICAL;
    }
    h->err = "non-finite singular values (A holds Inf / NaN, or the factorisation overflowed)";
    return RSVD_ERR_NUMERICAL;
}

int rsvd_sync(rsvd_handle_t h) {
    if (!h) return RSVD_ERR_INVALID_ARG;
    int flags[kFlagWords] = {0};
    return sync_flags(h, flags);
}

int rsvd_get_info(rsvd_handle_t h, rsvd_info_t* info) {
    if (!h || !info) return RSVD_ERR_INVALID_ARG;
    int flags[kFlagWords] = {0};
    RSVD_TRY(sync_flags(h, flags));
    int fallbacks = 0;
    for (int k = 4; k < 16; ++k) fallbacks += flags[k] != 0;
    h->info.cholqr_fallbacks = fallbacks;
    h->info.jacobi_sweeps = flags[1];
    h->info.power_kept = flags[16];
    *info = h->info;
    return RSVD_OK;
}

int rsvd_set_timing(rsvd_handle_t h, int enable) {
    if (!h) return RSVD_ERR_INVALID_ARG;
    RSVD_TRY(set_device(h));
    RSVD_CK(hipStreamSynchronize(h->stream));
    h->timing = enable != 0;
    h->ev_used.clear();
    h->ev_next = 0;
    for (int k = 0; k < 3; ++k) {
        h->acc_ms[k] = 0.0;
        h->acc_n[k] = 0;
    }
    return RSVD_OK;
}

int rsvd_get_timing(rsvd_handle_t h, rsvd_timing_t* t) {
    if (!h || !t) return RSVD_ERR_INVALID_ARG;
    RSVD_TRY(set_device(h));
    RSVD_CK(hipStreamSynchronize(h->stream));
    for (auto& u : h->ev_used) {
        float ms = 0.f;
        RSVD_CK(hipEventElapsedTime(&ms, h->ev_pool[u.second], h->ev_pool[u.second + 1]));
        h->acc_ms[u.first] += ms;
        h->acc_n[u.first] += 1;
        if (u.first == 2) {  // the sketch is also an A*X launch
            h->acc_ms[0] += ms;
            h->acc_n[0] += 1;
        }
    }
    h->ev_used.clear();
    h->ev_next = 0;
    t->nn_launches = h->acc_n[0];
    t->tn_launches = h->acc_n[1];
    t->nn_ms = h->acc_ms[0];
    t->tn_ms = h->acc_ms[1];
    t->sketch_launches = h->acc_n[2];
    t->reserved = 0;
    t->sketch_ms = h->acc_ms[2];
    return RSVD_OK;
}

int rsvd_set_workspace(rsvd_handle_t h, void* ptr, size_t bytes) {
    if (!h || (!ptr && bytes)) return RSVD_ERR_INVALID_ARG;
    if (h->ws && !h->ws_external) {
        (void)hipStreamSynchronize(h->stream);
        (void)hipFree(h->ws);
    }
    h->ws = reinterpret_cast<char*>(ptr);
    h->ws_bytes = ptr ? bytes : 0;
    h->ws_external = ptr != nullptr;
    return RSVD_OK;
}

int rsvd_set_comm(rsvd_handle_t h, int rank, int world, rsvd_allreduce_fn fn, void* user) {
    if (!h || world < 1 || world > 64 || rank < 0 || rank >= world || (world > 1 && !fn)) return RSVD_ERR_INVALID_ARG;
    release_comm(h);  // hooks replace a library-owned communicator
    h->rank = rank;
    h->world = world;
    h->allreduce = fn;
    h->ar_user = user;
    return RSVD_OK;
}

int rsvd_set_collectives(rsvd_handle_t h, rsvd_collective_fn fn, void* user) {
    if (!h) return RSVD_ERR_INVALID_ARG;
    h->coll = fn;
    h->coll_user = user;
    return RSVD_OK;
}

int rsvd_workspace_bytes(const rsvd_desc_t* d, size_t* bytes) {
    if (!d || !bytes) return RSVD_ERR_INVALID_ARG;
    const char* err = "";
    RSVD_TRY(check_desc_msg(d, &err, 0));
    if (d->l > 512) {  // dense_big.cpp
        *bytes = big_rsvd_workspace(d);
        return RSVD_OK;
    }
    RSVD_TRY(wide_workspace_bytes(d, bytes));
    if (wide_path(d)) return RSVD_OK;
    // narrow single-GPU layout, or the wide engine's when the handle is row-sharded: the larger
    const size_t narrow = d->dtype == RSVD_F64 ? Layout<double>(d->m, d->n, d->l).total
                                               : Layout<float>(d->m, d->n, d->l).total;
    *bytes = std::max(*bytes, narrow);
    return RSVD_OK;
}

int rsvd_run(rsvd_handle_t h, const rsvd_desc_t* d, const void* A, const void* omega, int64_t ldo, void* U,
             int64_t ldu, void* S, void* V, int64_t ldv) {
    if (!h) return RSVD_ERR_INVALID_ARG;
    RSVD_TRY(check_desc(h, d));
    if (!A || !U || !S || !V || ldu < d->m || ldv < d->n || (omega && ldo < d->n)) {
        h->err = "null pointer or bad leading dimension";
        return RSVD_ERR_INVALID_ARG;
    }
    RSVD_TRY(set_device(h));
    if (d->l > 512) return big_rsvd_run(h, d, A, omega, ldo, U, ldu, S, V, ldv, nullptr, 0);
    if (wide_path(d) || h->world > 1 || (d->flags & RSVD_FLAG_FORCE_NSHARD))
        return wide_run(h, d, A, omega, ldo, U, ldu, S, V, ldv, nullptr, 0);
    if (d->dtype == RSVD_F64) return run_typed<double>(h, d, A, omega, ldo, U, ldu, S, V, ldv, nullptr, 0);
    return run_typed<float>(h, d, A, omega, ldo, U, ldu, S, V, ldv, nullptr, 0);
}

int rsvd_range_finder(rsvd_handle_t h, const rsvd_desc_t* d, const void* A, const void* omega, int64_t ldo, void* Q,
                      int64_t ldq) {
    if (!h) return RSVD_ERR_INVALID_ARG;
    RSVD_TRY(check_desc(h, d));
    if (!A || !Q || ldq < d->m) {
        h->err = "null pointer or bad leading dimension";
        return RSVD_ERR_INVALID_ARG;
    }
    RSVD_TRY(set_device(h));
    if (d->l > 512) return big_rsvd_run(h, d, A, omega, ldo, nullptr, 0, nullptr, nullptr, 0, Q, ldq);
    if (wide_path(d) || h->world > 1) return wide_run(h, d, A, omega, ldo, nullptr, 0, nullptr, nullptr, 0, Q, ldq);
    if (d->dtype == RSVD_F64) return run_typed<double>(h, d, A, omega, ldo, nullptr, 0, nullptr, nullptr, 0, Q, ldq);
    return run_typed<float>(h, d, A, omega, ldo, nullptr, 0, nullptr, nullptr, 0, Q, ldq);
}

int rsvd_generate_omega(rsvd_handle_t h, int64_t n, int32_t l, uint64_t seed, int32_t dtype, void* omega) {
    if (!h || n <= 0 || l <= 0 || !omega) return RSVD_ERR_INVALID_ARG;
    RSVD_TRY(set_device(h));
    // Generate the row-major panel in the workspace, then write it out column-major:
    // Omega(i, j) is stream element i + n*j in both layouts.
    const int LP = lp_of(l);
    size_t bytes = (size_t)n * LP * (dtype == RSVD_F64 ? 8 : 4);
    RSVD_TRY(ensure_ws(h, bytes));
    if (dtype == RSVD_F64) {
        RSVD_CK(launch_philox_omega<double>(reinterpret_cast<double*>(h->ws), n, l, LP, seed, h->stream));
        RSVD_CK(launch_panel_to_colmajor<double>(reinterpret_cast<double*>(h->ws), n, l, LP,
                                                 reinterpret_cast<double*>(omega), n, h->stream));
    } else if (dtype == RSVD_F32) {
        RSVD_CK(launch_philox_omega<float>(reinterpret_cast<float*>(h->ws), n, l, LP, seed, h->stream));
        RSVD_CK(launch_panel_to_colmajor<float>(reinterpret_cast<float*>(h->ws), n, l, LP,
                                                reinterpret_cast<float*>(omega), n, h->stream));
    } else if (dtype == RSVD_BF16 || dtype == RSVD_FP8_E4M3) {
        // the Omega of the low-precision paths: Philox values rounded to bf16 / e4m3, as fp32
        RSVD_TRY(ensure_ws(h, (size_t)n * LP * 2));
        RSVD_CK(launch_omega_lowp(reinterpret_cast<bf16_t*>(h->ws), n, l, LP, seed, dtype == RSVD_FP8_E4M3,
                                  reinterpret_cast<float*>(omega), h->stream));
    } else {
        return RSVD_ERR_UNSUPPORTED;
    }
    return RSVD_OK;
}

// ---- host fp64 variants ----------------------------------------------------------------------
namespace {
struct DevBuf {
    void* p = nullptr;
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
};
}  // namespace

int rsvd_run_host_f64(rsvd_handle_t h, int64_t m, int64_t n, const double* A, int64_t lda, int32_t l, int32_t q,
                      int32_t method, const double* omega, uint64_t seed, double* U, double* S, double* V) {
    if (!h || !A || !U || !S || !V) return RSVD_ERR_INVALID_ARG;
    rsvd_desc_t d{};
    d.m = m; d.n = n; d.lda = m; d.l = l; d.q = q; d.dtype = RSVD_F64; d.method = method;
    d.qr_mode = RSVD_QR_AUTO; d.seed = seed;
    RSVD_TRY(check_desc(h, &d));
    if (lda < m) return RSVD_ERR_INVALID_ARG;
    RSVD_TRY(set_device(h));
    const int64_t dd = std::min<int64_t>(l, n);
    DevBuf dA, dO, dU, dS, dV;
    RSVD_CK(hipMalloc(&dA.p, sizeof(double) * m * n));
    RSVD_CK(hipMalloc(&dU.p, sizeof(double) * m * dd));
    RSVD_CK(hipMalloc(&dS.p, sizeof(double) * dd));
    RSVD_CK(hipMalloc(&dV.p, sizeof(double) * n * dd));
    RSVD_CK(hipMemcpy2DAsync(dA.p, sizeof(double) * m, A, sizeof(double) * lda, sizeof(double) * m, n,
                             hipMemcpyHostToDevice, h->stream));
    if (omega) {
        RSVD_CK(hipMalloc(&dO.p, sizeof(double) * n * l));
        RSVD_CK(hipMemcpyAsync(dO.p, omega, sizeof(double) * n * l, hipMemcpyHostToDevice, h->stream));
    }
    RSVD_TRY(rsvd_run(h, &d, dA.p, dO.p, n, dU.p, m, dS.p, dV.p, n));
    RSVD_CK(hipMemcpyAsync(U, dU.p, sizeof(double) * m * dd, hipMemcpyDeviceToHost, h->stream));
    RSVD_CK(hipMemcpyAsync(S, dS.p, sizeof(double) * dd, hipMemcpyDeviceToHost, h->stream));
    RSVD_CK(hipMemcpyAsync(V, dV.p, sizeof(double) * n * dd, hipMemcpyDeviceToHost, h->stream));
    return rsvd_sync(h);
}

int rsvd_range_finder_host_f64(rsvd_handle_t h, int64_t m, int64_t n, const double* A, int64_t lda,
                               const double* omega, int32_t l, int32_t q, double* Q) {
    if (!h || !A || !Q || !omega) return RSVD_ERR_INVALID_ARG;
    rsvd_desc_t d{};
    d.m = m; d.n = n; d.lda = m; d.l = l; d.q = q; d.dtype = RSVD_F64; d.method = RSVD_SVD_JACOBI;
    RSVD_TRY(check_desc(h, &d));
    if (lda < m) return RSVD_ERR_INVALID_ARG;
    RSVD_TRY(set_device(h));
    DevBuf dA, dO, dQ;
    RSVD_CK(hipMalloc(&dA.p, sizeof(double) * m * n));
    RSVD_CK(hipMalloc(&dO.p, sizeof(double) * n * l));
    RSVD_CK(hipMalloc(&dQ.p, sizeof(double) * m * l));
    RSVD_CK(hipMemcpy2DAsync(dA.p, sizeof(double) * m, A, sizeof(double) * lda, sizeof(double) * m, n,
                             hipMemcpyHostToDevice, h->stream));
    RSVD_CK(hipMemcpyAsync(dO.p, omega, sizeof(double) * n * l, hipMemcpyHostToDevice, h->stream));
    RSVD_TRY(rsvd_range_finder(h, &d, dA.p, dO.p, n, dQ.p, m));
    RSVD_CK(hipMemcpyAsync(Q, dQ.p, sizeof(double) * m * l, hipMemcpyDeviceToHost, h->stream));
    return rsvd_sync(h);
}

int rsvd_generate_omega_host_f64(rsvd_handle_t h, int64_t n, int32_t l, uint64_t seed, double* omega) {
    if (!h || !omega || n <= 0 || l <= 0) return RSVD_ERR_INVALID_ARG;
    RSVD_TRY(set_device(h));
    DevBuf dO;
    RSVD_CK(hipMalloc(&dO.p, sizeof(double) * n * l));
    RSVD_TRY(rsvd_generate_omega(h, n, l, seed, RSVD_F64, dO.p));
    RSVD_CK(hipMemcpyAsync(omega, dO.p, sizeof(double) * n * l, hipMemcpyDeviceToHost, h->stream));
    RSVD_CK(hipStreamSynchronize(h->stream));
    return RSVD_OK;
}

}  // extern "C"
