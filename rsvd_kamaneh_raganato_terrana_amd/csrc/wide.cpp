// wide.cpp -- host orchestration of the wide rSVD engine (l up to 512; bf16 / fp8 / fp32 / fp64 A).
//
// Same algorithm and op order as the narrow engine (driver.cpp) and the reference
// (src/rSVD.cpp:57-133):
//   Omega                                              generateOmega        src/rSVD.cpp:81
//   Y = A Omega ; Q = orth(Y)                          intermediate_step    src/rSVD.cpp:59-61
//   q x { Z = A^T Q ; X = orth(Z) ; Y = A X ; Q = orth(Y) }                 src/rSVD.cpp:62-69
//   B^T = A^T Q ; Q_B = orth(B^T) ; R = Q_B^T B^T      B = Q^T A + QR       src/rSVD.cpp:89, SVD_class.hpp:116-123
//   W = R^T = U_w S V_w^T                              SVD<Jacobi>          SVD_class.hpp:126-178
//   U = Q U_w ; V = Q_B V_w                            U = Q * Utilde       src/rSVD.cpp:128
// with the wide kernels (wide.hpp): bf16-MFMA projections for bf16 / fp8 A (fp32 / fp64 A use the
// narrow MFMA kernels per 64-column group), CholeskyQR(2) with fp64 Grams for any LP <= 512, and
// the block Jacobi small SVD for LP >= 128 (jacobi.hip's one-workgroup kernel below).
// Row sharding (world > 1): m-side Grams are summed through the all-reduce hook; every rank
// holds S, V and its rows of U.  The n side is either replicated (A^T Q all-reduced, every rank
// orthonormalises the whole n x l panel) or -- with the collective hook (rsvd_set_collectives) --
// sharded: rank r owns n-side rows [r nc, (r + 1) nc) (nc = n / world rounded up to 32, the
// panels zero-padded to world nc rows).  A^T Q is reduce-scattered, each rank runs the CholeskyQR
// of its rows (l x l Gram all-reduced, like the m side), the bf16 hi / lo panels of the next
// skinny operand are all-gathered for A X, and V = Q_B V_w is formed per shard and all-gathered.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <string>

#include "handle.hpp"
#include "dense.hpp"
#include "kernels.hpp"
#include "wide.hpp"

namespace rsvd {

namespace {

inline int64_t rup(int64_t x, int64_t q) { return (x + q - 1) / q * q; }

bool lowp_dtype(int dt) { return dt == RSVD_BF16 || dt == RSVD_FP8_E4M3; }

int wide_lp(int l, int dtype) {
    if (lowp_dtype(dtype)) {
        int lp = 16;
        while (lp < l) lp *= 2;
        return lp;  // the bf16 projection kernels are built for 16 .. 512
    }
    return (int)rup(l, 64);  // 64-column groups of the fp32 / fp64 projection kernels
}

template <typename T>
struct WideLayout {
    int64_t m, n;
    int l, LP;
    bool lowp;
    WProjPlan wnn, wtn;
    ProjPlan pnn, ptn;
    GramPlan gm, gn, gx;
    size_t off_Xn, off_Zn, off_Ym, off_Qm, off_T1, off_Xh, off_Xl, off_Qh, off_Ql, off_X8, off_pslab, off_gslab;
    size_t off_G, off_R, off_Rinv, off_W, off_R1, off_Uw, off_Vw, off_JX, off_JJ, off_M32, off_MS, off_colflag, off_sync,
        off_E, total;
    // the deferred second CholeskyQR pass (fp32 results): the factor's R (scratch), R2^-1 of the m and n
    // output panels, their products with U_w / V_w and a temp
    size_t off_R2s = 0, off_R2m = 0, off_R2n = 0, off_Mu = 0, off_Mv = 0, off_Tmp = 0;

    int64_t mpad, npad;  // bf16 panel rows, zero-padded to a multiple of 32 (wproj2 reads whole k-steps)
    bool s8 = false;     // the sketch runs e4m3 x e4m3 on the fp8 MFMA
    // n-side sharding: chunk rows nc per rank, the n-side panels hold nfull = world nc rows
    bool nsh = false;
    int64_t nc = 0, nfull = 0;
    GramPlan gnc, gxc;

    // a_aligned: A's base is 16-B aligned (the LDS-DMA projection kernel needs 16-B source chunks);
    // shard: the n side is sharded over `world` ranks (world 1 only under RSVD_FLAG_FORCE_NSHARD)
    WideLayout(const rsvd_desc_t* d, bool a_aligned = true, int world = 1, bool shard = false)
        : m(d->m), n(d->n), l(d->l), LP(wide_lp(d->l, d->dtype)) {
        lowp = lowp_dtype(d->dtype);
        mpad = rup(m, 32);
        nsh = shard;
        nc = nsh ? rup((n + world - 1) / world, 32) : n;
        nfull = nsh ? nc * world : n;
        npad = std::max(rup(n, 32), nfull);
        int64_t pslab = 1;
        if (lowp) {
            // (m a multiple of the 16-B chunk: a chunk is either inside A's rows or wholly past them,
            // where the clamped read lands on zero S rows / unstored output rows)
            const bool v2 = a_aligned && ((d->dtype == RSVD_BF16 && d->lda % 8 == 0 && m % 8 == 0 && m >= 8) ||
                                          (d->dtype == RSVD_FP8_E4M3 && d->lda % 16 == 0 && m % 16 == 0 && m >= 16));
            wnn = plan_wproj(m, n, LP, v2, true, d->dtype == RSVD_FP8_E4M3);
            wtn = plan_wproj(n, m, LP, v2, false, d->dtype == RSVD_FP8_E4M3);
            pslab = std::max<int64_t>(wnn.splits > 1 ? wnn.splits * m : 0, wtn.splits > 1 ? wtn.splits * n : 0);
        } else {
            pnn = plan_proj_nn<T>(m, n, 64);
            ptn = plan_proj_tn<T>(m, n, 64);
            pslab = std::max<int64_t>(pnn.splits > 1 ? pnn.splits * m : 0, ptn.splits > 1 ? ptn.splits * n : 0);
        }
        gm = plan_gram_wide(m, LP, 0);
        gn = plan_gram_wide(n, LP, 0);
        gx = plan_gram_wide(n, LP, 1);
        gnc = plan_gram_wide(nc, LP, 0);
        gxc = plan_gram_wide(nc, LP, 1);
        const size_t gslab = (size_t)std::max({(int64_t)gm.blocks * gm.chunks, (int64_t)gn.blocks * gn.chunks,
                                               (int64_t)gx.blocks * gx.chunks, (int64_t)gnc.blocks * gnc.chunks,
                                               (int64_t)gxc.blocks * gxc.chunks}) * 1024;
        const int64_t mx = std::max({m, n, nc});
        const size_t L2 = (size_t)LP * LP;
        size_t o = 0;
        auto take = [&](size_t bytes) {
            const size_t at = o;
            o = align256(o + bytes);
            return at;
        };
        off_Xn = take(sizeof(T) * nfull * LP);
        off_Zn = take(sizeof(T) * nfull * LP);
        off_Ym = take(sizeof(T) * m * LP);
        off_Qm = take(sizeof(T) * m * LP);
        off_T1 = take(sizeof(T) * mx * LP);
        const size_t bn = lowp ? 2 * npad * LP : 0, bm = lowp ? 2 * mpad * LP : 0;
        off_Xh = take(bn);
        off_Xl = take(bn);
        off_Qh = take(bm);
        off_Ql = take(bm);
        // e4m3 A: the sketch Omega as an e4m3 panel (the fp8-MFMA sketch product, launch_wproj_s8)
        s8 = d->dtype == RSVD_FP8_E4M3 && wproj_s8_supported(wnn, LP);
        off_X8 = take(s8 ? (size_t)npad * LP : 0);
        off_pslab = take(sizeof(T) * std::max<int64_t>(pslab, 1) * LP);
        off_gslab = take(sizeof(double) * gslab);
        off_G = take(sizeof(double) * (L2 + 1));  // (+1: the global row count rides the first m-side all-reduce)
        off_R = take(sizeof(double) * L2);
        off_Rinv = take(sizeof(double) * L2);
        off_W = take(sizeof(double) * L2);
        off_R1 = take(sizeof(double) * L2);
        off_Uw = take(sizeof(double) * L2);
        off_Vw = take(sizeof(double) * L2);
        // (also the two-level Cholesky's scratch during the QR chain, up to 3 levels at LP = 512)
        off_JX = take(sizeof(double) * std::max<size_t>(2 * L2, LP >= 256 ? chol_2level_scratch_doubles(LP, 1) : 0));
        off_JJ = take(sizeof(double) * 2 * L2);
        off_M32 = take(sizeof(float) * 3 * L2);  // Rinv, Uw, Vw in fp32 (panel_gemm operand for fp32 panels)
        // the three bf16 pieces of panel_gemm's M (twice: U_w's and V_w's for the two final products)
        off_MS = take(sizeof(T) == 4 ? sizeof(bf16_t) * 6 * L2 : 0);
        off_colflag = take(sizeof(int) * LP);
        off_sync = take(sizeof(unsigned) * kBJSyncWords);
        // the eigensolver's small SVD (fp32 results, 128 <= LP <= 512: wide_eig.hip)
        off_E = take(sizeof(T) == 4 && LP >= 128 && LP <= 512 ? sizeof(double) * eig_svd_ws_doubles(LP) : 0);
        if (sizeof(T) == 4) {
            off_R2s = take(sizeof(double) * L2);
            off_R2m = take(sizeof(double) * L2);
            off_R2n = take(sizeof(double) * L2);
            off_Mu = take(sizeof(double) * L2);
            off_Mv = take(sizeof(double) * L2);
            off_Tmp = take(sizeof(double) * L2);
        }
        total = o;
    }
};

template <typename T>
struct WideEngine {
    rsvd_handle_t h;
    const WideLayout<T>& L;
    hipStream_t s;
    int dtype;
    T *Xn, *Zn, *Ym, *Qm, *T1, *pslab;
    bf16_t *Xh, *Xl, *Qh, *Ql;
    fp8_t* X8;
    double *gslab, *G, *R, *Rinv, *W, *R1, *Uw, *Vw, *JX, *JJ;
    float *Rinv32, *Uw32, *Vw32;
    int* colflag;
    unsigned* sync;
    int inter_passes = 1;  // power-iteration intermediates only carry a subspace (driver.cpp)
    bool lowp_inter = false;  // RSVD_FLAG_LOWP_INTERMEDIATES
    int qr_mode = RSVD_QR_AUTO;
    int orth_index = 0;
    // Repair draws of the m side: rank g's rows are stream rows [g 2^40, g 2^40 + m_g) of a
    // world x 2^40-row stream (disjoint for any shard sizes, src/rSVD.cpp:20-23 remainders included),
    // normalised by the global row count estimate world * m_g.
    int64_t row_off = 0, m_total = 0, m_norm = 0;
    uint64_t seed = 0;
    bool nsh = false;  // n side sharded (L.nsh and a run that supports it)
    int64_t c0 = 0;    // first n-side row of this rank's shard (rank nc)

    WideEngine(rsvd_handle_t h_, const WideLayout<T>& L_, int dtype_) : h(h_), L(L_), s(h_->stream), dtype(dtype_) {
        char* b = h->ws;
        Xn = reinterpret_cast<T*>(b + L.off_Xn);
        Zn = reinterpret_cast<T*>(b + L.off_Zn);
        Ym = reinterpret_cast<T*>(b + L.off_Ym);
        Qm = reinterpret_cast<T*>(b + L.off_Qm);
        T1 = reinterpret_cast<T*>(b + L.off_T1);
        pslab = reinterpret_cast<T*>(b + L.off_pslab);
        Xh = L.lowp ? reinterpret_cast<bf16_t*>(b + L.off_Xh) : nullptr;
        Xl = L.lowp ? reinterpret_cast<bf16_t*>(b + L.off_Xl) : nullptr;
        Qh = L.lowp ? reinterpret_cast<bf16_t*>(b + L.off_Qh) : nullptr;
        Ql = L.lowp ? reinterpret_cast<bf16_t*>(b + L.off_Ql) : nullptr;
        X8 = L.s8 ? reinterpret_cast<fp8_t*>(b + L.off_X8) : nullptr;
        gslab = reinterpret_cast<double*>(b + L.off_gslab);
        G = reinterpret_cast<double*>(b + L.off_G);
        R = reinterpret_cast<double*>(b + L.off_R);
        Rinv = reinterpret_cast<double*>(b + L.off_Rinv);
        W = reinterpret_cast<double*>(b + L.off_W);
        R1 = reinterpret_cast<double*>(b + L.off_R1);
        Uw = reinterpret_cast<double*>(b + L.off_Uw);
        Vw = reinterpret_cast<double*>(b + L.off_Vw);
        JX = reinterpret_cast<double*>(b + L.off_JX);
        JJ = reinterpret_cast<double*>(b + L.off_JJ);
        Rinv32 = reinterpret_cast<float*>(b + L.off_M32);
        Uw32 = Rinv32 + (size_t)L.LP * L.LP;
        Vw32 = Uw32 + (size_t)L.LP * L.LP;
        Ms = sizeof(T) == 4 ? reinterpret_cast<bf16_t*>(b + L.off_MS) : nullptr;
        colflag = reinterpret_cast<int*>(b + L.off_colflag);
        sync = reinterpret_cast<unsigned*>(b + L.off_sync);
        if (sizeof(T) == 4) {
            R2s = reinterpret_cast<double*>(b + L.off_R2s);
            R2m = reinterpret_cast<double*>(b + L.off_R2m);
            R2n = reinterpret_cast<double*>(b + L.off_R2n);
            Mu = reinterpret_cast<double*>(b + L.off_Mu);
            Mv = reinterpret_cast<double*>(b + L.off_Mv);
            Tmp = reinterpret_cast<double*>(b + L.off_Tmp);
        }
    }

    // Output panels (final Q, Q_B) of fp32-result runs defer CholeskyQR2's second pass (round 6):
    // pass 1 gives T1 (orthonormal to ~eps_G cond^2, repaired when rank-deficient), and the exact
    // basis Q = T1 R2^-1 (R2 = chol(T1^T T1)) is never formed: the next projection reads T1 itself
    // (B^T = A^T Q = (A^T T1) R2^-1 -- T1 is as well conditioned as Q for the hi / lo operand), and
    // R2^-1 enters only the l x l matrices: R = Q_B^T B^T = R2n^-T (T1z^T A^T T1) R2m^-1,
    // U = T1 (R2m^-1 U_w), V = T1z (R2n^-1 V_w).  Same span, same R up to rounding (src/rSVD.cpp:60-68,
    // 89, 128); two m x l / n x l panel products per rSVD become four l x l GEMMs (C5 -0.33 ms, C3
    // -0.28 ms on one box).  Measured and dropped: the pass-2 Gram + factor on a side stream beside the
    // next projection -- the projections run one workgroup per CU in a single wave of workgroups, so
    // a CU the side stream holds delays the whole projection by about as long (C4 +0.03, C5 +0.08 ms).
    // R2^-1 need not be triangular: any M with (T1 M)^T (T1 M) = I will do, and G = T1^T T1 = I + E is
    // near the identity, so M = G^-1/2 by its series (wide_eig.hip launch_isqrt_near_identity: four
    // l^3 MFMA products instead of the factor's pivot chain; the Cholesky factor, predicated, when
    // |E|_F > 0.1).  RSVD_ISQRT=0: the Cholesky factor always (A/B).
    bool defer = false, isqrt = true;
    double *R2s = nullptr, *R2m = nullptr, *R2n = nullptr, *Mu = nullptr, *Mv = nullptr, *Tmp = nullptr;

    // world > 1: G[LP^2] holds this rank's row count until the first m-side Gram all-reduce sums it
    // with the Gram; a global count below l then raises kFlagFewRows (rsvd_sync: RSVD_ERR_UNSUPPORTED)
    bool count_pending = false;

    int allreduce(void* buf, int64_t count, int32_t dt) {
        if (h->world <= 1 || !h->allreduce) return RSVD_OK;
        if (h->allreduce(buf, count, dt, (void*)s, h->ar_user) != 0) {
            h->err = "all-reduce hook failed";
            return RSVD_ERR_COMM;
        }
        return RSVD_OK;
    }

    int collective(int op, void* send, void* recv, int64_t count, int32_t dt) {
        if (h->coll(op, send, recv, count, dt, (void*)s, h->coll_user) != 0) {
            h->err = op == RSVD_COLL_REDUCE_SCATTER ? "reduce-scatter hook failed" : "all-gather hook failed";
            return RSVD_ERR_COMM;
        }
        return RSVD_OK;
    }
    int32_t tdt() const { return sizeof(T) == 8 ? RSVD_F64 : RSVD_F32; }
    // the next skinny operand of A X to every rank: its bf16 hi / lo panels (or the T panel)
    int gather_x() {
        if (!nsh) return RSVD_OK;
        const int64_t cnt = L.nc * L.LP;
        if (L.lowp) {
            RSVD_TRY(collective(RSVD_COLL_ALL_GATHER, Xh + c0 * L.LP, Xh, cnt, RSVD_BF16));
            return collective(RSVD_COLL_ALL_GATHER, Xl + c0 * L.LP, Xl, cnt, RSVD_BF16);
        }
        return collective(RSVD_COLL_ALL_GATHER, Xn + c0 * L.LP, Xn, cnt, tdt());
    }

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

    // Y = A X (X: bf16 panels for low precision, T panel otherwise)
    int proj_nn(const void* A, int64_t lda, const T* X, const bf16_t* xh, const bf16_t* xl, T* Y, int kind = 0) {
        int ev;
        RSVD_TRY(ev_begin(kind, ev));
        hipEvent_t done = ev >= 0 ? h->ev_pool[ev + 1] : nullptr;
        if (L.lowp) {
            RSVD_CK(launch_wproj(1, dtype == RSVD_FP8_E4M3, A, lda, L.m, L.n, xh, xl, L.LP, L.wnn,
                                 reinterpret_cast<float*>(pslab), reinterpret_cast<float*>(Y), s, done));
        } else {
            RSVD_CK(launch_proj_nn<T>(reinterpret_cast<const T*>(A), lda, L.m, L.n, X, L.LP, L.pnn, pslab, Y, s, done));
        }
        return RSVD_OK;
    }
    // Y = A Omega with e4m3 A and the e4m3 sketch in X8: both operands exact e4m3 on the fp8 MFMA
    int proj_nn_s8(const void* A, int64_t lda, T* Y) {
        int ev;
        RSVD_TRY(ev_begin(2, ev));
        hipEvent_t done = ev >= 0 ? h->ev_pool[ev + 1] : nullptr;
        RSVD_CK(launch_wproj_s8(A, lda, L.m, L.n, X8, L.LP, L.wnn, reinterpret_cast<float*>(pslab),
                                reinterpret_cast<float*>(Y), s, done));
        return RSVD_OK;
    }
    // Z = A^T Q, summed over the row shards
    int proj_tn(const void* A, int64_t lda, const T* Q, const bf16_t* qh, const bf16_t* ql, T* Z) {
        int ev;
        RSVD_TRY(ev_begin(1, ev));
        hipEvent_t done = ev >= 0 ? h->ev_pool[ev + 1] : nullptr;
        if (L.lowp) {
            RSVD_CK(launch_wproj(0, dtype == RSVD_FP8_E4M3, A, lda, L.m, L.n, qh, ql, L.LP, L.wtn,
                                 reinterpret_cast<float*>(pslab), reinterpret_cast<float*>(Z), s, done));
        } else {
            RSVD_CK(launch_proj_tn<T>(reinterpret_cast<const T*>(A), lda, L.m, L.n, Q, L.LP, L.ptn, pslab, Z, s, done));
        }
        // sharded n side: this rank keeps the sum of its rows [c0, c0 + nc) (rows >= n are zero)
        if (nsh) return collective(RSVD_COLL_REDUCE_SCATTER, Z, Z + c0 * L.LP, L.nc * L.LP, tdt());
        return allreduce(Z, L.n * L.LP, tdt());
    }

    double tol() const { return sizeof(T) == 4 ? 1e-13 : 1e-28; }
    // the split Gram's entry error is ~3e-8 of sqrt(G_ii G_jj).  A pivot ratio d_k / G_kk above 1e-6
    // is then known to a few per cent, and the factor's only use -- Q = P R^-1 spanning span(P) --
    // tolerates that: Q's departure from orthonormality is ~eps_G cond(P)^2 <= 0.03 (intermediate
    // panels; output panels take a second pass).  Below it (cond(P) past ~1e3, breakdowns) the
    // fp64 Gram and factor run again.
    static constexpr double kSplitIllTol = 1e-7;
    bool split_gram = false;
    static constexpr int split_cross = 3;  // bits: 1 the split cross Gram at LP = 256, 2 at LP = 512
    bool split_panel = false;  // panel products on the bf16 MFMA, three-piece split (fp32 panels of bf16 / e4m3 A)
    bf16_t* Ms = nullptr;
    bf16_t* ms() const { return split_panel ? Ms : nullptr; }
    // two-level factor: bit 0 at LP = 512, bit 1 at LP = 256 (0 would be one level
    // everywhere).  Round 4 default 3: with the K-split 128^3 / 256^3 products (four waves per tile)
    // and the DPP diagonal factor, tools/wide_lab chol: LP = 256 one level 157.8 us vs two levels
    // 145.5 us; LP = 512 two levels 350.2 us vs three (each 256 level itself two-level) 321.8 us
    static constexpr int chol2 = 3;
    // LP = 512 with bit 1 also set: each 256-column level is itself two-level (three levels of 128)
    int chol_depth() const { return (L.LP == 512 && (chol2 & 2)) ? 1 : 0; }
    static constexpr int bj_groups = 0;  // block-Jacobi row groups (0: auto)
    bool eig_svd = true;  // fp32 results: the small SVD through the eigensolver (RSVD_SMALL_SVD=jacobi: block Jacobi)
    // panel_gemm's operand in the panel precision: fp64 matrices as-is, fp32 copies for fp32 panels
    const T* mat(const double* m64, const float* m32) const {
        if constexpr (sizeof(T) == 8) return m64; else return m32;
    }

    // The split Gram runs on unpredicated passes of one rank (RSVD_GRAM_SPLIT_SHARDED=1: of every rank).
    // Priced at world 8 from the per-rank kernels (bench.py --emulate-world 8, round 6): C5 -0.40 ms,
    // C4 -0.05 ms of kernel time per rSVD, but its predicated fallback Gram has to be summed whether or
    // not it runs -- eight more LP^2 all-reduces per rSVD, ~+0.42 / +0.34 ms at the model's RCCL cost
    // (tools/model8.py) -- so sharded passes keep the fp64 Gram.
    bool split_sharded = false;
    bool split_path(bool sharded, const int* pred) const { return split_gram && !pred && (!sharded || split_sharded); }

    // R = chol(P^T P) and R^-1 (Ro, Rio; with the fp32 copy and bf16 pieces of R^-1 when r32 / mt).
    int gram_factor(const T* P, int64_t rows, const GramPlan& gp, bool sharded, int* flag, const int* pred, double* Ro,
                    double* Rio, float* r32, bf16_t* mt) {
        // LP = 256 / 512, l > LP / 2: the two-level factor (wide_qr.hip launch_chol_wide_2level; JX is
        // free scratch until the small SVD) for unpredicated passes
        const bool two = (chol2 & (L.LP == 512 ? 1 : (L.LP == 256 ? 2 : 0))) && L.l > L.LP / 2;
        auto factor = [&](int* fl, double ill_tol, int* ill) -> hipError_t {
            if (two)
                return launch_chol_wide_2level(G, L.l, L.LP, tol(), Ro, Rio, r32, colflag, fl, W, JX, s, ill_tol, ill,
                                               nullptr, chol_depth(), mt);
            return launch_chol_wide(G, L.l, L.LP, tol(), Ro, Rio, r32, colflag, fl, W, nullptr, s, ill_tol, ill,
                                    nullptr, mt);
        };
        // sharded: the rank's Gram summed over the ranks (the first m-side sum carries the global row count)
        auto sum_ranks = [&]() -> int {
            if (!sharded) return RSVD_OK;
            const bool cnt = count_pending && rows == L.m && !pred;
            RSVD_TRY(allreduce(G, (int64_t)L.LP * L.LP + (cnt ? 1 : 0), RSVD_F64));
            if (cnt) {
                count_pending = false;
                RSVD_CK(launch_check_rows(G + (size_t)L.LP * L.LP, L.l, h->dflags + kFlagFewRows, s));
            }
            return RSVD_OK;
        };
        if (split_path(sharded, pred)) {
            int* ill = h->dflags + kFlagSplitIll;
            RSVD_CK(launch_gram_split(reinterpret_cast<const float*>(P), rows, L.LP, gp, gslab, G, s));
            RSVD_TRY(sum_ranks());
            RSVD_CK(factor(h->dflags + kFlagSplitScratch, kSplitIllTol, ill));
            RSVD_CK(launch_gram_wide<T>(P, nullptr, rows, L.LP, gp, gslab, G, ill, s));
            // sharded: the fallback Gram's sum is issued whether or not `ill` is raised (a device word the
            // host does not read; every rank factors the same summed G, so the ranks' words agree).  When
            // it is clear, G is dead and so is this sum.
            RSVD_TRY(sum_ranks());
            RSVD_CK(launch_chol_wide(G, L.l, L.LP, tol(), Ro, Rio, r32, colflag, flag, W, ill, s, 0.0, nullptr, nullptr,
                                     mt));
            return RSVD_OK;
        }
        RSVD_CK(launch_gram_wide<T>(P, nullptr, rows, L.LP, gp, gslab, G, pred, s));
        RSVD_TRY(sum_ranks());
        if (pred)
            RSVD_CK(launch_chol_wide(G, L.l, L.LP, tol(), Ro, Rio, r32, colflag, flag, W, pred, s, 0.0, nullptr, nullptr,
                                     mt));
        else
            RSVD_CK(factor(flag, 0.0, nullptr));
        return RSVD_OK;
    }

    // One CholeskyQR pass Out = P chol(P^T P)^-1 (+ bf16 hi/lo of Out).  `pred`: predicated pass.
    // fp32 panels of bf16 / e4m3 A (unpredicated passes, any world size): the Gram by the three-piece bf16
    // split (wide_qr.hip gram_split_kernel, |dG| ~ 1e-8 |G|); when a pivot of its factor falls below
    // kSplitIllTol of its diagonal (cond(P) beyond ~1e3, or a breakdown) the fp64 Gram and factor
    // run again, predicated on that test (h->dflags[kFlagSplitIll]), and their R / R^-1 / flags stand.
    int cholqr_pass(const T* P, int64_t rows, const GramPlan& gp, T* Out, bool sharded, bf16_t* hi, bf16_t* lo,
                    int* flag, const int* pred) {
        float* r32 = sizeof(T) == 4 ? Rinv32 : nullptr;
        // the split panel product's pieces of R^-1, written by the factor with its fp32 copy (no
        // split_mat launch per pass; bit-identical)
        bf16_t* mt = (ms() && L.LP >= 128) ? ms() : nullptr;
        RSVD_TRY(gram_factor(P, rows, gp, sharded, flag, pred, R, Rinv, r32, mt));
        const bool split_p = split_path(sharded, pred);
        RSVD_CK(launch_panel_gemm<T>(P, rows, L.LP, mat(Rinv, Rinv32), 1, Out, 0, 0, hi, lo, split_p ? nullptr : pred,
                                     s, ms(), mt != nullptr));
        return RSVD_OK;
    }

    // The rank-deficiency completion of an output panel Q (rows of this rank), predicated on `flag`
    // (a breakdown in its orthonormalisation): flagged columns replaced by Philox Gaussian rows, one
    // predicated CholeskyQR pass back into Q (+ hi / lo).
    int repair(T* Q, int64_t rows, const GramPlan& gp, bool sharded, bf16_t* hi, bf16_t* lo, int* flag, bool mside,
               bool nshard) {
        // sharded panels draw disjoint stream rows per rank (rank 2^40 + local row), as the m side
        const int64_t off = (mside || nshard) ? row_off : 0, tot = (mside || nshard) ? m_total : L.n;
        const int64_t nrm = mside ? m_norm : L.n;
        const int64_t valid = nshard ? std::max<int64_t>(0, std::min<int64_t>(L.nc, L.n - c0)) : rows;
        RSVD_CK(launch_repair_panel<T>(Q, rows, L.l, L.LP, colflag, flag, seed ^ (0x5EEDull + orth_index), off, tot,
                                       nrm, T1, s, valid));
        // a breakdown in the repaired pass is reported (sticky) by rsvd_sync as RSVD_ERR_NUMERICAL
        return cholqr_pass(T1, rows, gp, Q, sharded, hi, lo, h->dflags + kFlagUnrepaired, flag);
    }

    // The deferred form of an output panel's CholeskyQR2 (see `defer`): T1out = pass 1 (+ hi / lo, the
    // repair), then R2^-1 = chol(T1^T T1)^-1 into r2inv.
    int orth2_deferred(const T* P, bool mside, T* T1out, bf16_t* hi, bf16_t* lo, double* r2inv) {
        const bool nshard = !mside && nsh;
        const int64_t rows = mside ? L.m : (nshard ? L.nc : L.n);
        const GramPlan& gp = mside ? L.gm : (nshard ? L.gnc : L.gn);
        const bool sharded = (mside || nshard) && h->world > 1;
        if (nshard) {
            P += c0 * L.LP;
            T1out += c0 * L.LP;
            if (hi) hi += c0 * L.LP;
            if (lo) lo += c0 * L.LP;
        }
        int* flag = h->dflags + 4 + (orth_index < 12 ? orth_index : 11);
        ++orth_index;
        RSVD_TRY(cholqr_pass(P, rows, gp, T1out, sharded, hi, lo, flag, nullptr));
        RSVD_TRY(repair(T1out, rows, gp, sharded, hi, lo, flag, mside, nshard));
        // pass 2's factor: T1 is orthonormal to ~eps_G cond^2 (or repaired), so a breakdown here means the
        // panel could not be orthonormalised -- reported through the sticky kFlagUnrepaired
        if (!isqrt)
            return gram_factor(T1out, rows, gp, sharded, h->dflags + kFlagUnrepaired, nullptr, R2s, r2inv, nullptr,
                               nullptr);
        // G = T1^T T1 (split Gram: its ~3e-8 entry error is what the factor of that Gram carried too)
        if (split_gram) RSVD_CK(launch_gram_split(reinterpret_cast<const float*>(T1out), rows, L.LP, gp, gslab, G, s));
        else RSVD_CK(launch_gram_wide<T>(T1out, nullptr, rows, L.LP, gp, gslab, G, nullptr, s));
        if (sharded) RSVD_TRY(allreduce(G, (int64_t)L.LP * L.LP, RSVD_F64));
        int* fl = h->dflags + kFlagIsqrt;
        // E = G - I and the cut-off test; past it the Cholesky factor (predicated), then G is scratch
        RSVD_CK(launch_isqrt_near_identity(G, L.l, L.LP, Mu, Mv, nullptr, nullptr, nullptr, nullptr, fl, s, true,
                                           false));
        RSVD_CK(launch_chol_wide(G, L.l, L.LP, tol(), R2s, r2inv, nullptr, colflag, h->dflags + kFlagUnrepaired, W,
                                 fl + 1, s, 0.0, nullptr, nullptr, nullptr));
        RSVD_CK(launch_isqrt_near_identity(nullptr, L.l, L.LP, Mu, Mv, Tmp, R2s, G, r2inv, fl, s, false, true));
        return RSVD_OK;
    }

    // Q = orth(P): CholeskyQR (passes = 1) or CholeskyQR2; output panels (repair = true) get the
    // rank-deficiency completion (predicated on the breakdown flag of this orth).
    // The n side, sharded: P, Q, hi, lo are the full panels; this rank's rows [c0, c0 + nc) are used.
    int orth(const T* P, bool mside, T* Q, int passes, bf16_t* hi, bf16_t* lo, bool repair_out) {
        const bool nshard = !mside && nsh;
        const int64_t rows = mside ? L.m : (nshard ? L.nc : L.n);
        const GramPlan& gp = mside ? L.gm : (nshard ? L.gnc : L.gn);
        const bool sharded = (mside || nshard) && h->world > 1;
        if (nshard) {
            P += c0 * L.LP;
            Q += c0 * L.LP;
            if (hi) hi += c0 * L.LP;
            if (lo) lo += c0 * L.LP;
        }
        int* flag = h->dflags + 4 + (orth_index < 12 ? orth_index : 11);
        ++orth_index;
        if (qr_mode == RSVD_QR_CHOLQR2 || qr_mode == RSVD_QR_GS2) passes = 2;
        if (passes <= 1) {
            // bf16 / e4m3 A: a power-iteration intermediate is consumed only through its bf16 hi/lo
            // panels (the wproj kernels), so its fp32 copy is not written (-1/2 of the panel's writes)
            T* out = (L.lowp && !repair_out && hi && lo) ? nullptr : Q;
            RSVD_TRY(cholqr_pass(P, rows, gp, out, sharded, hi, lo, flag, nullptr));
        } else {
            RSVD_TRY(cholqr_pass(P, rows, gp, T1, sharded, nullptr, nullptr, flag, nullptr));
            RSVD_TRY(cholqr_pass(T1, rows, gp, Q, sharded, hi, lo, flag, nullptr));
        }
        if (repair_out) RSVD_TRY(repair(Q, rows, gp, sharded, hi, lo, flag, mside, nshard));
        return RSVD_OK;
    }

    int load_omega(const void* omega, int64_t ldo, uint64_t sd) {
        if (L.lowp) {
            const int f8 = dtype == RSVD_FP8_E4M3;
            if (omega) {
                RSVD_CK(launch_omega_lowp_from(reinterpret_cast<const float*>(omega), ldo, L.n, L.l, L.LP, f8, Xh, s));
            } else {
                RSVD_CK(launch_omega_lowp(Xh, L.n, L.l, L.LP, sd, f8, nullptr, s));
            }
        } else if (omega) {
            RSVD_CK(launch_colmajor_to_panel<T>(reinterpret_cast<const T*>(omega), ldo, L.n, L.l, L.LP, Xn, s));
        } else {
            RSVD_CK(launch_philox_omega<T>(Xn, L.n, L.l, L.LP, sd, s));
        }
        return RSVD_OK;
    }

    int range_finder(const void* A, int64_t lda, int q) {
        if (L.s8) {  // the sketch: Omega is exactly e4m3 -- fp8 MFMA
            RSVD_CK(launch_bf16_to_fp8(Xh, L.npad * L.LP, X8, s));
            RSVD_TRY(proj_nn_s8(A, lda, Ym));
        } else {
            RSVD_TRY(proj_nn(A, lda, Xn, Xh, nullptr, Ym, 2));  // the sketch: Omega is exactly bf16 (lowp)
        }
        if (q == 0 && defer)
            RSVD_TRY(orth2_deferred(Ym, true, Qm, Qh, Ql, R2m));
        else
            RSVD_TRY(orth(Ym, true, Qm, q == 0 ? 2 : inter_passes, Qh, Ql, q == 0));
        for (int i = 0; i < q; ++i) {
            const bool last = i == q - 1;
            // RSVD_FLAG_LOWP_INTERMEDIATES: iterations before the last take the bf16 operand alone
            const bool one = L.lowp && lowp_inter && !last;
            RSVD_TRY(proj_tn(A, lda, Qm, Qh, one ? nullptr : Ql, Zn));
            RSVD_TRY(orth(Zn, false, Xn, inter_passes, Xh, Xl, false));
            RSVD_TRY(gather_x());
            RSVD_TRY(proj_nn(A, lda, Xn, Xh, one ? nullptr : Xl, Ym));
            if (last && defer)
                RSVD_TRY(orth2_deferred(Ym, true, Qm, Qh, Ql, R2m));
            else
                RSVD_TRY(orth(Ym, true, Qm, last ? 2 : inter_passes, Qh, Ql, last));
        }
        return RSVD_OK;
    }

    // SVDMethod::Power on B = Q^T A in Q_B coordinates (driver.cpp power_stage, dense.hip).
    int power_stage(const rsvd_desc_t* d, void* U, int64_t ldu, T* S, void* V, int64_t ldv) {
        double *Y0 = G, *Pp = R, *X0s = Rinv, *Bpm = W, *Up = Uw, *Vc = Vw, *Sd = JX;
        RSVD_CK(launch_power_start<T>(T1, L.n, L.l, L.LP, power_seed(d->seed), s));
        RSVD_CK(launch_gram_wide<T>(Xn, T1, L.n, L.LP, L.gx, gslab, Y0, nullptr, s));  // Y0 = Q_B^T X0
        RSVD_CK(launch_power_prep(R1, Y0, L.l, L.LP, Pp, X0s, Bpm, s));
        RSVD_CK(launch_power_svd(Pp, L.l, L.l, L.LP, Bpm, L.l, 0, power_iterations(L.n), Up, Vc, Sd, h->dflags + 16,
                                 s, X0s, d->method == RSVD_SVD_POWER_IC ? 2 : 1));
        RSVD_CK(launch_convert_scale<T>(Sd, S, L.l, std::fabs(a_scale(d)), s));
        if (sizeof(T) == 4) {
            const int L2 = L.LP * L.LP;
            RSVD_CK(launch_convert_scale<float>(Up, Uw32, L2, 1.0, s));
            RSVD_CK(launch_convert_scale<float>(Vc, Vw32, L2, 1.0, s));
        }
        RSVD_CK(launch_panel_gemm<T>(Qm, L.m, L.LP, mat(Up, Uw32), 0, reinterpret_cast<T*>(U), ldu, L.l, nullptr,
                                     nullptr, nullptr, s, ms()));
        RSVD_CK(launch_panel_gemm<T>(Xn, L.n, L.LP, mat(Vc, Vw32), 0, reinterpret_cast<T*>(V), ldv, L.l, nullptr,
                                     nullptr, nullptr, s, ms()));
        return finish(d, S, V, ldv);
    }

    static double a_scale(const rsvd_desc_t* d) { return d->a_scale != 0.0 ? d->a_scale : 1.0; }
    // A = a_scale * (stored A) = U (|a_scale| S) (sign(a_scale) V)^T; then the finite check of S.
    int finish(const rsvd_desc_t* d, T* S, void* V, int64_t ldv) {
        if (a_scale(d) < 0.0) RSVD_CK(launch_scale_cols<T>(reinterpret_cast<T*>(V), L.n, L.l, ldv, -1.0, s));
        RSVD_CK(launch_check_finite<T>(S, L.l, h->dflags + kFlagNonFinite, s));
        return RSVD_OK;
    }

    int run(const rsvd_desc_t* d, const void* A, void* U, int64_t ldu, T* S, void* V, int64_t ldv) {
        RSVD_TRY(range_finder(A, d->lda, d->q));
        RSVD_TRY(proj_tn(A, d->lda, Qm, Qh, Ql, Zn));  // B^T = A^T Q (deferred: A^T T1 = B^T R2m)
        if (defer)
            RSVD_TRY(orth2_deferred(Zn, false, Xn, nullptr, nullptr, R2n));  // T1z (Q_B = T1z R2n^-1)
        else
            RSVD_TRY(orth(Zn, false, Xn, 2, nullptr, nullptr, true));  // Q_B
        if (nsh) {  // R = Q_B^T B^T summed over the n shards
            RSVD_CK(launch_gram_wide<T>(Xn + c0 * L.LP, Zn + c0 * L.LP, L.nc, L.LP, L.gxc, gslab, R1, nullptr, s));
            RSVD_TRY(allreduce(R1, (int64_t)L.LP * L.LP, RSVD_F64));
        } else {
            // R = Q_B^T B^T: fp32 panels of bf16 / e4m3 A at LP = 256 / 512 by the three-piece bf16 split
            // (the entries to ~1e-8 of |Q_B| |B^T|, as the split Grams; RSVD_GRAM_SPLIT=0: fp64 MFMA)
            if (split_gram && ((L.LP == 256 && (split_cross & 1)) || (L.LP == 512 && (split_cross & 2))))
                RSVD_CK(launch_gram_split_cross(reinterpret_cast<const float*>(Xn), reinterpret_cast<const float*>(Zn),
                                                L.n, L.LP, L.gx, gslab, R1, s));
            else
                RSVD_CK(launch_gram_wide<T>(Xn, Zn, L.n, L.LP, L.gx, gslab, R1, nullptr, s));
        }
        if (defer) {  // R = R2n^-T (T1z^T A^T T1) R2m^-1
            RSVD_CK(launch_gemm_rm(0, 0, L.LP, R1, L.LP, R2m, L.LP, Tmp, L.LP, s));
            RSVD_CK(launch_gemm_rm(1, 0, L.LP, R2n, L.LP, Tmp, L.LP, R1, L.LP, s));
        }
        // Inf / NaN in A reach R through B^T = A^T Q whatever the orthonormalisations did with them
        RSVD_CK(launch_check_finite<double>(R1, L.LP * L.LP, h->dflags + kFlagNonFinite, s));
        if (d->method == RSVD_SVD_POWER || d->method == RSVD_SVD_POWER_IC) return power_stage(d, U, ldu, S, V, ldv);
        // the small SVD always runs in fp64 (U_w, V_w feed the fp32 panel products of U and V)
        double* Sd = G;  // free scratch by now
        if (L.LP <= 64) {
            RSVD_CK(launch_small_svd<double>(R1, L.l, L.LP, Uw, Vw, Sd, h->dflags + 1, s));
        } else if (sizeof(T) == 4 && eig_svd && L.l >= 3 && L.LP >= 128 && L.LP <= 512) {
            // fp32 results: G = W^T W, tridiagonalisation, multisection + inverse iteration, the
            // back-transformation, X = W V_w, then the block Jacobi's orthogonality check at the same
            // cos <= 1e-6 (wide_eig.hip; sweeps run only if the check fails)
            double* E = reinterpret_cast<double*>(h->ws + L.off_E);
            RSVD_CK(launch_eig_svd<double>(R1, L.l, L.LP, E, JX, JJ, Uw, Vw, Sd, sync, h->dflags + 1, s, kBJTolF32));
        } else {
            // fp32 results (fp32 / bf16 / e4m3 A): converged at cos <= 1e-6 -- 16 fp32 ulps, far below
            // the 1e-4 bar -- one or two sweeps fewer than the fp64 results' 1e-12
            const int bjg = bj_groups > 0 && block_jacobi_groups(L.LP, L.LP, bj_groups) ? bj_groups : 0;
            RSVD_CK(launch_block_jacobi<double>(R1, L.l, L.LP, JX, JJ, Uw, Vw, Sd, sync, h->dflags + 1, s,
                                                sizeof(T) == 4 ? 1e-8 : 1e-16, sizeof(T) == 4 ? kBJTolF32 : kBJTolF64,
                                                bjg));
        }
        // deferred: U = T1 (R2m^-1 U_w), V = T1z (R2n^-1 V_w)
        double* Uw = this->Uw;
        double* Vw = this->Vw;
        if (defer) {
            RSVD_CK(launch_gemm_rm(0, 0, L.LP, R2m, L.LP, Uw, L.LP, Mu, L.LP, s));
            RSVD_CK(launch_gemm_rm(0, 0, L.LP, R2n, L.LP, Vw, L.LP, Mv, L.LP, s));
            Uw = Mu;
            Vw = Mv;
        }
        // U_w / V_w pieces for the split final products, written with their fp32 copies and S (one launch)
        bf16_t* mu = (ms() && L.LP >= 128) ? Ms : nullptr;
        bf16_t* mv = mu ? Ms + (size_t)3 * L.LP * L.LP : nullptr;
        if (sizeof(T) == 4 && mu) {
            RSVD_CK(launch_finish_convert(Sd, reinterpret_cast<float*>(S), L.l, std::fabs(a_scale(d)), Uw, Uw32, mu, Vw,
                                          Vw32, mv, L.LP, s));
        } else {
            RSVD_CK(launch_convert_scale<T>(Sd, S, L.l, std::fabs(a_scale(d)), s));
            if (sizeof(T) == 4) {
                const int L2 = L.LP * L.LP;
                RSVD_CK(launch_convert_scale<float>(Uw, Uw32, L2, 1.0, s));
                RSVD_CK(launch_convert_scale<float>(Vw, Vw32, L2, 1.0, s));
            }
        }
        RSVD_CK(launch_panel_gemm<T>(Qm, L.m, L.LP, mat(Uw, Uw32), 0, reinterpret_cast<T*>(U), ldu, L.l, nullptr,
                                     nullptr, nullptr, s, mu ? mu : ms(), mu != nullptr));
        if (nsh) {  // V rows of this shard as a panel (in Zn, free by now), all-gathered, then V
            RSVD_CK(launch_panel_gemm<T>(Xn + c0 * L.LP, L.nc, L.LP, mat(Vw, Vw32), 0, Zn + c0 * L.LP, 0, 0, nullptr,
                                         nullptr, nullptr, s, mv ? mv : ms(), mv != nullptr));
            RSVD_TRY(collective(RSVD_COLL_ALL_GATHER, Zn + c0 * L.LP, Zn, L.nc * L.LP, tdt()));
            RSVD_CK(launch_panel_to_colmajor<T>(Zn, L.n, L.l, L.LP, reinterpret_cast<T*>(V), ldv, s));
        } else {
            RSVD_CK(launch_panel_gemm<T>(Xn, L.n, L.LP, mat(Vw, Vw32), 0, reinterpret_cast<T*>(V), ldv, L.l, nullptr,
                                         nullptr, nullptr, s, mv ? mv : ms(), mv != nullptr));
        }
        return finish(d, S, V, ldv);
    }
};

template <typename T>
int wide_typed(rsvd_handle_t h, const rsvd_desc_t* d, const void* A, const void* omega, int64_t ldo, void* U,
               int64_t ldu, void* S, void* V, int64_t ldv, void* Qout, int64_t ldq) {
    // n-side sharding: a collective hook on a sharded handle, not for SVDMethod::Power (its stage
    // runs on the whole Q_B) nor for the range-finder-only entry point (Qout)
    // (RSVD_FLAG_FORCE_NSHARD: the same code path at world 1, so one GPU runs the RCCL calls)
    // (past 64 ranks the n side stays replicated: rsvd_workspace_bytes sizes the padded n-side
    // panels for worlds up to 64, and a caller-provided workspace is sized by it)
    const bool nshard = (h->world > 1 || (d->flags & RSVD_FLAG_FORCE_NSHARD)) && h->world <= 64 && h->coll && !Qout &&
                        d->method != RSVD_SVD_POWER && d->method != RSVD_SVD_POWER_IC;
    WideLayout<T> L(d, (reinterpret_cast<uintptr_t>(A) & 15) == 0, h->world, nshard);
    RSVD_TRY(ensure_ws(h, L.total));
    RSVD_CK(reset_run_flags(h->dflags, h->stream));
    if (L.nsh && L.nfull > L.n) {  // the zero rows past n of the sharded n-side panels (A^T Q, Q_B)
        const size_t bpr = sizeof(T) * L.LP;
        for (size_t off : {L.off_Zn, L.off_Xn})
            RSVD_CK(hipMemsetAsync(h->ws + off + L.n * bpr, 0, (L.nfull - L.n) * bpr, h->stream));
    }
    if (L.lowp) {  // the zero padding rows of the bf16 panels (never written by the kernels)
        const size_t bpr = (size_t)2 * L.LP;
        for (size_t off : {L.off_Xh, L.off_Xl})
            if (L.npad > L.n) RSVD_CK(hipMemsetAsync(h->ws + off + L.n * bpr, 0, (L.npad - L.n) * bpr, h->stream));
        for (size_t off : {L.off_Qh, L.off_Ql})
            if (L.mpad > L.m) RSVD_CK(hipMemsetAsync(h->ws + off + L.m * bpr, 0, (L.mpad - L.m) * bpr, h->stream));
    }
    h->info.n_shard_rows = L.nsh ? (int32_t)L.nc : 0;
    h->info.splits_nn = L.lowp ? L.wnn.splits : L.pnn.splits;
    h->info.splits_tn = L.lowp ? L.wtn.splits : L.ptn.splits;
    WideEngine<T> E(h, L, d->dtype);
    E.qr_mode = d->qr_mode;
    // the split Gram: fp32 panels of bf16 / e4m3 A.  Diagnostic switches (each pinned against the oracle
    // by tests/test_gpu_switches.py): RSVD_GRAM_SPLIT=0 fp64 Grams only, RSVD_SMALL_SVD=jacobi the block
    // Jacobi small SVD for fp32 results instead of the eigensolver.
    {
        static const int env = [] {
            const char* v = std::getenv("RSVD_GRAM_SPLIT");
            return v ? std::atoi(v) : 1;
        }();
        E.split_gram = env != 0 && sizeof(T) == 4 && L.lowp && gram_split_ok(L.LP);
        E.split_panel = sizeof(T) == 4 && L.lowp && L.LP % 32 == 0 && L.LP >= 128;
        static const int env6 = [] {
            const char* v = std::getenv("RSVD_GRAM_SPLIT_SHARDED");
            return v ? std::atoi(v) : 0;
        }();
        E.split_sharded = env6 != 0;
        static const bool env5 = [] {
            const char* v = std::getenv("RSVD_SMALL_SVD");
            return !(v && std::string(v) == "jacobi");
        }();
        E.eig_svd = env5;
    }
    E.lowp_inter = (d->flags & RSVD_FLAG_LOWP_INTERMEDIATES) != 0;
    {
        // fp32 results, the rSVD proper (not the range finder's Q, not the power method: both use Q / Q_B
        // themselves).  RSVD_DEFER2=0: Q and Q_B formed by the second passes, as before round 6 (A/B).
        static const int env = [] {
            const char* v = std::getenv("RSVD_DEFER2");
            return v ? std::atoi(v) : 1;
        }();
        E.defer = env != 0 && sizeof(T) == 4 && !Qout && d->method != RSVD_SVD_POWER &&
                  d->method != RSVD_SVD_POWER_IC && d->qr_mode == RSVD_QR_AUTO;
        static const int env2 = [] {
            const char* v = std::getenv("RSVD_ISQRT");
            return v ? std::atoi(v) : 1;
        }();
        E.isqrt = env2 != 0;
    }
    E.seed = d->seed;
    E.nsh = L.nsh;
    E.c0 = L.nsh ? (int64_t)h->rank * L.nc : 0;
    if (h->world > 1) {
        E.row_off = (int64_t)h->rank << 40;
        E.m_total = (int64_t)h->world << 40;
    } else {
        E.m_total = d->m;
    }
    E.m_norm = (int64_t)h->world * d->m;
    if (h->world > 1 && h->allreduce) {
        RSVD_CK(launch_set_count(E.G + (size_t)L.LP * L.LP, d->m, h->stream));
        E.count_pending = true;
    }
    RSVD_TRY(E.load_omega(omega, ldo, d->seed));
    if (Qout) {
        RSVD_TRY(E.range_finder(A, d->lda, d->q));
        RSVD_CK(launch_panel_to_colmajor<T>(E.Qm, L.m, L.l, L.LP, reinterpret_cast<T*>(Qout), ldq, h->stream));
        return RSVD_OK;
    }
    return E.run(d, A, U, ldu, reinterpret_cast<T*>(S), V, ldv);
}

}  // namespace

bool wide_path(const rsvd_desc_t* d) { return lowp_dtype(d->dtype) || d->l > 64; }

int wide_workspace_bytes(const rsvd_desc_t* d, size_t* bytes) {
    // the largest over the projection plans (LDS-DMA kernel or not: decided per run by alignment)
    // and over n-side shardings of up to 64 ranks (the zero-padded n-side panels; the handle's
    // world is not known here)
    size_t b = 0;
    for (int world = 1; world <= 64; ++world) {
        const bool shard = world > 1 || (d->flags & RSVD_FLAG_FORCE_NSHARD);
        if (d->dtype == RSVD_F64)
            b = std::max(b, WideLayout<double>(d, true, world, shard).total);
        else
            b = std::max({b, WideLayout<float>(d, true, world, shard).total,
                          WideLayout<float>(d, false, world, shard).total});
    }
    *bytes = b;
    return RSVD_OK;
}

int wide_run(rsvd_handle_t h, const rsvd_desc_t* d, const void* A, const void* omega, int64_t ldo, void* U,
             int64_t ldu, void* S, void* V, int64_t ldv, void* Qout, int64_t ldq) {
    if (d->dtype == RSVD_F64) return wide_typed<double>(h, d, A, omega, ldo, U, ldu, S, V, ldv, Qout, ldq);
    return wide_typed<float>(h, d, A, omega, ldo, U, ldu, S, V, ldv, Qout, ldq);
}

}  // namespace rsvd
