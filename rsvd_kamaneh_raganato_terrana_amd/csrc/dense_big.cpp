// dense_big.cpp -- the QR() and SVD<Jacobi> drop-ins past the 512-column panels (SURVEY.md §8 rows
// f1, f2): the reference's qr_decomposition_reduced / _full (src/QR.cpp:22-80) and SVD<Jacobi>
// (include/SVD_class.hpp:100-180) take any size; dense_api.cpp's panel paths stop at 512 columns
// (the CholeskyQR and block-Jacobi kernels of the rSVD engine hold an LP x LP fp64 factor).
//
// QR, any m x n (reduced: m >= n; full: Q m x m).  Q's columns are built in blocks of <= 512:
// block b = the next columns of the basis [A | e_n .. e_{m-1}] (the identity completion the
// reference's Q_temp starts from, src/QR.cpp:49), projected out of the previous blocks by block
// classical Gram-Schmidt twice (two MFMA GEMMs per pass, gemm.hip), orthonormalised by the shifted
// CholeskyQR3 + rank-deficiency repair of dense_api.cpp, then projected and orthonormalised once
// more (a repaired column is random, not yet orthogonal to the earlier blocks).  The Givens sign rule
// of untouched leading columns, det(Q) = +1 for a square Q (the reference's Q is a product of
// rotations; gemm.hip's LU sign), and R = Q^T A with the strictly lower part zeroed.  For full-rank
// A the reduced factors are the unique QR with R(j, j) > 0, i.e. the reference's.
//
// SVD<Jacobi>, min(m, n) > 512: one-sided block Jacobi directly on P = A (m >= n) or A^T (the
// generalised wide_svd.hip kernel with MR = rows > 512, the pair columns read from global memory):
// P J = U S, V = J -- the converged SVD, which is what the reference's QR-preconditioned two-sided
// Jacobi returns (up to the signs of singular-vector pairs).  ParallelJacobi past 512 returns the
// same converged SVD (its own weight-ordered iteration stops at an absolute 1e-12 weight, which only
// differs below that level; dense_api.cpp runs that exact iteration up to 512).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <string>

#include "dense.hpp"
#include "handle.hpp"
#include "kernels.hpp"
#include "wide.hpp"

namespace rsvd {

namespace {

inline int64_t rup(int64_t x, int64_t q) { return (x + q - 1) / q * q; }
constexpr int kQrBlock = 512;

// The panel machinery of one <= 512-column block (as dense_api.cpp's DenseWs / orth).
template <typename T>
struct BlockOrth {
    int64_t rows;
    int LP;
    GramPlan gp;
    size_t off_P, off_Q, off_T1, off_T2, off_gslab, off_G, off_R, off_Rinv, off_W, off_R32, off_colflag, total;
    BlockOrth(int64_t rows_, int LP_) : rows(rows_), LP(LP_) {
        gp = plan_gram_wide(rows, LP, 0);
        const size_t panel = sizeof(T) * rows * LP, L2 = (size_t)LP * LP;
        size_t o = 0;
        auto take = [&](size_t bytes) {
            const size_t at = o;
            o = align256(o + bytes);
            return at;
        };
        off_P = take(panel);
        off_Q = take(panel);
        off_T1 = take(panel);
        off_T2 = take(panel);
        off_gslab = take(sizeof(double) * (size_t)gp.blocks * gp.chunks * 1024);
        off_G = take(sizeof(double) * L2);
        off_R = take(sizeof(double) * L2);
        off_Rinv = take(sizeof(double) * L2);
        off_W = take(sizeof(double) * L2);
        off_R32 = take(sizeof(float) * L2);
        off_colflag = take(sizeof(int) * LP);
        total = o;
    }
};

template <typename T>
struct QrBigWs {
    BlockOrth<T> bo;
    size_t off_bo, off_Y, off_C, off_W, off_sgn, total;
    QrBigWs(int64_t m, int64_t K) : bo(m, (int)rup(std::min<int64_t>(K, kQrBlock), 32)) {
        size_t o = 0;
        auto take = [&](size_t bytes) {
            const size_t at = o;
            o = align256(o + bytes);
            return at;
        };
        off_bo = take(bo.total);
        off_Y = take(sizeof(T) * m * kQrBlock);
        off_C = take(sizeof(T) * K * kQrBlock);
        off_W = take(K == m ? sizeof(double) * 2 * (size_t)m * m : 0);  // det sign of a square Q
        off_sgn = take(sizeof(int) * 4);
        total = o;
    }
};

template <typename T>
struct QrBig {
    rsvd_handle_t h;
    hipStream_t s;
    const QrBigWs<T>& L;
    T *P, *Q, *T1, *T2, *Y, *C;
    double *gslab, *G, *R, *Rinv, *W;
    float* R32;
    int* colflag;

    QrBig(rsvd_handle_t h_, const QrBigWs<T>& L_, char* base = nullptr) : h(h_), s(h_->stream), L(L_) {
        if (!base) base = h->ws;
        char* b = base + L.off_bo;
        P = reinterpret_cast<T*>(b + L.bo.off_P);
        Q = reinterpret_cast<T*>(b + L.bo.off_Q);
        T1 = reinterpret_cast<T*>(b + L.bo.off_T1);
        T2 = reinterpret_cast<T*>(b + L.bo.off_T2);
        gslab = reinterpret_cast<double*>(b + L.bo.off_gslab);
        G = reinterpret_cast<double*>(b + L.bo.off_G);
        R = reinterpret_cast<double*>(b + L.bo.off_R);
        Rinv = reinterpret_cast<double*>(b + L.bo.off_Rinv);
        W = reinterpret_cast<double*>(b + L.bo.off_W);
        R32 = reinterpret_cast<float*>(b + L.bo.off_R32);
        colflag = reinterpret_cast<int*>(b + L.bo.off_colflag);
        Y = reinterpret_cast<T*>(base + L.off_Y);
        C = reinterpret_cast<T*>(base + L.off_C);
    }

    double tol() const { return sizeof(T) == 4 ? 1e-13 : 1e-28; }

    // Row-sharded panels (rSVD() past 512 columns at world > 1): this rank holds rows of a global
    // panel; the Grams and the block projections Qp^T Y are summed over the ranks (the all-reduce hook,
    // src/rSVD.cpp:20-23's row partition), and repair draws use disjoint stream rows per rank.
    bool shard = false;
    int64_t row_off = 0, rows_total = 0, norm_rows = 0, rows_global = 0;
    int allreduce(void* buf, int64_t count, int32_t dt) {
        if (!shard || h->world <= 1 || !h->allreduce) return RSVD_OK;
        if (h->allreduce(buf, count, dt, (void*)s, h->ar_user) != 0) {
            h->err = "all-reduce hook failed";
            return RSVD_ERR_COMM;
        }
        return RSVD_OK;
    }

    // one CholeskyQR pass on a k-column panel (forward substitution: backward stable)
    int pass(const T* In, int k, T* Out, bool shift, const int* pred) {
        const int64_t rows = L.bo.rows;
        const int LP = L.bo.LP;
        int* flag = h->dflags + 4;
        RSVD_CK(launch_gram_wide<T>(In, nullptr, rows, LP, L.bo.gp, gslab, G, pred, s));
        RSVD_TRY(allreduce(G, (int64_t)LP * LP, RSVD_F64));
        if (shift)
            RSVD_CK(launch_shift_diag(G, LP, k, shard ? rows_global : rows, sizeof(T) == 4 ? 0x1p-24 : 0x1p-53, s));
        RSVD_CK(launch_chol_wide(G, k, LP, tol(), R, Rinv, sizeof(T) == 4 ? R32 : nullptr, colflag, flag, W, pred, s));
        RSVD_CK(launch_trsm_rows<T>(In, rows, k, LP, R, Out, pred, s));
        return RSVD_OK;
    }
    // Q = orth(P[:, :k]): shifted CholeskyQR3 + the predicated repair (dense_api.cpp DenseEngine::orth)
    int orth(int k, uint64_t seed) {
        const int64_t rows = L.bo.rows;
        RSVD_TRY(pass(P, k, T1, true, nullptr));
        RSVD_TRY(pass(T1, k, T2, false, nullptr));
        RSVD_TRY(pass(T2, k, Q, false, nullptr));
        if (shard)
            RSVD_CK(launch_repair_panel<T>(Q, rows, k, L.bo.LP, colflag, h->dflags + 4, seed, row_off, rows_total,
                                           norm_rows, T1, s));
        else
            RSVD_CK(launch_repair_panel<T>(Q, rows, k, L.bo.LP, colflag, h->dflags + 4, seed, 0, rows, rows, T1, s));
        RSVD_TRY(pass(T1, k, Q, false, h->dflags + 4));
        return RSVD_OK;
    }
    // Y (m x w, ld m) -= Qp (Qp^T Y), Qp = the first c0 columns of Q (ld ldq)
    int project(const T* Qp, int64_t ldq, int64_t m, int64_t c0, int w) {
        if (c0 == 0) return RSVD_OK;
        RSVD_CK(launch_gemm<T>(1, 0, c0, w, m, T(1), Qp, ldq, Y, m, T(0), C, c0, s));
        RSVD_TRY(allreduce(C, c0 * w, sizeof(T) == 8 ? RSVD_F64 : RSVD_F32));
        RSVD_CK(launch_gemm<T>(0, 0, m, w, c0, T(-1), Qp, ldq, C, c0, T(1), Y, m, s));
        return RSVD_OK;
    }
    // Qo (rows x K, ld rows) = an orthonormal basis of span(Src[:, :K]) (K <= rows), 512-column
    // blocks: CGS2 against the earlier blocks, shifted CholeskyQR3 + repair, and (past the first
    // block) one more projection + orthonormalisation, as qr_big_typed
    int orth_cols(const T* Src, int64_t lds, int64_t K, T* Qo, uint64_t seed) {
        const int64_t rows = L.bo.rows;
        const int LPb = L.bo.LP;
        for (int64_t c0 = 0; c0 < K; c0 += kQrBlock) {
            const int w = (int)std::min<int64_t>(kQrBlock, K - c0);
            RSVD_CK(hipMemsetAsync(h->dflags + 4, 0, sizeof(int), s));  // this block's breakdown count
            RSVD_CK(hipMemcpy2DAsync(Y, sizeof(T) * rows, Src + c0 * lds, sizeof(T) * lds, sizeof(T) * rows, w,
                                     hipMemcpyDeviceToDevice, s));
            RSVD_TRY(project(Qo, rows, rows, c0, w));
            RSVD_TRY(project(Qo, rows, rows, c0, w));
            RSVD_CK(launch_colmajor_to_panel<T>(Y, rows, rows, w, LPb, P, s));
            RSVD_TRY(orth(w, seed + 2 * (uint64_t)c0));
            if (c0 > 0) {
                RSVD_CK(launch_panel_to_colmajor<T>(Q, rows, w, LPb, Y, rows, s));
                RSVD_TRY(project(Qo, rows, rows, c0, w));
                RSVD_CK(launch_colmajor_to_panel<T>(Y, rows, rows, w, LPb, P, s));
                RSVD_TRY(orth(w, seed + 2 * (uint64_t)c0 + 1));
            }
            RSVD_CK(launch_panel_to_colmajor<T>(Q, rows, w, LPb, Qo + c0 * rows, rows, s));
        }
        return RSVD_OK;
    }
};

template <typename T>
int qr_big_typed(rsvd_handle_t h, int64_t m, int64_t n, const T* A, int64_t lda, int full, T* Qo, int64_t ldq, T* Ro,
                 int64_t ldr) {
    const int64_t K = full ? m : n;  // columns of Q
    QrBigWs<T> L(m, K);
    RSVD_CK(hipSetDevice(h->device));
    RSVD_TRY(ensure_ws(h, L.total));
    RSVD_CK(reset_run_flags(h->dflags, h->stream));
    QrBig<T> E(h, L);
    hipStream_t s = h->stream;
    const int LPb = L.bo.LP;
    for (int64_t c0 = 0; c0 < K; c0 += kQrBlock) {
        const int w = (int)std::min<int64_t>(kQrBlock, K - c0);
        // the basis columns c0 .. c0 + w: A's (j < n), then the identity completion e_j (j >= n)
        const int na = (int)std::max<int64_t>(0, std::min<int64_t>(n, c0 + w) - c0);
        // this block's breakdown word (as orth_cols): an earlier block's breakdown must not predicate
        // this block's repair pass
        RSVD_CK(hipMemsetAsync(h->dflags + 4, 0, sizeof(int), s));
        if (na > 0)
            RSVD_CK(hipMemcpy2DAsync(E.Y, sizeof(T) * m, A + c0 * lda, sizeof(T) * lda, sizeof(T) * m, na,
                                     hipMemcpyDeviceToDevice, s));
        if (na < w) RSVD_CK(launch_identity_cols<T>(E.Y + (int64_t)na * m, m, m, w - na, c0 + na, s));
        const uint64_t seed = 0x51A7ull + (uint64_t)m * 131 + (uint64_t)n + 7919ull * (uint64_t)c0;
        // CGS2 against the earlier blocks, then the block's own orthonormalisation
        RSVD_TRY(E.project(Qo, ldq, m, c0, w));
        RSVD_TRY(E.project(Qo, ldq, m, c0, w));
        RSVD_CK(launch_colmajor_to_panel<T>(E.Y, m, m, w, LPb, E.P, s));
        RSVD_TRY(E.orth(w, seed));
        if (c0 > 0) {  // once more: a repaired (random) column is not yet orthogonal to the earlier blocks
            RSVD_CK(launch_panel_to_colmajor<T>(E.Q, m, w, LPb, E.Y, m, s));
            RSVD_TRY(E.project(Qo, ldq, m, c0, w));
            RSVD_CK(launch_colmajor_to_panel<T>(E.Y, m, m, w, LPb, E.P, s));
            RSVD_TRY(E.orth(w, seed + 1));
        }
        RSVD_CK(launch_panel_to_colmajor<T>(E.Q, m, w, LPb, Qo + c0 * ldq, ldq, s));
    }
    RSVD_CK(launch_qr_signs_cm<T>(A, lda, m, n, Qo, ldq, s));
    if (K == m) {  // a square Q: det +1, as the reference's product of rotations
        RSVD_CK(launch_det_sign_cm<T>(Qo, ldq, (int)m, reinterpret_cast<double*>(h->ws + L.off_W),
                                      reinterpret_cast<int*>(h->ws + L.off_sgn), s));
    }
    RSVD_CK(launch_gemm<T>(1, 0, K, n, m, T(1), Qo, ldq, A, lda, T(0), Ro, ldr, s));  // R = Q^T A
    RSVD_CK(launch_zero_below<T>(Ro, ldr, K, n, s));
    return RSVD_OK;
}

struct SvdBigWs {
    int MR, LP;
    size_t off_A64, off_X, off_J, off_Uw, off_Vw, off_Uw32, off_S, off_sync, total;
    SvdBigWs(int64_t m, int64_t n, int dtype) {
        const int64_t k = std::min(m, n), rows = std::max(m, n);
        MR = (int)rup(rows, 32);
        LP = (int)rup(k, 32);
        size_t o = 0;
        auto take = [&](size_t bytes) {
            const size_t at = o;
            o = align256(o + bytes);
            return at;
        };
        off_A64 = take(dtype == RSVD_F32 ? sizeof(double) * (size_t)m * n : 0);
        off_X = take(sizeof(double) * 2 * (size_t)MR * LP);
        off_J = take(sizeof(double) * 2 * (size_t)LP * LP);
        off_Uw = take(sizeof(double) * (size_t)MR * LP);
        off_Vw = take(sizeof(double) * (size_t)LP * LP);
        off_Uw32 = take(dtype == RSVD_F32 ? sizeof(float) * (size_t)MR * LP : 0);
        off_S = take(sizeof(double) * LP);
        off_sync = take(sizeof(unsigned) * kBJSyncWords);
        total = o;
    }
};

template <typename T>
int svd_big_typed(rsvd_handle_t h, int64_t m, int64_t n, const T* A, int64_t lda, T* U, int64_t ldu, T* S, T* V,
                  int64_t ldv) {
    const int dtype = sizeof(T) == 8 ? RSVD_F64 : RSVD_F32;
    SvdBigWs L(m, n, dtype);
    RSVD_CK(hipSetDevice(h->device));
    RSVD_TRY(ensure_ws(h, L.total));
    RSVD_CK(reset_run_flags(h->dflags, h->stream));
    hipStream_t s = h->stream;
    char* b = h->ws;
    const double* src = reinterpret_cast<const double*>(A);
    int64_t lds = lda;
    if (sizeof(T) == 4) {  // the Jacobi arithmetic is fp64: widen A once
        double* A64 = reinterpret_cast<double*>(b + L.off_A64);
        RSVD_CK(launch_widen<T>(A, lda, m, n, A64, s));
        src = A64;
        lds = m;
    }
    const bool tall = m >= n;
    const int64_t k = std::min(m, n), rows = std::max(m, n);
    double* X = reinterpret_cast<double*>(b + L.off_X);
    double* J = reinterpret_cast<double*>(b + L.off_J);
    double* Uw = reinterpret_cast<double*>(b + L.off_Uw);
    double* Vw = reinterpret_cast<double*>(b + L.off_Vw);
    double* Sd = reinterpret_cast<double*>(b + L.off_S);
    unsigned* sync = reinterpret_cast<unsigned*>(b + L.off_sync);
    // P = A (tall: X column c = A column c) or A^T (wide: X column c = A row c, a row-major read)
    RSVD_CK(launch_block_jacobi_ex<double>(src, lds, tall ? 0 : 1, (int)rows, (int)k, L.MR, L.LP, X, J, Uw, Vw, Sd, sync,
                                           h->dflags + 1, s, sizeof(T) == 4 ? 1e-8 : 1e-16,
                                           sizeof(T) == 4 ? kBJTolF32 : kBJTolF64));
    RSVD_CK(launch_convert_scale<T>(Sd, S, (int)k, 1.0, s));
    // P J = (Uw) S: tall -> U = Uw (m rows), V = J; wide -> U = J (m = k rows), V = Uw (n rows)
    T* xside = tall ? U : V;
    const int64_t ldx = tall ? ldu : ldv;
    T* jside = tall ? V : U;
    const int64_t ldj = tall ? ldv : ldu;
    if constexpr (sizeof(T) == 8) {
        RSVD_CK(launch_panel_to_colmajor<double>(Uw, rows, (int)k, L.LP, xside, ldx, s));
        RSVD_CK(launch_panel_to_colmajor<double>(Vw, k, (int)k, L.LP, jside, ldj, s));
    } else {
        float* U32 = reinterpret_cast<float*>(b + L.off_Uw32);
        RSVD_CK(launch_convert_scale<float>(Uw, U32, (int)((int64_t)L.MR * L.LP), 1.0, s));
        RSVD_CK(launch_panel_to_colmajor<float>(U32, rows, (int)k, L.LP, xside, ldx, s));
        RSVD_CK(launch_convert_scale<float>(Vw, U32, L.LP * L.LP, 1.0, s));
        RSVD_CK(launch_panel_to_colmajor<float>(U32, k, (int)k, L.LP, jside, ldj, s));
    }
    return RSVD_OK;
}


// ---- rSVD() past 512 sketch columns (src/rSVD.cpp:72-133 has no cap on l) ------------------------
// The same algorithm as the wide engine, in column-major blocks: Omega (Philox, or the caller's;
// rounded to bf16 / e4m3 for those A types as rsvd_generate_omega documents), Y = A Omega,
// Q = orth(Y), q x {Z = A^T Q, X = orth(Z), Y = A X, Q = orth(Y)}, B^T = A^T Q, Q_B = orth(B^T),
// R = Q_B^T B^T, W = R^T = U_w S V_w^T (block Jacobi, l <= 4096), U = Q U_w, V = Q_B V_w.  Products
// on the MFMA GEMM (gemm.hip) in the panel precision (fp64 for fp64 A, fp32 otherwise; bf16 / e4m3
// A widened to fp32 once -- exact), orthonormalisations by orth_cols (block CGS2 + CholeskyQR3).
template <typename T>
struct BigLWs {
    QrBigWs<T> qm, qn;
    int MR, LP;
    size_t off_qm, off_qn, off_A32, off_Om, off_Y, off_Q, off_Z, off_X, off_R, off_R64, off_JX, off_JJ, off_Uw, off_Vw,
        off_U32, off_S, off_sync, off_om16, total;
    BigLWs(const rsvd_desc_t* d)
        // (the m-side basis has l columns even where a row shard holds fewer than l rows: its Grams and
        // block projections are summed over the ranks)
        : qm(d->m, d->l), qn(d->n, std::min<int64_t>(d->l, d->n)) {
        const int64_t m = d->m, n = d->n, l = d->l;
        MR = (int)rup(l, 32);
        LP = (int)rup(l, 32);
        const bool lowp = d->dtype == RSVD_BF16 || d->dtype == RSVD_FP8_E4M3;
        size_t o = 0;
        auto take = [&](size_t bytes) {
            const size_t at = o;
            o = align256(o + bytes);
            return at;
        };
        off_qm = take(qm.total);
        off_qn = take(qn.total);
        off_A32 = take(lowp ? sizeof(float) * (size_t)m * n : 0);
        off_Om = take(sizeof(T) * (size_t)n * l);
        off_Y = take(sizeof(T) * (size_t)m * l);
        off_Q = take(sizeof(T) * (size_t)m * l);
        off_Z = take(sizeof(T) * (size_t)n * l);
        off_X = take(sizeof(T) * (size_t)n * rup(l, 32));  // (also the Philox panel, pitch rup(l, 32))
        off_R = take(sizeof(T) * (size_t)l * l);
        off_R64 = take(sizeof(T) == 4 ? sizeof(double) * (size_t)l * l : 0);
        off_JX = take(sizeof(double) * 2 * (size_t)MR * LP);
        off_JJ = take(sizeof(double) * 2 * (size_t)LP * LP);
        off_Uw = take(sizeof(double) * (size_t)MR * LP);
        off_Vw = take(sizeof(double) * (size_t)LP * LP);
        off_U32 = take(sizeof(T) == 4 ? sizeof(float) * (size_t)MR * LP : 0);
        off_S = take(sizeof(double) * LP);
        off_sync = take(sizeof(unsigned) * kBJSyncWords);
        off_om16 = take(lowp ? (size_t)2 * n * rup(l, 16) : 0);
        total = o;
    }
};

template <typename T>
int big_rsvd_typed(rsvd_handle_t h, const rsvd_desc_t* d, const void* Av, const void* omega, int64_t ldo, void* U,
                   int64_t ldu, void* S, void* V, int64_t ldv, void* Qout, int64_t ldq) {
    BigLWs<T> L(d);
    RSVD_TRY(ensure_ws(h, L.total));
    RSVD_CK(reset_run_flags(h->dflags, h->stream));
    hipStream_t s = h->stream;
    char* b = h->ws;
    const int64_t m = d->m, n = d->n, l = d->l;
    auto ptr = [&](size_t off) { return reinterpret_cast<T*>(b + off); };
    T *Om = ptr(L.off_Om), *Y = ptr(L.off_Y), *Q = ptr(L.off_Q), *Z = ptr(L.off_Z), *X = ptr(L.off_X), *R = ptr(L.off_R);
    QrBig<T> Em(h, L.qm, b + L.off_qm), En(h, L.qn, b + L.off_qn);
    const bool lowp = d->dtype == RSVD_BF16 || d->dtype == RSVD_FP8_E4M3;
    const int f8 = d->dtype == RSVD_FP8_E4M3;
    // A in the panel precision
    const T* A = reinterpret_cast<const T*>(Av);
    int64_t lda = d->lda;
    if (lowp) {
        float* A32 = reinterpret_cast<float*>(b + L.off_A32);
        RSVD_CK(launch_lowp_to_f32(Av, d->lda, m, n, f8, A32, s));
        A = reinterpret_cast<const T*>(A32);
        lda = m;
    }
    // Omega (n x l, column-major)
    if (lowp) {
        const int LP16 = (int)rup(l, 16);
        uint16_t* pan = reinterpret_cast<uint16_t*>(b + L.off_om16);
        if (omega) {
            RSVD_CK(launch_omega_lowp_from(reinterpret_cast<const float*>(omega), ldo, n, (int)l, LP16, f8, pan, s));
            RSVD_CK(launch_bf16_panel_to_f32(pan, n, (int)l, LP16, reinterpret_cast<float*>(Om), n, s));
        } else {
            RSVD_CK(launch_omega_lowp(pan, n, (int)l, LP16, d->seed, f8, reinterpret_cast<float*>(Om), s));
        }
    } else if (omega) {
        RSVD_CK(hipMemcpy2DAsync(Om, sizeof(T) * n, omega, sizeof(T) * ldo, sizeof(T) * n, l, hipMemcpyDeviceToDevice, s));
    } else {
        // Philox in the panel layout (ld LP = l rounded to 32: X is free scratch until the first orth)
        const int LPo = (int)rup(l, 32);
        RSVD_CK(launch_philox_omega<T>(X, n, (int)l, LPo, d->seed, s));
        RSVD_CK(launch_panel_to_colmajor<T>(X, n, (int)l, LPo, Om, n, s));
    }
    const uint64_t sd = d->seed ^ 0xB16Full;
    // world > 1: this rank's rows of A (src/rSVD.cpp:20-23); the m-side panels stay row-sharded
    // (their Grams and block projections all-reduced), A^T Q is all-reduced, the n side replicated
    const int32_t tdt = sizeof(T) == 8 ? RSVD_F64 : RSVD_F32;
    if (h->world > 1) {
        // the global row count, the SAME on every rank: it sets the CholeskyQR shift, which must give
        // bit-identical R factors everywhere (world * m differed by rank under the reference's
        // remainder rule -- 1001 / 1000 rows -- and the ranks' Q then disagreed at 1.7e-4)
        if (!h->allreduce) {
            h->err = "l > 512 on several ranks needs the all-reduce hook";
            return RSVD_ERR_COMM;
        }
        // (summed in fp64 -- exact for any row count -- in the S slot, written only at the end)
        double* cnt = reinterpret_cast<double*>(b + L.off_S);
        const double mloc = (double)m;
        RSVD_CK(hipMemcpyAsync(cnt, &mloc, sizeof(double), hipMemcpyHostToDevice, s));
        if (h->allreduce(cnt, 1, RSVD_F64, (void*)s, h->ar_user) != 0) {
            h->err = "all-reduce hook failed";
            return RSVD_ERR_COMM;
        }
        double mg = 0;
        RSVD_CK(hipMemcpyAsync(&mg, cnt, sizeof(double), hipMemcpyDeviceToHost, s));
        RSVD_CK(hipStreamSynchronize(s));
        const int64_t m_global = (int64_t)(mg + 0.5);
        if (l > m_global) {  // (every rank sees the same count: all refuse)
            h->err = "l > min(m, n) not supported (m: the global row count of the sharded A)";
            return RSVD_ERR_UNSUPPORTED;
        }
        Em.shard = true;
        Em.row_off = (int64_t)h->rank << 40;
        Em.rows_total = (int64_t)h->world << 40;
        Em.norm_rows = m_global;
        Em.rows_global = m_global;
    }
    auto reduce_z = [&]() -> int {
        if (h->world <= 1 || !h->allreduce) return RSVD_OK;
        if (h->allreduce(Z, n * l, tdt, (void*)s, h->ar_user) != 0) {
            h->err = "all-reduce hook failed";
            return RSVD_ERR_COMM;
        }
        return RSVD_OK;
    };
    // intermediate_step (src/rSVD.cpp:57-70)
    RSVD_CK(launch_gemm<T>(0, 0, m, l, n, T(1), A, lda, Om, n, T(0), Y, m, s));  // Y = A Omega
    RSVD_TRY(Em.orth_cols(Y, m, l, Q, sd));
    for (int i = 0; i < d->q; ++i) {
        RSVD_CK(launch_gemm<T>(1, 0, n, l, m, T(1), A, lda, Q, m, T(0), Z, n, s));  // Z = A^T Q
        RSVD_TRY(reduce_z());
        RSVD_TRY(En.orth_cols(Z, n, l, X, sd + 1000003ull * (2 * i + 1)));
        RSVD_CK(launch_gemm<T>(0, 0, m, l, n, T(1), A, lda, X, n, T(0), Y, m, s));  // Y = A X
        RSVD_TRY(Em.orth_cols(Y, m, l, Q, sd + 1000003ull * (2 * i + 2)));
    }
    if (Qout) {
        RSVD_CK(hipMemcpy2DAsync(Qout, sizeof(T) * ldq, Q, sizeof(T) * m, sizeof(T) * m, l, hipMemcpyDeviceToDevice, s));
        return RSVD_OK;
    }
    // B^T = A^T Q, Q_B = orth(B^T), R = Q_B^T B^T (src/rSVD.cpp:89, SVD_class.hpp:116-123)
    RSVD_CK(launch_gemm<T>(1, 0, n, l, m, T(1), A, lda, Q, m, T(0), Z, n, s));
    RSVD_TRY(reduce_z());
    RSVD_TRY(En.orth_cols(Z, n, l, X, sd + 7));
    RSVD_CK(launch_gemm<T>(1, 0, l, l, n, T(1), X, n, Z, n, T(0), R, l, s));
    const double* R64 = reinterpret_cast<const double*>(R);
    if (sizeof(T) == 4) {
        double* w = reinterpret_cast<double*>(b + L.off_R64);
        RSVD_CK(launch_widen<T>(R, l, l, l, w, s));
        R64 = w;
    }
    RSVD_CK(launch_check_finite<double>(R64, (int)(l * l), h->dflags + kFlagNonFinite, s));
    // W = R^T: X column c = row c of R (the row-major read of the column-major R)
    double* JXp = reinterpret_cast<double*>(b + L.off_JX);
    double* JJp = reinterpret_cast<double*>(b + L.off_JJ);
    double* Uw = reinterpret_cast<double*>(b + L.off_Uw);
    double* Vw = reinterpret_cast<double*>(b + L.off_Vw);
    double* Sd = reinterpret_cast<double*>(b + L.off_S);
    unsigned* sync = reinterpret_cast<unsigned*>(b + L.off_sync);
    const double asc = d->a_scale != 0.0 ? d->a_scale : 1.0;
    if (d->method == RSVD_SVD_POWER) {
        // SVDMethod::Power (src/rSVD.cpp:106-113) past 512 sketch columns, in the coordinates of Q_B as
        // the wide engine's power stage (wide.cpp power_stage): start vectors Philox(power_seed(seed) + i)
        // over the n coordinates, X0s = Q_B^T X0, then the power method with deflation on P = R^T,
        // B = R R^T on the grid (dense.hip launch_power_grid_rsvd; the one-workgroup kernel holds l <= 512)
        T* X0 = Om;  // (free after the sketch) X0[r l + i] = x0_i[r]: the column-major view is X0^T (l x n)
        RSVD_CK(launch_power_start<T>(X0, n, (int)l, (int)l, power_seed(d->seed), s));
        double* X0s = JXp;  // l x l: column i = Q_B^T x0_i
        double* part = JXp + l * l;
        double* Yw = part + (int64_t)power_grid_size(l) * (l + 2);
        if constexpr (sizeof(T) == 8) {
            RSVD_CK(launch_gemm<T>(1, 1, l, l, n, T(1), X, n, X0, l, T(0), reinterpret_cast<T*>(X0s), l, s));
        } else {
            T* y0 = reinterpret_cast<T*>(Vw);  // (free until the power method writes V_c)
            RSVD_CK(launch_gemm<T>(1, 1, l, l, n, T(1), X, n, X0, l, T(0), y0, l, s));
            RSVD_CK(launch_widen<T>(y0, l, l, l, X0s, s));
        }
        RSVD_CK(launch_gemm<double>(0, 1, l, l, l, 1.0, R64, l, R64, l, 0.0, JJp, l, s));  // B = R R^T
        RSVD_CK(launch_power_grid_rsvd(R64, (int)l, JJp, X0s, power_iterations(n), Uw, Vw, Sd, Yw, part, sync,
                                       h->dflags + 16, h->dflags + kFlagGramTimeout, s));
        RSVD_CK(launch_convert_scale<T>(Sd, reinterpret_cast<T*>(S), (int)l, std::fabs(asc), s));
        // U = Q U_p, V = Q_B V_c (column-major l x l, ld l)
        const T* up = reinterpret_cast<const T*>(Uw);
        const T* vc = reinterpret_cast<const T*>(Vw);
        if (sizeof(T) == 4) {
            float* u32 = reinterpret_cast<float*>(b + L.off_U32);
            float* v32 = reinterpret_cast<float*>(JXp);  // X0s / part are spent
            RSVD_CK(launch_convert_scale<float>(Uw, u32, (int)(l * l), 1.0, s));
            RSVD_CK(launch_convert_scale<float>(Vw, v32, (int)(l * l), 1.0, s));
            up = reinterpret_cast<const T*>(u32);
            vc = reinterpret_cast<const T*>(v32);
        }
        RSVD_CK(launch_gemm<T>(0, 0, m, l, l, T(1), Q, m, up, l, T(0), reinterpret_cast<T*>(U), ldu, s));
        RSVD_CK(launch_gemm<T>(0, 0, n, l, l, T(1), X, n, vc, l, T(0), reinterpret_cast<T*>(V), ldv, s));
    } else {
    RSVD_CK(launch_block_jacobi_ex<double>(R64, l, 1, (int)l, (int)l, L.MR, L.LP, JXp, JJp, Uw, Vw, Sd, sync,
                                           h->dflags + 1, s, sizeof(T) == 4 ? 1e-8 : 1e-16,
                                           sizeof(T) == 4 ? kBJTolF32 : kBJTolF64));
    RSVD_CK(launch_convert_scale<T>(Sd, reinterpret_cast<T*>(S), (int)l, std::fabs(asc), s));
    // U = Q U_w, V = Q_B V_w (U_w, V_w row-major with pitch LP: their column-major views are the transposes)
    const T* uw = reinterpret_cast<const T*>(Uw);
    const T* vw = reinterpret_cast<const T*>(Vw);
    if (sizeof(T) == 4) {
        float* u32 = reinterpret_cast<float*>(b + L.off_U32);
        float* v32 = reinterpret_cast<float*>(JXp);  // free after the Jacobi finish
        RSVD_CK(launch_convert_scale<float>(Uw, u32, L.MR * L.LP, 1.0, s));
        RSVD_CK(launch_convert_scale<float>(Vw, v32, L.LP * L.LP, 1.0, s));
        uw = reinterpret_cast<const T*>(u32);
        vw = reinterpret_cast<const T*>(v32);
    }
    RSVD_CK(launch_gemm<T>(0, 1, m, l, l, T(1), Q, m, uw, L.LP, T(0), reinterpret_cast<T*>(U), ldu, s));
    RSVD_CK(launch_gemm<T>(0, 1, n, l, l, T(1), X, n, vw, L.LP, T(0), reinterpret_cast<T*>(V), ldv, s));
    }
    if (asc < 0.0) RSVD_CK(launch_scale_cols<T>(reinterpret_cast<T*>(V), n, (int)l, ldv, -1.0, s));
    RSVD_CK(launch_check_finite<T>(reinterpret_cast<const T*>(S), (int)l, h->dflags + kFlagNonFinite, s));
    return RSVD_OK;
}
}  // namespace

size_t qr_big_workspace(int64_t m, int64_t n, int full, int dtype) {
    const int64_t K = full ? m : n;
    return dtype == RSVD_F64 ? QrBigWs<double>(m, K).total : QrBigWs<float>(m, K).total;
}

size_t svd_big_workspace(int64_t m, int64_t n, int dtype) { return SvdBigWs(m, n, dtype).total; }

int qr_big(rsvd_handle_t h, int64_t m, int64_t n, const void* A, int64_t lda, int dtype, int full, void* Q, int64_t ldq,
           void* R, int64_t ldr) {
    if (dtype == RSVD_F64)
        return qr_big_typed<double>(h, m, n, static_cast<const double*>(A), lda, full, static_cast<double*>(Q), ldq,
                                    static_cast<double*>(R), ldr);
    return qr_big_typed<float>(h, m, n, static_cast<const float*>(A), lda, full, static_cast<float*>(Q), ldq,
                               static_cast<float*>(R), ldr);
}

int svd_big(rsvd_handle_t h, int64_t m, int64_t n, const void* A, int64_t lda, int dtype, void* U, int64_t ldu,
            void* S, void* V, int64_t ldv) {
    if (std::min(m, n) > 4096) {
        h->err = "SVD<Jacobi> is built for min(m, n) <= 4096";
        return RSVD_ERR_UNSUPPORTED;
    }
    if (dtype == RSVD_F64)
        return svd_big_typed<double>(h, m, n, static_cast<const double*>(A), lda, static_cast<double*>(U), ldu,
                                     static_cast<double*>(S), static_cast<double*>(V), ldv);
    return svd_big_typed<float>(h, m, n, static_cast<const float*>(A), lda, static_cast<float*>(U), ldu,
                                static_cast<float*>(S), static_cast<float*>(V), ldv);
}

size_t big_rsvd_workspace(const rsvd_desc_t* d) {
    return d->dtype == RSVD_F64 ? BigLWs<double>(d).total : BigLWs<float>(d).total;
}

int big_rsvd_run(rsvd_handle_t h, const rsvd_desc_t* d, const void* A, const void* omega, int64_t ldo, void* U,
                 int64_t ldu, void* S, void* V, int64_t ldv, void* Qout, int64_t ldq) {
    if (d->l > kBigLMax) {
        h->err = "l > 4096 not supported (the block Jacobi small SVD is built for l <= 4096)";
        return RSVD_ERR_UNSUPPORTED;
    }
    if (h->world > 1 && !h->allreduce) {
        h->err = "a row-sharded rSVD needs the all-reduce hook (rsvd_set_comm / rsvd_comm_init)";
        return RSVD_ERR_INVALID_ARG;
    }
    if (d->flags & RSVD_FLAG_FORCE_NSHARD) {  // (the n side past 512 columns is replicated, A^T Q all-reduced)
        h->err = "RSVD_FLAG_FORCE_NSHARD: the sharded n-side path is built for l <= 512";
        return RSVD_ERR_UNSUPPORTED;
    }
    if (!Qout && d->method == RSVD_SVD_POWER_IC) {
        h->err = "RSVD_SVD_POWER_IC (image_compression's power method) is built for l <= 512";
        return RSVD_ERR_UNSUPPORTED;
    }
    if (d->dtype == RSVD_F64) return big_rsvd_typed<double>(h, d, A, omega, ldo, U, ldu, S, V, ldv, Qout, ldq);
    return big_rsvd_typed<float>(h, d, A, omega, ldo, U, ldu, S, V, ldv, Qout, ldq);
}

}  // namespace rsvd
