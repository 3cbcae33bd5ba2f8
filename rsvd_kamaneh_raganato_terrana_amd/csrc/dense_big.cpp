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

    QrBig(rsvd_handle_t h_, const QrBigWs<T>& L_) : h(h_), s(h_->stream), L(L_) {
        char* b = h->ws + L.off_bo;
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
        Y = reinterpret_cast<T*>(h->ws + L.off_Y);
        C = reinterpret_cast<T*>(h->ws + L.off_C);
    }

    double tol() const { return sizeof(T) == 4 ? 1e-13 : 1e-28; }

    // one CholeskyQR pass on a k-column panel (forward substitution: backward stable)
    int pass(const T* In, int k, T* Out, bool shift, const int* pred) {
        const int64_t rows = L.bo.rows;
        const int LP = L.bo.LP;
        int* flag = h->dflags + 4;
        RSVD_CK(launch_gram_wide<T>(In, nullptr, rows, LP, L.bo.gp, gslab, G, pred, s));
        if (shift) RSVD_CK(launch_shift_diag(G, LP, k, rows, sizeof(T) == 4 ? 0x1p-24 : 0x1p-53, s));
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
        RSVD_CK(launch_repair_panel<T>(Q, rows, k, L.bo.LP, colflag, h->dflags + 4, seed, 0, rows, rows, T1, s));
        RSVD_TRY(pass(T1, k, Q, false, h->dflags + 4));
        return RSVD_OK;
    }
    // Y (m x w, ld m) -= Qp (Qp^T Y), Qp = the first c0 columns of Q (ld ldq)
    int project(const T* Qp, int64_t ldq, int64_t m, int64_t c0, int w) {
        if (c0 == 0) return RSVD_OK;
        RSVD_CK(launch_gemm<T>(1, 0, c0, w, m, T(1), Qp, ldq, Y, m, T(0), C, c0, s));
        RSVD_CK(launch_gemm<T>(0, 0, m, w, c0, T(-1), Qp, ldq, C, c0, T(1), Y, m, s));
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

}  // namespace rsvd
