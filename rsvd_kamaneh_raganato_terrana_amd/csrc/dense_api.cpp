// dense.cpp -- the QR() and SVD<method> drop-ins on the wide engine's
// kernels.
//
// QR  (qr_decomposition_reduced / _full, src/QR.cpp:22-80).  The reference eliminates with
// Givens rotations, O(m^2 n) work on an m x m Q.  Here: Q = orth(A) by shifted CholeskyQR3 (a
// shifted first pass keeps the Gram positive definite up to cond(A) ~ 1/u, then CholeskyQR2),
// with the rank-deficiency repair of the rSVD panels; then R = Q^T A (cross Gram, fp64) with the
// strictly lower part zeroed.  For full rank A the QR with a positive diagonal is unique, so Q and
// R equal the reference's; the sign rule of Givens (a column whose sub-diagonal is already zero
// gets no rotation and keeps the sign of A(j,j)) is applied to the leading run of such columns
// (dense.hip qr_signs).  Full QR: the basis [A | e_n .. e_{m-1}] (identity completion, as the
// reference's Q starts from the identity) is orthonormalised the same way, so Q[:, :n] is the
// reduced Q and Q[:, n:] an orthonormal complement.
//
// SVD<Jacobi> / SVD<ParallelJacobi> (SVD_class.hpp:100-180, 223-333): the reference QR-
// preconditions a rectangular A (Householder) and runs two-sided Jacobi on the min(m,n)^2
// triangle.  Here: P = A (m >= n) or A^T (m < n) as a row-major panel, Q_P = orth(P) as above,
// W = Q_P^T P (cross Gram), the one-sided Jacobi small SVD of the wide engine (jacobi.hip for
// min(m,n) <= 64, the block Jacobi of wide_svd.hip up to 512): P = (Q_P U_w) S V_w^T -- the
// converged SVD, which is what the reference's Jacobi (cyclic, stop at 2 eps maxDiag) returns.
// ParallelJacobi stops at the ABSOLUTE weight 1e-12 (off-diagonals up to ~1e-6 survive), so its
// vectors depend on the rotation order; it runs the reference's own order here (dense.hip
// pjacobi_ref_kernel: weight-sorted, sequential, one workgroup) on W = R_P / R_P^T / A (square).
//
// SVD<Power> (SVD_class.hpp:183-219, src/PM.cpp:4-81): B = A^T A by the fp64 Gram kernel, then
// the power method with deflation in one workgroup (dense.hip power_svd_kernel).
//
// Past 512 columns (QR with max(Q columns, n) > 512, SVD<Jacobi / ParallelJacobi> with
// min(m, n) > 512) the blocked forms of dense_big.cpp take over.
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

// LP for a k-column factorisation: multiples of 16 up to 64 (jacobi.hip), of 32 beyond (block Jacobi).
int dense_lp(int64_t k) { return (int)(k <= 64 ? rup(std::max<int64_t>(k, 1), 16) : rup(k, 32)); }

template <typename T>
struct DenseWs {
    int64_t rows;
    int LP;
    GramPlan gp, gx;
    size_t off_P, off_Q, off_T1, off_T2, off_gslab, off_G, off_R, off_Rinv, off_W, off_R1, off_Uw, off_Vw, off_JX,
        off_JJ, off_M32, off_S, off_colflag, off_sync, total;
    DenseWs(int64_t rows_, int LP_) : rows(rows_), LP(LP_) {
        gp = plan_gram_wide(rows, LP, 0);
        gx = plan_gram_wide(rows, LP, 1);
        const size_t gslab = (size_t)std::max(gp.blocks * gp.chunks, gx.blocks * gx.chunks) * 1024;
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
        off_gslab = take(sizeof(double) * gslab);
        off_G = take(sizeof(double) * L2);
        off_R = take(sizeof(double) * L2);
        off_Rinv = take(sizeof(double) * L2);
        off_W = take(sizeof(double) * L2);
        off_R1 = take(sizeof(double) * L2);
        off_Uw = take(sizeof(double) * L2);
        off_Vw = take(sizeof(double) * L2);
        off_JX = take(sizeof(double) * 2 * L2);
        off_JJ = take(sizeof(double) * 2 * L2);
        off_M32 = take(sizeof(float) * 3 * L2);
        off_S = take(sizeof(double) * LP);
        off_colflag = take(sizeof(int) * LP);
        off_sync = take(sizeof(unsigned) * kBJSyncWords);
        total = o;
    }
};

template <typename T>
struct DenseEngine {
    rsvd_handle_t h;
    const DenseWs<T>& L;
    hipStream_t s;
    T *P, *Q, *T1, *T2;
    double *gslab, *G, *R, *Rinv, *W, *R1, *Uw, *Vw, *JX, *JJ, *Sd;
    float *Rinv32, *Uw32, *Vw32;
    int* colflag;
    unsigned* sync;
    int* flag;

    DenseEngine(rsvd_handle_t h_, const DenseWs<T>& L_) : h(h_), L(L_), s(h_->stream) {
        char* b = h->ws;
        P = reinterpret_cast<T*>(b + L.off_P);
        Q = reinterpret_cast<T*>(b + L.off_Q);
        T1 = reinterpret_cast<T*>(b + L.off_T1);
        T2 = reinterpret_cast<T*>(b + L.off_T2);
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
        Sd = reinterpret_cast<double*>(b + L.off_S);
        colflag = reinterpret_cast<int*>(b + L.off_colflag);
        sync = reinterpret_cast<unsigned*>(b + L.off_sync);
        flag = h->dflags + 4;
    }

    double tol() const { return sizeof(T) == 4 ? 1e-13 : 1e-28; }
    const T* mat(const double* m64, const float* m32) const {
        if constexpr (sizeof(T) == 8) return m64; else return m32;
    }

    int pass(const T* In, int k, T* Out, bool shift, const int* pred) {
        RSVD_CK(launch_gram_wide<T>(In, nullptr, L.rows, L.LP, L.gp, gslab, G, pred, s));
        if (shift) RSVD_CK(launch_shift_diag(G, L.LP, k, L.rows, sizeof(T) == 4 ? 0x1p-24 : 0x1p-53, s));
        RSVD_CK(launch_chol_wide(G, k, L.LP, tol(), R, Rinv, sizeof(T) == 4 ? Rinv32 : nullptr, colflag, flag, W, pred,
                                 s));
        // forward substitution rather than the R^-1 product: backward stable for ill-conditioned R
        RSVD_CK(launch_trsm_rows<T>(In, L.rows, k, L.LP, R, Out, pred, s));
        return RSVD_OK;
    }

    // Q = orth(In[:, :k]): shifted CholeskyQR3 + the predicated repair of flagged columns.
    int orth(const T* In, int k, uint64_t seed) {
        RSVD_TRY(pass(In, k, T1, true, nullptr));
        RSVD_TRY(pass(T1, k, T2, false, nullptr));
        RSVD_TRY(pass(T2, k, Q, false, nullptr));
        RSVD_CK(launch_repair_panel<T>(Q, L.rows, k, L.LP, colflag, flag, seed, 0, L.rows, L.rows, T1, s));
        RSVD_TRY(pass(T1, k, Q, false, flag));
        return RSVD_OK;
    }
};

bool ok_dtype(int dt) { return dt == RSVD_F64 || dt == RSVD_F32; }

int prepare(rsvd_handle_t h, size_t bytes) {
    RSVD_CK(hipSetDevice(h->device));
    RSVD_TRY(ensure_ws(h, bytes));
    RSVD_CK(reset_run_flags(h->dflags, h->stream));
    return RSVD_OK;
}

template <typename T>
int qr_typed(rsvd_handle_t h, int64_t m, int64_t n, const T* A, int64_t lda, int full, T* Qo, int64_t ldq, T* Ro,
             int64_t ldr) {
    const int64_t kq = full ? m : n;  // columns of Q (= rows of R)
    DenseWs<T> L(m, dense_lp(std::max(kq, n)));
    RSVD_TRY(prepare(h, L.total));
    DenseEngine<T> E(h, L);
    RSVD_CK(launch_colmajor_to_panel<T>(A, lda, m, (int)n, L.LP, E.P, h->stream));
    const T* basis = E.P;
    if (full && kq != n) {  // [A | e_n .. e_{m-1}], or the leading m columns of a wide A
        RSVD_CK(launch_colmajor_to_panel<T>(A, lda, m, (int)std::min(m, n), L.LP, E.T2, h->stream));
        RSVD_CK(launch_unit_columns<T>(E.T2, L.LP, (int)std::min(m, n), (int)m, h->stream));
        // T2 is scratch of orth(): park the basis in Q's slot first
        RSVD_CK(hipMemcpyAsync(E.Q, E.T2, sizeof(T) * m * L.LP, hipMemcpyDeviceToDevice, h->stream));
        basis = E.Q;
    }
    RSVD_TRY(E.orth(basis, (int)kq, 0x51A7ull + (uint64_t)m * 131 + (uint64_t)n));
    RSVD_CK(launch_qr_signs<T>(A, lda, m, (int)n, E.Q, L.LP, h->stream));
    if (kq == m) RSVD_CK(launch_det_sign<T>(E.Q, (int)m, L.LP, E.W, h->stream));  // square Q: det +1
    RSVD_CK(launch_gram_wide<T>(E.Q, E.P, m, L.LP, L.gx, E.gslab, E.R1, nullptr, h->stream));  // R = Q^T A
    RSVD_CK(launch_panel_to_colmajor<T>(E.Q, m, (int)kq, L.LP, Qo, ldq, h->stream));
    RSVD_CK(launch_upper_to_colmajor<T>(E.R1, L.LP, (int)kq, (int)n, Ro, ldr, h->stream));
    return RSVD_OK;
}

template <typename T>
int svd_jacobi_typed(rsvd_handle_t h, int64_t m, int64_t n, const T* A, int64_t lda, T* U, int64_t ldu, T* S, T* V,
                     int64_t ldv, bool reference_order) {
    const bool tall = m >= n;
    const int64_t k = std::min(m, n), rows = std::max(m, n);
    DenseWs<T> L(rows, dense_lp(k));
    RSVD_TRY(prepare(h, L.total));
    DenseEngine<T> E(h, L);
    hipStream_t s = h->stream;
    if (reference_order && m == n) {  // square: Jacobi on A itself (SVD_class.hpp:246-249), U = Jl, V = Jr
        RSVD_CK(launch_pjacobi_ref<T>(A, 1, lda, 0, (int)k, L.LP, E.W, E.Uw, E.Vw, E.Sd, E.JX, h->dflags + 1, s));
        RSVD_CK(launch_convert_scale<T>(E.Sd, S, (int)k, 1.0, s));
        if (sizeof(T) == 4) {
            const int L2 = L.LP * L.LP;
            RSVD_CK(launch_convert_scale<float>(E.Uw, E.Uw32, L2, 1.0, s));
            RSVD_CK(launch_convert_scale<float>(E.Vw, E.Vw32, L2, 1.0, s));
        }
        RSVD_CK(launch_panel_to_colmajor<T>(E.mat(E.Uw, E.Uw32), k, (int)k, L.LP, U, ldu, s));
        RSVD_CK(launch_panel_to_colmajor<T>(E.mat(E.Vw, E.Vw32), k, (int)k, L.LP, V, ldv, s));
        return RSVD_OK;
    }
    if (tall)
        RSVD_CK(launch_colmajor_to_panel<T>(A, lda, m, (int)n, L.LP, E.P, s));
    else
        RSVD_CK(launch_transpose_to_panel<T>(A, lda, m, n, L.LP, E.P, s));
    RSVD_TRY(E.orth(E.P, (int)k, 0x5BDull + (uint64_t)rows));
    RSVD_CK(launch_gram_wide<T>(E.P, E.Q, rows, L.LP, L.gx, E.gslab, E.R1, nullptr, s));  // R1 = P^T Q = R_P^T
    if (reference_order)  // W = R_P (tall) or R_P^T (wide, SVD_class.hpp:230-245) in R1 = R_P^T
        RSVD_CK(launch_pjacobi_ref<double>(E.R1, tall ? 1 : L.LP, tall ? L.LP : 1, tall ? 1 : -1, (int)k, L.LP, E.W, E.Uw, E.Vw, E.Sd,
                                           E.JX, h->dflags + 1, s));
    else if (L.LP <= 64)
        RSVD_CK(launch_small_svd<double>(E.R1, (int)k, L.LP, E.Uw, E.Vw, E.Sd, h->dflags + 1, s));
    else
        RSVD_CK(launch_block_jacobi<double>(E.R1, (int)k, L.LP, E.JX, E.JJ, E.Uw, E.Vw, E.Sd, E.sync, h->dflags + 1, s));
    RSVD_CK(launch_convert_scale<T>(E.Sd, S, (int)k, 1.0, s));
    if (sizeof(T) == 4) {
        const int L2 = L.LP * L.LP;
        RSVD_CK(launch_convert_scale<float>(E.Uw, E.Uw32, L2, 1.0, s));
        RSVD_CK(launch_convert_scale<float>(E.Vw, E.Vw32, L2, 1.0, s));
    }
    const T* Uwt = E.mat(E.Uw, E.Uw32);
    const T* Vwt = E.mat(E.Vw, E.Vw32);
    // P = (Q U_w) S V_w^T;  A = P (tall) or P^T (wide).  Reference order: W = Jl S Jr^T with W = R_P
    // (tall: A = (Q Jl) S Jr^T) or W = R_P^T (wide: A = Jl S (Q Jr)^T)
    T* left = tall ? U : V;
    const int64_t ldl = tall ? ldu : ldv;
    T* right = tall ? V : U;
    const int64_t ldr = tall ? ldv : ldu;
    const T* Qside = (reference_order && !tall) ? Vwt : Uwt;
    const T* Kside = (reference_order && !tall) ? Uwt : Vwt;
    RSVD_CK(launch_panel_gemm<T>(E.Q, rows, L.LP, Qside, 0, left, ldl, (int)k, nullptr, nullptr, nullptr, s));
    RSVD_CK(launch_panel_to_colmajor<T>(Kside, k, (int)k, L.LP, right, ldr, s));
    return RSVD_OK;
}

int svd_power(rsvd_handle_t h, int64_t m, int64_t n, const double* A, int64_t lda, int dim, uint64_t seed, double* U,
              int64_t ldu, double* S, double* V, int64_t ldv, int32_t* kept) {
    DenseWs<double> L(m, (int)rup(n, 16));
    RSVD_TRY(prepare(h, L.total));
    DenseEngine<double> E(h, L);
    hipStream_t s = h->stream;
    RSVD_CK(launch_colmajor_to_panel<double>(A, lda, m, (int)n, L.LP, E.P, s));
    RSVD_CK(launch_gram_wide<double>(E.P, nullptr, m, L.LP, L.gp, E.gslab, E.G, nullptr, s));  // B = A^T A (:193)
    RSVD_CK(hipMemsetAsync(E.Q, 0, sizeof(double) * m * L.LP, s));
    int* dk = h->dflags + 16;
    RSVD_CK(launch_power_svd(E.P, m, (int)n, L.LP, E.G, dim, seed, power_iterations(n), E.Q, E.Vw, E.Sd, dk, s));
    int k = 0;
    RSVD_CK(hipMemcpyAsync(&k, dk, sizeof(int), hipMemcpyDeviceToHost, s));
    RSVD_CK(hipStreamSynchronize(s));
    *kept = k;
    if (k == 0) return RSVD_OK;
    RSVD_CK(launch_panel_to_colmajor<double>(E.Q, m, k, L.LP, U, ldu, s));
    RSVD_CK(hipMemcpy2DAsync(V, sizeof(double) * ldv, E.Vw, sizeof(double) * L.LP, sizeof(double) * n, k,
                             hipMemcpyDeviceToDevice, s));  // column i of V = row i of V_r
    RSVD_CK(hipMemcpyAsync(S, E.Sd, sizeof(double) * k, hipMemcpyDeviceToDevice, s));
    return RSVD_OK;
}

// SVD<Power> with n > 512: B (n x n), the iterate pair, the grid partials, the barrier words, kept
struct PowerGridWs {
    size_t off_B, off_Y, off_part, off_sync, off_kept, total;
    PowerGridWs(int64_t n, int64_t dim) {
        size_t o = 0;
        auto take = [&](size_t bytes) {
            const size_t at = o;
            o = align256(o + bytes);
            return at;
        };
        off_B = take(sizeof(double) * (size_t)n * n);
        off_Y = take(sizeof(double) * 2 * (size_t)n);
        off_part = take(sizeof(double) * (size_t)power_grid_size(n) * (dim + 2));
        off_sync = take(8 * sizeof(unsigned));
        off_kept = take(sizeof(int));
        total = o;
    }
};

int svd_power_grid(rsvd_handle_t h, int64_t m, int64_t n, const double* A, int64_t lda, int dim, uint64_t seed,
                   double* U, int64_t ldu, double* S, double* V, int64_t ldv, int32_t* kept) {
    PowerGridWs L(n, dim);
    RSVD_TRY(prepare(h, L.total));
    hipStream_t s = h->stream;
    char* b = h->ws;
    double* B = reinterpret_cast<double*>(b + L.off_B);
    int* dk = reinterpret_cast<int*>(b + L.off_kept);
    RSVD_CK(launch_gram_colmajor(A, lda, m, n, B, s));  // B = A^T A (SVD_class.hpp:193)
    RSVD_CK(launch_power_grid(A, lda, m, n, B, dim, seed, power_iterations(n), U, ldu, V, ldv, S,
                              reinterpret_cast<double*>(b + L.off_Y), reinterpret_cast<double*>(b + L.off_part),
                              reinterpret_cast<unsigned*>(b + L.off_sync), dk, h->dflags + kFlagGramTimeout, s));
    int k = 0;
    RSVD_CK(hipMemcpyAsync(&k, dk, sizeof(int), hipMemcpyDeviceToHost, s));
    RSVD_CK(hipStreamSynchronize(s));
    *kept = k;
    return RSVD_OK;
}

size_t ws_bytes(int64_t rows, int LP, int dtype) {
    return dtype == RSVD_F64 ? DenseWs<double>(rows, LP).total : DenseWs<float>(rows, LP).total;
}

struct DevBuf {
    void* p = nullptr;
    ~DevBuf() {
        if (p) (void)hipFree(p);
    }
};

}  // namespace

// dense_big.cpp: past the 512-column panels
size_t qr_big_workspace(int64_t m, int64_t n, int full, int dtype);
size_t svd_big_workspace(int64_t m, int64_t n, int dtype);
int qr_big(rsvd_handle_t h, int64_t m, int64_t n, const void* A, int64_t lda, int dtype, int full, void* Q, int64_t ldq,
           void* R, int64_t ldr);
int svd_big(rsvd_handle_t h, int64_t m, int64_t n, const void* A, int64_t lda, int dtype, void* U, int64_t ldu,
            void* S, void* V, int64_t ldv);

}  // namespace rsvd

using namespace rsvd;

extern "C" {

int rsvd_qr_workspace_bytes(int64_t m, int64_t n, int32_t dtype, int32_t full, size_t* bytes) {
    if (!bytes || m < 1 || n < 1) return RSVD_ERR_INVALID_ARG;
    if (!ok_dtype(dtype)) return RSVD_ERR_UNSUPPORTED;
    const int64_t kq = full ? m : n;
    *bytes = std::max(kq, n) > 512 ? qr_big_workspace(m, n, full, dtype) : ws_bytes(m, dense_lp(std::max(kq, n)), dtype);
    return RSVD_OK;
}

int rsvd_svd_workspace_bytes(int64_t m, int64_t n, int32_t dtype, int32_t method, size_t* bytes) {
    if (!bytes || m < 1 || n < 1) return RSVD_ERR_INVALID_ARG;
    if (!ok_dtype(dtype)) return RSVD_ERR_UNSUPPORTED;
    if (method == RSVD_SVD_POWER)
        *bytes = n > 512 ? PowerGridWs(n, std::min(m, n)).total : ws_bytes(m, (int)rup(n, 16), RSVD_F64);
    else if (std::min(m, n) > 512)
        *bytes = svd_big_workspace(m, n, dtype);
    else
        *bytes = ws_bytes(std::max(m, n), dense_lp(std::min(m, n)), dtype);
    return RSVD_OK;
}

int rsvd_qr(rsvd_handle_t h, int64_t m, int64_t n, const void* A, int64_t lda, int32_t dtype, int32_t full, void* Q,
            int64_t ldq, void* R, int64_t ldr) {
    if (!h) return RSVD_ERR_INVALID_ARG;
    if (!A || !Q || !R || m < 1 || n < 1 || lda < m) {
        h->err = "null pointer or bad size";
        return RSVD_ERR_INVALID_ARG;
    }
    if (!ok_dtype(dtype)) {
        h->err = "QR supports F64 and F32";
        return RSVD_ERR_UNSUPPORTED;
    }
    const int64_t kq = full ? m : n;
    if (!full && m < n) {
        h->err = "qr_decomposition_reduced requires rows >= cols";  // Q_temp.leftCols(n), src/QR.cpp:78
        return RSVD_ERR_INVALID_ARG;
    }
    if (ldq < m || ldr < kq) {
        h->err = "bad leading dimension";
        return RSVD_ERR_INVALID_ARG;
    }
    if (std::max(kq, n) > 512) return qr_big(h, m, n, A, lda, dtype, full, Q, ldq, R, ldr);  // dense_big.cpp
    if (dtype == RSVD_F64)
        return qr_typed<double>(h, m, n, static_cast<const double*>(A), lda, full, static_cast<double*>(Q), ldq,
                                static_cast<double*>(R), ldr);
    return qr_typed<float>(h, m, n, static_cast<const float*>(A), lda, full, static_cast<float*>(Q), ldq,
                           static_cast<float*>(R), ldr);
}

int rsvd_svd(rsvd_handle_t h, int64_t m, int64_t n, const void* A, int64_t lda, int32_t dtype, int32_t method,
             int32_t r, uint64_t seed, void* U, int64_t ldu, void* S, void* V, int64_t ldv, int32_t* kept) {
    if (!h) return RSVD_ERR_INVALID_ARG;
    if (!A || !U || !S || !V || !kept || m < 1 || n < 1 || lda < m || ldu < m || ldv < n) {
        h->err = "null pointer or bad size";
        return RSVD_ERR_INVALID_ARG;
    }
    if (method != RSVD_SVD_JACOBI && method != RSVD_SVD_PARALLEL_JACOBI && method != RSVD_SVD_POWER) {
        h->err = "Unsupported SVD method";
        return RSVD_ERR_UNSUPPORTED;
    }
    if (!ok_dtype(dtype) || (method == RSVD_SVD_POWER && dtype != RSVD_F64)) {
        h->err = "SVD supports F64 and F32 (Power: F64)";
        return RSVD_ERR_UNSUPPORTED;
    }
    const int64_t k = std::min(m, n);
    if (method == RSVD_SVD_POWER) {
        const int64_t dim = r > 0 ? r : k;
        if (r < 0 || dim > k) {
            h->err = "r must be in [0, min(m, n)]";
            return RSVD_ERR_INVALID_ARG;
        }
        if (n > 512)  // B = A^T A no longer fits one workgroup: the grid power method
            return svd_power_grid(h, m, n, static_cast<const double*>(A), lda, (int)dim, seed, static_cast<double*>(U),
                                  ldu, static_cast<double*>(S), static_cast<double*>(V), ldv, kept);
        return svd_power(h, m, n, static_cast<const double*>(A), lda, (int)dim, seed, static_cast<double*>(U), ldu,
                         static_cast<double*>(S), static_cast<double*>(V), ldv, kept);
    }
    *kept = (int32_t)k;
    if (k > 512) return svd_big(h, m, n, A, lda, dtype, U, ldu, S, V, ldv);  // dense_big.cpp
    const bool ref_order = method == RSVD_SVD_PARALLEL_JACOBI;
    if (dtype == RSVD_F64)
        return svd_jacobi_typed<double>(h, m, n, static_cast<const double*>(A), lda, static_cast<double*>(U), ldu,
                                        static_cast<double*>(S), static_cast<double*>(V), ldv, ref_order);
    return svd_jacobi_typed<float>(h, m, n, static_cast<const float*>(A), lda, static_cast<float*>(U), ldu,
                                   static_cast<float*>(S), static_cast<float*>(V), ldv, ref_order);
}

int rsvd_qr_host_f64(rsvd_handle_t h, int64_t m, int64_t n, const double* A, int64_t lda, int32_t full, double* Q,
                     double* R) {
    if (!h || !A || !Q || !R || m < 1 || n < 1 || lda < m) return RSVD_ERR_INVALID_ARG;
    RSVD_CK(hipSetDevice(h->device));
    const int64_t kq = full ? m : n;
    DevBuf dA, dQ, dR;
    RSVD_CK(hipMalloc(&dA.p, sizeof(double) * m * n));
    RSVD_CK(hipMalloc(&dQ.p, sizeof(double) * m * kq));
    RSVD_CK(hipMalloc(&dR.p, sizeof(double) * kq * n));
    RSVD_CK(hipMemcpy2DAsync(dA.p, sizeof(double) * m, A, sizeof(double) * lda, sizeof(double) * m, n,
                             hipMemcpyHostToDevice, h->stream));
    RSVD_TRY(rsvd_qr(h, m, n, dA.p, m, RSVD_F64, full, dQ.p, m, dR.p, kq));
    RSVD_CK(hipMemcpyAsync(Q, dQ.p, sizeof(double) * m * kq, hipMemcpyDeviceToHost, h->stream));
    RSVD_CK(hipMemcpyAsync(R, dR.p, sizeof(double) * kq * n, hipMemcpyDeviceToHost, h->stream));
    return rsvd_sync(h);
}

int rsvd_svd_host_f64(rsvd_handle_t h, int64_t m, int64_t n, const double* A, int64_t lda, int32_t method, int32_t r,
                      uint64_t seed, double* U, double* S, double* V, int32_t* kept) {
    if (!h || !A || !U || !S || !V || !kept || m < 1 || n < 1 || lda < m) return RSVD_ERR_INVALID_ARG;
    RSVD_CK(hipSetDevice(h->device));
    const int64_t k = std::min(m, n);
    DevBuf dA, dU, dS, dV;
    RSVD_CK(hipMalloc(&dA.p, sizeof(double) * m * n));
    RSVD_CK(hipMalloc(&dU.p, sizeof(double) * m * k));
    RSVD_CK(hipMalloc(&dS.p, sizeof(double) * k));
    RSVD_CK(hipMalloc(&dV.p, sizeof(double) * n * k));
    RSVD_CK(hipMemcpy2DAsync(dA.p, sizeof(double) * m, A, sizeof(double) * lda, sizeof(double) * m, n,
                             hipMemcpyHostToDevice, h->stream));
    RSVD_TRY(rsvd_svd(h, m, n, dA.p, m, RSVD_F64, method, r, seed, dU.p, m, dS.p, dV.p, n, kept));
    const int64_t kk = *kept;
    RSVD_CK(hipMemcpyAsync(U, dU.p, sizeof(double) * m * kk, hipMemcpyDeviceToHost, h->stream));
    RSVD_CK(hipMemcpyAsync(S, dS.p, sizeof(double) * kk, hipMemcpyDeviceToHost, h->stream));
    RSVD_CK(hipMemcpyAsync(V, dV.p, sizeof(double) * n * kk, hipMemcpyDeviceToHost, h->stream));
    return rsvd_sync(h);
}

}  // extern "C"
