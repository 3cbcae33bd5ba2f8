// dense.hpp -- launch wrappers of dense.hip (the QR() and SVD<method> drop-ins, dense.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rsvd {

// P (n x LP row-major) = A^T for A m x n column-major (lda); columns m..LP-1 of P are zero.
template <typename T>
hipError_t launch_transpose_to_panel(const T* A, int64_t lda, int64_t m, int64_t n, int LP, T* P, hipStream_t s);
// P[j][j] = 1 for j in [c0, c1) (identity completion columns of the full QR basis).
template <typename T>
hipError_t launch_unit_columns(T* P, int LP, int c0, int c1, hipStream_t s);
// R (nr x nc column-major, ldr) = upper triangle of Rf (LP x LP fp64 row-major), zeros below.
template <typename T>
hipError_t launch_upper_to_colmajor(const double* Rf, int LP, int nr, int nc, T* R, int64_t ldr, hipStream_t s);
// G[:l,:l] += 11 (rows l + l (l+1)) u tr(G) I  (shifted CholeskyQR3, first pass)
hipError_t launch_shift_diag(double* G, int LP, int l, int64_t rows, double u, hipStream_t s);
// Givens sign convention (src/QR.cpp:31-39): a leading column whose sub-diagonal is already zero
// gets no rotation, so R(j,j) keeps the sign of A(j,j).  For the leading run of such columns of A
// (m x n, lda), negate column j of the Q panel (m x LP) where A(j,j) < 0.
template <typename T>
hipError_t launch_qr_signs(const T* A, int64_t lda, int64_t m, int n, T* Qp, int LP, hipStream_t s);
// Out (rows x LP) = In R^-1, R upper LP x LP fp64, by row-wise forward substitution (backward
// stable for any cond(R)); columns >= k of Out are 0.  `pred`: skip unless *pred != 0.
template <typename T>
hipError_t launch_trsm_rows(const T* In, int64_t rows, int k, int LP, const double* R, T* Out, const int* pred,
                            hipStream_t s);
// Square Q (m x m panel): negate column m-1 when det(Q) < 0 (the Givens Q has det +1).  W: LP x
// LP fp64 scratch.  One workgroup, LU with partial pivoting.
template <typename T>
hipError_t launch_det_sign(T* Qp, int m, int LP, double* W, hipStream_t s);
// SVD<Power> for any n (dense.hip power_grid_kernel): B = A^T A (n x n fp64, full) from A (m x n
// column-major), then the power method with deflation on a persistent grid of power_grid_size(n)
// workgroups (row partition of B as src/PM.cpp:31-35).  U m x dim (ldu), V n x dim (ldv, v_i in
// column i), S dim, *kept; Y: 2 n, part: grid x (dim + 2) doubles, sync: 8 words; *tmo |= 1 when a
// grid barrier times out.
hipError_t launch_gram_colmajor(const double* A, int64_t lda, int64_t m, int64_t n, double* B, hipStream_t s);
int power_grid_size(int64_t n);
hipError_t launch_power_grid(const double* A, int64_t lda, int64_t m, int64_t n, double* B, int dim, uint64_t seed,
                             int iters, double* U, int64_t ldu, double* V, int64_t ldv, double* S, double* Y,
                             double* part, unsigned* sync, int* kept, int* tmo, hipStream_t s);
// SVDMethod::Power of the rSVD in the coordinates of Q_B on the grid (any l; the one-workgroup
// launch_power_svd holds l <= 512): P = R^T for the column-major l x l R = Q_B^T B^T (ld l), B = R R^T,
// start vectors X0s (column i = Q_B^T x0_i), U_p / V_c column-major l x l (u_i, v_i in column i;
// zero past an early stop), S (l).  Work as launch_power_grid (Y 2 l, part power_grid_size(l) (l + 2), sync 8).
hipError_t launch_power_grid_rsvd(const double* R, int l, double* B, const double* X0s, int iters, double* Up,
                                  double* Vc, double* S, double* Y, double* part, unsigned* sync, int* kept, int* tmo,
                                  hipStream_t s);
// SVD<ParallelJacobi> with the reference's iteration (weight-sorted sequential two-sided Jacobi,
// SVD_class.hpp:223-333): W(p, q) = Win[p sp + q sq] (d x d; tri > 0 / < 0: upper / lower
// triangular) copied to W (LP pitch); Jl / Jr (LP x
// LP row-major) accumulate the left / right rotations; S (d) sorted descending with Jl / Jr columns
// permuted alike; info[0] = sweeps.  list: pjacobi_ref_list_bytes(d) of scratch.  One workgroup.
size_t pjacobi_ref_list_bytes(int d);
template <typename TI>
hipError_t launch_pjacobi_ref(const TI* Win, int64_t sp, int64_t sq, int tri, int d, int LP, double* W, double* Jl,
                              double* Jr, double* S, void* list, int* info, hipStream_t s);
// Iterations per singular value of the reference power method (src/PM.cpp:25-28).
int power_iterations(int64_t n);
// SVD<Power> on A (m x LP fp64 panel, n used columns) with B = A^T A (LP x LP, overwritten):
// u_i -> column i of Up (m x LP panel), v_i -> row i of Vr (LP x LP), S[i]; *kept = triplets
// found (< dim when sigma < 1e-12 stops it).  One workgroup.  n <= LP <= 512.
// x0 (nullable): start vectors as rows of an LP x LP matrix instead of Philox(seed + i).
// rsvd_mode: v_i goes to COLUMN i of Vr, and triplets past an early stop are written as zeros;
// rsvd_mode 2: image_compression's deflation (B recomputed as A_i^T A_i, no sigma < 1e-12 stop).
hipError_t launch_power_svd(const double* P, int64_t m, int n, int LP, double* B, int dim, uint64_t seed, int iters,
                            double* Up, double* Vr, double* S, int* kept, hipStream_t s, const double* x0 = nullptr,
                            int rsvd_mode = 0);
// rSVD(..., SVDMethod::Power) in Q_B coordinates (dense.hip power_prep_kernel): from R = Q_B^T B^T
// and Y0 = Q_B^T X0 build P = R^T, the start-vector rows X0s and Bpm = R R^T (all LP x LP fp64).
hipError_t launch_power_prep(const double* R, const double* Y0, int l, int LP, double* P, double* X0s, double* Bpm,
                             hipStream_t s);
// X0 (rows x LP): column i = Philox stream (seed + i), the reference's random start vectors.
template <typename T>
hipError_t launch_power_start(T* X0, int64_t rows, int l, int LP, uint64_t seed, hipStream_t s);
// The Philox key of the power method's start vectors inside rSVD (documented in rsvd_c.h).
uint64_t power_seed(uint64_t seed);

// ---- gemm.hip: column-major building blocks of the drop-ins past 512 columns (dense_big.cpp) ----
// C = alpha op(A) op(B) + beta C, op = transpose when ta / tb; column-major, any sizes (MFMA).
template <typename T>
hipError_t launch_gemm(int ta, int tb, int64_t M, int64_t N, int64_t K, T alpha, const T* A, int64_t lda, const T* B,
                       int64_t ldb, T beta, T* C, int64_t ldc, hipStream_t s);
// The Givens sign rule on a column-major Q (flip the leading run of untouched columns where A(j,j) < 0).
template <typename T>
hipError_t launch_qr_signs_cm(const T* A, int64_t lda, int64_t m, int64_t n, T* Q, int64_t ldq, hipStream_t s);
// det(Q) > 0 for a square column-major Q (m x m): LU with partial pivoting (one launch per step,
// W: 2 m^2 doubles, sgn: one int of workspace); flips column m - 1 when the determinant is negative.
template <typename T>
hipError_t launch_det_sign_cm(T* Q, int64_t ldq, int m, double* W, int* sgn, hipStream_t s);
// Y[:, j] = e_{e0 + j} (rows x cols, column-major)
template <typename T>
hipError_t launch_identity_cols(T* Y, int64_t ldy, int64_t rows, int cols, int64_t e0, hipStream_t s);
// zero the strictly lower part of a column-major rows x cols matrix
template <typename T>
hipError_t launch_zero_below(T* R, int64_t ldr, int64_t rows, int64_t cols, hipStream_t s);
// D (m x n fp32, ld m) = bf16 (fp8 = 0) or OCP e4m3 (fp8 = 1) A (column-major, ld lda), exactly
hipError_t launch_lowp_to_f32(const void* A, int64_t lda, int64_t m, int64_t n, int fp8, float* D, hipStream_t s);
// D (rows x cols fp32, column-major, ld) = a bf16 row-major panel (rows x LP)
hipError_t launch_bf16_panel_to_f32(const uint16_t* P, int64_t rows, int cols, int LP, float* D, int64_t ld,
                                    hipStream_t s);
// D (m x n fp64, ld m) = A (column-major, ld lda)
template <typename T>
hipError_t launch_widen(const T* A, int64_t lda, int64_t m, int64_t n, double* D, hipStream_t s);

}  // namespace rsvd
