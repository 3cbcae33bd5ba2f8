/*
 * rsvd_oracle.h -- CPU restatement of the reference randomized-SVD hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This is the parity oracle for the MI355X engine in
 * rsvd_kamaneh_raganato_terrana_amd/; only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load it.  The product path never calls it.
 *
 * Restates, in plain C99 + OpenMP, fp64, column-major storage (Eigen's default):
 *   - generateOmega            src/rSVD.cpp:12-55   (Gaussian N(0,1) n x l; here drawn from a
 *                                                    counter-based Philox4x32-10 stream so the
 *                                                    GPU and the oracle can see the same Omega)
 *   - intermediate_step        src/rSVD.cpp:57-70
 *   - rSVD                     src/rSVD.cpp:72-133
 *   - Eigen::HouseholderQR +   src/rSVD.cpp:60-61 (Eigen makeHouseholder convention:
 *     householderQ()*Identity    beta = -sign(x0)*||x||, tau = (beta-x0)/beta; == LAPACK dlarfg)
 *   - SVD<Jacobi>::jacobiSVD   include/SVD_class.hpp:100-180
 *   - SVD<ParallelJacobi>      include/SVD_class.hpp:223-333
 *   - SVD<Power> + PM          include/SVD_class.hpp:183-219, src/PM.cpp:4-81
 *   - JacobiOperations         src/JacobiOperations.cpp:6-103, 120-203
 *   - Givens QR                src/QR.cpp:12-80
 *
 * Parity pinning: see tests/test_oracle.py (known answers of the reference's committed inputs
 * input/ *.mtx and image_compression/data/input/mat/ *.mtx, plus LAPACK SVD/QR golden vectors
 * produced by the same numpy calls as python/test_run_rSVD.py:41-57 and test_run_QR.py:25-40).
 * The reference C++ itself cannot be compiled here (Eigen is absent), so oracle/_ref is not built.
 */
#ifndef RSVD_ORACLE_H
#define RSVD_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { ORC_SVD_JACOBI = 0, ORC_SVD_POWER = 1, ORC_SVD_PARALLEL_JACOBI = 2 };

/* Threads used by the OpenMP regions (0 = OpenMP default). Returns the count in effect. */
int orc_set_threads(int nthreads);

/* Philox4x32-10 Gaussian stream (CPU twin of the device generator).
 * out[e] for e in [0,count): element e of the stream for `seed`, e = i + n*j for an n x l
 * column-major Omega.  Box-Muller on two 53-bit uniforms per Philox block. */
void orc_philox_gaussian(uint64_t seed, int64_t first, int64_t count, double *out);

/* C = op(A) * op(B) (+ beta*C), column-major, op = 'N' or 'T'. */
void orc_gemm(char ta, char tb, int64_t m, int64_t n, int64_t k, const double *A, int64_t lda,
              const double *B, int64_t ldb, double beta, double *C, int64_t ldc);

/* In-place Householder QR (Eigen/LAPACK convention): R in the upper triangle, essential parts
 * of the reflectors below the diagonal, tau[min(m,n)]. */
void orc_householder_qr(int64_t m, int64_t n, double *A, int64_t lda, double *tau);
/* Q(:,0:cols) = H_0 ... H_{r-1} * I(m, cols), r = min(m, n). */
void orc_householder_q(int64_t m, int64_t n, const double *QR, int64_t ldqr, const double *tau,
                       int64_t cols, double *Q, int64_t ldq);
/* Thin Q of Y (m x l): Eigen::HouseholderQR<Mat_m> qr(Y); Q = qr.householderQ()*Identity(m,l). */
void orc_thin_q(int64_t m, int64_t l, const double *Y, int64_t ldy, double *Q, int64_t ldq);

/* Givens QR of src/QR.cpp. reduced: Q m x n, R n x n (requires m >= n); full: Q m x m, R m x n.
 * Returns 0 on success, -1 on a shape error. */
int orc_givens_qr_reduced(int64_t m, int64_t n, const double *A, int64_t lda, double *Q, double *R);
int orc_givens_qr_full(int64_t m, int64_t n, const double *A, int64_t lda, double *Q, double *R);

/* SVD<Jacobi> / SVD<ParallelJacobi> of data (m x n).  d = min(m, n).
 * Outputs: U (m x d), S (d), V (n x d), column-major with ld = rows.
 * Returns the number of sweeps. */
int orc_jacobi_svd(int64_t m, int64_t n, const double *data, int64_t ld, int parallel_variant,
                   double *U, double *S, double *V);

/* SVD<Power> of data (m x n) with r (0 => min(m,n)) deflation steps; the PM start vectors are
 * drawn from orc_philox_gaussian(seed + i) instead of std::random_device (src/PM.cpp:15-22).
 * Reference layouts (include/SVD_class.hpp:82-84,213-214): U m x m, S min(m,n), V n x n with
 * v_i^T stored in ROW i.  Returns k = number of singular triplets kept (early exit when
 * sigma < 1e-12, include/SVD_class.hpp:198-208); k == 0 encodes the i == 0 zero case. */
int64_t orc_power_svd(int64_t m, int64_t n, const double *data, int64_t ld, int64_t r,
                      uint64_t seed, double *U, double *S, double *V);

/* intermediate_step: Q (m x l) from A (m x n) and Omega (n x l), q power iterations. */
void orc_intermediate_step(int64_t m, int64_t n, const double *A, int64_t lda,
                           const double *Omega, int64_t ldo, int64_t l, int64_t q,
                           double *Q, int64_t ldq);

/* rSVD with Jacobi / ParallelJacobi small SVD.  d = min(l, n).
 * U (m x d), S (d), V (n x d), ld = rows.  Returns 0, or -1 for an unsupported method. */
int orc_rsvd(int64_t m, int64_t n, const double *A, int64_t lda, int64_t l, int64_t q,
             const double *Omega, int64_t ldo, int method, double *U, double *S, double *V);
/* rSVD with SVDMethod::Power (src/rSVD.cpp:106-113); start vectors Philox(pm_seed + i).
 * U m x l, S l, V n x n (v_i in rows); returns the triplets kept. */
int64_t orc_rsvd_power(int64_t m, int64_t n, const double *A, int64_t lda, int64_t l, int64_t q,
                       const double *Omega, int64_t ldo, uint64_t pm_seed, double *U, double *S, double *V);

#ifdef __cplusplus
}
#endif
/* image_compression's power-method SVD (image_compression/src/SVD.cpp:30-55, PowerMethod.cpp:3-43):
 * B recomputed as A^T A after every deflation, no sigma < 1e-12 stop; V (n x dim) in columns; start
 * vectors orc_philox_gaussian(seed + i).  Returns the triplets written (dim unless a sigma is 0). */
int64_t orc_ic_power_svd(int64_t m, int64_t n, const double *data, int64_t ld, int64_t dim, uint64_t seed,
                         double *U, double *S, double *V);
/* image_compression's 5-argument rSVD (image_compression/src/rSVD.cpp:77-118): q = 1, the power-method
 * SVD above on B = Q^T A with dim = min(l, n).  U m x d, S d, V n x d (d = min(l, n)). */
int64_t orc_ic_rsvd(int64_t m, int64_t n, const double *A, int64_t lda, int64_t l, const double *Omega, int64_t ldo,
                    uint64_t pm_seed, double *U, double *S, double *V);

#endif
