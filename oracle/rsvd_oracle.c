/*
 * rsvd_oracle.c -- CPU restatement of the reference rSVD hot path.  TEST INFRASTRUCTURE ONLY
 * (see rsvd_oracle.h for the contract and the list of reference functions restated).
 *
 * Storage is column-major fp64 everywhere, as Eigen::MatrixXd in the reference.
 */
#include "rsvd_oracle.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define IDX(i, j, ld) ((i) + (int64_t)(j) * (ld))

int orc_set_threads(int nthreads) {
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
    return omp_get_max_threads();
#else
    (void)nthreads;
    return 1;
#endif
}

/* ------------------------------------------------------------------------------------------ */
/* Philox4x32-10 (Salmon et al., SC'11).  The device twin lives in csrc/util.hip.                */
/* ------------------------------------------------------------------------------------------ */
static inline void philox_round(uint32_t c[4], const uint32_t k[2]) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
    const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    const uint32_t n0 = hi1 ^ c[1] ^ k[0];
    const uint32_t n2 = hi0 ^ c[3] ^ k[1];
    c[0] = n0; c[1] = lo1; c[2] = n2; c[3] = lo0;
}

static inline void philox4x32_10(uint64_t ctr, uint64_t seed, uint32_t out[4]) {
    uint32_t c[4] = {(uint32_t)ctr, (uint32_t)(ctr >> 32), 0x52535644u /* "RSVD" */, 0u};
    uint32_t k[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
    for (int r = 0; r < 10; ++r) {
        philox_round(c, k);
        k[0] += 0x9E3779B9u;
        k[1] += 0xBB67AE85u;
    }
    out[0] = c[0]; out[1] = c[1]; out[2] = c[2]; out[3] = c[3];
}

/* One Philox block -> two N(0,1) doubles (Box-Muller on 53-bit uniforms in (0,1)). */
static inline void gauss_pair(uint64_t pair, uint64_t seed, double *z0, double *z1) {
    uint32_t x[4];
    philox4x32_10(pair, seed, x);
    const double two_m53 = 1.1102230246251565404e-16; /* 2^-53 */
    const double u1 = ((double)(((uint64_t)(x[0] >> 5) << 26) | (x[1] >> 6)) + 0.5) * two_m53;
    const double u2 = ((double)(((uint64_t)(x[2] >> 5) << 26) | (x[3] >> 6)) + 0.5) * two_m53;
    const double r = sqrt(-2.0 * log(u1));
    const double th = 6.283185307179586476925286766559 * u2;
    *z0 = r * cos(th);
    *z1 = r * sin(th);
}

void orc_philox_gaussian(uint64_t seed, int64_t first, int64_t count, double *out) {
#pragma omp parallel for schedule(static)
    for (int64_t t = 0; t < count; ++t) {
        const int64_t e = first + t;
        double z0, z1;
        gauss_pair((uint64_t)(e >> 1), seed, &z0, &z1);
        out[t] = (e & 1) ? z1 : z0;
    }
}

/* ------------------------------------------------------------------------------------------ */
/* GEMM (stands in for Eigen's products at src/rSVD.cpp:59,63,66,89,128).                      */
/* ------------------------------------------------------------------------------------------ */
void orc_gemm(char ta, char tb, int64_t m, int64_t n, int64_t k, const double *A, int64_t lda,
              const double *B, int64_t ldb, double beta, double *C, int64_t ldc) {
    const int tA = (ta == 'T' || ta == 't');
    const int tB = (tb == 'T' || tb == 't');
    if (!tA) {
        /* C(:,j) = beta*C(:,j) + sum_p A(:,p) * op(B)(p,j): axpy form, rows split over threads. */
        const int64_t RB = 512;
        const int64_t nrb = (m + RB - 1) / RB;
#pragma omp parallel for collapse(2) schedule(static)
        for (int64_t rb = 0; rb < nrb; ++rb) {
            for (int64_t j = 0; j < n; ++j) {
                const int64_t i0 = rb * RB, i1 = (i0 + RB < m) ? i0 + RB : m;
                double acc[512];
                for (int64_t i = i0; i < i1; ++i) acc[i - i0] = (beta == 0.0) ? 0.0 : beta * C[IDX(i, j, ldc)];
                for (int64_t p = 0; p < k; ++p) {
                    const double b = tB ? B[IDX(j, p, ldb)] : B[IDX(p, j, ldb)];
                    const double *a = A + (int64_t)p * lda;
                    for (int64_t i = i0; i < i1; ++i) acc[i - i0] += a[i] * b;
                }
                for (int64_t i = i0; i < i1; ++i) C[IDX(i, j, ldc)] = acc[i - i0];
            }
        }
    } else {
        /* C(i,j) = beta*C(i,j) + dot(A(:,i), op(B)(:,j)). */
#pragma omp parallel for collapse(2) schedule(static)
        for (int64_t j = 0; j < n; ++j) {
            for (int64_t i = 0; i < m; ++i) {
                const double *a = A + (int64_t)i * lda;
                double s = 0.0;
                if (!tB) {
                    const double *b = B + (int64_t)j * ldb;
                    for (int64_t p = 0; p < k; ++p) s += a[p] * b[p];
                } else {
                    for (int64_t p = 0; p < k; ++p) s += a[p] * B[IDX(j, p, ldb)];
                }
                C[IDX(i, j, ldc)] = (beta == 0.0) ? s : beta * C[IDX(i, j, ldc)] + s;
            }
        }
    }
}

/* ------------------------------------------------------------------------------------------ */
/* Householder QR, Eigen convention (makeHouseholder: tol = numeric_limits<double>::min()).     */
/* ------------------------------------------------------------------------------------------ */
void orc_householder_qr(int64_t m, int64_t n, double *A, int64_t lda, double *tau) {
    const int64_t r = m < n ? m : n;
    for (int64_t k = 0; k < r; ++k) {
        double *x = A + IDX(k, k, lda);
        const double c0 = x[0];
        double tail = 0.0;
        for (int64_t i = 1; i < m - k; ++i) tail += x[i] * x[i];
        double beta, t;
        if (tail <= DBL_MIN) {
            t = 0.0;
            beta = c0;
            for (int64_t i = 1; i < m - k; ++i) x[i] = 0.0;
        } else {
            beta = sqrt(c0 * c0 + tail);
            if (c0 >= 0.0) beta = -beta;
            const double inv = 1.0 / (c0 - beta);
            for (int64_t i = 1; i < m - k; ++i) x[i] *= inv;
            t = (beta - c0) / beta;
        }
        x[0] = beta;
        tau[k] = t;
        if (t == 0.0) continue;
        /* Apply H = I - t v v^T, v = [1; x(1:)], to A(k:m, k+1:n). */
#pragma omp parallel for schedule(static) if ((m - k) * (n - k) > 65536)
        for (int64_t j = k + 1; j < n; ++j) {
            double *a = A + IDX(k, j, lda);
            double w = a[0];
            for (int64_t i = 1; i < m - k; ++i) w += x[i] * a[i];
            w *= t;
            a[0] -= w;
            for (int64_t i = 1; i < m - k; ++i) a[i] -= w * x[i];
        }
    }
}

void orc_householder_q(int64_t m, int64_t n, const double *QR, int64_t ldqr, const double *tau,
                       int64_t cols, double *Q, int64_t ldq) {
    const int64_t r = m < n ? m : n;
    for (int64_t j = 0; j < cols; ++j)
        for (int64_t i = 0; i < m; ++i) Q[IDX(i, j, ldq)] = (i == j) ? 1.0 : 0.0;
    for (int64_t k = r - 1; k >= 0; --k) {
        const double t = tau[k];
        if (t == 0.0) continue;
        const double *v = QR + IDX(k, k, ldqr);
#pragma omp parallel for schedule(static) if ((m - k) * cols > 65536)
        for (int64_t j = 0; j < cols; ++j) {
            double *q = Q + IDX(k, j, ldq);
            double w = q[0];
            for (int64_t i = 1; i < m - k; ++i) w += v[i] * q[i];
            w *= t;
            q[0] -= w;
            for (int64_t i = 1; i < m - k; ++i) q[i] -= w * v[i];
        }
    }
}

void orc_thin_q(int64_t m, int64_t l, const double *Y, int64_t ldy, double *Q, int64_t ldq) {
    double *work = (double *)malloc(sizeof(double) * (size_t)m * (size_t)l);
    const int64_t r = m < l ? m : l;
    double *tau = (double *)malloc(sizeof(double) * (size_t)(r > 0 ? r : 1));
    for (int64_t j = 0; j < l; ++j) memcpy(work + IDX(0, j, m), Y + IDX(0, j, ldy), sizeof(double) * (size_t)m);
    orc_householder_qr(m, l, work, m, tau);
    orc_householder_q(m, l, work, m, tau, l, Q, ldq);
    free(tau);
    free(work);
}

/* ------------------------------------------------------------------------------------------ */
/* Givens QR, src/QR.cpp:12-80.                                                                */
/* ------------------------------------------------------------------------------------------ */
static void givens_qr(int64_t m, int64_t n, double *Qf /* m x m */, double *R /* m x n, ld m */) {
    for (int64_t j = 0; j < m * m; ++j) Qf[j] = 0.0;
    for (int64_t i = 0; i < m; ++i) Qf[IDX(i, i, m)] = 1.0;
    const int64_t r = m < n ? m : n;
    for (int64_t j = 0; j < r; ++j) {
        for (int64_t i = m - 1; i > j; --i) {
            if (R[IDX(i, j, m)] != 0.0) {
                /* givens_rotation: r = hypot(a,b), c = a/r, s = -b/r, G = [[c,-s],[s,c]] */
                const double a = R[IDX(i - 1, j, m)], b = R[IDX(i, j, m)];
                const double rr = hypot(a, b);
                const double c = a / rr, s = -b / rr;
                for (int64_t jj = j; jj < n; ++jj) { /* R(i-1:i, j:) = G * R(i-1:i, j:) */
                    const double x = R[IDX(i - 1, jj, m)], y = R[IDX(i, jj, m)];
                    R[IDX(i - 1, jj, m)] = c * x - s * y;
                    R[IDX(i, jj, m)] = s * x + c * y;
                }
                for (int64_t ii = 0; ii < m; ++ii) { /* Q(:, i-1:i) = Q(:, i-1:i) * G^T */
                    const double x = Qf[IDX(ii, i - 1, m)], y = Qf[IDX(ii, i, m)];
                    Qf[IDX(ii, i - 1, m)] = x * c - y * s;
                    Qf[IDX(ii, i, m)] = x * s + y * c;
                }
            }
        }
    }
}

int orc_givens_qr_reduced(int64_t m, int64_t n, const double *A, int64_t lda, double *Q, double *R) {
    if (m < n) return -1; /* Q_temp.leftCols(n) needs n <= m (src/QR.cpp:78) */
    double *Qf = (double *)malloc(sizeof(double) * (size_t)(m * m));
    double *Rf = (double *)malloc(sizeof(double) * (size_t)(m * n));
    for (int64_t j = 0; j < n; ++j) memcpy(Rf + IDX(0, j, m), A + IDX(0, j, lda), sizeof(double) * (size_t)m);
    givens_qr(m, n, Qf, Rf);
    for (int64_t j = 0; j < n; ++j) memcpy(Q + IDX(0, j, m), Qf + IDX(0, j, m), sizeof(double) * (size_t)m);
    for (int64_t j = 0; j < n; ++j)
        for (int64_t i = 0; i < n; ++i) R[IDX(i, j, n)] = Rf[IDX(i, j, m)];
    free(Qf);
    free(Rf);
    return 0;
}

int orc_givens_qr_full(int64_t m, int64_t n, const double *A, int64_t lda, double *Q, double *R) {
    for (int64_t j = 0; j < n; ++j) memcpy(R + IDX(0, j, m), A + IDX(0, j, lda), sizeof(double) * (size_t)m);
    givens_qr(m, n, Q, R);
    return 0;
}

/* ------------------------------------------------------------------------------------------ */
/* Jacobi SVD, include/SVD_class.hpp:100-180 / 223-333 and src/JacobiOperations.cpp.          */
/* ------------------------------------------------------------------------------------------ */
typedef struct { double *p; int64_t rows, cols; } mat_t; /* column-major, ld = rows */
#define M_(M, i, j) ((M).p[IDX(i, j, (M).rows)])

static void apply_left(mat_t M, int64_t p, int64_t q, double c, double s) { /* :6-14 */
    for (int64_t i = 0; i < M.cols; ++i) {
        const double xi = M_(M, p, i), yi = M_(M, q, i);
        M_(M, p, i) = c * xi + s * yi;
        M_(M, q, i) = -s * xi + c * yi;
    }
}

static void apply_right(mat_t M, int64_t p, int64_t q, double c, double s) { /* :16-24 */
    for (int64_t i = 0; i < M.rows; ++i) {
        const double xi = M_(M, i, p), yi = M_(M, i, q);
        M_(M, i, p) = c * xi + (-s) * yi;
        M_(M, i, q) = s * xi + c * yi;
    }
}

/* real_2x2_jacobi_svd (:25-88); deno_min = DBL_MIN (serial) or 1e-10 (the _par variant :168). */
static void real_2x2_jacobi_svd(mat_t W, int64_t p, int64_t q, double deno_min, double *cl,
                                double *sl, double *cr, double *sr) {
    double m00 = M_(W, p, p), m01 = M_(W, p, q), m10 = M_(W, q, p), m11 = M_(W, q, q);
    const double t = m00 + m11;
    const double d = m10 - m01;
    double c1 = 1.0, s1 = 0.0;
    if (d != 0.0) {
        const double u = t / d;
        const double tmp = sqrt(1.0 + u * u);
        s1 = 1.0 / tmp;
        c1 = u / tmp;
    }
    { /* applyOnTheLeft(m, 0, 1, c1, s1) on the 2x2 block */
        const double x0 = m00, y0 = m10, x1 = m01, y1 = m11;
        m00 = c1 * x0 + s1 * y0;
        m10 = -s1 * x0 + c1 * y0;
        m01 = c1 * x1 + s1 * y1;
        m11 = -s1 * x1 + c1 * y1;
    }
    const double deno = 2.0 * fabs(m01);
    if (deno < deno_min) {
        *cr = 1.0;
        *sr = 0.0;
    } else {
        const double tau = (m00 - m11) / deno;
        const double w = sqrt(tau * tau + 1.0);
        const double t2 = (tau > 0.0) ? 1.0 / (tau + w) : 1.0 / (tau - w);
        const double segno = t2 > 0.0 ? 1.0 : -1.0;
        const double nn = 1.0 / sqrt(t2 * t2 + 1.0);
        *sr = -segno * (m01 / fabs(m01)) * fabs(t2) * nn;
        *cr = nn;
    }
    /* left = rot_to_eigen * j_right^T, rot_to_eigen = [[c1,s1],[-s1,c1]], j_right = [[cr,sr],[-sr,cr]] */
    *cl = c1 * (*cr) + s1 * (*sr);
    *sl = c1 * (-(*sr)) + s1 * (*cr);
}

static int precondition_2x2(mat_t W, int64_t p, int64_t q, double maxDiag) { /* :89-103 */
    return !(fabs(M_(W, p, q)) < maxDiag * DBL_EPSILON && fabs(M_(W, q, p)) < maxDiag * DBL_EPSILON);
}

typedef struct { double w; int64_t p, q; } wpq_t;
static int cmp_wpq_desc(const void *a, const void *b) { /* std::sort(..., std::greater<>()) on tuple */
    const wpq_t *x = (const wpq_t *)a, *y = (const wpq_t *)b;
    if (x->w != y->w) return x->w > y->w ? -1 : 1;
    if (x->p != y->p) return x->p > y->p ? -1 : 1;
    if (x->q != y->q) return x->q > y->q ? -1 : 1;
    return 0;
}

int orc_jacobi_svd(int64_t m, int64_t n, const double *data, int64_t ld, int parallel_variant,
                   double *Uout, double *Sout, double *Vout) {
    const int64_t d = m < n ? m : n;
    /* working matrix (d x d after preconditioning, or m x n when square) */
    mat_t W = {NULL, 0, 0}, U = {NULL, m, d}, V = {NULL, n, d};
    U.p = (double *)calloc((size_t)(m * d), sizeof(double));
    V.p = (double *)calloc((size_t)(n * d), sizeof(double));
    for (int64_t i = 0; i < d; ++i) { M_(U, i, i) = 1.0; M_(V, i, i) = 1.0; }
    if (m > n) { /* :110-115: QR of data, W = R (n x n upper), U = Q_thin, V = I */
        double *work = (double *)malloc(sizeof(double) * (size_t)(m * n));
        double *tau = (double *)malloc(sizeof(double) * (size_t)n);
        for (int64_t j = 0; j < n; ++j) memcpy(work + IDX(0, j, m), data + IDX(0, j, ld), sizeof(double) * (size_t)m);
        orc_householder_qr(m, n, work, m, tau);
        W.rows = W.cols = n;
        W.p = (double *)calloc((size_t)(n * n), sizeof(double));
        for (int64_t j = 0; j < n; ++j)
            for (int64_t i = 0; i <= j; ++i) M_(W, i, j) = work[IDX(i, j, m)];
        orc_householder_q(m, n, work, m, tau, n, U.p, m);
        free(tau);
        free(work);
    } else if (n > m) { /* :116-123: QR of data^T, W = R^T (m x m lower), V = Q_thin (n x m) */
        double *work = (double *)malloc(sizeof(double) * (size_t)(m * n));
        double *tau = (double *)malloc(sizeof(double) * (size_t)m);
        for (int64_t j = 0; j < m; ++j)
            for (int64_t i = 0; i < n; ++i) work[IDX(i, j, n)] = data[IDX(j, i, ld)];
        orc_householder_qr(n, m, work, n, tau);
        W.rows = W.cols = m;
        W.p = (double *)calloc((size_t)(m * m), sizeof(double));
        for (int64_t j = 0; j < m; ++j)
            for (int64_t i = 0; i <= j; ++i) M_(W, j, i) = work[IDX(i, j, n)];
        orc_householder_q(n, m, work, n, tau, m, V.p, n);
        free(tau);
        free(work);
    } else {
        W.rows = W.cols = m;
        W.p = (double *)malloc(sizeof(double) * (size_t)(m * m));
        for (int64_t j = 0; j < m; ++j) memcpy(W.p + IDX(0, j, m), data + IDX(0, j, ld), sizeof(double) * (size_t)m);
    }

    const double considerAsZero = parallel_variant ? 1e-12 : DBL_MIN;
    const double precision = parallel_variant ? 1e-12 : 2.0 * DBL_EPSILON;
    const double deno_min = parallel_variant ? 1e-10 : DBL_MIN;
    double maxDiag = 0.0;
    for (int64_t i = 0; i < d; ++i) maxDiag = fmax(maxDiag, fabs(M_(W, i, i)));
    double cl, sl, cr, sr;
    int sweeps = 0;
    int finished = 0;
    wpq_t *list = parallel_variant ? (wpq_t *)malloc(sizeof(wpq_t) * (size_t)(d * (d > 1 ? d - 1 : 1) / 2 + 1)) : NULL;
    while (!finished) {
        finished = 1;
        ++sweeps;
        if (!parallel_variant) { /* :132-155, cyclic by rows */
            for (int64_t p = 1; p < d; ++p) {
                for (int64_t q = 0; q < p; ++q) {
                    const double threshold = fmax(considerAsZero, precision * maxDiag);
                    if (fabs(M_(W, p, q)) > threshold || fabs(M_(W, q, p)) > threshold) {
                        finished = 0;
                        if (precondition_2x2(W, p, q, maxDiag)) {
                            real_2x2_jacobi_svd(W, p, q, deno_min, &cl, &sl, &cr, &sr);
                            apply_left(W, p, q, cl, sl);
                            apply_right(U, p, q, cl, -sl);
                            apply_right(W, p, q, cr, sr);
                            apply_right(V, p, q, cr, sr);
                            maxDiag = fmax(maxDiag, fmax(fabs(M_(W, p, p)), fabs(M_(W, q, q))));
                        }
                    }
                }
            }
        } else { /* :261-305, weight-sorted order */
            int64_t cnt = 0;
            const double threshold = fmax(considerAsZero, precision * maxDiag);
            for (int64_t p = 1; p < d; ++p)
                for (int64_t q = 0; q < p; ++q) {
                    const double w = M_(W, p, q) * M_(W, p, q) + M_(W, q, p) * M_(W, q, p);
                    if (w > threshold) { finished = 0; list[cnt].w = w; list[cnt].p = p; list[cnt].q = q; ++cnt; }
                }
            qsort(list, (size_t)cnt, sizeof(wpq_t), cmp_wpq_desc);
            for (int64_t e = 0; e < cnt; ++e) {
                const int64_t p = list[e].p, q = list[e].q;
                if (precondition_2x2(W, p, q, maxDiag)) {
                    real_2x2_jacobi_svd(W, p, q, deno_min, &cl, &sl, &cr, &sr);
                    apply_left(W, p, q, cl, sl);
                    apply_right(U, p, q, cl, -sl);
                    apply_right(W, p, q, cr, sr);
                    apply_right(V, p, q, cr, sr);
                    maxDiag = fmax(maxDiag, fmax(fabs(M_(W, p, p)), fabs(M_(W, q, q))));
                }
            }
        }
        if (sweeps > 10000) break; /* the reference loops forever here; the oracle refuses to */
    }
    free(list);
    /* :158-162 sign fix, :164-178 selection sort */
    for (int64_t i = 0; i < d; ++i) {
        const double a = M_(W, i, i);
        Sout[i] = fabs(a);
        if (a < 0) for (int64_t r = 0; r < m; ++r) M_(U, r, i) = -M_(U, r, i);
    }
    for (int64_t i = 0; i < d; ++i) {
        int64_t pos = 0;
        double mx = Sout[i];
        for (int64_t t = 1; t < d - i; ++t)
            if (Sout[i + t] > mx) { mx = Sout[i + t]; pos = t; }
        if (mx == 0.0) break;
        if (pos) {
            pos += i;
            const double ts = Sout[i]; Sout[i] = Sout[pos]; Sout[pos] = ts;
            for (int64_t r = 0; r < m; ++r) { const double x = M_(U, r, pos); M_(U, r, pos) = M_(U, r, i); M_(U, r, i) = x; }
            for (int64_t r = 0; r < n; ++r) { const double x = M_(V, r, pos); M_(V, r, pos) = M_(V, r, i); M_(V, r, i) = x; }
        }
    }
    memcpy(Uout, U.p, sizeof(double) * (size_t)(m * d));
    memcpy(Vout, V.p, sizeof(double) * (size_t)(n * d));
    free(U.p);
    free(V.p);
    free(W.p);
    return sweeps;
}

/* ------------------------------------------------------------------------------------------ */
/* SVD<Power>, include/SVD_class.hpp:183-219, with PM from src/PM.cpp:4-81.                   */
/* ------------------------------------------------------------------------------------------ */
static void nrm(double *x, int64_t n) {
    double s = 0.0;
    for (int64_t i = 0; i < n; ++i) s += x[i] * x[i];
    s = sqrt(s);
    for (int64_t i = 0; i < n; ++i) x[i] /= s;
}

int64_t orc_power_svd(int64_t m, int64_t n, const double *data_in, int64_t ld, int64_t r,
                      uint64_t seed, double *U, double *S, double *V) {
    const int64_t mn = m < n ? m : n;
    const int64_t dim = (r == 0) ? mn : r;
    double *data = (double *)malloc(sizeof(double) * (size_t)(m * n));
    for (int64_t j = 0; j < n; ++j) memcpy(data + IDX(0, j, m), data_in + IDX(0, j, ld), sizeof(double) * (size_t)m);
    /* compute(): U_ = I(m,m), V_ = I(n,n), S_ = 0 (:82-84) */
    for (int64_t i = 0; i < m * m; ++i) U[i] = 0.0;
    for (int64_t i = 0; i < m; ++i) U[IDX(i, i, m)] = 1.0;
    for (int64_t i = 0; i < n * n; ++i) V[i] = 0.0;
    for (int64_t i = 0; i < n; ++i) V[IDX(i, i, n)] = 1.0;
    for (int64_t i = 0; i < mn; ++i) S[i] = 0.0;
    double *B = (double *)malloc(sizeof(double) * (size_t)(n * n));
    orc_gemm('T', 'N', n, n, m, data, m, data, m, 0.0, B, n); /* B = data^T data (:193) */
    double *x0 = (double *)malloc(sizeof(double) * (size_t)n);
    double *res = (double *)malloc(sizeof(double) * (size_t)n);
    double *u = (double *)malloc(sizeof(double) * (size_t)m);
    /* s = ceil(log(4 log(2n/delta) / (eps delta)) / (2 lambda)), src/PM.cpp:25-28 */
    const double eps = 1.e-10, delta = 0.05, lambda = 0.1;
    const int s = (int)ceil(log(4.0 * log(2.0 * (double)n / delta) / (eps * delta)) / (2.0 * lambda));
    int64_t kept = dim;
    for (int64_t i = 0; i < dim; ++i) {
        orc_philox_gaussian(seed + (uint64_t)i, 0, n, x0);
        nrm(x0, n);
        for (int it = 1; it <= s; ++it) {
            orc_gemm('N', 'N', n, 1, n, B, n, x0, n, 0.0, res, n);
            memcpy(x0, res, sizeof(double) * (size_t)n);
            nrm(x0, n);
        }
        nrm(x0, n); /* v = x0.normalized() */
        orc_gemm('N', 'N', m, 1, n, data, m, x0, n, 0.0, u, m);
        double sigma = 0.0;
        for (int64_t t = 0; t < m; ++t) sigma += u[t] * u[t];
        sigma = sqrt(sigma);
        for (int64_t t = 0; t < m; ++t) u[t] /= sigma;
        if (sigma < 1e-12) { kept = i; break; }
        /* deflation (:210-212): data -= sigma u v^T; B -= (sigma u v^T)^T (sigma u v^T) */
        for (int64_t c = 0; c < n; ++c)
            for (int64_t t = 0; t < m; ++t) data[IDX(t, c, m)] -= sigma * u[t] * x0[c];
        double uu = 0.0;
        for (int64_t t = 0; t < m; ++t) uu += u[t] * u[t];
        for (int64_t c = 0; c < n; ++c)
            for (int64_t t = 0; t < n; ++t) B[IDX(t, c, n)] -= sigma * sigma * uu * x0[t] * x0[c];
        for (int64_t t = 0; t < m; ++t) U[IDX(t, i, m)] = u[t]; /* U_.col(i) = u */
        for (int64_t c = 0; c < n; ++c) V[IDX(i, c, n)] = x0[c]; /* V_.row(i) = v */
        S[i] = sigma;
    }
    free(u); free(res); free(x0); free(B); free(data);
    return kept;
}

/* ------------------------------------------------------------------------------------------ */
/* intermediate_step (src/rSVD.cpp:57-70) and rSVD (src/rSVD.cpp:72-133).                      */
/* ------------------------------------------------------------------------------------------ */
void orc_intermediate_step(int64_t m, int64_t n, const double *A, int64_t lda,
                           const double *Omega, int64_t ldo, int64_t l, int64_t q,
                           double *Q, int64_t ldq) {
    double *Ym = (double *)malloc(sizeof(double) * (size_t)(m * l));
    double *Yn = (double *)malloc(sizeof(double) * (size_t)(n * l));
    double *Qn = (double *)malloc(sizeof(double) * (size_t)(n * l));
    orc_gemm('N', 'N', m, l, n, A, lda, Omega, ldo, 0.0, Ym, m); /* Y = A * Omega (:59) */
    orc_thin_q(m, l, Ym, m, Q, ldq);                             /* (:60-61) */
    for (int64_t i = 0; i < q; ++i) {
        orc_gemm('T', 'N', n, l, m, A, lda, Q, ldq, 0.0, Yn, n);   /* Y = A^T Q (:63) */
        orc_thin_q(n, l, Yn, n, Qn, n);                            /* (:64-65) */
        orc_gemm('N', 'N', m, l, n, A, lda, Qn, n, 0.0, Ym, m);    /* Y = A Q (:66) */
        orc_thin_q(m, l, Ym, m, Q, ldq);                           /* (:67-68) */
    }
    free(Qn); free(Yn); free(Ym);
}

int orc_rsvd(int64_t m, int64_t n, const double *A, int64_t lda, int64_t l, int64_t q,
             const double *Omega, int64_t ldo, int method, double *U, double *S, double *V) {
    if (method != ORC_SVD_JACOBI && method != ORC_SVD_PARALLEL_JACOBI) return -1;
    double *Q = (double *)malloc(sizeof(double) * (size_t)(m * l));
    orc_intermediate_step(m, n, A, lda, Omega, ldo, l, q, Q, m);
    double *B = (double *)malloc(sizeof(double) * (size_t)(l * n));
    orc_gemm('T', 'N', l, n, m, Q, m, A, lda, 0.0, B, l); /* B = Q^T A (:89) */
    const int64_t d = l < n ? l : n;
    double *Ut = (double *)malloc(sizeof(double) * (size_t)(l * d));
    orc_jacobi_svd(l, n, B, l, method == ORC_SVD_PARALLEL_JACOBI, Ut, S, V);
    orc_gemm('N', 'N', m, d, l, Q, m, Ut, l, 0.0, U, m); /* U = Q * Utilde (:128) */
    free(Ut); free(B); free(Q);
    return 0;
}

/* rSVD with SVDMethod::Power (src/rSVD.cpp:106-113): SVD<Power> svd(B) on B = Q^T A (l x n), start
 * vectors Philox(pm_seed + i); Utilde = U_ (l x l), V = V_ (n x n, v_i in rows), U = Q Utilde.
 * U: m x l, S: l, V: n x n (all written in full, as before any conservativeResize); returns the
 * number of triplets kept (the caller cuts to it as SVD_class.hpp:198-208 does). */
int64_t orc_rsvd_power(int64_t m, int64_t n, const double *A, int64_t lda, int64_t l, int64_t q,
                       const double *Omega, int64_t ldo, uint64_t pm_seed, double *U, double *S, double *V) {
    double *Q = (double *)malloc(sizeof(double) * (size_t)(m * l));
    orc_intermediate_step(m, n, A, lda, Omega, ldo, l, q, Q, m);
    double *B = (double *)malloc(sizeof(double) * (size_t)(l * n));
    orc_gemm('T', 'N', l, n, m, Q, m, A, lda, 0.0, B, l); /* B = Q^T A (:89) */
    double *Ut = (double *)malloc(sizeof(double) * (size_t)(l * l));
    const int64_t kept = orc_power_svd(l, n, B, l, 0, pm_seed, Ut, S, V);
    orc_gemm('N', 'N', m, l, l, Q, m, Ut, l, 0.0, U, m); /* U = Q * Utilde (:128) */
    free(Ut); free(B); free(Q);
    return kept;
}

/* ------------------------------------------------------------------------------------------ */
/* image_compression's power-method SVD (image_compression/src/SVD.cpp:30-55 with powerMethod,   */
/* PowerMethod.cpp:3-43) and its 5-argument rSVD (image_compression/src/rSVD.cpp:77-118).        */
/* Differences from SVD<Power> above: after every triplet A -= sigma u v^T and B = A^T A is       */
/* RECOMPUTED (SVD.cpp:47-48), and there is no sigma < 1e-12 stop (a sigma of 0 makes the         */
/* reference divide by zero; the oracle stops there and reports the triplets written).           */
/* U: m x dim, S: dim, V: n x dim with v_i in column i (V = VT^T, SVD.cpp:54).                   */
/* ------------------------------------------------------------------------------------------ */
int64_t orc_ic_power_svd(int64_t m, int64_t n, const double *data_in, int64_t ld, int64_t dim, uint64_t seed,
                         double *U, double *S, double *V) {
    double *A = (double *)malloc(sizeof(double) * (size_t)(m * n));
    for (int64_t j = 0; j < n; ++j) memcpy(A + IDX(0, j, m), data_in + IDX(0, j, ld), sizeof(double) * (size_t)m);
    double *B = (double *)malloc(sizeof(double) * (size_t)(n * n));
    double *x0 = (double *)malloc(sizeof(double) * (size_t)n);
    double *res = (double *)malloc(sizeof(double) * (size_t)n);
    double *u = (double *)malloc(sizeof(double) * (size_t)m);
    orc_gemm('T', 'N', n, n, m, A, m, A, m, 0.0, B, n); /* B = A^T A (SVD.cpp:40) */
    const double eps = 1.e-10, delta = 0.05, lambda = 0.1; /* PowerMethod.cpp:24-27 */
    const int s = (int)ceil(log(4.0 * log(2.0 * (double)n / delta) / (eps * delta)) / (2.0 * lambda));
    for (int64_t i = 0; i < m * dim; ++i) U[i] = 0.0;
    for (int64_t i = 0; i < n * dim; ++i) V[i] = 0.0;
    for (int64_t i = 0; i < dim; ++i) S[i] = 0.0;
    int64_t kept = dim;
    for (int64_t i = 0; i < dim; ++i) {
        orc_philox_gaussian(seed + (uint64_t)i, 0, n, x0);
        nrm(x0, n);
        for (int it = 1; it <= s; ++it) { /* x0 = B x0; x0.normalize() (:29-32) */
            orc_gemm('N', 'N', n, 1, n, B, n, x0, n, 0.0, res, n);
            memcpy(x0, res, sizeof(double) * (size_t)n);
            nrm(x0, n);
        }
        nrm(x0, n); /* v = x0.normalized() (:35-36) */
        orc_gemm('N', 'N', m, 1, n, A, m, x0, n, 0.0, u, m);
        double sigma = 0.0;
        for (int64_t t = 0; t < m; ++t) sigma += u[t] * u[t];
        sigma = sqrt(sigma); /* sigma = (A v).norm() (:39) */
        if (!(sigma > 0.0)) { kept = i; break; }
        for (int64_t t = 0; t < m; ++t) u[t] /= sigma; /* u = A v / sigma (:42) */
        for (int64_t c = 0; c < n; ++c) /* A -= sigma u v^T (SVD.cpp:47) */
            for (int64_t t = 0; t < m; ++t) A[IDX(t, c, m)] -= sigma * u[t] * x0[c];
        orc_gemm('T', 'N', n, n, m, A, m, A, m, 0.0, B, n); /* B = A^T A (:48) */
        for (int64_t t = 0; t < m; ++t) U[IDX(t, i, m)] = u[t];
        for (int64_t c = 0; c < n; ++c) V[IDX(c, i, n)] = x0[c];
        S[i] = sigma;
    }
    free(u); free(res); free(x0); free(B); free(A);
    return kept;
}

int64_t orc_ic_rsvd(int64_t m, int64_t n, const double *A, int64_t lda, int64_t l, const double *Omega, int64_t ldo,
                    uint64_t pm_seed, double *U, double *S, double *V) {
    double *Q = (double *)malloc(sizeof(double) * (size_t)(m * l));
    orc_intermediate_step(m, n, A, lda, Omega, ldo, l, 1, Q, m); /* q = 1 (image_compression/src/rSVD.cpp:103) */
    double *B = (double *)malloc(sizeof(double) * (size_t)(l * n));
    orc_gemm('T', 'N', l, n, m, Q, m, A, lda, 0.0, B, l); /* B = Q^T A (:109) */
    const int64_t d = l < n ? l : n;                      /* min_dim (:112) */
    double *Ut = (double *)malloc(sizeof(double) * (size_t)(l * d));
    const int64_t kept = orc_ic_power_svd(l, n, B, l, d, pm_seed, Ut, S, V);
    orc_gemm('N', 'N', m, d, l, Q, m, Ut, l, 0.0, U, m); /* U = Q * Utilde (:117) */
    free(Ut); free(B); free(Q);
    return kept;
}
