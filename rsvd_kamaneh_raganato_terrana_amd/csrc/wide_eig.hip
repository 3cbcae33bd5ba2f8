// wide_eig.hip -- the small SVD of the rSVD through a symmetric eigensolver (fp32 results, l > 64).
//
// SVD<Jacobi>::compute on B (include/SVD_class.hpp:100-180) needs W = U_w S V_w^T for the l x l
// W = R^T (R = Q_B^T B^T, wide.cpp).  The block one-sided Jacobi of wide_svd.hip reaches it through
// ~8 sweeps of (LP / 16 - 1) grid-synchronised rounds, each a serial 31-step inner sweep: a latency
// chain of ~ 2 LP x sweeps dependent steps (C4 3.6 ms, C5 10.6 ms per rSVD).  This
// file replaces the iteration by a direct method with ONE dependent step per column:
//   1. G = W^T W (fp64 MFMA GEMM, gemm.hip);
//   2. G = Q_H T Q_H^T, Householder tridiagonalisation (tridiag_kernel): NW workgroups each hold
//      rows of G in registers; per column one hand-off (all-gather of the matrix-vector product
//      p = tau G v and of the next pivot row), everything else is replicated per workgroup;
//   3. the eigenvalues of T by Sturm-count multisection (tridiag_bisect_kernel: one wave per
//      eigenvalue, 64 shifts per round, three-term recurrence with power-of-two rescaling);
//   4. the eigenvectors of T by inverse iteration (tridiag_invit_kernel: one thread per vector,
//      LU with partial pivoting of T - lambda I, LAPACK dlagtf/dlagts semantics); vectors whose
//      eigenvalues are closer than kClusterTol |lambda|_max are re-orthogonalised (CGS2,
//      cluster_orth_kernel) -- inverse iteration only needs that inside clusters;
//   5. V_w = Q_H Z: compact-WY blocks of 32 reflectors (wy_t_kernel builds T_b, wy_apply_kernel
//      applies them to 16-column blocks of Z held in LDS, fp64 MFMA);
//   6. X = W V_w (fp64 MFMA GEMM); then wide_svd.hip's block Jacobi runs in "given" mode: it
//      measures the largest cosine between the columns of X (an LP x LP fp64 Gram over the grid)
//      and stops at once when it is below the fp32-result tolerance -- otherwise it polishes X, V_w
//      by ordinary sweeps, which converge quadratically from there.  The finish (S = |x_k|,
//      U_w = X / S sorted descending, zero-S completion) is wide_svd.hip's.
// Accuracy: the Gram squares the condition number, so small singular values lose relative accuracy
// (absolute error ~ eps |W|^2 / s_k in s_k); the Jacobi check bounds the non-orthogonality of the
// resulting U_w, and the results are delivered in fp32 anyway (1e-4 bar).  fp64 results keep the
// block Jacobi (its relative accuracy for small singular values is what the fp64 tests pin).
// numpy model of the same algorithm (Householder + multisection + inverse iteration + CGS2 in
// clusters + back-transformation) on the C4 small matrix: max cos between the columns of X 9e-15,
// |S - S_lapack| / |S| 6e-16.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "common.hpp"
#include "kernels.hpp"
#include "wide.hpp"
#include "dense.hpp"

namespace rsvd {

namespace {

typedef Mfma<double> MD;
constexpr double kEpsE = 2.220446049250313e-16;
constexpr int kEigThreads = 512;
constexpr int kEigMaxN = 512;
// eigenvalues within kClusterTol * max|lambda| of their neighbour: re-orthogonalised vectors
constexpr double kClusterTol = 1e-9;
// sync words (in the block-Jacobi sync block, past its own 384): hand-off counter, abort
constexpr int kTriCtr = 448, kTriAbort = 449;

__device__ __forceinline__ void st_wt(double* p, double v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_wt(const double* p) {
    return __hip_atomic_load(const_cast<double*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Sum over the 512-thread workgroup in a fixed order (bit-identical on every workgroup for
// identical inputs); two alternating halves of red[16], so back-to-back calls need one barrier each.
__device__ __forceinline__ double block_sum512(double x, double* red, int& tog) {
    x = warp_sum(x);
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    double* r = red + 8 * tog;
    tog ^= 1;
    if (lane == 0) r[w] = x;
    __syncthreads();
    double t = 0.0;
#pragma unroll
    for (int k = 0; k < 8; ++k) t += r[k];
    return t;
}

// The fence-free group hand-off of wide_svd.hip (MI355X_MICROARCH.md "Hand-offs measured with sc1
// loads", first row): sc1 stores, vmcnt(0) in every storing wave, one agent-scope add, sc1 poll.
__device__ bool tri_barrier(unsigned* sync, unsigned target) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    __shared__ int ok;
    if (threadIdx.x == 0) {
        unsigned* ctr = sync + kTriCtr;
        __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        int good = 1;
        long spins = 0;
        while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
            __builtin_amdgcn_s_sleep(1);
            if ((++spins & 1023) == 0 &&
                (__hip_atomic_load(sync + kTriAbort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0 ||
                 spins > (1l << 26))) {
                __hip_atomic_store(sync + kTriAbort, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                good = 0;
                break;
            }
        }
        ok = good;
    }
    __syncthreads();
    return ok != 0;
}

// Householder reflector of the row `row` (LDS, this row of the current matrix) for column k:
// x = row[k+1 .. n), H = I - tau v v^T with v[k+1] = 1, H x = beta e_{k+1} (LAPACK dlarfg: tau = 0
// when x[k+2 ..] = 0).  Writes v into vout[0 .. n) (zeros up to k); returns tau, beta.
__device__ __forceinline__ void house(const double* row, int k, int n, double* vout, double* red, int& tog,
                                      double& tau, double& beta) {
    const int tid = threadIdx.x;
    double xj = 0.0;
    for (int j = tid; j < n; j += kEigThreads)
        if (j > k + 1) xj += row[j] * row[j];
    const double xn2 = block_sum512(xj, red, tog);
    const double a0 = row[k + 1];
    double scal = 0.0;
    if (xn2 == 0.0) {
        tau = 0.0;
        beta = a0;
    } else {
        const double nr = sqrt(a0 * a0 + xn2);
        beta = a0 >= 0.0 ? -nr : nr;
        tau = (beta - a0) / beta;
        scal = 1.0 / (a0 - beta);
    }
    for (int j = tid; j < kEigMaxN; j += kEigThreads)
        vout[j] = (j == k + 1) ? 1.0 : ((j > k + 1 && j < n) ? row[j] * scal : 0.0);
}

// Householder tridiagonalisation of the symmetric n x n G (column-major, ld; n <= 512) by NW
// workgroups.  Row i belongs to workgroup i % NW (cyclic: every member keeps active rows to the
// end), local row li = i / NW held by wave li % 8 in register slot li / 8; lane holds columns
// lane + 64 u.  Step k (A_k -> A_{k+1} = H_k A_k H_k):
//   p = tau_k A_k v_k       each member its rows, published (row-group hand-off, double-buffered by
//                           step parity) with the pivot row k + 1 of A_k by its owner;
//   K = tau_k / 2 v_k.p, w = p - K v_k, row k+1 of A_{k+1} = row - w - w_{k+1} v_k;
//   v_{k+1}, tau_{k+1}      from that row, identical on every member (fixed-order sums);
//   A_{k+1} = A_k - v w^T - w v^T on the registers, fused with the next partial product.
// Out: d (n), e (n - 1), tau (n - 2) and the reflectors as columns of Y (ld; v_k[k+1] = 1).
template <int RT, int CT, int NW>
__global__ __launch_bounds__(kEigThreads) void tridiag_kernel(const double* __restrict__ G, int ld, int n,
                                                              double* __restrict__ Y, double* __restrict__ dvec,
                                                              double* __restrict__ evec, double* __restrict__ taus,
                                                              double* __restrict__ xch, unsigned* __restrict__ sync,
                                                              int* __restrict__ info) {
    constexpr int RPW = 8 * RT;                  // rows per member
    constexpr int XS = NW * RPW + kEigMaxN;      // one parity's exchange slots: p, then the pivot row
    __shared__ double vb[2][kEigMaxN];
    __shared__ double ps[kEigMaxN], ws[kEigMaxN], rs[kEigMaxN];
    __shared__ double red[16];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int g = blockIdx.x;
    int tog = 0;
    if (n <= 2) {
        if (g == 0 && tid == 0) {
            dvec[0] = G[0];
            if (n == 2) {
                dvec[1] = G[(int64_t)ld + 1];
                evec[0] = G[1];
            }
        }
        return;
    }
    double a[RT][CT];
#pragma unroll
    for (int t = 0; t < RT; ++t) {
        const int i = (w + 8 * t) * NW + g;
#pragma unroll
        for (int u = 0; u < CT; ++u) {
            const int j = lane + 64 * u;
            a[t][u] = (i < n && j < n) ? G[(int64_t)i * ld + j] : 0.0;  // G(j, i) = G(i, j)
        }
    }
    for (int j = tid; j < kEigMaxN; j += kEigThreads) rs[j] = j < n ? G[j] : 0.0;  // row 0
    __syncthreads();
    double tau, beta;
    house(rs, 0, n, vb[0], red, tog, tau, beta);
    if (g == 0) {
        for (int j = tid; j < ld; j += kEigThreads) Y[j] = j < n ? vb[0][j] : 0.0;
        if (tid == 0) {
            dvec[0] = rs[0];
            evec[0] = beta;
            taus[0] = tau;
        }
    }
    __syncthreads();
    double s[RT];
#pragma unroll
    for (int t = 0; t < RT; ++t) {
        double acc = 0.0;
#pragma unroll
        for (int u = 0; u < CT; ++u) acc += a[t][u] * vb[0][lane + 64 * u];
        s[t] = acc;
    }
    int cur = 0;
    for (int k = 0; k <= n - 3; ++k) {
        const double* vc = vb[cur];
        double* vn = vb[cur ^ 1];
        double* xp = xch + (int64_t)(k & 1) * XS;  // this step's slots
        // A. publish p = tau A_k v_k (rows > k; zero for rows <= k) and the pivot row k + 1
#pragma unroll
        for (int t = 0; t < RT; ++t) {
            const double tot = warp_sum(s[t]);
            const int li = w + 8 * t, i = li * NW + g;
            if (lane == 0 && i < n) {
                const double pv = i > k ? tau * tot : 0.0;
                if constexpr (NW == 1) ps[i] = pv;
                else st_wt(xp + g * RPW + li, pv);
            }
        }
        if ((k + 1) % NW == g) {
            const int li1 = (k + 1) / NW;
            if (w == (li1 & 7)) {
#pragma unroll
                for (int t = 0; t < RT; ++t) {
                    if (t == (li1 >> 3)) {
#pragma unroll
                        for (int u = 0; u < CT; ++u) {
                            const int j = lane + 64 * u;
                            if (j < n) {
                                if constexpr (NW == 1) rs[j] = a[t][u];
                                else st_wt(xp + NW * RPW + j, a[t][u]);
                            }
                        }
                    }
                }
            }
        }
        // B. the hand-off
        if constexpr (NW > 1) {
            if (!tri_barrier(sync, (unsigned)NW * (unsigned)(k + 1))) {
                if (tid == 0) info[2] = 1;
                return;
            }
            for (int j = tid; j < n; j += kEigThreads) {
                ps[j] = ld_wt(xp + (j % NW) * RPW + j / NW);
                rs[j] = ld_wt(xp + NW * RPW + j);
            }
        }
        __syncthreads();
        // C. K, w, the pivot row of A_{k+1}, the next reflector
        double dv = 0.0;
        for (int j = tid; j < n; j += kEigThreads) dv += vc[j] * ps[j];
        const double K = 0.5 * tau * block_sum512(dv, red, tog);
        const double wk1 = ps[k + 1] - K * vc[k + 1];
        for (int j = tid; j < kEigMaxN; j += kEigThreads) {
            const double wj = j < n ? ps[j] - K * vc[j] : 0.0;
            ws[j] = wj;
            if (j > k && j < n) rs[j] = rs[j] - wj - wk1 * vc[j];  // row k + 1 of A_{k+1} (own j only)
        }
        __syncthreads();
        double taun = 0.0, betan = 0.0;
        if (k + 1 <= n - 3) {
            house(rs, k + 1, n, vn, red, tog, taun, betan);
            if (g == 0) {
                for (int j = tid; j < ld; j += kEigThreads) Y[(int64_t)(k + 1) * ld + j] = j < n ? vn[j] : 0.0;
                if (tid == 0) {
                    dvec[k + 1] = rs[k + 1];
                    evec[k + 1] = betan;
                    taus[k + 1] = taun;
                }
            }
        } else {
            for (int j = tid; j < kEigMaxN; j += kEigThreads) vn[j] = 0.0;
            if (g == 0 && tid == 0) {
                dvec[n - 2] = rs[n - 2];
                evec[n - 2] = rs[n - 1];
            }
        }
        __syncthreads();
        // D. A_{k+1} = A_k - v w^T - w v^T on the registers, and the next partial product
        double vj[CT], wj[CT], vnj[CT];
#pragma unroll
        for (int u = 0; u < CT; ++u) {
            vj[u] = vc[lane + 64 * u];
            wj[u] = ws[lane + 64 * u];
            vnj[u] = vn[lane + 64 * u];
        }
#pragma unroll
        for (int t = 0; t < RT; ++t) {
            const int i = (w + 8 * t) * NW + g;
            const int ii = i < kEigMaxN ? i : kEigMaxN - 1;
            const double vi = i < n ? vc[ii] : 0.0, wi = i < n ? ws[ii] : 0.0;
            double acc = 0.0;
#pragma unroll
            for (int u = 0; u < CT; ++u) {
                a[t][u] -= vi * wj[u] + wi * vj[u];
                acc += a[t][u] * vnj[u];
            }
            s[t] = acc;
            if (k == n - 3 && i == n - 1) {  // the last diagonal entry, from its owner
#pragma unroll
                for (int u = 0; u < CT; ++u)
                    if (lane + 64 * u == n - 1) dvec[n - 1] = a[t][u];
            }
        }
        tau = taun;
        cur ^= 1;
    }
}

// Number of eigenvalues of T (d, e2 = e^2, both LDS) below x: sign changes of the leading principal
// minors p_i = (d_i - x) p_{i-1} - e2_{i-1} p_{i-2} (Sturm sequence; an exact zero counts as a change),
// with a power-of-two rescale every 8 steps (the ratios -- all the count uses -- are unchanged).
__device__ __forceinline__ int sturm_count(const double* d, const double* e2, int n, double x) {
    double p0 = 1.0, p1 = d[0] - x;
    if (p1 == 0.0) p1 = -1e-300;
    int c = p1 < 0.0;
    int i = 1;
    while (i < n) {
        const int iend = min(n, i + 8);
        for (; i < iend; ++i) {
            double p2 = (d[i] - x) * p1 - e2[i - 1] * p0;
            if (p2 == 0.0) p2 = p1 < 0.0 ? 1e-300 : -1e-300;
            c += (p2 < 0.0) != (p1 < 0.0);
            p0 = p1;
            p1 = p2;
        }
        const int ex = __builtin_amdgcn_frexp_exp(fmax(fabs(p0), fabs(p1)));
        p0 = __builtin_ldexp(p0, -ex);
        p1 = __builtin_ldexp(p1, -ex);
    }
    return c;
}

// Eigenvalues of the symmetric tridiagonal T (d: n, e: n - 1), descending into lam; one wave per
// eigenvalue: 64 shifts per round split the bracket into 65 parts (9-11 rounds to an fp64 bracket).
// T is scaled by its Gershgorin bound first; tnorm[0] = that bound (inverse iteration's scale).
__global__ __launch_bounds__(256) void tridiag_bisect_kernel(const double* __restrict__ dg, const double* __restrict__ eg,
                                                             int n, double* __restrict__ lam, double* __restrict__ tnorm) {
    __shared__ double d[kEigMaxN], e2[kEigMaxN];
    __shared__ double rlo[4], rhi[4];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    double lo = 1e300, hi = -1e300;
    for (int i = tid; i < n; i += 256) {
        const double el = i > 0 ? fabs(eg[i - 1]) : 0.0, er = i + 1 < n ? fabs(eg[i]) : 0.0;
        lo = fmin(lo, dg[i] - el - er);
        hi = fmax(hi, dg[i] + el + er);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        lo = fmin(lo, __shfl_xor(lo, o, 64));
        hi = fmax(hi, __shfl_xor(hi, o, 64));
    }
    if (lane == 0) rlo[wv] = lo, rhi[wv] = hi;
    __syncthreads();
    lo = fmin(fmin(rlo[0], rlo[1]), fmin(rlo[2], rlo[3]));
    hi = fmax(fmax(rhi[0], rhi[1]), fmax(rhi[2], rhi[3]));
    const double nrm = fmax(fabs(lo), fabs(hi));
    const double inv = nrm > 0.0 ? 1.0 / nrm : 0.0;
    for (int i = tid; i < n; i += 256) {
        d[i] = dg[i] * inv;
        const double es = i + 1 < n ? eg[i] * inv : 0.0;
        e2[i] = es * es;
    }
    if (blockIdx.x == 0 && tid == 0) tnorm[0] = nrm;
    __syncthreads();
    const int jd = blockIdx.x * 4 + wv;  // descending index
    if (jd >= n) return;
    if (nrm == 0.0) {
        if (lane == 0) lam[jd] = 0.0;
        return;
    }
    const int r = n - 1 - jd;  // ascending rank: the eigenvalue x with count(x-) <= r < count(x+)
    const double pad = 4.0 * n * kEpsE;
    double a = lo * inv - pad, b = hi * inv + pad;
    for (int round = 0; round < 14; ++round) {
        const double x = a + (b - a) * (double)(lane + 1) * (1.0 / 65.0);
        const int c = sturm_count(d, e2, n, x);
        const unsigned long long m = __ballot(c > r);
        const int ms = m ? __ffsll((long long)m) - 1 : 64;
        const double xa = __shfl(x, ms > 0 ? ms - 1 : 0, 64), xb = __shfl(x, ms < 64 ? ms : 63, 64);
        const double na = ms > 0 ? xa : a, nb = ms < 64 ? xb : b;
        a = na;
        b = nb;
        if (b - a <= 2.0 * kEpsE * fmax(fabs(a), fabs(b)) || b - a <= 1e-3 * kEpsE) break;
    }
    if (lane == 0) lam[jd] = 0.5 * (a + b) * nrm;
}

__device__ __forceinline__ double unit_hash(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    x ^= x >> 31;
    return (double)(x >> 11) * (2.0 / 9007199254740992.0) - 1.0;  // uniform in [-1, 1)
}

// Inverse iteration for every eigenvalue: thread k factors T - lam_k I = P L U (partial pivoting,
// LAPACK dlagtf; |u_ii| below eps |T| is replaced by +-eps |T|) and runs three solves from a
// pseudo-random start, rescaling by the largest entry between solves; the unit vector goes to
// row-major Z (Z[i][k], ld ldz).  Scratch: six n x ldz arrays laid out [i][k] (coalesced over k).
__global__ __launch_bounds__(64) void tridiag_invit_kernel(const double* __restrict__ dg, const double* __restrict__ eg,
                                                           const double* __restrict__ lam, const double* __restrict__ tnorm,
                                                           int n, int ldz, double* __restrict__ Z,
                                                           double* __restrict__ scr) {
    const int k = blockIdx.x * 64 + threadIdx.x;
    if (k >= n) return;
    const int64_t S = (int64_t)n * ldz;
    double* U0i = scr;
    double* U1 = scr + S;
    double* U2 = scr + 2 * S;
    double* Lm = scr + 3 * S;
    double* Pv = scr + 4 * S;
    double* X = scr + 5 * S;
    auto at = [&](int i) { return (int64_t)i * ldz + k; };
    const double lk = lam[k];
    const double tol = kEpsE * fmax(tnorm[0], 1e-300);
    auto pivot_inv = [&](double u) {
        if (fabs(u) < tol) u = u < 0.0 ? -tol : tol;
        return 1.0 / u;
    };
    // factor
    double cd = dg[0] - lk, cu = n > 1 ? eg[0] : 0.0;
    for (int i = 0; i < n - 1; ++i) {
        const double bi = eg[i], an = dg[i + 1] - lk, cn = i + 1 < n - 1 ? eg[i + 1] : 0.0;
        if (fabs(bi) > fabs(cd)) {
            const double m = cd / bi;
            U0i[at(i)] = pivot_inv(bi);
            U1[at(i)] = an;
            U2[at(i)] = cn;
            Lm[at(i)] = m;
            Pv[at(i)] = 1.0;
            cd = cu - m * an;
            cu = -m * cn;
        } else {
            const double m = cd != 0.0 ? bi / cd : 0.0;
            U0i[at(i)] = pivot_inv(cd);
            U1[at(i)] = cu;
            U2[at(i)] = 0.0;
            Lm[at(i)] = m;
            Pv[at(i)] = 0.0;
            cd = an - m * cu;
            cu = cn;
        }
    }
    U0i[at(n - 1)] = pivot_inv(cd);
    for (int i = 0; i < n; ++i) X[at(i)] = unit_hash(((uint64_t)k << 32) ^ (uint64_t)i ^ 0x5EED5EEDull);
    double sc = 1.0;
    for (int it = 0; it < 3; ++it) {
        // forward: y = L^-1 P x (in place)
        double yc = X[at(0)] * sc;
        for (int i = 0; i < n - 1; ++i) {
            const double yn = X[at(i + 1)] * sc, m = Lm[at(i)];
            if (Pv[at(i)] != 0.0) {
                X[at(i)] = yn;
                yc = yc - m * yn;
            } else {
                X[at(i)] = yc;
                yc = yn - m * yc;
            }
        }
        X[at(n - 1)] = yc;
        // back: U z = y (z into X), tracking max |z|
        double z1 = 0.0, z2 = 0.0, zmax = 0.0;
        for (int i = n - 1; i >= 0; --i) {
            const double z = (X[at(i)] - U1[at(i)] * z1 - U2[at(i)] * z2) * U0i[at(i)];
            X[at(i)] = z;
            zmax = fmax(zmax, fabs(z));
            z2 = z1;
            z1 = z;
        }
        sc = zmax > 0.0 ? 1.0 / zmax : 1.0;
    }
    double nn = 0.0;
    for (int i = 0; i < n; ++i) {
        const double z = X[at(i)] * sc;
        nn += z * z;
    }
    const double f = sc / sqrt(nn);
    for (int i = 0; i < n; ++i) Z[at(i)] = X[at(i)] * f;
}

// Re-orthogonalise the vectors of eigenvalue clusters (neighbours within kClusterTol max|lam|):
// CGS2 of each member against the earlier members of its cluster, in order.  One workgroup; no
// work when there are no clusters.
__global__ __launch_bounds__(1024) void cluster_orth_kernel(const double* __restrict__ lam, int n, int ldz,
                                                            double* __restrict__ Z) {
    __shared__ double coef[kEigMaxN];
    __shared__ int link[kEigMaxN];
    __shared__ double red[16];
    __shared__ int any;
    const int tid = threadIdx.x, nt = blockDim.x;
    double lmax = 0.0;
    for (int k = 0; k < n; ++k) lmax = fmax(lmax, fabs(lam[k]));
    if (tid == 0) any = 0;
    __syncthreads();
    for (int k = tid; k < n; k += nt) {
        const int l = k + 1 < n && (lam[k] - lam[k + 1]) <= kClusterTol * lmax;
        link[k] = l;
        if (l) any = 1;
    }
    __syncthreads();
    if (!any) return;
    int c0 = 0;
    for (int a = 1; a < n; ++a) {
        if (!link[a - 1]) {
            c0 = a;
            continue;
        }
        for (int pass = 0; pass < 2; ++pass) {
            for (int b = c0 + tid; b < a; b += nt) {
                double dsum = 0.0;
                for (int i = 0; i < n; ++i) dsum += Z[(int64_t)i * ldz + b] * Z[(int64_t)i * ldz + a];
                coef[b - c0] = dsum;
            }
            __syncthreads();
            for (int i = tid; i < n; i += nt) {
                double z = Z[(int64_t)i * ldz + a];
                for (int b = c0; b < a; ++b) z -= coef[b - c0] * Z[(int64_t)i * ldz + b];
                Z[(int64_t)i * ldz + a] = z;
            }
            __syncthreads();
        }
        double part = 0.0;
        for (int i = tid; i < n; i += nt) part += Z[(int64_t)i * ldz + a] * Z[(int64_t)i * ldz + a];
        part = warp_sum(part);
        if ((tid & 63) == 0) red[tid >> 6] = part;
        __syncthreads();
        double nn = 0.0;
        for (int q = 0; q < nt / 64; ++q) nn += red[q];
        const double f = nn > 0.0 ? 1.0 / sqrt(nn) : 0.0;
        for (int i = tid; i < n; i += nt) Z[(int64_t)i * ldz + a] *= f;
        __syncthreads();
    }
}

constexpr int kWY = 32;  // reflectors per compact-WY block

// T_b of block b (reflectors 32 b .. 32 b + 31; tau = 0 past the last one): the upper triangular
// factor of H_{32b} ... H_{32b+31} = I - Y_b T_b Y_b^T (LAPACK dlarft, forward, columnwise).
__global__ __launch_bounds__(256) void wy_t_kernel(const double* __restrict__ Y, int ld, int n, int nref,
                                                   const double* __restrict__ taus, double* __restrict__ Tg) {
    __shared__ double Sg[kWY][kWY + 1], T[kWY][kWY + 1];
    const int b = blockIdx.x, tid = threadIdx.x;
    const int k0 = kWY * b;
    for (int e = tid; e < kWY * kWY; e += 256) {
        const int p = e / kWY, q = e % kWY;
        double sdot = 0.0;
        if (p <= q && k0 + q < nref) {
            const double* yp = Y + (int64_t)(k0 + p) * ld;
            const double* yq = Y + (int64_t)(k0 + q) * ld;
            for (int j = k0 + q + 1; j < n; ++j) sdot += yp[j] * yq[j];  // v_q is zero above q + 1
        }
        Sg[p][q] = sdot;
        T[p][q] = 0.0;
    }
    __syncthreads();
    if (tid == 0) T[0][0] = k0 < nref ? taus[k0] : 0.0;
    __syncthreads();
    for (int i = 1; i < kWY; ++i) {
        const double ti = k0 + i < nref ? taus[k0 + i] : 0.0;
        double acc = 0.0;
        if (tid < i) {
            for (int q = tid; q < i; ++q) acc += T[tid][q] * Sg[q][i];
        }
        __syncthreads();
        if (tid < i) T[tid][i] = -ti * acc;
        if (tid == i) T[i][i] = ti;
        __syncthreads();
    }
    for (int e = tid; e < kWY * kWY; e += 256) Tg[(int64_t)b * kWY * kWY + e] = T[e / kWY][e % kWY];
}

// V = Q_H Z for one 16-column block of the row-major Z (ld ldz), held in LDS: blocks of 32
// reflectors from the last to the first, Z <- Z - Y_b (T_b (Y_b^T Z)) on the fp64 MFMA; then V
// into the column-major Vout (ld ldv; rows >= n written as zero).  256 threads.
__global__ __launch_bounds__(256) void wy_apply_kernel(const double* __restrict__ Y, int ld, int n, int nref,
                                                       const double* __restrict__ Tg, const double* __restrict__ Z,
                                                       int ldz, double* __restrict__ Vout, int ldv) {
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    double* Zs = reinterpret_cast<double*>(smem_raw);  // [n][17]
    __shared__ double Ms[2][kWY][17];
    __shared__ double Ts[kWY][kWY + 1];
    constexpr int ZP = 17;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int r = lane & 15, h = lane >> 4;
    const int c0 = 16 * blockIdx.x;
    for (int e = tid; e < n * 16; e += 256) {
        const int i = e >> 4, c = e & 15;
        Zs[i * ZP + c] = c0 + c < n ? Z[(int64_t)i * ldz + c0 + c] : 0.0;
    }
    const int nb = (nref + kWY - 1) / kWY;
    for (int b = nb - 1; b >= 0; --b) {
        const int k0 = kWY * b;
        const int j0 = k0 + 1;  // first row any reflector of the block touches
        for (int e = tid; e < kWY * kWY; e += 256) Ts[e / kWY][e % kWY] = Tg[(int64_t)b * kWY * kWY + e];
        __syncthreads();
        // M = Y_b^T Z (32 x 16): wave w -> tile rows (w & 1), k (row) quarter... halves (w >> 1)
        {
            const int rt = w & 1, half = w >> 1;
            const int len = n - j0;
            const int q0 = j0 + ((len + 7) / 8 * 4) * half;  // 4-aligned split of [j0, n)
            const int q1 = half ? n : min(n, q0 + (len + 7) / 8 * 4);
            f64x4 acc = MD::zero();
            const int col = k0 + 16 * rt + r;  // reflector of this lane's A row
            const double* yc = Y + (int64_t)col * ld;
            for (int j = q0; j < q1; j += 4) {
                const int jj = j + h;
                const double av = (jj < q1 && col < nref) ? yc[jj] : 0.0;
                const double bv = jj < q1 ? Zs[jj * ZP + r] : 0.0;
                acc = MD::mma(av, bv, acc);
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) Ms[half][16 * rt + MD::row(h, q)][r] = acc[q];
        }
        __syncthreads();
        // M2 = T_b M (upper triangular T), into Ms[0]
        double m2[2];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int e = tid + 256 * q, rr = e >> 4, cc = e & 15;
            double acc = 0.0;
            for (int p = rr; p < kWY; ++p) acc += Ts[rr][p] * (Ms[0][p][cc] + Ms[1][p][cc]);
            m2[q] = acc;
        }
        __syncthreads();
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int e = tid + 256 * q;
            Ms[0][e >> 4][e & 15] = m2[q];
        }
        __syncthreads();
        // Z -= Y_b M2: 16-row tiles of rows [j0, n), wave w -> tiles w, w + 4, ...
        const int t0 = j0 & ~15;
        for (int ti = t0 + 16 * w; ti < n; ti += 64) {
            f64x4 acc = MD::zero();
            const int row = ti + r;
#pragma unroll
            for (int s = 0; s < kWY / 4; ++s) {
                const int kk = 4 * s + h;
                const double av = (row < n && row >= j0 && k0 + kk < nref) ? Y[(int64_t)(k0 + kk) * ld + row] : 0.0;
                acc = MD::mma(av, Ms[0][kk][r], acc);
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int rr = ti + MD::row(h, q);
                if (rr < n) Zs[rr * ZP + r] -= acc[q];
            }
        }
        __syncthreads();
    }
    for (int c = 0; c < 16; ++c) {
        if (c0 + c >= n) break;
        for (int i = tid; i < ldv; i += 256) Vout[(int64_t)(c0 + c) * ldv + i] = i < n ? Zs[i * ZP + c] : 0.0;
    }
}

template <int RT, int CT, int NW>
hipError_t launch_tridiag(const double* G, int ld, int n, double* Y, double* d, double* e, double* taus, double* xch,
                          unsigned* sync, int* info, hipStream_t s) {
    return launch_coresident(tridiag_kernel<RT, CT, NW>, dim3(NW), dim3(kEigThreads), 0, s, G, ld, n, Y, d, e, taus,
                             xch, sync, info);
}

}  // namespace

size_t eig_svd_ws_doubles(int LP) {
    const size_t L2 = (size_t)LP * LP;
    const size_t nb = (LP + kWY - 1) / kWY;
    return 9 * L2 + nb * kWY * kWY + 4 * (size_t)LP + 64 + 2 * (size_t)(2 * kEigMaxN);
}

template <typename T>
hipError_t launch_eig_svd(const double* R, int l, int LP, double* ews, double* X, double* J, double* Uw, double* Vw,
                          T* S, unsigned* sync, int* info, hipStream_t s, double tol_chk) {
    if (l < 3 || l > kEigMaxN || LP < l || LP % 32 || LP > kEigMaxN) return hipErrorInvalidValue;
    const size_t L2 = (size_t)LP * LP;
    double* G = ews;
    double* Y = G + L2;
    double* Z = Y + L2;
    double* scr = Z + L2;  // 6 L2
    double* Tg = scr + 6 * L2;
    const int nb = (LP + kWY - 1) / kWY;
    double* d = Tg + (size_t)nb * kWY * kWY;
    double* e = d + LP;
    double* taus = e + LP;
    double* lam = taus + LP;
    double* tnorm = lam + LP;
    double* xch = tnorm + 64;
    const int n = l, nref = n - 2;
    hipError_t er;
    // 1. G = W^T W, W = the column-major view of R (ld LP)
    if ((er = launch_gemm<double>(1, 0, n, n, n, 1.0, R, LP, R, LP, 0.0, G, LP, s)) != hipSuccess) return er;
    // 2. tridiagonalisation
    if ((er = hipMemsetAsync(Y, 0, L2 * sizeof(double), s)) != hipSuccess) return er;
    if ((er = hipMemsetAsync(taus, 0, LP * sizeof(double), s)) != hipSuccess) return er;
    if ((er = hipMemsetAsync(sync + kTriCtr, 0, 2 * sizeof(unsigned), s)) != hipSuccess) return er;
    if (LP <= 128)
        er = launch_tridiag<16, 2, 1>(G, LP, n, Y, d, e, taus, xch, sync, info, s);
    else if (LP <= 256)
        er = launch_tridiag<8, 4, 4>(G, LP, n, Y, d, e, taus, xch, sync, info, s);
    else
        er = launch_tridiag<4, 8, 16>(G, LP, n, Y, d, e, taus, xch, sync, info, s);
    if (er != hipSuccess) return er;
    // 3. eigenvalues (descending), 4. eigenvectors of T (row-major Z), cluster re-orthogonalisation
    hipLaunchKernelGGL(tridiag_bisect_kernel, dim3((n + 3) / 4), dim3(256), 0, s, d, e, n, lam, tnorm);
    hipLaunchKernelGGL(tridiag_invit_kernel, dim3((n + 63) / 64), dim3(64), 0, s, d, e, lam, tnorm, n, LP, Z, scr);
    hipLaunchKernelGGL(cluster_orth_kernel, dim3(1), dim3(1024), 0, s, lam, n, LP, Z);
    // 5. V_w = Q_H Z into J (buffer 0, column-major LP x LP; columns >= n zero)
    if ((er = hipMemsetAsync(J, 0, L2 * sizeof(double), s)) != hipSuccess) return er;
    if (nref > 0) hipLaunchKernelGGL(wy_t_kernel, dim3((nref + kWY - 1) / kWY), dim3(256), 0, s, Y, LP, n, nref, taus, Tg);
    hipLaunchKernelGGL(wy_apply_kernel, dim3((n + 15) / 16), dim3(256), (size_t)n * 17 * sizeof(double), s, Y, LP, n,
                       nref, Tg, Z, LP, J, LP);
    if ((er = hipGetLastError()) != hipSuccess) return er;
    // 6. X = W V_w into X (buffer 0, column-major), then the checked block-Jacobi finish
    if ((er = hipMemsetAsync(X, 0, L2 * sizeof(double), s)) != hipSuccess) return er;
    if ((er = launch_gemm<double>(0, 0, n, n, n, 1.0, R, LP, J, LP, 0.0, X, LP, s)) != hipSuccess) return er;
    return launch_block_jacobi_given<T>(l, LP, X, J, Uw, Vw, S, sync, info, s, tol_chk);
}

template hipError_t launch_eig_svd<float>(const double*, int, int, double*, double*, double*, double*, double*, float*,
                                          unsigned*, int*, hipStream_t, double);
template hipError_t launch_eig_svd<double>(const double*, int, int, double*, double*, double*, double*, double*,
                                           double*, unsigned*, int*, hipStream_t, double);

}  // namespace rsvd
