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
//      cluster_orth_kernel), then one Newton-Schulz step over all of Z (two GEMMs) removes the
//      eps / gap_rel non-orthogonality of close but separated pairs;
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
// eigenvalues within kClusterTol * max|lambda| of their neighbour (exact or near-exact
// degeneracies, where inverse iteration from random starts returns random vectors of the
// eigenspace): CGS2 of the cluster's vectors, in order.  Every other pair is orthogonal to
// ~eps / gap_rel <= 2e-4 after inverse iteration, and one Newton-Schulz step Z (3 I - Z^T Z) / 2 over
// the whole Z squares that (its mixing of a pair i, j is ~eps |G| / |lam_i - lam_j|, so the eigen
// residuals stay at eps |G|).
constexpr double kClusterTol = 1e-12;
constexpr double kSturmPadD = 4.0;  // the padding steps' diagonal in sturm_count (scaled units)
constexpr double kE2Min = 1e-300;  // smallest squared off-diagonal in the Sturm counts (T scaled to |T| <= 1)
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
// `inject` (RSVD_TRI_FORCE_ABORT, fault injection for the tests): this member arrives, then takes the
// timeout branch at once -- the abort word goes up and every other member leaves at its next spin check.
__device__ bool tri_barrier(unsigned* sync, unsigned target, bool inject = false) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    __shared__ int ok;
    if (threadIdx.x == 0) {
        unsigned* ctr = sync + kTriCtr;
        __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        int good = 1;
        long spins = 0;
        if (inject) {
            __hip_atomic_store(sync + kTriAbort, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            good = 0;
        }
        while (good && __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
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

// fp64 reciprocal / reciprocal square root from the hardware estimates (two Newton steps each)
__device__ __forceinline__ double rcp_f64(double d) {
    double y = __builtin_amdgcn_rcp(d);
    y = y * fma(-d, y, 2.0);
    return y * fma(-d, y, 2.0);
}
__device__ __forceinline__ double rsqrt_f64(double d) {
    double y = __builtin_amdgcn_rsq(d);
    y = y * fma(-0.5 * d * y, y, 1.5);
    return y * fma(-0.5 * d * y, y, 1.5);
}

// RSVD_TRI_PROF (lab builds only): shader-cycle totals of the step phases of tridiag_kernel,
// workgroup 0 thread 0, read back by tri_prof_read (tools/eig_lab.cpp)
#ifdef RSVD_TRI_PROF
__device__ long long g_tri_prof[16];  // [0, 4): multi-workgroup steps, [8, 12): one workgroup; [4, 8): inverse iteration
#define TRI_INIT() long long tri_last_ = __builtin_amdgcn_s_memtime()
#define TRI_TS(i)                                                        \
    do {                                                                 \
        if (blockIdx.x == 0 && threadIdx.x == 0) {                       \
            const long long now_ = __builtin_amdgcn_s_memtime();         \
            g_tri_prof[(i) + (NW == 1 ? 8 : 0)] += now_ - tri_last_;     \
            tri_last_ = now_;                                            \
        }                                                                \
    } while (0)
#define TRI_DONE() \
    do {           \
    } while (0)
#define INV_INIT() long long inv_last_ = __builtin_amdgcn_s_memtime()
#define INV_TS(i)                                                        \
    do {                                                                 \
        if (blockIdx.x == 0 && threadIdx.x == 0) {                       \
            __builtin_amdgcn_s_waitcnt(0);                               \
            const long long now_ = __builtin_amdgcn_s_memtime();         \
            g_tri_prof[(i)] += now_ - inv_last_;                         \
            inv_last_ = now_;                                            \
        }                                                                \
    } while (0)
#else
#define INV_INIT() \
    do {           \
    } while (0)
#define INV_TS(i) \
    do {          \
    } while (0)
#define TRI_INIT() \
    do {           \
    } while (0)
#define TRI_TS(i) \
    do {          \
    } while (0)
#define TRI_DONE() \
    do {           \
    } while (0)
#endif

// Cross-lane fp64 sums on DPP (two v_mov_dpp per step, no LDS round trip -- a __shfl_xor is a
// ds_bpermute pair, ~100 cycles of latency per step, and a 6-step wave sum of those sat on the
// tridiagonalisation's critical path three times per column).
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, 0xf, 0xf, true);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, 0xf, 0xf, true);
    return __hiloint2double(hi, lo);
}
constexpr int kDppXor1 = 0xB1, kDppXor2 = 0x4E, kDppHalfMirror = 0x141, kDppMirror = 0x140;
__device__ __forceinline__ double readlane_f64(double v, int lane) {
    const int lo = __builtin_amdgcn_readlane(__double2loint(v), lane);
    const int hi = __builtin_amdgcn_readlane(__double2hiint(v), lane);
    return __hiloint2double(hi, lo);
}
// Sum over the LPR lanes of an aligned lane group (LPR in {8, 16, 32}); every lane of the group gets
// the same total (each step adds two partial sums: commutative, so all lanes agree bit for bit).
template <int LPR>
__device__ __forceinline__ double group_sum(double v) {
    v += dpp_f64<kDppXor1>(v);
    v += dpp_f64<kDppXor2>(v);
    v += dpp_f64<kDppHalfMirror>(v);
    if constexpr (LPR >= 16) v += dpp_f64<kDppMirror>(v);
    if constexpr (LPR >= 32) v += __shfl_xor(v, 16, 64);
    return v;
}
// Sum over the whole wave, wave-uniform (the four 16-lane row totals read back in a fixed order).
__device__ __forceinline__ double wave_total(double v) {
    v = group_sum<16>(v);
    return (readlane_f64(v, 0) + readlane_f64(v, 16)) + (readlane_f64(v, 32) + readlane_f64(v, 48));
}

// Householder tridiagonalisation of the symmetric G (LAPACK dsytd2's reflectors, v_k[k+1] = 1), in
// one or two launches:
//   phase 1: NW workgroups hold the rows of G in registers (row i on workgroup i % NW: every member
//            keeps active rows to the end) and run steps 0 .. kend - 1 with ONE hand-off per step,
//            then dump the trailing block (rows / columns >= kend + 1) of A_kend;
//   phase 2: one workgroup loads that block (t <= 192 rows: it fits the registers) and finishes the
//            steps kend .. n - 3 with workgroup barriers only.
// Register layout: a wave is G = 64 / LPR groups of LPR lanes (lane = g LPR + c); lane (g, c) holds
// RPL rows -- local row q (8 G) + w G + g of the workgroup -- at the CPL columns c + LPR u.  Local row
// li of workgroup wg is row off + li NW + wg of the matrix, local column j is column off + j.
// Step k (A_k -> A_{k+1} = H_k A_k H_k, LAPACK dsytd2 / dlatrd without the blocking):
//   [A] p = tau_k A_k v_k (each member its rows: a reduction over LPR lanes per row), the per-wave
//       partials of v_k . p, and the pivot row k + 1 of A_k by its owner -- to LDS (one workgroup) or
//       published (sc1 stores, the row-group hand-off, double-buffered by step parity);
//   [C] K = tau_k / 2 v_k . p (the partials summed in one fixed order: bit-identical on every
//       member), w = p - K v_k, the pivot row of A_{k+1} = row - w - w_{k+1} v_k, |row[k+3 ..]|^2;
//   [E] v_{k+1}, tau_{k+1}, beta (= e_{k+1}) from that row, identical on every member;
//   [D] A_{k+1} = A_k - v w^T - w v^T on the registers, fused with the next partial products.
// Out: d (n), e (n - 1), tau (n - 2) and the reflectors as the columns of Y (ldy; v_k[k+1] = 1).
template <int RPL, int CPL, int LPR, int NW>
__global__ __launch_bounds__(kEigThreads) void tridiag_kernel(const double* __restrict__ src, int lds, int n, int off,
                                                              int kend, double* __restrict__ Y, int ldy,
                                                              double* __restrict__ dvec, double* __restrict__ evec,
                                                              double* __restrict__ taus, double* __restrict__ dump,
                                                              double* __restrict__ xch, unsigned* __restrict__ sync,
                                                              int* __restrict__ info, int noskip, int abort_at) {
    constexpr int G = 64 / LPR;
    constexpr int RPW = 8 * G * RPL;                     // rows per member
    constexpr int XS = NW * RPW + 8 * NW + kEigMaxN;     // one parity's exchange slots: p, v.p partials, row
    __shared__ double vb[2][kEigMaxN];
    __shared__ double ps[kEigMaxN], ws[kEigMaxN], rs[kEigMaxN], rb[kEigMaxN];
    __shared__ double rv[kEigMaxN];  // rb past index k + 2 (else 0): v_{k+1} = scal rv + e_{k+2}
    __shared__ double vpw[8 * NW];
    __shared__ double red[8];
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: the row-slot tests stay scalar
    const int g = lane / LPR, c = lane % LPR;
    const int wg = blockIdx.x;
    const int t = n - off;  // local size
    if (n <= 2) {
        if (wg == 0 && tid == 0) {
            dvec[0] = src[0];
            if (n == 2) {
                dvec[1] = src[(int64_t)lds + 1];
                evec[0] = src[1];
            }
        }
        return;
    }
    auto lrow = [&](int q) { return (q * (8 * G) + w * G + g) * NW + wg; };  // local row of slot q
    double a[RPL][CPL];
#pragma unroll
    for (int q = 0; q < RPL; ++q) {
        const int i = lrow(q);
#pragma unroll
        for (int u = 0; u < CPL; ++u) {
            const int j = c + LPR * u;
            a[q][u] = (i < t && j < t) ? src[(int64_t)i * lds + j] : 0.0;  // symmetric: row i = column i
        }
    }
    const int kbeg = off == 0 ? 0 : off - 1;
    double tau;
    if (off == 0) {
        // v_0 from row 0 (LAPACK dlarfg: tau = 0 when the column below the subdiagonal is zero)
        for (int j = tid; j < kEigMaxN; j += kEigThreads) rs[j] = j < n ? src[j] : 0.0;
        __syncthreads();
        double xj = 0.0;
        for (int j = tid; j < n; j += kEigThreads)
            if (j > 1) xj += rs[j] * rs[j];
        xj = warp_sum(xj);
        if (lane == 0) red[w] = xj;
        __syncthreads();
        double xn2 = 0.0;
#pragma unroll
        for (int q = 0; q < 8; ++q) xn2 += red[q];
        const double a0 = rs[1];
        double beta = a0, scal = 0.0;
        tau = 0.0;
        if (xn2 != 0.0) {
            const double nr = sqrt(a0 * a0 + xn2);
            beta = a0 >= 0.0 ? -nr : nr;
            tau = (beta - a0) / beta;
            scal = 1.0 / (a0 - beta);
        }
        for (int j = tid; j < kEigMaxN; j += kEigThreads) {
            const double v = (j == 1) ? 1.0 : ((j > 1 && j < n) ? rs[j] * scal : 0.0);
            vb[0][j] = v;
            if (wg == 0 && j < n) Y[j] = v;
        }
        if (wg == 0 && tid == 0) {
            dvec[0] = rs[0];
            evec[0] = beta;
            taus[0] = tau;
        }
    } else {
        // phase 2: v_kbeg (written to Y by phase 1) in local coordinates
        for (int j = tid; j < kEigMaxN; j += kEigThreads) vb[0][j] = j < t ? Y[(int64_t)kbeg * ldy + off + j] : 0.0;
        tau = taus[kbeg];
    }
    __syncthreads();
    double s[RPL];
#pragma unroll
    for (int q = 0; q < RPL; ++q) {
        double acc = 0.0;
#pragma unroll
        for (int u = 0; u < CPL; ++u) acc += a[q][u] * vb[0][c + LPR * u];
        s[q] = acc;
    }
    int cur = 0;
    double scal = 0.0;  // v_k = scal * rb past its leading 1 (rb: row k of A_k, from the previous step)
    TRI_INIT();
    for (int k = kbeg; k < kend; ++k) {
        double* vc = vb[cur];
        double* vn = vb[cur ^ 1];
        const int l1 = k + 1 - off;  // local index of the pivot row k + 1
        double* xp = xch + (int64_t)((k - kbeg) & 1) * XS;
        // [A] p, the v.p partials and the pivot row.  v_k[li] of other threads' rows: from LDS in the
        // first step, afterwards re-formed from rb (the previous pivot row) -- its vb copy is written
        // without a barrier before this point
        double pv = 0.0;
#pragma unroll
        for (int q = 0; q < RPL; ++q) {
            const double tot = group_sum<LPR>(s[q]);
            const int li = lrow(q);
            const double p = (li < t && li > l1 - 1) ? tau * tot : 0.0;  // rows > k
            const int lc = li < kEigMaxN ? li : 0;
            double vli;
            if (k == kbeg) {  // (uniform branch)
                vli = vc[lc];
            } else {  // the LDS read is unconditional (a select around it became a branch + wait)
                vli = fma(rv[lc], scal, li == l1 ? 1.0 : 0.0);
            }
            pv += vli * p;
            if (c == 0 && li < t) {
                if constexpr (NW == 1) ps[li] = p;
                else st_wt(xp + wg * RPW + (li - wg) / NW, p);
            }
        }
        // wave partial of v.p over the group leaders (fixed order: identical on every member)
        pv = wave_total(c == 0 ? pv : 0.0);
        if (lane == 0) {
            if constexpr (NW == 1) vpw[w] = pv;
            else st_wt(xp + NW * RPW + wg * 8 + w, pv);
        }
        if (l1 % NW == wg) {
            const int li1 = l1 / NW;
            const int q1 = li1 / (8 * G), rem = li1 % (8 * G);
            if (w == rem / G && g == rem % G) {
#pragma unroll
                for (int q = 0; q < RPL; ++q)
                    if (q == q1) {
#pragma unroll
                        for (int u = 0; u < CPL; ++u) {
                            const int j = c + LPR * u;
                            if (j < t) {
                                if constexpr (NW == 1) rs[j] = a[q][u];
                                else st_wt(xp + NW * RPW + 8 * NW + j, a[q][u]);
                            }
                        }
                    }
            }
        }
        TRI_TS(0);
        // [B] the hand-off; thread j takes p_j and the pivot row's entry j
        double pj = 0.0, rj = 0.0, pl1, kk = 0.0;
        const int j = tid;  // t <= 512 = kEigThreads
        if constexpr (NW > 1) {
            if (!tri_barrier(sync, (unsigned)NW * (unsigned)(k - kbeg + 1), k == abort_at && wg == 0)) {
                if (tid == 0) info[2] = 1;
                return;
            }
            if (j < t) {
                pj = ld_wt(xp + (j % NW) * RPW + j / NW);
                rj = ld_wt(xp + NW * RPW + 8 * NW + j);
            }
            pl1 = ld_wt(xp + (l1 % NW) * RPW + l1 / NW);
#pragma unroll
            for (int q = 0; q < 8 * NW; q += 64) kk += lane + q < 8 * NW ? ld_wt(xp + NW * RPW + lane + q) : 0.0;
            kk = wave_total(kk);  // the same order in every wave and member
        } else {
            __syncthreads();
            if (j < t) {
                pj = ps[j];
                rj = rs[j];
            }
            pl1 = ps[l1];
#pragma unroll
            for (int q = 0; q < 8; ++q) kk += vpw[q];
        }
        TRI_TS(1);
        // [C] K, w, the pivot row of A_{k+1} (into rb), |row[k+3 ..]|^2
        const double K = 0.5 * tau * kk;
        const double wk1 = pl1 - K;  // v_k[k+1] = 1
        double xq;
        {
            const double vj = vc[j];
            const double wjv = j < t ? pj - K * vj : 0.0;
            ws[j] = wjv;
            double rn = rj - wjv - wk1 * vj;
            rn = (j >= l1 && j < t) ? rn : 0.0;
            const double rt = j > l1 + 1 ? rn : 0.0;
            xq = rt * rt;
            rb[j] = rn;
            rv[j] = rt;
        }
        xq = wave_total(xq);
        if (lane == 0) red[w] = xq;
        __syncthreads();
        TRI_TS(2);
        // [E] the next reflector (every thread; v_{k+1} is formed where it is used)
        double taun = 0.0;
        const bool more = k + 1 <= n - 3;
        {
            double xn2 = 0.0;
#pragma unroll
            for (int q = 0; q < 8; ++q) xn2 += red[q];
            const double a0 = rb[l1 + 1];
            double beta = a0;
            scal = 0.0;
            if (more && xn2 != 0.0) {
                const double x2 = a0 * a0 + xn2;
                const double nr = x2 * rsqrt_f64(x2);
                beta = a0 >= 0.0 ? -nr : nr;
                taun = (beta - a0) * rcp_f64(beta);
                scal = rcp_f64(a0 - beta);
            }
            if (wg == 0 && tid == 0) {
                if (more) {
                    dvec[k + 1] = rb[l1];
                    evec[k + 1] = beta;
                    taus[k + 1] = taun;
                } else {
                    dvec[n - 2] = rb[l1];
                    evec[n - 2] = rb[l1 + 1];
                }
            }
        }
        const double one = more ? 1.0 : 0.0;
        auto vnext = [&](int jj) -> double {  // v_{k+1}[jj] (scal = 0 when !more); the read is unconditional
            return fma(rv[jj], scal, jj == l1 + 1 ? one : 0.0);
        };
        {
            const double v = vnext(j);
            vn[j] = v;  // own entry: read back by this thread only until the next barrier
            if (more && wg == 0 && j < t) Y[(int64_t)(k + 1) * ldy + off + j] = v;
        }
        // [D] A_{k+1} = A_k - v w^T - w v^T on the registers, and the next partial products; column
        // groups of 4 whose columns are all <= k + 1 (dead from here on) are skipped (a scalar
        // branch).  Dead rows are updated too: v and w vanish there (v_k[i] = p_i = 0 for i <= k),
        // so the update leaves them exactly as they are -- cheaper than per-element predication.
        // The LDS reads are unconditional (v, w, rv are 0 past t), and a compiler memory barrier
        // between column groups keeps their reads from being hoisted together (that spilled).
        double vi[RPL], wi[RPL];
#pragma unroll
        for (int q = 0; q < RPL; ++q) {
            const int li = lrow(q);  // < RPL 8 G NW <= kEigMaxN
            vi[q] = vc[li];
            wi[q] = ws[li];
            s[q] = 0.0;
        }
        // Row slots die in order: slot q holds local rows [8 G NW q, 8 G NW (q + 1)), all dead (< l1)
        // once 8 G NW (q + 1) <= l1 -- the same for every thread and member.  The loop runs from the
        // first live slot Q0 (one instantiation per Q0: no per-row branches); a dead row is never read
        // again (p is masked there, the pivot row and the dump take live rows), and its s stays 0.
        auto update = [&](auto q0c) {
            constexpr int Q0 = decltype(q0c)::value;
#pragma unroll
            for (int u0 = 0; u0 < CPL; u0 += 4) {
                const int u1 = u0 + 4 < CPL ? u0 + 4 : CPL;
                if (LPR * (u1 - 1) + LPR - 1 > l1) {
#pragma unroll
                    for (int u = u0; u < u1; ++u) {
                        const int jj = c + LPR * u;
                        const double wj = ws[jj], vj = vc[jj], vnj = vnext(jj);
#pragma unroll
                        for (int q = Q0; q < RPL; ++q) {
                            a[q][u] -= vi[q] * wj + wi[q] * vj;
                            s[q] += a[q][u] * vnj;
                        }
                    }
                }
                asm volatile("" ::: "memory");
            }
        };
        // (the three-slot phase-2 shape keeps the one instantiation: a second one spilled it)
        const int q0 = (noskip || RPL > 2) ? 0 : l1 / (8 * G * NW);  // first slot with a live row
        if (RPL > 2 || q0 <= 0) update(std::integral_constant<int, 0>{});
        else if constexpr (RPL > 1) {
            if (q0 == 1) update(std::integral_constant<int, 1>{});
        }
        if (k == n - 3) {  // the last diagonal entry, from its owner
#pragma unroll
            for (int q = 0; q < RPL; ++q)
                if (lrow(q) == t - 1) {
#pragma unroll
                    for (int u = 0; u < CPL; ++u)
                        if (c + LPR * u == t - 1) dvec[n - 1] = a[q][u];
                }
        }
        TRI_TS(3);
        tau = taun;
        cur ^= 1;
    }
    TRI_DONE();
    if (kend < n - 2) {  // phase 1 ends: the trailing block of A_kend (rows / columns >= kend + 1)
        const int o2 = kend + 1 - off;
#pragma unroll
        for (int q = 0; q < RPL; ++q) {
            const int li = lrow(q);
            if (li >= o2 && li < t) {
#pragma unroll
                for (int u = 0; u < CPL; ++u) {
                    const int j = c + LPR * u;
                    if (j >= o2 && j < t) dump[(int64_t)(li - o2) * lds + (j - o2)] = a[q][u];
                }
            }
        }
    }
}

// Number of eigenvalues of T (d, e2 = e^2, both LDS) below x: sign changes of the leading principal
// minors p_i = (d_i - x) p_{i-1} - e2_{i-1} p_{i-2} (Sturm sequence; an exact zero counts as a change),
// with a power-of-two rescale every 8 steps (the ratios -- all the count uses -- are unchanged).
// The chain is one dependent FMA per step; the LDS operands of the next 8 steps are read into
// registers (ds_read_b128 pairs) while the current 8 run, so no step waits on an LDS round trip.
// d[i] = kSturmPadD and e2[i - 1] = kE2Min for n <= i < n + 16 (padding steps that leave the count
// unchanged: the loop runs whole chunks of 8 without a per-step bound test).
__device__ __forceinline__ int sturm_count(const double* d, const double* e2, int n, double x) {
    double p0 = 1.0, p1 = d[0] - x;
    if (p1 == 0.0) p1 = -1e-300;
    int c = p1 < 0.0;
    // chunk i0 = 1 + 8 q covers steps i0 .. i0 + 7 (d[i], e2[i - 1])
    double dn[8], en[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
        dn[u] = d[1 + u];
        en[u] = e2[u];
    }
    for (int i0 = 1; i0 < n; i0 += 8) {
        double dc[8], ec[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            dc[u] = dn[u] - x;
            ec[u] = en[u];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            dn[u] = d[i0 + 8 + u];
            en[u] = e2[i0 + 7 + u];
        }
        // (whole chunks: the steps past n - 1 are padding, d = kSturmPadD and e2 = kE2Min, which
        // keep the sign -- (kSturmPadD - x) > 2 for the scaled |x| <= 1.01 -- and so the count)
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            // no zero guard on the chain (it was a compare and two selects per step): an exact
            // p_i = 0 reads as positive, and p_{i+1} = -e2_i p_{i-1} then has the sign the guard's
            // +-tiny p_i would have led to, so the count over (p_{i-1}, p_i, p_{i+1}) is the same;
            // e2 has no exact zeros (clamped to kE2Min below), so p_{i+1} != 0
            const double p2 = fma(dc[u], p1, -ec[u] * p0);
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
    __shared__ double d[kEigMaxN + 16], e2[kEigMaxN + 16];  // + the prefetch overrun of sturm_count
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
    for (int i = tid; i < kEigMaxN + 16; i += 256) {
        d[i] = i < n ? dg[i] * inv : kSturmPadD;
        const double es = i + 1 < n ? eg[i] * inv : 0.0;
        e2[i] = fmax(es * es, kE2Min);  // a split (e = 0) couples at 1e-300: |dlambda| <= 1e-150
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
// LAPACK dlagtf; |u_ii| below eps |T| is replaced by +-eps |T|) and runs two solves from a
// pseudo-random start -- the first forward elimination fused into the factorisation, the second
// solve rescaled by the first's largest entry -- and writes the unit vector to row-major Z
// (Z[i][k], ld ldz).  Scratch: six n x ldz arrays laid out [i][k] (a wave's 64 vectors read and
// write 512 contiguous bytes per step).  Stores and loads share vmcnt, so a load issued after a
// store waits for it: the solve loops read the operands of the NEXT 8 steps before storing the
// current 8, and the factorisation's multipliers come from a Newton reciprocal, not a division.

constexpr int kInvitSets = 4;  // register sets of the solves' operand ring (3 chunks of 8 steps ahead)

__global__ __launch_bounds__(64) void tridiag_invit_kernel(const double* __restrict__ dg, const double* __restrict__ eg,
                                                           const double* __restrict__ lam, const double* __restrict__ tnorm,
                                                           int n, int ldz, double* __restrict__ Z,
                                                           double* __restrict__ scr) {
    // T's diagonal and off-diagonal in LDS: the factorisation reads d[i + 1], e[i], e[i + 1] every
    // step, and from global memory each step's loads sat on an L2 round trip
    __shared__ double sdg[kEigMaxN], seg[kEigMaxN];
    for (int i = threadIdx.x; i < n; i += 64) {
        sdg[i] = dg[i];
        seg[i] = i < n - 1 ? eg[i] : 0.0;
    }
    __syncthreads();
    const int k = blockIdx.x * 64 + threadIdx.x;
    if (k >= n) return;
    const int64_t S = (int64_t)n * ldz;
    double* __restrict__ U0i = scr;
    double* __restrict__ U1 = scr + S;
    double* __restrict__ U2 = scr + 2 * S;
    double* __restrict__ Lm = scr + 3 * S;
    double* __restrict__ Pv = scr + 4 * S;
    double* __restrict__ X = scr + 5 * S;
    auto at = [&](int i) { return (int64_t)i * ldz + k; };
    const double lk = lam[k];
    const double tol = kEpsE * fmax(tnorm[0], 1e-300);
    auto pivot_inv = [&](double u) {
        if (fabs(u) < tol) u = u < 0.0 ? -tol : tol;
        return 1.0 / u;
    };
    auto rnd = [&](int i) { return unit_hash(((uint64_t)k << 32) ^ (uint64_t)i ^ 0x5EED5EEDull); };
    INV_INIT();
    // pass 1: factor, forward elimination of the random right-hand side on the fly (y into X)
    double cd = sdg[0] - lk, cu = n > 1 ? seg[0] : 0.0, yc = rnd(0);
#pragma unroll 4
    for (int i = 0; i < n - 1; ++i) {
        const double bi = seg[i], an = sdg[i + 1] - lk, cn = i + 1 < n - 1 ? seg[i + 1] : 0.0, yn = rnd(i + 1);
        const bool piv = fabs(bi) > fabs(cd);
        const double m = piv ? cd * rcp_f64(bi) : (cd != 0.0 ? bi * rcp_f64(cd) : 0.0);
        U0i[at(i)] = pivot_inv(piv ? bi : cd);
        U1[at(i)] = piv ? an : cu;
        U2[at(i)] = piv ? cn : 0.0;
        Lm[at(i)] = m;
        Pv[at(i)] = piv ? 1.0 : 0.0;
        X[at(i)] = piv ? yn : yc;
        const double ycn = piv ? yc - m * yn : yn - m * yc;
        const double cdn = piv ? cu - m * an : an - m * cu;
        cu = piv ? -m * cn : cn;
        cd = cdn;
        yc = ycn;
    }
    U0i[at(n - 1)] = pivot_inv(cd);
    INV_TS(4);
    X[at(n - 1)] = yc;
    // back substitution U z = y (z into X): max |z| and sum z^2.  The operands are read in chunks of
    // 8 steps through a ring of kInvitSets register sets, kInvitSets - 1 chunks ahead of the chunk being
    // solved (one chunk ahead left one memory round trip exposed per 8 steps -- the solves were
    // latency-bound).  Only whole chunks go through the ring, with unpredicated loads (a chunk past
    // the end reads clamped rows it never uses): per-element guards there turned every chunk into
    // branches and full vmcnt drains.  The last n % 8 steps run on their own; the arithmetic is
    // unchanged, step by step.
    constexpr int NS = kInvitSets;
    auto back = [&](double& norm2) {
        double z1 = 0.0, z2 = 0.0, zmax = 0.0, nn = 0.0;
        double xr[NS][8], u1r[NS][8], u2r[NS][8], uir[NS][8];
        const int nfull = n / 8;  // whole chunks; chunk c: rows n - 1 - 8 c down to n - 8 - 8 c
        auto load = [&](int c, auto sc) {
            constexpr int st = decltype(sc)::value;
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int i = max(n - 1 - 8 * c - u, 0);
                xr[st][u] = X[at(i)];
                u1r[st][u] = U1[at(i)];
                u2r[st][u] = U2[at(i)];
                uir[st][u] = U0i[at(i)];
            }
        };
        auto step = [&](int i, double x, double u1, double u2, double ui) {
            const double z = (x - u1 * z1 - u2 * z2) * ui;
            X[at(i)] = z;
            zmax = fmax(zmax, fabs(z));
            nn += z * z;
            z2 = z1;
            z1 = z;
        };
        auto chunk = [&](int c, auto sc) {
            constexpr int st = decltype(sc)::value;
            load(c + NS - 1, std::integral_constant<int, (st + NS - 1) % NS>{});
            const int i0 = n - 1 - 8 * c;
#pragma unroll
            for (int u = 0; u < 8; ++u) step(i0 - u, xr[st][u], u1r[st][u], u2r[st][u], uir[st][u]);
        };
        load(0, std::integral_constant<int, 0>{});
        load(1, std::integral_constant<int, 1>{});
        load(2, std::integral_constant<int, 2>{});
        int c = 0;
        for (; c + NS <= nfull; c += NS) {
            chunk(c, std::integral_constant<int, 0>{});
            chunk(c + 1, std::integral_constant<int, 1>{});
            chunk(c + 2, std::integral_constant<int, 2>{});
            chunk(c + 3, std::integral_constant<int, 3>{});
        }
        if (c < nfull) chunk(c++, std::integral_constant<int, 0>{});
        if (c < nfull) chunk(c++, std::integral_constant<int, 1>{});
        if (c < nfull) chunk(c++, std::integral_constant<int, 2>{});
        for (int i = n - 1 - 8 * c; i >= 0; --i) step(i, X[at(i)], U1[at(i)], U2[at(i)], U0i[at(i)]);
        norm2 = nn;
        return zmax;
    };
    double nn;
    const double zmax = back(nn);
    INV_TS(5);
    // pass 3: forward elimination of sc x (in place), sc = 1 / max |x| (the same ring, whole chunks)
    const double sc = zmax > 0.0 ? 1.0 / zmax : 1.0;
    if (n > 1) {
        double ycur = X[at(0)] * sc;
        double xr[NS][8], lr[NS][8], pr[NS][8];
        const int nfull = (n - 1) / 8;  // whole chunks; chunk c: steps i = 8 c .. 8 c + 7 (i < n - 1)
        auto load = [&](int c, auto sc_) {
            constexpr int st = decltype(sc_)::value;
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int i = min(8 * c + u, n - 2);
                xr[st][u] = X[at(i + 1)];
                lr[st][u] = Lm[at(i)];
                pr[st][u] = Pv[at(i)];
            }
        };
        auto step = [&](int i, double x, double l, double p) {
            const double yn = x * sc;
            const bool pv = p != 0.0;
            X[at(i)] = pv ? yn : ycur;
            ycur = pv ? ycur - l * yn : yn - l * ycur;
        };
        auto chunk = [&](int c, auto sc_) {
            constexpr int st = decltype(sc_)::value;
            load(c + NS - 1, std::integral_constant<int, (st + NS - 1) % NS>{});
#pragma unroll
            for (int u = 0; u < 8; ++u) step(8 * c + u, xr[st][u], lr[st][u], pr[st][u]);
        };
        load(0, std::integral_constant<int, 0>{});
        load(1, std::integral_constant<int, 1>{});
        load(2, std::integral_constant<int, 2>{});
        int c = 0;
        for (; c + NS <= nfull; c += NS) {
            chunk(c, std::integral_constant<int, 0>{});
            chunk(c + 1, std::integral_constant<int, 1>{});
            chunk(c + 2, std::integral_constant<int, 2>{});
            chunk(c + 3, std::integral_constant<int, 3>{});
        }
        if (c < nfull) chunk(c++, std::integral_constant<int, 0>{});
        if (c < nfull) chunk(c++, std::integral_constant<int, 1>{});
        if (c < nfull) chunk(c++, std::integral_constant<int, 2>{});
        for (int i = 8 * c; i < n - 1; ++i) step(i, X[at(i + 1)], Lm[at(i)], Pv[at(i)]);
        X[at(n - 1)] = ycur;
    } else {
        X[at(0)] = X[at(0)] * sc;
    }
    INV_TS(6);
    back(nn);
    INV_TS(7);
    const double f = nn > 0.0 ? 1.0 / sqrt(nn) : 0.0;
    for (int i = 0; i < n; i += 8) {
        double xv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u)
            if (i + u < n) xv[u] = X[at(i + u)];
#pragma unroll
        for (int u = 0; u < 8; ++u)
            if (i + u < n) Z[at(i + u)] = xv[u] * f;
    }
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

constexpr int kWY = 32;     // reflectors per compact-WY block
constexpr int kWYRows = 128;  // Y rows staged in LDS per chunk

// Y rows [r0, r0 + kWYRows) of the block's 32 reflector columns (column-major Y, ld) -> Ys[row][refl]
// (pitch 33), zero past n / nref; 16 values per thread, consecutive threads along the rows.
__device__ __forceinline__ void wy_stage(const double* __restrict__ Y, int ld, int n, int nref, int k0, int r0,
                                         double (&v)[kWYRows * kWY / 256]) {
#pragma unroll
    for (int q = 0; q < kWYRows * kWY / 256; ++q) {
        const int e = threadIdx.x + 256 * q, rr = e % kWYRows, c = e / kWYRows;
        const int row = r0 + rr;
        v[q] = (row < n && k0 + c < nref) ? Y[(int64_t)(k0 + c) * ld + row] : 0.0;
    }
}
__device__ __forceinline__ void wy_put(double* Ys, const double (&v)[kWYRows * kWY / 256]) {
#pragma unroll
    for (int q = 0; q < kWYRows * kWY / 256; ++q) {
        const int e = threadIdx.x + 256 * q, rr = e % kWYRows, c = e / kWYRows;
        Ys[rr * (kWY + 1) + c] = v[q];
    }
}

// T_b of block b (reflectors 32 b .. 32 b + 31; tau = 0 past the last one): the upper triangular
// factor of H_{32b} ... H_{32b+31} = I - Y_b T_b Y_b^T (LAPACK dlarft, forward, columnwise).  The
// Gram Y_b^T Y_b over coalesced 128-row chunks staged in LDS.
__global__ __launch_bounds__(256) void wy_t_kernel(const double* __restrict__ Y, int ld, int n, int nref,
                                                   const double* __restrict__ taus, double* __restrict__ Tg) {
    __shared__ double Ys[kWYRows * (kWY + 1)];
    __shared__ double Sg[kWY][kWY + 1], T[kWY][kWY + 1];
    const int b = blockIdx.x, tid = threadIdx.x;
    const int k0 = kWY * b;
    double acc[4] = {0.0, 0.0, 0.0, 0.0};
    double v[kWYRows * kWY / 256];
    for (int r0 = k0 + 1; r0 < n; r0 += kWYRows) {
        wy_stage(Y, ld, n, nref, k0, r0, v);
        __syncthreads();
        wy_put(Ys, v);
        __syncthreads();
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int e = tid + 256 * q, pp = e / kWY, qq = e % kWY;
            if (pp <= qq) {
                double a = 0.0;
                for (int rr = 0; rr < kWYRows; ++rr) a += Ys[rr * (kWY + 1) + pp] * Ys[rr * (kWY + 1) + qq];
                acc[q] += a;
            }
        }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int e = tid + 256 * q;
        Sg[e / kWY][e % kWY] = acc[q];
        T[e / kWY][e % kWY] = 0.0;
    }
    __syncthreads();
    if (tid == 0) T[0][0] = k0 < nref ? taus[k0] : 0.0;
    __syncthreads();
    for (int i = 1; i < kWY; ++i) {
        const double ti = k0 + i < nref ? taus[k0 + i] : 0.0;
        double a = 0.0;
        if (tid < i) {
            for (int q = tid; q < i; ++q) a += T[tid][q] * Sg[q][i];
        }
        __syncthreads();
        if (tid < i) T[tid][i] = -ti * a;
        if (tid == i) T[i][i] = ti;
        __syncthreads();
    }
    for (int e = tid; e < kWY * kWY; e += 256) Tg[(int64_t)b * kWY * kWY + e] = T[e / kWY][e % kWY];
}

// V = Q_H Z for one 16-column block of the row-major Z (ld ldz), held in LDS: blocks of 32
// reflectors from the last to the first, Z <- Z - Y_b (T_b (Y_b^T Z)) on the fp64 MFMA, Y_b staged
// through LDS in 128-row chunks; then V into the column-major Vout (ld ldv; rows >= n written as
// zero).  A whole Y block (rows k0 + 1 .. n - 1, up to kWYCh chunks) lives in registers; both
// passes over it (Y_b^T Z, then Z -= Y_b M2) put its chunks from there, and pass 2 refills each
// chunk's registers with the next block's chunk as soon as it has been put, so the loads of block
// b - 1 (and its T) fly while block b finishes (round 5: one chunk ahead left a round trip
// exposed per chunk and pass -- 223 us at n = 512; a second register block spilled to AGPRs and
// drained every load).  Same operations in the same order: bit-identical.
constexpr int kWYCh = kEigMaxN / kWYRows;  // Y chunks per block, at most
__global__ __launch_bounds__(256) void wy_apply_kernel(const double* __restrict__ Y, int ld, int n, int nref,
                                                       const double* __restrict__ Tg, const double* __restrict__ Z,
                                                       int ldz, double* __restrict__ Vout, int ldv) {
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    constexpr int ZP = 17, YP = kWY + 1, NV = kWYRows * kWY / 256;
    double* Zs = reinterpret_cast<double*>(smem_raw);  // [n][17]
    __shared__ double Ys[kWYRows * YP];
    __shared__ double Ms[2][kWY][17];
    __shared__ double Ts[kWY][kWY + 1];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int r = lane & 15, h = lane >> 4;
    const int c0 = 16 * blockIdx.x;
    for (int e = tid; e < n * 16; e += 256) {
        const int i = e >> 4, c = e & 15;
        Zs[i * ZP + c] = c0 + c < n ? Z[(int64_t)i * ldz + c0 + c] : 0.0;
    }
    const int nb = (nref + kWY - 1) / kWY;
    double ya[kWYCh][NV];
    // unpredicated loads: every load is issued before its first use, so the waits count them
    // (loads under a branch made the compiler drain vmcnt(0) after each one).  Rows past n read row
    // n - 1 scaled by 0.0 (Y is finite); columns nref .. 32 nb - 1 < LP are zero in Y (tri_zero)
    auto load_chunk = [&](int b, int c, double (&yc)[NV]) {
        const int k0 = kWY * b, j0 = k0 + 1;
#pragma unroll
        for (int q = 0; q < NV; ++q) {
            const int e = tid + 256 * q, rr = e % kWYRows, cc = e / kWYRows;
            const int row = j0 + kWYRows * c + rr;
            const double x = Y[(int64_t)(k0 + cc) * ld + (row < n ? row : n - 1)];
            yc[q] = x * (row < n ? 1.0 : 0.0);
        }
    };
    double tsv[kWY * kWY / 256];
    auto load_t = [&](int b) {
#pragma unroll
        for (int q = 0; q < kWY * kWY / 256; ++q) tsv[q] = Tg[(int64_t)b * kWY * kWY + tid + 256 * q];
    };
    // block b from ya (loaded while block b + 1 was applied); ya is refilled with block max(b - 1, 0)
    // chunk by chunk as pass 2 releases it, and tsv with its T
    auto apply_blk = [&](int b) {
        const int k0 = kWY * b;
        const int j0 = k0 + 1;  // first row any reflector of the block touches
        const int bn = b > 0 ? b - 1 : 0;
#pragma unroll
        for (int q = 0; q < kWY * kWY / 256; ++q) {
            const int e = tid + 256 * q;
            Ts[e / kWY][e % kWY] = tsv[q];
        }
        // M = Y_b^T Z (32 x 16): per chunk, wave w -> reflector tile (w & 1), chunk rows half (w >> 1)
        f64x4 acc = MD::zero();
        const int rt = w & 1, half = w >> 1;
#pragma unroll
        for (int c = 0; c < kWYCh; ++c) {
            const int r0 = j0 + kWYRows * c;
            if (r0 < n) {
                __syncthreads();
                wy_put(Ys, ya[c]);
                __syncthreads();
#pragma unroll 4
                for (int j = 64 * half; j < 64 * half + 64; j += 4) {
                    const int row = r0 + j + h;
                    const double av = Ys[(j + h) * YP + 16 * rt + r];
                    const double bv = row < n ? Zs[row * ZP + r] : 0.0;
                    acc = MD::mma(av, bv, acc);
                }
            }
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) Ms[half][16 * rt + MD::row(h, q)][r] = acc[q];
        __syncthreads();
        // M2 = T_b M (upper triangular T), into Ms[0].  The sum runs over all 32 p, the terms below
        // the diagonal skipped by a select (the same terms in the same order), so the loop unrolls
        // and its LDS reads pipeline (the triangular bound left an LDS round trip per term exposed)
        double m2[2];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int e = tid + 256 * q, rr = e >> 4, cc = e & 15;
            double a = 0.0;
#pragma unroll
            for (int p = 0; p < kWY; ++p) {
                const double t = Ts[rr][p], mm = Ms[0][p][cc] + Ms[1][p][cc];
                a = p >= rr ? a + t * mm : a;
            }
            m2[q] = a;
        }
        __syncthreads();
        load_t(bn);
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const int e = tid + 256 * q;
            Ms[0][e >> 4][e & 15] = m2[q];
        }
        // Z -= Y_b M2: per chunk, wave w -> 16-row tiles w, w + 4 of the 128 chunk rows
#pragma unroll
        for (int c = 0; c < kWYCh; ++c) {
            const int r0 = j0 + kWYRows * c;
            if (r0 < n) {
                __syncthreads();
                wy_put(Ys, ya[c]);
                __syncthreads();
            }
            load_chunk(bn, c, ya[c]);  // (the put above has read ya[c])
            if (r0 < n) {
#pragma unroll
                for (int t = 0; t < 2; ++t) {
                    const int tr = 16 * (w + 4 * t);
                    f64x4 a = MD::zero();
#pragma unroll
                    for (int s = 0; s < kWY / 4; ++s) a = MD::mma(Ys[(tr + r) * YP + 4 * s + h], Ms[0][4 * s + h][r], a);
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const int row = r0 + tr + MD::row(h, q);
                        if (row < n) Zs[row * ZP + r] -= a[q];
                    }
                }
            }
        }
        __syncthreads();
    };
    if (nb > 0) {
#pragma unroll
        for (int c = 0; c < kWYCh; ++c) load_chunk(nb - 1, c, ya[c]);
        load_t(nb - 1);
    }
    for (int b = nb - 1; b >= 0; --b) apply_blk(b);
    for (int c = 0; c < 16; ++c) {
        if (c0 + c >= n) break;
        for (int i = tid; i < ldv; i += 256) Vout[(int64_t)(c0 + c) * ldv + i] = i < n ? Zs[i * ZP + c] : 0.0;
    }
}

// C = alpha op(A) op(B) + beta C for the eigensolver's small fp64 products (column-major, M, N,
// K <= a few hundred): one workgroup per 16 x 16 tile of C (1024 at 512^2 -- gemm.hip's 64 x 64
// tiles gave 64 workgroups there and ran 55 / 100 us at 256^3 / 512^3).  Within a 16-deep k chunk
// the MFMA k order is k0 + 4 h + s (step s, lane half h): the A and B operands only have to agree on
// it, and then a transposed operand (op = T: contiguous along k) is read as 32-B runs per lane,
// a plain one (contiguous along i / j) as 128-B rows per 16 lanes.
// (Cin: the beta term's C when it is not the output, same ld -- C = alpha op(A) op(B) + beta Cin)
template <int TA, int TB>
__global__ __launch_bounds__(256) void sqgemm_f64_kernel(int M, int N, int K, double alpha, const double* __restrict__ A,
                                                         int lda, const double* __restrict__ B, int ldb, double beta,
                                                         double* C, int ldc, const double* Cin) {
    // round 6: four waves per tile, wave w taking every fourth 32-deep k chunk, the partial tiles summed
    // in wave order through LDS (the one-wave form walked K = 512 as 16 dependent L2 round trips: 23 us)
    __shared__ f64x4 part[3][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, r = lane & 15, h = lane >> 4;
    const int tm = (M + 15) / 16;
    const int bi = blockIdx.x % tm, bj = blockIdx.x / tm;
    const int i = 16 * bi + r, j = 16 * bj + r;
    const bool iv = i < M, jv = j < N;
    auto ld_a = [&](int k) -> double {  // op(A)(i, k)
        if (!iv || k >= K) return 0.0;
        return TA ? A[(int64_t)i * lda + k] : A[(int64_t)k * lda + i];
    };
    auto ld_b = [&](int k) -> double {  // op(B)(k, j)
        if (!jv || k >= K) return 0.0;
        return TB ? B[(int64_t)k * ldb + j] : B[(int64_t)j * ldb + k];
    };
    f64x4 acc0 = MD::zero(), acc1 = MD::zero();
    for (int k0 = 32 * w; k0 < K; k0 += 128) {
        double a[8], b[8];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            a[s] = ld_a(k0 + 4 * h + s);
            b[s] = ld_b(k0 + 4 * h + s);
            a[4 + s] = ld_a(k0 + 16 + 4 * h + s);
            b[4 + s] = ld_b(k0 + 16 + 4 * h + s);
        }
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            acc0 = MD::mma(a[s], b[s], acc0);
            acc1 = MD::mma(a[4 + s], b[4 + s], acc1);
        }
    }
    f64x4 t;
#pragma unroll
    for (int q = 0; q < 4; ++q) t[q] = acc0[q] + acc1[q];
    if (w > 0) part[w - 1][lane] = t;
    __syncthreads();
    if (w != 0) return;
#pragma unroll
    for (int q = 0; q < 4; ++q) t[q] = ((t[q] + part[0][lane][q]) + part[1][lane][q]) + part[2][lane][q];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int ii = 16 * bi + MD::row(h, q);
        if (ii < M && jv) {
            double* c = C + (int64_t)j * ldc + ii;
            const double v = alpha * t[q];
            *c = beta != 0.0 ? v + beta * (Cin ? Cin[(int64_t)j * ldc + ii] : *c) : v;
        }
    }
}

// Round 6: 32 x 32 tiles of C (2 x 2 MFMA tiles per wave), K split in four contiguous ranges over the
// waves, partials summed in wave order.  Per 16-deep chunk a wave issues 8 + 8 loads for 16 MFMAs
// (the 16 x 16 form: 8 + 8 for 4), a k-contiguous operand as 32-B vector loads; the L2 reads of A and
// B halve (each tile row / column is read by half as many workgroups).
template <int TA, int TB>
__global__ __launch_bounds__(256) void sqgemm2_f64_kernel(int M, int N, int K, double alpha,
                                                          const double* __restrict__ A, int lda,
                                                          const double* __restrict__ B, int ldb, double beta,
                                                          double* C, int ldc, const double* Cin) {
    __shared__ f64x4 part[3][4][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, r = lane & 15, h = lane >> 4;
    const int tm = (M + 31) / 32;
    const int i0 = 32 * (blockIdx.x % tm), j0 = 32 * (blockIdx.x / tm);
    const int kper = (K + 63) / 64 * 16;  // each wave's K range: a multiple of 16
    const int kb = w * kper, ke = min(K, kb + kper);
    // op(A)(i, k0 .. k0 + 3) and op(B)(k0 .. k0 + 3, j) (zero outside the matrix and the wave's range)
    auto ld_a4 = [&](int i, int k0, double (&v)[4]) {
        if (TA && i < M && k0 + 3 < ke && ((lda | k0) & 1) == 0) {
            const double2 x = *reinterpret_cast<const double2*>(A + (int64_t)i * lda + k0);
            const double2 y = *reinterpret_cast<const double2*>(A + (int64_t)i * lda + k0 + 2);
            v[0] = x.x; v[1] = x.y; v[2] = y.x; v[3] = y.y;
            return;
        }
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const int k = k0 + s;
            v[s] = (i < M && k < ke) ? (TA ? A[(int64_t)i * lda + k] : A[(int64_t)k * lda + i]) : 0.0;
        }
    };
    auto ld_b4 = [&](int j, int k0, double (&v)[4]) {
        if (!TB && j < N && k0 + 3 < ke && ((ldb | k0) & 1) == 0) {
            const double2 x = *reinterpret_cast<const double2*>(B + (int64_t)j * ldb + k0);
            const double2 y = *reinterpret_cast<const double2*>(B + (int64_t)j * ldb + k0 + 2);
            v[0] = x.x; v[1] = x.y; v[2] = y.x; v[3] = y.y;
            return;
        }
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const int k = k0 + s;
            v[s] = (j < N && k < ke) ? (TB ? B[(int64_t)k * ldb + j] : B[(int64_t)j * ldb + k]) : 0.0;
        }
    };
    f64x4 acc[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) acc[a][b] = MD::zero();
    // the next chunk's operands are loaded while this chunk's MFMAs run
    double av[2][4], bv[2][4];
    auto load = [&](int kc) {
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            ld_a4(i0 + 16 * t + r, kc + 4 * h, av[t]);
            ld_b4(j0 + 16 * t + r, kc + 4 * h, bv[t]);
        }
    };
    if (kb < ke) load(kb);
    for (int kc = kb; kc < ke; kc += 16) {
        double ac[2][4], bc[2][4];
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                ac[t][s] = av[t][s];
                bc[t][s] = bv[t][s];
            }
        if (kc + 16 < ke) load(kc + 16);
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
            for (int a = 0; a < 2; ++a)
#pragma unroll
                for (int b = 0; b < 2; ++b) acc[a][b] = MD::mma(ac[a][s], bc[b][s], acc[a][b]);
    }
    if (w > 0) {
#pragma unroll
        for (int t = 0; t < 4; ++t) part[w - 1][t][lane] = acc[t >> 1][t & 1];
    }
    __syncthreads();
    if (w != 0) return;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        f64x4 v = acc[t >> 1][t & 1];
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = ((v[q] + part[0][t][lane][q]) + part[1][t][lane][q]) + part[2][t][lane][q];
        const int j = j0 + 16 * (t & 1) + r;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int ii = i0 + 16 * (t >> 1) + MD::row(h, q);
            if (ii < M && j < N) {
                double* c = C + (int64_t)j * ldc + ii;
                const double x = alpha * v[q];
                *c = beta != 0.0 ? x + beta * (Cin ? Cin[(int64_t)j * ldc + ii] : *c) : x;
            }
        }
    }
}

hipError_t launch_sqgemm(int ta, int tb, int M, int N, int K, double alpha, const double* A, int lda, const double* B,
                         int ldb, double beta, double* C, int ldc, hipStream_t s, const double* Cin = nullptr) {
    // 32 x 32 tiles from 384 x 384 up (LP = 512: 23 -> 15 us per 512^3 product); below, the 16 x 16 tiles
    // keep more workgroups in flight (LP = 256: 6.2 us against 9.9 us on 64 tiles of 32 x 32)
    const bool big = M >= 384 && N >= 384;
    const dim3 grid(big ? ((M + 31) / 32) * ((N + 31) / 32) : ((M + 15) / 16) * ((N + 15) / 16));
#define SQG(X, Y)                                                                                                      \
    if (ta == X && tb == Y) {                                                                                          \
        if (big)                                                                                                       \
            hipLaunchKernelGGL((sqgemm2_f64_kernel<X, Y>), grid, dim3(256), 0, s, M, N, K, alpha, A, lda, B, ldb, beta, \
                               C, ldc, Cin);                                                                           \
        else                                                                                                           \
            hipLaunchKernelGGL((sqgemm_f64_kernel<X, Y>), grid, dim3(256), 0, s, M, N, K, alpha, A, lda, B, ldb, beta,  \
                               C, ldc, Cin);                                                                           \
        return hipGetLastError();                                                                                      \
    }
    SQG(0, 0) SQG(0, 1) SQG(1, 0) SQG(1, 1)
#undef SQG
    return hipErrorInvalidValue;
}

template <int RPL, int CPL, int LPR, int NW>
hipError_t launch_tridiag(const double* src, int lds, int n, int off, int kend, double* Y, int ldy, double* d, double* e,
                          double* taus, double* dump, double* xch, unsigned* sync, int* info, hipStream_t s) {
    static_assert(8 * (64 / LPR) * RPL * NW <= kEigMaxN && LPR * CPL <= kEigMaxN, "tridiag layout");
    static const int noskip = [] {  // RSVD_TRI_NOSKIP=1 (A/B): update the dead row slots too
        const char* v = std::getenv("RSVD_TRI_NOSKIP");
        return v ? std::atoi(v) : 0;
    }();
    // RSVD_TRI_FORCE_ABORT=k (fault injection, tests/test_gpu_eig.py): member 0 of the multi-workgroup
    // phase takes the hand-off's timeout branch at step k, as if a member had stalled -- the abort word,
    // the sticky timeout flag (rsvd_sync: RSVD_ERR_HIP) and every member's exit are exercised
    static const int abort_at = [] {
        const char* v = std::getenv("RSVD_TRI_FORCE_ABORT");
        return v ? std::atoi(v) : -1;
    }();
    return launch_coresident(tridiag_kernel<RPL, CPL, LPR, NW>, dim3(NW), dim3(kEigThreads), 0, s, src, lds, n, off,
                             kend, Y, ldy, d, e, taus, dump, xch, sync, info, noskip, abort_at);
}

constexpr int kTailRows = 192;  // phase 2 (one workgroup) takes the last kTailRows rows

// the tridiagonalisation's zeroed inputs in one launch: the reflector matrix Y (n1 doubles), tau (n2),
// the hand-off counter words (nw)
__global__ void tri_zero_kernel(double* __restrict__ Y, int64_t n1, double* __restrict__ taus, int n2,
                                unsigned* __restrict__ ctr, int nw) {
    const int64_t t0 = blockIdx.x * (int64_t)blockDim.x + threadIdx.x, st = (int64_t)gridDim.x * blockDim.x;
    for (int64_t e = t0; e < n1; e += st) Y[e] = 0.0;
    for (int64_t e = t0; e < n2; e += st) taus[e] = 0.0;
    for (int64_t e = t0; e < nw; e += st) ctr[e] = 0u;
}

}  // namespace

#ifdef RSVD_TRI_PROF
void tri_prof_read(long long* out) {
    (void)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_tri_prof), sizeof(long long) * 16);
    long long z[16] = {};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_tri_prof), z, sizeof(z));
}
#endif

// ---- G^-1/2 of a Gram near the identity (round 6; the deferred second CholeskyQR pass, wide.cpp) ----
// The second pass's Gram G = T1^T T1 of an already orthonormalised panel is I + E with |E|_F <~ 0.03
// (the split Gram's entry error times cond(P)^2, bounded by its fallback test).  Any M with
// (T1 M)^T (T1 M) = I serves the deferred algebra (it only needs span(T1 M) = span(T1)), and
// M = G^-1/2 = sum_k binom(-1/2, k) E^k converges fast there: to degree 8 the remainder is below
// 0.19 |E|^9 (2e-10 at |E|_F = 0.1, the cut-off).  Paterson-Stockmeyer on E, E^2, E^3:
//     M = B0 + E^3 (B1 + E^3 B2),   B_i = c_{3i} I + c_{3i+1} E + c_{3i+2} E^2
// -- four l^3 products on the MFMA and three element-wise passes, against the Cholesky factor's
// dependent pivot chain (C5: ~285 us per LP = 512 factor).  Past the cut-off (or a non-finite E)
// flags[1] is raised and the caller's predicated Cholesky factor runs instead.
constexpr double kIsqrtCut = 0.1;
constexpr double kIsqrtC[9] = {1.0,          -0.5,         0.375,         -0.3125,           0.2734375,
                               -0.24609375, 0.2255859375, -0.20947265625, 0.196380615234375};

// E = G - I on the l x l block, 0 outside, 256 entries per workgroup; part[b] = the block's sum of squares
__global__ __launch_bounds__(256) void isqrt_prep_kernel(const double* __restrict__ G, int l, int LP,
                                                         double* __restrict__ E, double* __restrict__ part) {
    __shared__ double red[4];
    const int64_t e = blockIdx.x * 256 + threadIdx.x;
    double v = 0.0;
    if (e < (int64_t)LP * LP) {
        const int i = (int)(e / LP), j = (int)(e - (int64_t)i * LP);
        v = (i < l && j < l) ? G[e] - (i == j ? 1.0 : 0.0) : 0.0;
        E[e] = v;
    }
    double ss = v * v;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) ss += __shfl_xor(ss, o);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ss;
    __syncthreads();
    if (threadIdx.x == 0) part[blockIdx.x] = ((red[0] + red[1]) + red[2]) + red[3];
}
// flags[0] = |E|_F <= cut (finite), flags[1] = !flags[0] from the nb block sums (fixed order)
__global__ __launch_bounds__(256) void isqrt_flags_kernel(const double* __restrict__ part, int nb,
                                                          int* __restrict__ flags, double cut) {
    __shared__ double red[4];
    double ss = 0.0;
    for (int b = threadIdx.x; b < nb; b += 256) ss += part[b];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) ss += __shfl_xor(ss, o);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ss;
    __syncthreads();
    if (threadIdx.x == 0) {
        const double t = ((red[0] + red[1]) + red[2]) + red[3];
        const int small = (t <= cut * cut) ? 1 : 0;  // NaN: not small
        flags[0] = small;
        flags[1] = 1 - small;
    }
}

// out = a I + b E + c E2 (+ X) on the l x l block; outside it the identity (`pad_id`) or 0
__global__ __launch_bounds__(256) void isqrt_poly_kernel(double* __restrict__ out, const double* __restrict__ E,
                                                         const double* __restrict__ E2, const double* __restrict__ X,
                                                         double a, double b, double c, int l, int LP, int pad_id,
                                                         const int* __restrict__ pred) {
    if (pred && *pred == 0) return;
    const int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (e >= (int64_t)LP * LP) return;
    const int i = (int)(e / LP), j = (int)(e - (int64_t)i * LP);
    double v;
    if (i < l && j < l) {
        v = fma(c, E2[e], fma(b, E[e], i == j ? a : 0.0));
        if (X) v += X[e];
    } else {
        v = (pad_id && i == j) ? 1.0 : 0.0;
    }
    out[e] = v;
}

// M = G^-1/2 into `out` (pred flags[0]); scratch: E, E2, E3, B, T (LP x LP each, T may be G itself once
// the caller's predicated fallback has read it).  The l x l products run on the sqgemm (column-major:
// every operand is a polynomial in the symmetric E, so the layout does not matter).
hipError_t launch_isqrt_near_identity(const double* G, int l, int LP, double* E, double* E2, double* E3, double* B,
                                      double* T, double* out, int* flags, hipStream_t s, bool prep_only,
                                      bool series_only) {
    hipError_t er;
    const dim3 grid((unsigned)(((int64_t)LP * LP + 255) / 256));
    if (!series_only) {  // (the block sums in E2, free until the series)
        hipLaunchKernelGGL(isqrt_prep_kernel, grid, dim3(256), 0, s, G, l, LP, E, E2);
        // RSVD_ISQRT_CUT (debugging, tests/test_gpu_switches.py): another cut-off; 0 sends every second pass
        // to the predicated Cholesky factor
        static const double cut = [] {
            const char* v = std::getenv("RSVD_ISQRT_CUT");
            return v ? std::atof(v) : kIsqrtCut;
        }();
        hipLaunchKernelGGL(isqrt_flags_kernel, dim3(1), dim3(256), 0, s, E2, (int)grid.x, flags, cut);
        if ((er = hipGetLastError()) != hipSuccess || prep_only) return er;
    }
    const double* c = kIsqrtC;
    if ((er = launch_sqgemm(0, 0, l, l, l, 1.0, E, LP, E, LP, 0.0, E2, LP, s)) != hipSuccess) return er;
    if ((er = launch_sqgemm(0, 0, l, l, l, 1.0, E2, LP, E, LP, 0.0, E3, LP, s)) != hipSuccess) return er;
    hipLaunchKernelGGL(isqrt_poly_kernel, grid, dim3(256), 0, s, B, E, E2, nullptr, c[6], c[7], c[8], l, LP, 0, nullptr);
    if ((er = launch_sqgemm(0, 0, l, l, l, 1.0, E3, LP, B, LP, 0.0, T, LP, s)) != hipSuccess) return er;
    hipLaunchKernelGGL(isqrt_poly_kernel, grid, dim3(256), 0, s, B, E, E2, T, c[3], c[4], c[5], l, LP, 0, nullptr);
    if ((er = launch_sqgemm(0, 0, l, l, l, 1.0, E3, LP, B, LP, 0.0, T, LP, s)) != hipSuccess) return er;
    hipLaunchKernelGGL(isqrt_poly_kernel, grid, dim3(256), 0, s, out, E, E2, T, c[0], c[1], c[2], l, LP, 1, flags);
    return hipGetLastError();
}

// Z = op(X) op(Y), n x n fp64 row-major (lds ldx / ldy / ldz): the column-major sqgemm on the
// transposed views (Z^T = op(Y)^T op(X)^T)
hipError_t launch_gemm_rm(int tx, int ty, int n, const double* X, int ldx, const double* Y, int ldy, double* Z, int ldz,
                          hipStream_t s) {
    return launch_sqgemm(ty, tx, n, n, n, 1.0, Y, ldy, X, ldx, 0.0, Z, ldz, s);
}

size_t eig_svd_ws_doubles(int LP) {
    const size_t L2 = (size_t)LP * LP;
    const size_t nb = (LP + kWY - 1) / kWY;
    // exchange: 2 parities x (p of n rows + 8 NW v.p partials + one row), NW <= 16
    return 9 * L2 + nb * kWY * kWY + 4 * (size_t)LP + 64 + 2 * (size_t)(2 * kEigMaxN + 8 * 16);
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
    if ((er = launch_sqgemm(1, 0, n, n, n, 1.0, R, LP, R, LP, 0.0, G, LP, s)) != hipSuccess) return er;
    // 2. tridiagonalisation
    hipLaunchKernelGGL(tri_zero_kernel, dim3((unsigned)std::min<size_t>((L2 + 255) / 256, 1024)), dim3(256), 0, s, Y,
                       (int64_t)L2, taus, LP, sync + kTriCtr, 2);
    if ((er = hipGetLastError()) != hipSuccess) return er;
    // the one-workgroup steps on a local block of n - off <= kTailRows rows: the three-slot shape while
    // more than 128 rows are active, then the two-slot shape <2, 16, 8, 1> on the last 128 (its steps
    // do 32 instead of 72 elements per thread: round 5, RSVD_TRI_SPLIT2=0 keeps one launch)
    static const bool split2 = [] {
        const char* v = std::getenv("RSVD_TRI_SPLIT2");
        return v ? std::atoi(v) != 0 : true;
    }();
    auto one_wg = [&](const double* src, int off) -> hipError_t {
        if (split2 && n - off > 128) {
            const int kend2 = n - 128 - 1;
            double* dump2 = scr + L2;  // (scr: free until the inverse iteration)
            hipError_t e2 = launch_tridiag<3, 24, 8, 1>(src, LP, n, off, kend2, Y, LP, d, e, taus, dump2, xch, sync,
                                                        info, s);
            if (e2 != hipSuccess) return e2;
            return launch_tridiag<2, 16, 8, 1>(dump2, LP, n, kend2 + 1, n - 2, Y, LP, d, e, taus, nullptr, xch, sync,
                                               info, s);
        }
        return launch_tridiag<3, 24, 8, 1>(src, LP, n, off, n - 2, Y, LP, d, e, taus, nullptr, xch, sync, info, s);
    };
    if (n <= 128) {
        er = launch_tridiag<2, 16, 8, 1>(G, LP, n, 0, n - 2, Y, LP, d, e, taus, nullptr, xch, sync, info, s);
    } else if (n <= kTailRows) {
        er = one_wg(G, 0);
    } else {
        // phase 1 on NW workgroups up to the step that leaves kTailRows trailing rows, phase 2 on one
        double* dump = scr;  // free until the inverse iteration
        const int kend = n - kTailRows - 1;
        if (n <= 256)
            er = launch_tridiag<2, 16, 16, 4>(G, LP, n, 0, kend, Y, LP, d, e, taus, dump, xch, sync, info, s);
        else
            er = launch_tridiag<2, 16, 32, 16>(G, LP, n, 0, kend, Y, LP, d, e, taus, dump, xch, sync, info, s);
        if (er != hipSuccess) return er;
        er = one_wg(dump, kend + 1);
    }
    if (er != hipSuccess) return er;
    // 3. eigenvalues (descending), 4. eigenvectors of T (row-major Z), cluster re-orthogonalisation
    hipLaunchKernelGGL(tridiag_bisect_kernel, dim3((n + 3) / 4), dim3(256), 0, s, d, e, n, lam, tnorm);
    hipLaunchKernelGGL(tridiag_invit_kernel, dim3((n + 63) / 64), dim3(64), 0, s, d, e, lam, tnorm, n, LP, Z, scr);
    hipLaunchKernelGGL(cluster_orth_kernel, dim3(1), dim3(1024), 0, s, lam, n, LP, Z);
    // one Newton-Schulz step: Z' = Z (3 I - Z^T Z) / 2.  Row-major Z read column-major (ld LP) is
    // Zc = Z^T, so M = Z^T Z = Zc Zc^T and Zc' = 1.5 Zc - 0.5 M Zc (M symmetric); Zc' into Z2 (scratch)
    double* M = scr;
    double* Z2 = scr + L2;
    if ((er = launch_sqgemm(0, 1, n, n, n, 1.0, Z, LP, Z, LP, 0.0, M, LP, s)) != hipSuccess) return er;
    if ((er = launch_sqgemm(0, 0, n, n, n, -0.5, M, LP, Z, LP, 1.5, Z2, LP, s, Z)) != hipSuccess) return er;
    Z = Z2;
    // 5. V_w = Q_H Z into J (buffer 0, column-major LP x LP; columns >= n zero)
    // (wy_apply writes every row of the n columns; only columns past n need the zeros)
    if (n < LP && (er = hipMemsetAsync(J, 0, L2 * sizeof(double), s)) != hipSuccess) return er;
    if (nref > 0) hipLaunchKernelGGL(wy_t_kernel, dim3((nref + kWY - 1) / kWY), dim3(256), 0, s, Y, LP, n, nref, taus, Tg);
    hipLaunchKernelGGL(wy_apply_kernel, dim3((n + 15) / 16), dim3(256), (size_t)n * 17 * sizeof(double), s, Y, LP, n,
                       nref, Tg, Z, LP, J, LP);
    if ((er = hipGetLastError()) != hipSuccess) return er;
    // 6. X = W V_w into X (buffer 0, column-major), then the checked block-Jacobi finish
    if (n < LP && (er = hipMemsetAsync(X, 0, L2 * sizeof(double), s)) != hipSuccess) return er;
    if ((er = launch_sqgemm(0, 0, n, n, n, 1.0, R, LP, J, LP, 0.0, X, LP, s)) != hipSuccess) return er;
    return launch_block_jacobi_given<T>(l, LP, X, J, Uw, Vw, S, sync, info, s, tol_chk);
}

template hipError_t launch_eig_svd<float>(const double*, int, int, double*, double*, double*, double*, double*, float*,
                                          unsigned*, int*, hipStream_t, double);
template hipError_t launch_eig_svd<double>(const double*, int, int, double*, double*, double*, double*, double*,
                                           double*, unsigned*, int*, hipStream_t, double);

}  // namespace rsvd
