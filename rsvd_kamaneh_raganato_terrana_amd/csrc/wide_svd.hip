// wide_svd.hip -- the small SVD of the rSVD for sketch widths 128..512 (SVD<Jacobi>::compute on B,
// include/SVD_class.hpp:100-180).
//
// As in jacobi.hip, W = R^T (R = Q_B^T B^T, so B = W Q_B^T) is diagonalised by one-sided
// (Hestenes) Jacobi: X = W, J = I, rotate column pairs until the columns of X are orthogonal;
// then S = column norms (descending, the reference's selection sort :164-178), U_w = X / S,
// V_w = J.  For l > 64 the l x l problem no longer fits one workgroup, so the columns are cut
// into NB = LP/16 blocks of 16 and paired round-robin (NB/2 disjoint block pairs per round,
// NB - 1 rounds per sweep) over a persistent grid of NB/2 workgroups:
//   1. Gp = X_pair^T X_pair (32 x 32, fp64 MFMA over the MR rows; exact column dot products, the
//      same quantities the one-sided rotation angles use);
//   2. the 32 x 32 symmetric eigenproblem of Gp by one cyclic Jacobi sweep in LDS (16 disjoint
//      rotations per inner round, accumulated into Jp) -- each inner rotation is the one-sided
//      rotation of the corresponding column pair of X, with the same angle formula as jacobi.hip;
//   3. X_pair <- X_pair Jp, J_pair <- J_pair Jp (fp64 MFMA), into the other half of a double
//      buffer (every column is owned by exactly one pair per round).
// (Measured and reverted, profiles/r03_bj_cross_deadend.txt: rotating only the 16 x 16 cross pairs
// per outer round plus one intra-block round per sweep -- half the inner rounds -- needs 1-2 sweeps
// more on clustered spectra and its inner round was no faster.  Also reverted, profiles/r03_bj_rowgroups.txt:
// one barrier per inner round with wave 7 deriving the next round's angles from the current Gram
// while the others rotate -- the look-ahead's 12 extra LDS reads and three 2 x 2 products made it
// the longer path, 0.93 vs 0.67 us per inner round.)
// Row groups: each block pair is served by G workgroups (G = 1, 2, 4), member g owning rows
// [g MR / G, (g + 1) MR / G) of X and [g LP / G, (g + 1) LP / G) of J.  The members publish their
// partial pair Grams, meet at a group barrier, sum the G partials in a fixed order and then run the
// SAME inner sweep on the same Gram (bit-identical Jp, no broadcast), each applying it to its own
// rows.  The staging, Gram and rotation traffic per workgroup shrink by G; the inner sweep is
// replicated.
// Rounds are separated by an agent-scope grid barrier (MI355X_MICROARCH.md "Workgroup dispatch
// ... inter-workgroup visibility": plain stores -> vmcnt(0) -> barrier -> release fence -> relaxed
// counter; acquire fence after the poll).  The grid (<= 64 workgroups at LP = 512) is launched
// cooperatively (launch_coresident): co-resident by the runtime's guarantee; every spin is still
// bounded and reports a timeout instead of hanging.
// Convergence: a sweep whose rotations all had cos^2 = g^2 / (ab) <= quad2 ends the iteration (the
// next would only square them); and when a sweep's largest pre-rotation cosine is <= 10 sqrt(tol_chk)
// (quadratic convergence: close to having squared below tol_chk), the whole grid checks max cos
// over ALL column pairs of the new X
// (an LP x LP fp64 MFMA Gram, every workgroup a 32-column slice) and stops at <= tol_chk -- which
// saves the confirming sweep the first rule needs.
#include <algorithm>
#include <cstdlib>

#include "common.hpp"
#include "kernels.hpp"
#include "wide.hpp"

namespace rsvd {

namespace {

typedef Mfma<double> MD;
constexpr double kEps = 2.220446049250313e-16;
constexpr int kMaxSweeps = 30;
// sync layout (unsigned words): [0] barrier counter, [1] abort, [2] final parity, [4 + s] sweep s
// rotated, [36 + s] sweep s had rotations outside the quadratic regime; u64 slots (8-B aligned):
// [80 + 2 s] sweep s's largest pre-rotation cos^2, [144 + 2 s] the global check's max cos^2 after it,
// [kGroupWord + pair] the row-group barrier counters (one per block pair, up to 128 pairs)
constexpr int kGroupWord = 256;
constexpr int kSyncWords = 384;
static_assert(kSyncWords <= kBJSyncWords, "block Jacobi sync words");

__device__ __forceinline__ void rr_pair(int round, int k, int N, int& p, int& q) {
    if (k == 0) {
        p = round;
        q = N - 1;
    } else {
        p = (round + k) % (N - 1);
        q = (round - k + (N - 1)) % (N - 1);
    }
}

// rr_pair for N = 32 without the modulo (round < 31, k < 16): the same pairs
__device__ __forceinline__ void rr_pair32(int round, int k, int& p, int& q) {
    int a = round + k, b = round - k;
    a = a >= 31 ? a - 31 : a;
    b = b < 0 ? b + 31 : b;
    p = k == 0 ? round : a;
    q = k == 0 ? 31 : b;
}

// Returns false on timeout (then every workgroup bails out through the abort word sync[1]).
// ctr: the arrival counter (sync[0] for the grid, a group word for a row group).
__device__ bool grid_barrier(unsigned* sync, unsigned target, unsigned* ctr = nullptr) {
    if (!ctr) ctr = sync;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    __shared__ int ok;
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        int good = 1;
        long spins = 0;
        while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
            __builtin_amdgcn_s_sleep(2);
            if ((++spins & 1023) == 0 &&
                (__hip_atomic_load(sync + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0 || spins > (1l << 26))) {
                __hip_atomic_store(sync + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                good = 0;
                break;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        ok = good;
    }
    __syncthreads();
    return ok != 0;
}

// The row-group hand-off of the partial pair Grams, fence-free (MI355X_MICROARCH.md, "Hand-offs
// measured with sc1 loads", first row): every byte stored `sc1` (st_wt) and loaded `sc1`
// (ld_wt), every storing wave's vmcnt(0) before the workgroup barrier, one lane's agent-scope add
// to the group counter, an `sc1` poll, then a workgroup barrier before any load.  No release /
// acquire fence: each costs ~1.7 us, and the group meets once per round.
__device__ bool group_barrier(unsigned* sync, unsigned* ctr, unsigned target) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    __shared__ int ok;
    if (threadIdx.x == 0) {
        __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        int good = 1;
        long spins = 0;
        while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
            __builtin_amdgcn_s_sleep(1);
            if ((++spins & 1023) == 0 &&
                (__hip_atomic_load(sync + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0 || spins > (1l << 26))) {
                __hip_atomic_store(sync + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                good = 0;
                break;
            }
        }
        ok = good;
    }
    __syncthreads();
    return ok != 0;
}

constexpr int GS = 33;  // LDS pitch of the 32 x 32 blocks

// Stores of the round's X / J columns and partial Grams: `sc1` (write-through; the line leaves the
// XCD's L2 clean).  The next reader of a column is almost always a workgroup on another XCD, so
// keeping the line in this L2 buys nothing, while a dirty line makes the agent release of the next
// barrier write it back on the critical path (MI355X_MICROARCH.md: 1.7 us clean vs 6.5 us with
// 16 KB dirty per block; a round dirtied 64 KB per workgroup at LP = 512).
__device__ __forceinline__ void st_wt(double* p, double v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_wt(double* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

// Full-precision fp64 reciprocal square root / reciprocal from the hardware estimates (two
// Newton steps each): the inner rotations need c^2 + s^2 = 1 to rounding, not IEEE division.
__device__ __forceinline__ double rsqrt_nr(double d) {
    double y = __builtin_amdgcn_rsq(d);
    y = y * (1.5 - 0.5 * d * y * y);
    return y * (1.5 - 0.5 * d * y * y);
}
__device__ __forceinline__ double rcp_nr(double d) {
    double y = __builtin_amdgcn_rcp(d);
    y = y * (2.0 - d * y);
    return y * (2.0 - d * y);
}

// Rotation of the pair (a = |x_p|^2, b = |x_q|^2, g = x_p.x_q): x_p' = c x_p - s x_q, x_q' = s x_p + c x_q
// zeroes the cross term (jacobi.hip formula: t = sign(d g) |2g| / (|d| + sqrt(d^2 + 4 g^2)), d = b - a,
// c = (1 + t^2)^-1/2, s = c t), evaluated on operands scaled by max(|d|, |2g|) (no overflow / underflow
// for any finite a, b, g)
__device__ __forceinline__ void pair_angle(const double* G, int p, int q, double tol2, double negl, double& c,
                                           double& s, bool& rot) {
    const double a = G[p * GS + p], b = G[q * GS + q], g = G[p * GS + q];
    rot = g != 0.0 && g * g > tol2 * a * b && a > negl && b > negl;
    const double d = b - a, g2 = 2.0 * g;
    const double inv = rcp_nr(fmax(fmax(fabs(d), fabs(g2)), 1e-300));
    const double ds = fabs(d) * inv, gs = fabs(g2) * inv;
    const double hyp2 = ds * ds + gs * gs;  // in [1, 2]
    const double tmag = gs * rcp_nr(ds + hyp2 * rsqrt_nr(hyp2));
    const double t = ((d >= 0.0) == (g >= 0.0)) ? tmag : -tmag;
    const double cc = rsqrt_nr(1.0 + t * t);
    c = rot ? cc : 1.0;
    s = rot ? cc * t : 0.0;
}

// The same rotation with a shorter dependent chain: the operands are scaled by the power of two of
// max(|d|, |2g|) (exact, v_ldexp) instead of a Newton reciprocal, and with u = ds + sqrt(ds^2 + gs^2)
// (so t = gs / u) the pair c = (1 + t^2)^-1/2, s = c t is c = u w, s = gs w with
// w = (u^2 + gs^2)^-1/2 -- one reciprocal square root instead of a reciprocal and a reciprocal square
// root.  c^2 + s^2 = 1 to rounding as before; the angle differs from pair_angle's in the last bits.
__device__ __forceinline__ void pair_angle_fast(const double* G, int p, int q, double tol2, double negl, double& c,
                                                double& s, bool& rot) {
    const double a = G[p * GS + p], b = G[q * GS + q], g = G[p * GS + q];
    rot = g != 0.0 && g * g > tol2 * a * b && a > negl && b > negl;
    const double d = b - a, g2 = 2.0 * g;
    const int e = __builtin_amdgcn_frexp_exp(fmax(fmax(fabs(d), fabs(g2)), 1e-300));
    const double ds = __builtin_ldexp(fabs(d), -e), gs = __builtin_ldexp(fabs(g2), -e);  // max in [0.5, 1)
    const double hyp2 = ds * ds + gs * gs;
    const double u = ds + hyp2 * rsqrt_nr(hyp2);
    const double w = rsqrt_nr(u * u + gs * gs);
    const double sg = ((d >= 0.0) == (g >= 0.0)) ? w : -w;
    c = rot ? u * w : 1.0;
    s = rot ? gs * sg : 0.0;
}

// rows: the rows one workgroup stages (MR / G)
size_t block_jacobi_lds(int rows) { return ((rows <= 512 ? (size_t)32 * (rows + 1) : 0) + 3 * 32 * GS) * sizeof(double); }

constexpr int kBJThreads = 512;  // 8 waves: 2 per SIMD for the MFMA phases

// One cyclic sweep of the 32 x 32 pair Gram (round-robin: 16 disjoint rotations per inner round,
// 31 rounds), ONE barrier per inner round: every thread derives the angle of its column pair k2
// itself (32 threads per pair, identical inputs, so identical c, s); thread (k, k2) < 256 takes
// the angle of its row pair k from a lane of its wave that computed it (a register shuffle) and
// rotates the 2 x 2 block (pair k rows, pair k2 columns) from both sides into the other G buffer,
// while threads 256.. rotate the columns of Jp (Jp <- Jp J).  Returns the buffer holding the final
// Gram.  (Round 3: replaces 16 lanes writing the angles to LDS behind a barrier of their own --
// bit-identical outputs, neutral in the bench: C4 27.72 -> 27.59 ms, C5 29.60 -> 29.57 ms, C3 equal;
// the inner round is bound by neither that barrier nor the angle hand-off.)
template <bool FAST>
__device__ __forceinline__ double* inner_sweep(double* Ga, double* Gb, double* Jp, int tid, double tol2, double negl) {
    for (int e = tid; e < 32 * 32; e += kBJThreads) Jp[(e / 32) * GS + e % 32] = (e / 32 == e % 32) ? 1.0 : 0.0;
    __syncthreads();
    const int k = (tid >> 4) & 15, k2 = tid & 15;
    const int src = (tid & 0x30) | k;  // a lane of this wave with k2 == k
    double* cur = Ga;
    double* nxt = Gb;
    for (int ir = 0; ir < 31; ++ir) {
        int p2, q2;
        rr_pair32(ir, k2, p2, q2);
        double c2, s2;
        bool rt2;
        if constexpr (FAST)
            pair_angle_fast(cur, p2, q2, tol2, negl, c2, s2, rt2);
        else
            pair_angle(cur, p2, q2, tol2, negl, c2, s2, rt2);
        const double c1 = __shfl(c2, src, 64), s1 = __shfl(s2, src, 64);
        if (tid < 256) {
            int p, q;
            rr_pair32(ir, k, p, q);
            const double b00 = cur[p * GS + p2], b01 = cur[p * GS + q2];
            const double b10 = cur[q * GS + p2], b11 = cur[q * GS + q2];
            const double l00 = c1 * b00 - s1 * b10, l01 = c1 * b01 - s1 * b11;
            const double l10 = s1 * b00 + c1 * b10, l11 = s1 * b01 + c1 * b11;
            nxt[p * GS + p2] = c2 * l00 - s2 * l01;
            nxt[p * GS + q2] = s2 * l00 + c2 * l01;
            nxt[q * GS + p2] = c2 * l10 - s2 * l11;
            nxt[q * GS + q2] = s2 * l10 + c2 * l11;
        } else if (rt2) {
#pragma unroll
            for (int rr = 0; rr < 2; ++rr) {
                const int row = k + 16 * rr;
                const double jp = Jp[row * GS + p2], jq = Jp[row * GS + q2];
                Jp[row * GS + p2] = c2 * jp - s2 * jq;
                Jp[row * GS + q2] = s2 * jp + c2 * jq;
            }
        }
        __syncthreads();
        double* t = cur;
        cur = nxt;
        nxt = t;
    }
    return cur;
}

// The same sweep on the first four waves only (one per SIMD): thread (k, k2) < 256 also rotates
// rows k and k + 16 of Jp's column pair k2, so the round's VALU work (angle, index arithmetic,
// 2 x 2 updates) is issued once per SIMD instead of twice; waves 4..7 only meet the barriers.
// Same arithmetic as inner_sweep up to the compiler's FMA contraction choices.
template <bool FAST>
__device__ __forceinline__ double* inner_sweep4(double* Ga, double* Gb, double* Jp, int tid, double tol2, double negl) {
    for (int e = tid; e < 32 * 32; e += kBJThreads) Jp[(e / 32) * GS + e % 32] = (e / 32 == e % 32) ? 1.0 : 0.0;
    __syncthreads();
    const int k = (tid >> 4) & 15, k2 = tid & 15;
    const int src = (tid & 0x30) | k;
    double* cur = Ga;
    double* nxt = Gb;
    for (int ir = 0; ir < 31; ++ir) {
        if (tid < 256) {
            int p2, q2, p, q;
            rr_pair32(ir, k2, p2, q2);
            rr_pair32(ir, k, p, q);
            double c2, s2;
            bool rt2;
            if constexpr (FAST)
                pair_angle_fast(cur, p2, q2, tol2, negl, c2, s2, rt2);
            else
                pair_angle(cur, p2, q2, tol2, negl, c2, s2, rt2);
            const double c1 = __shfl(c2, src, 64), s1 = __shfl(s2, src, 64);
            const double b00 = cur[p * GS + p2], b01 = cur[p * GS + q2];
            const double b10 = cur[q * GS + p2], b11 = cur[q * GS + q2];
            const double l00 = c1 * b00 - s1 * b10, l01 = c1 * b01 - s1 * b11;
            const double l10 = s1 * b00 + c1 * b10, l11 = s1 * b01 + c1 * b11;
            nxt[p * GS + p2] = c2 * l00 - s2 * l01;
            nxt[p * GS + q2] = s2 * l00 + c2 * l01;
            nxt[q * GS + p2] = c2 * l10 - s2 * l11;
            nxt[q * GS + q2] = s2 * l10 + c2 * l11;
            if (rt2) {
#pragma unroll
                for (int rr = 0; rr < 2; ++rr) {
                    const int row = k + 16 * rr;
                    const double jp = Jp[row * GS + p2], jq = Jp[row * GS + q2];
                    Jp[row * GS + p2] = c2 * jp - s2 * jq;
                    Jp[row * GS + q2] = s2 * jp + c2 * jq;
                }
            }
        }
        __syncthreads();
        double* t = cur;
        cur = nxt;
        nxt = t;
    }
    return cur;
}

// inner_sweep4 with the rotation of Jp moved to the idle waves 4..7, one round behind: wave 0's
// k == 0 lanes leave each round's (c, s) in a two-slot LDS table, and in round ir + 1 threads 256..
// apply round ir's rotations to rows k, k + 16 of Jp (c = 1, s = 0 for a skipped pair: the
// identity).  The first four waves' round is then the angle and the 2 x 2 Gram update only.
template <bool FAST>
__device__ __forceinline__ double* inner_sweep4j(double* Ga, double* Gb, double* Jp, double* AngB, int tid, double tol2,
                                                 double negl) {
    for (int e = tid; e < 32 * 32; e += kBJThreads) Jp[(e / 32) * GS + e % 32] = (e / 32 == e % 32) ? 1.0 : 0.0;
    __syncthreads();
    const int k = (tid >> 4) & 15, k2 = tid & 15;
    const int src = (tid & 0x30) | k;
    double* cur = Ga;
    double* nxt = Gb;
    for (int ir = 0; ir < 32; ++ir) {
        if (tid < 256) {
            if (ir < 31) {
                int p2, q2, p, q;
                rr_pair32(ir, k2, p2, q2);
                rr_pair32(ir, k, p, q);
                double c2, s2;
                bool rt2;
                if constexpr (FAST)
                    pair_angle_fast(cur, p2, q2, tol2, negl, c2, s2, rt2);
                else
                    pair_angle(cur, p2, q2, tol2, negl, c2, s2, rt2);
                // (evaluating the row pair's angle here too instead of the shuffle: C5 28.5 -> 29.3 ms,
                // the round is VALU-issue-bound)
                const double c1 = __shfl(c2, src, 64), s1 = __shfl(s2, src, 64);
                const double b00 = cur[p * GS + p2], b01 = cur[p * GS + q2];
                const double b10 = cur[q * GS + p2], b11 = cur[q * GS + q2];
                const double l00 = c1 * b00 - s1 * b10, l01 = c1 * b01 - s1 * b11;
                const double l10 = s1 * b00 + c1 * b10, l11 = s1 * b01 + c1 * b11;
                nxt[p * GS + p2] = c2 * l00 - s2 * l01;
                nxt[p * GS + q2] = s2 * l00 + c2 * l01;
                nxt[q * GS + p2] = c2 * l10 - s2 * l11;
                nxt[q * GS + q2] = s2 * l10 + c2 * l11;
                if (tid < 16) {
                    AngB[(ir & 1) * 32 + k2] = c2;
                    AngB[(ir & 1) * 32 + 16 + k2] = s2;
                }
            }
        } else if (ir > 0) {
            int p2, q2;
            rr_pair32(ir - 1, k2, p2, q2);
            const double c2 = AngB[((ir - 1) & 1) * 32 + k2], s2 = AngB[((ir - 1) & 1) * 32 + 16 + k2];
#pragma unroll
            for (int rr = 0; rr < 2; ++rr) {
                const int row = k + 16 * rr;
                const double jp = Jp[row * GS + p2], jq = Jp[row * GS + q2];
                Jp[row * GS + p2] = c2 * jp - s2 * jq;
                Jp[row * GS + q2] = s2 * jp + c2 * jq;
            }
        }
        __syncthreads();
        if (ir < 31) {
            double* t = cur;
            cur = nxt;
            nxt = t;
        }
    }
    return cur;
}

// Stage rows [row0, row0 + nr) of the 32 columns col(0..31) of a column-major matrix (ld rows per
// column) into LDS rows of pitch nr + 1; 32 nr / 2 double2, each thread keeping up to 4 loads in flight.
template <typename F>
__device__ __forceinline__ void stage_pair(double* Xs, const double* __restrict__ S, int ld, int row0, int nr, F col) {
    const int XP = nr + 1;
    const int per = nr / 2;  // double2 per column
    const int tot = 32 * per;
    for (int e0 = threadIdx.x; e0 < tot; e0 += 4 * kBJThreads) {
        double2 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int e = e0 + kBJThreads * u;
            if (e < tot) {
                const int k = e / per, i = 2 * (e % per);
                v[u] = *reinterpret_cast<const double2*>(S + (int64_t)col(k) * ld + row0 + i);
            }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int e = e0 + kBJThreads * u;
            if (e < tot) {
                const int k = e / per, i = 2 * (e % per);
                Xs[k * XP + i] = v[u].x;
                Xs[k * XP + i + 1] = v[u].y;
            }
        }
    }
}

// D[row0 + i, col(j)] = sum_k Xs[k][i] Jp[k][j], i < nr, for the 32 pair columns (fp64 MFMA; D has
// ld rows per column), wave w -> row tiles w, w + 8, ...
template <typename F>
__device__ __forceinline__ void apply_pair(const double* Xs, const double* Jp, double* __restrict__ D, int ld, int row0,
                                           int nr, F col, int w, int r, int h) {
    const int XP = nr + 1;
    for (int it = w; it < nr / 16; it += kBJThreads / 64) {
        const int i0 = 16 * it;
        f64x4 acc0 = MD::zero(), acc1 = MD::zero();
#pragma unroll
        for (int kk = 0; kk < 8; ++kk) {
            const double a = Xs[(4 * kk + h) * XP + i0 + r];
            acc0 = MD::mma(a, Jp[(4 * kk + h) * GS + r], acc0);
            acc1 = MD::mma(a, Jp[(4 * kk + h) * GS + 16 + r], acc1);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            st_wt(D + (int64_t)col(r) * ld + row0 + i0 + MD::row(h, j), acc0[j]);
            st_wt(D + (int64_t)col(16 + r) * ld + row0 + i0 + MD::row(h, j), acc1[j]);
        }
    }
}

// The same product with the pair's columns read straight from global memory (column-major source:
// the 16 lanes of an MFMA row read 128 contiguous bytes of one column), all 8 k-steps in flight.
template <typename F>
__device__ __forceinline__ void apply_pair_global(const double* __restrict__ Src, const double* Jp,
                                                  double* __restrict__ D, int ld, int row0, int nr, F col, int w, int r,
                                                  int h) {
    for (int it = w; it < nr / 16; it += kBJThreads / 64) {
        const int i0 = row0 + 16 * it;
        double a[8];
#pragma unroll
        for (int kk = 0; kk < 8; ++kk) a[kk] = Src[(int64_t)col(4 * kk + h) * ld + i0 + r];
        f64x4 acc0 = MD::zero(), acc1 = MD::zero();
#pragma unroll
        for (int kk = 0; kk < 8; ++kk) {
            acc0 = MD::mma(a[kk], Jp[(4 * kk + h) * GS + r], acc0);
            acc1 = MD::mma(a[kk], Jp[(4 * kk + h) * GS + 16 + r], acc1);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            st_wt(D + (int64_t)col(r) * ld + i0 + MD::row(h, j), acc0[j]);
            st_wt(D + (int64_t)col(16 + r) * ld + i0 + MD::row(h, j), acc1[j]);
        }
    }
}

#ifdef RSVD_BJ_PROF
__device__ long long g_bj_prof[8];
#define BJ_T(k)                                                \
    do {                                                       \
        if (wg == 0 && tid == 0) {                             \
            const long long now_ = wall_clock64();             \
            bj_acc[(k)] += now_ - bj_last;                     \
            bj_last = now_;                                    \
        }                                                      \
    } while (0)
#else
#define BJ_T(k) \
    do {        \
    } while (0)
#endif

// Gp = X_pair^T X_pair with the pair's columns read from global memory (MR > 512 rows: no LDS
// image), wave w -> tile ((w >> 1) & 1, w & 1) over row half w >> 2; the halves land in Ga / Gb.
template <typename F>
__device__ __forceinline__ void pair_gram_global(const double* __restrict__ X, int MR, int row0, int nr, F col, int w,
                                                 int r, int h, double* Ga, double* Gb) {
    const int ta = (w >> 1) & 1, tb = w & 1, half = w >> 2;
    const double* xa = X + (int64_t)col(16 * ta + r) * MR + 4 * h;
    const double* xb = X + (int64_t)col(16 * tb + r) * MR + 4 * h;
    f64x4 acc[2] = {MD::zero(), MD::zero()};
    const int ibeg = row0 + half * (nr / 2), iend = ibeg + nr / 2;
    for (int i0 = ibeg; i0 < iend; i0 += 16) {
        const double2 a01 = *reinterpret_cast<const double2*>(xa + i0);
        const double2 a23 = *reinterpret_cast<const double2*>(xa + i0 + 2);
        const double2 b01 = *reinterpret_cast<const double2*>(xb + i0);
        const double2 b23 = *reinterpret_cast<const double2*>(xb + i0 + 2);
        acc[0] = MD::mma(a01.x, b01.x, acc[0]);
        acc[1] = MD::mma(a01.y, b01.y, acc[1]);
        acc[0] = MD::mma(a23.x, b23.x, acc[0]);
        acc[1] = MD::mma(a23.y, b23.y, acc[1]);
    }
    double* Gd = half ? Gb : Ga;
#pragma unroll
    for (int j = 0; j < 4; ++j) Gd[(16 * ta + MD::row(h, j)) * GS + 16 * tb + r] = acc[0][j] + acc[1][j];
}

__device__ __forceinline__ double u64_as_double(unsigned long long v) { return __longlong_as_double((long long)v); }

// max cos^2 over the column pairs (a, b), a in this workgroup's 32 columns [32 wg, 32 wg + 32), b any,
// of the MR x LP column-major X (global, after an acquire): 16 x 16 Gram tiles on the fp64 MFMA,
// the column norms accumulated from the same operand loads.  Columns with norm^2 <= negl (and the
// zero padding) are excluded, as the rotations exclude them.
__device__ double slice_max_cos2(const double* __restrict__ X, int MR, int LP, int slice, int g, int G, int w, int lane,
                                 double negl) {
    const int r = lane & 15, h = lane >> 4;
    double mx = 0.0;
    const int ntile = 2 * (LP / 16);
    for (int t = w + (kBJThreads / 64) * g; t < ntile; t += (kBJThreads / 64) * G) {
        const int a0 = 32 * slice + 16 * (t & 1), b0 = 16 * (t >> 1);
        const double* xa = X + (int64_t)(a0 + r) * MR + 4 * h;
        const double* xb = X + (int64_t)(b0 + r) * MR + 4 * h;
        f64x4 acc = MD::zero();
        double na = 0.0, nb = 0.0;
        for (int i0 = 0; i0 < MR; i0 += 16) {
            const double2 a01 = *reinterpret_cast<const double2*>(xa + i0);
            const double2 a23 = *reinterpret_cast<const double2*>(xa + i0 + 2);
            const double2 b01 = *reinterpret_cast<const double2*>(xb + i0);
            const double2 b23 = *reinterpret_cast<const double2*>(xb + i0 + 2);
            // k order inside the 16-row chunk is 4h + j for both operands (the sum is order-free)
            acc = MD::mma(a01.x, b01.x, acc);
            acc = MD::mma(a01.y, b01.y, acc);
            acc = MD::mma(a23.x, b23.x, acc);
            acc = MD::mma(a23.y, b23.y, acc);
            na += a01.x * a01.x + a01.y * a01.y + a23.x * a23.x + a23.y * a23.y;
            nb += b01.x * b01.x + b01.y * b01.y + b23.x * b23.x + b23.y * b23.y;
        }
        na += __shfl_xor(na, 16, 64);
        na += __shfl_xor(na, 32, 64);
        nb += __shfl_xor(nb, 16, 64);
        nb += __shfl_xor(nb, 32, 64);
        // C/D (f64): col = lane & 15 (b0 + col), row = h + 4 reg (a0 + row)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int row = MD::row(h, j);
            const double nar = __shfl(na, row, 64);
            const double g = acc[j];
            if (a0 + row != b0 + r && nar > negl && nb > negl) mx = fmax(mx, (g * g) / (nar * nb));
        }
    }
    return mx;
}

// X = the mrv x l source (column-major with ld lds, or row-major when src_rowmajor: X = src^T),
// zero-padded to MR x LP (MR, LP multiples of 32); J = I (LP x LP).  Grid: (LP / 32) pairs x G
// row-group members (MR % 32 G == 0, LP % 16 G == 0).  MR / G <= 512: the member's rows of the pair
// columns are staged in LDS; beyond, the pair Gram and the X product read them from global memory.
// scratch: nwg + 1024 nwg doubles (||W||_F partials, then the partial pair Grams when G > 1).
__global__ __launch_bounds__(kBJThreads) void block_jacobi_kernel(const double* __restrict__ R, int64_t lds,
                                                           int src_rowmajor, int mrv, int l, int MR, int LP, int G,
                                                           double* __restrict__ Xb, double* __restrict__ Jb,
                                                           double* __restrict__ scratch, unsigned* __restrict__ sync,
                                                           int* __restrict__ info, double quad2, double tol_chk2,
                                                           int inner_v, int given) {
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    const int rpg = MR / G, jpg = LP / G;  // rows of X / J per group member
    const bool staged = rpg <= 512;
    const int XP = rpg + 1;
    double* Xs = reinterpret_cast<double*>(smem_raw);  // [32][MR + 1]: the pair's columns (staged)
    double* Ga = Xs + (staged ? 32 * XP : 0);          // [32][GS] x 2: the pair Gram (Gb: the MFMA half)
    double* Gb = Ga + 32 * GS;
    double* Jp = Gb + 32 * GS;                         // [32][GS] accumulated inner rotation
    __shared__ int flags[8];
    __shared__ double AngB[64];  // inner_sweep4j: (c, s) of two inner rounds
    __shared__ double fro;
    __shared__ unsigned long long lmax;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int r = lane & 15, h = lane >> 4;
    const int nwg = gridDim.x, wg = blockIdx.x;
    const int pr = wg / G, g = wg - pr * G;  // block pair (round-robin slot), row-group member
    const int xr0 = g * rpg, jr0 = g * jpg;
    unsigned* gctr = sync + kGroupWord + pr;
    double* gpart = scratch + ((nwg + 31) & ~31);  // [pair][member] 32 x 32 partial Grams
    const int NB = LP / 16;
    const int64_t L2 = (int64_t)LP * LP, L2X = (int64_t)MR * LP;
    const double tol = (double)l * kEps, tol2 = tol * tol;
    unsigned long long* smax = reinterpret_cast<unsigned long long*>(sync + 80);
    unsigned long long* cmax = reinterpret_cast<unsigned long long*>(sync + 144);
#ifdef RSVD_BJ_PROF
    long long bj_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    long long bj_last = wall_clock64();
#endif

    // X (column-major, X[c][i] = W[i][c] = R[c][i]) and J = I into buffer 0: columns of this
    // workgroup; this workgroup's part of ||W||_F^2 to scratch[wg]
    // (given: X and J are already in buffer 0 -- wide_eig.hip's X = W V_w, J = V_w -- and |X|_F = |W|_F)
    {
        double part = 0.0;
        for (int c = wg; c < LP; c += nwg) {
            for (int i = tid; i < MR; i += kBJThreads) {
                double v;
                if (given) {
                    v = Xb[(int64_t)c * MR + i];
                } else {
                    v = (c < l && i < mrv) ? (src_rowmajor ? R[(int64_t)i * lds + c] : R[(int64_t)c * lds + i]) : 0.0;
                    Xb[(int64_t)c * MR + i] = v;
                }
                part += v * v;
            }
            if (!given)
                for (int i = tid; i < LP; i += kBJThreads) Jb[(int64_t)c * LP + i] = (c == i && c < l) ? 1.0 : 0.0;
        }
        if (tid == 0) fro = 0.0;
        __syncthreads();
        part = warp_sum(part);
        if (lane == 0) atomicAdd(&fro, part);
        __syncthreads();
        if (tid == 0) scratch[wg] = fro;
    }
    unsigned bar = 0;
    if (!grid_barrier(sync, (unsigned)nwg * ++bar)) {
        if (tid == 0) info[2] = 1;
        return;
    }
    // ||W||_F^2 in a fixed order (every workgroup the same value) -> negligible-column threshold
    double frot = 0.0;
    for (int k = 0; k < nwg; ++k) frot += scratch[k];
    const double negl = frot * (double)l * l * kEps * kEps;

    BJ_T(0);
    int par = 0, sweeps = 0;
    bool done = false;
    if (given == 1 && tol_chk2 > 0.0) {
        // the given X may already be orthogonal to the tolerance: the global check first (slot 31)
        // (given == 2: the check is skipped and the sweeps run -- RSVD_EIG_FORCE_POLISH, tests only)
        const double mx = slice_max_cos2(Xb, MR, LP, pr, g, G, w, lane, negl);
        if (tid == 0) lmax = 0ull;
        __syncthreads();
        atomicMax(&lmax, (unsigned long long)__double_as_longlong(mx));
        __syncthreads();
        if (tid == 0) atomicMax(cmax + 31, lmax);
        if (!grid_barrier(sync, (unsigned)nwg * ++bar)) {
            if (tid == 0) info[2] = 1;
            return;
        }
        done = u64_as_double(__hip_atomic_load(cmax + 31, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) <= tol_chk2;
    }
    for (int sweep = 0; sweep < kMaxSweeps && !done; ++sweep) {
        for (int round = 0; round < NB - 1; ++round) {
            int P, Q;
            rr_pair(round, pr, NB, P, Q);
            const double* Xsrc = Xb + (size_t)par * L2X;
            const double* Jsrc = Jb + (size_t)par * L2;
            double* Xd = Xb + (size_t)(1 - par) * L2X;
            double* Jd = Jb + (size_t)(1 - par) * L2;
            auto col = [&](int k) { return k < 16 ? 16 * P + k : 16 * Q + k - 16; };
            // 1. the pair's columns of X into LDS
            if (staged) stage_pair(Xs, Xsrc, MR, xr0, rpg, col);
            if (tid < 8) flags[tid] = 0;
            if (tid == 0) lmax = 0ull;
            __syncthreads();
            BJ_T(1);
            // 2. Gp = X_pair^T X_pair: wave w -> tile ((w >> 1) & 1, w & 1) over row half w >> 2 (four
            //    independent MFMA chains); the halves meet in Ga (half 0) + Gb (half 1)
            if (!staged) {
                pair_gram_global(Xsrc, MR, xr0, rpg, col, w, r, h, Ga, Gb);
            } else {
                const int ta = (w >> 1) & 1, tb = w & 1, half = w >> 2;
                const double* xa = Xs + (16 * ta + r) * XP + h;
                const double* xb = Xs + (16 * tb + r) * XP + h;
                f64x4 acc[4] = {MD::zero(), MD::zero(), MD::zero(), MD::zero()};
                const int ibeg = half * (rpg / 2), iend = ibeg + rpg / 2;
                for (int i0 = ibeg; i0 < iend; i0 += 16) {
#pragma unroll
                    for (int u = 0; u < 4; ++u) acc[u] = MD::mma(xa[i0 + 4 * u], xb[i0 + 4 * u], acc[u]);
                }
                double* Gd = half ? Gb : Ga;
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    Gd[(16 * ta + MD::row(h, j)) * GS + 16 * tb + r] = (acc[0][j] + acc[1][j]) + (acc[2][j] + acc[3][j]);
            }
            __syncthreads();
            if (G == 1) {
                for (int e = tid; e < 32 * 32; e += kBJThreads) {
                    const int i = e / 32, j = e % 32;
                    Ga[i * GS + j] += Gb[i * GS + j];
                }
            } else {
                // publish this member's rows' Gram, meet the group, sum the G partials in member order
                double* mine = gpart + (int64_t)wg * 1024;
                for (int e = tid; e < 32 * 32; e += kBJThreads) {
                    const int i = e / 32, j = e % 32;
                    st_wt(mine + e, Ga[i * GS + j] + Gb[i * GS + j]);
                }
                if (!group_barrier(sync, gctr, (unsigned)G * (unsigned)(sweep * (NB - 1) + round + 1))) {
                    if (tid == 0) info[2] = 1;
                    return;
                }
                double* grp = gpart + (int64_t)pr * G * 1024;
                for (int e = tid; e < 32 * 32; e += kBJThreads) {
                    const int i = e / 32, j = e % 32;
                    double v = ld_wt(grp + e);
                    for (int m = 1; m < G; ++m) v += ld_wt(grp + (int64_t)m * 1024 + e);
                    Ga[i * GS + j] = v;
                }
            }
            __syncthreads();
            BJ_T(2);
            // 3. convergence test on the fresh Gram (and this round's largest cos^2, one LDS atomic per wave)
            {
                double cm = 0.0;
                for (int e = tid; e < 32 * 32; e += kBJThreads) {
                    const int i = e / 32, j = e % 32;
                    if (i < j) {
                        const double a = Ga[i * GS + i], b = Ga[j * GS + j], g = Ga[i * GS + j];
                        if (a > negl && b > negl) {
                            cm = fmax(cm, (g * g) / (a * b));
                            if (g != 0.0 && g * g > tol2 * a * b) {
                                flags[0] = 1;
                                if (g * g > quad2 * a * b) flags[1] = 1;
                            }
                        }
                    }
                }
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) cm = fmax(cm, __shfl_xor(cm, o, 64));
                if (lane == 0 && cm > 0.0) atomicMax(&lmax, (unsigned long long)__double_as_longlong(cm));
            }
            __syncthreads();
            if (tid == 0 && lmax) atomicMax(smax + sweep, lmax);
            if (flags[0]) {
                if (tid == 0) {
                    __hip_atomic_store(sync + 4 + sweep, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (flags[1]) __hip_atomic_store(sync + 36 + sweep, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                // 4. the inner sweep on Gp (in place; Jp from the register wave)
                switch (inner_v) {
                    case 1: inner_sweep4<false>(Ga, Gb, Jp, tid, tol2, negl); break;
                    case 2: inner_sweep<true>(Ga, Gb, Jp, tid, tol2, negl); break;
                    case 3: inner_sweep4<true>(Ga, Gb, Jp, tid, tol2, negl); break;
                    case 5: inner_sweep4j<false>(Ga, Gb, Jp, AngB, tid, tol2, negl); break;
                    case 7: inner_sweep4j<true>(Ga, Gb, Jp, AngB, tid, tol2, negl); break;
                    default: inner_sweep<false>(Ga, Gb, Jp, tid, tol2, negl);
                }
                BJ_T(3);
                // 5. X_pair Jp and J_pair Jp -> destination buffer
                if (staged)
                    apply_pair(Xs, Jp, Xd, MR, xr0, rpg, col, w, r, h);
                else
                    apply_pair_global(Xsrc, Jp, Xd, MR, xr0, rpg, col, w, r, h);
                BJ_T(4);
                apply_pair_global(Jsrc, Jp, Jd, LP, jr0, jpg, col, w, r, h);
                BJ_T(5);
            } else {
                for (int e = tid; e < 32 * (rpg / 2); e += kBJThreads) {
                    const int kk = e / (rpg / 2), i = 2 * (e % (rpg / 2));
                    const int64_t o = (int64_t)col(kk) * MR + xr0 + i;
                    const double2 v = *reinterpret_cast<const double2*>(Xsrc + o);
                    st_wt(Xd + o, v.x);
                    st_wt(Xd + o + 1, v.y);
                }
                for (int e = tid; e < 32 * (jpg / 2); e += kBJThreads) {
                    const int kk = e / (jpg / 2), i = 2 * (e % (jpg / 2));
                    const int64_t o = (int64_t)col(kk) * LP + jr0 + i;
                    const double2 v = *reinterpret_cast<const double2*>(Jsrc + o);
                    st_wt(Jd + o, v.x);
                    st_wt(Jd + o + 1, v.y);
                }
            }
            par = 1 - par;
            BJ_T(7);
            if (!grid_barrier(sync, (unsigned)nwg * ++bar)) {
                if (tid == 0) info[2] = 1;
                return;
            }
            BJ_T(6);
        }
        ++sweeps;
        const unsigned rot = __hip_atomic_load(sync + 4 + sweep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned big = __hip_atomic_load(sync + 36 + sweep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (rot == 0 || big == 0) break;
        // the global check, once the sweep's rotations were small enough to have squared below tol_chk2
        const double pre = u64_as_double(__hip_atomic_load(smax + sweep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        // (triggered at a pre-rotation cos^2 100x above sqrt(tol): a failed check costs one LP x LP
        // Gram and a barrier, a missed one a whole sweep -- the C4 solve sat on the 7 / 8 sweep border)
        if (tol_chk2 > 0.0 && pre <= 100.0 * sqrt(tol_chk2)) {
            const double mx = slice_max_cos2(Xb + (size_t)par * L2X, MR, LP, pr, g, G, w, lane, negl);
            if (tid == 0) lmax = 0ull;
            __syncthreads();
            atomicMax(&lmax, (unsigned long long)__double_as_longlong(mx));
            __syncthreads();
            if (tid == 0) atomicMax(cmax + sweep, lmax);
            if (!grid_barrier(sync, (unsigned)nwg * ++bar)) {
                if (tid == 0) info[2] = 1;
                return;
            }
            const double post = u64_as_double(__hip_atomic_load(cmax + sweep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
            if (post <= tol_chk2) break;
        }
    }
    if (wg == 0 && tid == 0) {
        sync[2] = (unsigned)par;
        info[0] = sweeps;
#ifdef RSVD_BJ_PROF
        for (int k = 0; k < 8; ++k) g_bj_prof[k] = bj_acc[k];
#endif
    }
}

// S, U_w = X / S (sorted descending, completed to orthonormal where S = 0), V_w = J, in four
// launches: (1) one workgroup: column norms, descending ranks, S, and the sorted norms + inverse
// permutation to scratch (the free half of the X double buffer); (2, 3) grids of 64 x 64 tiles:
// U_w[i][k] = X[inv[k]][i] / s_k (MR rows), V_w[i][k] = J[inv[k]][i] (LP rows), through an LDS
// transpose (coalesced reads along i and writes along k -- one workgroup scattering 8-B values down
// the columns of row-major U_w / V_w ran 0.7 ms at LP = 512); (4) one workgroup: completion of U_w
// for zero singular values (returns at once when there are none).  U_w row-major [row][col], MR x LP;
// V_w LP x LP.
template <typename T>
__global__ __launch_bounds__(1024) void block_jacobi_finish_kernel(const double* __restrict__ Xb, int l, int MR,
                                                                   int LP, const unsigned* __restrict__ sync,
                                                                   T* __restrict__ S) {
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    double* sig = reinterpret_cast<double*>(smem_raw);  // [LP]
    double* v = sig + LP;                               // [LP]
    int* rank = reinterpret_cast<int*>(v + LP);         // [LP]
    int* misc = rank + LP;                              // [4]
    const int tid = threadIdx.x, nt = blockDim.x;
    const int64_t L2X = (int64_t)MR * LP;
    const int par = (int)sync[2];
    const double* X = Xb + (size_t)par * L2X;
    double* sigk = const_cast<double*>(Xb) + (size_t)(1 - par) * L2X;  // scratch: [LP] sorted norms
    int* inv = reinterpret_cast<int*>(sigk + LP);                      // [LP] column of rank k
    // squared column norms: one wave per column, coalesced loads + a wave reduction, four columns
    // per wave in flight (a column at a time left every wave waiting out one L2 round trip per column)
    const int lane = tid & 63, wv = tid >> 6, nw = nt >> 6;
    for (int c0 = wv; c0 < LP; c0 += 4 * nw) {
        double s2[4] = {0.0, 0.0, 0.0, 0.0};
        for (int i = lane; i < MR; i += 64) {
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int c = c0 + u * nw;
                const double x = (c < l) ? X[(int64_t)c * MR + i] : 0.0;
                s2[u] += x * x;
            }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const double t = warp_sum(s2[u]);
            if (lane == 0 && c0 + u * nw < LP) sig[c0 + u * nw] = t;
        }
    }
    __syncthreads();
    if (wv == 0) {
        double f = 0.0;
        for (int c = lane; c < l; c += 64) f += sig[c];
        f = warp_sum(f);
        if (lane == 0) {
            misc[1] = 0;
            v[0] = f * (double)l * l * kEps * kEps;  // negligible column norm^2
        }
    }
    __syncthreads();
    const double negl = v[0];
    __syncthreads();
    for (int c = tid; c < LP; c += nt) {
        const double s2 = sig[c];
        const double sv = sqrt(s2);
        sig[c] = (c < l && isfinite(sv) && s2 > negl) ? sv : 0.0;
    }
    __syncthreads();
    for (int c = tid; c < l; c += nt) {
        int rk = 0;
        const double sc = sig[c];
        for (int d = 0; d < l; ++d) rk += (sig[d] > sc) || (sig[d] == sc && d < c);
        S[rk] = (T)sc;
        sigk[rk] = sc;
        inv[rk] = c;
    }
}

// Dst[i][k] = Src[inv[k]][i] (/ s_k when scale), i < rows (rows >= rows_valid are zero), k < LP
__global__ __launch_bounds__(256) void block_jacobi_scatter_kernel(const double* __restrict__ base, int64_t buf_stride,
                                                                   const double* __restrict__ Xb, int64_t x_stride,
                                                                   int rows_valid, int rows, int l, int LP,
                                                                   const unsigned* __restrict__ sync, int scale,
                                                                   double* __restrict__ Dst) {
    __shared__ double tile[64][65];
    __shared__ double rs[64];
    __shared__ int col[64];
    const int tid = threadIdx.x;
    const int nbk = (LP + 63) / 64;  // LP is a multiple of 32: the last tile column may be half
    const int k0 = 64 * (blockIdx.x % nbk), i0 = 64 * (blockIdx.x / nbk);
    const int par = (int)sync[2];
    const double* src = base + (size_t)par * buf_stride;
    const double* sigk = Xb + (size_t)(1 - par) * x_stride;
    const int* inv = reinterpret_cast<const int*>(sigk + LP);
    if (tid < 64) {
        const int k = k0 + tid;
        const double sc = k < l ? sigk[k] : 0.0;
        col[tid] = k < l ? inv[k] : -1;
        rs[tid] = !scale ? 1.0 : (sc > 0.0 ? 1.0 / sc : 0.0);
    }
    __syncthreads();
    for (int e = tid; e < 64 * 64; e += 256) {
        const int kk = e >> 6, ii = e & 63;
        const int c = col[kk], i = i0 + ii;
        double x = 0.0;
        if (c >= 0 && i < rows_valid) x = src[(int64_t)c * rows + i] * rs[kk];
        tile[kk][ii] = x;
    }
    __syncthreads();
    for (int e = tid; e < 64 * 64; e += 256) {
        const int ii = e >> 6, kk = e & 63;
        if (i0 + ii < rows && k0 + kk < LP) Dst[(int64_t)(i0 + ii) * LP + k0 + kk] = tile[kk][ii];
    }
}

template <typename T>
__global__ __launch_bounds__(1024) void block_jacobi_complete_kernel(const T* __restrict__ S, int l, int rows_valid,
                                                                     int LP, double* __restrict__ Uw) {
    // LDS is sized by LP, not by rows (the standalone SVD<Jacobi> has rows = max(m, n), unbounded):
    // v[j] (j < LP) holds the CGS2 coefficients; the least-covered row is a block argmin reduction
    // of per-thread (coverage, row) minima over the rows in global memory
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    double* v = reinterpret_cast<double*>(smem_raw);  // [max(LP, 1024)]
    int* vi = reinterpret_cast<int*>(v + (LP > 1024 ? LP : 1024));  // [1024]
    __shared__ int misc[2];
    const int tid = threadIdx.x, nt = blockDim.x;
    if (tid == 0) misc[1] = 0;
    __syncthreads();
    int mine = 0;
    for (int c = tid; c < l; c += nt) mine += (S[c] > (T)0);
    if (mine) atomicAdd(&misc[1], mine);
    __syncthreads();
    const int nz = misc[1];
    // complete U_w for zero singular values (as jacobi.hip): least-covered unit vector, CGS2
    for (int k = nz; k < l; ++k) {
        double best_c = 1e300;
        int best_i = 0x7fffffff;
        for (int i = tid; i < rows_valid; i += nt) {
            double cov = 0.0;
            for (int j = 0; j < k; ++j) cov += Uw[(int64_t)i * LP + j] * Uw[(int64_t)i * LP + j];
            if (cov < best_c) best_c = cov, best_i = i;  // rows visited in ascending order: first minimum
        }
        v[tid] = best_c;
        vi[tid] = best_i;
        __syncthreads();
        for (int o = nt / 2; o > 0; o >>= 1) {
            if (tid < o) {
                const double c2 = v[tid + o];
                const int i2 = vi[tid + o];
                if (c2 < v[tid] || (c2 == v[tid] && i2 < vi[tid])) v[tid] = c2, vi[tid] = i2;
            }
            __syncthreads();
        }
        const int cand = vi[0];
        __syncthreads();
        for (int i = tid; i < rows_valid; i += nt) Uw[(int64_t)i * LP + k] = (i == cand) ? 1.0 : 0.0;
        __syncthreads();
        for (int pass = 0; pass < 2; ++pass) {
            for (int j = tid; j < k; j += nt) {
                double d = 0.0;
                for (int i = 0; i < rows_valid; ++i) d += Uw[(int64_t)i * LP + j] * Uw[(int64_t)i * LP + k];
                v[j] = d;
            }
            __syncthreads();
            for (int i = tid; i < rows_valid; i += nt) {
                double x = Uw[(int64_t)i * LP + k];
                for (int j = 0; j < k; ++j) x -= v[j] * Uw[(int64_t)i * LP + j];
                Uw[(int64_t)i * LP + k] = x;
            }
            __syncthreads();
        }
        if (tid == 0) {
            double nv = 0.0;
            for (int i = 0; i < rows_valid; ++i) nv += Uw[(int64_t)i * LP + k] * Uw[(int64_t)i * LP + k];
            v[0] = 1.0 / sqrt(nv);
        }
        __syncthreads();
        const double sc = v[0];
        for (int i = tid; i < rows_valid; i += nt) Uw[(int64_t)i * LP + k] *= sc;
        __syncthreads();
    }
}

}  // namespace

// inner sweep form: bit 0 = the first four waves only (inner_sweep4), bit 1 = pair_angle_fast,
// bit 2 (with bit 0) = Jp rotated by waves 4..7 one round behind (inner_sweep4j).
// Same box A/B (round 3, variants 0/1/2/3): C5 29.77 / 29.25 / 29.48 / 29.14 ms, C3 7.15 / 6.99 / 7.04 /
// 6.99 ms, C4 28.02 / 28.05 / 28.06 / 27.92 ms (8 sweeps in every case); another box, 3 / 5 / 7:
// C5 28.91 / 28.51 / 28.34, C4 27.67 / 27.35 / 27.27, C3 6.96 / 6.92 / 6.88.  Default: 7 for the
// fp32-result tolerance; the fp64-result runs (tol_chk <= 1e-9: the standalone fp64 SVD, fp64 A)
// keep 0, whose V is orthogonal to the 1e-12 the fp64 SVD tests hold (3 gave 1.6e-12 on a
// 1200 x 900 SVD).
static int bj_inner_variant(double tol_chk) { return tol_chk > 1e-9 ? 7 : 0; }

int block_jacobi_groups(int MR, int LP, int G) {
    // scratch (U_w, MR x LP doubles) must hold nwg + 1024 nwg doubles; members split MR and LP rows
    // into whole 32- / 16-row tiles
    auto ok = [&](int g) {
        const int64_t nwg = (int64_t)(LP / 32) * g;
        return MR % (32 * g) == 0 && LP % (16 * g) == 0 && ((nwg + 31) & ~31) + 1024 * nwg <= (int64_t)MR * LP;
    };
    if (G > 0) return ok(G) ? G : 0;
    for (int g : {4, 2}) {
        if (ok(g)) return g;
    }
    return 1;
}

template <typename T>
hipError_t bj_launch(const double* src, int64_t lds, int src_rowmajor, int mrv, int l, int MR, int LP, double* X,
                     double* J, double* Uw, double* Vw, T* S, unsigned* sync, int* info, hipStream_t s, double quad2,
                     double tol_chk, int G, int given) {
    if (LP % 32 || LP < 64 || LP > 4096 || MR % 32 || MR < 32 || l > LP || mrv > MR) return hipErrorInvalidValue;
    G = block_jacobi_groups(MR, LP, G);
    if (G < 1) return hipErrorInvalidValue;
    // the persistent grid (LP / 32 pair slots x G row-group members) must be co-resident: fewer
    // members per pair when the device cannot hold it (LP = 4096: 128 x 4 workgroups of 512
    // threads), and a refusal when even one member per pair does not fit
    auto cap = [&](int g) { return coresident_capacity(block_jacobi_kernel, kBJThreads, block_jacobi_lds(MR / g)); };
    int64_t c = cap(G);
    while (c >= 0 && G > 1 && (int64_t)(LP / 32) * G > c) {
        G = G / 2 >= 1 && block_jacobi_groups(MR, LP, G / 2) ? G / 2 : 1;
        c = cap(G);
    }
    if (c < 0) return (hipError_t)(-c);  // the occupancy query failed (not a size problem)
    if ((int64_t)(LP / 32) * G > c) return hipErrorCooperativeLaunchTooLarge;
    hipError_t e = hipMemsetAsync(sync, 0, kSyncWords * sizeof(unsigned), s);
    if (e != hipSuccess) return e;
    e = launch_coresident(block_jacobi_kernel, dim3(LP / 32 * G), dim3(kBJThreads), block_jacobi_lds(MR / G), s, src,
                          lds, src_rowmajor, mrv, l, MR, LP, G, X, J, Uw, sync, info, quad2, tol_chk * tol_chk,
                          bj_inner_variant(tol_chk), given);
    if (e != hipSuccess) return e;
    const size_t lds_fin = (size_t)LP * 8 * 2 + (size_t)LP * 4 + 64;
    hipLaunchKernelGGL((block_jacobi_finish_kernel<T>), dim3(1), dim3(1024), lds_fin, s, X, l, MR, LP, sync, S);
    const int64_t sx = (int64_t)MR * LP, sj = (int64_t)LP * LP;
    const int nbk = (LP + 63) / 64;
    hipLaunchKernelGGL(block_jacobi_scatter_kernel, dim3(nbk * ((LP + 63) / 64)), dim3(256), 0, s, J, sj, X, sx, l, LP,
                       l, LP, sync, 0, Vw);
    hipLaunchKernelGGL(block_jacobi_scatter_kernel, dim3(nbk * ((MR + 63) / 64)), dim3(256), 0, s, X, sx, X, sx, mrv, MR,
                       l, LP, sync, 1, Uw);
    hipLaunchKernelGGL((block_jacobi_complete_kernel<T>), dim3(1), dim3(1024), (size_t)std::max(LP, 1024) * 8 + 1024 * 4,
                       s, S, l, mrv, LP, Uw);
    return hipGetLastError();
}

template <typename T>
hipError_t launch_block_jacobi_ex(const double* src, int64_t lds, int src_rowmajor, int mrv, int l, int MR, int LP,
                                  double* X, double* J, double* Uw, double* Vw, T* S, unsigned* sync, int* info,
                                  hipStream_t s, double quad2, double tol_chk, int G) {
    return bj_launch<T>(src, lds, src_rowmajor, mrv, l, MR, LP, X, J, Uw, Vw, S, sync, info, s, quad2, tol_chk, G, 0);
}

template <typename T>
hipError_t launch_block_jacobi_given(int l, int LP, double* X, double* J, double* Uw, double* Vw, T* S, unsigned* sync,
                                     int* info, hipStream_t s, double tol_chk) {
    if (LP > 512) return hipErrorInvalidValue;
    // RSVD_EIG_FORCE_POLISH=1 (tests): skip the orthogonality check, so the Jacobi polish of the
    // eigensolver's X always runs -- the path a failed check takes
    static const int force = [] {
        const char* v = std::getenv("RSVD_EIG_FORCE_POLISH");
        return v ? std::atoi(v) : 0;
    }();
    return bj_launch<T>(nullptr, LP, 0, l, l, LP, LP, X, J, Uw, Vw, S, sync, info, s,
                        tol_chk > 1e-9 ? 1e-8 : 1e-16, tol_chk, 0, force ? 2 : 1);
}
template hipError_t launch_block_jacobi_given<float>(int, int, double*, double*, double*, double*, float*, unsigned*,
                                                     int*, hipStream_t, double);
template hipError_t launch_block_jacobi_given<double>(int, int, double*, double*, double*, double*, double*,
                                                      unsigned*, int*, hipStream_t, double);

template <typename T>
hipError_t launch_block_jacobi(const double* R, int l, int LP, double* X, double* J, double* Uw, double* Vw, T* S,
                               unsigned* sync, int* info, hipStream_t s, double quad2, double tol_chk, int G) {
    if (LP > 512) return hipErrorInvalidValue;
    return launch_block_jacobi_ex<T>(R, LP, 0, l, l, LP, LP, X, J, Uw, Vw, S, sync, info, s, quad2, tol_chk, G);
}

template hipError_t launch_block_jacobi<float>(const double*, int, int, double*, double*, double*, double*, float*,
                                               unsigned*, int*, hipStream_t, double, double, int);
template hipError_t launch_block_jacobi<double>(const double*, int, int, double*, double*, double*, double*, double*,
                                                unsigned*, int*, hipStream_t, double, double, int);
template hipError_t launch_block_jacobi_ex<float>(const double*, int64_t, int, int, int, int, int, double*, double*,
                                                  double*, double*, float*, unsigned*, int*, hipStream_t, double, double,
                                                  int);
template hipError_t launch_block_jacobi_ex<double>(const double*, int64_t, int, int, int, int, int, double*, double*,
                                                   double*, double*, double*, unsigned*, int*, hipStream_t, double,
                                                   double, int);

#ifdef RSVD_BJ_PROF
void bj_prof_dump() {
    long long t[8];
    (void)hipMemcpyFromSymbol(t, HIP_SYMBOL(g_bj_prof), sizeof(t));
    printf("  block_jacobi phases (us, wg 0): init %.1f stage %.1f gram %.1f test %.1f inner %.1f applyX %.1f "
           "stageJ+applyJ %.1f tail %.1f barrier %.1f\n", t[0] * 0.01, t[1] * 0.01, t[2] * 0.01, 0.0, t[3] * 0.01,
           t[4] * 0.01, t[5] * 0.01, t[7] * 0.01, t[6] * 0.01);
}
#endif
}  // namespace rsvd
