// qr.hip -- tall-skinny orthonormalisation by CholeskyQR with an fp64 Gram, the cross-Gram used
// for the small SVD's input, and the "panel x small matrix" MFMA kernel used for Q = Y R^-1 and
// the back-projections U = Q U_w (src/rSVD.cpp:128) and V = Q_B V_w.
//
// The reference orthonormalises with Eigen::HouseholderQR + householderQ()*Identity
// (src/rSVD.cpp:60-61,64-65,67-68).  rSVD's outputs depend only on span(Q), so
// any numerically orthonormal basis of span(Y) is a drop-in.  One CholeskyQR pass is
//     G = Y^T Y (fp64 MFMA on exactly up-converted entries), R = chol(G), Q = Y R^-1 (fp64 MFMA)
// and CholeskyQR2 repeats it on Q.  Because Q is applied in fp64, span(Q) = span(Y) to working
// accuracy for ANY well-conditioned triangular R: the factorisation itself only has to make Q
// well conditioned, so on the fp32 path it runs in fp32 (4x shorter dependent-latency chains
// than fp64 on gfx950); the fp64 path factors in fp64.  A pivot below 1e-10 (fp64) / 1e-6 (fp32)
// of its original diagonal raises a device flag (rank loss / cond(Y) beyond the method's range).
// The small SVD does not use this R: it factors W = (Q_B^T B^T)^T computed exactly by the
// cross-Gram mode below, so its accuracy does not depend on the Cholesky precision.
//
// gram_kernel does the whole small side of a pass in ONE launch: every workgroup reduces its
// row block to partial 16x16 Gram tiles and publishes them (cdna_hip_programming.md §6
// Guideline 16: plain stores, per-wave vmcnt(0), barrier, agent release, relaxed counter add);
// one workgroup per tile waits for all slabs (bounded spin, agent acquire), sums its tile over
// the slabs in a FIXED order (bitwise reproducible) and publishes it; the last tile reducer
// assembles the Gram and (mode 1) factors it: R and R^-1 together by symmetric elimination on
// [G | I], register-tiled over 256 threads, one barrier per block of 4 pivots.
#include <algorithm>

#include "common.hpp"
#include "kernels.hpp"

namespace rsvd {

namespace {

constexpr int kGramWaves = 4;
constexpr int kMaxGramBlocks = 32;
// A final fp32 panel factored in fp64 is orthonormal to ~u64 cond(R)^2 after ONE pass: below this
// Frobenius condition estimate (u64 * 2e4^2 ~ 4e-8 < fp32 storage rounding) the second CholeskyQR
// pass is skipped (gram_kernel `refine`).
constexpr double kRefineCond = 2e4;  // plan_gram_blocks() cap: the tile reducers keep one load per slab in flight

template <int LP, bool FULL>
struct Tiles {
    static constexpr int G = LP / 16;
    static constexpr int NT = FULL ? G * G : G * (G + 1) / 2;  // full (cross) or upper tiles
};

__device__ __forceinline__ double rsqrt_c(double d) {
    const double y = __builtin_amdgcn_rsq(d);
    return y * (1.5 - 0.5 * d * y * y);
}
__device__ __forceinline__ float rsqrt_c(float d) {
    const float y = __builtin_amdgcn_rsqf(d);
    return y * (1.5f - 0.5f * d * y * y);
}
template <typename C> struct PivTol;
template <> struct PivTol<double> { static constexpr double v = 1e-10; };
template <> struct PivTol<float> { static constexpr double v = 1e-6; };

// ---- R = chol(G) and R^-1 together, all 256 threads, one barrier per 4 pivots ----------------
// Symmetric Gaussian elimination on [G | I]: after step k, row k of G is row k of D L^T and row k
// of the identity block is row k of L^-1 (G = L D L^T, L unit lower), so
//     R[k][j]     = M[k][j] / sqrt(M[k][k])        (j >= k)
//     R^-1[j][k]  = W[k][j] / sqrt(M[k][k])        (j <= k).
// Thread (ti, tj) of a 16 x 16 grid keeps M[i][j] and W[i][j] for i = ti + 16a, j = tj + 16b in
// registers (compute type C).  Pivots go in blocks of PB = 4: the owners publish the PB raw block
// rows (double-buffered LDS), then EVERY thread replays the PB elimination steps of the block on
// just the columns it needs -- its NB columns j, its NB rows i (by symmetry M[i][k] = M[k][i]) and
// the PB diagonal-block columns -- and applies the rank-PB update to its registers.  One barrier
// per block instead of per pivot; the replay is a few dozen redundant FMAs per thread.
// The padding is treated as [G_ll 0; 0 I]; outputs are zeroed outside the leading l x l block.
// LDS: rows (2 x 2 x PB x LP of C), d0 (LP of C), Rs and RIs (LP*LP doubles each).
constexpr int kPivBlock = 4;

// Pivots 16*AK .. 16*AK+15 (four blocks of PB).  AK is a compile-time constant, so the live
// register tiles are known: rows a < AK are finished, M's columns b < AK are dead, and W's rows
// are lower triangular (W[k][j] = 0 for j > k) so W only changes in columns b <= AK.
template <typename C, int LP, int AK>
__device__ __forceinline__ void chol_group(C (&M)[LP / 16][LP / 16], C (&W)[LP / 16][LP / 16], C* rows,
                                           const C* d0, double* Rs, double* RIs, int lend, int& buf, bool& bad) {
    constexpr int NB = LP / 16, PB = kPivBlock;
    const int tid = threadIdx.x;
    const int ti = tid >> 4, tj = tid & 15;
    for (int tk0 = 0; tk0 < 16; tk0 += PB, buf ^= 1) {
        const int k0 = 16 * AK + tk0;
        if (k0 >= lend) break;
        C* PMr = rows + buf * (2 * PB * LP);  // [PB][LP] raw block rows of M
        C* PWr = PMr + PB * LP;               // [PB][LP] raw block rows of W
        if (ti >= tk0 && ti < tk0 + PB) {
            const int t = ti - tk0;
#pragma unroll
            for (int b = AK; b < NB; ++b) PMr[t * LP + tj + 16 * b] = M[AK][b];
#pragma unroll
            for (int b = 0; b <= AK; ++b) PWr[t * LP + tj + 16 * b] = W[AK][b];
        }
        __syncthreads();
        // replay the block's PB steps on the needed columns (indices b / a below AK are dead)
        C pm[PB][NB], pr[PB][NB], pd[PB][PB], pw[PB][NB];
#pragma unroll
        for (int t = 0; t < PB; ++t) {
#pragma unroll
            for (int b = AK; b < NB; ++b) {
                pm[t][b] = PMr[t * LP + tj + 16 * b];
                pr[t][b] = PMr[t * LP + ti + 16 * b];
            }
#pragma unroll
            for (int b = 0; b <= AK; ++b) pw[t][b] = PWr[t * LP + tj + 16 * b];
#pragma unroll
            for (int u = 0; u < PB; ++u) pd[t][u] = PMr[t * LP + k0 + u];
        }
        C fr[PB][NB];
#pragma unroll
        for (int t = 0; t < PB; ++t) {
            const int k = k0 + t;
            C piv = pd[t][t];
            const C d0k = d0[k];
            const bool ok = (piv > (C)PivTol<C>::v * d0k) && (d0k > C(0)) && isfinite(piv);
            bad |= !ok;
            piv = ok ? piv : ((d0k > C(0) && isfinite(d0k)) ? d0k : C(1));  // keep going without NaNs; flagged
            const C inv = rsqrt_c(piv);
            const C ipiv = inv * inv;
            if (ti == t) {  // 16 writer threads per pivot row
                if (Rs) {
#pragma unroll
                    for (int b = AK; b < NB; ++b) {
                        const int j = tj + 16 * b;
                        Rs[k * LP + j] = (j >= k) ? (double)(pm[t][b] * inv) : 0.0;
                    }
                }
#pragma unroll
                for (int b = 0; b <= AK; ++b) {
                    const int j = tj + 16 * b;
                    RIs[j * LP + k] = (j <= k) ? (double)(pw[t][b] * inv) : 0.0;
                }
            }
            // multipliers of this thread's rows (i > k) for step t
#pragma unroll
            for (int a = AK; a < NB; ++a) fr[t][a] = (a > AK || ti > tk0 + t) ? pr[t][a] * ipiv : C(0);
            // eliminate column k from the later block rows s > t
#pragma unroll
            for (int s2 = t + 1; s2 < PB; ++s2) {
                const C f = pd[t][s2] * ipiv;
#pragma unroll
                for (int u = t + 1; u < PB; ++u) pd[s2][u] -= f * pd[t][u];
                pm[s2][AK] -= (tj > tk0 + t) ? f * pm[t][AK] : C(0);
                pr[s2][AK] -= (ti > tk0 + t) ? f * pr[t][AK] : C(0);
#pragma unroll
                for (int b = AK + 1; b < NB; ++b) {
                    pm[s2][b] -= f * pm[t][b];
                    pr[s2][b] -= f * pr[t][b];
                }
#pragma unroll
                for (int b = 0; b <= AK; ++b) pw[s2][b] -= f * pw[t][b];
            }
        }
        // rank-PB update of the live trailing registers
#pragma unroll
        for (int a = AK; a < NB; ++a) {
            {
                C mv = M[a][AK];
#pragma unroll
                for (int t = 0; t < PB; ++t) mv -= (tj > tk0 + t) ? fr[t][a] * pm[t][AK] : C(0);
                M[a][AK] = mv;
            }
#pragma unroll
            for (int b = AK + 1; b < NB; ++b) {
                C mv = M[a][b];
#pragma unroll
                for (int t = 0; t < PB; ++t) mv -= fr[t][a] * pm[t][b];
                M[a][b] = mv;
            }
#pragma unroll
            for (int b = 0; b <= AK; ++b) {
                C wv = W[a][b];
#pragma unroll
                for (int t = 0; t < PB; ++t) wv -= fr[t][a] * pw[t][b];
                W[a][b] = wv;
            }
        }
    }
}

template <typename C, int LP, int AK>
__device__ __forceinline__ void chol_groups(C (&M)[LP / 16][LP / 16], C (&W)[LP / 16][LP / 16], C* rows,
                                            const C* d0, double* Rs, double* RIs, int lend, int& buf, bool& bad) {
    if constexpr (AK < LP / 16) {
        if (16 * AK < lend) {
            chol_group<C, LP, AK>(M, W, rows, d0, Rs, RIs, lend, buf, bad);
            chol_groups<C, LP, AK + 1>(M, W, rows, d0, Rs, RIs, lend, buf, bad);
        }
    }
}

// Rs may be null (R itself not wanted); RIs always receives R^-1.
template <typename C, int LP>
__device__ __forceinline__ bool tile_cholesky_inverse(const double* Gs, C* rows, C* d0, double* Rs, double* RIs,
                                                      int l) {
    constexpr int NB = LP / 16;
    const int tid = threadIdx.x;
    const int ti = tid >> 4, tj = tid & 15;
    C M[NB][NB], W[NB][NB];
#pragma unroll
    for (int a = 0; a < NB; ++a)
#pragma unroll
        for (int b = 0; b < NB; ++b) {
            const int i = ti + 16 * a, j = tj + 16 * b;
            M[a][b] = (i < l && j < l) ? (C)Gs[i * LP + j] : ((i == j) ? C(1) : C(0));
            W[a][b] = (i == j) ? C(1) : C(0);
        }
    for (int e = tid; e < LP * LP; e += blockDim.x) {
        if (Rs) Rs[e] = 0.0;
        RIs[e] = 0.0;
    }
    for (int k = tid; k < LP; k += blockDim.x) d0[k] = (k < l) ? (C)Gs[k * LP + k] : C(1);
    bool bad = false;
    int buf = 0;
    const int lend = (l + kPivBlock - 1) / kPivBlock * kPivBlock;  // padded pivots beyond are exact 1s
    chol_groups<C, LP, 0>(M, W, rows, d0, Rs, RIs, lend, buf, bad);
    __syncthreads();
    return bad;
}

template <int LP>
__device__ __forceinline__ void write_factor(const double* Rs, const double* RIs, int l, double* __restrict__ Rout,
                                             double* __restrict__ Rinv) {
    for (int e = threadIdx.x; e < LP * LP; e += blockDim.x) {
        const int i = e / LP, j = e % LP;
        const bool in = i < l && j < l;
        if (Rout) Rout[e] = in ? Rs[e] : 0.0;
        Rinv[e] = in ? RIs[e] : 0.0;
    }
}

__device__ __forceinline__ bool spin_until(unsigned* ctr, unsigned target, int* tmo) {
    unsigned spins = 0;
    while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > (1u << 26)) {  // ~seconds: never expected; report (sticky word) instead of hanging
            atomicOr(tmo, 1);
            return false;
        }
    }
    return true;
}

// Doubles of LDS the factorisation phase needs (Gs + Rs + RIs, rows + d0).
template <int LP>
constexpr size_t factor_lds_doubles() { return (size_t)3 * LP * LP + (4 * kPivBlock + 1) * LP; }

// ------------------------------------------------------------------------------------------------
// grid = max(nb, NT) workgroups.  Phase 1 (blocks < nb): partial Gram of a row block -> slab
// (CROSS: P^T P2, all G x G tiles; else P^T P, upper tiles).  Phase 2 (blocks < NT): wait for all
// nb slabs (cumulative counter ctr[0] >= target0), reduce tile `blockIdx.x` over the slabs in fixed
// order.  Phase 3 (the last tile reducer, ctr[1] == target1 - 1): mode 1 factors (R, R^-1), mode 0
// writes the Gram (zero outside l x l) to Gsum.  Counters are zeroed by the driver at the start of
// every run; targets are run-cumulative (no in-kernel reset).
template <typename T, typename C, int LP, bool CROSS>
__global__ __launch_bounds__(kWave* kGramWaves) void gram_kernel(
    const T* __restrict__ P, const T* __restrict__ P2, int64_t rows, int64_t chunk, int nb,
    double* __restrict__ slabs, double* __restrict__ tiles, unsigned* __restrict__ ctr, unsigned target0,
    unsigned target1, int mode, double* __restrict__ Gsum, int l, double* __restrict__ Rout,
    double* __restrict__ Rinv, int* __restrict__ flag, int* __restrict__ tmo, const int* __restrict__ pred,
    int* __restrict__ refine) {
    constexpr int G = Tiles<LP, CROSS>::G, NT = Tiles<LP, CROSS>::NT;
    if (pred && *pred == 0) return;  // predicated pass (private counters: skipping disturbs no other launch)
    typedef Mfma<double> M;
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    double* red = reinterpret_cast<double*>(smem_raw);  // [kGramWaves][NT][256]
    constexpr size_t red_doubles = (size_t)kGramWaves * NT * 256;
    constexpr size_t area = red_doubles > factor_lds_doubles<LP>() ? red_doubles : factor_lds_doubles<LP>();
    int* ticket = reinterpret_cast<int*>(red + area);
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int r = lane & 15, h = lane >> 4;
    const int b = blockIdx.x;

    if (b < nb) {
        const int64_t rbeg = (int64_t)b * chunk;
        const int64_t rend = (rbeg + chunk < rows) ? rbeg + chunk : rows;
        f64x4 acc[NT];
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[t] = M::zero();
        constexpr int U = CROSS ? 2 : 4;  // k-steps (4 rows each) per wave per iteration, loads first
        for (int64_t i0 = rbeg + 4 * w; i0 < rend; i0 += 4 * kGramWaves * U) {
            double y[U][G], z[U][G];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int64_t i = i0 + 4 * kGramWaves * u + h;
#pragma unroll
                for (int g = 0; g < G; ++g) {
                    y[u][g] = (i < rend) ? (double)P[i * LP + 16 * g + r] : 0.0;
                    z[u][g] = (CROSS && i < rend) ? (double)P2[i * LP + 16 * g + r] : 0.0;
                }
            }
#pragma unroll
            for (int u = 0; u < U; ++u) {
                int t = 0;
#pragma unroll
                for (int a = 0; a < G; ++a)
#pragma unroll
                    for (int bb = (CROSS ? 0 : a); bb < G; ++bb, ++t)
                        acc[t] = M::mma(y[u][a], CROSS ? z[u][bb] : y[u][bb], acc[t]);
            }
        }
        // tile (a, bb) element (row 16a + R, col 16bb + C) sits at red[w][t][R*16 + C]
        double* mine = red + (size_t)w * NT * 256;
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) mine[t * 256 + M::row(h, jj) * 16 + r] = acc[t][jj];
        __syncthreads();
        double* myslab = slabs + (size_t)b * NT * 256;
        for (int e = threadIdx.x; e < NT * 256; e += blockDim.x) {
            double s = 0.0;
#pragma unroll
            for (int ww = 0; ww < kGramWaves; ++ww) s += red[(size_t)ww * NT * 256 + e];
            myslab[e] = s;
        }
        // publish (cdna_hip_programming.md §6 Guideline 16, counter form)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    if (b >= NT) return;
    // ---- phase 2: tile reducer ----
    if (threadIdx.x == 0) {
        *ticket = spin_until(ctr, target0, tmo) ? 1 : 0;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    if (*ticket == 0) return;
    {
        const int e = threadIdx.x;  // 256 elements per tile, one per thread
        // every slab load in flight at once (nb <= kMaxGramBlocks): one L2 round trip instead
        // of nb / 4 dependent ones; then a fixed-order sum (bitwise reproducible)
        double v[kMaxGramBlocks];
#pragma unroll
        for (int sb = 0; sb < kMaxGramBlocks; ++sb)
            v[sb] = (sb < nb) ? slabs[(size_t)sb * NT * 256 + b * 256 + e] : 0.0;
        double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
#pragma unroll
        for (int sb = 0; sb < kMaxGramBlocks; sb += 4) {
            s0 += v[sb];
            s1 += v[sb + 1];
            s2 += v[sb + 2];
            s3 += v[sb + 3];
        }
        tiles[b * 256 + e] = (s0 + s1) + (s2 + s3);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned tk = __hip_atomic_fetch_add(ctr + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *ticket = (tk == target1 - 1) ? 1 : 0;
        if (*ticket) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
    }
    __syncthreads();
    if (*ticket == 0) return;
    // ---- phase 3: the last tile reducer assembles the Gram ----
    double* Gs = red;                    // [LP][LP]   (reuses the reduction area)
    double* Rs = Gs + LP * LP;           // [LP][LP]
    double* RIs = Rs + LP * LP;          // [LP][LP]
    C* prow = reinterpret_cast<C*>(RIs + LP * LP);  // [2][2][PB][LP]
    C* d0 = prow + 4 * kPivBlock * LP;              // [LP]
    for (int e = threadIdx.x; e < NT * 256; e += blockDim.x) {
        const double s = tiles[e];
        int t = e >> 8, a = 0, bb;
        if (CROSS) {
            a = t / G;
            bb = t % G;
        } else {
            while (t >= G - a) { t -= G - a; ++a; }
            bb = a + t;
        }
        const int R_ = (e & 255) >> 4, C_ = e & 15;
        const int row = 16 * a + R_, col = 16 * bb + C_;
        Gs[row * LP + col] = s;
        if (!CROSS) Gs[col * LP + row] = s;
    }
    __syncthreads();
    if (mode == 0) {
        for (int e = threadIdx.x; e < LP * LP; e += blockDim.x) {
            const int row = e / LP, col = e % LP;
            Gsum[e] = (row < l && col < l) ? Gs[e] : 0.0;
        }
        return;
    }
    const bool bad = tile_cholesky_inverse<C, LP>(Gs, prow, d0, Rout ? Rs : nullptr, RIs, l);
    write_factor<LP>(Rs, RIs, l, Rout, Rinv);
    if (threadIdx.x == 0 && bad) atomicAdd(flag, 1);
    if (refine) {
        // cond_F(R) = |R|_F |R^-1|_F >= cond_2(R): one pass left Q orthonormal to ~u cond^2, so a
        // second pass is requested when that exceeds what the panel's storage precision resolves
        double a = 0.0, c = 0.0;
        for (int e = threadIdx.x; e < LP * LP; e += blockDim.x) {
            const int i = e / LP, j = e % LP;
            if (i < l && j < l) {
                a += Rs[e] * Rs[e];
                c += RIs[e] * RIs[e];
            }
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            a += __shfl_xor(a, o);
            c += __shfl_xor(c, o);
        }
        double* part = reinterpret_cast<double*>(prow);
        if (lane == 0) {
            part[w] = a;
            part[kGramWaves + w] = c;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            double sa = 0.0, sc = 0.0;
            for (int t = 0; t < kGramWaves; ++t) {
                sa += part[t];
                sc += part[kGramWaves + t];
            }
            const double cond = sqrt(sa * sc);
            *refine = (bad || !(cond <= kRefineCond)) ? 1 : 0;
        }
    }
}

// Factor an already-summed Gram (distributed path: after the all-reduce).
template <typename C, int LP>
__global__ __launch_bounds__(256) void chol_kernel(const double* __restrict__ Gin, int l, double* __restrict__ Rout,
                                                   double* __restrict__ Rinv, int* __restrict__ flag) {
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    double* Gs = reinterpret_cast<double*>(smem_raw);
    double* Rs = Gs + LP * LP;
    double* RIs = Rs + LP * LP;
    C* prow = reinterpret_cast<C*>(RIs + LP * LP);
    C* d0 = prow + 4 * kPivBlock * LP;
    for (int e = threadIdx.x; e < LP * LP; e += blockDim.x) {
        const int row = e / LP, col = e % LP;
        Gs[e] = (row < l && col < l) ? Gin[e] : 0.0;
    }
    __syncthreads();
    const bool bad = tile_cholesky_inverse<C, LP>(Gs, prow, d0, Rout ? Rs : nullptr, RIs, l);
    write_factor<LP>(Rs, RIs, l, Rout, Rinv);
    if (threadIdx.x == 0 && bad) atomicAdd(flag, 1);
}

// Out = In * M (M: LP x LP fp64): one wave per 16 x 16 output tile (rows/16 x LP/16 waves, four
// per workgroup), so even a 4096-row panel spreads over every CU.  A wave issues all of its
// operand loads at once -- LP/4 In values (converted to fp64) and LP/4 M values per lane, M
// being L2-resident -- and then runs LP/4 f64 MFMAs: applying R^-1 in fp64 keeps storage
// rounding from being amplified by cond(R); only the result is rounded to T.
template <typename T, int LP>
__global__ __launch_bounds__(256) void panel_small_kernel(const T* __restrict__ In, int64_t rows,
                                                          const double* __restrict__ Mg, T* __restrict__ Out,
                                                          int out_colmajor, int cols, int64_t ld,
                                                          const int* __restrict__ pred) {
    if (pred && *pred == 0) return;
    typedef Mfma<double> M;
    constexpr int G = LP / 16, KS = LP / 4;
    const int lane = threadIdx.x & 63;
    const int r = lane & 15, h = lane >> 4;
    const int64_t wave = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int g = (int)(wave % G);
    const int64_t r0 = (wave / G) * 16;
    if (r0 >= rows) return;
    const int64_t arow = r0 + r;
    double a[KS], b[KS];
#pragma unroll
    for (int k = 0; k < KS; ++k) {
        a[k] = (arow < rows) ? (double)In[arow * LP + 4 * k + h] : 0.0;
        b[k] = Mg[(4 * k + h) * LP + 16 * g + r];
    }
    f64x4 acc = M::zero();
#pragma unroll
    for (int k = 0; k < KS; ++k) acc = M::mma(a[k], b[k], acc);
    const int col = 16 * g + r;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int64_t row = r0 + M::row(h, j);
        if (row >= rows) continue;
        if (!out_colmajor)
            Out[row * LP + col] = (T)acc[j];
        else if (col < cols)
            Out[row + (int64_t)col * ld] = (T)acc[j];
    }
}

template <int LP, bool CROSS>
size_t gram_lds_bytes() {
    const size_t red = (size_t)kGramWaves * Tiles<LP, CROSS>::NT * 256;
    return std::max(red, factor_lds_doubles<LP>()) * sizeof(double) + 16;
}

template <typename T, typename C, int LP, bool CROSS>
hipError_t gram_launch(const T* P, const T* P2, int64_t rows, int nb, double* slabs, double* tiles, unsigned* ctr,
                       unsigned t0, unsigned t1, int mode, double* Gsum, int l, double* R, double* Rinv, int* flag,
                       int* tmo, hipStream_t s, const int* pred = nullptr, int* refine = nullptr) {
    const int64_t chunk = (rows + nb - 1) / nb;
    const int NT = Tiles<LP, CROSS>::NT;
    const int grid = nb > NT ? nb : NT;
    hipLaunchKernelGGL((gram_kernel<T, C, LP, CROSS>), dim3(grid), dim3(kWave * kGramWaves), (gram_lds_bytes<LP, CROSS>()),
                       s, P, P2, rows, chunk, nb, slabs, tiles, ctr, t0, t1, mode, Gsum, l, R, Rinv, flag, tmo, pred, refine);
    return hipGetLastError();
}

}  // namespace

int plan_gram_blocks(int64_t rows) {
    int64_t blocks = (rows + 127) / 128;  // >= 128 rows per workgroup
    if (blocks > kMaxGramBlocks) blocks = kMaxGramBlocks;
    if (blocks < 1) blocks = 1;
    return (int)blocks;
}

int gram_tiles(int LP, int cross) {
    const int G = LP / 16;
    return cross ? G * G : G * (G + 1) / 2;
}

template <typename T>
hipError_t launch_gram_chol(const T* P, int64_t rows, int LP, int nb, double* slabs, double* tiles, unsigned* ctr,
                            unsigned t0, unsigned t1, int mode, int compute_f32, double* Gsum, int l, double* R,
                            double* Rinv, int* flag, int* tmo, hipStream_t s, const int* pred, int* refine) {
    switch (LP) {
#define CASE(L)                                                                                                   \
    case L:                                                                                                       \
        return compute_f32 ? gram_launch<T, float, L, false>(P, nullptr, rows, nb, slabs, tiles, ctr, t0, t1, mode, \
                                                              Gsum, l, R, Rinv, flag, tmo, s, pred, refine)        \
                           : gram_launch<T, double, L, false>(P, nullptr, rows, nb, slabs, tiles, ctr, t0, t1, mode, \
                                                               Gsum, l, R, Rinv, flag, tmo, s, pred, refine);
        CASE(16) CASE(32) CASE(48) CASE(64)
#undef CASE
        default: return hipErrorInvalidValue;
    }
}

template <typename T>
hipError_t launch_cross_gram(const T* P, const T* P2, int64_t rows, int LP, int nb, double* slabs, double* tiles,
                             unsigned* ctr, unsigned t0, unsigned t1, double* Gout, int l, int* tmo, hipStream_t s) {
    switch (LP) {
#define CASE(L)                                                                                                 \
    case L:                                                                                                     \
        return gram_launch<T, double, L, true>(P, P2, rows, nb, slabs, tiles, ctr, t0, t1, 0, Gout, l, nullptr, \
                                               nullptr, nullptr, tmo, s);
        CASE(16) CASE(32) CASE(48) CASE(64)
#undef CASE
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_chol(const double* G, int l, int LP, int compute_f32, double* R, double* Rinv, int* flag,
                       hipStream_t s) {
    const size_t lds = factor_lds_doubles<64>() * sizeof(double) + 16;
    switch (LP) {
#define CASE(L)                                                                                                    \
    case L:                                                                                                        \
        if (compute_f32)                                                                                           \
            hipLaunchKernelGGL((chol_kernel<float, L>), dim3(1), dim3(256), lds, s, G, l, R, Rinv, flag);          \
        else                                                                                                       \
            hipLaunchKernelGGL((chol_kernel<double, L>), dim3(1), dim3(256), lds, s, G, l, R, Rinv, flag);         \
        break;
        CASE(16) CASE(32) CASE(48) CASE(64)
#undef CASE
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

template <typename T>
hipError_t launch_panel_small(const T* In, int64_t rows, int LP, const double* Mat, T* Out, int out_colmajor,
                              int cols, int64_t ld, hipStream_t s, const int* pred) {
    const int64_t waves = (rows + 15) / 16 * (LP / 16);
    const int blocks = (int)((waves + 3) / 4);
    switch (LP) {
#define CASE(L)                                                                                          \
    case L:                                                                                              \
        hipLaunchKernelGGL((panel_small_kernel<T, L>), dim3(blocks), dim3(256), 0, s, In, rows, Mat, Out, \
                           out_colmajor, cols, ld, pred);                                                \
        break;
        CASE(16) CASE(32) CASE(48) CASE(64)
#undef CASE
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

#define RSVD_INST(T)                                                                                             \
    template hipError_t launch_gram_chol<T>(const T*, int64_t, int, int, double*, double*, unsigned*, unsigned,    \
                                            unsigned, int, int, double*, int, double*, double*, int*, int*, hipStream_t, \
                                            const int*, int*);                                                    \
    template hipError_t launch_cross_gram<T>(const T*, const T*, int64_t, int, int, double*, double*, unsigned*,   \
                                             unsigned, unsigned, double*, int, int*, hipStream_t);               \
    template hipError_t launch_panel_small<T>(const T*, int64_t, int, const double*, T*, int, int, int64_t,       \
                                              hipStream_t, const int*);
RSVD_INST(float)
RSVD_INST(double)
#undef RSVD_INST

}  // namespace rsvd
