// wide_qr.hip -- tall-skinny orthonormalisation for sketch widths up to 512 (gfx950).
//
// The reference takes a Householder thin Q of every tall-skinny panel (src/rSVD.cpp:60-61,
// 64-65, 67-68); only span(Q) reaches the outputs.  Here: CholeskyQR(2) --
//   G = P^T P            gram_wide_kernel: fp64 MFMA (v_mfma_f64_16x16x4_f64) on 32 x 32 blocks of
//                        the upper triangle, one wave per (block, row chunk), + a fixed-order
//                        chunk reduction (deterministic);
//   R = chol(G), R^-1    chol_wide_kernel: ONE workgroup, 16-column blocks, fp64 MFMA trailing
//                        updates, breakdown detection per pivot;
//   Q = P R^-1           panel_gemm_kernel: fp32 MFMA (fp64 for fp64 panels) that also writes the
//                        bf16 hi/lo panels the next projection reads (wide_proj.hip) and, for the
//                        final U = Q U_w / V = Q_B V_w, the caller's column-major matrix.
// Rank deficiency (a pivot below tol * G_kk): R row k := e_k and column k is flagged; the
// driver then replaces flagged columns by Philox Gaussian vectors and re-orthonormalises
// (repair_kernel + one predicated CholeskyQR pass) -- an orthonormal basis completed like the
// reference's Householder Q.
#include <algorithm>
#include <cstdlib>
#include <string>
#include <utility>

#include "common.hpp"
#include "dense.hpp"
#include "kernels.hpp"
#include "wide.hpp"

namespace rsvd {

namespace {

typedef Mfma<double> MD;

constexpr bool gram_sym_ok(int LP) { return LP == 64 || LP == 128 || LP == 256 || LP == 512; }

template <typename T> struct Pair;
template <> struct Pair<float> { typedef float2 type; };
template <> struct Pair<double> { typedef double2 type; };

// ------------------------------------------------------------------------------------------------
// Gram: one wave per (32x32 block, row chunk).  Tile (ta, tb) of the block holds columns
// a0 + 2i + ta (i = MFMA row) and b0 + 2j + tb (j = MFMA col): each lane's 2-element vector load
// feeds both tiles of its side.
template <typename T, bool CROSS>
__global__ __launch_bounds__(256) void gram_wide_kernel(const T* __restrict__ P, const T* __restrict__ P2,
                                                        int64_t rows, int LP, int nblk, int nchunk, int64_t rpc,
                                                        double* __restrict__ slabs, const int* __restrict__ pred) {
    if (pred && *pred == 0) return;
    typedef typename Pair<T>::type V2;
    const int lane = threadIdx.x & 63;
    const int gw = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int blk = gw % nblk, chunk = gw / nblk;
    if (chunk >= nchunk) return;
    const int nb = (LP + 31) / 32;
    int a, b;
    if (CROSS) {
        a = blk / nb;
        b = blk % nb;
    } else {
        int rem = blk;
        a = 0;
        while (rem >= nb - a) {
            rem -= nb - a;
            ++a;
        }
        b = a + rem;
    }
    const int r = lane & 15, h = lane >> 4;
    const int ca = 32 * a + 2 * r, cb = 32 * b + 2 * r;
    const bool oka = ca < LP, okb = cb < LP;  // LP is a multiple of 16: pairs never straddle it
    const int64_t beg = (int64_t)chunk * rpc;
    const int64_t end = (beg + rpc < rows) ? beg + rpc : rows;
    f64x4 acc[2][2];
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y) acc[x][y] = MD::zero();
    for (int64_t i0 = beg; i0 < end; i0 += 16) {
        V2 va[4], vb[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int64_t row = i0 + 4 * u + h;
            va[u].x = va[u].y = vb[u].x = vb[u].y = T(0);
            if (row < end) {
                if (oka) va[u] = *reinterpret_cast<const V2*>(P + row * LP + ca);
                if (okb) vb[u] = *reinterpret_cast<const V2*>((CROSS ? P2 : P) + row * LP + cb);
            }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const double a0 = (double)va[u].x, a1 = (double)va[u].y;
            const double b0 = (double)vb[u].x, b1 = (double)vb[u].y;
            acc[0][0] = MD::mma(a0, b0, acc[0][0]);
            acc[0][1] = MD::mma(a0, b1, acc[0][1]);
            acc[1][0] = MD::mma(a1, b0, acc[1][0]);
            acc[1][1] = MD::mma(a1, b1, acc[1][1]);
        }
    }
    double* dst = slabs + ((int64_t)chunk * nblk + blk) * 1024;
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int i = MD::row(h, j);
                dst[(2 * i + x) * 32 + 2 * r + y] = acc[x][y][j];
            }
}

// ------------------------------------------------------------------------------------------------
// Symmetric Gram of a tall panel, LP in {64, 128, 256}: ONE 512-thread workgroup per row chunk reads
// its rows once (16-B loads, register-prefetched one step ahead, staged in LDS 32 rows per step) and
// computes every upper 16x16 tile pair (ta <= tb) of the chunk on the fp64 MFMA (LP = 256: two workgroups per chunk).  For G = P^T P both
// MFMA operands are "row k, column c" reads of the panel (A: P^T[c][k], B: P[k][c]), so a tile pair
// costs two LDS reads per 4 rows.  Pairs are dealt round-robin to the waves (9 per wave at
// LP = 256).  The old kernel gave each 32x32 block its own wave and chunk walk, re-reading every
// panel row LP/32 + 1 times from HBM; here each byte is read once and the MFMA issue rate is the
// bound.  Partial tiles land in the (chunk, 32x32 block) slab layout gram_reduce4_kernel sums; the
// lower 16x16 sub-tile of a diagonal 32x32 block is written as the transpose of the upper one.
// (ta, tb) of upper tile pair p (row-major over the upper triangle of NT x NT tiles); p >= NP -> (0, 0)
constexpr int pair_ta(int NT, int p) {
    if (p >= NT * (NT + 1) / 2) return 0;
    int a = 0;
    while (p >= NT - a) { p -= NT - a; ++a; }
    return a;
}
constexpr int pair_tb(int NT, int p) {
    if (p >= NT * (NT + 1) / 2) return 0;
    int a = 0;
    while (p >= NT - a) { p -= NT - a; ++a; }
    return a + p;
}

template <int NT, int P> struct PairOf {  // forces compile-time evaluation of the tile indices
    static constexpr int a = pair_ta(NT, P), b = pair_tb(NT, P);
};

template <int LP> struct GramSym {
    static constexpr int NH = LP == 512 ? 8 : (LP == 256 ? 2 : 1);  // workgroups per chunk
    static constexpr int LNH = LP == 512 ? 3 : (LP == 256 ? 1 : 0);
    // panel rows per LDS step (static LDS <= 64 KB)
    template <typename T> static constexpr int rs() { return LP == 512 ? (sizeof(T) == 8 ? 8 : 16) : ((sizeof(T) == 8 && LP == 256) ? 16 : 32); }
    static constexpr int NT = LP / 16, NP = NT * (NT + 1) / 2, NW = 8 * NH, PPW = (NP + NW - 1) / NW;
    static constexpr int NB = LP / 32, NBLK = NB * (NB + 1) / 2;
};

// slot I of dealer WG: pair WG + NW I (compile-time tile indices, so v[] stays in registers)
template <int LP, int WG, int... I>
__device__ __forceinline__ void gram_sym_mma(const double (&v)[LP / 16], f64x4 (&acc)[GramSym<LP>::PPW],
                                             std::integer_sequence<int, I...>) {
    typedef GramSym<LP> G;
    ((acc[I] = (WG + G::NW * I < G::NP) ? MD::mma(v[PairOf<G::NT, WG + G::NW * I>::a], v[PairOf<G::NT, WG + G::NW * I>::b], acc[I])
                                        : acc[I]),
     ...);
}

// does dealer WG touch tile t?
template <int LP, int WG>
constexpr bool gram_sym_needs(int t) {
    typedef GramSym<LP> G;
    for (int i = 0; i < G::PPW; ++i)
        if (WG + G::NW * i < G::NP && (pair_ta(G::NT, WG + G::NW * i) == t || pair_tb(G::NT, WG + G::NW * i) == t))
            return true;
    return false;
}

template <int LP, int WG, int t> struct NeedOf {  // compile-time gram_sym_needs
    static constexpr bool value = gram_sym_needs<LP, WG>(t);
};
// the panel values of the tiles dealer WG touches, for the 4 rows of one MFMA step
template <typename T, int LP, int WG, int... I>
__device__ __forceinline__ void gram_sym_loadv(const T* rowp, double (&v)[LP / 16], std::integer_sequence<int, I...>) {
    ((v[I] = NeedOf<LP, WG, I>::value ? (double)rowp[16 * I] : 0.0), ...);
}

template <typename T, int LP, int WG>
__device__ __forceinline__ void gram_sym_body(const T* __restrict__ P, int64_t beg, int64_t end, int chunk,
                                              double* __restrict__ slabs, T* tile) {
    typedef GramSym<LP> G;
    constexpr int NT = G::NT, PPW = G::PPW, NTH = 512;
    constexpr int RS = G::template rs<T>();  // panel rows per step
    constexpr int VE = 16 / sizeof(T);                            // elements per 16-B load
    constexpr int CPR = LP / VE;                                  // 16-B chunks per row
    constexpr int LPT = RS * CPR / NTH;                           // loads per thread per step
    static_assert(LPT >= 1 && (RS * CPR) % NTH == 0, "step tiling");
    constexpr int PITCH = LP + 64 / (int)sizeof(T);  // row pitch: the 4 rows of an MFMA read hit different banks
    typedef typename Vec16<T>::type V;
    const int tid = threadIdx.x, lane = tid & 63;
    const int r = lane & 15, h = lane >> 4;
    f64x4 acc[PPW];
#pragma unroll
    for (int i = 0; i < PPW; ++i) acc[i] = MD::zero();

    V reg[LPT];
    auto load = [&](int64_t r0) {
#pragma unroll
        for (int t = 0; t < LPT; ++t) {
            const int u = tid + NTH * t;
            const int64_t row = r0 + u / CPR;
            V v;
            if constexpr (sizeof(T) == 4) v = make_float4(0.f, 0.f, 0.f, 0.f);
            else v = make_double2(0.0, 0.0);
            if (row < end) v = *reinterpret_cast<const V*>(P + row * LP + (u % CPR) * VE);
            reg[t] = v;
        }
    };
    if (beg < end) load(beg);
    for (int64_t r0 = beg; r0 < end; r0 += RS) {
        __syncthreads();  // the previous step's LDS reads are done
#pragma unroll
        for (int t = 0; t < LPT; ++t) {
            const int u = tid + NTH * t;
            *reinterpret_cast<V*>(tile + (u / CPR) * PITCH + (u % CPR) * VE) = reg[t];
        }
        __syncthreads();
        if (r0 + RS < end) load(r0 + RS);
#pragma unroll 2
        for (int g = 0; g < RS / 4; ++g) {
            const T* rowp = tile + (4 * g + h) * PITCH + r;
            double v[NT];
            gram_sym_loadv<T, LP, WG>(rowp, v, std::make_integer_sequence<int, NT>{});
            gram_sym_mma<LP, WG>(v, acc, std::make_integer_sequence<int, PPW>{});
        }
    }

#pragma unroll
    for (int i = 0; i < PPW; ++i) {
        const int p = WG + G::NW * i;
        if (p < G::NP) {
            const int ta = pair_ta(NT, p), tb = pair_tb(NT, p);
            const int a = ta >> 1, b = tb >> 1;
            const int blk = a * G::NB - a * (a - 1) / 2 + (b - a);
            double* dst = slabs + ((int64_t)chunk * G::NBLK + blk) * 1024;
            const bool mirror = (a == b) && (ta != tb);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int li = 16 * (ta & 1) + MD::row(h, j), lj = 16 * (tb & 1) + r;
                dst[li * 32 + lj] = acc[i][j];
                if (mirror) dst[lj * 32 + li] = acc[i][j];
            }
        }
    }
}

template <typename T, int LP, int... W>
__device__ __forceinline__ void gram_sym_dispatch(int wg, const T* P, int64_t beg, int64_t end, int chunk, double* slabs,
                                                  T* tile, std::integer_sequence<int, W...>) {
    ((wg == W ? gram_sym_body<T, LP, W>(P, beg, end, chunk, slabs, tile) : void()), ...);
}

template <typename T, int LP>
__global__ __launch_bounds__(512) void gram_sym_kernel(const T* __restrict__ P, int64_t rows, int64_t rpc, int nchunk,
                                                       double* __restrict__ slabs, const int* __restrict__ pred) {
    if (pred && *pred == 0) return;
    typedef GramSym<LP> G;
    // NH workgroups share a chunk (LP = 256: 2, LP = 512: 8, dealing the pairs between them), all on one
    // XCD (block ids b, b + 8, ...) so the repeated reads of the rows are L2 hits.
    constexpr int RS = G::template rs<T>();
    constexpr int PITCH = LP + 64 / (int)sizeof(T);
    __shared__ __attribute__((aligned(16))) T tile[RS * PITCH];
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform: scalar branch to the dealer body
    const int hb = G::NH == 1 ? 0 : (blockIdx.x >> 3) & (G::NH - 1);
    const int chunk = G::NH == 1 ? blockIdx.x : ((blockIdx.x & 7) | ((blockIdx.x >> (3 + G::LNH)) << 3));
    if (chunk >= nchunk) return;
    const int64_t beg = (int64_t)chunk * rpc;
    const int64_t end = (beg + rpc < rows) ? beg + rpc : rows;
    // dealer index: pairs WG, WG + NW, ... belong to wave w of half hb
    gram_sym_dispatch<T, LP>(w * G::NH + hb, P, beg, end, chunk, slabs, tile, std::make_integer_sequence<int, G::NW>{});
}

// ------------------------------------------------------------------------------------------------
// Split Gram of an fp32 panel on the bf16 MFMA.  Every fp32 value is EXACTLY h + m + t with
// h = bf16(v), m = bf16(v - h), t = bf16(v - h - m) (8 + 8 + 8 significant bits), and the six
// products hh, hm, mh, mm, ht, th carry P_ki P_kj to ~2^-24 of |P_ki P_kj| (the dropped mt, tm,
// tt are below it).  Each bf16 product is exact in fp32; the v_mfma_f32_16x16x32_bf16 chains sum a
// row chunk (<= 1024 rows at the configs' sizes) in fp32 and the chunk partials are summed in fp64,
// so the rounding does not grow with the panel height: numpy model of the same arithmetic on a
// cond 1e3 panel (65536 x 256): |G_split - G|_F / |G|_F ~ 1e-8, max |dG_ij| / sqrt(G_ii G_jj) ~ 3e-8.  Six bf16 MFMAs at 32x the fp64 MFMA rate: the Gram becomes an HBM read of the panel
// (C4 65536 x 256: ~100 -> ~20 us).  It is only used where its accuracy is enough -- CholeskyQR of
// the fp32 panels of bf16 / e4m3 A, with the factor's pivots checked against kSplitIllTol
// (launch_chol_wide, `ill`) and the fp64 Gram + factor re-run (predicated) when one is below it.
// Layout: a 32-row step is staged as three [LP column][32 row] bf16 images (64-B columns, 16-B
// unit u of column c at u ^ ((c >> 1) & 3): the 16-lane ds_read_b128 of one tile is conflict-free);
// lane (r, h) of tile t reads rows 8h .. 8h + 7 of column 16t + r -- the A and the B fragment of
// v_mfma_f32_16x16x32_bf16 alike (G = P^T P: both operands are "column, rows k" reads).
// Upper tile pairs (ta <= tb) are dealt to the NH x 8 waves of a chunk at compile time; the
// partial tiles go to gram_sym's (chunk, 32x32 block) slab layout, summed by gram_reduce4_kernel.
typedef __attribute__((ext_vector_type(8))) short bf16x8s;

// Work split: the tiles are cut into groups of TG (4; 2 at LP = 128) and each wave owns one
// group pair (A <= B) -- TG x TG tile pairs whose A-side fragments stay in registers for the step
// while the B-side ones stream (each fragment feeds TG x 6 MFMAs: ~0.25 KB of LDS reads per MFMA;
// one fragment pair per tile pair read 1 KB per MFMA and made the kernel LDS-bound).  Diagonal
// group pairs compute their TG^2 tile pairs in full and store the upper ones.  The fp32 MFMA
// accumulators run over the whole row chunk (<= 1024 rows for the panels of the bf16 / e4m3
// configs) and the chunk partials are summed in fp64 by gram_reduce4_kernel.
template <int LP> struct GramSplit {
    static constexpr int TG = LP == 128 ? 2 : 4;
    static constexpr int NT = LP / 16, NTG = NT / TG, NBK = NTG * (NTG + 1) / 2;
    static constexpr int NH = LP == 512 ? 4 : 1;  // workgroups per chunk
    static constexpr int LNH = LP == 512 ? 2 : 0;
    static constexpr int NWW = NBK / NH;          // waves per workgroup (10, 10, 9)
    static constexpr int THREADS = 64 * NWW;
    static constexpr int NB = LP / 32, NBLK = NB * (NB + 1) / 2;
    static constexpr int IMG = LP * 64;           // bytes of one piece image (LP columns x 32 rows bf16)
    static constexpr int STEP = 3 * IMG;          // the three pieces of a 32-row step
    static constexpr int NBUF = STEP * 2 <= 98304 ? 2 : 1;
    static constexpr int NU = 2 * LP;             // 4-row x 4-column units of a 32-row step
    static constexpr int LPT = (NU + THREADS - 1) / THREADS;
    static_assert(NBK % NH == 0, "group pairs per workgroup");
};

// two fp32 -> packed bf16 (round to nearest even): lo = a, hi = b
__device__ __forceinline__ uint32_t cvt_pk_bf16(float a, float b) {
    uint32_t r;
    asm volatile("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

// Loader groups (round 4): the NU units of a step are loaded by GSZ = NU / LPTG threads, LPTG units
// each; NLG such groups take the steps round robin, so a group issues its next load NLG steps ahead
// of the step it stages.  <1, 1> is the original one-step prefetch; at LP = 128 one step is 16 KB per
// CU and the 1-step prefetch left the kernel waiting on HBM latency (205 us for a 2^20-row panel).
template <int LP, int LPTG = GramSplit<LP>::LPT, int NLG = 1>
__global__ __launch_bounds__(GramSplit<LP>::THREADS) void gram_split_kernel(const float* __restrict__ P, int64_t rows,
                                                                          int64_t rpc, int nchunk,
                                                                          double* __restrict__ slabs) {
    typedef GramSplit<LP> G;
    constexpr int TG = G::TG, LPT = LPTG;
    constexpr int GSZ = (G::NU + LPTG - 1) / LPTG;  // threads of one loader group
    static_assert(NLG == 1 || (GSZ % 64 == 0 && NLG * GSZ <= G::THREADS), "loader groups");
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    const int tid = threadIdx.x, lane = tid & 63, r = lane & 15, h = lane >> 4;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int hb = G::NH == 1 ? 0 : (blockIdx.x >> 3) & (G::NH - 1);
    const int chunk = G::NH == 1 ? blockIdx.x : ((blockIdx.x & 7) | ((blockIdx.x >> (3 + G::LNH)) << 3));
    if (chunk >= nchunk) return;
    const int64_t beg = (int64_t)chunk * rpc;
    const int64_t end = (beg + rpc < rows) ? beg + rpc : rows;
    // this wave's group pair (GA <= GB), row-major over the upper triangle of NTG x NTG
    int GA = 0, GB = 0;
    {
        int rem = hb * G::NWW + w;
        while (rem >= G::NTG - GA) {
            rem -= G::NTG - GA;
            ++GA;
        }
        GB = GA + rem;
    }
    f32x4 acc[TG][TG];
#pragma unroll
    for (int i = 0; i < TG; ++i)
#pragma unroll
        for (int j = 0; j < TG; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    // thread unit u = tid + THREADS t (u < NU): rows kr = 4 (u & 7) .. + 3 of columns 4 (u >> 3) .. + 3
    float4 reg[LPT][4];
    // (the unit guard is wave-uniform -- NU is a multiple of 64 -- and a full step loads unguarded: a
    // per-load guard compiled to an exec branch per load; the partial last step clamps and zeroes)
    auto load = [&](int64_t r0) {
        const bool full = r0 + 32 <= end;
#pragma unroll
        for (int t = 0; t < LPT; ++t) {
            const int u = (NLG == 1 ? tid : tid % GSZ) + (NLG == 1 ? G::THREADS : GSZ) * t;
            if (u - lane >= G::NU) break;
            const int64_t row = r0 + 4 * (u & 7);
            const int c = 4 * (u >> 3);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                if (full) {
                    reg[t][q] = *reinterpret_cast<const float4*>(P + (row + q) * LP + c);
                } else {
                    const int64_t rr = row + q < end ? row + q : end - 1;
                    const float4 x = *reinterpret_cast<const float4*>(P + rr * LP + c);
                    reg[t][q] = row + q < end ? x : make_float4(0.f, 0.f, 0.f, 0.f);
                }
            }
        }
    };
    auto stage = [&](char* img) {
#pragma unroll
        for (int t = 0; t < LPT; ++t) {
            const int u = (NLG == 1 ? tid : tid % GSZ) + (NLG == 1 ? G::THREADS : GSZ) * t;
            if (u >= G::NU) break;
            const int kr = 4 * (u & 7);
            const int c0 = 4 * (u >> 3);
            const int rot = (u >> 3) & 3;  // octets write columns of alternating parity (LDS banks)
#pragma unroll
            for (int i0 = 0; i0 < 4; ++i0) {
                const int i = (i0 + rot) & 3;
                const int c = c0 + i;
                uint32_t pw[3][2];
#pragma unroll
                for (int q = 0; q < 4; q += 2) {
                    const float4 f0 = reg[t][q], f1 = reg[t][q + 1];
                    const float a = i == 0 ? f0.x : (i == 1 ? f0.y : (i == 2 ? f0.z : f0.w));
                    const float b = i == 0 ? f1.x : (i == 1 ? f1.y : (i == 2 ? f1.z : f1.w));
                    // exact three-piece split, two rows at a time: h = bf16(v), m = bf16(v - h), t = v - h - m
                    const uint32_t ph = cvt_pk_bf16(a, b);
                    const float ra = a - __uint_as_float(ph << 16), rb = b - __uint_as_float(ph & 0xffff0000u);
                    const uint32_t pm = cvt_pk_bf16(ra, rb);
                    const float ta = ra - __uint_as_float(pm << 16), tb = rb - __uint_as_float(pm & 0xffff0000u);
                    pw[0][q >> 1] = ph;
                    pw[1][q >> 1] = pm;
                    pw[2][q >> 1] = cvt_pk_bf16(ta, tb);
                }
                // rows kr .. kr + 3 of column c: 8 B inside 16-B unit kr >> 3 (swizzled), offset 8 ((kr >> 2) & 1)
                const int off = c * 64 + 16 * ((kr >> 3) ^ ((c >> 1) & 3)) + 8 * ((kr >> 2) & 1);
#pragma unroll
                for (int x = 0; x < 3; ++x)
                    *reinterpret_cast<uint2*>(img + x * G::IMG + off) = make_uint2(pw[x][0], pw[x][1]);
            }
        }
    };
    const uint32_t lo = (uint32_t)(r * 64 + 16 * (h ^ ((r >> 1) & 3)));
    auto frag = [&](const char* img, int piece, int t) {
        return *reinterpret_cast<const bf16x8s*>(img + piece * G::IMG + t * 1024 + lo);
    };
    int buf = 0;
    // loader group of this wave (NLG > 1): it stages steps lg, lg + NLG, ... and loads NLG ahead
    const int lg = NLG == 1 ? 0 : __builtin_amdgcn_readfirstlane(tid / GSZ);
    if (NLG == 1) {
        if (beg < end) load(beg);
    } else if (lg < NLG && beg + 32 * lg < end) {
        load(beg + 32 * lg);
    }
    int sm = 0;  // step index mod NLG
    for (int64_t r0 = beg; r0 < end; r0 += 32) {
        char* img = smem_raw + buf * G::STEP;
        if (G::NBUF == 1) __syncthreads();  // single buffer: the previous step's reads are done
        if (NLG == 1) {
            stage(img);
            __syncthreads();
            if (r0 + 32 < end) load(r0 + 32);
        } else {
            static_assert(NLG == 1 || G::NBUF == 2, "loader groups need two buffers");
            if (sm == lg) {
                stage(img);
                if (r0 + 32 * NLG < end) load(r0 + 32 * NLG);
            }
            sm = sm + 1 == NLG ? 0 : sm + 1;
            __syncthreads();
        }
        bf16x8s fa[TG][3];
#pragma unroll
        for (int i = 0; i < TG; ++i)
#pragma unroll
            for (int x = 0; x < 3; ++x) fa[i][x] = frag(img, x, GA * TG + i);
#pragma unroll
        for (int j = 0; j < TG; ++j) {
            const bf16x8s hb_ = frag(img, 0, GB * TG + j), mb = frag(img, 1, GB * TG + j), tb = frag(img, 2, GB * TG + j);
#pragma unroll
            for (int i = 0; i < TG; ++i) {
                f32x4 c = acc[i][j];
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][2], hb_, c, 0, 0, 0);  // smallest terms first
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][0], tb, c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][1], mb, c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][1], hb_, c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][0], mb, c, 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][0], hb_, c, 0, 0, 0);
            }
        }
        buf = G::NBUF - 1 - buf;
    }
#pragma unroll
    for (int i = 0; i < TG; ++i)
#pragma unroll
        for (int j = 0; j < TG; ++j) {
            const int ta = GA * TG + i, tb = GB * TG + j;
            if (ta > tb) continue;  // (diagonal group pairs) the mirror of an upper pair
            const int a = ta >> 1, b = tb >> 1;
            const int blk = a * G::NB - a * (a - 1) / 2 + (b - a);
            double* dst = slabs + ((int64_t)chunk * G::NBLK + blk) * 1024;
            const bool mirror = (a == b) && (ta != tb);
#pragma unroll
            for (int e = 0; e < 4; ++e) {  // bf16 MFMA D: col = lane & 15, row = 4 h + e
                const int li = 16 * (ta & 1) + 4 * h + e, lj = 16 * (tb & 1) + r;
                dst[li * 32 + lj] = (double)acc[i][j][e];
                if (mirror) dst[lj * 32 + li] = (double)acc[i][j][e];
            }
        }
}

// LP = 512, round 4: the same arithmetic (six bf16 products per tile pair, fp32 chunk accumulators,
// the same slabs) with each of a chunk's workgroups staging ONLY the column groups its group pairs
// read.  gram_split_kernel<512> staged all 512 columns (96 KB per 32-row step) in each of four
// workgroups: single-buffered, the VALU split work (430 instructions per wave per step) run 4x over
// between barriers, 168 VGPRs with spills at 9 waves -- rocprofv3: MFMA busy 23 %, waves parked
// 61 %, LDS 11 % busy.  Here the 36 group pairs of the 8 column groups (64 columns each) are dealt
// to five 8-wave workgroup types, each reading at most 6 groups:
//   0: groups {0,1,2,3}, pairs (0,0) (0,1) (0,2) (1,1) (1,2) (2,2) (0,3) (1,3)
//   1: groups {4,5,6,7}, the same pairs shifted by 4
//   2: {0,1} x {4,5,6,7}    3: {2,3} x {4,5,6,7}    4: (2,3) (3,3) (6,7) (7,7)
// so a step is at most 6 groups (72 KB): two buffers fit the LDS and the next step's split is
// staged while this step's MFMAs run (one barrier per step), at 2 waves per SIMD (256 VGPRs).
struct GramSplit4 {
    static constexpr int LP = 512, TG = 4, NB = 16, NBLK = NB * (NB + 1) / 2;
    static constexpr int TYPES = 5, WAVES = 12, THREADS = 64 * WAVES;  // 8 MFMA waves + 4 staging waves
    static constexpr int CWAVES = 8, SWAVES = WAVES - CWAVES;
    static constexpr int MAXG = 6;                 // staged groups (64 columns) per workgroup, at most
    static constexpr int IMG = MAXG * 64 * 64;     // bytes of one piece image (6 x 64 columns x 32 rows bf16)
    static constexpr int STEP = 3 * IMG;           // one 32-row step, three pieces (72 KB)
    static constexpr int LDS = 2 * STEP;           // double-buffered: 144 KB
    static constexpr int LPT = (MAXG * 64 * 4 + 64 * SWAVES - 1) / (64 * SWAVES);  // 8-row units per staging thread
};

// global group of local staged group lg, for workgroup type ty
__device__ __forceinline__ int gs4_group(int ty, int lg) {
    switch (ty) {
        case 0: return lg;
        case 1: return 4 + lg;
        case 2: return lg < 2 ? lg : 2 + lg;
        case 3: return 2 + lg;
        default: return lg < 2 ? 2 + lg : 4 + lg;
    }
}

__global__ __launch_bounds__(GramSplit4::THREADS) void gram_split4_kernel(const float* __restrict__ P, int64_t rows,
                                                                         int64_t rpc, int nchunk,
                                                                         double* __restrict__ slabs) {
    typedef GramSplit4 G;
    constexpr int TG = G::TG, LPT = G::LPT;
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    const int tid = threadIdx.x, lane = tid & 63, r = lane & 15, h = lane >> 4;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    // a chunk's five workgroups are 8 apart in dispatch order: one XCD (its L2 serves the repeats)
    const int v = blockIdx.x >> 3;
    const int ty = v % G::TYPES;
    const int chunk = ((v / G::TYPES) << 3) | (blockIdx.x & 7);
    if (chunk >= nchunk) return;
    const int64_t beg = (int64_t)chunk * rpc;
    const int64_t end = (beg + rpc < rows) ? beg + rpc : rows;
    const int ngl = (ty == 2 || ty == 3) ? 6 : 4;  // staged groups
    const int NU = ngl * 64 * 4;                  // units of a step
    // this wave's group pair: local (LA <= LB) and global (GA <= GB)
    int LA, LB;
    bool active = true;
    if (ty < 2) {
        LA = (0x10211000 >> (4 * w)) & 15;  // w = 0..7: 0 0 0 1 1 2 0 1
        LB = (0x33221210 >> (4 * w)) & 15;  //          0 1 2 1 2 2 3 3
    } else if (ty < 4) {
        LA = w >> 2;
        LB = 2 + (w & 3);
    } else {
        LA = w & 3;
        LB = (w & 2) ? 3 : 1;
        active = w < 4;
    }
    const bool stager = w >= G::CWAVES;
    if (stager) active = false;
    const int sid = tid - 64 * G::CWAVES;  // staging thread index (stagers only)
    const int GA = gs4_group(ty, LA), GB = gs4_group(ty, LB);
    f32x4 acc[TG][TG];
#pragma unroll
    for (int i = 0; i < TG; ++i)
#pragma unroll
        for (int j = 0; j < TG; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    if (stager) {  // the staging waves: their own loop, the same barriers as the MFMA waves'
        // unit u = sid + 256 t (u < NU): row octet u / ncol (8 rows) of local column u % ncol.  A wave's
        // lanes take 64 consecutive columns (256-B row segments per load), each lane splits its 8 rows into
        // the three pieces with no component selects, and writes one 16-B octet per piece.  LDS image as
        // gram_split_kernel's: column c's 32 rows as four 16-B octets, octet o at o ^ ((c >> 1) & 3) -- 8
        // consecutive columns of a ds_write_b128 lane group hit 8 distinct slots, the fragment reads'
        // 16-lane groups 16.  Offsets are fixed for the launch: computed once.
        const int ncol = ngl * 64;
        int64_t goff[LPT];
        int loff[LPT];
#pragma unroll
        for (int t = 0; t < LPT; ++t) {
            const int u = sid + 64 * G::SWAVES * t;
            const int oc = u / ncol, lc = u - oc * ncol;
            goff[t] = (int64_t)(8 * oc) * G::LP + ((gs4_group(ty, lc >> 6) << 6) | (lc & 63));
            loff[t] = u < NU ? lc * 64 + 16 * (oc ^ ((lc >> 1) & 3)) : -1;
        }
        // two steps of loads in flight (a step's stage is ~1 us of work, an HBM round trip under this
        // load longer): register sets A and B alternate, loads issued two steps ahead of their stage
        typedef float Regs[LPT][8];
        Regs ra, rb;
        // (every guard is wave-uniform: no per-load exec branches -- they were 10 instructions per load;
        // the rows of a chunk's partial last step are clamped and zeroed)
        const int tmax = ngl == 6 ? LPT : 4;  // units t >= tmax do not exist for the 4-group types
        auto load = [&](Regs& reg, int64_t r0) {
            const bool full = r0 + 32 <= end;
#pragma unroll
            for (int t = 0; t < LPT; ++t) {
                if (t >= tmax) break;
                if (full) {
                    const float* src = P + r0 * G::LP + goff[t];
#pragma unroll
                    for (int q = 0; q < 8; ++q) reg[t][q] = src[q * G::LP];
                } else {
                    const int64_t row = r0 + (goff[t] >> 9);  // + 8 oc (G::LP = 512)
                    const int gc = (int)(goff[t] & (G::LP - 1));
#pragma unroll
                    for (int q = 0; q < 8; ++q) {
                        const int64_t rr = row + q < end ? row + q : end - 1;
                        const float x = P[rr * G::LP + gc];
                        reg[t][q] = row + q < end ? x : 0.f;
                    }
                }
            }
        };
        auto stage = [&](const Regs& reg, char* img) {
#pragma unroll
            for (int t = 0; t < LPT; ++t) {
                if (t >= tmax) break;
                uint32_t pw[3][4];
#pragma unroll
                for (int q = 0; q < 8; q += 2) {
                    // exact three-piece split, two rows at a time: h = bf16(v), m = bf16(v - h), t = v - h - m
                    const float a = reg[t][q], b = reg[t][q + 1];
                    const uint32_t ph = cvt_pk_bf16(a, b);
                    const float ra_ = a - __uint_as_float(ph << 16), rb_ = b - __uint_as_float(ph & 0xffff0000u);
                    const uint32_t pm = cvt_pk_bf16(ra_, rb_);
                    const float ta = ra_ - __uint_as_float(pm << 16), tb = rb_ - __uint_as_float(pm & 0xffff0000u);
                    pw[0][q >> 1] = ph;
                    pw[1][q >> 1] = pm;
                    pw[2][q >> 1] = cvt_pk_bf16(ta, tb);
                }
#pragma unroll
                for (int x = 0; x < 3; ++x)
                    *reinterpret_cast<uint4*>(img + x * G::IMG + loff[t]) = make_uint4(pw[x][0], pw[x][1], pw[x][2], pw[x][3]);
            }
        };
        if (beg < end) {
            load(ra, beg);
            stage(ra, smem_raw);
            if (beg + 32 < end) load(rb, beg + 32);
            if (beg + 64 < end) load(ra, beg + 64);
        }
        __syncthreads();
        // iteration of step r0: stage step r0 + 32 into the other buffer (its last readers passed the
        // previous barrier) from the set loaded two iterations ago, then reload that set with r0 + 96
        auto iter = [&](Regs& reg, int64_t r0, int b) {
            if (r0 + 32 < end) {
                stage(reg, smem_raw + (b ^ 1) * G::STEP);
                if (r0 + 96 < end) load(reg, r0 + 96);
            }
            __syncthreads();
        };
        for (int64_t r0 = beg; r0 < end; r0 += 64) {
            iter(rb, r0, 0);
            if (r0 + 32 < end) iter(ra, r0 + 32, 1);
        }
        return;
    }
    const uint32_t lo = (uint32_t)(r * 64 + 16 * (h ^ ((r >> 1) & 3)));
    auto frag = [&](const char* img, int piece, int t) {  // t: local tile (16 columns)
        return *reinterpret_cast<const bf16x8s*>(img + piece * G::IMG + t * 1024 + lo);
    };
    __syncthreads();  // step 0 staged
    int buf = 0;
    for (int64_t r0 = beg; r0 < end; r0 += 32) {
        const char* img = smem_raw + buf * G::STEP;
        if (active) {
            bf16x8s fa[TG][3];
#pragma unroll
            for (int i = 0; i < TG; ++i)
#pragma unroll
                for (int x = 0; x < 3; ++x) fa[i][x] = frag(img, x, LA * TG + i);
#pragma unroll
            for (int j = 0; j < TG; ++j) {
                const bf16x8s hb_ = frag(img, 0, LB * TG + j), mb = frag(img, 1, LB * TG + j),
                              tb = frag(img, 2, LB * TG + j);
#pragma unroll
                for (int i = 0; i < TG; ++i) {
                    f32x4 c = acc[i][j];
                    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][2], hb_, c, 0, 0, 0);  // smallest terms first
                    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][0], tb, c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][1], mb, c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][1], hb_, c, 0, 0, 0);
                    c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][0], mb, c, 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][0], hb_, c, 0, 0, 0);
                }
            }
        }
        __syncthreads();
        buf ^= 1;
    }
    if (!active) return;
#pragma unroll
    for (int i = 0; i < TG; ++i)
#pragma unroll
        for (int j = 0; j < TG; ++j) {
            const int ta = GA * TG + i, tb = GB * TG + j;
            if (ta > tb) continue;  // (diagonal group pairs) the mirror of an upper pair
            const int a = ta >> 1, b = tb >> 1;
            const int blk = a * G::NB - a * (a - 1) / 2 + (b - a);
            double* dst = slabs + ((int64_t)chunk * G::NBLK + blk) * 1024;
            const bool mirror = (a == b) && (ta != tb);
#pragma unroll
            for (int e = 0; e < 4; ++e) {  // bf16 MFMA D: col = lane & 15, row = 4 h + e
                const int li = 16 * (ta & 1) + 4 * h + e, lj = 16 * (tb & 1) + r;
                dst[li * 32 + lj] = (double)acc[i][j][e];
                if (mirror) dst[lj * 32 + li] = (double)acc[i][j][e];
            }
        }
}

// Cross Gram R = X^T Y of two fp32 panels at LP = 256 / 512 by the same three-piece bf16 split (round
// 4: R = Q_B^T B^T, the fp64-MFMA gram_wide_kernel<float, true> took 237 us at C4 for 8.6 GFLOP).
// Workgroup types per row chunk: the 64 columns of X's group gx against 256 columns (half gy) of Y
// -- 4 types at LP = 256, 16 at LP = 512.  A step stages 64 + 256 columns (octet units as
// gram_split4_kernel, 60 KB, double-buffered); wave w takes X tiles 2 (w & 1) .. + 1 of the group and
// Y tiles 4 (w >> 1) .. + 3 of the half -- 8 tile pairs, six MFMAs each.  Partial 32 x 32 blocks go
// to the cross slab layout gram_reduce4_kernel sums (blk = a nb + b).
template <int LP_> struct GramSplitX {
    static constexpr int LP = LP_, NB = LP / 32, NBLK = NB * NB, WAVES = 8, THREADS = 64 * WAVES;
    static constexpr int GXN = LP / 64, GYN = LP / 256, TYPES = GXN * GYN;
    static constexpr int XC = 64, YC = 256;               // staged columns of X (one group) and Y (one half)
    static constexpr int XIMG = XC * 64, YIMG = YC * 64;  // bytes per piece image (32 rows bf16 per column)
    static constexpr int STEP = 3 * (XIMG + YIMG);        // 60 KB
    static constexpr int NU = 4 * (XC + YC);              // 8-row x 1-column units per step
    static constexpr int LPT = (NU + THREADS - 1) / THREADS;
};

template <int LP_>
__global__ __launch_bounds__(GramSplitX<LP_>::THREADS) void gram_split_cross_kernel(const float* __restrict__ X,
                                                                                   const float* __restrict__ Y,
                                                                                   int64_t rows, int64_t rpc,
                                                                                   int nchunk,
                                                                                   double* __restrict__ slabs) {
    typedef GramSplitX<LP_> G;
    constexpr int LPT = G::LPT;
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    const int tid = threadIdx.x, lane = tid & 63, r = lane & 15, h = lane >> 4;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int v = blockIdx.x >> 3;  // a chunk's types are 8 apart in dispatch order: one XCD
    const int ty = v % G::TYPES;
    const int gx = ty % G::GXN, gy = ty / G::GXN;
    const int chunk = ((v / G::TYPES) << 3) | (blockIdx.x & 7);
    if (chunk >= nchunk) return;
    const int64_t beg = (int64_t)chunk * rpc;
    const int64_t end = (beg + rpc < rows) ? beg + rpc : rows;
    const int xt0 = 2 * (w & 1), yt0 = 4 * (w >> 1);  // local X tiles (of the group), Y tiles
    f32x4 acc[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // unit u: units [0, 4 XC) are X's (octet u / XC of local column u % XC), the rest Y's
    int oct[LPT], coff[LPT], loff[LPT];
    bool isx[LPT];
#pragma unroll
    for (int t = 0; t < LPT; ++t) {
        const int u = tid + G::THREADS * t;
        const bool xu = u < 4 * G::XC;
        const int uu = xu ? u : u - 4 * G::XC;
        const int nc = xu ? G::XC : G::YC;
        const int oc = uu / nc, c = uu - oc * nc;
        isx[t] = xu;
        oct[t] = 8 * oc;
        coff[t] = xu ? 64 * gx + c : 256 * gy + c;
        loff[t] = (u < G::NU) ? (xu ? 0 : 3 * G::XIMG) + c * 64 + 16 * (oc ^ ((c >> 1) & 3)) : -1;
    }
    float reg[LPT][8];
    auto load = [&](int64_t r0) {
        const bool full = r0 + 32 <= end;
#pragma unroll
        for (int t = 0; t < LPT; ++t) {
            if (tid + G::THREADS * t - lane >= G::NU) break;  // wave-uniform (NU, THREADS multiples of 64)
            const float* base = isx[t] ? X : Y;
            const int64_t row = r0 + oct[t];
            if (full) {
                const float* src = base + row * G::LP + coff[t];
#pragma unroll
                for (int q = 0; q < 8; ++q) reg[t][q] = src[q * G::LP];
            } else {  // the chunk's partial last step: rows clamped and zeroed
#pragma unroll
                for (int q = 0; q < 8; ++q) {
                    const int64_t rr = row + q < end ? row + q : end - 1;
                    const float x = base[rr * G::LP + coff[t]];
                    reg[t][q] = row + q < end ? x : 0.f;
                }
            }
        }
    };
    auto stage = [&](char* img) {
#pragma unroll
        for (int t = 0; t < LPT; ++t) {
            if (loff[t] < 0) break;
            uint32_t pw[3][4];
#pragma unroll
            for (int q = 0; q < 8; q += 2) {
                const float a = reg[t][q], b = reg[t][q + 1];
                const uint32_t ph = cvt_pk_bf16(a, b);
                const float ra = a - __uint_as_float(ph << 16), rb = b - __uint_as_float(ph & 0xffff0000u);
                const uint32_t pm = cvt_pk_bf16(ra, rb);
                const float ta = ra - __uint_as_float(pm << 16), tb = rb - __uint_as_float(pm & 0xffff0000u);
                pw[0][q >> 1] = ph;
                pw[1][q >> 1] = pm;
                pw[2][q >> 1] = cvt_pk_bf16(ta, tb);
            }
            const int pstride = isx[t] ? G::XIMG : G::YIMG;
#pragma unroll
            for (int x = 0; x < 3; ++x)
                *reinterpret_cast<uint4*>(img + loff[t] + x * pstride) = make_uint4(pw[x][0], pw[x][1], pw[x][2], pw[x][3]);
        }
    };
    const uint32_t lo = (uint32_t)(r * 64 + 16 * (h ^ ((r >> 1) & 3)));
    if (beg < end) {
        load(beg);
        stage(smem_raw);
        if (beg + 32 < end) load(beg + 32);
    }
    __syncthreads();
    int buf = 0;
    for (int64_t r0 = beg; r0 < end; r0 += 32) {
        const char* img = smem_raw + buf * G::STEP;
        bf16x8s fa[2][3];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int x = 0; x < 3; ++x)
                fa[i][x] = *reinterpret_cast<const bf16x8s*>(img + x * G::XIMG + (xt0 + i) * 1024 + lo);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const char* yb = img + 3 * G::XIMG + (yt0 + j) * 1024 + lo;
            const bf16x8s yh = *reinterpret_cast<const bf16x8s*>(yb), ym = *reinterpret_cast<const bf16x8s*>(yb + G::YIMG),
                          yt = *reinterpret_cast<const bf16x8s*>(yb + 2 * G::YIMG);
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                f32x4 c = acc[i][j];
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][2], yh, c, 0, 0, 0);  // smallest terms first
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][0], yt, c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][1], ym, c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][1], yh, c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][0], ym, c, 0, 0, 0);
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i][0], yh, c, 0, 0, 0);
            }
        }
        if (r0 + 32 < end) {
            stage(smem_raw + (buf ^ 1) * G::STEP);
            if (r0 + 64 < end) load(r0 + 64);
        }
        __syncthreads();
        buf ^= 1;
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int ta = 4 * gx + xt0 + i, tb = 16 * gy + yt0 + j;  // global 16-column tiles of X, Y
            const int blk = (ta >> 1) * G::NB + (tb >> 1);
            double* dst = slabs + ((int64_t)chunk * G::NBLK + blk) * 1024;
#pragma unroll
            for (int e = 0; e < 4; ++e)  // bf16 MFMA D: col = lane & 15, row = 4 h + e
                dst[(16 * (ta & 1) + 4 * h + e) * 32 + 16 * (tb & 1) + r] = (double)acc[i][j][e];
        }
}

// The chunk partials summed in a fixed order (deterministic): one workgroup = 64 Gram entries x 4
// chunk ranges (wave k sums chunks [k n / 4, (k + 1) n / 4) with four interleaved partials, a wave's
// 64 entries one 512-B load per chunk), the ranges combined in wave order.  (Round 4 replaced a
// one-thread-per-entry sum: C3's LP = 128 Gram -- 10 blocks, 256 chunks -- ran that on 40 workgroups;
// this gives it 160: C4 23.81 -> 23.68 ms, C5 19.15 -> 19.13, C3 5.65 -> 5.62 on one box.)
__global__ __launch_bounds__(256) void gram_reduce4_kernel(const double* __restrict__ slabs, int nblk, int nchunk,
                                                           int LP, int cross, double* __restrict__ G,
                                                           const int* __restrict__ pred) {
    if (pred && *pred == 0) return;
    __shared__ double part[4][64];
    const int lane = threadIdx.x & 63, k = threadIdx.x >> 6;
    const int64_t e = blockIdx.x * (int64_t)64 + lane;
    bool ok = e < (int64_t)nblk * 1024;
    const int blk = ok ? (int)(e / 1024) : 0, loc = (int)(e % 1024);
    const int nb = (LP + 31) / 32;
    int a, b;
    if (cross) {
        a = blk / nb;
        b = blk % nb;
    } else {
        int rem = blk;
        a = 0;
        while (rem >= nb - a) {
            rem -= nb - a;
            ++a;
        }
        b = a + rem;
    }
    const int ra = 32 * a + loc / 32, cb = 32 * b + loc % 32;
    ok = ok && ra < LP && cb < LP;
    double sum = 0.0;
    if (ok) {
        const int64_t cs = (int64_t)nblk * 1024;
        const double* src = slabs + (int64_t)blk * 1024 + loc;
        const int c0 = (int)((int64_t)nchunk * k / 4), c1 = (int)((int64_t)nchunk * (k + 1) / 4);
        double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
        int c = c0;
        for (; c + 4 <= c1; c += 4) {
            s0 += src[(c + 0) * cs];
            s1 += src[(c + 1) * cs];
            s2 += src[(c + 2) * cs];
            s3 += src[(c + 3) * cs];
        }
        for (; c < c1; ++c) s0 += src[c * cs];
        sum = (s0 + s1) + (s2 + s3);
    }
    part[k][lane] = sum;
    __syncthreads();
    if (k == 0 && ok) {
        const double t = (part[0][lane] + part[1][lane]) + (part[2][lane] + part[3][lane]);
        G[(int64_t)ra * LP + cb] = t;
        if (!cross && a != b) G[(int64_t)cb * LP + ra] = t;
    }
}

hipError_t launch_gram_reduce(const double* slabs, int nblk, int nchunk, int LP, int cross, double* G, const int* pred,
                              hipStream_t s) {
    const int64_t tot = (int64_t)nblk * 1024;
    hipLaunchKernelGGL(gram_reduce4_kernel, dim3((int)((tot + 63) / 64)), dim3(256), 0, s, slabs, nblk, nchunk, LP,
                       cross, G, pred);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------------
// Cholesky, one workgroup of kCholThreads threads.  W (work) holds the Gram being reduced (upper
// block triangle only); R gets the factor's upper block triangle, Rinv the inverse diagonal blocks
// (rinv_wide_kernel fills the rest).  Per 16-column block p: the strip R[p][p+1..] = D_p^-T W[p][p+1..]
// (to global R and an LDS copy), then the trailing update W -= R[p]^T R[p] on the fp64 MFMA with both
// operands from the LDS strip, each wave keeping kCholBatch W tiles' read-modify-write in flight (one
// CU's update is latency-bound otherwise).  Look-ahead: wave 0 updates tile (p+1, p+1) first and
// factors it -- 16x16 upper Cholesky and inverse in registers, lane j owning column j, pivots and rows
// broadcast with v_readlane, rsqrt + Newton pivots -- while the other waves finish the update.  Two
// workgroup barriers per block.
constexpr int kCholThreads = 512;
constexpr int kCholBatch = 6;
constexpr int kCholPad = 16;  // LDS strip pitch LP + 16 doubles: the 4 k-rows of a tile read hit different banks

__device__ __forceinline__ double readlane_d(double v, int lane) {
    const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
    const unsigned lo = __builtin_amdgcn_readlane((unsigned)u, lane);
    const unsigned hi = __builtin_amdgcn_readlane((unsigned)(u >> 32), lane);
    return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}

__device__ __forceinline__ void tri_decode(int t, int nt2, int& ib, int& jb) {  // t -> (ib <= jb) in [0, nt2)
    int rem = t, i = 0;
    while (rem >= nt2 - i) {
        rem -= nt2 - i;
        ++i;
    }
    ib = i;
    jb = i + rem;
}

// 1/sqrt(d) to fp64 accuracy: hardware estimate + two Newton steps
__device__ __forceinline__ double rsqrt_nr(double d) {
    double y = __builtin_amdgcn_rsq(d);
    y = y * fma(-0.5 * d * y, y, 1.5);
    y = y * fma(-0.5 * d * y, y, 1.5);
    return y;
}

// Wave-level factor of a 16x16 diagonal block for the single-wave critical path of the block
// Cholesky (lane j: col[i] = T[i][j]; the upper part is valid).  Measured: the predicated form
// (`if (j >= i) col[i] -= ...`) followed by a separate back substitution ran 6 us per block, a
// dependent chain of ~2000 VALU/readlane instructions on one wave.  Here every update is
// unconditional (lanes j < i only carry lower-triangle values no later step reads), and D^-1 is
// formed in the same pivot loop: row k of Y = D^-T (lane j: Y[k][j] = D^-1[j][k]) is
// (e_j[k] - acc[k]) / D[k][k], and each broadcast D[k][i] feeds both the factor update and
// acc[i] += D[k][i] Y[k][j] -- one readlane per element for both.  Writes the R and R^-1 diagonal
// blocks (global), D^-1 (Di, LDS, row-major), the breakdown rows (bad) and flags.
__device__ __forceinline__ __attribute__((unused)) void chol_diag16_fast(double (&col)[16], int p16, int l, int LP, double tol,
                                                 const double* d0, double* Di, int* bad, double* R, double* Rinv,
                                                 int* colflag, int* flag, int lane) {
    const int j = lane & 15;
    int badmask = 0;
    double acc[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 0.0;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const int gk = p16 + k;
        const double dkk = readlane_d(col[k], k);
        const bool pad = gk >= l;
        const bool isbad = !pad && (!(dkk > tol * d0[gk]) || !(d0[gk] > 0.0) || !isfinite(dkk));
        if (isbad) badmask |= 1 << k;
        const bool unit = pad || isbad;
        const double y = unit ? 1.0 : rsqrt_nr(dkk);
        const double rk = unit ? 1.0 : dkk * y;
        const double v = unit ? 0.0 : col[k] * y;
        col[k] = (j == k) ? rk : v;
        const double yk = ((j == k ? 1.0 : 0.0) - acc[k]) * y;  // Y[k][j] = D^-1[j][k]
        if (lane < 16) Di[j * 16 + k] = yk;
#pragma unroll
        for (int i = k + 1; i < 16; ++i) {
            const double dki = readlane_d(col[k], i);  // D[k][i]
            col[i] = fma(-dki, col[k], col[i]);
            acc[i] = fma(dki, yk, acc[i]);
        }
    }
#pragma unroll
    for (int i = 0; i < 16; ++i)
        if (i > j) col[i] = 0.0;
    if (lane < 16) {
#pragma unroll
        for (int i = 0; i < 16; ++i) R[(int64_t)(p16 + i) * LP + p16 + j] = col[i];
        bad[lane] = (badmask >> lane) & 1;
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's D^-1 rows landed
    __builtin_amdgcn_wave_barrier();
    if (lane < 16) {
#pragma unroll
        for (int i = 0; i < 16; i += 2)
            *reinterpret_cast<double2*>(Rinv + (int64_t)(p16 + j) * LP + p16 + i) =
                *reinterpret_cast<const double2*>(Di + j * 16 + i);
    }
    if (lane == 0 && badmask) {
        atomicAdd(flag, __popc(badmask));
        for (int k = 0; k < 16; ++k)
            if (badmask & (1 << k)) colflag[p16 + k] = 1;
    }
}

// The same factor with the row broadcasts on the 64-bit DPP of gfx90a+ (row_newbcast:i -- lane i of
// every 16-lane row to the whole row): the tile is replicated in the wave's four rows (lane j of each
// row owns column j), so D[k][i] = lane i's col[k] reaches every lane of the row inside the FMA that
// uses it -- v_fmac_f64_dpp, ONE instruction per update instead of two v_readlane (SGPRs, which the
// compiler hoisted and spilled) and an FMA.  Same operations in the same order (fma(d, -c, x) rounds as
// fma(-d, c, x)): bit-identical to chol_diag16_fast.  The d0 diagonal of the block is read before the
// pivot chain (lane j: d0[p16 + j], broadcast per pivot).  The asm carries `s_nop 1` for the
// VALU-write -> DPP-read hazard (the compiler's hazard recognizer does not look into inline asm).
template <int I>
__device__ __forceinline__ double nbcast_f64(double v) {
    double r;
    asm("s_nop 1\n\tv_mov_b64_dpp %0, %1 row_newbcast:%2 row_mask:0xf bank_mask:0xf" : "=v"(r) : "v"(v), "i"(I));
    return r;
}
template <int I>
__device__ __forceinline__ void fmac_nbcast_f64(double& acc, double x, double y) {  // acc += x[lane I of the row] * y
    asm("s_nop 1\n\tv_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
        : "+v"(acc)
        : "v"(x), "v"(y), "i"(I));
}
template <int K, int I>
__device__ __forceinline__ void diag16_updates(double (&col)[16], double (&acc)[16], double ck, double nck, double yk) {
    if constexpr (I < 16) {
        fmac_nbcast_f64<I>(col[I], ck, nck);  // col[i] -= D[k][i] col[k]
        fmac_nbcast_f64<I>(acc[I], ck, yk);   // acc[i] += D[k][i] Y[k][j]
        diag16_updates<K, I + 1>(col, acc, ck, nck, yk);
    }
}
template <int K>
__device__ __forceinline__ void diag16_pivots(double (&col)[16], double (&acc)[16], int j, int p16, int l, double tol,
                                              double d0j, double* Di, int lane, int& badmask) {
    if constexpr (K < 16) {
        const int gk = p16 + K;
        const double dkk = nbcast_f64<K>(col[K]);
        const double d0k = nbcast_f64<K>(d0j);
        const bool pad = gk >= l;
        const bool isbad = !pad && (!(dkk > tol * d0k) || !(d0k > 0.0) || !isfinite(dkk));
        if (isbad) badmask |= 1 << K;
        const bool unit = pad || isbad;
        const double y = unit ? 1.0 : rsqrt_nr(dkk);
        const double rk = unit ? 1.0 : dkk * y;
        const double v = unit ? 0.0 : col[K] * y;
        col[K] = (j == K) ? rk : v;
        const double yk = ((j == K ? 1.0 : 0.0) - acc[K]) * y;  // Y[k][j] = D^-1[j][k]
        if (lane < 16) Di[j * 16 + K] = yk;
        diag16_updates<K, K + 1>(col, acc, col[K], -col[K], yk);
        diag16_pivots<K + 1>(col, acc, j, p16, l, tol, d0j, Di, lane, badmask);
    }
}
__device__ __forceinline__ void chol_diag16_dpp(double (&col)[16], int p16, int l, int LP, double tol, const double* d0,
                                                double* Di, int* bad, double* R, double* Rinv, int* colflag, int* flag,
                                                int lane) {
    const int j = lane & 15;
    const double d0j = d0[p16 + j];
    int badmask = 0;  // the same in every lane (uniform tests)
    double acc[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 0.0;
    diag16_pivots<0>(col, acc, j, p16, l, tol, d0j, Di, lane, badmask);
#pragma unroll
    for (int i = 0; i < 16; ++i)
        if (i > j) col[i] = 0.0;
    if (lane < 16) {
#pragma unroll
        for (int i = 0; i < 16; ++i) R[(int64_t)(p16 + i) * LP + p16 + j] = col[i];
        bad[lane] = (badmask >> lane) & 1;
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's D^-1 rows landed
    __builtin_amdgcn_wave_barrier();
    if (lane < 16) {
#pragma unroll
        for (int i = 0; i < 16; i += 2)
            *reinterpret_cast<double2*>(Rinv + (int64_t)(p16 + j) * LP + p16 + i) =
                *reinterpret_cast<const double2*>(Di + j * 16 + i);
    }
    if (lane == 0 && badmask) {
        atomicAdd(flag, __popc(badmask));
        for (int k = 0; k < 16; ++k)
            if (badmask & (1 << k)) colflag[p16 + k] = 1;
    }
}
// Round 5: the same factor with fewer instructions on the pivot loop.  One wave issues at most one
// instruction per four cycles, and the DPP form above spent 1686 instructions per factor (974 VALU,
// 712 SALU: s_nop hazards, exec-mask branches around the rsqrt and the D^-1 stores, per-pivot
// breakdown tests) -- 7844 cycles.  Here:
//  * the breakdown / finiteness tests leave the pivot loop: lane k keeps its pivot d_kk, and after
//    the loop one vector test (lane j judges pivot j) and a ballot decide; a bad or padding pivot
//    (rare: rank deficiency, l % 16) re-runs chol_diag16_dpp from the staged tile -- the only path
//    that needs the unit-pivot substitutions;
//  * rsqrt unconditional (no branch), the D^-1 rows stay in registers (lane j: row j of D^-1) and
//    are stored once after the loop (LDS Di and the global R^-1 block), no per-pivot exec masks;
//  * -col[K] is the DPP FMA's src1 negation modifier, and only the first DPP use of each pivot
//    row carries the `s_nop 1` (its source was just written); the later ones read it again.
// Same operations in the same order as chol_diag16_dpp on a pivot chain without breakdowns:
// bit-identical R and R^-1 (tools/wide_lab chol checks it).
template <int I>
__device__ __forceinline__ void fmsub_nbcast_nop(double& acc, double x, double y) {  // acc -= x[lane I] * y, hazard-safe
    asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, %1, -%2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
                 : "+v"(acc)
                 : "v"(x), "v"(y), "i"(I));
}
// (volatile: kept in program order, so every hazard-free use follows the s_nop'ed first use)
template <int I>
__device__ __forceinline__ void fmsub_nbcast(double& acc, double x, double y) {  // x written >= 2 instrs earlier
    asm volatile("v_fmac_f64_dpp %0, %1, -%2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
                 : "+v"(acc)
                 : "v"(x), "v"(y), "i"(I));
}
template <int I>
__device__ __forceinline__ void fmadd_nbcast(double& acc, double x, double y) {
    asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
                 : "+v"(acc)
                 : "v"(x), "v"(y), "i"(I));
}
template <int K, int I>
__device__ __forceinline__ void diag16v2_updates(double (&col)[16], double (&acc)[16], double ck, double yk) {
    if constexpr (I < 16) {
        if constexpr (I == K + 1) fmsub_nbcast_nop<I>(col[I], ck, ck);  // col[i] -= D[k][i] col[k]
        else fmsub_nbcast<I>(col[I], ck, ck);
        fmadd_nbcast<I>(acc[I], ck, yk);  // acc[i] += D[k][i] Y[k][j]
        diag16v2_updates<K, I + 1>(col, acc, ck, yk);
    }
}
// `careful` (uniform): the breakdown / padding tests of chol_diag16_dpp on every pivot; a unit pivot
// (padding row or breakdown) is the same arithmetic on the substituted row e_k with d_kk = 1 (then
// y = rk = 1, v = 0, exactly the unit-pivot values of the DPP form).
template <int K>
__device__ __forceinline__ void diag16v2_pivots(double (&col)[16], double (&acc)[16], double (&yrow)[16], int j,
                                                double& dsave, bool careful, int p16, int l, double tol, double d0j,
                                                int& badmask) {
    if constexpr (K < 16) {
        double dkk = nbcast_f64<K>(col[K]);
        if (careful) {
            const double d0k = nbcast_f64<K>(d0j);
            const bool pad = p16 + K >= l;
            const bool isbad = !pad && (!(dkk > tol * d0k) || !(d0k > 0.0) || !isfinite(dkk));
            if (isbad) badmask |= 1 << K;
            if (pad || isbad) {
                dkk = 1.0;
                col[K] = (j == K) ? 1.0 : 0.0;
            }
        }
        dsave = (j == K) ? dkk : dsave;
        const double y = rsqrt_nr(dkk);
        const double rk = dkk * y;
        const double v = col[K] * y;
        col[K] = (j == K) ? rk : v;
        const double yk = ((j == K ? 1.0 : 0.0) - acc[K]) * y;  // Y[k][j] = D^-1[j][k]
        yrow[K] = yk;
        diag16v2_updates<K, K + 1>(col, acc, col[K], yk);
        diag16v2_pivots<K + 1>(col, acc, yrow, j, dsave, careful, p16, l, tol, d0j, badmask);
    }
}
// src: the staged tile (LDS, [i][16] row-major: src[i * 16 + j] = T[i][j]).  Pass 0 runs without the
// per-pivot tests; if a pivot then fails them (ballot) -- or the block has padding rows -- the same
// unrolled body runs again from src with the tests on (pass 1).
__device__ __forceinline__ void chol_diag16_v2(double (&col)[16], int p16, int l, int LP, double tol, const double* d0,
                                               double* Di, int* bad, double* R, double* Rinv, int* colflag, int* flag,
                                               int lane, const double* src) {
    const int j = lane & 15;
    const double d0j = d0[p16 + j];
    double acc[16], yrow[16];
    int badmask = 0;
    for (int pass = p16 + 16 > l ? 1 : 0;; ++pass) {
#pragma unroll
        for (int i = 0; i < 16; ++i) acc[i] = 0.0;
        double dsave = 0.0;
        diag16v2_pivots<0>(col, acc, yrow, j, dsave, pass != 0, p16, l, tol, d0j, badmask);
        if (pass) break;
        // lane j judges its own pivot (the test chol_diag16_dpp applies per pivot)
        const bool isbad = !(dsave > tol * d0j) || !(d0j > 0.0) || !isfinite(dsave);
        if (!__ballot(isbad && lane < 16)) break;
#pragma unroll
        for (int i = 0; i < 16; ++i) col[i] = src[i * 16 + j];
    }
#pragma unroll
    for (int i = 0; i < 16; ++i)
        if (i > j) col[i] = 0.0;
    if (lane < 16) {
#pragma unroll
        for (int i = 0; i < 16; ++i) R[(int64_t)(p16 + i) * LP + p16 + j] = col[i];
#pragma unroll
        for (int k = 0; k < 16; k += 2) {
            const double2 v2 = make_double2(yrow[k], yrow[k + 1]);
            *reinterpret_cast<double2*>(Di + j * 16 + k) = v2;
            *reinterpret_cast<double2*>(Rinv + (int64_t)(p16 + j) * LP + p16 + k) = v2;
        }
        bad[lane] = (badmask >> lane) & 1;
    }
    if (lane == 0 && badmask) {
        atomicAdd(flag, __popc(badmask));
        for (int k = 0; k < 16; ++k)
            if (badmask & (1 << k)) colflag[p16 + k] = 1;
    }
}
#ifndef RSVD_CHOL_DIAG  // the register-resident factor's diagonal blocks
#define RSVD_CHOL_DIAG chol_diag16_v2
#endif

// The split-Gram fallback test after a factor (off the pivot chain): ill = some valid pivot broke
// down or R_kk^2 <= ill_tol G_kk.  Called by the whole workgroup after its last barrier (the R
// diagonal and colflag stores of the factor are then visible workgroup-wide).
__device__ __forceinline__ void chol_ill_test(const double* __restrict__ R, int LP, int l, const double* d0,
                                              const int* __restrict__ colflag, double ill_tol, int* ill,
                                              int* ill_s, int tid, int nthr) {
    int mine = 0;
    for (int k = tid; k < l; k += nthr) {
        const double rkk = R[(int64_t)k * LP + k];
        if (colflag[k] || !(rkk * rkk > ill_tol * d0[k])) mine = 1;
    }
    if (mine) *ill_s = 1;
    __syncthreads();
    if (tid == 0) *ill = *ill_s;
}

#ifdef RSVD_CHOL_PROF
__device__ long long g_chol_prof[256];
#define CHOL_TS(k)                                               \
    do {                                                         \
        if (threadIdx.x == 0) g_chol_prof[(k)] = wall_clock64(); \
    } while (0)
#else
#define CHOL_TS(k) \
    do {           \
    } while (0)
#endif

// Upper block-triangle walk (ib <= jb < n): advance by `step` tiles; ib >= n marks the end.
struct TriWalk {
    int ib, jb, n;
    __device__ __forceinline__ TriWalk(int t, int n_) : ib(n_), jb(0), n(n_) {
        if (t < n_ * (n_ + 1) / 2) tri_decode(t, n_, ib, jb);
    }
    __device__ __forceinline__ void advance(int step) {
        jb += step;
        while (ib < n && jb >= n) {
            const int over = jb - n;
            ++ib;
            jb = ib + over;
        }
    }
};

// W is kept tile-major in MFMA output order: tile (ib, jb) at (ib * np + jb) * 256, lane (r, h)'s
// four values (rows h + 4 j, column r) contiguous -- one 32-B access per lane per tile, and the
// same registers serve as the B operand (rows 4 kk + h) of the strip product.
__device__ __forceinline__ double* wtile(double* W, int np, int ib, int jb, int lane) {
    return W + ((int64_t)ib * np + jb) * 256 + lane * 4;
}

template <int NT, int B>
__global__ __launch_bounds__(NT) void chol_wide_kernel(const double* __restrict__ G, int l, int LP,
                                                                 double tol, double* __restrict__ W,
                                                                 double* __restrict__ R, double* __restrict__ Rinv,
                                                                 int* __restrict__ colflag, int* __restrict__ flag,
                                                                 const int* __restrict__ pred, double ill_tol,
                                                                 int* __restrict__ ill, const double* __restrict__ d0src,
                                                                 int ldg) {
    if (pred && *pred == 0) return;
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    __shared__ int ill_s;
    const int np = LP / 16;
    const int ldr = LP + kCholPad;
    constexpr int nw = NT / 64;
    double* Dd = reinterpret_cast<double*>(smem_raw);  // [2][16][16] D^-1 of blocks p, p+1
    double* d0 = Dd + 512;                             // [LP] original diagonal of G
    double* Rs = d0 + LP;                              // [16][ldr] current R row strip
    double* Tsc = Rs + 16 * ldr;                       // [16][16] wave 0's look-ahead tile
    int* bad = reinterpret_cast<int*>(Tsc + 256);      // [2][16]
    const int tid = threadIdx.x;
    const int lane = tid & 63, wv = tid >> 6;
    const int r = lane & 15, h = lane >> 4;
    CHOL_TS(97);

    // W := upper block triangle of G (zero beyond l), tile-major; B tiles per wave in flight
    {
        TriWalk tw(wv, np);
        while (tw.ib < np) {
            double v[B][4];
            int tix[B];
#pragma unroll
            for (int b = 0; b < B; ++b) {
                tix[b] = tw.ib < np ? tw.ib * 64 + tw.jb : -1;
                if (tw.ib < np) {
                    const int c = 16 * tw.jb + r;
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const int i = 16 * tw.ib + h + 4 * j;
                        v[b][j] = (i < l && c < l) ? G[(int64_t)i * ldg + c] : 0.0;
                    }
                }
                tw.advance(nw);
            }
#pragma unroll
            for (int b = 0; b < B; ++b)
                if (tix[b] >= 0) {
                    double* dst = wtile(W, np, tix[b] >> 6, tix[b] & 63, lane);
                    *reinterpret_cast<double2*>(dst) = make_double2(v[b][0], v[b][1]);
                    *reinterpret_cast<double2*>(dst + 2) = make_double2(v[b][2], v[b][3]);
                }
        }
    }
    for (int i = tid; i < LP; i += NT) {
        d0[i] = (i < l) ? (d0src ? d0src[i] : G[(int64_t)i * ldg + i]) : 0.0;
        colflag[i] = 0;
    }
    if (tid == 0) ill_s = 0;
    __syncthreads();
    CHOL_TS(0);

    for (int p = -1; p < np; ++p) {  // p = -1: only the factor of diagonal block 0
        const int p16 = 16 * p;
        const double* Di = Dd + (p & 1) * 256;
        const int* bd = bad + (p & 1) * 16;
        // (1) strip R[p][jb] = D_p^-T W[p][jb] (0 for rows that broke down), to R and the LDS strip
        if (p >= 0) {
            double x[4];
#pragma unroll
            for (int kk = 0; kk < 4; ++kk) x[kk] = Di[(4 * kk + h) * 16 + r];
            int zero_rows = 0;
#pragma unroll
            for (int j = 0; j < 4; ++j) zero_rows |= (bd[h + 4 * j] || p16 + h + 4 * j >= l) << j;
            for (int jb0 = p + 1 + wv; jb0 < np; jb0 += nw * 4) {
                double2 y[4][2];
#pragma unroll
                for (int b = 0; b < 4; ++b) {
                    const int jb = jb0 + nw * b;
                    if (jb < np) {
                        const double* src = wtile(W, np, p, jb, lane);
                        y[b][0] = *reinterpret_cast<const double2*>(src);
                        y[b][1] = *reinterpret_cast<const double2*>(src + 2);
                    }
                }
#pragma unroll
                for (int b = 0; b < 4; ++b) {
                    const int jb = jb0 + nw * b;
                    if (jb < np) {
                        f64x4 acc = MD::zero();
                        acc = MD::mma(x[0], y[b][0].x, acc);
                        acc = MD::mma(x[1], y[b][0].y, acc);
                        acc = MD::mma(x[2], y[b][1].x, acc);
                        acc = MD::mma(x[3], y[b][1].y, acc);
#pragma unroll
                        for (int j = 0; j < 4; ++j) {
                            const int i = h + 4 * j;
                            const double v = ((zero_rows >> j) & 1) ? 0.0 : acc[j];
                            R[(int64_t)(p16 + i) * LP + 16 * jb + r] = v;
                            Rs[i * ldr + 16 * jb + r] = v;
                        }
                    }
                }
            }
        }
        __syncthreads();
        if (p >= 0) CHOL_TS(1 + 2 * p);
        // (2) trailing update W[ib][jb] -= R[p][ib]^T R[p][jb], p < ib <= jb.  Tile (p+1, p+1) goes to
        // wave 0, which then factors it (look-ahead); the other tiles to waves 1.., software-pipelined
        // in batches of B (loads of batch i+1 in flight while batch i is updated and stored).
        const int nt2 = np - p - 1;
        if (nt2 > 0) {
            if (wv == 0) {
                const int b1 = p + 1;
                const double* src = wtile(W, np, b1, b1, lane);
                const double2 w0 = *reinterpret_cast<const double2*>(src);
                const double2 w1 = *reinterpret_cast<const double2*>(src + 2);
                f64x4 acc = MD::zero();
                if (p >= 0) {
#pragma unroll
                    for (int kk = 0; kk < 4; ++kk)
                        acc = MD::mma(Rs[(4 * kk + h) * ldr + 16 * b1 + r], Rs[(4 * kk + h) * ldr + 16 * b1 + r], acc);
                }
                Tsc[h * 16 + r] = w0.x - acc[0];
                Tsc[(h + 4) * 16 + r] = w0.y - acc[1];
                Tsc[(h + 8) * 16 + r] = w1.x - acc[2];
                Tsc[(h + 12) * 16 + r] = w1.y - acc[3];
                __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the wave's LDS stores landed
                __builtin_amdgcn_wave_barrier();
                double col[16];
#pragma unroll
                for (int i = 0; i < 16; ++i) col[i] = Tsc[i * 16 + r];
                __builtin_amdgcn_s_waitcnt(0xc07f);
                __builtin_amdgcn_wave_barrier();
                // (the DPP form here: this factor overlaps the other waves' trailing updates, and the v2
                // form's extra registers spilled in this kernel -- LP = 512 637 -> 809 us in the lab)
                chol_diag16_dpp(col, 16 * b1, l, LP, tol, d0, Dd + (b1 & 1) * 256, bad + (b1 & 1) * 16, R, Rinv,
                                colflag, flag, lane);
            } else if (p >= 0) {
                // local tile t of the (nt2 x nt2) upper triangle; t = 0 is wave 0's
                TriWalk tw(wv, nt2);
                double2 wa[B][2], wb[B][2];
                int ta[B], tb[B];
                auto load = [&](double2 (&w)[B][2], int (&tt)[B]) {
#pragma unroll
                    for (int b = 0; b < B; ++b) {
                        tt[b] = tw.ib < nt2 ? tw.ib * 64 + tw.jb : -1;
                        if (tw.ib < nt2) {
                            const double* src = wtile(W, np, p + 1 + tw.ib, p + 1 + tw.jb, lane);
                            w[b][0] = *reinterpret_cast<const double2*>(src);
                            w[b][1] = *reinterpret_cast<const double2*>(src + 2);
                        }
                        tw.advance(nw - 1);
                    }
                };
                auto update = [&](double2 (&w)[B][2], int (&tt)[B]) {
#pragma unroll
                    for (int b = 0; b < B; ++b)
                        if (tt[b] >= 0) {
                            const int ib = p + 1 + (tt[b] >> 6), jb = p + 1 + (tt[b] & 63);
                            f64x4 acc = MD::zero();
#pragma unroll
                            for (int kk = 0; kk < 4; ++kk)
                                acc = MD::mma(Rs[(4 * kk + h) * ldr + 16 * ib + r], Rs[(4 * kk + h) * ldr + 16 * jb + r],
                                              acc);
                            double* dst = wtile(W, np, ib, jb, lane);
                            *reinterpret_cast<double2*>(dst) = make_double2(w[b][0].x - acc[0], w[b][0].y - acc[1]);
                            *reinterpret_cast<double2*>(dst + 2) = make_double2(w[b][1].x - acc[2], w[b][1].y - acc[3]);
                        }
                };
                load(wa, ta);
                for (;;) {
                    if (ta[0] < 0) break;
                    load(wb, tb);
                    update(wa, ta);
                    if (tb[0] < 0) break;
                    load(wa, ta);
                    update(wb, tb);
                }
            }
        }
        __syncthreads();
        if (p >= 0) CHOL_TS(2 + 2 * p);
    }
    if (ill) chol_ill_test(R, LP, l, d0, colflag, ill_tol, ill, &ill_s, tid, NT);
}

size_t chol_lds_bytes(int LP) {
    return (size_t)512 * 8 + (size_t)LP * 8 + (size_t)16 * (LP + kCholPad) * 8 + 256 * 8 + 32 * 4 + 64;
}

// ------------------------------------------------------------------------------------------------
// Register-resident Cholesky (LP <= 256).  chol_wide_kernel keeps the Gram being reduced in global
// memory (L2), so every block step pays two L2 round trips per tile on top of its barriers
// (10 us per 16-column step at LP = 256).  Here the upper block triangle of G lives in the
// REGISTERS of one 512-thread workgroup: upper-triangle tile t (row-major order) belongs to wave
// t % 8, slot t / 8, in MFMA output layout (lane (r, h): rows h + 4 j, column r) -- LP = 256 is 136
// tiles, 17 slots = 136 VGPRs per lane.  Row-major dealing spreads every tile row over consecutive
// waves, so the trailing triangle of each step is balanced to one tile per row.  Per block step p:
//   (A) the owner of tile (p, p) factors it (16x16 upper Cholesky + inverse, lane j owning column j),
//       D^-1 to LDS;                                                              -- barrier
//   (B) the owners of row p form the strip R[p][jb] = D_p^-T W[p][jb] (4 MFMAs), to R and to LDS;
//                                                                                 -- barrier
//   (C) every wave updates its trailing tiles W[ib][jb] -= R[p][ib]^T R[p][jb] from the LDS strip.
// (C) of step p and (A) of step p + 1 touch only the owner's registers, so two barriers per step.
// Same operations in the same order as chol_wide_kernel: bit-identical R.
constexpr int kCholRegWaves = 8;

template <int NP> struct CholReg {
    static constexpr int LP = 16 * NP, NW = kCholRegWaves, NT = NP * (NP + 1) / 2, S = (NT + NW - 1) / NW;
    // the first SL slots of every wave (rows retired earliest) live in LDS: VGPR budget at 2 waves/SIMD
    static constexpr int SL = S > 10 ? S - 10 : 0;
    static constexpr int LDR = LP + kCholPad;
    static constexpr size_t lds_bytes = (size_t)(512 + 256 + LP + 16 * LDR + NW * SL * 256) * 8 + 32 * 4;
};

__device__ __forceinline__ bf16_t f2bf(float x) {  // round to nearest even
    const uint32_t u = __float_as_uint(x);
    if ((u & 0x7f800000u) == 0x7f800000u) return (bf16_t)(u >> 16);
    return (bf16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}
__device__ __forceinline__ float bf2f(bf16_t b) { return __uint_as_float((uint32_t)b << 16); }

// The three bf16 pieces of the fp32 element (row k, column c) of an LP x LP matrix in split_mat_kernel's
// transposed piece images (Mt[x][c][k], image pitch L2 = LP^2): the factor kernels that write R^-1's
// fp32 copy also write its pieces, so the split panel product needs no split_mat launch.
__device__ __forceinline__ void store_pieces(bf16_t* __restrict__ Mt, int64_t L2, int64_t idx, float v) {
    const bf16_t bh = f2bf(v);
    const float rm = v - bf2f(bh);
    const bf16_t bm = f2bf(rm);
    Mt[idx] = bh;
    Mt[L2 + idx] = bm;
    Mt[2 * L2 + idx] = f2bf(rm - bf2f(bm));
}

// R^-1 inside the factor's own launch (round 5; NP <= 8, every leaf of the two- and three-level
// factors): the products of rinv_wide_kernel in the same order, bit-identical, but one WAVE per
// 16-column block column jb instead of one workgroup.  X[k] never leaves the wave -- its MFMA output
// layout (row h + 4 j, column r) is the B operand (rows 4 kk + h) of the next product -- so the steps
// need no workgroup barrier, and R's upper block triangle (diagonal slots: D^-1 from Rinv) is staged
// once in LDS in A-operand order (tile t of the triangle at img + 256 t, lane L's four k-values
// contiguous).  Saves the rinv_wide launch (~14 us per leaf) for ~4 us here.
template <int NP> struct CholRegInv {
    static constexpr int NT = NP * (NP + 1) / 2, NTH = 64 * kCholRegWaves;
    static constexpr int NE = (NT * 256 + NTH - 1) / NTH;  // staged doubles per thread
    static constexpr size_t lds_bytes = (size_t)NT * 256 * 8;
};
__device__ __forceinline__ int tri_index(int p, int k, int np) { return p * np - p * (p - 1) / 2 + (k - p); }

// Below the block diagonal of an LP x LP factor: zeros in R, Rinv, Rinv32 (row-major) and the pieces
// (transposed), each array walked in its own layout so every store instruction is contiguous.
__device__ __forceinline__ void chol_lower_zeros(int LP, double* __restrict__ R, double* __restrict__ Rinv,
                                                 float* __restrict__ Rinv32, bf16_t* __restrict__ Mt, int t0,
                                                 int nthr) {
    const int64_t L2 = (int64_t)LP * LP;
    for (int e = t0; e < LP * LP; e += nthr) {
        const int a = e / LP, b = e % LP;
        if (a >= 16 * (b / 16 + 1)) {  // row a, column b
            R[e] = 0.0;
            Rinv[e] = 0.0;
            if (Rinv32) Rinv32[e] = 0.0f;
        }
        if (Mt && b >= 16 * (a / 16 + 1)) {  // column a, row b
            Mt[e] = 0;
            Mt[L2 + e] = 0;
            Mt[2 * L2 + e] = 0;
        }
    }
}

template <int NP>
__device__ __forceinline__ void chol_reg_rinv(double* __restrict__ img, double* __restrict__ R,
                                              double* __restrict__ Rinv, float* __restrict__ Rinv32,
                                              bf16_t* __restrict__ Mt, int tid, int wv, int lane) {
    typedef CholRegInv<NP> C;
    constexpr int LP = 16 * NP;
    const int64_t L2 = (int64_t)LP * LP;
    const int r = lane & 15, h = lane >> 4;
    __syncthreads();  // the factor's LDS is dead; its R / Rinv stores are visible workgroup-wide
    {
        // the full NP x NP tile grid, upper triangle kept: shifts only, every load issued before any store
        constexpr int NF = NP * NP * 256 / C::NTH;
        double v[NF];
#pragma unroll
        for (int i = 0; i < NF; ++i) {
            const int e = tid + i * C::NTH;
            const int t2 = e >> 8, p = t2 / NP, k = t2 % NP, L = (e >> 2) & 63, kk = e & 3;
            const int64_t src = (int64_t)(16 * p + (L & 15)) * LP + 16 * k + 4 * kk + (L >> 4);
            v[i] = 0.0;
            if (p < k) v[i] = R[src];
            else if (p == k) v[i] = Rinv[src];
        }
#pragma unroll
        for (int i = 0; i < NF; ++i) {
            const int e = tid + i * C::NTH;
            const int t2 = e >> 8, p = t2 / NP, k = t2 % NP;
            if (p <= k) img[tri_index(p, k, NP) * 256 + (e & 255)] = v[i];
        }
    }
    __syncthreads();
    CHOL_TS(210);
    // column jb's 2 jb^2 + 6 jb MFMAs: waves w and w + 4 share a SIMD, so pair the long columns with
    // the short ones (NP = 8: 7 + 0, 6 + 1, 5 + 2, 4 + 3; 140 MFMAs on the busiest SIMD instead of 176)
    const int jb = NP == 8 ? (wv < 4 ? 7 - wv : wv - 4) : wv, c0 = 16 * jb;
    if (jb >= NP) return;
    f64x4 T[NP];
#pragma unroll
    for (int s = 0; s < NP; ++s) T[s] = MD::zero();
    for (int k = jb; k >= 0; --k) {
        const double* dk = img + tri_index(k, k, NP) * 256;
        f64x4 x;
        if (k == jb) {  // D_jb^-1 in output layout: element (h + 4 j, r) sits in lane (h + 4 j) + 16 (r & 3), slot r >> 2
#pragma unroll
            for (int j = 0; j < 4; ++j) x[j] = dk[((h + 4 * j) + 16 * (r & 3)) * 4 + (r >> 2)];
        } else {
            f64x4 t = MD::zero();
#pragma unroll
            for (int s = 0; s < NP; ++s)
                if (s == k) t = T[s];
            const double2 d01 = *reinterpret_cast<const double2*>(dk + lane * 4);
            const double2 d23 = *reinterpret_cast<const double2*>(dk + lane * 4 + 2);
            f64x4 o = MD::zero();
            o = MD::mma(d01.x, t[0], o);
            o = MD::mma(d01.y, t[1], o);
            o = MD::mma(d23.x, t[2], o);
            o = MD::mma(d23.y, t[3], o);
#pragma unroll
            for (int j = 0; j < 4; ++j) x[j] = -o[j];
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int i = h + 4 * j;
            if (k != jb) Rinv[(int64_t)(16 * k + i) * LP + c0 + r] = x[j];
            if (Rinv32) Rinv32[(int64_t)(16 * k + i) * LP + c0 + r] = (float)x[j];
            if (Mt) store_pieces(Mt, L2, (int64_t)(c0 + r) * LP + 16 * k + i, (float)x[j]);
        }
#pragma unroll
        for (int s = NP - 1; s >= 0; --s)  // T[k - 1] first: the next step's product waits on it
            if (s < k) {
                const double* a = img + tri_index(s, k, NP) * 256 + lane * 4;
                const double2 a01 = *reinterpret_cast<const double2*>(a);
                const double2 a23 = *reinterpret_cast<const double2*>(a + 2);
                T[s] = MD::mma(a01.x, x[0], T[s]);
                T[s] = MD::mma(a01.y, x[1], T[s]);
                T[s] = MD::mma(a23.x, x[2], T[s]);
                T[s] = MD::mma(a23.y, x[3], T[s]);
            }
    }
#ifdef RSVD_CHOL_PROF
    if (lane == 0) g_chol_prof[211 + jb] = wall_clock64();
#endif
    // the zeros below the block diagonal: on the waves of the short columns, after their column
    if (2 * jb < NP) chol_lower_zeros(LP, R, Rinv, Rinv32, Mt, jb * 64 + lane, NP / 2 * 64);
}

template <int NP>
__global__ __launch_bounds__(64 * kCholRegWaves) void chol_reg_kernel(const double* __restrict__ G, int l, double tol,
                                                                      double* __restrict__ R, double* __restrict__ Rinv,
                                                                      int* __restrict__ colflag, int* __restrict__ flag,
                                                                      const int* __restrict__ pred, double ill_tol,
                                                                      int* __restrict__ ill, const double* __restrict__ d0src,
                                                                      int ldg, float* __restrict__ Rinv32,
                                                                      bf16_t* __restrict__ Mt, int fuse_rinv) {
    if (pred && *pred == 0) return;
    typedef CholReg<NP> C;
    __shared__ int ill_s;
    constexpr int LP = C::LP, NW = C::NW, NT = C::NT, S = C::S, SL = C::SL, LDR = C::LDR;
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    double* Di = reinterpret_cast<double*>(smem_raw);  // [2][256]
    double* Tsc = Di + 512;                            // [256]
    double* d0 = Tsc + 256;                            // [LP]
    double* Rs = d0 + LP;                              // [16][LDR]
    double* wl = Rs + 16 * LDR;                        // [NW][SL][64 lanes][4]
    int* bad = reinterpret_cast<int*>(wl + NW * SL * 256);  // [2][16]
    const int tid = threadIdx.x, lane = tid & 63;
    const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r = lane & 15, h = lane >> 4;
    double* wlw = wl + wv * SL * 256 + lane * 4;
    CHOL_TS(97);

    int tib[S], tjb[S];
    double wt[S - SL > 0 ? S - SL : 1][4];
#pragma unroll
    for (int s = 0; s < S; ++s) {
        tib[s] = NP;  // empty slot: never active
        tjb[s] = NP;
        const int t = s * NW + wv;
        if (t < NT) tri_decode(t, NP, tib[s], tjb[s]);
        double v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int i = 16 * tib[s] + h + 4 * j, c = 16 * tjb[s] + r;
            v[j] = (t < NT && i < l && c < l) ? G[(int64_t)i * ldg + c] : 0.0;
        }
        if (s < SL) {
            *reinterpret_cast<double2*>(wlw + s * 256) = make_double2(v[0], v[1]);
            *reinterpret_cast<double2*>(wlw + s * 256 + 2) = make_double2(v[2], v[3]);
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) wt[s < SL ? 0 : s - SL][j] = v[j];
        }
    }
    auto get = [&](int s, double (&v)[4]) {
        if (s < SL) {
            const double2 a = *reinterpret_cast<const double2*>(wlw + s * 256);
            const double2 b = *reinterpret_cast<const double2*>(wlw + s * 256 + 2);
            v[0] = a.x; v[1] = a.y; v[2] = b.x; v[3] = b.y;
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] = wt[s < SL ? 0 : s - SL][j];
        }
    };
    for (int i = tid; i < LP; i += 64 * NW) {
        d0[i] = (i < l) ? (d0src ? d0src[i] : G[(int64_t)i * ldg + i]) : 0.0;
        colflag[i] = 0;
    }
    if (tid == 0) ill_s = 0;
    __syncthreads();
    CHOL_TS(200);

    for (int p = 0; p < NP; ++p) {
        const int p16 = 16 * p;
        // (A) factor the diagonal tile (p, p) on its owner wave
        const int tpp = p * NP - p * (p - 1) / 2;
        if (wv == tpp % NW) {
            const int sp = tpp / NW;
#pragma unroll
            for (int s = 0; s < S; ++s)
                if (s == sp) {
                    double v[4];
                    get(s, v);
#pragma unroll
                    for (int j = 0; j < 4; ++j) Tsc[(h + 4 * j) * 16 + r] = v[j];
                }
            __builtin_amdgcn_s_waitcnt(0xc07f);
            __builtin_amdgcn_wave_barrier();
            double col[16];
#pragma unroll
            for (int i = 0; i < 16; ++i) col[i] = Tsc[i * 16 + r];
            __builtin_amdgcn_s_waitcnt(0xc07f);
            __builtin_amdgcn_wave_barrier();
            RSVD_CHOL_DIAG(col, p16, l, LP, tol, d0, Di + (p & 1) * 256, bad + (p & 1) * 16, R, Rinv,
                           colflag, flag, lane, Tsc);
        }
        __syncthreads();
        if (p < 32) CHOL_TS(1 + 3 * p);
        if (p == NP - 1) {
            if (ill) chol_ill_test(R, LP, l, d0, colflag, ill_tol, ill, &ill_s, tid, 64 * NW);
            break;
        }
        // (B) strip R[p][jb] = D_p^-T W[p][jb] (0 for rows that broke down or are padding)
        {
            const double* Dp = Di + (p & 1) * 256;
            const int* bd = bad + (p & 1) * 16;
            double x[4];
#pragma unroll
            for (int kk = 0; kk < 4; ++kk) x[kk] = Dp[(4 * kk + h) * 16 + r];
            int zero_rows = 0;
#pragma unroll
            for (int j = 0; j < 4; ++j) zero_rows |= (bd[h + 4 * j] || p16 + h + 4 * j >= l) << j;
#pragma unroll
            for (int s = 0; s < S; ++s)
                if (tib[s] == p && tjb[s] > p) {
                    double v[4];
                    get(s, v);
                    f64x4 acc = MD::zero();
#pragma unroll
                    for (int kk = 0; kk < 4; ++kk) acc = MD::mma(x[kk], v[kk], acc);
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const int i = h + 4 * j;
                        const double o = ((zero_rows >> j) & 1) ? 0.0 : acc[j];
                        R[(int64_t)(p16 + i) * LP + 16 * tjb[s] + r] = o;
                        Rs[i * LDR + 16 * tjb[s] + r] = o;
                    }
                }
        }
        __syncthreads();
        if (p < 32) CHOL_TS(2 + 3 * p);
        // (C) trailing update of the tiles below row p
#pragma unroll
        for (int s = 0; s < S; ++s)
            if (tib[s] > p && tib[s] < NP) {
                f64x4 acc = MD::zero();
#pragma unroll
                for (int kk = 0; kk < 4; ++kk)
                    acc = MD::mma(Rs[(4 * kk + h) * LDR + 16 * tib[s] + r], Rs[(4 * kk + h) * LDR + 16 * tjb[s] + r], acc);
                if (s < SL) {
                    double v[4];
                    get(s, v);
                    *reinterpret_cast<double2*>(wlw + s * 256) = make_double2(v[0] - acc[0], v[1] - acc[1]);
                    *reinterpret_cast<double2*>(wlw + s * 256 + 2) = make_double2(v[2] - acc[2], v[3] - acc[3]);
                } else {
#pragma unroll
                    for (int j = 0; j < 4; ++j) wt[s < SL ? 0 : s - SL][j] -= acc[j];
                }
            }
        if (p < 32) CHOL_TS(3 + 3 * p);
    }
    if constexpr (NP <= 8) {
        if (fuse_rinv) chol_reg_rinv<NP>(reinterpret_cast<double*>(smem_raw), R, Rinv, Rinv32, Mt, tid, wv, lane);
    }
}

// R^-1 = blocked back substitution, one workgroup (4 waves) per 16-column block jb, all block
// columns in parallel:  X[jb] = D_jb^-1,  X[p] = -D_p^-1 T[p],  T[p] = sum_{p<k<=jb} R[p][k] X[k].
// Right-looking: as soon as X[k] is known every wave adds R[p][k] X[k] to the accumulators T[p] it
// owns (p = wave + 4 s, in registers), so each step is one MFMA group per owned block, one 16x16
// product on the owner wave and ONE barrier (X double-buffered in LDS); the R tiles of the next step are loaded a step ahead.
// (An accumulator in MFMA output layout -- row h + 4 j, column r in lane (r, h) -- is already the
// B operand of the next product: rows 4 kk + h.)  Also: zeros below the block diagonal of R and
// R^-1, and the fp32 copy of this block column of R^-1.
constexpr int kRinvSlots = 8;  // LP <= 512: 32 block rows over 4 waves

__global__ __launch_bounds__(256) void rinv_wide_kernel(int LP, double* __restrict__ R, double* __restrict__ Rinv,
                                                        float* __restrict__ Rinv32, const int* __restrict__ pred,
                                                        bf16_t* __restrict__ Mt) {
    const int64_t L2 = (int64_t)LP * LP;
    if (pred && *pred == 0) return;
    __shared__ double Xs[2][256];  // X[k] of the current step (buffer k & 1), row-major
    const int jb = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int r = lane & 15, h = lane >> 4;
    const int c0 = 16 * jb;
    // below the block diagonal: zeros
    for (int e = tid; e < (LP - c0 - 16) * 16; e += 256) {
        const int i = c0 + 16 + e / 16, c = c0 + e % 16;
        R[(int64_t)i * LP + c] = 0.0;
        Rinv[(int64_t)i * LP + c] = 0.0;
        if (Rinv32) Rinv32[(int64_t)i * LP + c] = 0.0f;
        if (Mt) store_pieces(Mt, L2, (int64_t)c * LP + i, 0.0f);
    }
    f64x4 T[kRinvSlots];
    double Rc[kRinvSlots][4], Rn[kRinvSlots][4], Dn[4];
#pragma unroll
    for (int s = 0; s < kRinvSlots; ++s) T[s] = MD::zero();
    // R[p][k] A-operands (row r, column 4 kk + h) of the step k for the blocks p < k this wave owns
    auto load_r = [&](double (&dst)[kRinvSlots][4], int k) {
#pragma unroll
        for (int s = 0; s < kRinvSlots; ++s) {
            const int p = wv + 4 * s;
            if (p < k) {
#pragma unroll
                for (int kk = 0; kk < 4; ++kk) dst[s][kk] = R[(int64_t)(16 * p + r) * LP + 16 * k + 4 * kk + h];
            }
        }
    };
    // D_k^-1 as the A operand (row r, column 4 kk + h), loaded one owned step ahead
    auto load_d = [&](int k) {
        if (k >= 0) {
#pragma unroll
            for (int kk = 0; kk < 4; ++kk) Dn[kk] = Rinv[(int64_t)(16 * k + r) * LP + 16 * k + 4 * kk + h];
        }
    };
    {
        int k1 = jb - 1;
        while (k1 >= 0 && (k1 & 3) != wv) --k1;
        load_d(k1);
    }
    load_r(Rc, jb);
    for (int k = jb; k >= 0; --k) {
        const int own = k & 3;
        if (k > 0) load_r(Rn, k - 1);
        if (wv == own) {
            f64x4 x;
            if (k == jb) {
#pragma unroll
                for (int j = 0; j < 4; ++j) x[j] = Rinv[(int64_t)(c0 + h + 4 * j) * LP + c0 + r];
            } else {
                f64x4 t = MD::zero();
#pragma unroll
                for (int s = 0; s < kRinvSlots; ++s)
                    if (wv + 4 * s == k) t = T[s];
                f64x4 o = MD::zero();
#pragma unroll
                for (int kk = 0; kk < 4; ++kk) o = MD::mma(Dn[kk], t[kk], o);
#pragma unroll
                for (int j = 0; j < 4; ++j) x[j] = -o[j];
                load_d(k - 4);
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int i = h + 4 * j;
                Xs[k & 1][i * 16 + r] = x[j];
                if (k != jb) Rinv[(int64_t)(16 * k + i) * LP + c0 + r] = x[j];
                if (Rinv32) Rinv32[(int64_t)(16 * k + i) * LP + c0 + r] = (float)x[j];
                if (Mt) store_pieces(Mt, L2, (int64_t)(c0 + r) * LP + 16 * k + i, (float)x[j]);
            }
        }
        __syncthreads();
        if (k > 0) {
            double xb[4];
#pragma unroll
            for (int kk = 0; kk < 4; ++kk) xb[kk] = Xs[k & 1][(4 * kk + h) * 16 + r];
#pragma unroll
            for (int s = 0; s < kRinvSlots; ++s) {
                const int p = wv + 4 * s;
                if (p < k) {
#pragma unroll
                    for (int kk = 0; kk < 4; ++kk) T[s] = MD::mma(Rc[s][kk], xb[kk], T[s]);
                }
            }
#pragma unroll
            for (int s = 0; s < kRinvSlots; ++s)
#pragma unroll
                for (int kk = 0; kk < 4; ++kk) Rc[s][kk] = Rn[s][kk];
        }
    }
}

// ------------------------------------------------------------------------------------------------
// Out = In * M.  Workgroup = 64 rows x CT columns (4 waves x 16 rows; LP > CT -> column blocks,
// adjacent on one XCD so In rows are re-read from L2).  K runs in chunks staged through LDS with
// 16-B loads of M (given in T precision); a lane's In vector (float4 / double2) feeds VW MFMAs
// (k-slot h of MFMA t <-> k = k0 + VW h + t), the chunk's In vectors are loaded before the M
// staging so their latency overlaps it.  fp32: v_mfma_f32_16x16x4_f32; fp64: the f64 form.
// Upper-triangular M (R^-1): K stops at the block's last column (no per-tile skipping inside the
// unrolled MFMA loop: a data-dependent skip there makes hipcc shuffle the accumulators).
template <typename T> struct PG;
template <> struct PG<float> {
    typedef float4 V;
    static constexpr int VW = 4, PAD = 4;  // pitch CT+4: the two k-rows of a half-wave hit disjoint banks
    typedef Mfma<float> M;
};
template <> struct PG<double> {
    typedef double2 V;
    static constexpr int VW = 2, PAD = 8;
    typedef Mfma<double> M;
};


template <typename T, int CT>
__global__ __launch_bounds__(256) void panel_gemm_kernel(const T* __restrict__ In, int64_t rows, int LP,
                                                         const T* __restrict__ Mm, int upper, T* __restrict__ Out,
                                                         int64_t ldo, int cols, bf16_t* __restrict__ hi,
                                                         bf16_t* __restrict__ lo, int ncb,
                                                         const int* __restrict__ pred) {
    if (pred && *pred == 0) return;
    typedef PG<T> C;
    typedef typename C::M M;
    typedef typename C::V V;
    constexpr int VW = C::VW;
    constexpr int G = CT / 16;
    constexpr int NJ = 4;             // k-steps of 4 VW per chunk
    constexpr int KC = NJ * 4 * VW;   // 64 (fp32) / 32 (fp64)
    constexpr int MP = CT + C::PAD;   // LDS pitch of the M chunk
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    T* Ms = reinterpret_cast<T*>(smem_raw);  // [KC][MP]
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int r = lane & 15, h = lane >> 4;
    const int bid = xcd_remap(blockIdx.x, gridDim.x);
    const int cb = bid % ncb;
    const int64_t row0 = (int64_t)(bid / ncb) * 64;
    const int c0 = cb * CT;
    const int64_t row = row0 + 16 * w + r;
    const bool rok = row < rows;
    const int kmax = upper ? ((c0 + CT < LP) ? c0 + CT : LP) : LP;
    typename M::acc_t acc[G];
#pragma unroll
    for (int g = 0; g < G; ++g) acc[g] = M::zero();
    for (int kc = 0; kc < kmax; kc += KC) {
        V a[NJ];
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const int k = kc + 4 * VW * j + VW * h;
            if (rok && k < LP) {
                a[j] = *reinterpret_cast<const V*>(In + row * LP + k);
            } else {
                T* e = reinterpret_cast<T*>(&a[j]);
#pragma unroll
                for (int t = 0; t < VW; ++t) e[t] = T(0);
            }
        }
        __syncthreads();  // the previous chunk's LDS reads are done
        for (int e = tid; e < KC * CT / VW; e += 256) {
            const int kr = e / (CT / VW), cv = (e % (CT / VW)) * VW;
            V v;
            if (kc + kr < LP && c0 + cv < LP) {
                v = *reinterpret_cast<const V*>(Mm + (int64_t)(kc + kr) * LP + c0 + cv);
            } else {
                T* x = reinterpret_cast<T*>(&v);
#pragma unroll
                for (int t = 0; t < VW; ++t) x[t] = T(0);
            }
            *reinterpret_cast<V*>(Ms + kr * MP + cv) = v;
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
            const int k0 = kc + 4 * VW * j;
            if (k0 >= kmax) break;
            const T* ae = reinterpret_cast<const T*>(&a[j]);
#pragma unroll
            for (int t = 0; t < VW; ++t) {
                const T* mrow = Ms + (4 * VW * j + VW * h + t) * MP + r;
#pragma unroll
                for (int g = 0; g < G; ++g) acc[g] = M::mma(ae[t], mrow[16 * g], acc[g]);
            }
        }
    }
    // epilogue.  D: col = r (output column), row = M::row(h, j) (output row within the wave's 16)
    if (ldo == 0) {
#pragma unroll
        for (int g = 0; g < G; ++g)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int64_t orow = row0 + 16 * w + M::row(h, j);
                const int c = c0 + 16 * g + r;
                if (orow < rows && c < LP) {
                    const T v = (T)acc[g][j];
                    if (Out) Out[orow * LP + c] = v;  // null: only the bf16 hi / lo panels are wanted
                    if (hi) {
                        const bf16_t bh = f2bf((float)v);
                        hi[orow * LP + c] = bh;
                        if (lo) lo[orow * LP + c] = f2bf((float)v - bf2f(bh));
                    }
                }
            }
        return;
    }
    // column-major caller output: transpose through LDS, store column segments contiguously
    __syncthreads();
    T* Ts = Ms;  // [CT][64 + 1]  (fits: KC * MP >= CT * 65 is checked at launch)
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
        for (int j = 0; j < 4; ++j) Ts[(16 * g + r) * 65 + 16 * w + M::row(h, j)] = acc[g][j];
    __syncthreads();
    for (int e = tid; e < CT * 64; e += 256) {
        const int c = e / 64, lr = e % 64;
        if (c0 + c < cols && row0 + lr < rows) Out[row0 + lr + (int64_t)(c0 + c) * ldo] = Ts[c * 65 + lr];
    }
}

// ------------------------------------------------------------------------------------------------
// Out = In * M for fp32 panels on the bf16 MFMA (panel_split_kernel): the three-piece split of
// the Gram kernel on both operands (In = h + m + t per element in registers, M pre-split into
// transposed piece images Mt[x][c][k] by split_mat_kernel) and the six products hH, hM, mH, mM,
// hT, tH per 32-deep k-step -- each term exact in fp32, the fp32 accumulation as the fp32 MFMA's.
// Six bf16 MFMAs cost 6/16 of one fp32 MFMA of the same shape: the product becomes a read of In
// plus the writes.  Workgroup: 128 rows x 128 columns (4 waves x 32 rows, 8 column tiles), M's
// 32 x 128 piece chunk staged in LDS per k-step (double-buffered, 64-B columns, 16-B units
// swizzled by (c >> 1) & 3 as the Gram images), In's fragment (8 consecutive k of one row) loaded
// one k-step ahead.  Upper-triangular M: K stops at the block's last column.
__global__ void split_mat_kernel(const float* __restrict__ M, int LP, bf16_t* __restrict__ Mt) {
    // Mt[x][c][k] = piece x of M[k][c]
    const int64_t L2 = (int64_t)LP * LP;
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < L2; e += (int64_t)gridDim.x * blockDim.x) {
        const int c = (int)(e / LP), k = (int)(e % LP);
        const float v = M[(int64_t)k * LP + c];
        const bf16_t bh = f2bf(v);
        const float rm = v - bf2f(bh);
        const bf16_t bm = f2bf(rm);
        Mt[e] = bh;
        Mt[L2 + e] = bm;
        Mt[2 * L2 + e] = f2bf(rm - bf2f(bm));
    }
}

// RT2 row tiles (16 rows each) per wave, CT output columns per workgroup: the workgroup covers
// 64 RT2 rows x CT columns.  M's next chunk is loaded into registers while the current one is
// multiplied and written to the free LDS buffer after the MFMAs; the first version loaded and
// wrote it in one place before the MFMAs, exposing the L2 latency every step, and transposed
// column-major outputs through LDS.  Same shape (RT2 = 2, CT = 128), same box: C5 m-side product
// 454 -> 318 us, n side 51 -> 31 us, C4 74 -> 59 us (C5 31.0 -> 30.1 ms, C3 7.90 -> 7.50 ms).
template <typename F, int... I>
__device__ __forceinline__ void qr_static_for_impl(F& f, std::integer_sequence<int, I...>) {
    (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void qr_static_for(F& f) {
    qr_static_for_impl(f, std::make_integer_sequence<int, N>{});
}

// PD: In's fragments come through a ring of PD register sets, PD - 1 k-steps ahead (round 5: one
// step ahead left an HBM round trip exposed in every step of the short LP = 128 products).  The
// loads are unpredicated so the waits count them: rows past `rows` read the last row again, which
// only reaches output rows that are never stored (an MFMA output row depends on its A row alone).
template <int RT2, int CT, int PD = 2>
__global__ __launch_bounds__(256, 2) void panel_split_kernel(const float* __restrict__ In, int64_t rows, int LP,
                                                          const bf16_t* __restrict__ Mt, int upper,
                                                          float* __restrict__ Out, int64_t ldo, int cols,
                                                          bf16_t* __restrict__ hi, bf16_t* __restrict__ lo, int ncb,
                                                          const int* __restrict__ pred) {
    if (pred && *pred == 0) return;
    constexpr int G = CT / 16, IMG = CT * 64, STEPB = 3 * IMG, WR = 64 * RT2, NU = 3 * CT / 64;
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int r = lane & 15, h = lane >> 4;
    const int bid = xcd_remap(blockIdx.x, gridDim.x);
    const int cb = bid % ncb;
    const int64_t row0 = (int64_t)(bid / ncb) * WR;
    const int c0 = cb * CT;
    const int kmax = upper ? ((c0 + CT < LP) ? c0 + CT : LP) : LP;
    const int nk = (kmax + 31) / 32;
    const int64_t L2 = (int64_t)LP * LP;
    f32x4 acc[RT2][G];
#pragma unroll
    for (int t = 0; t < RT2; ++t)
#pragma unroll
        for (int g = 0; g < G; ++g) acc[t][g] = f32x4{0.f, 0.f, 0.f, 0.f};
    // M chunk: 3 pieces x CT columns x 64 B = 12 CT 16-B units, NU per thread
    uint4 mreg[NU];
    auto loadM = [&](int ks) {
#pragma unroll
        for (int t = 0; t < NU; ++t) {
            const int u = tid + 256 * t;
            const int x = u / (4 * CT), rem = u % (4 * CT), c = rem >> 2, un = rem & 3;
            mreg[t] = make_uint4(0u, 0u, 0u, 0u);
            if (c0 + c < LP) mreg[t] = *reinterpret_cast<const uint4*>(Mt + x * L2 + (int64_t)(c0 + c) * LP + 32 * ks + 8 * un);
        }
    };
    auto writeM = [&](char* img) {
#pragma unroll
        for (int t = 0; t < NU; ++t) {
            const int u = tid + 256 * t;
            const int x = u / (4 * CT), rem = u % (4 * CT), c = rem >> 2, un = rem & 3;
            *reinterpret_cast<uint4*>(img + x * IMG + c * 64 + 16 * (un ^ ((c >> 1) & 3))) = mreg[t];
        }
    };
    // In's fragments (8 consecutive k of the lane's row per row tile), ring of PD sets
    float4 ab[PD][RT2][2];
    auto loadA = [&](int ks, float4 (&a)[RT2][2]) {
        const int k = 32 * (ks < nk ? ks : nk - 1) + 8 * h;
#pragma unroll
        for (int t = 0; t < RT2; ++t) {
            const int64_t row = row0 + 16 * RT2 * w + 16 * t + r;
            const float* src = In + (row < rows ? row : rows - 1) * LP + k;
            a[t][0] = *reinterpret_cast<const float4*>(src);
            a[t][1] = *reinterpret_cast<const float4*>(src + 4);
        }
    };
    const uint32_t lofs = (uint32_t)(r * 64 + 16 * (h ^ ((r >> 1) & 3)));
    if (nk > 0) {
#pragma unroll
        for (int j = 0; j < PD - 1; ++j) loadA(j, ab[j]);
        loadM(0);
        writeM(smem_raw);
    }
    auto step = [&](int ks, float4 (&cur)[RT2][2], float4 (&ahead)[RT2][2]) __attribute__((always_inline)) {
        const char* img = smem_raw + (ks & 1) * STEPB;
        __syncthreads();  // chunk ks written; the readers of chunk ks - 1 (the other buffer) are done
        const bool more = ks + 1 < nk;
        loadA(ks + PD - 1, ahead);
        if (more) loadM(ks + 1);
        // In fragments of this k-step: three pieces of 8 consecutive k of the lane's row, per row tile
        bf16x8s fa[RT2][3];
#pragma unroll
        for (int t = 0; t < RT2; ++t) {
            const float v[8] = {cur[t][0].x, cur[t][0].y, cur[t][0].z, cur[t][0].w,
                                cur[t][1].x, cur[t][1].y, cur[t][1].z, cur[t][1].w};
            uint32_t ph[4], pm[4], pt[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                ph[j] = cvt_pk_bf16(v[2 * j], v[2 * j + 1]);
                const float ra = v[2 * j] - __uint_as_float(ph[j] << 16);
                const float rb = v[2 * j + 1] - __uint_as_float(ph[j] & 0xffff0000u);
                pm[j] = cvt_pk_bf16(ra, rb);
                pt[j] = cvt_pk_bf16(ra - __uint_as_float(pm[j] << 16), rb - __uint_as_float(pm[j] & 0xffff0000u));
            }
            fa[t][0] = __builtin_bit_cast(bf16x8s, make_uint4(ph[0], ph[1], ph[2], ph[3]));
            fa[t][1] = __builtin_bit_cast(bf16x8s, make_uint4(pm[0], pm[1], pm[2], pm[3]));
            fa[t][2] = __builtin_bit_cast(bf16x8s, make_uint4(pt[0], pt[1], pt[2], pt[3]));
        }
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const char* base = img + g * 1024 + lofs;
            const bf16x8s bh = *reinterpret_cast<const bf16x8s*>(base);
            const bf16x8s bm = *reinterpret_cast<const bf16x8s*>(base + IMG);
            const bf16x8s bt = *reinterpret_cast<const bf16x8s*>(base + 2 * IMG);
#pragma unroll
            for (int t = 0; t < RT2; ++t) {
                f32x4 c = acc[t][g];
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[t][2], bh, c, 0, 0, 0);  // smallest terms first
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[t][0], bt, c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[t][1], bm, c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[t][1], bh, c, 0, 0, 0);
                c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[t][0], bm, c, 0, 0, 0);
                acc[t][g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[t][0], bh, c, 0, 0, 0);
            }
        }
        if (more) writeM(smem_raw + ((ks + 1) & 1) * STEPB);
    };
    // whole groups of PD steps (each set at a fixed position in the ring), then the rest
    int ks0 = 0;
    for (; ks0 + PD <= nk; ks0 += PD) {
        auto one = [&](auto jc) {
            constexpr int j = decltype(jc)::value;
            step(ks0 + j, ab[j], ab[(j + PD - 1) % PD]);
        };
        qr_static_for<PD>(one);
    }
    {
        auto one = [&](auto jc) {
            constexpr int j = decltype(jc)::value;
            if (ks0 + j < nk) step(ks0 + j, ab[j], ab[(j + PD - 1) % PD]);
        };
        qr_static_for<PD>(one);
    }
    // epilogue.  bf16 MFMA D: col = r (output column c0 + 16 g + r), row = 4 h + j within the 16-row tile.
    // Row-major outputs go through LDS, 64 rows at a time (in the M buffers): a lane then owns 8
    // consecutive columns of one row and stores them as 32 B of fp32 and 16 B each of hi / lo --
    // from the accumulators a lane's values sit in 4 different rows, i.e. 2-byte hi / lo stores.
    if (ldo == 0) {
        constexpr int TP = CT + 4;  // fp32 pitch of the staged rows
        static_assert(64 * TP * 4 <= 2 * STEPB, "epilogue tile fits the M buffers");
        float* Ts = reinterpret_cast<float*>(smem_raw);
#pragma unroll
        for (int ch = 0; ch < RT2; ++ch) {  // 64-row chunks of the 64 RT2-row tile
            __syncthreads();                // the M buffers / the previous chunk are free
#pragma unroll
            for (int t = 0; t < RT2; ++t) {
                const int rt = 16 * RT2 * w + 16 * t;  // this row tile's first row in the workgroup
                if (rt / 64 != ch) continue;
#pragma unroll
                for (int g = 0; g < G; ++g)
#pragma unroll
                    for (int j = 0; j < 4; ++j) Ts[(rt % 64 + 4 * h + j) * TP + 16 * g + r] = acc[t][g][j];
            }
            __syncthreads();
            for (int e = tid; e < 64 * (CT / 8); e += 256) {
                const int lr = e / (CT / 8), c8 = 8 * (e % (CT / 8));
                const int64_t orow = row0 + 64 * ch + lr;
                const int c = c0 + c8;
                if (orow >= rows || c >= LP) continue;
                const float4 v0 = *reinterpret_cast<const float4*>(Ts + lr * TP + c8);
                const float4 v1 = *reinterpret_cast<const float4*>(Ts + lr * TP + c8 + 4);
                if (Out) {
                    *reinterpret_cast<float4*>(Out + orow * LP + c) = v0;
                    *reinterpret_cast<float4*>(Out + orow * LP + c + 4) = v1;
                }
                if (hi) {
                    const float v[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
                    uint32_t ph[4], pl[4];
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const bf16_t h0 = f2bf(v[2 * q]), h1 = f2bf(v[2 * q + 1]);
                        ph[q] = (uint32_t)h0 | ((uint32_t)h1 << 16);
                        pl[q] = (uint32_t)f2bf(v[2 * q] - bf2f(h0)) | ((uint32_t)f2bf(v[2 * q + 1] - bf2f(h1)) << 16);
                    }
                    *reinterpret_cast<uint4*>(hi + orow * LP + c) = make_uint4(ph[0], ph[1], ph[2], ph[3]);
                    if (lo) *reinterpret_cast<uint4*>(lo + orow * LP + c) = make_uint4(pl[0], pl[1], pl[2], pl[3]);
                }
            }
        }
        return;
    }
    // column-major caller output: a lane holds 4 consecutive rows of one column -- one 16-B store
    // when Out and ldo allow it (4 lanes then write 64 contiguous bytes of the column)
    const bool vec = ((reinterpret_cast<uintptr_t>(Out) | (uintptr_t)(ldo * 4)) & 15) == 0;
#pragma unroll
    for (int t = 0; t < RT2; ++t)
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const int64_t orow = row0 + 16 * RT2 * w + 16 * t + 4 * h;
            const int c = c0 + 16 * g + r;
            if (c >= cols) continue;
            float* dst = Out + orow + (int64_t)c * ldo;
            if (vec && orow + 3 < rows) {
                *reinterpret_cast<f32x4*>(dst) = acc[t][g];
            } else {
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    if (orow + j < rows) dst[j] = acc[t][g][j];
            }
        }
}

// ------------------------------------------------------------------------------------------------
template <typename T>
__global__ void repair_kernel(const T* __restrict__ Q, int64_t rows, int l, int LP, const int* __restrict__ colflag,
                              const int* __restrict__ flag, uint64_t seed, int64_t row_off, int64_t rows_total,
                              int64_t norm_rows, int64_t valid_rows, T* __restrict__ Out) {
    if (*flag == 0) return;
    const double sc = 1.0 / sqrt((double)norm_rows);
    const int64_t total = rows * LP;
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = e / LP;
        const int c = (int)(e - i * LP);
        T v = Q[e];
        if (c < l && colflag[c])  // (rows past valid_rows: the zero padding of a sharded panel stays zero)
            v = i < valid_rows ? (T)(gauss_elem((uint64_t)(row_off + i + rows_total * (int64_t)c), seed) * sc) : (T)0;
        Out[e] = v;
    }
}

template <typename T>
__global__ void split_bf16_kernel(const T* __restrict__ P, int64_t count, bf16_t* __restrict__ hi,
                                  bf16_t* __restrict__ lo) {
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < count; e += (int64_t)gridDim.x * blockDim.x) {
        const float v = (float)P[e];
        const bf16_t bh = f2bf(v);
        hi[e] = bh;
        if (lo) lo[e] = f2bf(v - bf2f(bh));
    }
}

// Round x to `bits` significant bits (round half to even), e4m3: saturate at 448 and keep the
// subnormal quantum 2^-9.  Mirrored bit for bit by the oracle's Python front end.
__device__ __forceinline__ double round_sig(double x, int fp8) {
    if (x == 0.0 || !isfinite(x)) return x;
    int e;
    (void)frexp(x, &e);  // |x| = m 2^e, m in [0.5, 1)
    int ex = e - 1;      // floor(log2 |x|)
    int bits = fp8 ? 3 : 7;
    if (fp8 && ex < -6) ex = -6;
    const double qn = ldexp(1.0, ex - bits);
    double y = rint(x / qn) * qn;
    if (fp8) y = fmin(fmax(y, -448.0), 448.0);
    return y;
}

// One thread per PAIR of stream elements (e, e + 1) = rows (i, i + 1) of column c (n even, i even):
// the two share the Philox block, log and square root of gauss_elem -- the same operations, so the
// values are bit-identical to gauss_elem's (cos for the even element, sin for the odd one); an odd n
// falls back to one element per thread.  C4's 65536 x 256 Omega: half the Philox / log / sqrt work.
__device__ __forceinline__ void gauss_pair(uint64_t e, uint64_t seed, double& g0, double& g1) {
    uint32_t x[4];
    philox4x32_10(e >> 1, seed, x);
    const double two_m53 = 1.1102230246251565404e-16;
    const double u1 = ((double)(((uint64_t)(x[0] >> 5) << 26) | (x[1] >> 6)) + 0.5) * two_m53;
    const double u2 = ((double)(((uint64_t)(x[2] >> 5) << 26) | (x[3] >> 6)) + 0.5) * two_m53;
    const double rr = sqrt(-2.0 * log(u1));
    const double th = 6.283185307179586476925286766559 * u2;
    g0 = rr * cos(th);
    g1 = rr * sin(th);
}

__global__ void omega_lowp_kernel(bf16_t* __restrict__ panel, int64_t n, int l, int LP, uint64_t seed, int fp8,
                                  float* __restrict__ f) {
    if ((n & 1) == 0) {
        const int64_t total = (n >> 1) * LP;  // (row pair, column)
        for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total;
             e += (int64_t)gridDim.x * blockDim.x) {
            const int64_t i = 2 * (e / LP);
            const int c = (int)(e % LP);
            float v0 = 0.f, v1 = 0.f;
            if (c < l) {
                double g0, g1;
                gauss_pair((uint64_t)(i + n * (int64_t)c), seed, g0, g1);  // even stream index
                v0 = (float)round_sig(g0, fp8);
                v1 = (float)round_sig(g1, fp8);
                if (f) {
                    f[i + n * (int64_t)c] = v0;
                    f[i + 1 + n * (int64_t)c] = v1;
                }
            }
            panel[i * LP + c] = (bf16_t)(__float_as_uint(v0) >> 16);  // exact: <= 8 significant bits
            panel[(i + 1) * LP + c] = (bf16_t)(__float_as_uint(v1) >> 16);
        }
        return;
    }
    const int64_t total = n * LP;
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = e / LP;
        const int c = (int)(e - i * LP);
        float v = 0.f;
        if (c < l) {
            v = (float)round_sig(gauss_elem((uint64_t)(i + n * (int64_t)c), seed), fp8);
            if (f) f[i + n * (int64_t)c] = v;
        }
        panel[e] = (bf16_t)(__float_as_uint(v) >> 16);  // exact: v has <= 8 significant bits
    }
}

__global__ void omega_lowp_from_kernel(const float* __restrict__ om, int64_t ld, int64_t n, int l, int LP, int fp8,
                                       bf16_t* __restrict__ panel) {
    const int64_t total = n * LP;
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = e / LP;
        const int c = (int)(e - i * LP);
        const float v = (c < l) ? (float)round_sig((double)om[i + ld * c], fp8) : 0.f;
        panel[e] = (bf16_t)(__float_as_uint(v) >> 16);
    }
}

// bf16 values that are exactly e4m3 -> e4m3 codes, 4 per thread (exact: no rounding happens)
__global__ void bf16_to_fp8_kernel(const bf16_t* __restrict__ in, int64_t count4, uint32_t* __restrict__ out) {
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < count4; e += (int64_t)gridDim.x * blockDim.x) {
        const uint2 v = reinterpret_cast<const uint2*>(in)[e];
        const float f0 = __uint_as_float(v.x << 16), f1 = __uint_as_float(v.x & 0xFFFF0000u);
        const float f2 = __uint_as_float(v.y << 16), f3 = __uint_as_float(v.y & 0xFFFF0000u);
        int w = __builtin_amdgcn_cvt_pk_fp8_f32(f0, f1, 0, false);
        w = __builtin_amdgcn_cvt_pk_fp8_f32(f2, f3, w, true);
        out[e] = (uint32_t)w;
    }
}

template <typename T>
__global__ void convert_scale_kernel(const double* __restrict__ x, T* __restrict__ y, int n, double sc) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) y[i] = (T)(x[i] * sc);
}

// The small SVD's outputs for the fp32 final products in one launch: S (scaled), U_w and V_w in fp32
// and, for the split panel products, their bf16 piece images (split_mat_kernel's layout)
__global__ void finish_convert_kernel(const double* __restrict__ Sd, float* __restrict__ S, int l, double sc,
                                      const double* __restrict__ Uw, float* __restrict__ Uw32, bf16_t* __restrict__ Mu,
                                      const double* __restrict__ Vw, float* __restrict__ Vw32, bf16_t* __restrict__ Mv,
                                      int LP) {
    const int64_t L2 = (int64_t)LP * LP;
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < L2; e += (int64_t)gridDim.x * blockDim.x) {
        const int k = (int)(e / LP), c = (int)(e - (int64_t)k * LP);
        const int64_t t = (int64_t)c * LP + k;
        const float u = (float)Uw[e], v = (float)Vw[e];
        Uw32[e] = u;
        Vw32[e] = v;
        store_pieces(Mu, L2, t, u);
        store_pieces(Mv, L2, t, v);
        if (e < l) S[e] = (float)(Sd[e] * sc);
    }
}

inline int grid_1d(int64_t work) {
    int64_t g = (work + 255) / 256;
    return (int)(g > 8192 ? 8192 : (g < 1 ? 1 : g));
}

}  // namespace

GramPlan plan_gram_wide(int64_t rows, int LP, int cross) {
    GramPlan g;
    const int nb = (LP + 31) / 32;
    g.blocks = cross ? nb * nb : nb * (nb + 1) / 2;
    if (!cross && gram_sym_ok(LP)) {  // gram_sym_kernel: one workgroup per chunk, >= 64 rows each, <= 256 chunks
        // >= max(64, LP) rows per chunk: a chunk's slab (LP^2 / 2 doubles) must not outweigh its rows
        const int64_t rmin = LP > 64 ? LP : 64;
        int64_t chunks = (rows + rmin - 1) / rmin;
        const int64_t cap = LP == 512 ? 128 : 256;  // LP = 512: 8 workgroups per chunk, 1 MB of slab per chunk
        if (chunks > cap) chunks = cap;
        if (chunks < 1) chunks = 1;
        int64_t rpc = (rows + chunks - 1) / chunks;
        rpc = (rpc + 31) / 32 * 32;  // a multiple of every RS
        g.rows_per_chunk = rpc;
        g.chunks = (int)((rows + rpc - 1) / rpc);
        if (g.chunks < 1) g.chunks = 1;
        return g;
    }
    int64_t chunks = (4096 + g.blocks - 1) / g.blocks;
    const int64_t max_by_rows = (rows + 255) / 256;
    if (chunks > max_by_rows) chunks = max_by_rows;
    if (chunks > 512) chunks = 512;
    if (chunks < 1) chunks = 1;
    int64_t rpc = (rows + chunks - 1) / chunks;
    rpc = (rpc + 15) / 16 * 16;
    g.rows_per_chunk = rpc;
    g.chunks = (int)((rows + rpc - 1) / rpc);
    if (g.chunks < 1) g.chunks = 1;
    return g;
}

template <typename T>
hipError_t launch_gram_wide(const T* P, const T* P2, int64_t rows, int LP, const GramPlan& gp, double* slabs,
                            double* G, const int* pred, hipStream_t s) {
    const int waves = gp.blocks * gp.chunks;
    const int wgs = (waves + 3) / 4;
    if (P2)
        hipLaunchKernelGGL((gram_wide_kernel<T, true>), dim3(wgs), dim3(256), 0, s, P, P2, rows, LP, gp.blocks,
                           gp.chunks, gp.rows_per_chunk, slabs, pred);
    else if (gram_sym_ok(LP)) {
        if (LP == 64)
            hipLaunchKernelGGL((gram_sym_kernel<T, 64>), dim3(gp.chunks), dim3(512), 0, s, P, rows, gp.rows_per_chunk, gp.chunks,
                               slabs, pred);
        else if (LP == 128)
            hipLaunchKernelGGL((gram_sym_kernel<T, 128>), dim3(gp.chunks), dim3(512), 0, s, P, rows,
                               gp.rows_per_chunk, gp.chunks, slabs, pred);
        else if (LP == 256)
            hipLaunchKernelGGL((gram_sym_kernel<T, 256>), dim3((gp.chunks + 7) / 8 * 16), dim3(512), 0, s, P,
                               rows, gp.rows_per_chunk, gp.chunks, slabs, pred);
        else
            hipLaunchKernelGGL((gram_sym_kernel<T, 512>), dim3((gp.chunks + 7) / 8 * 64), dim3(512), 0, s, P,
                               rows, gp.rows_per_chunk, gp.chunks, slabs, pred);
    } else
        hipLaunchKernelGGL((gram_wide_kernel<T, false>), dim3(wgs), dim3(256), 0, s, P, P, rows, LP, gp.blocks,
                           gp.chunks, gp.rows_per_chunk, slabs, pred);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return launch_gram_reduce(slabs, gp.blocks, gp.chunks, LP, P2 ? 1 : 0, G, pred, s);
}

bool gram_split_ok(int LP) { return LP == 128 || LP == 256 || LP == 512; }

hipError_t launch_gram_split_cross(const float* X, const float* Y, int64_t rows, int LP, const GramPlan& gp,
                                   double* slabs, double* G, hipStream_t s) {
    if ((LP != 256 && LP != 512) || gp.blocks != (LP / 32) * (LP / 32)) return hipErrorInvalidValue;
    // >= 256 rows per chunk, at most the plan's chunk count (its slabs), ~256 workgroups
    const int types = LP == 256 ? GramSplitX<256>::TYPES : GramSplitX<512>::TYPES;
    int64_t ch = (rows + 255) / 256;
    if (ch > 256 / types) ch = 256 / types;
    if (ch > gp.chunks) ch = gp.chunks;
    if (ch < 1) ch = 1;
    int64_t rpc = (rows + ch - 1) / ch;
    rpc = (rpc + 31) / 32 * 32;
    // each fp32 MFMA accumulator sums one chunk's rows; past kSplitCrossRows per chunk (n > 262144 at
    // LP = 256, n > 65536 at LP = 512) its error would grow with n -- the fp64 cross Gram instead
    if (rpc > kSplitCrossRows) return launch_gram_wide<float>(X, Y, rows, LP, gp, slabs, G, nullptr, s);
    const int nchunk = (int)((rows + rpc - 1) / rpc);
    const dim3 grid((unsigned)((nchunk + 7) / 8 * 8 * types));
    if (LP == 256)
        hipLaunchKernelGGL(gram_split_cross_kernel<256>, grid, dim3(GramSplitX<256>::THREADS), 2 * GramSplitX<256>::STEP,
                           s, X, Y, rows, rpc, nchunk, slabs);
    else
        hipLaunchKernelGGL(gram_split_cross_kernel<512>, grid, dim3(GramSplitX<512>::THREADS), 2 * GramSplitX<512>::STEP,
                           s, X, Y, rows, rpc, nchunk, slabs);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return launch_gram_reduce(slabs, gp.blocks, nchunk, LP, 1, G, nullptr, s);
}

hipError_t launch_gram_split(const float* P, int64_t rows, int LP, const GramPlan& gp, double* slabs, double* G,
                             hipStream_t s) {
    if (!gram_split_ok(LP)) return hipErrorInvalidValue;
    auto go = [&](auto lpc) {
        constexpr int L = decltype(lpc)::value;
        typedef GramSplit<L> GS;
        const int grid = GS::NH == 1 ? gp.chunks : (gp.chunks + 7) / 8 * 8 * GS::NH;
        if constexpr (L == 128) {  // two loader groups taking the steps in turn (round 4, 220 -> 180 us at C3)
            hipLaunchKernelGGL((gram_split_kernel<L, 1, 2>), dim3(grid), dim3(GS::THREADS), GS::NBUF * GS::STEP, s, P,
                               rows, gp.rows_per_chunk, gp.chunks, slabs);
            return;
        }
        hipLaunchKernelGGL(gram_split_kernel<L>, dim3(grid), dim3(GS::THREADS), GS::NBUF * GS::STEP, s, P, rows,
                           gp.rows_per_chunk, gp.chunks, slabs);
    };
    if (LP == 128) go(std::integral_constant<int, 128>{});
    else if (LP == 256) go(std::integral_constant<int, 256>{});
    int nchunk = gp.chunks;
    if (LP == 512) {
        // one round of 5-workgroup chunks on the 256 CUs (51 x 5 = 255), >= 512 rows each, within the
        // plan's slab count (the fp32 accumulators then run over up to ~2600 rows, as C3's 4096 do)
        int64_t ch = (rows + 511) / 512;
        if (ch > 51) ch = 51;
        if (ch > gp.chunks) ch = gp.chunks;
        if (ch < 1) ch = 1;
        int64_t rpc = (rows + ch - 1) / ch;
        rpc = rpc < 32 ? 32 : (rpc + 31) / 32 * 32;  // (a rank's shard may hold no rows: one empty chunk)
        nchunk = rows > 0 ? (int)((rows + rpc - 1) / rpc) : 1;
        hipLaunchKernelGGL(gram_split4_kernel, dim3((nchunk + 7) / 8 * 8 * GramSplit4::TYPES),
                           dim3(GramSplit4::THREADS), GramSplit4::LDS, s, P, rows, rpc, nchunk, slabs);
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return launch_gram_reduce(slabs, gp.blocks, nchunk, LP, 0, G, nullptr, s);
}

int chol_variant = 1;

hipError_t launch_chol_wide(const double* G, int l, int LP, double tol, double* R, double* Rinv, float* Rinv32,
                            int* colflag, int* flag, double* work, const int* pred, hipStream_t s, double ill_tol,
                            int* ill, const double* d0src, bf16_t* Mt, int ldg) {
    if (LP % 16 || LP > 512) return hipErrorInvalidValue;
    if (ldg == 0) ldg = LP;
    // LP = 256: chol_wide_kernel (its wave-0 look-ahead overlaps the diagonal factor with the other waves'
    // updates; the register-resident kernel spills there, 174 vs 161 us measured); LP <= 128: chol_reg_kernel
    // (LP = 128: 63 vs 71 us, LP = 64: 31 vs 37 us, tools/wide_lab chol)
    // R^-1 by the triangular inverse in the same launch after the register-resident factor (round 6 tried
    // eliminating [G | I] in the factor's own sweep instead: 256 VGPRs + 112 B/lane scratch at NP = 8,
    // +6 us per launch measured; DESIGN.md §9c dead end 17)
    const int fuse = (chol_variant >= 1 && (LP == 128 || LP == 64)) ? 1 : 0;
    if (chol_variant >= 1 && LP == 128)
        hipLaunchKernelGGL(chol_reg_kernel<8>, dim3(1), dim3(64 * kCholRegWaves),
                           std::max(CholReg<8>::lds_bytes, fuse ? CholRegInv<8>::lds_bytes : 0), s, G, l, tol, R, Rinv,
                           colflag, flag, pred, ill_tol, ill, d0src, ldg, Rinv32, Mt, fuse);
    else if (chol_variant >= 1 && LP == 64)
        hipLaunchKernelGGL(chol_reg_kernel<4>, dim3(1), dim3(64 * kCholRegWaves),
                           std::max(CholReg<4>::lds_bytes, fuse ? CholRegInv<4>::lds_bytes : 0), s, G, l, tol, R, Rinv,
                           colflag, flag, pred, ill_tol, ill, d0src, ldg, Rinv32, Mt, fuse);
#ifdef RSVD_LAB
    else if (chol_variant == 2 && LP == 256)  // the lab's register-resident LP = 256 factor (it spills)
        hipLaunchKernelGGL(chol_reg_kernel<16>, dim3(1), dim3(64 * kCholRegWaves), CholReg<16>::lds_bytes, s, G, l,
                           tol, R, Rinv, colflag, flag, pred, ill_tol, ill, d0src, ldg, Rinv32, Mt, 0);
#endif
    else
        hipLaunchKernelGGL((chol_wide_kernel<kCholThreads, kCholBatch>), dim3(1), dim3(kCholThreads), chol_lds_bytes(LP),
                           s, G, l, LP, tol, work, R, Rinv, colflag, flag, pred, ill_tol, ill, d0src, ldg);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess || fuse) return e;
    hipLaunchKernelGGL(rinv_wide_kernel, dim3(LP / 16), dim3(256), 0, s, LP, R, Rinv, Rinv32, pred, Mt);
    return hipGetLastError();
}

// ---- two-level factor, LP = 2 B (launch_chol_wide_2level) ----------------------------------------
// The levels read G11 and G22 in place (row pitch ldg); d0b = diag(G22), written by the S product's
// diagonal tiles: the breakdown / ill tests of the second level judge S's pivots against G's own
// diagonal, as the one-level factor does (d0src: that diagonal when this factor is itself a level).

// R / Rinv (2B x 2B row-major) from the level blocks; Rinv32 the fp32 copy; ill = ill1 | ill2.
// Run by extra workgroups of the Rinv12 GEMM (gemmsq_f64_kernel with a Chol2Asm job, round 5: one
// launch fewer per two-level block); the GEMM's own workgroups write Rinv12's fp32 copy and pieces.
struct Chol2Asm {
    const double* R11;
    const double* Ri11;
    const double* R22;
    const double* Ri22;
    int B;  // 0: no assembly job
    double* R;
    double* Rinv;
    float* Rinv32;
    const int* ill2;
    int* ill;
    bf16_t* Mt;
};
// element (row i of 2B, column c of B): columns c (and c + B for i >= B) of row i
__device__ __forceinline__ void chol2_assemble_elem(const Chol2Asm& a, int i, int c) {
    const int B = a.B;
    const int64_t o = (int64_t)i * 2 * B, L2 = (int64_t)4 * B * B;
    if (i < B) {
        a.R[o + c] = a.R11[i * B + c];
        a.Rinv[o + c] = a.Ri11[i * B + c];
        if (a.Rinv32) a.Rinv32[o + c] = (float)a.Ri11[i * B + c];
        if (a.Mt) store_pieces(a.Mt, L2, (int64_t)c * 2 * B + i, (float)a.Ri11[i * B + c]);
    } else {
        const int i2 = i - B;
        a.R[o + c] = 0.0;
        a.Rinv[o + c] = 0.0;
        a.R[o + B + c] = a.R22[i2 * B + c];
        a.Rinv[o + B + c] = a.Ri22[i2 * B + c];
        if (a.Rinv32) {
            a.Rinv32[o + c] = 0.f;
            a.Rinv32[o + B + c] = (float)a.Ri22[i2 * B + c];
        }
        if (a.Mt) {
            store_pieces(a.Mt, L2, (int64_t)c * 2 * B + i, 0.0f);
            store_pieces(a.Mt, L2, (int64_t)(B + c) * 2 * B + i, (float)a.Ri22[i2 * B + c]);
        }
    }
    if (a.ill && i == 0 && c == 0 && *a.ill2) *a.ill = 1;
}

// row-major C (N x N, ldc) = alpha op(A) B + beta C, N = K in {128, 256} (op(A) = A or A^T; A, B
// row-major with ld lda / ldb): one wave per 16 x 16 output tile ((N / 16)^2 workgroups -- the
// 64 x 64-tile general GEMM kept 16 CUs busy, 56 us per 256^3 product), four independent fp64 MFMA
// chains over K, every operand an L2 hit.
// K is split over the workgroup's four waves (a quarter each, four chains per wave: the one-wave form
// was a 16-deep dependent MFMA chain per accumulator behind L2 loads, 24 us per 256^3 product); the
// wave partials are summed through LDS in wave order.
constexpr int kGemmSqWaves = 4;
// zrow (nullable): output rows i with zrow[i] != 0 are written as zeros (R12's broken-down rows).
// Cin (nullable): the beta term's C when it is not the output (ld ldcin); d0out (nullable): the
// diagonal-tile workgroups also write d0out[i] = d0in ? d0in[i] : Cin[i][i] (a level's pivot reference)
struct GemmSqJob {
    int N = 0, ta = 0;  // N = 0: no job
    double alpha = 1.0;
    const double* A = nullptr;
    int lda = 0;
    const double* B = nullptr;
    int ldb = 0;
    double beta = 0.0;
    double* C = nullptr;
    int ldc = 0;
    const int* zrow = nullptr;
    const double* Cin = nullptr;
    int ldcin = 0;
    double* d0out = nullptr;
    const double* d0in = nullptr;
};
// One launch runs up to two independent products (j1.N = 0: one) and, on extra workgroups, a
// two-level factor's assembly job (round 6: the two-level factor's T = Ri11 R12 rides the S product's
// launch -- one dependent launch fewer per two-level block).
__global__ __launch_bounds__(64 * kGemmSqWaves) void gemmsq_f64_kernel(GemmSqJob j0, GemmSqJob j1, Chol2Asm aj) {
    __shared__ double part[kGemmSqWaves - 1][4][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, r = lane & 15, h = lane >> 4;
    const int nb0 = (j0.N / 16) * (j0.N / 16), nb1 = (j1.N / 16) * (j1.N / 16);
    int b = (int)blockIdx.x;
    if (b >= nb0 + nb1) {  // an assembly workgroup (the Rinv12 product's launch)
        const int e = (b - nb0 - nb1) * 64 * kGemmSqWaves + (int)threadIdx.x;
        if (aj.B && e < 2 * aj.B * aj.B) chol2_assemble_elem(aj, e / aj.B, e % aj.B);
        return;
    }
    const bool second = b >= nb0;
    const GemmSqJob& J = second ? j1 : j0;
    if (second) b -= nb0;
    const int N = J.N, nt = N / 16;
    const int i0 = 16 * (b / nt), j0c = 16 * (b % nt);
    const int kq = N / kGemmSqWaves;  // N % 64 == 0
    const double* __restrict__ A = J.A;
    const double* __restrict__ B = J.B;
    const int lda = J.lda, ldb = J.ldb, ta = J.ta;
    f64x4 acc[4] = {MD::zero(), MD::zero(), MD::zero(), MD::zero()};
#pragma unroll 2
    for (int k0 = w * kq; k0 < (w + 1) * kq; k0 += 16) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int k = k0 + 4 * u + h;
            const double a = ta ? A[(int64_t)k * lda + i0 + r] : A[(int64_t)(i0 + r) * lda + k];
            acc[u] = MD::mma(a, B[(int64_t)k * ldb + j0c + r], acc[u]);
        }
    }
    double v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = (acc[0][j] + acc[1][j]) + (acc[2][j] + acc[3][j]);
    if (w > 0) {
#pragma unroll
        for (int j = 0; j < 4; ++j) part[w - 1][j][lane] = v[j];
    }
    __syncthreads();
    if (w != 0) return;
    const int ldc = J.ldc;
#pragma unroll
    for (int j = 0; j < 4; ++j) {  // f64 D: col = r, row = h + 4 j
#pragma unroll
        for (int q = 0; q < kGemmSqWaves - 1; ++q) v[j] += part[q][j][lane];
        const int ii = i0 + MD::row(h, j), jj = j0c + r;
        double* c = J.C + (int64_t)ii * ldc + jj;
        const double o = J.alpha * v[j];
        const double cin = J.beta == 0.0 ? 0.0 : (J.Cin ? J.Cin[(int64_t)ii * J.ldcin + jj] : *c);
        const double out = (J.zrow && J.zrow[ii]) ? 0.0 : (J.beta == 0.0 ? o : o + J.beta * cin);
        *c = out;
        if (J.d0out && ii == jj) J.d0out[ii] = J.d0in ? J.d0in[ii] : J.Cin[(int64_t)ii * J.ldcin + ii];
        if (!second && aj.B) {  // (the Rinv12 product: C = Rinv + B, ldc = 2 B) its fp32 copy and pieces
            if (aj.Rinv32) aj.Rinv32[(int64_t)ii * ldc + aj.B + jj] = (float)out;
            if (aj.Mt) store_pieces(aj.Mt, (int64_t)4 * aj.B * aj.B, (int64_t)(aj.B + jj) * 2 * aj.B + ii, (float)out);
        }
    }
}

static GemmSqJob sq_job(int N, int ta, double alpha, const double* A, int lda, const double* B, int ldb, double beta,
                        double* C, int ldc, const int* zrow = nullptr, const double* Cin = nullptr, int ldcin = 0,
                        double* d0out = nullptr, const double* d0in = nullptr) {
    GemmSqJob j;
    j.N = N, j.ta = ta, j.alpha = alpha, j.A = A, j.lda = lda, j.B = B, j.ldb = ldb, j.beta = beta, j.C = C, j.ldc = ldc;
    j.zrow = zrow, j.Cin = Cin, j.ldcin = ldcin, j.d0out = d0out, j.d0in = d0in;
    return j;
}

static hipError_t gemm_sq2(const GemmSqJob& j0, const GemmSqJob& j1, hipStream_t s, const Chol2Asm* aj = nullptr) {
    if (j0.N % (16 * kGemmSqWaves) || j1.N % (16 * kGemmSqWaves)) return hipErrorInvalidValue;
    Chol2Asm job{};
    int extra = 0;
    if (aj) {
        job = *aj;
        extra = (2 * job.B * job.B + 64 * kGemmSqWaves - 1) / (64 * kGemmSqWaves);
    }
    const int nb = (j0.N / 16) * (j0.N / 16) + (j1.N / 16) * (j1.N / 16) + extra;
    hipLaunchKernelGGL(gemmsq_f64_kernel, dim3(nb), dim3(64 * kGemmSqWaves), 0, s, j0, j1, job);
    return hipGetLastError();
}

static hipError_t gemm_sq(int N, int ta, double alpha, const double* A, int lda, const double* B, int ldb, double beta,
                          double* C, int ldc, hipStream_t s, const int* zrow = nullptr, const double* Cin = nullptr,
                          int ldcin = 0, double* d0out = nullptr, const double* d0in = nullptr,
                          const Chol2Asm* aj = nullptr) {
    return gemm_sq2(sq_job(N, ta, alpha, A, lda, B, ldb, beta, C, ldc, zrow, Cin, ldcin, d0out, d0in), GemmSqJob{}, s,
                    aj);
}

size_t chol_2level_scratch_doubles(int LP, int depth) {
    const size_t B = LP / 2;
    const size_t own = 7 * B * B + B + 64;  // Ga R11 Ri11 Sb R22 Ri22 T, d0b, ill2 (+ alignment)
    return own + (depth > 0 && B >= 256 ? chol_2level_scratch_doubles((int)B, depth - 1) : 0);
}

// One level of the factor: the two-level form (recursing `depth` more times) when LP >= 256 and more
// than half the columns are valid, else the one-workgroup kernel.
static hipError_t chol_level(const double* G, int ldg, int l, int LP, double tol, double* R, double* Rinv,
                             int* colflag, int* flag, double* work, double* scratch, hipStream_t s, double ill_tol,
                             int* ill, const double* d0src, int depth) {
    if (depth >= 0 && LP >= 256 && l > LP / 2)
        return launch_chol_wide_2level(G, l, LP, tol, R, Rinv, nullptr, colflag, flag, work, scratch, s, ill_tol, ill,
                                       d0src, depth, nullptr, ldg);
    return launch_chol_wide(G, l, LP, tol, R, Rinv, nullptr, colflag, flag, work, nullptr, s, ill_tol, ill, d0src,
                            nullptr, ldg);
}

hipError_t launch_chol_wide_2level(const double* G, int l, int LP, double tol, double* R, double* Rinv,
                                   float* Rinv32, int* colflag, int* flag, double* work, double* scratch,
                                   hipStream_t s, double ill_tol, int* ill, const double* d0src, int depth,
                                   bf16_t* Mt, int ldg) {
    if ((LP != 256 && LP != 512) || l <= LP / 2 || l > LP) return hipErrorInvalidValue;
    if (ldg == 0) ldg = LP;
    const int B = LP / 2, B2 = B * B;
    double *Ga = scratch, *R11 = Ga + B2, *Ri11 = R11 + B2, *Sb = Ri11 + B2, *R22 = Sb + B2, *Ri22 = R22 + B2,
           *T = Ri22 + B2, *d0b = T + B2;
    int* ill2 = reinterpret_cast<int*>(d0b + B);
    double* inner = d0b + B + 64;  // the next level's scratch (depth > 0)
    const int sub = depth - 1;     // < 0: the levels below are one-workgroup factors
    (void)Ga;  // (round 5: the levels read G11 and G22 in place -- no copy launch)
    // level 1: R11, Ri11 = chol(G11) (columns 0 .. B - 1 of colflag), G11 read in place (pitch ldg)
    hipError_t e = chol_level(G, ldg, B, B, tol, R11, Ri11, colflag, flag, work, inner, s, ill_tol, ill, d0src, sub);
    if (e != hipSuccess) return e;
    // R12 = Ri11^T G12 -> R[:B, B:] (ld LP); the rows whose first-level pivot broke down are zero, as
    // the one-level factor's strips are (written so by the product's epilogue)
    if ((e = gemm_sq(B, 1, 1.0, Ri11, B, G + B, ldg, 0.0, R + B, LP, s, colflag)) != hipSuccess) return e;
    // S = G22 - R12^T R12 into Sb (the beta term read from G22 in place), and d0b = diag(G22) (or the
    // caller's d0src[B ..]) from the diagonal tiles; in the same launch T = Ri11 R12 (independent of S)
    if ((e = gemm_sq2(sq_job(B, 1, -1.0, R + B, LP, R + B, LP, 1.0, Sb, B, nullptr, G + (int64_t)B * ldg + B, ldg, d0b,
                             d0src ? d0src + B : nullptr),
                      sq_job(B, 0, 1.0, Ri11, B, R + B, LP, 0.0, T, B), s)) != hipSuccess)
        return e;
    // level 2 on the l - B valid columns of S, tested against diag(G22) (or the caller's d0src)
    e = chol_level(Sb, B, l - B, B, tol, R22, Ri22, colflag + B, flag, work, inner, s, ill_tol, ill ? ill2 : nullptr,
                   d0b, sub);
    if (e != hipSuccess) return e;
    // Rinv12 = -(Ri11 R12) Ri22 -> Rinv[:B, B:], with the blocks' assembly into R / Rinv (+ Rinv32,
    // pieces, ill) on extra workgroups
    const Chol2Asm job{R11, Ri11, R22, Ri22, B, R, Rinv, Rinv32, ill2, ill, Mt};
    return gemm_sq(B, 0, -1.0, T, B, Ri22, B, 0.0, Rinv + B, LP, s, nullptr, nullptr, 0, nullptr, nullptr, &job);
}


// panel_split_kernel shape: 2 row tiles x 128 columns (4 x 128 runs at one wave per SIMD and loses
// the gain of its halved LDS reads, 4 x 64 ties with 2 x 128 in the bench: round 3)
template <typename T>
hipError_t launch_panel_gemm(const T* In, int64_t rows, int LP, const T* Mm, int upper, T* Out, int64_t ldo,
                             int cols, bf16_t* hi, bf16_t* lo, const int* pred, hipStream_t s, bf16_t* msplit,
                             bool msplit_ready) {
    if (!Mm || LP % 16 || (!Out && (ldo != 0 || !hi))) return hipErrorInvalidValue;
    const int64_t rb = (rows + 63) / 64;
    if constexpr (sizeof(T) == 4) {
        if (msplit && LP % 32 == 0 && LP >= 128) {  // the bf16-split product (panel_split_kernel)
            const int64_t L2 = (int64_t)LP * LP;
            if (!msplit_ready)  // (else the factor that wrote M's fp32 copy wrote its pieces too)
                hipLaunchKernelGGL(split_mat_kernel, dim3((unsigned)std::min<int64_t>((L2 + 255) / 256, 1024)), dim3(256),
                                   0, s, reinterpret_cast<const float*>(Mm), LP, msplit);
#define PSPLIT(RT2, CT, PD)                                                                                    \
    {                                                                                                          \
        const int ncb = (LP + CT - 1) / CT;                                                                    \
        const int64_t rb2 = (rows + 64 * RT2 - 1) / (64 * RT2);                                                \
        hipLaunchKernelGGL((panel_split_kernel<RT2, CT, PD>), dim3((unsigned)(rb2 * ncb)), dim3(256),          \
                           (size_t)2 * 3 * CT * 64, s, reinterpret_cast<const float*>(In), rows, LP, msplit,   \
                           upper, reinterpret_cast<float*>(Out), ldo, cols, hi, lo, ncb, pred);                \
        return hipGetLastError();                                                                              \
    }
            // In prefetch ring depth (RSVD_PANEL_PD overrides): 4 at LP = 512 (16 k-steps: C5 18.38 ->
            // 18.19 ms, gpurun_out r6k), 2 (one step ahead) below, where 3 / 4 measured no gain
            static const int pd_env = [] {
                const char* e = std::getenv("RSVD_PANEL_PD");
                return e ? std::atoi(e) : 0;
            }();
            const int pd = pd_env ? pd_env : (LP >= 512 ? 4 : 2);
            if (pd == 3) PSPLIT(2, 128, 3)
            if (pd == 4) PSPLIT(2, 128, 4)
            PSPLIT(2, 128, 2)
#undef PSPLIT
        }
    }
#define GO(CT)                                                                                                  \
    {                                                                                                           \
        const int ncb = (LP + CT - 1) / CT;                                                                     \
        constexpr int KC = 16 * PG<T>::VW;                                                                      \
        const size_t lds = std::max<size_t>((size_t)KC * (CT + PG<T>::PAD), (size_t)CT * 65) * sizeof(T);       \
        hipLaunchKernelGGL((panel_gemm_kernel<T, CT>), dim3((unsigned)(rb * ncb)), dim3(256), lds, s, In, rows, \
                           LP, Mm, upper, Out, ldo, cols, hi, lo, ncb, pred);                                   \
        return hipGetLastError();                                                                               \
    }
    if (LP <= 16) GO(16)
    if (LP <= 32) GO(32)
    if (LP <= 64) GO(64)
    GO(128)
#undef GO
}

template <typename T>
hipError_t launch_repair_panel(const T* Q, int64_t rows, int l, int LP, const int* colflag, const int* flag,
                               uint64_t seed, int64_t row_off, int64_t rows_total, int64_t norm_rows, T* Out,
                               hipStream_t s, int64_t valid_rows) {
    hipLaunchKernelGGL((repair_kernel<T>), dim3(grid_1d(rows * LP)), dim3(256), 0, s, Q, rows, l, LP, colflag, flag,
                       seed, row_off, rows_total, norm_rows, valid_rows < 0 ? rows : valid_rows, Out);
    return hipGetLastError();
}

template <typename T>
hipError_t launch_split_bf16(const T* P, int64_t rows, int LP, bf16_t* hi, bf16_t* lo, hipStream_t s) {
    hipLaunchKernelGGL((split_bf16_kernel<T>), dim3(grid_1d(rows * LP)), dim3(256), 0, s, P, rows * LP, hi, lo);
    return hipGetLastError();
}

hipError_t launch_omega_lowp(bf16_t* panel, int64_t n, int l, int LP, uint64_t seed, int round_fp8, float* f,
                             hipStream_t s) {
    hipLaunchKernelGGL(omega_lowp_kernel, dim3(grid_1d(n * LP)), dim3(256), 0, s, panel, n, l, LP, seed, round_fp8,
                       f);
    return hipGetLastError();
}

hipError_t launch_bf16_to_fp8(const bf16_t* in, int64_t count, fp8_t* out, hipStream_t s) {
    if (count % 4) return hipErrorInvalidValue;
    hipLaunchKernelGGL(bf16_to_fp8_kernel, dim3(grid_1d(count / 4)), dim3(256), 0, s, in, count / 4,
                       reinterpret_cast<uint32_t*>(out));
    return hipGetLastError();
}

hipError_t launch_omega_lowp_from(const float* om, int64_t ld, int64_t n, int l, int LP, int round_fp8,
                                  bf16_t* panel, hipStream_t s) {
    hipLaunchKernelGGL(omega_lowp_from_kernel, dim3(grid_1d(n * LP)), dim3(256), 0, s, om, ld, n, l, LP, round_fp8,
                       panel);
    return hipGetLastError();
}

hipError_t launch_finish_convert(const double* Sd, float* S, int l, double sc, const double* Uw, float* Uw32, bf16_t* Mu,
                                 const double* Vw, float* Vw32, bf16_t* Mv, int LP, hipStream_t s) {
    const int64_t L2 = (int64_t)LP * LP;
    hipLaunchKernelGGL(finish_convert_kernel, dim3((unsigned)std::min<int64_t>((L2 + 255) / 256, 1024)), dim3(256), 0, s,
                       Sd, S, l, sc, Uw, Uw32, Mu, Vw, Vw32, Mv, LP);
    return hipGetLastError();
}

template <typename T>
hipError_t launch_convert_scale(const double* x, T* y, int n, double sc, hipStream_t s) {
    hipLaunchKernelGGL((convert_scale_kernel<T>), dim3((n + 255) / 256), dim3(256), 0, s, x, y, n, sc);
    return hipGetLastError();
}

#define RSVD_INST(T)                                                                                               \
    template hipError_t launch_convert_scale<T>(const double*, T*, int, double, hipStream_t);                                             \
    template hipError_t launch_gram_wide<T>(const T*, const T*, int64_t, int, const GramPlan&, double*, double*,    \
                                            const int*, hipStream_t);                                               \
    template hipError_t launch_panel_gemm<T>(const T*, int64_t, int, const T*, int, T*, int64_t, int, bf16_t*,      \
                                             bf16_t*, const int*, hipStream_t, bf16_t*, bool);                      \
    template hipError_t launch_repair_panel<T>(const T*, int64_t, int, int, const int*, const int*, uint64_t,       \
                                               int64_t, int64_t, int64_t, T*, hipStream_t, int64_t);                \
    template hipError_t launch_split_bf16<T>(const T*, int64_t, int, bf16_t*, bf16_t*, hipStream_t);
RSVD_INST(float)
RSVD_INST(double)
#undef RSVD_INST

}  // namespace rsvd

#ifdef RSVD_CHOL_PROF
#include <vector>
namespace rsvd {
namespace {
// one wave factors a 16 x 16 SPD tile `reps` times (the diagonal factor alone, no barriers): cycles per factor
template <int V>
__global__ __launch_bounds__(64) void diag_bench_kernel(const double* __restrict__ T, int reps, double* R, double* Rinv,
                                                        int* colflag, int* flag, long long* out) {
    __shared__ double Di[256], d0[16], Ts[256];
    __shared__ int bad[16];
    const int lane = threadIdx.x, r = lane & 15;
    if (lane < 16) d0[lane] = T[lane * 16 + lane];
    for (int e = lane; e < 256; e += 64) Ts[e] = T[e];
    __syncthreads();
    double col0[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) col0[i] = T[i * 16 + r];
    double sink = 0.0;
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < reps; ++it) {
        double col[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) col[i] = col0[i] + sink * 1e-300;
        if constexpr (V == 0) chol_diag16_fast(col, 0, 16, 16, 1e-13, d0, Di, bad, R, Rinv, colflag, flag, lane);
        else if constexpr (V == 1) chol_diag16_dpp(col, 0, 16, 16, 1e-13, d0, Di, bad, R, Rinv, colflag, flag, lane);
        else chol_diag16_v2(col, 0, 16, 16, 1e-13, d0, Di, bad, R, Rinv, colflag, flag, lane, Ts);
        sink += col[15];
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) out[V] = (t1 - t0) / reps + (sink == 12345.0 ? 1 : 0);
}
}  // namespace
void chol_diag_bench() {
    std::vector<double> h(256);
    for (int i = 0; i < 16; ++i)
        for (int j = 0; j < 16; ++j) h[i * 16 + j] = (i == j ? 20.0 : 0.0) + 1.0 / (1 + i + j);
    double *T, *R, *Ri;
    int *cf, *fl;
    long long* out;
    (void)hipMalloc(&T, 256 * 8);
    (void)hipMalloc(&R, 256 * 8);
    (void)hipMalloc(&Ri, 256 * 8);
    (void)hipMalloc(&cf, 64);
    (void)hipMalloc(&fl, 64);
    (void)hipMalloc(&out, 24);
    (void)hipMemcpy(T, h.data(), 256 * 8, hipMemcpyHostToDevice);
    long long o[3];
    std::vector<double> r1(256), r2(256), i1(256), i2(256);
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(diag_bench_kernel<0>, dim3(1), dim3(64), 0, 0, T, 256, R, Ri, cf, fl, out);
        hipLaunchKernelGGL(diag_bench_kernel<1>, dim3(1), dim3(64), 0, 0, T, 256, R, Ri, cf, fl, out);
        (void)hipMemcpy(r1.data(), R, 256 * 8, hipMemcpyDeviceToHost);
        (void)hipMemcpy(i1.data(), Ri, 256 * 8, hipMemcpyDeviceToHost);
        hipLaunchKernelGGL(diag_bench_kernel<2>, dim3(1), dim3(64), 0, 0, T, 256, R, Ri, cf, fl, out);
        (void)hipMemcpy(r2.data(), R, 256 * 8, hipMemcpyDeviceToHost);
        (void)hipMemcpy(i2.data(), Ri, 256 * 8, hipMemcpyDeviceToHost);
        (void)hipMemcpy(o, out, 24, hipMemcpyDeviceToHost);
    }
    printf("  16x16 diagonal factor, one wave: readlane form %lld cycles, DPP form %lld cycles, v2 %lld cycles "
           "(v2 bit-identical to DPP: R %d, R^-1 %d)\n", o[0], o[1], o[2], (int)(r1 == r2), (int)(i1 == i2));
    (void)hipFree(T); (void)hipFree(R); (void)hipFree(Ri); (void)hipFree(cf); (void)hipFree(fl); (void)hipFree(out);
}
void chol_prof_dump(int LP) {
    long long t[256];
    (void)hipMemcpyFromSymbol(t, HIP_SYMBOL(g_chol_prof), sizeof(t));
    const int np = LP / 16;
    double strip = 0, trail = 0;
    const double us = 0.01;  // wall_clock64 runs at 100 MHz
    long long prev = t[0];
    for (int p = 0; p < np; ++p) {
        strip += (t[1 + 2 * p] - prev) * us;
        trail += (t[2 + 2 * p] - t[1 + 2 * p]) * us;
        prev = t[2 + 2 * p];
    }
    if (chol_variant == 0) {
        printf("  LP=%d factor phases (us): init+diag0 %.1f strip %.1f trailing+diag %.1f\n", LP, (t[0] - t[97]) * us,
               strip, trail);
        return;
    }
    double A = 0, B = 0, Cc = 0;
    prev = t[200];
    for (int p = 0; p < np && p < 32; ++p) {
        A += (t[1 + 3 * p] - prev) * us;
        if (p == np - 1) break;
        B += (t[2 + 3 * p] - t[1 + 3 * p]) * us;
        Cc += (t[3 + 3 * p] - t[2 + 3 * p]) * us;
        prev = t[3 + 3 * p];
    }
    printf("  LP=%d reg phases (us, wave 0): init %.1f  diag+wait %.1f  strip %.1f  update %.1f\n", LP,
           (t[200] - t[97]) * us, A, B, Cc);
    if (np <= 8) {
        const long long f = t[1 + 3 * (np - 1)];
        printf("  LP=%d fused R^-1 (us after the factor): staged %.2f, columns", LP, (t[210] - f) * us);
        for (int j = 0; j < np; ++j) printf(" %.2f", (t[211 + j] - f) * us);
        printf("\n");
    }
}
}  // namespace rsvd
#endif
