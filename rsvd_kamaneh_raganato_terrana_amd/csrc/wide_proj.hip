// wide_proj.hip -- bf16 / fp8 A projections on the bf16 MFMA (gfx950), sketch width LP <= 512.
//
//   NN:  Y = A * S     (A m x n column-major, S n x LP panel)    src/rSVD.cpp:59,66
//   TN:  Z = A^T * S   (S m x LP panel, Z n x LP)                 src/rSVD.cpp:63,89 (B^T = A^T Q)
//
// The skinny operand S arrives as bf16 panels: "hi" (and "lo" with S ~= hi + lo) -- two MFMAs
// per product keep 16 significant bits of S, which is what the 1e-4 parity bar needs (SURVEY.md
// §7 "Hard parts"); the Gaussian sketch is itself bf16 (or e4m3) so A*Omega is one pass.  A is
// read from HBM exactly once per launch; fp8 A is widened to bf16 on the way (exact).
//
// v_mfma_f32_16x16x32_bf16 operand maps (cdna_hip_programming.md §3): lane l holds
// A[row l&15][k = 8(l>>4) + j] and B[k = 8(l>>4) + j][col l&15], j = 0..7; D: col = l&15,
// row = 4(l>>4) + reg.  The contraction index k is the A column index for NN (strided in HBM)
// and the A row index for TN (contiguous):
//  * S (both) and A (NN) are staged per 32-deep k-step into LDS as row-major [k][...] tiles
//    (16-B padded rows, 2-way bank conflicts at most) and read with ds_read_b64_tr_b16, which
//    hands each lane 4 consecutive k of one column -- the fragment shape, no shuffles.
//  * A (TN) goes straight from HBM to the fragment: 8 consecutive rows of one A column.
// Staging is register-prefetched one k-step ahead (loads for step s+1 in flight while step s
// computes).  Workgroup = 4 waves as WR (rows) x WC (columns); a wave owns 64 output rows x
// 16 G columns (acc = 4 x G MFMA tiles).  K is split over workgroups into fp32 slabs
// (launch_sum_slabs) when the row blocks alone cannot fill the chip; the XCD-aware remap puts
// the row blocks of one K chunk on one XCD so their shared S chunk is an L2 hit.
#include <type_traits>

#include <cstdlib>

#include "common.hpp"
#include "kernels.hpp"
#include "wide.hpp"

#include <utility>

namespace rsvd {

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_t;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(8))) short s16x8;

template <int LP> struct WCfg;
template <> struct WCfg<16> { static constexpr int WR = 4, WC = 1, G = 1; };
template <> struct WCfg<32> { static constexpr int WR = 4, WC = 1, G = 2; };
template <> struct WCfg<64> { static constexpr int WR = 4, WC = 1, G = 4; };
template <> struct WCfg<128> { static constexpr int WR = 4, WC = 1, G = 8; };
template <> struct WCfg<256> { static constexpr int WR = 2, WC = 2, G = 8; };
template <> struct WCfg<512> { static constexpr int WR = 1, WC = 4, G = 8; };

constexpr int RT = 4;   // 16-row MFMA tiles per wave
constexpr int KS = 32;  // k per step (one MFMA deep)

__device__ __forceinline__ s16x4 tr_read(const bf16_t* p) {
    typedef s16x4 __attribute__((address_space(3))) * lds_ptr;
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_ptr)(const_cast<bf16_t*>(p)));
}
__device__ __forceinline__ bf16x8_t join(s16x4 a, s16x4 b) {
    return __builtin_bit_cast(bf16x8_t, __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7));
}
// 4 e4m3 bytes -> 4 bf16 (exact: e4m3 has 4 significant bits)
__device__ __forceinline__ uint2 fp8x4_to_bf16x4(uint32_t v) {
    const bf16x2_t a = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(v, 1.0f, false);
    const bf16x2_t b = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(v, 1.0f, true);
    return make_uint2(__builtin_bit_cast(uint32_t, a), __builtin_bit_cast(uint32_t, b));
}

template <bool FP8, bool NN, int LP, bool SPLIT>
constexpr size_t wproj_lds() {
    constexpr int WI = WCfg<LP>::WR * 64;
    return (size_t)(SPLIT ? 2 : 1) * KS * (LP + 8) * 2 + (NN ? (size_t)KS * (WI + 8) * 2 : 0);
}

template <bool FP8, bool NN, int LP, bool SPLIT>
__global__ __launch_bounds__(256) void wproj_kernel(const void* __restrict__ Av, int64_t lda, int64_t rows_out,
                                                    int64_t K, const bf16_t* __restrict__ Shi,
                                                    const bf16_t* __restrict__ Slo, float* __restrict__ out,
                                                    int64_t slab_stride, int64_t kchunk, int nrowblk, int vec_ok) {
    typedef WCfg<LP> C;
    constexpr int WR = C::WR, G = C::G;
    constexpr int WI = WR * 64;
    constexpr int PS = LP + 8;  // S tile row pitch (bf16 elements)
    constexpr int PA = WI + 8;  // A tile row pitch (NN)
    constexpr int NS = SPLIT ? 2 : 1;
    constexpr int SCH = KS * LP / 8;  // 16-B chunks of one S tile
    constexpr int SPT = (SCH + 255) / 256;
    constexpr int AEL = FP8 ? 16 : 8;  // A elements per 16-B chunk
    constexpr int ACH = KS * WI / AEL;
    constexpr int APT = NN ? (ACH + 255) / 256 : 1;
    typedef typename std::conditional<FP8, uint2, uint4>::type AF;  // 8 A elements along k
    typedef typename std::conditional<FP8, fp8_t, bf16_t>::type TA;
    const TA* __restrict__ A = reinterpret_cast<const TA*>(Av);

    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    bf16_t* Ss = reinterpret_cast<bf16_t*>(smem_raw);  // [NS][KS][PS]
    bf16_t* As = Ss + NS * KS * PS;                    // [KS][PA]   (NN)

    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int r = lane & 15, h = lane >> 4, q = r >> 2, p = r & 3;
    const int wr = w % WR, wc = w / WR;
    const int bid = xcd_remap(blockIdx.x, gridDim.x);
    const int rb = bid % nrowblk, sp = bid / nrowblk;
    const int64_t row0 = (int64_t)rb * WI;
    const int64_t kbeg = (int64_t)sp * kchunk;
    const int64_t kend = (kbeg + kchunk < K) ? kbeg + kchunk : K;
    const bf16_t* Sarr[2] = {Shi, Slo};

    uint4 sreg[NS][SPT];
    uint4 areg[APT];
    AF afr[NN ? 1 : RT];

    auto load_S = [&](int64_t kk) {
#pragma unroll
        for (int a = 0; a < NS; ++a)
#pragma unroll
            for (int t = 0; t < SPT; ++t) {
                const int u = tid + 256 * t;
                const int krow = u / (LP / 8), c8 = u % (LP / 8);
                const int64_t k = kk + krow;
                uint4 v = make_uint4(0, 0, 0, 0);
                if (u < SCH && k < kend) v = *reinterpret_cast<const uint4*>(Sarr[a] + k * LP + c8 * 8);
                sreg[a][t] = v;
            }
    };
    auto store_S = [&]() {
#pragma unroll
        for (int a = 0; a < NS; ++a)
#pragma unroll
            for (int t = 0; t < SPT; ++t) {
                const int u = tid + 256 * t;
                if (u < SCH) {
                    const int krow = u / (LP / 8), c8 = u % (LP / 8);
                    *reinterpret_cast<uint4*>(Ss + (a * KS + krow) * PS + c8 * 8) = sreg[a][t];
                }
            }
    };
    auto load_A_nn = [&](int64_t kk) {
#pragma unroll
        for (int t = 0; t < APT; ++t) {
            const int u = tid + 256 * t;
            const int j = u / (WI / AEL), ic = u % (WI / AEL);
            const int64_t jj = kk + j, i = row0 + (int64_t)ic * AEL;
            uint4 v = make_uint4(0, 0, 0, 0);
            if (u < ACH && jj < kend) {
                const TA* src = A + jj * lda + i;
                if (vec_ok && i + AEL <= rows_out) {
                    v = *reinterpret_cast<const uint4*>(src);
                } else {
                    TA* e = reinterpret_cast<TA*>(&v);
#pragma unroll
                    for (int x = 0; x < AEL; ++x) e[x] = (i + x < rows_out) ? src[x] : TA(0);
                }
            }
            areg[t] = v;
        }
    };
    auto store_A_nn = [&]() {
#pragma unroll
        for (int t = 0; t < APT; ++t) {
            const int u = tid + 256 * t;
            if (u < ACH) {
                const int j = u / (WI / AEL), ic = u % (WI / AEL);
                if (FP8) {
                    const uint2 b0 = fp8x4_to_bf16x4(areg[t].x), b1 = fp8x4_to_bf16x4(areg[t].y);
                    const uint2 b2 = fp8x4_to_bf16x4(areg[t].z), b3 = fp8x4_to_bf16x4(areg[t].w);
                    uint4* d = reinterpret_cast<uint4*>(As + j * PA + ic * AEL);
                    d[0] = make_uint4(b0.x, b0.y, b1.x, b1.y);
                    d[1] = make_uint4(b2.x, b2.y, b3.x, b3.y);
                } else {
                    *reinterpret_cast<uint4*>(As + j * PA + ic * AEL) = areg[t];
                }
            }
        }
    };
    auto load_A_tn = [&](int64_t kk) {
#pragma unroll
        for (int t = 0; t < (NN ? 1 : RT); ++t) {
            const int64_t jc = row0 + wr * 64 + 16 * t + r;  // output row = column of A
            const int64_t i = kk + 8 * h;
            AF v;
            TA* e = reinterpret_cast<TA*>(&v);
#pragma unroll
            for (int x = 0; x < 8; ++x) e[x] = TA(0);
            if (jc < rows_out) {
                const TA* src = A + jc * lda + i;
                if (vec_ok && i + 8 <= kend) {
                    v = *reinterpret_cast<const AF*>(src);
                } else {
#pragma unroll
                    for (int x = 0; x < 8; ++x) e[x] = (i + x < kend) ? src[x] : TA(0);
                }
            }
            afr[t] = v;
        }
    };

    f32x4 acc[RT][G];
#pragma unroll
    for (int t = 0; t < RT; ++t)
#pragma unroll
        for (int g = 0; g < G; ++g) acc[t][g] = f32x4{0.f, 0.f, 0.f, 0.f};

    if (kbeg < kend) {
        load_S(kbeg);
        if (NN) load_A_nn(kbeg); else load_A_tn(kbeg);
    }
    for (int64_t kk = kbeg; kk < kend; kk += KS) {
        __syncthreads();  // previous step's LDS reads are done
        store_S();
        if (NN) store_A_nn();
        AF acur[NN ? 1 : RT];
        if (!NN) {
#pragma unroll
            for (int t = 0; t < (NN ? 1 : RT); ++t) acur[t] = afr[t];
        }
        __syncthreads();
        if (kk + KS < kend) {  // prefetch the next step while this one computes
            load_S(kk + KS);
            if (NN) load_A_nn(kk + KS); else load_A_tn(kk + KS);
        }
        bf16x8_t af[RT];
#pragma unroll
        for (int t = 0; t < RT; ++t) {
            if (NN) {
                const bf16_t* b = As + (8 * h + q) * PA + wr * 64 + 16 * t + 4 * p;
                af[t] = join(tr_read(b), tr_read(b + 4 * PA));
            } else if (FP8) {
                const uint2 x = *reinterpret_cast<const uint2*>(&acur[t]);
                const uint2 lo = fp8x4_to_bf16x4(x.x), hi = fp8x4_to_bf16x4(x.y);
                af[t] = __builtin_bit_cast(bf16x8_t, make_uint4(lo.x, lo.y, hi.x, hi.y));
            } else {
                af[t] = __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const uint4*>(&acur[t]));
            }
        }
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const int col = wc * G * 16 + 16 * g + 4 * p;
            const bf16_t* b = Ss + (8 * h + q) * PS + col;
            const bf16x8_t bh = join(tr_read(b), tr_read(b + 4 * PS));
            bf16x8_t bl;
            if (SPLIT) {
                const bf16_t* c = b + KS * PS;
                bl = join(tr_read(c), tr_read(c + 4 * PS));
            }
#pragma unroll
            for (int t = 0; t < RT; ++t) {
                acc[t][g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[t], bh, acc[t][g], 0, 0, 0);
                if (SPLIT) acc[t][g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[t], bl, acc[t][g], 0, 0, 0);
            }
        }
    }

    float* dst = out + (int64_t)sp * slab_stride;
#pragma unroll
    for (int t = 0; t < RT; ++t)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int64_t row = row0 + wr * 64 + 16 * t + 4 * h + j;
            if (row < rows_out) {
#pragma unroll
                for (int g = 0; g < G; ++g) dst[row * LP + wc * G * 16 + 16 * g + r] = acc[t][g][j];
            }
        }
}

// ------------------------------------------------------------------------------------------------
// v2 (bf16 A, LP in {128, 256, 512}): the same products on a 512-thread workgroup fed by an
// LDS-DMA pipeline.  Every operand tile of a 32-deep k-step -- the S hi / lo tiles [32][LP] and the
// A tile ([32 j][WI i] for NN, [WI j][32 i] for TN) -- is copied HBM -> LDS with
// global_load_lds_dwordx4 into a ring of NST stages (2-4 by LDS size), NST - 1 steps ahead, with
// one raw s_barrier per k-step and a counted vmcnt wait (cdna_hip_programming.md §5 "Pipelining
// across barriers").  glds writes lane-linear LDS, so the images are swizzled through the per-lane
// SOURCE address: 16-B chunk c of row k lands at chunk c ^ f(k), f(k) = 2((k & 3) | ((k >> 3) & 1) << 2)
// for the [32][...] images (ds_read_b64_tr_b16 conflict-free) and c ^ ((j >> 1) & 3) for the TN A
// image (ds_read_b128 conflict-free; tools/ check in DESIGN.md §3.6).  The S panels must be
// zero-padded to a multiple of 32 rows; A indices are clamped in bounds (the zero S rows cancel
// whatever the clamped A values are).
//
// DS ("double step", bf16 TN at LP = 128): a stage holds TWO 32-deep k-steps, so every A column
// contributes one 128-B run per stage -- a full-line fabric request instead of two 64-B ones (the
// TN A image is [WI j][64 i], unit c of row j holding rows 32 (c >> 2) + 8 ((c & 3) ^ ((j >> 1) & 3))
// .. +7, ds_read_b128 conflict-free per 8 lanes).  To fit two stages in LDS the workgroup takes 256
// output rows (4 x 2 waves, 64 S columns each).  Needs K and the K chunks multiples of 64.
template <int LP, bool DS> struct W2Cfg;
template <> struct W2Cfg<128, false> { static constexpr int WR = 8, WC = 1, G = 8; };
template <> struct W2Cfg<128, true> { static constexpr int WR = 4, WC = 2, G = 4; };
template <> struct W2Cfg<256, false> { static constexpr int WR = 4, WC = 2, G = 8; };
template <> struct W2Cfg<512, false> { static constexpr int WR = 2, WC = 4, G = 8; };

template <int LP, bool SPLIT, bool FP8, bool DS = false, bool S8 = false, bool SC = false>
struct W2Shape {
    static constexpr int WR = W2Cfg<LP, DS>::WR, WC = W2Cfg<LP, DS>::WC, G = W2Cfg<LP, DS>::G;
    static constexpr int WI = WR * 64;            // output rows per workgroup
    static constexpr int NS = SPLIT ? 2 : 1;
    static constexpr int KSS = SC ? 4 * KS : (DS ? 2 * KS : KS);  // k rows per stage (SC: one K = 128 MFMA)
    static constexpr int SBYTES = KSS * LP * (S8 ? 1 : 2);  // one S panel tile (e4m3 S: one byte per element)
    static constexpr int ABYTES = KSS * WI * (FP8 ? 1 : 2);  // the A tile
    static constexpr int STAGE = NS * SBYTES + ABYTES;
    static constexpr int NST0 = 147456 / STAGE;
    static constexpr int NST = NST0 > 4 ? 4 : (NST0 < 2 ? 2 : NST0);
    static constexpr int SGL = SBYTES / 8192;     // glds per thread per S tile (512 threads x 16 B)
    static constexpr int NAI = ABYTES / 1024;     // wave-level glds instructions per A tile
    static constexpr int AGL = NAI / 8;           // ... per wave (every wave)
    static constexpr int AEX = NAI % 8;           // waves 0 .. AEX-1 issue one more
    static constexpr int GL = NS * SGL + AGL;     // glds per thread per stage (waves >= AEX)
    static constexpr size_t LDS = (size_t)NST * STAGE;
};

// fp8 A images: 16-B unit swizzles that keep the fragment reads conflict-free.  NN [32 k][WI i]
// bytes, read by ds_read_b64_tr_b8 (16 lanes = 8 k-rows x 16 bytes; lane r supplies row r >> 1,
// byte 8 (r & 1), and receives the 8 k of column r); TN [WI j][32 k] bytes read by ds_read_b64.
template <int WI>
__device__ __forceinline__ int swz8(int k) { return WI == 128 ? ((k >> 1) & 7) : (k & 15); }

__device__ __forceinline__ int swz(int row) { return 2 * ((row & 3) | (((row >> 3) & 1) << 2)); }

typedef __attribute__((address_space(3))) void* lds_void_ptr;

template <int AUX = 0>
__device__ __forceinline__ void glds16(const void* g, char* lds_wave_base) {
    __builtin_amdgcn_global_load_lds(g, (lds_void_ptr)lds_wave_base, 16, 0, AUX);
}

// LDS reads of the v2 kernel are inline asm: hipcc's waitcnt pass treats a compiler-visible LDS
// read as possibly aliasing the in-flight LDS-DMA and drains vmcnt(0) before it, which would
// serialise the ring (cdna_hip_programming.md §5, "Three .s-level traps").  The asm reads are
// ordered among themselves (volatile) and retired by explicit lgkmcnt waits.
__device__ __forceinline__ uint32_t lds_addr(const void* p) { return (uint32_t)(uintptr_t)(lds_void_ptr)p; }
typedef __attribute__((ext_vector_type(2))) int i32x2;  // asm operands: int vectors stay in registers
typedef __attribute__((ext_vector_type(4))) int i32x4;
__device__ __forceinline__ i32x2 tr_read_a(uint32_t a) {
    i32x2 v;
    asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v) : "v"(a));
    return v;
}
__device__ __forceinline__ i32x4 read128_a(uint32_t a) {
    i32x4 v;
    asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(a));
    return v;
}
__device__ __forceinline__ bf16x8_t join2(i32x2 a, i32x2 b) {
    return __builtin_bit_cast(bf16x8_t, __builtin_shufflevector(a, b, 0, 1, 2, 3));
}
// The wait names the registers it retires as in/out operands, so hipcc cannot read (copy, pack)
// an asm-loaded register before the data has landed.
__device__ __forceinline__ void wait_lgkm0(i32x2& a, i32x2& b, i32x2& c, i32x2& d) {
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a), "+v"(b), "+v"(c), "+v"(d)::"memory");
}
__device__ __forceinline__ void wait_lgkm0(i32x2& a, i32x2& b) {
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a), "+v"(b)::"memory");
}
__device__ __forceinline__ void wait_lgkm0(i32x2& a) { asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a)::"memory"); }
__device__ __forceinline__ void wait_lgkm0(i32x4& a) { asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a)::"memory"); }

template <int N>
__device__ __forceinline__ void wait_vm() {  // s_waitcnt vmcnt(N), expcnt / lgkmcnt untouched
    static_assert(N >= 0 && N < 64, "vmcnt range");
    __builtin_amdgcn_s_waitcnt((N & 0xF) | ((N >> 4) << 14) | (0x7 << 4) | (0xF << 8));
}

__device__ __forceinline__ i32x2 tr8_read_a(uint32_t a) {
    i32x2 v;
    asm volatile("ds_read_b64_tr_b8 %0, %1" : "=v"(v) : "v"(a));
    return v;
}
__device__ __forceinline__ i32x2 read64_a(uint32_t a) {
    i32x2 v;
    asm volatile("ds_read_b64 %0, %1" : "=v"(v) : "v"(a));
    return v;
}
// 8 e4m3 bytes (k order) -> the bf16x8 fragment (exact)
__device__ __forceinline__ bf16x8_t fp8x8_to_bf16x8(i32x2 v) {
    const uint2 a = fp8x4_to_bf16x4((uint32_t)v.x), b = fp8x4_to_bf16x4((uint32_t)v.y);
    return __builtin_bit_cast(bf16x8_t, make_uint4(a.x, a.y, b.x, b.y));
}

// KN (tuning knobs): bit 0 -- A (read once per launch) with the non-temporal policy (aux = 2) so
// the panel S, re-read by every workgroup, keeps the L2; bit 1 -- s_setprio 1 for waves 4-7.
// S8 (e4m3 A, NN, single pass, LP >= 256): S is an e4m3 panel -- the exactly-e4m3 Gaussian sketch
// Omega -- so both operands stay e4m3 and the product runs on v_mfma_f32_16x16x32_fp8_fp8: no
// widening of A, half the S bytes through L2 and LDS.  The S image is [32 k][LP] bytes swizzled
// like the e4m3 A image and read with ds_read_b64_tr_b8.
// SC (with S8; K and the K chunks multiples of 128): 128-deep stages on the block-scaled
// v_mfma_scale_f32_16x16x128_f8f6f4 with unit E8M0 scales (127) -- e4m3 x e4m3 exact, twice the
// non-scaled fp8 form's rate (MI355X_MICROARCH.md "Matrix cores").  A lane's 32-byte fragment is
// four ds_read_b64_tr_b8 at k rows 32 i + 8 h + (r >> 1), i = 0..3 (k = 32 i + 8 h .. + 7 of its
// column), the same k set for the A and the B operand -- the contraction only needs the two
// operands' k orders to agree (tools/mfma_scale_probe.hip: exact against a host product).
template <bool FP8, bool NN, int LP, bool SPLIT, bool DS = false, int KN = 0, bool S8 = false, bool SC = false>
__global__ __launch_bounds__(512) void wproj2_kernel(const void* __restrict__ Av, int64_t lda, int64_t rows_out,
                                                     int64_t K, int64_t arows, const bf16_t* __restrict__ Shi,
                                                     const bf16_t* __restrict__ Slo, float* __restrict__ out,
                                                     int64_t slab_stride, int64_t kchunk, int nrowblk, int s_pitch,
                                                     int o_pitch, int halves) {
    typedef W2Shape<LP, SPLIT, FP8, DS, S8, SC> SH;
    static_assert(!SC || S8, "scaled fp8 MFMA: e4m3 x e4m3 sketch only");
    static_assert(!DS || (!NN && !FP8), "double-step stages: bf16 TN only");
    static_assert(!S8 || (FP8 && NN && !SPLIT && LP >= 256), "e4m3 S: single-pass e4m3 NN at LP >= 256");
    constexpr int KSS = SH::KSS;
    const bf16_t* __restrict__ A = reinterpret_cast<const bf16_t*>(Av);
    const uint8_t* __restrict__ A8 = reinterpret_cast<const uint8_t*>(Av);
    constexpr int WR = SH::WR, G = SH::G, WI = SH::WI, NS = SH::NS, NST = SH::NST;
    extern __shared__ __attribute__((aligned(1024))) char smem_raw[];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int r = lane & 15, h = lane >> 4, q = r >> 2, p = r & 3;
    const int wr = w % WR, wc = w / WR;
    // halves = 2: the two 256-column halves of an LP = 512 product in one launch, as neighbouring
    // logical blocks (same XCD, dispatched together), so the twin's A reads hit the L2
    const int bid2 = xcd_remap(blockIdx.x, gridDim.x);
    const int hf = bid2 % halves, bid = bid2 / halves;
    if (hf) {
        Shi = S8 ? reinterpret_cast<const bf16_t*>(reinterpret_cast<const uint8_t*>(Shi) + 256 * hf) : Shi + 256 * hf;
        if (Slo) Slo += 256 * hf;
        out += 256 * hf;
    }
    const int rb = bid % nrowblk, sp = bid / nrowblk;
    const int64_t row0 = (int64_t)rb * WI;
    const int64_t kbeg = (int64_t)sp * kchunk;
    const int64_t kend = (kbeg + kchunk < K) ? kbeg + kchunk : K;
    const int nsteps = (int)((kend - kbeg + KSS - 1) / KSS);

    // issue the glds of step `st` into ring slot st % NST
    auto issue = [&](int st) {
        char* slot = smem_raw + (size_t)(st % NST) * SH::STAGE;
        const int64_t k0 = kbeg + (int64_t)st * KSS;
        if constexpr (S8) {  // [32 k][LP] bytes: 16-B chunk cp of row k at cp ^ swz8<LP>(k)
            const uint8_t* S = reinterpret_cast<const uint8_t*>(Shi);
#pragma unroll
            for (int t = 0; t < SH::SGL; ++t) {
                const int gi = t * 8 + w;
                const int u = gi * 64 + lane;
                constexpr int CPR = LP / 16;
                const int k = u / CPR, cp = u % CPR;
                glds16(S + (k0 + k) * s_pitch + 16 * (cp ^ swz8<LP>(k)), slot + gi * 1024);
            }
        } else {
#pragma unroll
        for (int a = 0; a < NS; ++a) {
            const bf16_t* S = a ? Slo : Shi;
#pragma unroll
            for (int t = 0; t < SH::SGL; ++t) {
                const int gi = t * 8 + w;             // wave instruction index within the tile
                const int u = gi * 64 + lane;         // 16-B chunk of the LDS image
                const int row = u / (LP / 8), cc = u % (LP / 8);
                glds16(S + (k0 + row) * s_pitch + 8 * (cc ^ swz(row)), slot + a * SH::SBYTES + gi * 1024);
            }
        }
        }
        char* at = slot + NS * SH::SBYTES;
        if constexpr (FP8) {
#pragma unroll
            for (int t = 0; t < (SH::NAI + 7) / 8; ++t) {
                const int gi = t * 8 + w;
                if (SH::NAI % 8 == 0 || gi < SH::NAI) {
                    const int u = gi * 64 + lane;
                    const uint8_t* src;
                    if (NN) {  // [32 k][WI i] bytes: unit u -> k row, swizzled 16-row chunk
                        constexpr int CPR = WI / 16;
                        const int k = u / CPR, cp = u % CPR;
                        int64_t kk = k0 + k;
                        kk = kk < K ? kk : K - 1;
                        int64_t i = row0 + 16 * (cp ^ swz8<WI>(k));
                        i = (i + 16 <= arows) ? i : arows - 16;
                        src = A8 + kk * lda + i;
                    } else {  // [WI j][32 k] bytes: 2 units per column j, swapped on (j >> 3) & 1
                        const int j = u >> 1, cc = u & 1;
                        int64_t jc = row0 + j;
                        jc = jc < rows_out ? jc : rows_out - 1;
                        int64_t i = k0 + 16 * (cc ^ ((j >> 3) & 1));
                        i = (i + 16 <= arows) ? i : arows - 16;
                        src = A8 + jc * lda + i;
                    }
                    glds16<(KN & 1) ? 2 : 0>(src, at + gi * 1024);
                }
            }
            return;
        }
#pragma unroll
        for (int t = 0; t < SH::AGL; ++t) {
            const int gi = t * 8 + w;
            const int u = gi * 64 + lane;
            const bf16_t* src;
            if (NN) {  // [32 j][WI i]: row = A column k0 + j, 8 rows i per chunk
                const int j = u / (WI / 8), cc = u % (WI / 8);
                int64_t jj = k0 + j;
                jj = jj < K ? jj : K - 1;
                int64_t i = row0 + 8 * (cc ^ swz(j));
                i = (i + 8 <= arows) ? i : arows - 8;
                src = A + jj * lda + i;
            } else if (DS) {  // [WI j][64 i]: 8 units of 8 rows i, swizzled within each 32-row half
                const int j = u >> 3, c8 = u & 7;
                int64_t jc = row0 + j;
                jc = jc < rows_out ? jc : rows_out - 1;
                int64_t i = k0 + 32 * (c8 >> 2) + 8 * ((c8 & 3) ^ ((j >> 1) & 3));
                i = (i + 8 <= arows) ? i : arows - 8;
                src = A + jc * lda + i;
            } else {  // [WI j][32 i]: row = A column row0 + j, 4 chunks of 8 rows i
                const int j = u >> 2, cc = u & 3;
                int64_t jc = row0 + j;
                jc = jc < rows_out ? jc : rows_out - 1;
                int64_t i = k0 + 8 * (cc ^ ((j >> 1) & 3));
                i = (i + 8 <= arows) ? i : arows - 8;
                src = A + jc * lda + i;
            }
            glds16<(KN & 1) ? 2 : 0>(src, at + gi * 1024);
        }
    };

    f32x4 acc[RT][G];
#pragma unroll
    for (int t = 0; t < RT; ++t)
#pragma unroll
        for (int g = 0; g < G; ++g) acc[t][g] = f32x4{0.f, 0.f, 0.f, 0.f};

    if ((KN & 2) && w >= 4) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int st = 0; st < NST - 1; ++st)
        if (st < nsteps) issue(st);

    for (int st = 0; st < nsteps; ++st) {
        // stage st has landed once at most the younger stages' glds are outstanding
        if (st + NST - 2 < nsteps) {
            if (SH::AEX && w < SH::AEX) wait_vm<(NST - 2) * (SH::GL + 1)>();
            else wait_vm<(NST - 2) * SH::GL>();
        } else {
            wait_vm<0>();
        }
        __builtin_amdgcn_s_barrier();
        if (st + NST - 1 < nsteps) issue(st + NST - 1);
        const uint32_t slot = lds_addr(smem_raw) + (uint32_t)((st % NST) * SH::STAGE);
        const uint32_t At = slot + NS * SH::SBYTES;
#pragma unroll
        for (int ss = 0; ss < KSS / KS; ++ss) {  // the k-steps of the stage
            if constexpr (SC) {  // one 128-deep step: A fragments [RT][4 x 8 B], B per column tile, double-buffered
                typedef __attribute__((ext_vector_type(8))) int i32x8;
                const int kb = 8 * h + (r >> 1);
                i32x2 a8[RT][4];
#pragma unroll
                for (int t = 0; t < RT; ++t)
#pragma unroll
                    for (int i4 = 0; i4 < 4; ++i4) {
                        const int k = kb + 32 * i4;
                        a8[t][i4] = tr8_read_a(At + k * WI + 16 * ((4 * wr + t) ^ swz8<WI>(k)) + 8 * (r & 1));
                    }
                auto bread8 = [&](int g, i32x2 (&b)[4]) {
#pragma unroll
                    for (int i4 = 0; i4 < 4; ++i4) {
                        const int k = kb + 32 * i4;
                        b[i4] = tr8_read_a(slot + k * LP + 16 * ((wc * G + g) ^ swz8<LP>(k)) + 8 * (r & 1));
                    }
                };
                i32x2 b8[2][4];
                bread8(0, b8[0]);
#pragma unroll
                for (int t = 0; t < RT; ++t) wait_lgkm0(a8[t][0], a8[t][1], a8[t][2], a8[t][3]);
                wait_lgkm0(b8[0][0], b8[0][1], b8[0][2], b8[0][3]);
                i32x8 af8[RT];
#pragma unroll
                for (int t = 0; t < RT; ++t)
                    af8[t] = i32x8{a8[t][0].x, a8[t][0].y, a8[t][1].x, a8[t][1].y,
                                   a8[t][2].x, a8[t][2].y, a8[t][3].x, a8[t][3].y};
#pragma unroll
                for (int g = 0; g < G; ++g) {
                    if (g + 1 < G) bread8(g + 1, b8[(g + 1) & 1]);
                    __builtin_amdgcn_sched_barrier(0);
                    const i32x2* b = b8[g & 1];
                    const i32x8 bf = i32x8{b[0].x, b[0].y, b[1].x, b[1].y, b[2].x, b[2].y, b[3].x, b[3].y};
#pragma unroll
                    for (int t = 0; t < RT; ++t)
                        acc[t][g] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(af8[t], bf, acc[t][g], 0, 0, 0,
                                                                                     127, 0, 127);
                    __builtin_amdgcn_sched_barrier(0);
                    if (g + 1 < G) {
                        i32x2(&n)[4] = b8[(g + 1) & 1];
                        wait_lgkm0(n[0], n[1], n[2], n[3]);
                    }
                }
                break;  // the whole 128-deep stage
            }
            bf16x8_t af[RT];
            i32x2 a1[RT], a2[RT];
            i32x4 a4[RT];
#pragma unroll
            for (int t = 0; t < RT; ++t) {
                if (FP8) {
                    if (NN) {
                        const int k = 8 * h + (r >> 1);
                        const int c = 4 * wr + t;  // 16-row chunk of the tile
                        a1[t] = tr8_read_a(At + k * WI + 16 * (c ^ swz8<WI>(k)) + 8 * (r & 1));
                    } else {
                        const int j = wr * 64 + 16 * t + r;
                        a1[t] = read64_a(At + j * 32 + 8 * (h ^ (2 * ((j >> 3) & 1))));
                    }
                } else if (NN) {
                    const int col = wr * 64 + 16 * t + 4 * p;  // i within the tile
                    const int k1 = 8 * h + q, k2 = k1 + 4;
                    a1[t] = tr_read_a(At + k1 * (WI * 2) + 16 * ((col >> 3) ^ swz(k1)) + 2 * (col & 7));
                    a2[t] = tr_read_a(At + k2 * (WI * 2) + 16 * ((col >> 3) ^ swz(k2)) + 2 * (col & 7));
                } else {
                    const int j = wr * 64 + 16 * t + r;
                    a4[t] = read128_a(At + j * (KSS * 2) + 16 * (4 * ss + (h ^ ((j >> 1) & 3))));
                }
            }
            if constexpr (S8) {  // both operands e4m3: fragments are the raw 8 bytes of k 8h .. 8h + 7
                i32x2 bv[G];
                const int k = 8 * h + (r >> 1);
#pragma unroll
                for (int g = 0; g < G; ++g)  // every B fragment in flight, then one wait
                    bv[g] = tr8_read_a(slot + k * LP + 16 * ((wc * G + g) ^ swz8<LP>(k)) + 8 * (r & 1));
#pragma unroll
                for (int t = 0; t < RT; ++t) wait_lgkm0(a1[t]);
#pragma unroll
                for (int g = 0; g < G; ++g) wait_lgkm0(bv[g]);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int g = 0; g < G; ++g)
#pragma unroll
                    for (int t = 0; t < RT; ++t)
                        acc[t][g] = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(__builtin_bit_cast(long, a1[t]),
                                                                              __builtin_bit_cast(long, bv[g]), acc[t][g],
                                                                              0, 0, 0);
                continue;
            }
            // B fragments of column tile g: hi (and lo) halves of the transposed S rows 8h+q, 8h+q+4
            auto bread = [&](int g, i32x2* b) {
                const int col = wc * G * 16 + 16 * g + 4 * p;
                const int k1 = 8 * h + q + 32 * ss, k2 = k1 + 4;
                const uint32_t o1 = 2 * (k1 * LP + 8 * ((col >> 3) ^ swz(k1)) + (col & 7));
                const uint32_t o2 = 2 * (k2 * LP + 8 * ((col >> 3) ^ swz(k2)) + (col & 7));
                b[0] = tr_read_a(slot + o1);
                b[1] = tr_read_a(slot + o2);
                if (SPLIT) {
                    b[2] = tr_read_a(slot + SH::SBYTES + o1);
                    b[3] = tr_read_a(slot + SH::SBYTES + o2);
                }
            };
            i32x2 bb[2][4];
            bread(0, bb[0]);
            auto wait_b = [&](i32x2* b) {
                if (SPLIT) wait_lgkm0(b[0], b[1], b[2], b[3]);
                else wait_lgkm0(b[0], b[1]);
            };
            wait_b(bb[0]);
#pragma unroll
            for (int t = 0; t < RT; ++t) {  // (retired by the wait above; these waits are no-ops that pin the order)
                if (FP8) {
                    wait_lgkm0(a1[t]);
                    af[t] = fp8x8_to_bf16x8(a1[t]);
                } else {
                    if (NN) wait_lgkm0(a1[t], a2[t]);
                    else wait_lgkm0(a4[t]);
                    af[t] = NN ? join2(a1[t], a2[t]) : __builtin_bit_cast(bf16x8_t, a4[t]);
                }
            }
#pragma unroll
            for (int g = 0; g < G; ++g) {
                if (g + 1 < G) bread(g + 1, bb[(g + 1) & 1]);  // next tile's fragments in flight
                const i32x2* b = bb[g & 1];
                const bf16x8_t bh = join2(b[0], b[1]);
#pragma unroll
                for (int t = 0; t < RT; ++t) acc[t][g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[t], bh, acc[t][g], 0, 0, 0);
                if (SPLIT) {
                    const bf16x8_t bl = join2(b[2], b[3]);
#pragma unroll
                    for (int t = 0; t < RT; ++t)
                        acc[t][g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[t], bl, acc[t][g], 0, 0, 0);
                }
                if (g + 1 < G) wait_b(bb[(g + 1) & 1]);
            }
        }
    }

    float* dst = out + (int64_t)sp * slab_stride;
#pragma unroll
    for (int t = 0; t < RT; ++t)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int64_t row = row0 + wr * 64 + 16 * t + 4 * h + j;
            if (row < rows_out) {
#pragma unroll
                for (int g = 0; g < G; ++g) dst[row * o_pitch + wc * G * 16 + 16 * g + r] = acc[t][g][j];
            }
        }
}

// ------------------------------------------------------------------------------------------------
// v3 (bf16 A, LP in {256, 512}).  Two changes against v2, both measured at C4 (wide_lab):
// (1) Every LDS fragment read is (per-lane base, fixed for the launch) + (slot offset, one v_add
//     per base and step) + (immediate tile offset).  v2's XOR swizzle put the tile index inside the
//     XOR, so the compiler rebuilt 80+ addresses per k-step -- 110 VALU per 64 MFMA, 57 % MFMA
//     busy.  The row images are conflict-free by PLACEMENT instead: a [32 k][RB bytes] image is cut
//     into 1-KiB LDS-DMA pieces of 1024 / RB rows at a 1056-B pitch, and k row r goes to piece slot
//     sigma(r) (bits 2 and 3 swapped), so the eight rows one ds_read_b64_tr_b16 touches ({0-3,
//     8-11} + 4 j + 16 i) start at eight different 32-B bank offsets; columns stay in natural
//     order, so a tile index is a constant offset.  (A 32x32x16-MFMA form of the same kernel, which
//     blocks issue for 8 of 32 cycles instead of 8 of 16, measured 5 % slower: dropped.)
// (2) A and S have separate LDS rings.  Ablations (nobar / nodma / nolds) showed the DMA stream,
//     not the MFMA or the LDS reads, bounding the kernel: bytes in flight per CU were capped by
//     the shared ring (two 48-KiB stages), ~16 B/clk/CU at HBM latency.  A (HBM, read once) now
//     runs DA steps ahead in its own ring, S (L2-resident panel re-read by every workgroup) SD
//     steps ahead in a smaller one.
// The TN A image ([WI j][32 i], 64-B rows, read by ds_read_b128) keeps an XOR swizzle whose term
// depends on the lane only.  LDS: [A ring: NA x AIMG][S ring: (SD + 1) x NS x SIMG].
__host__ __device__ constexpr int v3_sigma(int r) { return (r & ~12) | ((r >> 1) & 4) | ((r << 1) & 8); }

template <int RB>  // a [32 k][RB bytes] image, RB in {256, 512, 1024}
struct RowImg {
    static constexpr int RP = 1024 / RB, PITCH = 1056, PIECES = 32 / RP;
    static constexpr int BYTES = PIECES * PITCH;
    __host__ __device__ static constexpr int off(int r) {
        const int s = v3_sigma(r), G = s >> 3, idx = s & 7;
        return ((G / RP) * 8 + idx) * PITCH + (G % RP) * RB;
    }
    __host__ __device__ static constexpr int row_of(int pc, int part) {  // the row piece pc holds in `part`
        return v3_sigma(((pc >> 3) * RP + part) * 8 + (pc & 7));
    }
};

template <int LP, bool NN, bool SPLIT, int SD>
struct W3Shape {
    static constexpr int WR = W2Cfg<LP, false>::WR, WC = W2Cfg<LP, false>::WC, G = W2Cfg<LP, false>::G;
    static constexpr int WI = WR * 64;
    static constexpr int NS = SPLIT ? 2 : 1;
    typedef RowImg<LP * 2> SImg;
    typedef RowImg<WI * 2> AImg;
    static constexpr int SIMG = SImg::BYTES;
    static constexpr int AIMG0 = NN ? AImg::BYTES : KS * WI * 2;
    static constexpr int AIMG = (AIMG0 + 255) / 256 * 256;
    static constexpr int SPC = SImg::PIECES;                   // pieces per S image
    static constexpr int APC = NN ? AImg::PIECES : AIMG0 / 1024;  // pieces of the A image
    static constexpr int SPW = SPC / 8, APW = APC / 8;          // ... per wave
    static constexpr int APITCH = NN ? AImg::PITCH : 1024;
    static constexpr int SSLOT = (NS * SIMG + 255) / 256 * 256;
    static constexpr int NSS = SD + 1;                         // S ring slots
    static constexpr int NA0 = (163840 - NSS * SSLOT) / AIMG;
    static constexpr int NA = NA0 > 8 ? 8 : NA0;               // A ring slots
    static constexpr int DA = NA - 1;                          // A prefetch distance (steps)
    static constexpr int SBASE = NA * AIMG;
    static constexpr int GL = NS * SPW + APW;                  // glds per thread per step
    static constexpr size_t LDS = (size_t)SBASE + (size_t)NSS * SSLOT;
    static_assert(SPC % 8 == 0 && APC % 8 == 0, "v3 piece split");
    // DA > SD: A(st) must be issued before S(st) -- the steady-state wait counts only what follows S(st)
    static_assert(DA > SD && LDS <= 163840, "v3 rings");
    static_assert((NS - 1) * SIMG + 32 * G < 65536, "immediate offsets");
};

template <typename F, int... I>
__device__ __forceinline__ void static_for_impl(F& f, std::integer_sequence<int, I...>) {
    (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F& f) {
    static_for_impl(f, std::make_integer_sequence<int, N>{});
}

template <int OFF>
__device__ __forceinline__ i32x2 tr_read_o(uint32_t a) {
    i32x2 v;
    asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(v) : "v"(a), "i"(OFF));
    return v;
}
template <int OFF>
__device__ __forceinline__ i32x4 read128_o(uint32_t a) {
    i32x4 v;
    asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(a), "i"(OFF));
    return v;
}

// ABL (lab ablations, results meaningless): bit 0 no barrier / DMA waits, bit 1 no DMA, bit 2 no
// LDS fragment reads.  The product path instantiates ABL = 0 only.
// AR (lab only, abl 16): A staged through registers -- the LDS-DMA stream then carries only the
// L2-resident S panels and the HBM-sourced A goes global -> VGPR -> ds_write.  Bit-identical; in the
// isolated kernel loop it is 7 % faster (tools/wide_lab areg: NN2 3324 -> 3084 us, TN2 3383 -> 3136
// us), but inside the 29-ms rSVD loop 2.4 % slower on the same box (C4 28.06-28.11 ms with DMA A vs
// 28.77-28.83 ms, TN 3555 vs 3680 us; profiles/r02_v6_areg_ab.txt), so the engine keeps DMA A.
template <bool NN, int LP, bool SPLIT, int KN, int SD, int ABL = 0, bool AR = false>
__global__ __launch_bounds__(512) void wproj3_kernel(const bf16_t* __restrict__ A, int64_t lda, int64_t rows_out,
                                                     int64_t K, int64_t arows, const bf16_t* __restrict__ Shi,
                                                     const bf16_t* __restrict__ Slo, float* __restrict__ out,
                                                     int64_t slab_stride, int64_t kchunk, int nrowblk) {
    typedef W3Shape<LP, NN, SPLIT, SD> SH;
    typedef typename SH::SImg SImg;
    typedef typename SH::AImg AImg;
    constexpr int WR = SH::WR, G = SH::G, WI = SH::WI, NS = SH::NS, NA = SH::NA, DA = SH::DA, NSS = SH::NSS;
    extern __shared__ __attribute__((aligned(1024))) char smem_raw[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r = lane & 15, h = lane >> 4, q = r >> 2, p = r & 3;
    const int wr = w % WR, wc = w / WR;
    const int bid = xcd_remap(blockIdx.x, gridDim.x);
    const int rb = bid % nrowblk, sp = bid / nrowblk;
    const int64_t row0 = (int64_t)rb * WI;
    const int64_t kbeg = (int64_t)sp * kchunk;
    const int64_t kend = (kbeg + kchunk < K) ? kbeg + kchunk : K;
    const int nsteps = (int)((kend - kbeg + KS - 1) / KS);

    // per-lane source offsets of this wave's pieces (elements; fixed for the launch)
    int32_t soff[SH::SPW];
#pragma unroll
    for (int t = 0; t < SH::SPW; ++t) {
        constexpr int LPR = 64 / SImg::RP;  // lanes per row
        const int pc = t * 8 + w;
        soff[t] = SImg::row_of(pc, lane / LPR) * LP + 8 * (lane % LPR);
    }
    int64_t aoff[SH::APW];  // NN: A column k0 + r, rows i;  TN: A column row0 + j, rows k0 + i
    int arow[SH::APW];      // NN: r (k row of the image);  TN: i (k row offset within the step)
#pragma unroll
    for (int t = 0; t < SH::APW; ++t) {
        const int pc = t * 8 + w;
        if constexpr (NN) {
            constexpr int LPR = 64 / AImg::RP;
            const int rr = AImg::row_of(pc, lane / LPR);
            int64_t i = row0 + 8 * (lane % LPR);
            i = (i + 8 <= arows) ? i : arows - 8;
            aoff[t] = (int64_t)rr * lda + i;
            arow[t] = rr;
        } else {  // 16 rows j x 4 chunks; chunk position cc holds rows 8 (cc ^ ((j >> 1) & 3))
            const int u = pc * 64 + lane, j = u >> 2, cc = u & 3;
            int64_t jc = row0 + j;
            jc = jc < rows_out ? jc : rows_out - 1;
            const int i = 8 * (cc ^ ((j >> 1) & 3));
            aoff[t] = jc * lda + i;
            arow[t] = i;
        }
    }

    auto issueS = [&](int st) {
        if constexpr ((ABL & 2) != 0) return;
        char* slot = smem_raw + SH::SBASE + (st % NSS) * SH::SSLOT;
        const int64_t k0 = kbeg + (int64_t)st * KS;
#pragma unroll
        for (int a = 0; a < NS; ++a) {
            const bf16_t* S = (a ? Slo : Shi) + k0 * LP;
#pragma unroll
            for (int t = 0; t < SH::SPW; ++t) glds16(S + soff[t], slot + a * SH::SIMG + (t * 8 + w) * SImg::PITCH);
        }
    };
    auto asrc = [&](int st, int t) {
        const int64_t k0 = kbeg + (int64_t)st * KS;
        const bool tail = k0 + KS > K;  // (uniform) the last step of a ragged K: clamp the A reads
        const bf16_t* src;
        if constexpr (NN) {
            src = A + k0 * lda + aoff[t];
            if (tail && k0 + arow[t] >= K) src = A + (K - 1 - arow[t]) * lda + aoff[t];
        } else {
            src = A + k0 + aoff[t];
            if (tail && k0 + arow[t] + 8 > arows) src = A + (arows - 8 - arow[t]) + aoff[t];
        }
        return src;
    };
    auto issueA = [&](int st) {
        if constexpr ((ABL & 2) != 0) return;
        char* slot = smem_raw + (st % NA) * SH::AIMG;
#pragma unroll
        for (int t = 0; t < SH::APW; ++t) glds16<(KN & 1) ? 2 : 0>(asrc(st, t), slot + (t * 8 + w) * SH::APITCH);
    };
    // KN bit 2 (IL): the step's LDS-DMA one piece per column group inside the MFMA loop (the same
    // issue order as the burst after the barrier, so the waits count the same)
    constexpr bool IL = (KN & 4) != 0 && !AR && ABL == 0;
    constexpr int NSP = NS * SH::SPW;
    static_assert(!IL || NSP + SH::APW <= G, "interleaved DMA: one piece per column group");
    auto issueS_piece = [&](int st, int i) {
        char* slot = smem_raw + SH::SBASE + (st % NSS) * SH::SSLOT;
        const int a = i / SH::SPW, t = i % SH::SPW;
        const bf16_t* S = (a ? Slo : Shi) + (kbeg + (int64_t)st * KS) * LP;
        glds16(S + soff[t], slot + a * SH::SIMG + (t * 8 + w) * SImg::PITCH);
    };
    auto issueA_piece = [&](int st, int t) {
        glds16<(KN & 1) ? 2 : 0>(asrc(st, t), smem_raw + (st % NA) * SH::AIMG + (t * 8 + w) * SH::APITCH);
    };
    // AR: A through registers instead of LDS-DMA -- global_load_dwordx4 four steps ahead,
    // ds_write_b128 of the same 16 B to the same LDS address two steps ahead; S stays on the DMA.
    // Loads and writes are inline asm: the compiler's waitcnt pass cannot count the in-flight DMA
    // across the loop and drained vmcnt(0) before every write; the explicit wait_vm below covers them.
    static_assert(!AR || (SD == 1 && NA >= 3), "register-staged A: SD = 1, >= 3 A slots");
    i32x4 areg[2][SH::APW];
    auto loadA = [&](int st, i32x4 (&dst)[SH::APW]) {
#pragma unroll
        for (int t = 0; t < SH::APW; ++t) {
            if constexpr ((KN & 1) != 0)
                asm volatile("global_load_dwordx4 %0, %1, off nt" : "=v"(dst[t]) : "v"(asrc(st, t)) : "memory");
            else
                asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(dst[t]) : "v"(asrc(st, t)) : "memory");
        }
    };
    auto writeA = [&](int st, const i32x4 (&src)[SH::APW]) {
        const uint32_t slot = lds_addr(smem_raw) + (uint32_t)((st % NA) * SH::AIMG) + 16 * lane;
#pragma unroll
        for (int t = 0; t < SH::APW; ++t)
            asm volatile("ds_write_b128 %0, %1" ::"v"(slot + (uint32_t)((t * 8 + w) * SH::APITCH)), "v"(src[t]) : "memory");
    };

    // per-lane LDS read bases within a slot
    const int colS = wc * G * 16 + 4 * p;
    const int k1 = 8 * h + q, k2 = k1 + 4;
    const uint32_t lS1 = SImg::off(k1) + 2 * colS, lS2 = SImg::off(k2) + 2 * colS;
    uint32_t lA1, lA2;
    if constexpr (NN) {
        const int colA = wr * 64 + 4 * p;
        lA1 = AImg::off(k1) + 2 * colA;
        lA2 = AImg::off(k2) + 2 * colA;
    } else {
        lA1 = (wr * 64 + r) * 64 + 16 * (h ^ ((r >> 1) & 3));
        lA2 = 0;
    }

    f32x4 acc[RT][G];
#pragma unroll
    for (int t = 0; t < RT; ++t)
#pragma unroll
        for (int g = 0; g < G; ++g) acc[t][g] = f32x4{0.f, 0.f, 0.f, 0.f};

    if ((KN & 2) && w >= 4) __builtin_amdgcn_s_setprio(1);
    // prologue: the issues of the virtual iterations -DA .. -1 (S(i + SD), A(i + DA)), so that the
    // steady-state wait below counts the same glds in every iteration
    if constexpr (AR) {  // A(0), A(1) by DMA, S(0), then A(2), A(3) into registers
        for (int i = 0; i < 2 && i < nsteps; ++i) issueA(i);
        if (nsteps > 0) issueS(0);
        if (2 < nsteps) loadA(2, areg[0]);
        if (3 < nsteps) loadA(3, areg[1]);
    } else {
        for (int i = -DA; i < 0; ++i) {
            if (i + SD >= 0 && i + SD < nsteps) issueS(i + SD);
            if (i + DA < nsteps) issueA(i + DA);
        }
    }

    const uint32_t lds0 = lds_addr(smem_raw);
    auto iter = [&](int st, i32x4 (&ar)[SH::APW]) {
        if constexpr (AR) {
            // S(st) (issued last iteration) and the register loads of A(st + 2) have landed once at
            // most the APW loads of A(st + 3) are in flight
            if (st + 3 < nsteps) wait_vm<SH::APW>();
            else wait_vm<0>();
            __builtin_amdgcn_s_barrier();
            if (st + 2 < nsteps) writeA(st + 2, ar);
            if (st + 1 < nsteps) issueS(st + 1);
            if (st + 4 < nsteps) loadA(st + 4, ar);
        } else {
            if constexpr ((ABL & 1) == 0) {
                // S(st) and A(st) have landed once at most the glds issued after S(st) are in flight:
                // A(st - SD + DA) and the SD - 1 full iterations since (conservatively all, at the end)
                if (st - 1 + DA < nsteps) wait_vm<SH::APW + (SD - 1) * SH::GL>();
                else wait_vm<0>();
                __builtin_amdgcn_s_barrier();
            }
            if constexpr (!IL) {
                if (st + SD < nsteps) issueS(st + SD);
                if (st + DA < nsteps) issueA(st + DA);
            }
        }
        const bool il_s = st + SD < nsteps, il_a = st + DA < nsteps;
        const uint32_t sS = lds0 + SH::SBASE + (uint32_t)((st % NSS) * SH::SSLOT);
        const uint32_t sA = lds0 + (uint32_t)((st % NA) * SH::AIMG);
        const uint32_t bS1 = sS + lS1, bS2 = sS + lS2, bA1 = sA + lA1, bA2 = sA + lA2;
        auto wait_b = [&](i32x2* b) {
            if (SPLIT) wait_lgkm0(b[0], b[1], b[2], b[3]);
            else wait_lgkm0(b[0], b[1]);
        };
        i32x2 a1[RT], a2[RT];
        i32x4 a4[RT];
        bf16x8_t af[RT];
        auto aread = [&](auto tc) {
            constexpr int t = decltype(tc)::value;
            if constexpr ((ABL & 4) != 0) {
                a1[t] = a2[t] = i32x2{(int)lS1 + t, (int)bA1};
                a4[t] = i32x4{(int)lS2, t, (int)bA1, (int)bA2};
            } else if constexpr (NN) {  // 32 B per 16-row tile
                a1[t] = tr_read_o<32 * t>(bA1);
                a2[t] = tr_read_o<32 * t>(bA2);
            } else {  // 1 KiB per 16-row tile
                a4[t] = read128_o<1024 * t>(bA1);
            }
        };
        static_for<RT>(aread);
        auto bread = [&](auto gc, i32x2* b) {
            constexpr int g = decltype(gc)::value;
            if constexpr ((ABL & 4) != 0) {
                b[0] = b[2] = i32x2{(int)bS1 + g, (int)bS2};
                b[1] = b[3] = i32x2{(int)bS2 + g, (int)bS1};
                return;
            }
            b[0] = tr_read_o<32 * g>(bS1);
            b[1] = tr_read_o<32 * g>(bS2);
            if constexpr (SPLIT) {
                b[2] = tr_read_o<SH::SIMG + 32 * g>(bS1);
                b[3] = tr_read_o<SH::SIMG + 32 * g>(bS2);
            }
        };
        i32x2 bb[2][4];
        bread(std::integral_constant<int, 0>{}, bb[0]);
        wait_b(bb[0]);
#pragma unroll
        for (int t = 0; t < RT; ++t) {
            if (NN) wait_lgkm0(a1[t], a2[t]);
            else wait_lgkm0(a4[t]);
            af[t] = NN ? join2(a1[t], a2[t]) : __builtin_bit_cast(bf16x8_t, a4[t]);
        }
        auto gstep = [&](auto gc) {
            constexpr int g = decltype(gc)::value;
            if constexpr (g + 1 < G) bread(std::integral_constant<int, g + 1>{}, bb[(g + 1) & 1]);
            if constexpr (IL) {
                if constexpr (g < NSP) {
                    if (il_s) issueS_piece(st + SD, g);
                } else if constexpr (g < NSP + SH::APW) {
                    if (il_a) issueA_piece(st + DA, g - NSP);
                }
            }
            __builtin_amdgcn_sched_barrier(0);  // the next tile's reads go out before this tile's MFMAs
            const i32x2* b = bb[g & 1];
            const bf16x8_t bh = join2(b[0], b[1]);
#pragma unroll
            for (int t = 0; t < RT; ++t) acc[t][g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[t], bh, acc[t][g], 0, 0, 0);
            if constexpr (SPLIT) {
                const bf16x8_t bl = join2(b[2], b[3]);
#pragma unroll
                for (int t = 0; t < RT; ++t) acc[t][g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[t], bl, acc[t][g], 0, 0, 0);
            }
            __builtin_amdgcn_sched_barrier(0);  // ... and are waited for only after them
            if constexpr (g + 1 < G) wait_b(bb[(g + 1) & 1]);
        };
        static_for<G>(gstep);
    };
    if constexpr (AR) {  // unrolled by two: each register buffer stays in fixed VGPRs (asm-loaded)
        for (int st = 0; st < nsteps; st += 2) {
            iter(st, areg[0]);
            if (st + 1 < nsteps) iter(st + 1, areg[1]);
        }
    } else {
        for (int st = 0; st < nsteps; ++st) iter(st, areg[0]);
    }

    float* dst = out + (int64_t)sp * slab_stride;
#pragma unroll
    for (int t = 0; t < RT; ++t)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int64_t row = row0 + wr * 64 + 16 * t + 4 * h + j;
            if (row < rows_out) {
#pragma unroll
                for (int g = 0; g < G; ++g) dst[row * LP + wc * G * 16 + 16 * g + r] = acc[t][g][j];
            }
        }
}

template <bool NN, int LP, bool SPLIT, int SD, int ABL = 0>
hipError_t wproj3_go(const void* A, int64_t lda, int64_t m, int64_t n, const bf16_t* Shi, const bf16_t* Slo,
                     const WProjPlan& p, float* slabs, float* Out, hipStream_t s, hipEvent_t done) {
    typedef W3Shape<LP, NN, SPLIT, SD> SH;
    const int64_t rows_out = NN ? m : n, K = NN ? n : m;
    float* o = p.splits == 1 ? Out : slabs;
    const int64_t stride = rows_out * LP;
    // as v2 (profiles/r02_wide_lab_knobs.txt), plus the interleaved DMA (bit 2, round 6) for the LP = 256 NN
    // (C4 -0.23 ms on one box, bit-identical; the LP = 128 NN measured 4.99 -> 5.01 ms at C3 with it)
    constexpr int KN = NN ? ((LP == 256 && ABL == 0) ? 7 : 3) : 0;
#ifdef RSVD_LAB
    constexpr bool ar_ok = ABL == 0 && SD == 1 && SH::NA >= 3;  // register-staged A fits
#else
    constexpr bool ar_ok = false;  // (the lab-only variants are built into tools/wide_lab alone)
#endif
    auto go = [&](auto knc) {
        if constexpr (ar_ok) {
            if (p.abl & 16) {  // abl 16 (lab only): register-staged A
                hipLaunchKernelGGL((wproj3_kernel<NN, LP, SPLIT, decltype(knc)::value, SD, 0, true>),
                                   dim3(p.blocks * p.splits), dim3(512), SH::LDS, s, reinterpret_cast<const bf16_t*>(A),
                                   lda, rows_out, K, m, Shi, Slo, o, stride, p.chunk, p.blocks);
                return;
            }
        }
        hipLaunchKernelGGL((wproj3_kernel<NN, LP, SPLIT, decltype(knc)::value, SD, ABL>), dim3(p.blocks * p.splits),
                           dim3(512), SH::LDS, s, reinterpret_cast<const bf16_t*>(A), lda, rows_out, K, m, Shi, Slo, o,
                           stride, p.chunk, p.blocks);
    };
#ifdef RSVD_LAB
    if constexpr (LP == 256 && ABL == 0 && SD == 1) {  // lab knob sweep (p.kn >= 0); the engine uses KN
        switch (p.kn < 0 ? KN : p.kn) {
            case 0: go(std::integral_constant<int, 0>{}); break;
            case 1: go(std::integral_constant<int, 1>{}); break;
            case 2: go(std::integral_constant<int, 2>{}); break;
            case 3: go(std::integral_constant<int, 3>{}); break;
            default: go(std::integral_constant<int, KN>{}); break;
        }
    } else {
        go(std::integral_constant<int, KN>{});
    }
#else
    go(std::integral_constant<int, KN>{});
#endif
    hipError_t e = hipGetLastError();
    if (e == hipSuccess && done) e = hipEventRecord(done, s);
    if (e != hipSuccess || p.splits == 1) return e;
    return launch_sum_slabs<float>(slabs, stride, p.splits, stride, Out, s);
}

// v3 TN at LP = 256 with two k-steps per A slot: the A image of a slot is [WI j][64 i] (128-B
// rows), so every A column contributes ONE full 128-B line per slot instead of two 64-B halves in
// consecutive steps (v2's DS idea, affordable here because A and S have separate rings: A 2 x 32 KiB,
// S 2 x 33 KiB per hi / lo pair).  Row j's 16-B unit u (rows 8 u .. 8 u + 7 of the 64) sits at unit
// u ^ ((j >> 1) & 7): a ds_read_b128 of 16 lanes (rows r = 0..15, one unit) covers all 16 bank
// positions.  The S images are v3's (32-step, row placement by sigma).
template <bool SPLIT, int KN, bool AR>
__global__ __launch_bounds__(512) void wproj3tn2_kernel(const bf16_t* __restrict__ A, int64_t lda, int64_t rows_out,
                                                        int64_t K, int64_t arows, const bf16_t* __restrict__ Shi,
                                                        const bf16_t* __restrict__ Slo, float* __restrict__ out,
                                                        int64_t slab_stride, int64_t kchunk, int nrowblk) {
    constexpr int LP = 256;
    typedef W3Shape<LP, false, SPLIT, 1> SH;
    typedef typename SH::SImg SImg;
    constexpr int WR = SH::WR, G = SH::G, WI = SH::WI, NS = SH::NS;
    constexpr int ASLOT = WI * 128, APW2 = ASLOT / 1024 / 8;  // A slot bytes; pieces per wave
    constexpr int SBASE = 2 * ASLOT;                           // [A 2 slots][S 2 slots]
    extern __shared__ __attribute__((aligned(1024))) char smem_raw[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r = lane & 15, h = lane >> 4, q = r >> 2, p = r & 3;
    const int wr = w % WR, wc = w / WR;
    const int bid = xcd_remap(blockIdx.x, gridDim.x);
    const int rb = bid % nrowblk, sp = bid / nrowblk;
    const int64_t row0 = (int64_t)rb * WI;
    const int64_t kbeg = (int64_t)sp * kchunk;
    const int64_t kend = (kbeg + kchunk < K) ? kbeg + kchunk : K;
    const int nsteps = (int)((kend - kbeg + KS - 1) / KS);
    const int nd = (nsteps + 1) / 2;

    int32_t soff[SH::SPW];
#pragma unroll
    for (int t = 0; t < SH::SPW; ++t) {
        constexpr int LPR = 64 / SImg::RP;
        const int pc = t * 8 + w;
        soff[t] = SImg::row_of(pc, lane / LPR) * LP + 8 * (lane % LPR);
    }
    int64_t aoff[APW2];
    int arow[APW2];
#pragma unroll
    for (int t = 0; t < APW2; ++t) {
        const int u = (t * 8 + w) * 64 + lane, j = u >> 3, pu = u & 7;
        int64_t jc = row0 + j;
        jc = jc < rows_out ? jc : rows_out - 1;
        const int i = 8 * (pu ^ ((j >> 1) & 7));
        aoff[t] = jc * lda + i;
        arow[t] = i;
    }
    auto issueS = [&](int st) {
        char* slot = smem_raw + SBASE + (st & 1) * SH::SSLOT;
        const int64_t k0 = kbeg + (int64_t)st * KS;
#pragma unroll
        for (int a = 0; a < NS; ++a) {
            const bf16_t* S = (a ? Slo : Shi) + k0 * LP;
#pragma unroll
            for (int t = 0; t < SH::SPW; ++t) glds16(S + soff[t], slot + a * SH::SIMG + (t * 8 + w) * SImg::PITCH);
        }
    };
    auto asrc = [&](int d, int t) {
        const int64_t k0 = kbeg + (int64_t)d * 2 * KS;
        const bool tail = k0 + 2 * KS > arows;
        const bf16_t* src = A + k0 + aoff[t];
        if (tail && k0 + arow[t] + 8 > arows) src = A + (arows - 8 - arow[t]) + aoff[t];
        return src;
    };
    auto issueA = [&](int d) {
        char* slot = smem_raw + (d & 1) * ASLOT;
#pragma unroll
        for (int t = 0; t < APW2; ++t) glds16<(KN & 1) ? 2 : 0>(asrc(d, t), slot + (t * 8 + w) * 1024);
    };
    // KN bit 2 (IL): the step's LDS-DMA goes out one piece per column group inside the MFMA loop
    // instead of as a burst of NS SPW + APW2 right after the barrier (the same issue order, so the
    // waits count the same).  Piece i < NS SPW: S(st + 1) image i / SPW, piece i % SPW; the next APW2:
    // the A slot's pieces.
    constexpr bool IL = (KN & 4) != 0;
    constexpr int NSP = NS * SH::SPW;
    static_assert(!IL || NSP + APW2 <= G, "interleaved DMA: one piece per column group");
    auto issueS_piece = [&](int st, int i) {
        char* slot = smem_raw + SBASE + (st & 1) * SH::SSLOT;
        const int a = i / SH::SPW, t = i % SH::SPW;
        const bf16_t* S = (a ? Slo : Shi) + (kbeg + (int64_t)st * KS) * LP;
        glds16(S + soff[t], slot + a * SH::SIMG + (t * 8 + w) * SImg::PITCH);
    };
    auto issueA_piece = [&](int d, int t) {
        glds16<(KN & 1) ? 2 : 0>(asrc(d, t), smem_raw + (d & 1) * ASLOT + (t * 8 + w) * 1024);
    };
    // AR: A(d + 1) is ds_written at step 2d from registers loaded at step 2d - 2 (one A buffer: the
    // write of A(d + 1) precedes the load of A(d + 2) in the same step); see wproj3_kernel.
    i32x4 areg[APW2];
    auto loadA = [&](int d) {
#pragma unroll
        for (int t = 0; t < APW2; ++t) {
            if constexpr ((KN & 1) != 0)
                asm volatile("global_load_dwordx4 %0, %1, off nt" : "=v"(areg[t]) : "v"(asrc(d, t)) : "memory");
            else
                asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(areg[t]) : "v"(asrc(d, t)) : "memory");
        }
    };
    auto writeA = [&](int d) {
        const uint32_t slot = lds_addr(smem_raw) + (uint32_t)((d & 1) * ASLOT) + 16 * lane;
#pragma unroll
        for (int t = 0; t < APW2; ++t)
            asm volatile("ds_write_b128 %0, %1" ::"v"(slot + (uint32_t)((t * 8 + w) * 1024)), "v"(areg[t]) : "memory");
    };

    const int colS = wc * G * 16 + 4 * p;
    const int k1 = 8 * h + q, k2 = k1 + 4;
    const uint32_t lS1 = SImg::off(k1) + 2 * colS, lS2 = SImg::off(k2) + 2 * colS;
    const int sw = (r >> 1) & 7;
    const uint32_t lA0 = (wr * 64 + r) * 128 + 16 * (h ^ sw), lA1 = (wr * 64 + r) * 128 + 16 * ((4 + h) ^ sw);

    f32x4 acc[RT][G];
#pragma unroll
    for (int t = 0; t < RT; ++t)
#pragma unroll
        for (int g = 0; g < G; ++g) acc[t][g] = f32x4{0.f, 0.f, 0.f, 0.f};

    if ((KN & 2) && w >= 4) __builtin_amdgcn_s_setprio(1);
    if (nsteps > 0) {
        issueS(0);
        issueA(0);
        if (AR && 1 < nd) loadA(1);
    }
    const uint32_t lds0 = lds_addr(smem_raw);
    for (int st = 0; st < nsteps; ++st) {
        const int d = st >> 1, hs = st & 1;
        // step 2d needs A(d) and S(2d) (AR: and the registers of A(d + 1)): nothing younger is in
        // flight; step 2d + 1 needs S(2d + 1), issued before A(d + 1) (AR: A(d + 2)) in step 2d
        if (hs == 0 || d + 1 + (AR ? 1 : 0) >= nd) wait_vm<0>();
        else wait_vm<SH::APW * 0 + APW2>();
        __builtin_amdgcn_s_barrier();
        if constexpr (AR) {
            if (hs == 0 && d + 1 < nd) writeA(d + 1);
            if (st + 1 < nsteps) issueS(st + 1);
            if (hs == 0 && d + 2 < nd) loadA(d + 2);
        } else if constexpr (!IL) {
            if (st + 1 < nsteps) issueS(st + 1);
            if (hs == 0 && d + 1 < nd) issueA(d + 1);
        }
        const bool il_s = st + 1 < nsteps, il_a = hs == 0 && d + 1 < nd;
        const uint32_t sS = lds0 + SBASE + (uint32_t)((st & 1) * SH::SSLOT);
        const uint32_t sA = lds0 + (uint32_t)((d & 1) * ASLOT);
        const uint32_t bS1 = sS + lS1, bS2 = sS + lS2, bA = sA + (hs ? lA1 : lA0);
        auto wait_b = [&](i32x2* b) {
            if (SPLIT) wait_lgkm0(b[0], b[1], b[2], b[3]);
            else wait_lgkm0(b[0], b[1]);
        };
        i32x4 a4[RT];
        bf16x8_t af[RT];
        auto aread = [&](auto tc) {
            constexpr int t = decltype(tc)::value;
            a4[t] = read128_o<2048 * t>(bA);
        };
        static_for<RT>(aread);
        auto bread = [&](auto gc, i32x2* b) {
            constexpr int g = decltype(gc)::value;
            b[0] = tr_read_o<32 * g>(bS1);
            b[1] = tr_read_o<32 * g>(bS2);
            if constexpr (SPLIT) {
                b[2] = tr_read_o<SH::SIMG + 32 * g>(bS1);
                b[3] = tr_read_o<SH::SIMG + 32 * g>(bS2);
            }
        };
        i32x2 bb[2][4];
        bread(std::integral_constant<int, 0>{}, bb[0]);
        wait_b(bb[0]);
#pragma unroll
        for (int t = 0; t < RT; ++t) {
            wait_lgkm0(a4[t]);
            af[t] = __builtin_bit_cast(bf16x8_t, a4[t]);
        }
        auto gstep = [&](auto gc) {
            constexpr int g = decltype(gc)::value;
            if constexpr (g + 1 < G) bread(std::integral_constant<int, g + 1>{}, bb[(g + 1) & 1]);
            if constexpr (IL && !AR) {
                if constexpr (g < NSP) {
                    if (il_s) issueS_piece(st + 1, g);
                } else if constexpr (g < NSP + APW2) {
                    if (il_a) issueA_piece(d + 1, g - NSP);
                }
            }
            __builtin_amdgcn_sched_barrier(0);
            const i32x2* b = bb[g & 1];
            const bf16x8_t bh = join2(b[0], b[1]);
#pragma unroll
            for (int t = 0; t < RT; ++t) acc[t][g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[t], bh, acc[t][g], 0, 0, 0);
            if constexpr (SPLIT) {
                const bf16x8_t bl = join2(b[2], b[3]);
#pragma unroll
                for (int t = 0; t < RT; ++t) acc[t][g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[t], bl, acc[t][g], 0, 0, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (g + 1 < G) wait_b(bb[(g + 1) & 1]);
        };
        static_for<G>(gstep);
    }

    float* dst = out + (int64_t)sp * slab_stride;
#pragma unroll
    for (int t = 0; t < RT; ++t)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int64_t row = row0 + wr * 64 + 16 * t + 4 * h + j;
            if (row < rows_out) {
#pragma unroll
                for (int g = 0; g < G; ++g) dst[row * LP + wc * G * 16 + 16 * g + r] = acc[t][g][j];
            }
        }
}

// v3 TN for e4m3 A at LP = 256 (and LP = 512 as two column halves): FOUR 32-deep k-steps per A
// slot, so every A column contributes one full 128-B line per slot -- the e4m3 TN of wproj2 read
// 32-B column runs per k-step, which the fabric fetched about 4x over (C5: 4.3-4.5 GB per launch
// against 1.07 GB of A, profiles/r03_v1_c5_traffic.json).  A slot: [WI j][128 i] bytes, row j's
// 16-B unit u (rows 16 u .. 16 u + 15) at unit u ^ ((j >> 1) & 7); a lane's step-hs fragment is the
// 8 bytes of k 32 hs + 8 h .. + 7 of its column (ds_read_b64), widened to bf16 exactly.  S (the
// bf16 hi / lo panels) keeps v3's 32-step row images, with a row pitch s_pitch (512 for a half of
// an LP = 512 panel) and the output pitch o_pitch.  K chunks are multiples of 128 rows.
// Ring: A 2 slots x 32 KiB, S 2 slots (hi + lo) x 33 KiB.  A(d + 1) is issued in step 4 d + 1 behind
// S(4 d + 2), so step 4 d + 2 waits for all but it and step 4 d + 3 for everything.
template <int OFF>
__device__ __forceinline__ i32x2 read64_o(uint32_t a) {
    i32x2 v;
    asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(v) : "v"(a), "i"(OFF));
    return v;
}

template <bool SPLIT>
__global__ __launch_bounds__(512) void wproj3tn4_kernel(const uint8_t* __restrict__ A, int64_t lda, int64_t rows_out,
                                                        int64_t K, int64_t arows, const bf16_t* __restrict__ Shi,
                                                        const bf16_t* __restrict__ Slo, float* __restrict__ out,
                                                        int64_t slab_stride, int64_t kchunk, int nrowblk, int s_pitch,
                                                        int o_pitch, int halves) {
    constexpr int LP = 256;
    typedef W3Shape<LP, false, SPLIT, 1> SH;
    typedef typename SH::SImg SImg;
    constexpr int WR = SH::WR, G = SH::G, WI = SH::WI, NS = SH::NS;
    constexpr int ASLOT = WI * 128, APW2 = ASLOT / 1024 / 8;
    constexpr int SBASE = 2 * ASLOT;
    extern __shared__ __attribute__((aligned(1024))) char smem_raw[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r = lane & 15, h = lane >> 4, q = r >> 2, p = r & 3;
    const int wr = w % WR, wc = w / WR;
    const int bid2 = xcd_remap(blockIdx.x, gridDim.x);  // halves: as wproj2_kernel
    const int hf = bid2 % halves, bid = bid2 / halves;
    if (hf) {
        Shi += 256 * hf;
        if (Slo) Slo += 256 * hf;
        out += 256 * hf;
    }
    const int rb = bid % nrowblk, sp = bid / nrowblk;
    const int64_t row0 = (int64_t)rb * WI;
    const int64_t kbeg = (int64_t)sp * kchunk;
    const int64_t kend = (kbeg + kchunk < K) ? kbeg + kchunk : K;
    const int nsteps = (int)((kend - kbeg + KS - 1) / KS);
    const int nd = (nsteps + 3) / 4;

    int32_t soff[SH::SPW];
#pragma unroll
    for (int t = 0; t < SH::SPW; ++t) {
        constexpr int LPR = 64 / SImg::RP;
        const int pc = t * 8 + w;
        soff[t] = SImg::row_of(pc, lane / LPR) * s_pitch + 8 * (lane % LPR);
    }
    int64_t aoff[APW2];
    int arow[APW2];
#pragma unroll
    for (int t = 0; t < APW2; ++t) {
        const int u = (t * 8 + w) * 64 + lane, j = u >> 3, pu = u & 7;
        int64_t jc = row0 + j;
        jc = jc < rows_out ? jc : rows_out - 1;
        const int i = 16 * (pu ^ ((j >> 1) & 7));
        aoff[t] = jc * lda + i;
        arow[t] = i;
    }
    auto issueS = [&](int st) {
        char* slot = smem_raw + SBASE + (st & 1) * SH::SSLOT;
        const int64_t k0 = kbeg + (int64_t)st * KS;
#pragma unroll
        for (int a = 0; a < NS; ++a) {
            const bf16_t* S = (a ? Slo : Shi) + k0 * s_pitch;
#pragma unroll
            for (int t = 0; t < SH::SPW; ++t) glds16(S + soff[t], slot + a * SH::SIMG + (t * 8 + w) * SImg::PITCH);
        }
    };
    auto issueA = [&](int d) {
        char* slot = smem_raw + (d & 1) * ASLOT;
        const int64_t k0 = kbeg + (int64_t)d * 4 * KS;
        const bool tail = k0 + 4 * KS > arows;
#pragma unroll
        for (int t = 0; t < APW2; ++t) {
            const uint8_t* src = A + k0 + aoff[t];
            if (tail && k0 + arow[t] + 16 > arows) src = A + (arows - 16 - arow[t]) + aoff[t];
            glds16(src, slot + (t * 8 + w) * 1024);
        }
    };

    const int colS = wc * G * 16 + 4 * p;
    const int k1 = 8 * h + q, k2 = k1 + 4;
    const uint32_t lS1 = SImg::off(k1) + 2 * colS, lS2 = SImg::off(k2) + 2 * colS;
    const int sw = (r >> 1) & 7;
    uint32_t lA[4];
#pragma unroll
    for (int hs = 0; hs < 4; ++hs) lA[hs] = (wr * 64 + r) * 128 + 16 * ((2 * hs + (h >> 1)) ^ sw) + 8 * (h & 1);

    f32x4 acc[RT][G];
#pragma unroll
    for (int t = 0; t < RT; ++t)
#pragma unroll
        for (int g = 0; g < G; ++g) acc[t][g] = f32x4{0.f, 0.f, 0.f, 0.f};

    if (nsteps > 0) {
        issueA(0);
        issueS(0);
    }
    const uint32_t lds0 = lds_addr(smem_raw);
    for (int st = 0; st < nsteps; ++st) {
        const int d = st >> 2, hs = st & 3;
        if (hs == 2 && d + 1 < nd) wait_vm<APW2>();
        else wait_vm<0>();
        __builtin_amdgcn_s_barrier();
        if (st + 1 < nsteps) issueS(st + 1);
        if (hs == 1 && d + 1 < nd) issueA(d + 1);
        const uint32_t sS = lds0 + SBASE + (uint32_t)((st & 1) * SH::SSLOT);
        const uint32_t sA = lds0 + (uint32_t)((d & 1) * ASLOT);
        const uint32_t bS1 = sS + lS1, bS2 = sS + lS2;
        const uint32_t bA = sA + (hs == 0 ? lA[0] : (hs == 1 ? lA[1] : (hs == 2 ? lA[2] : lA[3])));
        auto wait_b = [&](i32x2* b) {
            if (SPLIT) wait_lgkm0(b[0], b[1], b[2], b[3]);
            else wait_lgkm0(b[0], b[1]);
        };
        i32x2 a2[RT];
        bf16x8_t af[RT];
        auto aread = [&](auto tc) {
            constexpr int t = decltype(tc)::value;
            a2[t] = read64_o<2048 * t>(bA);
        };
        static_for<RT>(aread);
        auto bread = [&](auto gc, i32x2* b) {
            constexpr int g = decltype(gc)::value;
            b[0] = tr_read_o<32 * g>(bS1);
            b[1] = tr_read_o<32 * g>(bS2);
            if constexpr (SPLIT) {
                b[2] = tr_read_o<SH::SIMG + 32 * g>(bS1);
                b[3] = tr_read_o<SH::SIMG + 32 * g>(bS2);
            }
        };
        i32x2 bb[2][4];
        bread(std::integral_constant<int, 0>{}, bb[0]);
        wait_b(bb[0]);
#pragma unroll
        for (int t = 0; t < RT; ++t) {
            wait_lgkm0(a2[t]);
            af[t] = fp8x8_to_bf16x8(a2[t]);
        }
        auto gstep = [&](auto gc) {
            constexpr int g = decltype(gc)::value;
            if constexpr (g + 1 < G) bread(std::integral_constant<int, g + 1>{}, bb[(g + 1) & 1]);
            __builtin_amdgcn_sched_barrier(0);
            const i32x2* b = bb[g & 1];
            const bf16x8_t bh = join2(b[0], b[1]);
#pragma unroll
            for (int t = 0; t < RT; ++t) acc[t][g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[t], bh, acc[t][g], 0, 0, 0);
            if constexpr (SPLIT) {
                const bf16x8_t bl = join2(b[2], b[3]);
#pragma unroll
                for (int t = 0; t < RT; ++t) acc[t][g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[t], bl, acc[t][g], 0, 0, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (g + 1 < G) wait_b(bb[(g + 1) & 1]);
        };
        static_for<G>(gstep);
    }

    float* dst = out + (int64_t)sp * slab_stride;
#pragma unroll
    for (int t = 0; t < RT; ++t)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int64_t row = row0 + wr * 64 + 16 * t + 4 * h + j;
            if (row < rows_out) {
#pragma unroll
                for (int g = 0; g < G; ++g) dst[row * o_pitch + wc * G * 16 + 16 * g + r] = acc[t][g][j];
            }
        }
}

// v3 NN for e4m3 A (C5's NN products, LP = 512 as two 256-column halves).  The v2 e4m3 NN spent
// 114 VALU per 64 MFMA (the XOR-swizzled S and A addresses rebuilt per tile and step); here S uses
// v3's placed row images (per-lane bases + immediate tile offsets, as wproj3_kernel) and A keeps
// v2's [32 k][256 i] byte image with its conflict-free unit swizzle (unit c of row k at c ^ (k & 15))
// -- the tile index sits inside that XOR, so each lane keeps one base per 16-row tile (four VGPRs,
// fixed for the launch; one v_add each per step).  A lane's fragment is ds_read_b64_tr_b8 of k rows
// 8 h .. 8 h + 7 of its column, widened to bf16 exactly.  Rings: A NA x 8 KiB (read DA = NA - 1
// steps ahead), S 2 x (hi + lo) images.  Same k order and MFMA order as v2: bit-identical.
template <bool SPLIT, bool IL = false>
__global__ __launch_bounds__(512) void wproj3nn8_kernel(const uint8_t* __restrict__ A, int64_t lda, int64_t rows_out,
                                                        int64_t K, int64_t arows, const bf16_t* __restrict__ Shi,
                                                        const bf16_t* __restrict__ Slo, float* __restrict__ out,
                                                        int64_t slab_stride, int64_t kchunk, int nrowblk, int s_pitch,
                                                        int o_pitch, int halves) {
    constexpr int LP = 256;
    typedef W3Shape<LP, false, SPLIT, 1> SH;
    typedef typename SH::SImg SImg;
    constexpr int WR = SH::WR, G = SH::G, WI = SH::WI, NS = SH::NS;
    constexpr int AIMG = KS * WI;  // 8 KiB: one 1-KiB piece per wave
    static_assert(AIMG == 8 * 1024, "one A piece per wave");
    constexpr int NA0 = (163840 - 2 * SH::SSLOT) / AIMG;
    constexpr int NA = NA0 > 8 ? 8 : NA0, DA = NA - 1;
    constexpr int SBASE = NA * AIMG;
    extern __shared__ __attribute__((aligned(1024))) char smem_raw[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r = lane & 15, h = lane >> 4, q = r >> 2, p = r & 3;
    const int wr = w % WR, wc = w / WR;
    const int bid2 = xcd_remap(blockIdx.x, gridDim.x);  // halves: as wproj2_kernel
    const int hf = bid2 % halves, bid = bid2 / halves;
    if (hf) {
        Shi += 256 * hf;
        if (Slo) Slo += 256 * hf;
        out += 256 * hf;
    }
    const int rb = bid % nrowblk, sp = bid / nrowblk;
    const int64_t row0 = (int64_t)rb * WI;
    const int64_t kbeg = (int64_t)sp * kchunk;
    const int64_t kend = (kbeg + kchunk < K) ? kbeg + kchunk : K;
    const int nsteps = (int)((kend - kbeg + KS - 1) / KS);

    int32_t soff[SH::SPW];
#pragma unroll
    for (int t = 0; t < SH::SPW; ++t) {
        constexpr int LPR = 64 / SImg::RP;
        const int pc = t * 8 + w;
        soff[t] = SImg::row_of(pc, lane / LPR) * s_pitch + 8 * (lane % LPR);
    }
    // A piece w: LDS units u = 64 w + lane -> k row u / 16, unit cp = u % 16 holding source rows
    // row0 + 16 (cp ^ (k & 15)) .. + 15 of A column k0 + k
    const int ka = (w * 64 + lane) >> 4, cpa = lane & 15;
    int64_t ia = row0 + 16 * (cpa ^ (ka & 15));
    ia = (ia + 16 <= arows) ? ia : arows - 16;
    auto issueS = [&](int st) {
        char* slot = smem_raw + SBASE + (st & 1) * SH::SSLOT;
        const int64_t k0 = kbeg + (int64_t)st * KS;
#pragma unroll
        for (int a = 0; a < NS; ++a) {
            const bf16_t* S = (a ? Slo : Shi) + k0 * s_pitch;
#pragma unroll
            for (int t = 0; t < SH::SPW; ++t) glds16(S + soff[t], slot + a * SH::SIMG + (t * 8 + w) * SImg::PITCH);
        }
    };
    auto issueA = [&](int st) {
        int64_t kk = kbeg + (int64_t)st * KS + ka;
        kk = kk < K ? kk : K - 1;
        glds16<2>(A + kk * lda + ia, smem_raw + (st % NA) * AIMG + w * 1024);  // read once: non-temporal
    };

    const int colS = wc * G * 16 + 4 * p;
    const int k1 = 8 * h + q, k2 = k1 + 4;
    const uint32_t lS1 = SImg::off(k1) + 2 * colS, lS2 = SImg::off(k2) + 2 * colS;
    const int kr = 8 * h + (r >> 1);
    uint32_t lA[RT];
#pragma unroll
    for (int t = 0; t < RT; ++t) lA[t] = kr * WI + 16 * ((4 * wr + t) ^ (kr & 15)) + 8 * (r & 1);

    f32x4 acc[RT][G];
#pragma unroll
    for (int t = 0; t < RT; ++t)
#pragma unroll
        for (int g = 0; g < G; ++g) acc[t][g] = f32x4{0.f, 0.f, 0.f, 0.f};

    if (w >= 4) __builtin_amdgcn_s_setprio(1);
    // prologue: A(0 .. DA - 1) and S(0), in the order the steady-state wait counts
    for (int i = -DA; i < 0; ++i) {
        if (i == -1 && nsteps > 0) issueS(0);
        if (i + DA < nsteps) issueA(i + DA);
    }
    // IL (round 6, the engine's form): the step's LDS-DMA one piece per column group inside the MFMA
    // loop instead of a burst after the barrier, the same issue order (the waits count the same);
    // bit-identical, C5 17.16 -> 17.07 ms on one box.  (The e4m3 TN measured slower with it: its A
    // slot spans four steps, 1639 -> 1678 us.)
    constexpr int NSP = NS * SH::SPW;
    static_assert(!IL || NSP + 1 <= G, "interleaved DMA: one piece per column group");
    auto issueS_piece = [&](int st, int i) {
        char* slot = smem_raw + SBASE + (st & 1) * SH::SSLOT;
        const int a = i / SH::SPW, t = i % SH::SPW;
        const bf16_t* S = (a ? Slo : Shi) + (kbeg + (int64_t)st * KS) * s_pitch;
        glds16(S + soff[t], slot + a * SH::SIMG + (t * 8 + w) * SImg::PITCH);
    };
    const uint32_t lds0 = lds_addr(smem_raw);
    for (int st = 0; st < nsteps; ++st) {
        // S(st) and A(st) have landed once at most A(st - 1 + DA), issued behind S(st), is in flight
        if (st - 1 + DA < nsteps) wait_vm<1>();
        else wait_vm<0>();
        __builtin_amdgcn_s_barrier();
        if constexpr (!IL) {
            if (st + 1 < nsteps) issueS(st + 1);
            if (st + DA < nsteps) issueA(st + DA);
        }
        const bool il_s = st + 1 < nsteps, il_a = st + DA < nsteps;
        const uint32_t sS = lds0 + SBASE + (uint32_t)((st & 1) * SH::SSLOT);
        const uint32_t sA = lds0 + (uint32_t)((st % NA) * AIMG);
        const uint32_t bS1 = sS + lS1, bS2 = sS + lS2;
        auto wait_b = [&](i32x2* b) {
            if (SPLIT) wait_lgkm0(b[0], b[1], b[2], b[3]);
            else wait_lgkm0(b[0], b[1]);
        };
        i32x2 a2[RT];
        bf16x8_t af[RT];
#pragma unroll
        for (int t = 0; t < RT; ++t) a2[t] = tr8_read_a(sA + lA[t]);
        auto bread = [&](auto gc, i32x2* b) {
            constexpr int g = decltype(gc)::value;
            b[0] = tr_read_o<32 * g>(bS1);
            b[1] = tr_read_o<32 * g>(bS2);
            if constexpr (SPLIT) {
                b[2] = tr_read_o<SH::SIMG + 32 * g>(bS1);
                b[3] = tr_read_o<SH::SIMG + 32 * g>(bS2);
            }
        };
        i32x2 bb[2][4];
        bread(std::integral_constant<int, 0>{}, bb[0]);
        wait_b(bb[0]);
#pragma unroll
        for (int t = 0; t < RT; ++t) {
            wait_lgkm0(a2[t]);
            af[t] = fp8x8_to_bf16x8(a2[t]);
        }
        auto gstep = [&](auto gc) {
            constexpr int g = decltype(gc)::value;
            if constexpr (g + 1 < G) bread(std::integral_constant<int, g + 1>{}, bb[(g + 1) & 1]);
            if constexpr (IL) {
                if constexpr (g < NSP) {
                    if (il_s) issueS_piece(st + 1, g);
                } else if constexpr (g == NSP) {
                    if (il_a) issueA(st + DA);
                }
            }
            __builtin_amdgcn_sched_barrier(0);
            const i32x2* b = bb[g & 1];
            const bf16x8_t bh = join2(b[0], b[1]);
#pragma unroll
            for (int t = 0; t < RT; ++t) acc[t][g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[t], bh, acc[t][g], 0, 0, 0);
            if constexpr (SPLIT) {
                const bf16x8_t bl = join2(b[2], b[3]);
#pragma unroll
                for (int t = 0; t < RT; ++t) acc[t][g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[t], bl, acc[t][g], 0, 0, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (g + 1 < G) wait_b(bb[(g + 1) & 1]);
        };
        static_for<G>(gstep);
    }

    float* dst = out + (int64_t)sp * slab_stride;
#pragma unroll
    for (int t = 0; t < RT; ++t)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int64_t row = row0 + wr * 64 + 16 * t + 4 * h + j;
            if (row < rows_out) {
#pragma unroll
                for (int g = 0; g < G; ++g) dst[row * o_pitch + wc * G * 16 + 16 * g + r] = acc[t][g][j];
            }
        }
}

template <bool SPLIT>
constexpr size_t nn8_lds() {
    typedef W3Shape<256, false, SPLIT, 1> SH;
    constexpr int NA0 = (163840 - 2 * SH::SSLOT) / (KS * 256);
    return (size_t)(NA0 > 8 ? 8 : NA0) * KS * 256 + 2 * (size_t)SH::SSLOT;
}

// e4m3 NN through wproj3nn8_kernel: LP = 512 as two 256-column halves (merged: one launch)
template <bool SPLIT>
hipError_t wproj3nn8_go(const void* A, int64_t lda, int64_t m, int64_t n, const bf16_t* Shi, const bf16_t* Slo,
                        const WProjPlan& p, float* slabs, float* Out, hipStream_t s, hipEvent_t done) {
    constexpr size_t lds = nn8_lds<SPLIT>();
    static_assert(lds <= 163840, "NN8 LDS");
    const int64_t rows_out = m, K = n;
    float* o = p.splits == 1 ? Out : slabs;
    const int64_t stride = rows_out * 512;
    if (p.merge) {
        hipLaunchKernelGGL((wproj3nn8_kernel<SPLIT, true>), dim3(2 * p.blocks * p.splits), dim3(512), lds, s,
                           reinterpret_cast<const uint8_t*>(A), lda, rows_out, K, m, Shi, Slo, o, stride, p.chunk,
                           p.blocks, 512, 512, 2);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    } else {
        for (int hf = 0; hf < 2; ++hf) {
            hipLaunchKernelGGL((wproj3nn8_kernel<SPLIT, true>), dim3(p.blocks * p.splits), dim3(512), lds, s,
                               reinterpret_cast<const uint8_t*>(A), lda, rows_out, K, m, Shi + 256 * hf,
                               Slo ? Slo + 256 * hf : nullptr, o + 256 * hf, stride, p.chunk, p.blocks, 512, 512, 1);
            hipError_t e = hipGetLastError();
            if (e != hipSuccess) return e;
        }
    }
    hipError_t e = hipSuccess;
    if (done) e = hipEventRecord(done, s);
    if (e != hipSuccess || p.splits == 1) return e;
    return launch_sum_slabs<float>(slabs, stride, p.splits, stride, Out, s);
}

// e4m3 TN through wproj3tn4_kernel: LP = 256 in one dispatch, LP = 512 as two 256-column halves
// (S columns 256 hf .., pitch 512, into output columns 256 hf ..).
template <bool SPLIT>
hipError_t wproj3tn4_go(const void* A, int64_t lda, int64_t m, int64_t n, const bf16_t* Shi, const bf16_t* Slo, int LP,
                        const WProjPlan& p, float* slabs, float* Out, hipStream_t s, hipEvent_t done) {
    typedef W3Shape<256, false, SPLIT, 1> SH;
    constexpr size_t lds = 2 * (size_t)SH::WI * 128 + 2 * (size_t)SH::SSLOT;
    static_assert(lds <= 163840, "TN4 LDS");
    const int64_t rows_out = n, K = m;
    float* o = p.splits == 1 ? Out : slabs;
    const int64_t stride = rows_out * LP;
    if (LP == 512 && p.merge) {  // both halves in one launch (A read once, the twin from L2)
        hipLaunchKernelGGL((wproj3tn4_kernel<SPLIT>), dim3(2 * p.blocks * p.splits), dim3(512), lds, s,
                           reinterpret_cast<const uint8_t*>(A), lda, rows_out, K, m, Shi, Slo, o, stride, p.chunk,
                           p.blocks, LP, LP, 2);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    } else {
        for (int hf = 0; hf < LP / 256; ++hf) {
            hipLaunchKernelGGL((wproj3tn4_kernel<SPLIT>), dim3(p.blocks * p.splits), dim3(512), lds, s,
                               reinterpret_cast<const uint8_t*>(A), lda, rows_out, K, m, Shi + 256 * hf,
                               Slo ? Slo + 256 * hf : nullptr, o + 256 * hf, stride, p.chunk, p.blocks, LP, LP, 1);
            hipError_t e = hipGetLastError();
            if (e != hipSuccess) return e;
        }
    }
    hipError_t e = hipSuccess;
    if (done) e = hipEventRecord(done, s);
    if (e != hipSuccess || p.splits == 1) return e;
    return launch_sum_slabs<float>(slabs, stride, p.splits, stride, Out, s);
}

template <bool SPLIT>
hipError_t wproj3tn2_go(const void* A, int64_t lda, int64_t m, int64_t n, const bf16_t* Shi, const bf16_t* Slo,
                        const WProjPlan& p, float* slabs, float* Out, hipStream_t s, hipEvent_t done) {
    typedef W3Shape<256, false, SPLIT, 1> SH;
    constexpr size_t lds = 2 * (size_t)SH::WI * 128 + 2 * (size_t)SH::SSLOT;
    static_assert(lds <= 163840, "TN2 LDS");
    const int64_t rows_out = n, K = m;
    float* o = p.splits == 1 ? Out : slabs;
    const int64_t stride = rows_out * 256;
    auto go = [&](auto knc) {  // LDS-DMA A; register-staged A only for the lab (abl 16)
#ifdef RSVD_LAB
        if (p.abl & 16) {
            hipLaunchKernelGGL((wproj3tn2_kernel<SPLIT, decltype(knc)::value, true>), dim3(p.blocks * p.splits),
                               dim3(512), lds, s, reinterpret_cast<const bf16_t*>(A), lda, rows_out, K, m, Shi, Slo, o,
                               stride, p.chunk, p.blocks);
            return;
        }
#endif
        hipLaunchKernelGGL((wproj3tn2_kernel<SPLIT, decltype(knc)::value, false>), dim3(p.blocks * p.splits),
                           dim3(512), lds, s, reinterpret_cast<const bf16_t*>(A), lda, rows_out, K, m, Shi, Slo, o,
                           stride, p.chunk, p.blocks);
    };
#ifdef RSVD_LAB
    switch (p.kn < 0 ? 4 : p.kn) {  // KN 4 (interleaved DMA) in the engine; the others for the lab knob sweep
        case 0: go(std::integral_constant<int, 0>{}); break;
        case 1: go(std::integral_constant<int, 1>{}); break;
        case 2: go(std::integral_constant<int, 2>{}); break;
        case 3: go(std::integral_constant<int, 3>{}); break;
        default: go(std::integral_constant<int, 4>{}); break;
    }
#else
    go(std::integral_constant<int, 4>{});  // interleaved DMA (KN bit 2, round 6)
#endif
    hipError_t e = hipGetLastError();
    if (e == hipSuccess && done) e = hipEventRecord(done, s);
    if (e != hipSuccess || p.splits == 1) return e;
    return launch_sum_slabs<float>(slabs, stride, p.splits, stride, Out, s);
}

// bf16 TN at LP = 128 with separate A and S rings (C3: Z = A^T Q, 2^20 x 1024 A, K split 64 ways).
// The v2 double-step kernel it replaces stages A and S together in two 64-KiB stages, so one stage
// -- 32 KiB of A -- is in flight while the other computes, and every 64-k stage pays about one HBM
// latency (2.9 us per stage, 53 % of wave cycles in memory waits: 0.35 of HBM).  Here A has its
// own ring of NA slots of [256 j][64 i] (128-B lines, tn2's image), and S (hi / lo) a ring of NSS
// 32-step slots.  Every step issues S(st + SD) and HALF of A slot st / 2 + DA (SD = NSS - 1,
// DA = NA - 1), so the A stream goes out evenly and one counted wait serves both parities.  The S
// images are v2's [32 k][128] with the 16-B chunk XOR swizzle (no padding, so NA = 4 / NSS = 2
// fills exactly 160 KiB); the swizzle only moves the 32-B window of a column tile, so each of the
// G = 4 tiles gets its own per-lane base, fixed for the launch.  Wave tiles as v2's DS shape
// (4 x 2 waves, 64 rows x 64 columns each) with the same MFMA sequence per acc tile (k-step by
// k-step, hi then lo): bit-identical to the v2 kernel.
// Wait: at step st = 2d + hs, S(st) (issued at step st - SD) is younger than both halves of A(d)
// (steps 2d - 2DA, 2d - 2DA + 1; needs 2 DA - 1 > SD), and AH + (SD - 1)(S + AH) glds follow it.
template <int NA, int NSS>
struct Tn128Shape {
    static constexpr int NS_MAX = 2, SIMG = 32 * 128 * 2, ASLOT = 256 * 128;
    static constexpr size_t lds(int ns) { return (size_t)NA * ASLOT + (size_t)NSS * ns * SIMG; }
    static_assert(2 * (NA - 1) - 1 > NSS - 1, "A must be issued before S");
};

template <bool SPLIT, int NA, int NSS>
__global__ __launch_bounds__(512) void wproj3tn128_kernel(const bf16_t* __restrict__ A, int64_t lda, int64_t rows_out,
                                                          int64_t K, int64_t arows, const bf16_t* __restrict__ Shi,
                                                          const bf16_t* __restrict__ Slo, float* __restrict__ out,
                                                          int64_t slab_stride, int64_t kchunk, int nrowblk) {
    constexpr int LP = 128, WR = 4, G = 4, WI = 256, NS = SPLIT ? 2 : 1;
    constexpr int DA = NA - 1, SD = NSS - 1;
    typedef Tn128Shape<NA, NSS> SH;
    constexpr int SIMG = SH::SIMG, SSLOT = NS * SIMG, ASLOT = SH::ASLOT;
    constexpr int APW2 = ASLOT / 1024 / 8, AH = APW2 / 2;  // A glds per wave per slot / per half
    constexpr int SBASE = NA * ASLOT;
    constexpr int CNT = AH + (SD - 1) * (NS + AH);
    static_assert(SH::lds(NS) <= 163840, "TN128 LDS");
    extern __shared__ __attribute__((aligned(1024))) char smem_raw[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int r = lane & 15, h = lane >> 4, q = r >> 2, p = r & 3;
    const int wr = w % WR, wc = w / WR;
    const int bid = xcd_remap(blockIdx.x, gridDim.x);
    const int rb = bid % nrowblk, sp = bid / nrowblk;
    const int64_t row0 = (int64_t)rb * WI;
    const int64_t kbeg = (int64_t)sp * kchunk;
    const int64_t kend = (kbeg + kchunk < K) ? kbeg + kchunk : K;
    const int nsteps = (int)((kend - kbeg + KS - 1) / KS);
    const int nd = (nsteps + 1) / 2;

    // S: one glds per wave per image; lane's 16-B chunk cc of row srow holds source chunk cc ^ swz(srow)
    const int su = w * 64 + lane, srow = su >> 4;
    const int32_t soff = srow * LP + 8 * ((su & 15) ^ swz(srow));
    int64_t aoff[APW2];
    int arow[APW2];
#pragma unroll
    for (int t = 0; t < APW2; ++t) {
        const int u = (t * 8 + w) * 64 + lane, j = u >> 3, pu = u & 7;
        int64_t jc = row0 + j;
        jc = jc < rows_out ? jc : rows_out - 1;
        const int i = 8 * (pu ^ ((j >> 1) & 7));
        aoff[t] = jc * lda + i;
        arow[t] = i;
    }
    auto issueS = [&](int st) {
        char* slot = smem_raw + SBASE + (st % NSS) * SSLOT;
        const int64_t k0 = kbeg + (int64_t)st * KS;
        glds16(Shi + k0 * LP + soff, slot + w * 1024);
        if constexpr (SPLIT) glds16(Slo + k0 * LP + soff, slot + SIMG + w * 1024);
    };
    auto issueA = [&](int d, int half) {
        char* slot = smem_raw + (d % NA) * ASLOT;
        const int64_t k0 = kbeg + (int64_t)d * 2 * KS;
        const bool tail = k0 + 2 * KS > arows;
#pragma unroll
        for (int tt = 0; tt < AH; ++tt) {
            const int t = half * AH + tt;
            const bf16_t* src = A + k0 + aoff[t];
            if (tail && k0 + arow[t] + 8 > arows) src = A + (arows - 8 - arow[t]) + aoff[t];
            glds16(src, slot + (t * 8 + w) * 1024);
        }
    };
    // the issue rule of step st (also run over the virtual steps of the prologue)
    auto issue = [&](int st) {
        if (st + SD >= 0 && st + SD < nsteps) issueS(st + SD);
        const int d = (st >> 1) + DA;  // (arithmetic shift: floor for the negative virtual steps)
        if (d >= 0 && d < nd) {
            if (st & 1) issueA(d, 1);
            else issueA(d, 0);
        }
    };

    // per-lane S read bases of the G column tiles (row k1; row k2 = k1 + 4 is +1024, lo is +SIMG)
    const int k1 = 8 * h + q;
    uint32_t lS[G];
#pragma unroll
    for (int g = 0; g < G; ++g) lS[g] = k1 * 256 + 16 * (((wc * 8 + 2 * g) ^ swz(k1)) + (p >> 1)) + 8 * (p & 1);
    const int sw = (r >> 1) & 7;
    const uint32_t lA0 = (wr * 64 + r) * 128 + 16 * (h ^ sw), lA1 = (wr * 64 + r) * 128 + 16 * ((4 + h) ^ sw);

    f32x4 acc[RT][G];
#pragma unroll
    for (int t = 0; t < RT; ++t)
#pragma unroll
        for (int g = 0; g < G; ++g) acc[t][g] = f32x4{0.f, 0.f, 0.f, 0.f};

    for (int st = -(2 * DA > SD ? 2 * DA : SD); st < 0; ++st) issue(st);
    const uint32_t lds0 = lds_addr(smem_raw);
    for (int st = 0; st < nsteps; ++st) {
        const int d = st >> 1, hs = st & 1;
        if (st + 2 * DA + SD < nsteps) wait_vm<CNT>();
        else wait_vm<0>();
        __builtin_amdgcn_s_barrier();
        issue(st);
        const uint32_t sS = lds0 + SBASE + (uint32_t)((st % NSS) * SSLOT);
        const uint32_t sA = lds0 + (uint32_t)((d % NA) * ASLOT);
        const uint32_t bA = sA + (hs ? lA1 : lA0);
        auto wait_b = [&](i32x2* b) {
            if (SPLIT) wait_lgkm0(b[0], b[1], b[2], b[3]);
            else wait_lgkm0(b[0], b[1]);
        };
        i32x4 a4[RT];
        bf16x8_t af[RT];
        auto aread = [&](auto tc) {
            constexpr int t = decltype(tc)::value;
            a4[t] = read128_o<2048 * t>(bA);
        };
        static_for<RT>(aread);
        auto bread = [&](auto gc, i32x2* b) {
            constexpr int g = decltype(gc)::value;
            const uint32_t bs = sS + lS[g];
            b[0] = tr_read_o<0>(bs);
            b[1] = tr_read_o<1024>(bs);
            if constexpr (SPLIT) {
                b[2] = tr_read_o<SIMG>(bs);
                b[3] = tr_read_o<SIMG + 1024>(bs);
            }
        };
        i32x2 bb[2][4];
        bread(std::integral_constant<int, 0>{}, bb[0]);
        wait_b(bb[0]);
#pragma unroll
        for (int t = 0; t < RT; ++t) {
            wait_lgkm0(a4[t]);
            af[t] = __builtin_bit_cast(bf16x8_t, a4[t]);
        }
        auto gstep = [&](auto gc) {
            constexpr int g = decltype(gc)::value;
            if constexpr (g + 1 < G) bread(std::integral_constant<int, g + 1>{}, bb[(g + 1) & 1]);
            __builtin_amdgcn_sched_barrier(0);
            const i32x2* b = bb[g & 1];
            const bf16x8_t bh = join2(b[0], b[1]);
#pragma unroll
            for (int t = 0; t < RT; ++t) acc[t][g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[t], bh, acc[t][g], 0, 0, 0);
            if constexpr (SPLIT) {
                const bf16x8_t bl = join2(b[2], b[3]);
#pragma unroll
                for (int t = 0; t < RT; ++t) acc[t][g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[t], bl, acc[t][g], 0, 0, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (g + 1 < G) wait_b(bb[(g + 1) & 1]);
        };
        static_for<G>(gstep);
    }

    float* dst = out + (int64_t)sp * slab_stride;
#pragma unroll
    for (int t = 0; t < RT; ++t)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int64_t row = row0 + wr * 64 + 16 * t + 4 * h + j;
            if (row < rows_out) {
#pragma unroll
                for (int g = 0; g < G; ++g) dst[row * LP + wc * G * 16 + 16 * g + r] = acc[t][g][j];
            }
        }
}

// ring depths (A slots, S slots): 4 / 2 in the engine; 3 / 3 in the lab only (p.tn3 = 2, RSVD_LAB builds)
template <bool SPLIT>
hipError_t wproj3tn128_go(const void* A, int64_t lda, int64_t m, int64_t n, const bf16_t* Shi, const bf16_t* Slo,
                          const WProjPlan& p, float* slabs, float* Out, hipStream_t s, hipEvent_t done) {
    constexpr int NS = SPLIT ? 2 : 1;
    const int64_t rows_out = n, K = m;
    float* o = p.splits == 1 ? Out : slabs;
    const int64_t stride = rows_out * 128;
#ifdef RSVD_LAB
    if (p.tn3 == 2)
        hipLaunchKernelGGL((wproj3tn128_kernel<SPLIT, 3, 3>), dim3(p.blocks * p.splits), dim3(512),
                           (Tn128Shape<3, 3>::lds(NS)), s, reinterpret_cast<const bf16_t*>(A), lda, rows_out, K, m, Shi,
                           Slo, o, stride, p.chunk, p.blocks);
    else
#endif
        hipLaunchKernelGGL((wproj3tn128_kernel<SPLIT, 4, 2>), dim3(p.blocks * p.splits), dim3(512),
                           (Tn128Shape<4, 2>::lds(NS)), s, reinterpret_cast<const bf16_t*>(A), lda, rows_out, K, m, Shi,
                           Slo, o, stride, p.chunk, p.blocks);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess && done) e = hipEventRecord(done, s);
    if (e != hipSuccess || p.splits == 1) return e;
    return launch_sum_slabs<float>(slabs, stride, p.splits, stride, Out, s);
}


template <bool FP8, bool NN, int LP, bool SPLIT, bool DS = false, bool S8 = false, bool SC = false>
hipError_t wproj2_go(const void* A, int64_t lda, int64_t m, int64_t n, const bf16_t* Shi, const bf16_t* Slo,
                     const WProjPlan& p, float* slabs, float* Out, hipStream_t s, hipEvent_t done) {
    typedef W2Shape<LP, SPLIT, FP8, DS, S8, SC> SH;
    const int64_t rows_out = NN ? m : n, K = NN ? n : m;
    float* o = p.splits == 1 ? Out : slabs;
    const int64_t stride = rows_out * LP;
    // NN streams A in whole columns: non-temporal A (and the static priority) measured -9..-11 % on
    // the C3 / C4 / C5 NN launches; TN's short column runs need the L2 to keep the second half of
    // each line for the next k-step (non-temporal: +4..13 %), so TN keeps the default policy
    // (profiles/r02_wide_lab_knobs.txt).
    constexpr int KN = NN ? 3 : 0;
    hipLaunchKernelGGL((wproj2_kernel<FP8, NN, LP, SPLIT, DS, KN, S8, SC>), dim3(p.blocks * p.splits), dim3(512), SH::LDS,
                       s, A, lda, rows_out, K, m, Shi, Slo, o, stride, p.chunk, p.blocks, LP, LP, 1);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess && done) e = hipEventRecord(done, s);
    if (e != hipSuccess || p.splits == 1) return e;
    return launch_sum_slabs<float>(slabs, stride, p.splits, stride, Out, s);
}

// LP = 512 as two LP = 256 column halves (WProjPlan::half).  At LP = 512 the v2 tile is 128 output
// rows x 512 columns, so every workgroup re-reads 16x (NN) / 16x (TN) more S bytes from L2 than A
// bytes (C5 TN: 16 GB of S per launch against 1.07 GB of A, and the L2 pressure evicted A's line
// halves before the next k-step used them: 4x A traffic from HBM).  Each half runs the LP = 256
// tile (256 rows x 256 columns: S 2x A per k-step) on its 256 columns of S (pitch 512) into its
// 256 columns of the output / slabs (pitch 512).  Same per-element arithmetic: bit-identical.
template <bool FP8, bool NN, bool SPLIT, bool S8 = false, bool SC = false>
hipError_t wproj2_half_go(const void* A, int64_t lda, int64_t m, int64_t n, const bf16_t* Shi, const bf16_t* Slo,
                          const WProjPlan& p, float* slabs, float* Out, hipStream_t s, hipEvent_t done) {
    typedef W2Shape<256, SPLIT, FP8, false, S8, SC> SH;
    const int64_t rows_out = NN ? m : n, K = NN ? n : m;
    float* o = p.splits == 1 ? Out : slabs;
    const int64_t stride = rows_out * 512;
    constexpr int KN = NN ? 3 : 0;
    if (p.merge) {  // both halves in one launch: neighbouring blocks share the A tile through the L2
        hipLaunchKernelGGL((wproj2_kernel<FP8, NN, 256, SPLIT, false, KN, S8, SC>), dim3(2 * p.blocks * p.splits),
                           dim3(512), SH::LDS, s, A, lda, rows_out, K, m, Shi, Slo, o, stride, p.chunk, p.blocks, 512,
                           512, 2);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    } else {
        for (int hf = 0; hf < 2; ++hf) {
            // S column offset: 256 bf16 elements, or 256 bytes of an e4m3 panel (S8)
            const bf16_t* sh = S8 ? reinterpret_cast<const bf16_t*>(reinterpret_cast<const uint8_t*>(Shi) + 256 * hf)
                                  : Shi + 256 * hf;
            const bf16_t* sl = Slo ? Slo + 256 * hf : nullptr;
            hipLaunchKernelGGL((wproj2_kernel<FP8, NN, 256, SPLIT, false, KN, S8, SC>), dim3(p.blocks * p.splits),
                               dim3(512), SH::LDS, s, A, lda, rows_out, K, m, sh, sl, o + 256 * hf, stride, p.chunk,
                               p.blocks, 512, 512, 1);
            hipError_t e = hipGetLastError();
            if (e != hipSuccess) return e;
        }
    }
    hipError_t e = hipSuccess;
    if (done) e = hipEventRecord(done, s);
    if (e != hipSuccess || p.splits == 1) return e;
    return launch_sum_slabs<float>(slabs, stride, p.splits, stride, Out, s);
}

template <bool FP8, bool NN, int LP, bool SPLIT>
hipError_t wproj_go(const void* A, int64_t lda, int64_t m, int64_t n, const bf16_t* Shi, const bf16_t* Slo,
                    const WProjPlan& p, float* slabs, float* Out, hipStream_t s, hipEvent_t done) {
    const int64_t rows_out = NN ? m : n, K = NN ? n : m;
    float* o = p.splits == 1 ? Out : slabs;
    const int64_t stride = rows_out * LP;
    const int esz = FP8 ? 1 : 2;
    const int vec_ok = ((lda * esz) % 16 == 0) && ((reinterpret_cast<uintptr_t>(A) & 15) == 0);
    hipLaunchKernelGGL((wproj_kernel<FP8, NN, LP, SPLIT>), dim3(p.blocks * p.splits), dim3(256),
                       (wproj_lds<FP8, NN, LP, SPLIT>()), s, A, lda, rows_out, K, Shi, Slo, o, stride, p.chunk,
                       p.blocks, vec_ok);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess && done) e = hipEventRecord(done, s);
    if (e != hipSuccess || p.splits == 1) return e;
    return launch_sum_slabs<float>(slabs, stride, p.splits, stride, Out, s);
}

template <int LP>
hipError_t wproj_lp(int nn, int fp8, const void* A, int64_t lda, int64_t m, int64_t n, const bf16_t* Shi,
                    const bf16_t* Slo, const WProjPlan& p, float* slabs, float* Out, hipStream_t s, hipEvent_t d) {
    const bool split = Slo != nullptr;
    if constexpr (LP == 128) {
        // the v3 NN at LP = 128 (WI = 512 rows, A 3 / S 2 slots) for the hi / lo products: C3 5.40 ->
        // 5.35 ms (gpurun_out r6d, bit-identical); the single-pass sketch measured 468 -> 473 us on it
        // and keeps v2
        if (p.v2 && nn && !fp8 && p.nn3 && split)
            return wproj3_go<true, 128, true, 1>(A, lda, m, n, Shi, Slo, p, slabs, Out, s, d);
        if (p.v2 && p.ds && !nn && !fp8 && p.tn3)
            return split ? wproj3tn128_go<true>(A, lda, m, n, Shi, Slo, p, slabs, Out, s, d)
                         : wproj3tn128_go<false>(A, lda, m, n, Shi, Slo, p, slabs, Out, s, d);
        if (p.v2 && p.ds && !nn && !fp8)
            return split ? wproj2_go<false, false, 128, true, true>(A, lda, m, n, Shi, Slo, p, slabs, Out, s, d)
                         : wproj2_go<false, false, 128, false, true>(A, lda, m, n, Shi, Slo, p, slabs, Out, s, d);
    }
    if constexpr (LP == 256 || LP == 512) {
        if (p.v2 && p.v3 && !fp8) {
#define GO3(SD)                                                                                         \
    {                                                                                                   \
        if (nn) return split ? wproj3_go<true, LP, true, SD>(A, lda, m, n, Shi, Slo, p, slabs, Out, s, d) \
                             : wproj3_go<true, LP, false, SD>(A, lda, m, n, Shi, Slo, p, slabs, Out, s, d); \
        return split ? wproj3_go<false, LP, true, SD>(A, lda, m, n, Shi, Slo, p, slabs, Out, s, d)        \
                     : wproj3_go<false, LP, false, SD>(A, lda, m, n, Shi, Slo, p, slabs, Out, s, d);      \
    }
#ifdef RSVD_LAB
            if constexpr (LP == 256) {  // lab ablations of the C4 NN2 / TN2 kernels
                if (p.abl && split) {
#define AB(X) \
    case X: return nn ? wproj3_go<true, 256, true, 1, X>(A, lda, m, n, Shi, Slo, p, slabs, Out, s, d) \
                      : wproj3_go<false, 256, true, 1, X>(A, lda, m, n, Shi, Slo, p, slabs, Out, s, d);
                    switch (p.abl) { AB(1) AB(2) AB(3) AB(4) AB(5) AB(6) AB(7) default: break; }
#undef AB
                }
            }
#endif
            if constexpr (LP == 256) {
                // (round 6: the S panel two steps ahead instead of one -- sketch 1977 -> 2003 us at C4;
                // profiles/r06_deadends.txt 22 -- so every v3 product keeps SD = 1)
                if (!nn && p.tn2)
                    return split ? wproj3tn2_go<true>(A, lda, m, n, Shi, Slo, p, slabs, Out, s, d)
                                 : wproj3tn2_go<false>(A, lda, m, n, Shi, Slo, p, slabs, Out, s, d);
            }
            GO3(1);
#undef GO3
        }
    }
    if constexpr (LP == 256 || LP == 512) {
        if (p.tn4 && fp8 && !nn)
            return split ? wproj3tn4_go<true>(A, lda, m, n, Shi, Slo, LP, p, slabs, Out, s, d)
                         : wproj3tn4_go<false>(A, lda, m, n, Shi, Slo, LP, p, slabs, Out, s, d);
    }
    if constexpr (LP == 512) {
        if (p.v2 && p.half && fp8) {
            if (nn && p.nn8)
                return split ? wproj3nn8_go<true>(A, lda, m, n, Shi, Slo, p, slabs, Out, s, d)
                             : wproj3nn8_go<false>(A, lda, m, n, Shi, Slo, p, slabs, Out, s, d);
            // (RSVD_NN8=0, the round-4 kernel; every v2 e4m3 TN takes wproj3tn4 above)
            return split ? wproj2_half_go<true, true, true>(A, lda, m, n, Shi, Slo, p, slabs, Out, s, d)
                         : wproj2_half_go<true, true, false>(A, lda, m, n, Shi, Slo, p, slabs, Out, s, d);
        }
    }
    if constexpr (LP >= 128) {
        if (p.v2) {
#define GO2(F)                                                                                   \
    {                                                                                            \
        if (nn) return split ? wproj2_go<F, true, LP, true>(A, lda, m, n, Shi, Slo, p, slabs, Out, s, d) \
                             : wproj2_go<F, true, LP, false>(A, lda, m, n, Shi, Slo, p, slabs, Out, s, d); \
        return split ? wproj2_go<F, false, LP, true>(A, lda, m, n, Shi, Slo, p, slabs, Out, s, d)        \
                     : wproj2_go<F, false, LP, false>(A, lda, m, n, Shi, Slo, p, slabs, Out, s, d);      \
    }
            if (fp8) {  // (e4m3 at LP 256 / 512: the TN is wproj3tn4's, LP 512 runs as halves above)
                if constexpr (LP == 128) GO2(true);
                if constexpr (LP == 256) {
                    if (nn) return split ? wproj2_go<true, true, LP, true>(A, lda, m, n, Shi, Slo, p, slabs, Out, s, d)
                                         : wproj2_go<true, true, LP, false>(A, lda, m, n, Shi, Slo, p, slabs, Out, s, d);
                }
                return hipErrorInvalidValue;
            }
            if constexpr (LP == 128) GO2(false);  // (bf16 at LP 256 / 512: the v3 kernels above)
            return hipErrorInvalidValue;
#undef GO2
        }
    }
#define GO(F, N, SP) return wproj_go<F, N, LP, SP>(A, lda, m, n, Shi, Slo, p, slabs, Out, s, d)
    if (fp8) {
        if (nn) { if (split) GO(true, true, true); GO(true, true, false); }
        if (split) GO(true, false, true);
        GO(true, false, false);
    }
    if (nn) { if (split) GO(false, true, true); GO(false, true, false); }
    if (split) GO(false, false, true);
    GO(false, false, false);
#undef GO
}

}  // namespace

bool wproj_supported_lp(int LP) {
    return LP == 16 || LP == 32 || LP == 64 || LP == 128 || LP == 256 || LP == 512;
}

int wproj_rows_per_block(int LP) { return LP <= 128 ? 256 : (LP == 256 ? 128 : 64); }

static int tn128_mode() {  // RSVD_TN128: 0 the v2 double-step LP = 128 TN, 1 rings 4 / 2 (default)
    static const int env = [] {
        const char* v = std::getenv("RSVD_TN128");
        const int x = v ? std::atoi(v) : 1;
        return x == 0 ? 0 : 1;
    }();
    return env;
}

static bool nn8_enabled() {  // RSVD_NN8=0 in the environment: the v2 e4m3 NN (A/B)
    static const int env = [] {
        const char* v = std::getenv("RSVD_NN8");
        return v ? std::atoi(v) : 1;
    }();
    return env != 0;
}

static bool nn3_128_enabled() {  // RSVD_NN3_128=0 in the environment: the v2 bf16 NN at LP = 128 (A/B)
    static const int env = [] {
        const char* v = std::getenv("RSVD_NN3_128");
        return v ? std::atoi(v) : 1;
    }();
    return env != 0;
}

WProjPlan plan_wproj(int64_t rows_out, int64_t K, int LP, bool v2, bool nn, bool fp8) {
    WProjPlan p;
    p.v2 = v2 && LP >= 128;
    p.v3 = p.v2 && !fp8 && (LP == 256 || LP == 512);
    p.tn2 = p.v3 && !nn && LP == 256;  // two k-steps per A slot: K chunks of whole 64-row pairs
    p.ds = p.v2 && LP == 128 && !nn && !fp8 && K % 64 == 0;  // double-step TN stages (whole 64-row K chunks)
    p.tn3 = p.ds ? tn128_mode() : 0;
    p.nn3 = p.v2 && LP == 128 && nn && !fp8 && nn3_128_enabled();
    p.half = p.v2 && fp8 && LP == 512;  // two LP = 256 column halves (wproj2_half_go)
    p.nn8 = p.half && nn && nn8_enabled();  // ... the e4m3 NN on wproj3nn8_kernel
    // e4m3 TN: four k-steps per A slot (wproj3tn4_kernel; K chunks of whole 128-row slots)
    p.tn4 = p.v2 && fp8 && !nn && (LP == 256 || LP == 512);
    const int WI = p.v2 ? (LP == 128 ? (p.ds ? 256 : 512) : ((LP == 256 || p.half) ? 256 : 128))
                        : wproj_rows_per_block(LP);
    p.blocks = (int)((rows_out + WI - 1) / WI);
    // LP = 512 e4m3 products as two 256-column halves in one launch (twin workgroups adjacent)
    p.merge = p.half || (p.tn4 && LP == 512);
    // one workgroup per CU (LDS ring / registers); merged halves: two workgroups per (row block, split)
    const int target = p.merge ? 128 : ((p.v2 || LP >= 512) ? 256 : 512);
    int64_t splits = (target + p.blocks - 1) / p.blocks;
    const int64_t max_by_work = K / (KS * 8);
    if (splits > max_by_work) splits = max_by_work;
    if (splits > 128) splits = 128;
    if (splits < 1) splits = 1;
    int64_t chunk = (K + splits - 1) / splits;
    const int kq = p.tn4 ? 4 * KS : ((p.ds || p.tn2) ? 2 * KS : KS);
    chunk = (chunk + kq - 1) / kq * kq;
    p.chunk = chunk;
    p.splits = (int)((K + chunk - 1) / chunk);
    return p;
}

bool wproj_s8_supported(const WProjPlan& p, int LP) { return p.v2 && (LP == 256 || LP == 512); }

hipError_t launch_wproj_s8(const void* A, int64_t lda, int64_t m, int64_t n, const fp8_t* S8, int LP, const WProjPlan& p,
                           float* slabs, float* Out, hipStream_t s, hipEvent_t done) {
    if (!wproj_s8_supported(p, LP)) return hipErrorInvalidValue;
    const bf16_t* S = reinterpret_cast<const bf16_t*>(S8);
    // the block-scaled K = 128 form when every stage is whole (else the K = 32 form)
    const bool sc = n % 128 == 0 && p.chunk % 128 == 0;
    if (sc) {
        if (LP == 256) return wproj2_go<true, true, 256, false, false, true, true>(A, lda, m, n, S, nullptr, p, slabs, Out, s, done);
        if (p.half) return wproj2_half_go<true, true, false, true, true>(A, lda, m, n, S, nullptr, p, slabs, Out, s, done);
    }
    if (LP == 256) return wproj2_go<true, true, 256, false, false, true>(A, lda, m, n, S, nullptr, p, slabs, Out, s, done);
    if (p.half) return wproj2_half_go<true, true, false, true>(A, lda, m, n, S, nullptr, p, slabs, Out, s, done);
    return wproj2_go<true, true, 512, false, false, true>(A, lda, m, n, S, nullptr, p, slabs, Out, s, done);
}

hipError_t launch_wproj(int nn, int a_fp8, const void* A, int64_t lda, int64_t m, int64_t n, const bf16_t* Shi,
                        const bf16_t* Slo, int LP, const WProjPlan& p, float* slabs, float* Out, hipStream_t s,
                        hipEvent_t done) {
    switch (LP) {
        case 16: return wproj_lp<16>(nn, a_fp8, A, lda, m, n, Shi, Slo, p, slabs, Out, s, done);
        case 32: return wproj_lp<32>(nn, a_fp8, A, lda, m, n, Shi, Slo, p, slabs, Out, s, done);
        case 64: return wproj_lp<64>(nn, a_fp8, A, lda, m, n, Shi, Slo, p, slabs, Out, s, done);
        case 128: return wproj_lp<128>(nn, a_fp8, A, lda, m, n, Shi, Slo, p, slabs, Out, s, done);
        case 256: return wproj_lp<256>(nn, a_fp8, A, lda, m, n, Shi, Slo, p, slabs, Out, s, done);
        case 512: return wproj_lp<512>(nn, a_fp8, A, lda, m, n, Shi, Slo, p, slabs, Out, s, done);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace rsvd
