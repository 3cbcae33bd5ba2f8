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

#include "common.hpp"
#include "kernels.hpp"
#include "wide.hpp"

namespace rsvd {

namespace {

typedef Mfma<double> MD;

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

__global__ void gram_reduce_kernel(const double* __restrict__ slabs, int nblk, int nchunk, int LP, int cross,
                                   double* __restrict__ G, const int* __restrict__ pred) {
    if (pred && *pred == 0) return;
    const int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
    if (e >= (int64_t)nblk * 1024) return;
    const int blk = (int)(e / 1024), loc = (int)(e % 1024);
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
    if (ra >= LP || cb >= LP) return;
    double s = 0.0;
    for (int c = 0; c < nchunk; ++c) s += slabs[((int64_t)c * nblk + blk) * 1024 + loc];
    G[(int64_t)ra * LP + cb] = s;
    if (!cross && a != b) G[(int64_t)cb * LP + ra] = s;
}

// ------------------------------------------------------------------------------------------------
// Cholesky + inverse, one workgroup of kCholThreads threads.  W (work) holds the Gram being
// reduced; R and Rinv are the outputs; the 16x16 inverse diagonal blocks stay in LDS.  Per 16-
// column block p: wave 0 factors the diagonal block in registers (lane j owns column j, pivots and
// rows broadcast with v_readlane: no workgroup barriers inside), all waves then form the strip
// R[p][p+1..] = D^-T W[p][p+1..] and the trailing update W -= R[p]^T R[p] on the fp64 MFMA
// (3 barriers per block).  R^-1 is assembled bottom-up by block rows (1 barrier per block).
constexpr int kCholThreads = 512;

// acc += X^T Y for 16x16 fp64 blocks X (ldx), Y (ldy) given row-major: acc[i][j] += sum_k X[k][i] Y[k][j]
__device__ __forceinline__ f64x4 mma_tn16(const double* X, int64_t ldx, const double* Y, int64_t ldy, f64x4 acc,
                                          int r, int h) {
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) acc = MD::mma(X[(4 * kk + h) * ldx + r], Y[(4 * kk + h) * ldy + r], acc);
    return acc;
}
// acc += X Y for 16x16 blocks: acc[i][j] += sum_k X[i][k] Y[k][j]
__device__ __forceinline__ f64x4 mma_nn16(const double* X, int64_t ldx, const double* Y, int64_t ldy, f64x4 acc,
                                          int r, int h) {
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) acc = MD::mma(X[r * ldx + 4 * kk + h], Y[(4 * kk + h) * ldy + r], acc);
    return acc;
}

__device__ __forceinline__ double readlane_d(double v, int lane) {
    const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
    const unsigned lo = __builtin_amdgcn_readlane((unsigned)u, lane);
    const unsigned hi = __builtin_amdgcn_readlane((unsigned)(u >> 32), lane);
    return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}

__global__ __launch_bounds__(kCholThreads) void chol_wide_kernel(const double* __restrict__ G, int l, int LP,
                                                                 double tol, double* __restrict__ W,
                                                                 double* __restrict__ R, double* __restrict__ Rinv,
                                                                 float* __restrict__ Rinv32, int* __restrict__ colflag,
                                                                 int* __restrict__ flag, const int* __restrict__ pred) {
    if (pred && *pred == 0) return;
    extern __shared__ __attribute__((aligned(16))) char smem_raw[];
    const int np = LP / 16;
    double* Dinv = reinterpret_cast<double*>(smem_raw);  // [np][16][16]
    double* d0 = Dinv + np * 256;                        // [LP] original diagonal of G
    double* Tsc = d0 + LP;                               // [waves][16][16] per-wave scratch
    int* bad = reinterpret_cast<int*>(Tsc + (kCholThreads / 64) * 256);  // [16]
    const int tid = threadIdx.x, nt = blockDim.x;
    const int lane = tid & 63, wv = tid >> 6, nw = nt >> 6;
    const int r = lane & 15, h = lane >> 4;
    const int64_t L2 = (int64_t)LP * LP;

    for (int64_t e = tid; e < L2; e += nt) {
        const int i = (int)(e / LP), j = (int)(e % LP);
        W[e] = (i < l && j < l) ? G[e] : 0.0;
        R[e] = 0.0;
        Rinv[e] = 0.0;
    }
    for (int i = tid; i < LP; i += nt) {
        d0[i] = (i < l) ? G[(int64_t)i * LP + i] : 0.0;
        colflag[i] = 0;
    }
    __syncthreads();

    for (int p = 0; p < np; ++p) {
        const int p16 = 16 * p;
        double* Di = Dinv + p * 256;
        // (1) wave 0: upper Cholesky of the 16x16 diagonal block and its inverse, in registers
        if (wv == 0) {
            const int j = lane & 15;
            double col[16];
#pragma unroll
            for (int i = 0; i < 16; ++i) col[i] = W[(int64_t)(p16 + i) * LP + p16 + j];  // D[i][j]
            int badmask = 0;
#pragma unroll
            for (int k = 0; k < 16; ++k) {
                const int gk = p16 + k;
                const double dkk = readlane_d(col[k], k);
                const bool pad = gk >= l;
                const bool isbad = !pad && (!(dkk > tol * d0[gk]) || !(d0[gk] > 0.0) || !isfinite(dkk));
                if (isbad) badmask |= 1 << k;
                const bool unit = pad || isbad;
                const double rk = unit ? 1.0 : sqrt(dkk);
                const double inv = 1.0 / rk;
                if (j > k) col[k] = unit ? 0.0 : col[k] * inv;
                if (j == k) col[k] = rk;
#pragma unroll
                for (int i = k + 1; i < 16; ++i) {
                    const double dki = readlane_d(col[k], i);  // D[k][i]
                    if (j >= i) col[i] -= dki * col[k];
                }
            }
            // zero the strictly lower part of this column (it held the symmetric copy)
#pragma unroll
            for (int i = 0; i < 16; ++i)
                if (i > j) col[i] = 0.0;
            // Dinv column j by back substitution: x[i] = -(sum_{k>i} D[i][k] x[k]) / D[i][i]
            double x[16];
#pragma unroll
            for (int i = 15; i >= 0; --i) {
                double s = 0.0;
#pragma unroll
                for (int k = i + 1; k < 16; ++k) s += readlane_d(col[i], k) * x[k];  // D[i][k] from lane k
                const double dii = readlane_d(col[i], i);
                x[i] = (i == j) ? 1.0 / dii : ((i < j) ? -s / dii : 0.0);
            }
            if (lane < 16) {
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    Di[i * 16 + j] = x[i];
                    R[(int64_t)(p16 + i) * LP + p16 + j] = col[i];
                }
            }
            if (lane < 16) bad[lane] = (badmask >> lane) & 1;
            if (lane == 0 && badmask) {
                atomicAdd(flag, __popc(badmask));
                for (int k = 0; k < 16; ++k)
                    if (badmask & (1 << k)) colflag[p16 + k] = 1;
            }
        }
        __syncthreads();
        // (2) strip: R[p][jb] = Dinv^T W[p][jb], or 0 for rows that broke down (one wave per block)
        for (int jb = p + 1 + wv; jb < np; jb += nw) {
            f64x4 acc = MD::zero();
            acc = mma_tn16(Di, 16, W + (int64_t)p16 * LP + 16 * jb, LP, acc, r, h);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int i = MD::row(h, j);
                R[(int64_t)(p16 + i) * LP + 16 * jb + r] = (bad[i] || p16 + i >= l) ? 0.0 : acc[j];
            }
        }
        __syncthreads();
        // (3) trailing update W[ib][jb] -= R[p][ib]^T R[p][jb], p < ib <= jb
        const int nt2 = np - p - 1;
        const int ntri = nt2 * (nt2 + 1) / 2;
        for (int t = wv; t < ntri; t += nw) {
            int rem = t, ib = 0;
            while (rem >= nt2 - ib) {
                rem -= nt2 - ib;
                ++ib;
            }
            const int jb = ib + rem + p + 1;
            ib += p + 1;
            f64x4 acc = MD::zero();
            acc = mma_tn16(R + (int64_t)p16 * LP + 16 * ib, LP, R + (int64_t)p16 * LP + 16 * jb, LP, acc, r, h);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int i = MD::row(h, j);
                W[(int64_t)(16 * ib + i) * LP + 16 * jb + r] -= acc[j];
            }
        }
        __syncthreads();
    }
    // Rinv, bottom block row first: Rinv[p][p] = Dinv_p, Rinv[p][jb] = -Dinv_p sum_{p<k<=jb} R[p][k] Rinv[k][jb]
    double* Tw = Tsc + wv * 256;
    for (int p = np - 1; p >= 0; --p) {
        const double* Di = Dinv + p * 256;
        const int p16 = 16 * p;
        for (int e = tid; e < 256; e += nt) Rinv[(int64_t)(p16 + e / 16) * LP + p16 + e % 16] = Di[e];
        for (int jb = p + 1 + wv; jb < np; jb += nw) {
            f64x4 acc = MD::zero();
            for (int kb = p + 1; kb <= jb; ++kb)
                acc = mma_nn16(R + (int64_t)p16 * LP + 16 * kb, LP, Rinv + (int64_t)(16 * kb) * LP + 16 * jb, LP, acc,
                               r, h);
#pragma unroll
            for (int j = 0; j < 4; ++j) Tw[MD::row(h, j) * 16 + r] = acc[j];
            __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the wave's LDS stores landed
            __builtin_amdgcn_wave_barrier();
            f64x4 o = MD::zero();
            o = mma_nn16(Di, 16, Tw, 16, o, r, h);
#pragma unroll
            for (int j = 0; j < 4; ++j) Rinv[(int64_t)(p16 + MD::row(h, j)) * LP + 16 * jb + r] = -o[j];
            __builtin_amdgcn_wave_barrier();
        }
        __syncthreads();
    }
    if (Rinv32)
        for (int64_t e = tid; e < L2; e += nt) Rinv32[e] = (float)Rinv[e];
}

size_t chol_lds_bytes(int LP) {
    const int np = LP / 16;
    return (size_t)np * 256 * 8 + (size_t)LP * 8 + (size_t)(kCholThreads / 64) * 256 * 8 + 16 * 4 + 64;
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

__device__ __forceinline__ bf16_t f2bf(float x) {  // round to nearest even
    const uint32_t u = __float_as_uint(x);
    if ((u & 0x7f800000u) == 0x7f800000u) return (bf16_t)(u >> 16);
    return (bf16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}
__device__ __forceinline__ float bf2f(bf16_t b) { return __uint_as_float((uint32_t)b << 16); }

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
                    Out[orow * LP + c] = v;
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
template <typename T>
__global__ void repair_kernel(const T* __restrict__ Q, int64_t rows, int l, int LP, const int* __restrict__ colflag,
                              const int* __restrict__ flag, uint64_t seed, int64_t row_off, int64_t rows_total,
                              T* __restrict__ Out) {
    if (*flag == 0) return;
    const double sc = 1.0 / sqrt((double)rows_total);
    const int64_t total = rows * LP;
    for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = e / LP;
        const int c = (int)(e - i * LP);
        T v = Q[e];
        if (c < l && colflag[c]) v = (T)(gauss_elem((uint64_t)(row_off + i + rows_total * (int64_t)c), seed) * sc);
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

__global__ void omega_lowp_kernel(bf16_t* __restrict__ panel, int64_t n, int l, int LP, uint64_t seed, int fp8,
                                  float* __restrict__ f) {
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

template <typename T>
__global__ void convert_scale_kernel(const double* __restrict__ x, T* __restrict__ y, int n, double sc) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) y[i] = (T)(x[i] * sc);
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
    else
        hipLaunchKernelGGL((gram_wide_kernel<T, false>), dim3(wgs), dim3(256), 0, s, P, P, rows, LP, gp.blocks,
                           gp.chunks, gp.rows_per_chunk, slabs, pred);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const int64_t tot = (int64_t)gp.blocks * 1024;
    hipLaunchKernelGGL(gram_reduce_kernel, dim3((int)((tot + 255) / 256)), dim3(256), 0, s, slabs, gp.blocks,
                       gp.chunks, LP, P2 ? 1 : 0, G, pred);
    return hipGetLastError();
}

hipError_t launch_chol_wide(const double* G, int l, int LP, double tol, double* R, double* Rinv, float* Rinv32,
                            int* colflag, int* flag, double* work, const int* pred, hipStream_t s) {
    if (LP % 16 || LP > 512) return hipErrorInvalidValue;
    hipLaunchKernelGGL(chol_wide_kernel, dim3(1), dim3(kCholThreads), chol_lds_bytes(LP), s, G, l, LP, tol, work, R,
                       Rinv, Rinv32, colflag, flag, pred);
    return hipGetLastError();
}

template <typename T>
hipError_t launch_panel_gemm(const T* In, int64_t rows, int LP, const T* Mm, int upper, T* Out, int64_t ldo,
                             int cols, bf16_t* hi, bf16_t* lo, const int* pred, hipStream_t s) {
    if (!Mm || LP % 16) return hipErrorInvalidValue;
    const int64_t rb = (rows + 63) / 64;
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
                               uint64_t seed, int64_t row_off, int64_t rows_total, T* Out, hipStream_t s) {
    hipLaunchKernelGGL((repair_kernel<T>), dim3(grid_1d(rows * LP)), dim3(256), 0, s, Q, rows, l, LP, colflag, flag,
                       seed, row_off, rows_total, Out);
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

hipError_t launch_omega_lowp_from(const float* om, int64_t ld, int64_t n, int l, int LP, int round_fp8,
                                  bf16_t* panel, hipStream_t s) {
    hipLaunchKernelGGL(omega_lowp_from_kernel, dim3(grid_1d(n * LP)), dim3(256), 0, s, om, ld, n, l, LP, round_fp8,
                       panel);
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
                                             bf16_t*, const int*, hipStream_t);                                     \
    template hipError_t launch_repair_panel<T>(const T*, int64_t, int, int, const int*, const int*, uint64_t,       \
                                               int64_t, int64_t, T*, hipStream_t);                                  \
    template hipError_t launch_split_bf16<T>(const T*, int64_t, int, bf16_t*, bf16_t*, hipStream_t);
RSVD_INST(float)
RSVD_INST(double)
#undef RSVD_INST

}  // namespace rsvd
