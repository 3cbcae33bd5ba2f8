// common.hpp -- shared device helpers for the gfx950 (MI355X / CDNA4) rSVD kernels.
//
// Conventions used by every kernel in this directory:
//  * A (the big m x n operand) is column-major with leading dimension lda, exactly as the
//    reference's Eigen::MatrixXd (include/rSVD.hpp:9).
//  * "Skinny" panels (Omega, Y = A*Omega, Q, Z = A^T*Q, B^T) live in HBM ROW-major with a
//    padded width LP = 16*ceil(l/16): one panel row is one contiguous LP-vector, which is the
//    natural B-operand feed of the 16x16x4 MFMA (16 lanes read 16 consecutive columns) and the
//    row-per-thread feed of the QR kernels.  Columns l..LP-1 are kept exactly zero.
//  * Wave = 64 lanes.  lane = threadIdx.x & 63, r = lane & 15, h = lane >> 4.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rsvd {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef double f64x4 __attribute__((ext_vector_type(4)));

constexpr int kWave = 64;

// ---------------------------------------------------------------------------------------------
// MFMA 16x16x4 (f32-in exact f32, or f64).  Operand maps (cdna_hip_programming.md §3):
//   A: lane l holds A[row = l & 15][k = l >> 4];  B: lane l holds B[k = l >> 4][col = l & 15]
//   C/D f32: col = lane & 15, row = (lane >> 4) * 4 + reg
//   C/D f64: col = lane & 15, row = (lane >> 4) + 4 * reg
// ---------------------------------------------------------------------------------------------
template <typename T> struct Mfma;

template <> struct Mfma<float> {
    typedef f32x4 acc_t;
    static __device__ __forceinline__ acc_t zero() { return acc_t{0.f, 0.f, 0.f, 0.f}; }
    static __device__ __forceinline__ acc_t mma(float a, float b, acc_t c) {
        return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
    }
    // row of register `reg` for lane half h (= lane >> 4)
    static __device__ __forceinline__ int row(int h, int reg) { return h * 4 + reg; }
};

template <> struct Mfma<double> {
    typedef f64x4 acc_t;
    static __device__ __forceinline__ acc_t zero() { return acc_t{0.0, 0.0, 0.0, 0.0}; }
    static __device__ __forceinline__ acc_t mma(double a, double b, acc_t c) {
        return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
    }
    static __device__ __forceinline__ int row(int h, int reg) { return h + 4 * reg; }
};

// 16-byte vector of T: 4 floats or 2 doubles.
template <typename T> struct Vec16;
template <> struct Vec16<float> {
    static constexpr int N = 4;
    typedef float4 type;
    static __device__ __forceinline__ float get(const float4& v, int t) {
        return t == 0 ? v.x : (t == 1 ? v.y : (t == 2 ? v.z : v.w));
    }
};
template <> struct Vec16<double> {
    static constexpr int N = 2;
    typedef double2 type;
    static __device__ __forceinline__ double get(const double2& v, int t) { return t == 0 ? v.x : v.y; }
};

// XCD-aware bijective block remap (cdna_hip_programming.md §5 "XCD swizzle must be bijective"):
// blocks that the dispatcher deals to the same XCD (b % 8) get consecutive logical ids, so
// neighbouring tiles (which share A columns / panel rows) meet in one L2.
__device__ __forceinline__ int xcd_remap(int b, int nwg) {
    const int xcd = b & 7, q = nwg >> 3, r = nwg & 7;
    const int base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
    return base + (b >> 3);
}

__device__ __forceinline__ double warp_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

}  // namespace rsvd
