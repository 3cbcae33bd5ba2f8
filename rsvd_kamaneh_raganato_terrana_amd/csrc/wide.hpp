// wide.hpp -- launch wrappers of the "wide" rSVD path: sketch widths up to 512 and bf16 / fp8 A.
//
// Panels (Y, Q, Z, Omega, B^T, Q_B) are row-major `rows x LP` in fp32 (fp64 when A is fp64), as
// in the narrow path (common.hpp).  For bf16 / fp8 A the projections run on the bf16 MFMA
// (v_mfma_f32_16x16x32_bf16) and read the skinny operand as a bf16 "hi" panel plus, for the
// power-iteration and B projections, a bf16 "lo" panel (P ~= hi + lo, 16 significant bits; the
// Gaussian sketch Omega is itself rounded to bf16 / e4m3, so the first projection is exact in
// one pass).  The QR is CholeskyQR(2) with fp64 Grams on the fp64 MFMA, a one-workgroup blocked
// Cholesky + triangular inverse, and an MFMA panel product that also emits the next hi/lo
// panels.  The small SVD is a block one-sided Jacobi on a persistent grid (wide_svd.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "../../include/rsvd_c.h"

namespace rsvd {

typedef uint16_t bf16_t;  // storage of one bf16
typedef uint8_t fp8_t;    // storage of one OCP e4m3fn

// ---- wide_proj.hip -----------------------------------------------------------------------------
// Sketch widths the bf16 projection kernels are built for (LP = padded l).
bool wproj_supported_lp(int LP);
int wproj_rows_per_block(int LP);  // output rows per workgroup (256 / 128 / 64)
struct WProjPlan {
    int splits;      // K splits (1 = straight into the output panel)
    int64_t chunk;   // K range per workgroup (multiple of 32)
    int blocks;      // output row blocks
    bool v2;         // LDS-DMA pipelined kernel (bf16 / e4m3 A, LP >= 128, 16-B aligned columns)
    bool ds = false; // v2 TN at LP = 128 with two k-steps per stage (128-B A runs; K a multiple of 64)
    int tn3 = 0;      // ds with separate A / S rings (wproj3tn128_kernel): 1 = 4 A / 2 S slots, 2 = 3 / 3 (lab)
    bool nn3 = false;  // bf16 NN at LP = 128 on wproj3_kernel (RSVD_NN3_128=0: the v2 kernel)
    bool nn8 = false;  // e4m3 NN halves on the v3-style wproj3nn8_kernel (RSVD_NN8=0: the v2 kernel)
    bool v3 = false; // v2 with launch-constant LDS read bases (bf16 A, LP 256 / 512; wide_proj.hip)
    bool tn2 = false; // v3 TN at LP = 256 with two k-steps per A slot (128-B A lines)
    bool half = false; // e4m3 A at LP = 512: two LP = 256 column-half launches (256-row tiles)
    bool tn4 = false;  // e4m3 TN at LP 256 / 512: four k-steps per A slot (128-B A lines, wproj3tn4_kernel)
    bool merge = false; // LP = 512 halves (half / tn4) in ONE launch, twin blocks adjacent (A from HBM once)
    int abl = 0;      // lab-only ablations of the v3 kernel (tools/wide_lab.cpp), never set by the engine
    int kn = -1;      // lab-only knob override of the LP = 256 v3 kernels (-1: the engine's choice)
};
// v2 requires: a 16-B aligned base, bf16 A with lda and m multiples of 8 or e4m3 A with lda and m
// multiples of 16, and S panels zero-padded
// to a multiple of 32 rows (the engine allocates them so).
WProjPlan plan_wproj(int64_t rows_out, int64_t K, int LP, bool v2 = false, bool nn = true, bool fp8 = false);
// NN: Y (m x LP, fp32) = A (m x n) * S       S = n x LP bf16 panel(s)      src/rSVD.cpp:59,66
// TN: Z (n x LP, fp32) = A^T * S             S = m x LP bf16 panel(s)      src/rSVD.cpp:63,89
// A is column-major (lda) bf16 (a_fp8 = 0) or e4m3 (a_fp8 = 1).  Slo == nullptr: single pass.
// `done` (optional) is recorded after the MFMA kernel, before the slab reduction.
hipError_t launch_wproj(int nn, int a_fp8, const void* A, int64_t lda, int64_t m, int64_t n, const bf16_t* Shi,
                        const bf16_t* Slo, int LP, const WProjPlan& p, float* slabs, float* Out, hipStream_t s,
                        hipEvent_t done = nullptr);

// e4m3 A times an e4m3 panel S8 (n x LP bytes, rows zero-padded to a multiple of 32): the Gaussian
// sketch Y = A Omega of an e4m3 A on v_mfma_f32_16x16x32_fp8_fp8 (both operands exact e4m3).
// Needs an NN plan with v2 and LP in {256, 512} (wproj_s8_supported).
bool wproj_s8_supported(const WProjPlan& p, int LP);
hipError_t launch_wproj_s8(const void* A, int64_t lda, int64_t m, int64_t n, const fp8_t* S8, int LP, const WProjPlan& p,
                           float* slabs, float* Out, hipStream_t s, hipEvent_t done = nullptr);
// bf16 panel holding exactly-e4m3 values -> e4m3 codes (count elements)
hipError_t launch_bf16_to_fp8(const bf16_t* in, int64_t count, fp8_t* out, hipStream_t s);

// ---- wide_qr.hip -------------------------------------------------------------------------------
struct GramPlan {
    int blocks;   // 32 x 32 blocks of the Gram (upper triangle, or all for a cross Gram)
    int chunks;   // row chunks
    int64_t rows_per_chunk;
};
GramPlan plan_gram_wide(int64_t rows, int LP, int cross);
// Partial Grams of P^T P (cross: P^T P2) per (chunk, 32x32 block) into `slabs` (fp64), then
// G = sum over chunks (LP x LP fp64 row-major, mirrored when symmetric).  `pred` (nullable): skip
// both launches unless *pred != 0.
template <typename T>
hipError_t launch_gram_wide(const T* P, const T* P2, int64_t rows, int LP, const GramPlan& gp, double* slabs,
                            double* G, const int* pred, hipStream_t s);
// R = chol(G[:l,:l]) (upper) and Rinv = R^-1, LP x LP fp64 zero-padded, one workgroup.  A pivot
// d_k <= tol * G_kk (or not finite) is a breakdown: R row k := e_k, colflag[k] = 1, *flag += 1.
// Also writes Rinv as fp32 when Rinv32 != nullptr.  `work`: LP x LP fp64.  `pred`: as above.
// ill (nullable): set to 1 when a pivot d_k <= ill_tol * G_kk (else 0) -- the split-Gram fallback test.
hipError_t launch_chol_wide(const double* G, int l, int LP, double tol, double* R, double* Rinv, float* Rinv32,
                            int* colflag, int* flag, double* work, const int* pred, hipStream_t s,
                            double ill_tol = 0.0, int* ill = nullptr, const double* d0src = nullptr,
                            bf16_t* Mt = nullptr, int ldg = 0);  // ldg: G's row pitch (0: LP)
// The same factor at LP = 2 B (B = 128, 256; l > B) in two B-column levels: R11 = chol(G11) and
// S = G22 - R12^T R12 (R12 = R11^-T G12), the off-diagonal blocks R12 and Rinv12 = -Rinv11 R12 Rinv22
// on a B^3 fp64 MFMA GEMM, breakdowns judged against the diagonal of G (d0src when this factor is
// itself a level) as the one-level factor does.  The levels are the one-workgroup LP = B kernels,
// or (depth > 0, B = 256) two-level factors themselves.  scratch: chol_2level_scratch_doubles.
hipError_t launch_chol_wide_2level(const double* G, int l, int LP, double tol, double* R, double* Rinv,
                                   float* Rinv32, int* colflag, int* flag, double* work, double* scratch,
                                   hipStream_t s, double ill_tol = 0.0, int* ill = nullptr,
                                   const double* d0src = nullptr, int depth = 0, bf16_t* Mt = nullptr,
                                   int ldg = 0);  // ldg: G's row pitch (0: LP)
// (Mt, both factors, with Rinv32: R^-1's fp32 copy also as split_mat_kernel's three bf16 piece
// images, 3 LP^2 -- launch_panel_gemm's msplit with msplit_ready)
size_t chol_2level_scratch_doubles(int LP, int depth);
// G = P^T P of an fp32 panel by the three-piece bf16 split on the bf16 MFMA (fp32 chunk sums added
// in fp64; |dG| ~ 1e-8 |G|) -- same plan / slab layout as launch_gram_wide.  LP in {128, 256, 512}.
bool gram_split_ok(int LP);
hipError_t launch_gram_split(const float* P, int64_t rows, int LP, const GramPlan& gp, double* slabs, double* G,
                             hipStream_t s);
// R = X^T Y of two fp32 panels by the same split (LP = 256 / 512; gp: the cross plan, plan_gram_wide(rows, LP, 1));
// more than kSplitCrossRows rows per chunk fall back to the fp64 cross Gram (launch_gram_wide)
constexpr int64_t kSplitCrossRows = 4096;
hipError_t launch_gram_split_cross(const float* X, const float* Y, int64_t rows, int LP, const GramPlan& gp,
                                   double* slabs, double* G, hipStream_t s);
// 1 (default): chol_reg_kernel for LP <= 128, chol_wide_kernel above; 0: chol_wide_kernel everywhere;
// 2: also chol_reg_kernel at LP = 256 (lab A/B only).
extern int chol_variant;
// Out (rows x LP) = In (rows x LP) * M (LP x LP, row-major, in the panel precision T; `upper`:
// only k <= c of M is read).  Out may be null with ldo = 0 when only the hi / lo panels are wanted.
// Out layouts: row-major panel (ldo = 0) or the caller's column-major matrix (first
// `cols` columns, leading dimension ldo).  Optionally also writes the bf16 hi / lo panels of Out
// (row-major, LP wide).  `pred`: as above.
// msplit (fp32 panels, LP a multiple of 32 >= 128; 3 LP^2 bf16 of scratch): the product runs on the
// bf16 MFMA with both operands split in three bf16 pieces (panel_split_kernel) instead of the fp32 MFMA.
template <typename T>
hipError_t launch_panel_gemm(const T* In, int64_t rows, int LP, const T* M, int upper, T* Out, int64_t ldo,
                             int cols, bf16_t* hi, bf16_t* lo, const int* pred, hipStream_t s,
                             bf16_t* msplit = nullptr, bool msplit_ready = false);
// S = (float)(sc Sd) (l), U_w / V_w (LP x LP fp64) -> fp32 copies and their three bf16 piece images (Mu,
// Mv: 3 LP^2 each, launch_panel_gemm's msplit with msplit_ready) in one launch
hipError_t launch_finish_convert(const double* Sd, float* S, int l, double sc, const double* Uw, float* Uw32, bf16_t* Mu,
                                 const double* Vw, float* Vw32, bf16_t* Mv, int LP, hipStream_t s);
// y[0..n) = (T)(x * sc)
template <typename T>
hipError_t launch_convert_scale(const double* x, T* y, int n, double sc, hipStream_t s);
// Rank-deficiency repair of an orthonormalised panel: copies Q into Out, replacing every column
// k with colflag[k] != 0 by Philox Gaussian values / sqrt(norm_rows) (stream element
// row_off + i + rows_total * k: row shards of one global panel draw disjoint parts of one stream).
// No-op unless *flag != 0.
template <typename T>
hipError_t launch_repair_panel(const T* Q, int64_t rows, int l, int LP, const int* colflag, const int* flag,
                               uint64_t seed, int64_t row_off, int64_t rows_total, int64_t norm_rows, T* Out,
                               hipStream_t s, int64_t valid_rows = -1);
// fp32 / fp64 panel -> bf16 hi (+ lo) panels (rows x LP).
template <typename T>
hipError_t launch_split_bf16(const T* P, int64_t rows, int LP, bf16_t* hi, bf16_t* lo, hipStream_t s);
// Omega for bf16 / fp8 A: Philox N(0,1) rounded to bf16 (round_fp8 = 0) or e4m3 (= 1), written
// as the bf16 panel (n x LP) and, when `f` != nullptr, as fp32 column-major (ld n) for callers.
hipError_t launch_omega_lowp(bf16_t* panel, int64_t n, int l, int LP, uint64_t seed, int round_fp8, float* f,
                             hipStream_t s);
// Caller-supplied Omega (fp32 column-major, ld) -> bf16 panel, rounding to bf16 / e4m3.
hipError_t launch_omega_lowp_from(const float* om, int64_t ld, int64_t n, int l, int LP, int round_fp8,
                                  bf16_t* panel, hipStream_t s);

// ---- wide_svd.hip ------------------------------------------------------------------------------
// Block one-sided Jacobi of W (W[i][c] = R[c][i], l x l): X = W, J = I; rotate column blocks
// pairwise until orthogonal; then S (descending), Uw = X / S (completed to orthonormal when
// S = 0), Vw = J (both LP x LP fp64 row-major, [row][col]).  Work: X, J (2 LP^2 fp64 each:
// double buffers), sync (kBJSyncWords words, zeroed here).  LP in {64, 96, ..., 512}.  info[0] =
// sweeps; info[2] = 1 on a barrier timeout.
// quad2: a sweep whose rotations all have (g^2 / ab) <= quad2 ends the iteration (the next sweep would
// only square them): 1e-16 for fp64 results, 1e-8 for results delivered in fp32 (as jacobi.hip's fp32 path).
// tol_chk: after a sweep whose rotations were small enough, the largest cosine over ALL column pairs
// is measured and the iteration ends when it is <= tol_chk (0 disables the check).
constexpr int kBJSyncWords = 512;
constexpr double kBJTolF64 = 1e-12, kBJTolF32 = 1e-6;
template <typename T>
hipError_t launch_block_jacobi(const double* R, int l, int LP, double* X, double* J, double* Uw, double* Vw, T* S,
                               unsigned* sync, int* info, hipStream_t s, double quad2 = 1e-16,
                               double tol_chk = kBJTolF64, int G = 0);
// The general form: X = the mrv x l source (column-major with ld lds, or row-major: X = src^T when
// src_rowmajor), zero-padded to MR x LP (multiples of 32, LP <= 4096); X: 2 MR LP, J: 2 LP^2 doubles;
// U_w: MR x LP, V_w: LP x LP (row-major).  G: workgroups per block pair (row groups; 0 = the largest
// of 4, 2, 1 that block_jacobi_groups accepts).  MR / G > 512 reads the pair columns from global memory.
template <typename T>
hipError_t launch_block_jacobi_ex(const double* src, int64_t lds, int src_rowmajor, int mrv, int l, int MR, int LP,
                                  double* X, double* J, double* Uw, double* Vw, T* S, unsigned* sync, int* info,
                                  hipStream_t s, double quad2 = 1e-16, double tol_chk = kBJTolF64, int G = 0);
// The row-group count launch_block_jacobi_ex uses for G (0: auto), or 0 when G does not fit.
int block_jacobi_groups(int MR, int LP, int G);
// "Given" mode (LP <= 512): X = W V_w and J = V_w are already in buffer 0 of X / J (column-major,
// zero-padded); the kernel measures the largest cosine between the columns of X first and runs
// sweeps only while it exceeds tol_chk; then the same finish (S, U_w, V_w).
template <typename T>
hipError_t launch_block_jacobi_given(int l, int LP, double* X, double* J, double* Uw, double* Vw, T* S, unsigned* sync,
                                     int* info, hipStream_t s, double tol_chk);

// ---- wide_eig.hip ------------------------------------------------------------------------------
// The small SVD through the symmetric eigensolver (3 <= l <= 512, LP in {128, 256, 512}): G = W^T W,
// Householder tridiagonalisation, multisection eigenvalues, inverse-iteration eigenvectors, the
// compact-WY back-transformation, X = W V_w; then launch_block_jacobi_given's check (and polish if
// it fails) and finish.  ews: eig_svd_ws_doubles(LP) doubles; sync: kBJSyncWords words.
size_t eig_svd_ws_doubles(int LP);
// Z = op(X) op(Y) for n x n fp64 row-major matrices on the fp64 MFMA (tx / ty: transpose X / Y)
hipError_t launch_gemm_rm(int tx, int ty, int n, const double* X, int ldx, const double* Y, int ldy, double* Z, int ldz,
                          hipStream_t s);
// M = G^-1/2 for a Gram near the identity (|G - I|_F <= 0.1: flags[0] = 1, M into `out`; else flags[1] = 1
// and `out` is left alone).  prep_only: E = G - I and the flags; series_only: the rest (G no longer read).
hipError_t launch_isqrt_near_identity(const double* G, int l, int LP, double* E, double* E2, double* E3, double* B,
                                      double* T, double* out, int* flags, hipStream_t s, bool prep_only,
                                      bool series_only);
template <typename T>
hipError_t launch_eig_svd(const double* R, int l, int LP, double* ews, double* X, double* J, double* Uw, double* Vw,
                          T* S, unsigned* sync, int* info, hipStream_t s, double tol_chk);

// ---- wide.cpp: the host pipeline ------------------------------------------------------------------
// True when `d` runs on the wide engine (bf16 / fp8 A, or l > 64).
bool wide_path(const rsvd_desc_t* d);
int wide_workspace_bytes(const rsvd_desc_t* d, size_t* bytes);
// rSVD (Qout == nullptr) or intermediate_step (Q into Qout) on the handle's stream.
int wide_run(rsvd_handle_t h, const rsvd_desc_t* d, const void* A, const void* omega, int64_t ldo, void* U,
             int64_t ldu, void* S, void* V, int64_t ldv, void* Qout, int64_t ldq);

// ---- dense_big.cpp: rSVD() past the wide engine's 512 sketch columns --------------------------------
// One GPU, SVDMethod Jacobi / ParallelJacobi, l <= kBigLMax; column-major blocks on the MFMA GEMM
// (bf16 / e4m3 A widened to fp32 once), block CGS2 + CholeskyQR3 orthonormalisation, block Jacobi.
constexpr int kBigLMax = 4096;
int big_rsvd_run(rsvd_handle_t h, const rsvd_desc_t* d, const void* A, const void* omega, int64_t ldo, void* U,
                 int64_t ldu, void* S, void* V, int64_t ldv, void* Qout, int64_t ldq);
size_t big_rsvd_workspace(const rsvd_desc_t* d);

}  // namespace rsvd
