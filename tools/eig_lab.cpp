// eig_lab.cpp -- the eigensolver small SVD (wide_eig.hip) on a synthetic l x l W: wall time per call
// (hipEvents), sweeps taken by the block-Jacobi check, and -- built with RSVD_TRI_PROF -- the shader
// cycles of each phase of the tridiagonalisation steps (workgroup 0).
// Build: make -C rsvd_kamaneh_raganato_terrana_amd/csrc eiglab ; run on the GPU box:
//   tools/eig_lab [l] [LP] [reps]
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "../rsvd_kamaneh_raganato_terrana_amd/csrc/wide.hpp"

namespace rsvd {
void tri_prof_read(long long* out);
}
using namespace rsvd;

#define CK(x)                                                                                \
    do {                                                                                     \
        hipError_t e = (x);                                                                  \
        if (e != hipSuccess) {                                                               \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
            exit(1);                                                                         \
        }                                                                                    \
    } while (0)

int main(int argc, char** argv) {
    const int l = argc > 1 ? atoi(argv[1]) : 256;
    const int LP = argc > 2 ? atoi(argv[2]) : 256;
    const int reps = argc > 3 ? atoi(argv[3]) : 5;
    hipStream_t s;
    CK(hipStreamCreate(&s));
    // W = R^T-like: random with graded columns (0.97^j) plus a flat tail, as the rSVD's W
    std::mt19937_64 rng(7);
    std::normal_distribution<double> nd;
    std::vector<double> W((size_t)LP * LP, 0.0);
    for (int c = 0; c < l; ++c)
        for (int i = 0; i < l; ++i) W[(size_t)c * LP + i] = nd(rng) * std::max(std::pow(0.97, c), 2e-3);
    double *dW, *ews, *X, *J, *Uw, *Vw, *S;
    unsigned* sync;
    int* info;
    const size_t L2 = (size_t)LP * LP;
    CK(hipMalloc(&dW, L2 * 8));
    CK(hipMalloc(&ews, eig_svd_ws_doubles(LP) * 8));
    CK(hipMalloc(&X, 2 * L2 * 8));
    CK(hipMalloc(&J, 2 * L2 * 8));
    CK(hipMalloc(&Uw, L2 * 8));
    CK(hipMalloc(&Vw, L2 * 8));
    CK(hipMalloc(&S, LP * 8));
    CK(hipMalloc(&sync, kBJSyncWords * 4));
    CK(hipMalloc(&info, 16));
    CK(hipMemcpy(dW, W.data(), L2 * 8, hipMemcpyHostToDevice));
    CK(hipMemset(info, 0, 16));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int r = 0; r < reps; ++r) {
#ifdef RSVD_TRI_PROF
        long long junk[16];
        tri_prof_read(junk);
#endif
        CK(hipEventRecord(a, s));
        CK(launch_eig_svd<double>(dW, l, LP, ews, X, J, Uw, Vw, S, sync, info, s, kBJTolF32));
        CK(hipEventRecord(b, s));
        CK(hipStreamSynchronize(s));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        int hinfo[4];
        CK(hipMemcpy(hinfo, info, 16, hipMemcpyDeviceToHost));
        std::vector<double> Sh(l);
        CK(hipMemcpy(Sh.data(), S, l * 8, hipMemcpyDeviceToHost));
        printf("l=%d LP=%d rep %d: %.1f us, sweeps %d, timeout %d, S[0] %.6g S[l-1] %.6g\n", l, LP, r, ms * 1e3,
               hinfo[0], hinfo[2], Sh[0], Sh[l - 1]);
#ifdef RSVD_TRI_PROF
        long long p[16];
        tri_prof_read(p);
        printf("  tridiag phases (Mcycles, wg 0), multi-workgroup steps: A %.3f B %.3f C %.3f D %.3f\n", p[0] * 1e-6,
               p[1] * 1e-6, p[2] * 1e-6, p[3] * 1e-6);
        printf("  tridiag phases (Mcycles), one-workgroup steps: A %.3f B %.3f C %.3f D %.3f\n", p[8] * 1e-6,
               p[9] * 1e-6, p[10] * 1e-6, p[11] * 1e-6);
        printf("  inverse iteration (Mcycles, thread 0): factor %.3f back %.3f forward %.3f back %.3f\n",
               p[4] * 1e-6, p[5] * 1e-6, p[6] * 1e-6, p[7] * 1e-6);
#endif
    }
    return 0;
}
