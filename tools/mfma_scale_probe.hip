#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));
__global__ void k(const int* A, const int* B, float* D) {
  int l = threadIdx.x;
  v8i a, b;
  for (int i = 0; i < 8; ++i) { a[i] = A[l * 8 + i]; b[i] = B[l * 8 + i]; }
  v4f c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, 127, 0, 127);
  for (int i = 0; i < 4; ++i) D[l * 4 + i] = c[i];
}
int main() {
  const uint8_t enc[7] = {0xC4, 0xC0, 0xB8, 0x00, 0x38, 0x40, 0x44};  // -3..3
  uint8_t ha[64 * 32], hb[64 * 32];
  int va[64 * 32], vb[64 * 32];
  srand(1);
  for (int i = 0; i < 64 * 32; ++i) { va[i] = rand() % 7 - 3; vb[i] = rand() % 7 - 3; ha[i] = enc[va[i] + 3]; hb[i] = enc[vb[i] + 3]; }
  int *dA, *dB; float* dD;
  hipMalloc(&dA, sizeof ha); hipMalloc(&dB, sizeof hb); hipMalloc(&dD, 64 * 4 * 4);
  hipMemcpy(dA, ha, sizeof ha, hipMemcpyHostToDevice); hipMemcpy(dB, hb, sizeof hb, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dD);
  float hD[256]; hipMemcpy(hD, dD, sizeof hD, hipMemcpyDeviceToHost);
  // hypotheses: element j of lane l -> k
  for (int hyp = 0; hyp < 3; ++hyp) {
    int Am[16][128], Bm[128][16];
    for (int l = 0; l < 64; ++l) for (int j = 0; j < 32; ++j) {
      int kk;
      if (hyp == 0) kk = 32 * (l >> 4) + j;
      else if (hyp == 1) kk = 16 * (l >> 4) + (j & 15) + 64 * (j >> 4);
      else kk = 8 * (l >> 4) + (j & 7) + 32 * (j >> 3);
      Am[l & 15][kk] = va[l * 32 + j]; Bm[kk][l & 15] = vb[l * 32 + j];
    }
    int bad = 0;
    for (int l = 0; l < 64; ++l) for (int i = 0; i < 4; ++i) {
      int row = 4 * (l >> 4) + i, col = l & 15; long s = 0;
      for (int kk = 0; kk < 128; ++kk) s += Am[row][kk] * Bm[kk][col];
      if ((float)s != hD[l * 4 + i]) ++bad;
    }
    printf("hypothesis %d: %d mismatches of 256\n", hyp, bad);
  }
  printf("D[0..3] = %g %g %g %g\n", hD[0], hD[1], hD[2], hD[3]);
  return 0;
}
