// Layout probe for v_mfma_i32_16x16x64_i8 (gfx950): D = A . B + 0 with the fragment layout the
// Frodo kernels assume -- lane l supplies A[l & 15][16 (l >> 4) + j] and B[16 (l >> 4) + j][l & 15]
// (j = 0..15), and holds D[4 (l >> 4) + g][l & 15].  Prints max |D - A.B| over random int8 inputs.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
typedef int v4i __attribute__((ext_vector_type(4)));
__global__ void k(const signed char* A, const signed char* B, int* D) {
  const int l = threadIdx.x;
  v4i a, b;
  signed char* pa = (signed char*)&a;
  signed char* pb = (signed char*)&b;
  for (int j = 0; j < 16; ++j) {
    pa[j] = A[(l & 15) * 64 + 16 * (l >> 4) + j];
    pb[j] = B[(16 * (l >> 4) + j) * 16 + (l & 15)];
  }
  v4i c = {0, 0, 0, 0};
  v4i d = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c, 0, 0, 0);
  for (int g = 0; g < 4; ++g) D[(4 * (l >> 4) + g) * 16 + (l & 15)] = d[g];
}
int main() {
  signed char hA[16 * 64], hB[64 * 16];
  srand(7);
  for (int i = 0; i < 1024; ++i) hA[i] = (signed char)(rand() % 256 - 128), hB[i] = (signed char)(rand() % 256 - 128);
  signed char *dA, *dB;
  int* dD;
  hipMalloc(&dA, 1024); hipMalloc(&dB, 1024); hipMalloc(&dD, 1024);
  hipMemcpy(dA, hA, 1024, hipMemcpyHostToDevice);
  hipMemcpy(dB, hB, 1024, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dD);
  int hD[256];
  hipMemcpy(hD, dD, 1024, hipMemcpyDeviceToHost);
  long worst = 0, worstT = 0;
  for (int m = 0; m < 16; ++m)
    for (int n = 0; n < 16; ++n) {
      long s = 0, t = 0;
      for (int kk = 0; kk < 64; ++kk) s += hA[m * 64 + kk] * hB[kk * 16 + n], t += hA[n * 64 + kk] * hB[kk * 16 + m];
      long e = labs(s - hD[m * 16 + n]), et = labs(t - hD[m * 16 + n]);
      if (e > worst) worst = e;
      if (et > worstT) worstT = et;
    }
  printf("max|D-AB| = %ld   max|D-(AB)^T| = %ld\n", worst, worstT);
  return 0;
}
