// gfx950 v_permlane16_swap / v_permlane32_swap semantics: for x = lane id passed as both
// operands, print which source lane each output lane holds (first / second result).
#include <hip/hip_runtime.h>
#include <stdio.h>
__global__ void k(unsigned* o) {
  unsigned x = threadIdx.x;
  auto a = __builtin_amdgcn_permlane16_swap(x, x, false, false);
  auto b = __builtin_amdgcn_permlane32_swap(x, x, false, false);
  o[4 * threadIdx.x + 0] = a[0];
  o[4 * threadIdx.x + 1] = a[1];
  o[4 * threadIdx.x + 2] = b[0];
  o[4 * threadIdx.x + 3] = b[1];
}
int main() {
  unsigned* d;
  unsigned h[256];
  (void)hipMalloc(&d, sizeof(h));
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  const char* nm[4] = {"p16.0", "p16.1", "p32.0", "p32.1"};
  for (int r = 0; r < 4; ++r) {
    printf("%s:", nm[r]);
    for (int l = 0; l < 64; ++l) printf(" %u", h[4 * l + r]);
    printf("\n");
  }
  return 0;
}
