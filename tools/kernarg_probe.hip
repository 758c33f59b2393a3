// Does this stack launch a kernel whose by-value argument is 4.8 KB (more than the 4 KB often
// quoted)?  ML-KEM-1024 single-shot Decaps passes c || dk (4736 B) that way.  -> one JSON line
#include <hip/hip_runtime.h>
#include <stdio.h>
struct Big { unsigned long long w[600]; };  // 4800 B
__global__ void k(Big b, unsigned long long* out) { out[threadIdx.x] = b.w[threadIdx.x * 9]; }
int main() {
  Big b; for (int i = 0; i < 600; ++i) b.w[i] = i * 3 + 1;
  unsigned long long* d; (void)hipMalloc(&d, 64 * 8);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, b, d);
  hipError_t e = hipDeviceSynchronize();
  unsigned long long h[64]; (void)hipMemcpy(h, d, 64 * 8, hipMemcpyDeviceToHost);
  int bad = 0; for (int t = 0; t < 64; ++t) bad += h[t] != (unsigned long long)(t * 9 * 3 + 1);
  printf("{\"launch\": \"%s\", \"bad\": %d}\n", hipGetErrorString(e), bad);
  return 0;
}
