// Single-wave Keccak-f[1600] latency probe (the single-shot critical path): one wave, P
// permutations back to back on one state per lane, timed with HIP events and the shader clock.
//   ./keccak_latency  -> one JSON line: us and shader cycles per permutation for P = 1, 9, 90
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "../quantum-resistant-p2p_amd/csrc/keccak.cuh"
using namespace qrk;
__global__ void k_lat(int P, uint64_t* out, long long* cyc) {
  KState s;
  kzero(s);
  s.a[0].lo = threadIdx.x;
  const long long t0 = clock64();
  for (int i = 0; i < P; ++i) keccak_f(s);
  const long long t1 = clock64();
  out[threadIdx.x] = kword(s, 0) ^ kword(s, 7);
  if (threadIdx.x == 0) *cyc = t1 - t0;
}
int main() {
  uint64_t* out;
  long long* cyc;
  hipMalloc(&out, 64 * 8);
  hipMalloc(&cyc, 8);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL(k_lat, dim3(1), dim3(64), 0, 0, 4, out, cyc);  // warm-up
  hipDeviceSynchronize();
  printf("{");
  const int Ps[3] = {1, 9, 90};
  for (int i = 0; i < 3; ++i) {
    hipEventRecord(a, 0);
    hipLaunchKernelGGL(k_lat, dim3(1), dim3(64), 0, 0, Ps[i], out, cyc);
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    long long c = 0;
    hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    printf("%s\"P%d\": {\"kernel_us\": %.2f, \"clock64_per_perm\": %.0f}", i ? ", " : "", Ps[i], ms * 1e3, (double)c / Ps[i]);
  }
  printf("}\n");
  return 0;
}
