// Wave-cooperative Keccak-f[1600] (csrc/keccak_coop.cuh) against the lane-per-state one
// (csrc/keccak.cuh): correctness on random states, then single-wave latency per permutation.
//   ./keccak_coop_probe  -> one JSON line
#include <hip/hip_runtime.h>
#include <stdio.h>

#include "../quantum-resistant-p2p_amd/csrc/keccak_coop.cuh"
using namespace qrk;

// state s (25 words) -> P permutations, both ways; out_ref / out_coop 25 words each
__global__ void k_check(const uint64_t* in, int P, uint64_t* out_ref, uint64_t* out_coop) {
  const Coop c = coop_init();
  uint32_t lo = 0, hi = 0;
  if (c.idx >= 0) {
    lo = (uint32_t)in[c.idx];
    hi = (uint32_t)(in[c.idx] >> 32);
  }
  for (int p = 0; p < P; ++p) keccak_f_coop(lo, hi, c);
  if (c.idx >= 0) out_coop[c.idx] = ((uint64_t)hi << 32) | lo;
  if (threadIdx.x == 0) {
    KState s;
#pragma unroll
    for (int i = 0; i < 25; ++i) s.a[i] = {(uint32_t)in[i], (uint32_t)(in[i] >> 32)};
    for (int p = 0; p < P; ++p) keccak_f(s);
#pragma unroll
    for (int i = 0; i < 25; ++i) out_ref[i] = kword(s, i);
  }
}

__global__ void k_lat(int P, uint64_t* out, long long* cyc) {
  const Coop c = coop_init();
  uint32_t lo = c.idx >= 0 ? (uint32_t)c.idx : 0u, hi = 0;
  const long long t0 = clock64();
  for (int i = 0; i < P; ++i) keccak_f_coop(lo, hi, c);
  const long long t1 = clock64();
  out[threadIdx.x] = ((uint64_t)hi << 32) | lo;
  if (threadIdx.x == 0) *cyc = t1 - t0;
}

int main() {
  uint64_t h_in[25], h_ref[25], h_coop[25];
  uint64_t x = 0x9E3779B97F4A7C15ull;
  for (int i = 0; i < 25; ++i) {
    x ^= x << 13;
    x ^= x >> 7;
    x ^= x << 17;
    h_in[i] = x;
  }
  uint64_t *in, *ref, *coop, *out;
  long long* cyc;
  hipMalloc(&in, 25 * 8);
  hipMalloc(&ref, 25 * 8);
  hipMalloc(&coop, 25 * 8);
  hipMalloc(&out, 64 * 8);
  hipMalloc(&cyc, 8);
  hipMemcpy(in, h_in, 25 * 8, hipMemcpyHostToDevice);
  int bad = 0;
  for (int P = 1; P <= 3; ++P) {
    hipLaunchKernelGGL(k_check, dim3(1), dim3(64), 0, 0, in, P, ref, coop);
    hipMemcpy(h_ref, ref, 25 * 8, hipMemcpyDeviceToHost);
    hipMemcpy(h_coop, coop, 25 * 8, hipMemcpyDeviceToHost);
    for (int i = 0; i < 25; ++i) bad += h_ref[i] != h_coop[i];
  }
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL(k_lat, dim3(1), dim3(64), 0, 0, 4, out, cyc);  // warm-up
  hipDeviceSynchronize();
  printf("{\"mismatched_words\": %d", bad);
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
    printf(", \"P%d\": {\"kernel_us\": %.2f, \"clock64_per_perm\": %.0f}", Ps[i], ms * 1e3, (double)c / Ps[i]);
  }
  printf("}\n");
  return 0;
}
