// Cost of a cooperative sponge absorb beyond its permutations: SHA3-256 of a 1184-byte message
// held in LDS (the single-shot KeyGen's H(ek), 9 permutations) against 9 bare permutations, one
// wave, clock64 cycles.   ./coop_absorb_probe -> one JSON line
#include <hip/hip_runtime.h>
#include <stdio.h>

#include "../quantum-resistant-p2p_amd/csrc/keccak_coop.cuh"
using namespace qrk;

constexpr int NW = 1184 / 8;

__global__ void k_absorb(const uint64_t* msg, uint64_t* out, long long* cyc) {
  __shared__ uint64_t io[NW];
  for (int w = threadIdx.x; w < NW; w += 64) io[w] = msg[w];
  __syncthreads();
  const Coop c = coop_init();
  CState s;
  const long long t0 = clock64();
  coop_absorb<RW_SHA3_256, NW, DS_SHA3>(s, c, [&](int w) { return io[w]; });
  const long long t1 = clock64();
  if (coop_canon(c) && c.idx < 4) out[c.idx] = cs_word(s);
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

__global__ void k_bare(uint64_t* out, long long* cyc) {
  const Coop c = coop_init();
  CState s;
  s.lo = (uint32_t)c.idx;
  const long long t0 = clock64();
#pragma unroll 1
  for (int b = 0; b < 9; ++b) s = kf_coop(s, c);
  const long long t1 = clock64();
  out[threadIdx.x] = cs_word(s);
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

int main() {
  uint64_t h[NW];
  for (int i = 0; i < NW; ++i) h[i] = 0x0101010101010101ull * (uint64_t)(i & 0xFF);
  uint64_t *msg, *out;
  long long* cyc;
  (void)hipMalloc(&msg, sizeof(h));
  (void)hipMalloc(&out, 64 * 8);
  (void)hipMalloc(&cyc, 8);
  (void)hipMemcpy(msg, h, sizeof(h), hipMemcpyHostToDevice);
  long long ca[5], cb[5];
  for (int r = 0; r < 5; ++r) {
    hipLaunchKernelGGL(k_absorb, dim3(1), dim3(64), 0, 0, msg, out, cyc);
    (void)hipMemcpy(&ca[r], cyc, 8, hipMemcpyDeviceToHost);
    hipLaunchKernelGGL(k_bare, dim3(1), dim3(64), 0, 0, out, cyc);
    (void)hipMemcpy(&cb[r], cyc, 8, hipMemcpyDeviceToHost);
  }
  printf("{\"absorb_1184B_cycles\": [%lld, %lld, %lld, %lld, %lld], \"bare_9_perm_cycles\": [%lld, %lld, %lld, %lld, %lld]}\n",
         ca[0], ca[1], ca[2], ca[3], ca[4], cb[0], cb[1], cb[2], cb[3], cb[4]);
  return 0;
}
