// Latency of the instruction kinds the wave-cooperative Keccak round (csrc/keccak_coop.cuh) chains,
// on one wave alone on the GPU: shader clocks per dependent instruction (clock64 over a chain of
// 4096), and the issue interval of independent VALU work (8 interleaved chains).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/coop_lat_probe.hip -o tools/coop_lat_probe
#include <hip/hip_runtime.h>
#include <stdio.h>

#include <cstdint>

constexpr int N = 4096;

template <int KIND>
__global__ void k_chain(uint32_t seed, uint32_t* out, long long* cyc) {
  uint32_t v = seed + threadIdx.x, w = seed ^ threadIdx.x;
  const int addr = (int)(((threadIdx.x * 7) & 63) * 4);
  __syncthreads();
  const long long t0 = clock64();
#pragma unroll 64
  for (int i = 0; i < N; ++i) {
    if constexpr (KIND == 0) {  // v_xor_b32
      asm volatile("v_xor_b32 %0, %0, %1" : "+v"(v) : "v"(w));
    } else if constexpr (KIND == 1) {  // v_mov_b32 dpp row_shr:1
      v = (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x111, 0xF, 0xF, true);
    } else if constexpr (KIND == 2) {  // v_permlane32_swap
      const auto p = __builtin_amdgcn_permlane32_swap(v, w, false, false);
      v = p[0];
      w = p[1];
    } else if constexpr (KIND == 3) {  // v_permlane16_swap
      const auto p = __builtin_amdgcn_permlane16_swap(v, w, false, false);
      v = p[0];
      w = p[1];
    } else if constexpr (KIND == 4) {  // ds_bpermute_b32
      v = (uint32_t)__builtin_amdgcn_ds_bpermute(addr, (int)v);
    } else if constexpr (KIND == 5) {  // v_alignbit_b32
      asm volatile("v_alignbit_b32 %0, %0, %1, 7" : "+v"(v) : "v"(w));
    } else if constexpr (KIND == 6) {  // v_bitop3_b32
      v = __builtin_amdgcn_bitop3_b32(v, w, v, 0x96);
    } else if constexpr (KIND == 7) {  // ds_swizzle_b32 (swap adjacent 16-lane groups' lanes: offset 0x401f)
      v = (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x041F);
    } else if constexpr (KIND == 8) {  // v_mov_b32 dpp row_ror:8 then xor (the theta pattern)
      v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x128, 0xF, 0xF, true);
    }
  }
  const long long t1 = clock64();
  out[threadIdx.x] = v ^ w;
  if (threadIdx.x == 0) *cyc = t1 - t0;
}

// 8 independent v_xor chains interleaved: the issue interval of one wave alone
__global__ void k_issue(uint32_t seed, uint32_t* out, long long* cyc) {
  uint32_t v[8];
  for (int k = 0; k < 8; ++k) v[k] = seed + k * threadIdx.x;
  const uint32_t w = seed ^ threadIdx.x;
  const long long t0 = clock64();
#pragma unroll 8
  for (int i = 0; i < N / 8; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(v[k]) : "v"(w));
  }
  const long long t1 = clock64();
  uint32_t x = 0;
  for (int k = 0; k < 8; ++k) x ^= v[k];
  out[threadIdx.x] = x;
  if (threadIdx.x == 0) *cyc = t1 - t0;
}

template <int KIND>
double run(uint32_t* out, long long* cyc) {
  hipLaunchKernelGGL(k_chain<KIND>, dim3(1), dim3(64), 0, 0, 1u, out, cyc);
  hipLaunchKernelGGL(k_chain<KIND>, dim3(1), dim3(64), 0, 0, 2u, out, cyc);
  long long c = 0;
  hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
  return (double)c / N;
}

int main() {
  uint32_t* out;
  long long* cyc;
  hipMalloc(&out, 64 * 4);
  hipMalloc(&cyc, 8);
  const char* names[9] = {"v_xor",   "dpp_row_shr1", "permlane32_swap", "permlane16_swap", "ds_bpermute",
                          "v_alignbit", "v_bitop3", "ds_swizzle", "dpp_row_ror8_then_xor"};
  double r[9] = {run<0>(out, cyc), run<1>(out, cyc), run<2>(out, cyc), run<3>(out, cyc), run<4>(out, cyc),
                 run<5>(out, cyc), run<6>(out, cyc), run<7>(out, cyc), run<8>(out, cyc)};
  hipLaunchKernelGGL(k_issue, dim3(1), dim3(64), 0, 0, 1u, out, cyc);
  hipLaunchKernelGGL(k_issue, dim3(1), dim3(64), 0, 0, 2u, out, cyc);
  long long c = 0;
  hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
  printf("{\"clocks_per_dependent_instruction\": {");
  for (int i = 0; i < 9; ++i) printf("%s\"%s\": %.2f", i ? ", " : "", names[i], r[i]);
  printf("}, \"clocks_per_independent_v_xor\": %.2f, \"hip\": \"%s\"}\n", (double)c / N,
         hipGetErrorString(hipDeviceSynchronize()));
  return 0;
}
