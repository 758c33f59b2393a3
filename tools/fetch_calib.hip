// Calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE against known byte counts, in the access
// patterns the ML-KEM kernels actually use (MI355X_MICROARCH.md: FETCH_SIZE is exactly 1/2 of a
// 16 B/lane coalesced streaming read on gfx950; "other access widths are uncalibrated:
// calibrate on a known byte count in your own access pattern").
//
// Every kernel touches a distinct 1.2-2 GB region (far above the 256 MB Infinity Cache), once,
// and writes one word per wave or per handshake (a few MB, reported separately).  Run under
//   rocprofv3 --pmc FETCH_SIZE -- ./fetch_calib      and      rocprofv3 --pmc WRITE_SIZE -- ./fetch_calib
// then tools/fetch_calib_summary.py joins the counters with the byte counts printed here.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      return 1;                                                               \
    }                                                                         \
  } while (0)

// ---- reads
// coalesced streaming reads: W bytes per lane, consecutive lanes consecutive
template <typename T>
__global__ void r_coalesced(const T* __restrict__ in, size_t n, uint32_t* __restrict__ out) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t acc = 0;
  if (i < n) {
    const T v = in[i];
    const uint32_t* w = (const uint32_t*)&v;
#pragma unroll
    for (int j = 0; j < (int)(sizeof(T) / 4); ++j) acc ^= w[j];
  }
  if (acc == 0x9E3779B9u) out[i & 1023] = acc;  // practically never: keeps the loads alive
}

// k_encrypt_core's SampleNTT reads: 16 lanes per handshake, lane L reads 16-B chunks 2L, 2L+1 of
// entry (e C + hs) in the 64-instance tiled layout (chunk c of inst at ((inst/64) 32 + c) 64 + inst%64)
__global__ void r_core_xof(const uint4* __restrict__ xs, size_t C, int entries, uint32_t* __restrict__ out) {
  const size_t hs = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 4;
  const int L = threadIdx.x & 15;
  uint32_t acc = 0;
  if (hs < C) {
    for (int e = 0; e < entries; ++e) {
      const size_t inst = (size_t)e * C + hs;
      const uint4* base = xs + (inst / 64) * 32 * 64 + (inst % 64);
      const uint4 u = base[(2 * L) * 64], v = base[(2 * L + 1) * 64];
      acc ^= u.x ^ u.y ^ u.z ^ u.w ^ v.x ^ v.y ^ v.z ^ v.w;
    }
  }
  if (acc == 0x9E3779B9u) out[hs & 1023] = acc;
}

// k_front_encaps' H(ek) absorb: one lane per handshake reads its own AoS record of `rec` bytes
// with 16-B loads, front to back
template <int REC>
__global__ void r_lane_aos(const uint8_t* __restrict__ in, size_t n, uint32_t* __restrict__ out) {
  const size_t hs = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t acc = 0;
  if (hs < n) {
    const uint4* p = (const uint4*)(in + hs * REC);
#pragma unroll 4
    for (int j = 0; j < REC / 16; ++j) {
      const uint4 u = p[j];
      acc ^= u.x ^ u.y ^ u.z ^ u.w;
    }
  }
  if (acc == 0x9E3779B9u) out[hs & 1023] = acc;
}

// the cores' AoS reads (ek rows, ct rows): 16 lanes per handshake read dword L + 16 i of a REC-byte row
template <int REC>
__global__ void r_group_aos(const uint8_t* __restrict__ in, size_t n, uint32_t* __restrict__ out) {
  const size_t hs = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 4;
  const int L = threadIdx.x & 15;
  uint32_t acc = 0;
  if (hs < n) {
    const uint32_t* p = (const uint32_t*)(in + hs * REC);
    for (int i = L; i < REC / 4; i += 16) acc ^= p[i];
  }
  if (acc == 0x9E3779B9u) out[hs & 1023] = acc;
}

// ---- writes
template <typename T>
__global__ void w_coalesced(T* __restrict__ o, size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    T v;
    uint32_t* w = (uint32_t*)&v;
#pragma unroll
    for (int j = 0; j < (int)(sizeof(T) / 4); ++j) w[j] = (uint32_t)i + j;
    o[i] = v;
  }
}
// k_xof's stores: one 16-B chunk per lane into the 64-instance tiled layout, chunk by chunk
__global__ void w_xof_tiled(uint4* __restrict__ o, size_t ninst) {
  const size_t inst = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (inst >= ninst) return;
  uint4* dst = o + (inst / 64) * 32 * 64 + (inst % 64);
  for (int c = 0; c < 32; ++c) dst[c * 64] = make_uint4((uint32_t)inst, c, 1, 2);
}
// the cores' AoS row writes (ct): 16 lanes per handshake write dword L + 16 i of a REC-byte row
template <int REC>
__global__ void w_group_aos(uint8_t* __restrict__ o, size_t n) {
  const size_t hs = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 4;
  const int L = threadIdx.x & 15;
  if (hs >= n) return;
  uint32_t* p = (uint32_t*)(o + hs * REC);
  for (int i = L; i < REC / 4; i += 16) p[i] = (uint32_t)hs ^ i;
}

static unsigned blocks(size_t threads) { return (unsigned)((threads + 255) / 256); }

int main() {
  const size_t GB = (size_t)1 << 30;
  uint8_t *a, *b;
  uint32_t* sink;
  CHECK(hipMalloc(&a, 2 * GB));
  CHECK(hipMalloc(&b, 2 * GB));
  CHECK(hipMalloc(&sink, 4096 * 4));
  CHECK(hipMemset(a, 0x5A, 2 * GB));
  CHECK(hipMemset(b, 0xA5, 2 * GB));
  CHECK(hipDeviceSynchronize());
  // each read kernel reads the other buffer than the previous one, so no line is cache-resident
  // (the previous kernel's 1.2-2 GB evicted the 256 MB Infinity Cache)
  printf("{\"kernel\": \"r_coalesced16\", \"read_bytes\": %zu}\n", (size_t)GB);
  r_coalesced<uint4><<<blocks(GB / 16), 256>>>((const uint4*)a, GB / 16, sink);
  printf("{\"kernel\": \"r_coalesced8\", \"read_bytes\": %zu}\n", (size_t)GB);
  r_coalesced<uint2><<<blocks(GB / 8), 256>>>((const uint2*)b, GB / 8, sink);
  printf("{\"kernel\": \"r_coalesced4\", \"read_bytes\": %zu}\n", (size_t)GB);
  r_coalesced<uint32_t><<<blocks(GB / 4), 256>>>((const uint32_t*)a, GB / 4, sink);
  {
    const size_t C = (size_t)1 << 18;  // 9 entries x 2^18 x 512 B = 1.2 GB
    printf("{\"kernel\": \"r_core_xof\", \"read_bytes\": %zu}\n", (size_t)9 * C * 512);
    r_core_xof<<<blocks(16 * C), 256>>>((const uint4*)b, C, 9, sink);
  }
  {
    const size_t n = (size_t)1 << 20;  // ML-KEM-768 ek: 1184 B
    printf("{\"kernel\": \"r_lane_aos\", \"read_bytes\": %zu}\n", n * 1184);
    r_lane_aos<1184><<<blocks(n), 256>>>(a, n, sink);
    printf("{\"kernel\": \"r_group_aos\", \"read_bytes\": %zu}\n", n * 1088);  // ML-KEM-768 ct
    r_group_aos<1088><<<blocks(16 * n), 256>>>(b, n, sink);
  }
  printf("{\"kernel\": \"w_coalesced16\", \"write_bytes\": %zu}\n", (size_t)GB);
  w_coalesced<uint4><<<blocks(GB / 16), 256>>>((uint4*)a, GB / 16);
  printf("{\"kernel\": \"w_coalesced4\", \"write_bytes\": %zu}\n", (size_t)GB);
  w_coalesced<uint32_t><<<blocks(GB / 4), 256>>>((uint32_t*)b, GB / 4);
  {
    const size_t ninst = (size_t)9 << 18;
    printf("{\"kernel\": \"w_xof_tiled\", \"write_bytes\": %zu}\n", ninst * 512);
    w_xof_tiled<<<blocks(ninst), 256>>>((uint4*)a, ninst);
    const size_t n = (size_t)1 << 20;
    printf("{\"kernel\": \"w_group_aos\", \"write_bytes\": %zu}\n", n * 1088);
    w_group_aos<1088><<<blocks(16 * n), 256>>>(b, n);
  }
  CHECK(hipDeviceSynchronize());
  CHECK(hipFree(a));
  CHECK(hipFree(b));
  CHECK(hipFree(sink));
  return 0;
}
