// Diagnostic: where does k_xof's time go?  Same geometry as production
// (9 x 2^20 lanes, 256 per workgroup), variants:
//   0: 3 Keccak-f only            1: + split12 / compare / count (no LDS, no stores)
//   2: + LDS ring writes          3: + chunk flush to global (production-equivalent)
#include <cstdio>
#include "../quantum-resistant-p2p_amd/csrc/keccak.cuh"

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("err %s\n", hipGetErrorString(e_)); return 1; } } while (0)
using namespace qrk;
constexpr int Q = 3329;

__device__ __forceinline__ void split12(uint32_t w0, uint32_t w1, uint32_t w2, int c[8]) {
  c[0] = (int)(w0 & 0xFFF);
  c[1] = (int)((w0 >> 12) & 0xFFF);
  c[2] = (int)(__builtin_amdgcn_alignbit(w1, w0, 24) & 0xFFF);
  c[3] = (int)((w1 >> 4) & 0xFFF);
  c[4] = (int)((w1 >> 16) & 0xFFF);
  c[5] = (int)(__builtin_amdgcn_alignbit(w2, w1, 28) & 0xFFF);
  c[6] = (int)((w2 >> 8) & 0xFFF);
  c[7] = (int)(w2 >> 20);
}

template <int V>
__global__ __launch_bounds__(256) void k_probe(size_t total, uint4* __restrict__ out, uint32_t* sink) {
  __shared__ uint32_t ring_all[4 * 16 * 64];
  uint32_t* ring = ring_all + (threadIdx.x >> 6) * 16 * 64 + (threadIdx.x & 63);
  const size_t inst = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (inst >= total) return;
  uint4* dst = out + (inst >> 6) * 32 * 64 + (inst & 63);
  KState s;
  kzero(s);
  s.a[0].lo = (uint32_t)inst;
  s.a[4].lo ^= 0x1F0000u;
  s.a[20].hi ^= 0x80000000u;
  int cnt = 0;
  uint32_t acc = 0;
#pragma unroll 1
  for (int b = 0; b < 3; ++b) {
    keccak_f(s);
    if (V == 0) {
      acc ^= s.a[b].lo;
      continue;
    }
#pragma unroll
    for (int t = 0; t < 14; ++t) {
      uint32_t d[3];
#pragma unroll
      for (int e = 0; e < 3; ++e) {
        const int di = 3 * t + e;
        d[e] = (di & 1) ? s.a[di >> 1].hi : s.a[di >> 1].lo;
      }
      int c[8];
      split12(d[0], d[1], d[2], c);
      const int before = cnt;
      int pos = cnt << 8;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        if (V >= 2) *(uint32_t*)((char*)ring + (pos & 0xF00)) = (uint32_t)c[e];
        else acc += (uint32_t)c[e] ^ (uint32_t)pos;
        pos += c[e] < Q ? 256 : 0;
      }
      cnt = pos >> 8;
      const int ch = before >> 3;
      if (V == 3 && (cnt >> 3) != ch && ch < 32) {
        const uint32_t* r = ring + (ch & 1) * 8 * 64;
        uint32_t w[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) w[j] = r[(2 * j) * 64] | (r[(2 * j + 1) * 64] << 16);
        dst[ch * 64] = make_uint4(w[0], w[1], w[2], w[3]);
      }
    }
  }
  if (V == 2) acc ^= ring[(cnt & 15) * 64];
  if (acc == 0x12345678u) sink[0] = cnt;  // keep the work alive
}

int main() {
  const size_t total = (size_t)9 << 20;
  uint4* out;
  uint32_t* sink;
  CHECK(hipMalloc(&out, total * 512));
  CHECK(hipMalloc(&sink, 64));
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  void (*ks[4])(size_t, uint4*, uint32_t*) = {k_probe<0>, k_probe<1>, k_probe<2>, k_probe<3>};
  printf("{");
  for (int v = 0; v < 4; ++v) {
    float best = 1e30f;
    for (int r = 0; r < 6; ++r) {
      CHECK(hipEventRecord(a, 0));
      hipLaunchKernelGGL(ks[v], dim3((unsigned)(total / 256)), dim3(256), 0, 0, total, out, sink);
      CHECK(hipEventRecord(b, 0));
      CHECK(hipEventSynchronize(b));
      float ms;
      CHECK(hipEventElapsedTime(&ms, a, b));
      if (r) best = ms < best ? ms : best;
    }
    printf("%s\"variant%d_ms\": %.4f", v ? ", " : "", v, best);
  }
  printf("}\n");
  return 0;
}
