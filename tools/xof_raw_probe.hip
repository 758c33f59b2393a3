// SampleNTT placement: producer-side compaction (the product, k_xof's ring) against a raw squeeze +
// acceptance mask with the placement done by the consumer ("take SampleNTT
// acceptance and compaction out of k_xof, measured rather than estimated").
//
// Four kernels over the 2^20-handshake ML-KEM-768 matrix (9 entries per handshake):
//   ring   the product's SampleNTT role (mlkem.hip RXof, included as-is): 3 blocks, 12-bit chunk
//          pairs written by the per-lane LDS ring compaction
//   raw    3 blocks, the 504 squeezed bytes stored as 63 tiled u64 words + an 11-dword acceptance
//          mask (one v_cmp + one v_addc per candidate, bit-reversed per dword at the end)
//   load   the consumer as the encrypt core reads the product's output today: each of 16 lanes
//          per entry loads its 24 contiguous bytes and spreads them into 8 packed int16 pairs
//   place  the consumer on the raw layout: the group stages the entry's 504 B in LDS, each lane
//          finds the first of its 16 accepted candidates from popcount prefix sums of the mask and
//          extracts them (two LDS dwords + a funnel shift per coefficient)
// ring + load is the shipped pipeline's SampleNTT cost, raw + place the proposed one (fix-up
// entries, ~0.7 %, are excluded from the comparison of the two outputs, which must be equal).
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/xof_raw_probe.hip -o xof_raw_probe
#include "../quantum-resistant-p2p_amd/csrc/mlkem.hip"

#include <algorithm>
#include <cstdio>
#include <vector>

namespace qrk {
thread_local KernelTimer* g_timer = nullptr;
thread_local hipError_t g_launch_err = hipSuccess;
}  // namespace qrk
using namespace qrk;
using namespace qrk::mlkem;

constexpr int KK = 3;          // ML-KEM-768
constexpr int RAW_W = 63;      // u64 words per entry (3 SHAKE128 blocks of 21)
constexpr int MASK_W = 12;     // 11 mask dwords + 1 pad per entry

__global__ __launch_bounds__(256) void k_xof_raw(const uint8_t* __restrict__ rho, size_t n, size_t C,
                                                 uint64_t* __restrict__ raw, uint32_t* __restrict__ mask,
                                                 uint32_t* __restrict__ nfix) {
  const size_t inst = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (inst >= (size_t)KK * KK * C || inst % C >= n) return;
  KState s;
  xof_init(s, (const uint64_t*)(rho + (inst % C) * 32), (int)(inst / C), KK);
  uint32_t m[11];
#pragma unroll
  for (int d = 0; d < 11; ++d) m[d] = 0;
#pragma unroll 1
  for (int b = 0; b < 3; ++b) {
    keccak_f(s);
#pragma unroll
    for (int w = 0; w < 21; ++w) raw[tidx<64>(inst, 21 * b + w, RAW_W)] = kword(s, w);
    // m[d] = 2 m[d] + (c < q): candidate j of the entry ends at bit 31 - (j mod 32) after 32 steps
    // (blocks hold 112 candidates: 3.5 dwords, so the dword index is per block and candidate)
#pragma unroll
    for (int t = 0; t < 14; ++t) {
      uint32_t dd[3];
#pragma unroll
      for (int e = 0; e < 3; ++e) {
        const int di = 3 * t + e;
        dd[e] = (di & 1) ? s.a[di >> 1].hi : s.a[di >> 1].lo;
      }
      int c[8];
      split12(dd[0], dd[1], dd[2], c);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int j = 112 * b + 8 * t + e;
        m[j >> 5] = 2 * m[j >> 5] + (c[e] < Q ? 1u : 0u);
      }
    }
  }
  // the last dword holds 16 candidates (336 = 10 * 32 + 16): shift them to the top first
  m[10] <<= 16;
  int cnt = 0;
#pragma unroll
  for (int d = 0; d < 11; ++d) {
    m[d] = __builtin_bitreverse32(m[d]);  // candidate 32 d + k at bit k
    cnt += __builtin_popcount(m[d]);
  }
  uint32_t* mo = mask + inst * MASK_W;
#pragma unroll
  for (int d = 0; d < 11; ++d) mo[d] = m[d];
  if (cnt < 256) atomicAdd(nfix, 1u);
}

struct Pk8Out {
  uint4 a, b;
};

// the product's consumer read (mlkem.hip load_sampled on the packed 12-bit layout)
__global__ __launch_bounds__(256) void k_load(const uint64_t* __restrict__ xof, size_t nent, Pk8Out* __restrict__ out) {
  const size_t e = (size_t)blockIdx.x * 16 + (threadIdx.x >> 4);
  const int L = threadIdx.x & 15;
  if (e >= nent) return;
  const PK8 p = load_sampled<64, true>(xof, e, L);
  out[e * 16 + L] = {make_uint4(p.w[0], p.w[1], p.w[2], p.w[3]), make_uint4(p.w[4], p.w[5], p.w[6], p.w[7])};
}

// consumer-side placement on the raw layout
__global__ __launch_bounds__(256) void k_place(const uint64_t* __restrict__ raw, const uint32_t* __restrict__ mask,
                                               size_t nent, Pk8Out* __restrict__ out) {
  __shared__ uint32_t st[16][128];  // the group's entry: 126 dwords + 2 pad
  __shared__ uint32_t sm[16][12];
  const int g = threadIdx.x >> 4, L = threadIdx.x & 15;
  const size_t e = (size_t)blockIdx.x * 16 + g;
  const bool active = e < nent;
  const size_t es = active ? e : nent - 1;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int w = L + 16 * k;
    if (w < RAW_W) {
      const uint64_t v = raw[tidx<64>(es, w, RAW_W)];
      st[g][2 * w] = (uint32_t)v;
      st[g][2 * w + 1] = (uint32_t)(v >> 32);
    }
  }
  if (L < 12) sm[g][L] = mask[es * MASK_W + L];
  if (L < 2) st[g][126 + L] = 0;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  // popcount prefix: the dword holding accepted candidate number R = 16 L, and its rank there
  const uint32_t R = 16u * (uint32_t)L;
  uint32_t before = 0;
  int d0 = 0;
  uint32_t pre = 0;
#pragma unroll
  for (int d = 0; d < 11; ++d) {
    const uint32_t c = __builtin_popcount(sm[g][d]);
    const bool here = before <= R && R < before + c;
    d0 = here ? d : d0;
    pre = here ? before : pre;
    before += c;
  }
  int d = d0;
  uint32_t cur = sm[g][d];
  for (uint32_t skip = R - pre; skip; --skip) cur &= cur - 1;  // drop the lower-ranked ones
  uint32_t r[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    while (cur == 0 && d < 10) cur = sm[g][++d];  // bounded: a fix-up entry may run out
    if (cur == 0) {
      r[k] = 0;
      continue;
    }
    const uint32_t j = 32u * (uint32_t)d + (uint32_t)__builtin_ctz(cur);
    cur &= cur - 1;
    const uint32_t bo = j + (j >> 1);  // byte offset of candidate j: 12 j / 8
    const uint32_t w0 = st[g][bo >> 2], w1 = st[g][(bo >> 2) + 1];
    const uint32_t x = __builtin_amdgcn_alignbit(w1, w0, (bo & 3) * 8);
    r[k] = (x >> ((j & 1) * 4)) & 0xFFFu;
  }
  if (active) {
    uint32_t w[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) w[k] = r[2 * k] | (r[2 * k + 1] << 16);
    out[e * 16 + L] = {make_uint4(w[0], w[1], w[2], w[3]), make_uint4(w[4], w[5], w[6], w[7])};
  }
}

// entries whose 3 blocks hold fewer than 256 accepted values (the fix-up's) are skipped
__global__ void k_cmp(const Pk8Out* a, const Pk8Out* b, const uint32_t* mask, size_t nent, unsigned long long* bad,
                      unsigned long long* skipped) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= nent * 16) return;
  const size_t e = i / 16;
  int cnt = 0;
  for (int d = 0; d < 11; ++d) cnt += __builtin_popcount(mask[e * MASK_W + d]);
  if (cnt < 256) {
    if ((i & 15) == 0) atomicAdd(skipped, 1ull);
    return;
  }
  const Pk8Out x = a[i], y = b[i];
  if (x.a.x != y.a.x || x.a.y != y.a.y || x.a.z != y.a.z || x.a.w != y.a.w || x.b.x != y.b.x || x.b.y != y.b.y ||
      x.b.z != y.b.z || x.b.w != y.b.w)
    atomicAdd(bad, 1ull);
}

__global__ void k_rho(uint64_t* rho, size_t n) {  // synthetic per-handshake rho
  const size_t t = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (t < 4 * n) rho[t] = 0x9E3779B97F4A7C15ull * (t + 1) ^ (t << 29);
}

int main() {
  const size_t n = 1 << 20, C = n, nent = (size_t)KK * KK * C;
  uint64_t *rho, *xof, *raw;
  uint32_t *fix, *nfix, *mask;
  Pk8Out *oa, *ob;
  unsigned long long* dbg;
  hipMalloc(&rho, 32 * n);
  hipMalloc(&xof, nent * XOF_W * 8);
  hipMalloc(&raw, nent * RAW_W * 8 + 64 * 8);
  hipMalloc(&mask, nent * MASK_W * 4);
  hipMalloc(&fix, nent * 4);
  hipMalloc(&nfix, 8);
  hipMalloc(&oa, nent * 16 * sizeof(Pk8Out));
  hipMalloc(&ob, nent * 16 * sizeof(Pk8Out));
  hipMalloc(&dbg, 16);
  hipLaunchKernelGGL(k_rho, dim3((unsigned)((4 * n + 255) / 256)), dim3(256), 0, 0, rho, n);
  const RXof<KK, false> ring{{(const uint8_t*)rho, 32, n, C, (XUnit*)xof, fix, nfix}, (unsigned)((nent + 255) / 256)};
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const unsigned gx = (unsigned)((nent + 255) / 256), gc = (unsigned)((nent + 15) / 16);
  auto ring_l = [&] {
    hipMemsetAsync(nfix, 0, 4, 0);
    hipLaunchKernelGGL((k_role<RXof<KK, false>>), dim3(ring.nb), dim3(256), 0, 0, ring);
  };
  auto raw_l = [&] {
    hipMemsetAsync(nfix + 1, 0, 4, 0);
    hipLaunchKernelGGL(k_xof_raw, dim3(gx), dim3(256), 0, 0, (const uint8_t*)rho, n, C, raw, mask, nfix + 1);
  };
  auto load_l = [&] { hipLaunchKernelGGL(k_load, dim3(gc), dim3(256), 0, 0, xof, nent, oa); };
  auto place_l = [&] { hipLaunchKernelGGL(k_place, dim3(gc), dim3(256), 0, 0, raw, mask, nent, ob); };
  // warm-up (clocks up, every kernel's code loaded), then 7 rounds with the four kernels
  // interleaved, 5 launches each; the median round is reported
  for (int i = 0; i < 20; ++i) ring_l(), raw_l(), load_l(), place_l();
  std::vector<float> tr, tw, tl, tp;
  auto timeit = [&](auto launch) {
    hipEventRecord(e0, 0);
    for (int i = 0; i < 5; ++i) launch();
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    return ms / 5;
  };
  for (int r = 0; r < 7; ++r) {
    tr.push_back(timeit(ring_l));
    tw.push_back(timeit(raw_l));
    tl.push_back(timeit(load_l));
    tp.push_back(timeit(place_l));
  }
  auto med = [](std::vector<float> v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
  };
  const float t_ring = med(tr), t_raw = med(tw), t_load = med(tl), t_place = med(tp);
  // the outputs compared below come from the last launch of each kernel
  ring_l();
  raw_l();
  load_l();
  place_l();
  hipMemset(dbg, 0, 16);
  hipLaunchKernelGGL(k_cmp, dim3((unsigned)((nent * 16 + 255) / 256)), dim3(256), 0, 0, oa, ob, mask, nent, dbg, dbg + 1);
  unsigned long long h[2];
  uint32_t nf[2];
  hipMemcpy(h, dbg, 16, hipMemcpyDeviceToHost);
  hipMemcpy(nf, nfix, 8, hipMemcpyDeviceToHost);
  const hipError_t err = hipDeviceSynchronize();
  printf("{\"alg\": \"ML-KEM-768\", \"handshakes\": %zu, \"entries\": %zu, \"ms_per_launch\": {\"ring_producer\": %.4f, "
         "\"raw_producer\": %.4f, \"load_consumer\": %.4f, \"place_consumer\": %.4f}, "
         "\"shipped_ring_plus_load\": %.4f, \"proposed_raw_plus_place\": %.4f, \"fixup_entries\": [%u, %u], "
         "\"compared_lanes_mismatched\": %llu, \"entries_skipped_need_4th_block\": %llu, \"hip\": \"%s\"}\n",
         n, nent, t_ring, t_raw, t_load, t_place, t_ring + t_load, t_raw + t_place, nf[0], nf[1], h[0], h[1],
         hipGetErrorString(err));
  return err == hipSuccess && h[0] == 0 ? 0 : 1;
}
