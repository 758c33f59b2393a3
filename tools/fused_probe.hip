// SampleNTT -> K-PKE.Encrypt fused in one launch, the sampled matrix kept in LDS (VERDICT r4 item 1:
// "measure a fused, wave-specialised SampleNTT -> encrypt-core kernel that keeps A-hat on chip").
//
// k_fused<T, NP, NB>: one persistent workgroup per CU.  Waves 0 .. NP-1 are producers (lane-per-entry
// SHAKE128 with the product's per-lane LDS ring compaction, mlkem.hip compact_block, but the 12-bit
// chunks go to an LDS ring of row-tiles instead of HBM); the other T / 4 waves are consumers, one
// 16-lane group per handshake of a T-handshake tile, running the product's encrypt core
// (mlkem.hip encrypt_core_hs) with the matrix rows read from that ring.  The matrix is streamed one
// row at a time: row-tile r = (tile, row i) holds A[j][i] = SampleNTT(rho || i || j) for the K
// columns j of the T handshakes (K T entries, 384 B each at a 392-B stride).  A producer round fills
// 64 NP / (K T) row-tiles; NB row-tile buffers form the ring.  Hand-off by monotonic LDS counters:
// a producer wave bumps full[b] after its stores (workgroup release), a consumer wave bumps free[b]
// once its four groups hold the row in registers (they read the next row right after the current
// row's basemul, as the product core's prefetch does).  Producers run at s_setprio 2, so the consumer
// waves take the issue slots the producers leave.  Entries that need a 4th SHAKE128 block (~0.7 %,
// the product's fix-up list) are not completed here (FIX4 = false: their handshakes are excluded
// from the comparison) or are completed in the producer lane itself (FIX4 = true: the wave runs the
// extra block whenever any of its lanes needs it).
//
// LDS per CU bounds the producers: every producer lane holds its entry (384 B) for the ~3-block life
// of the entry, so NB row-tile buffers + the compaction rings + the consumer groups' NTT images
// must fit 160 KiB: T = 32, NP = 3, NB = 2 (11 waves, 135 KiB) and T = 16, NP = 3, NB = 6 (7 waves,
// 149 KiB).  k_xof_occ measures what that producer count costs SampleNTT alone: the product's
// SampleNTT role with its workgroups padded to 1..5 per CU (4..20 waves per CU).
//
// Baseline: the product's serial launches k_xof (SampleNTT, 3 blocks), k_xof_fix, k_encrypt_core on
// the same 2^20-handshake ML-KEM-768 chunk; reference ciphertexts from mlkem.hip encaps_impl.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/fused_probe.hip -o tools/fused_probe
#include "../quantum-resistant-p2p_amd/csrc/mlkem.hip"

#include <algorithm>
#include <cstdio>
#include <functional>
#include <set>
#include <string>
#include <vector>

namespace qrk {
thread_local KernelTimer* g_timer = nullptr;
thread_local hipError_t g_launch_err = hipSuccess;
}  // namespace qrk
using namespace qrk;
using namespace qrk::mlkem;

constexpr int KK = 3;      // ML-KEM-768
constexpr int ESTR = 392;  // LDS stride of one entry: 384 B + 8 (consecutive entries 34 banks apart)

template <int T, int NP, int NB>
struct FCfg {
  static constexpr int RT = KK * T;         // entries per row-tile
  static constexpr int RPR = 64 * NP / RT;  // row-tiles per producer round
  static_assert(64 * NP % RT == 0, "a producer round must cover whole row-tiles");
  static_assert(NB >= RPR, "the ring must hold one round");
  static constexpr int NCW = T / 4;  // consumer waves
  static constexpr int THREADS = 64 * (NP + NCW);
  static constexpr int RING = NB * RT * ESTR;
};

__device__ __forceinline__ void wait_ge(uint32_t* c, uint32_t v) {
  while (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < v) __builtin_amdgcn_s_sleep(1);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}
__device__ __forceinline__ void signal(uint32_t* c) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// ---- producer: the product's compaction (mlkem.hip compact_block) into an LDS entry
struct PendL {
  uint32_t r[8];
  int ch = -1;
};
__device__ __forceinline__ void lchunk_store(char* ent, int ch, const uint32_t r[8]) {
  chunk_store((XChunk*)(ent + (ch >> 1) * 24 + (ch & 1) * 12), r);
}
__device__ __forceinline__ void pend_store(PendL& pd, char* ent) {
  if (pd.ch >= 0) {
    lchunk_store(ent, pd.ch, pd.r);
    pd.ch = -1;
  }
}
__device__ __forceinline__ void compact_l(const KState& s, char* ring_all, uint32_t rb, int& cnt, char* ent, PendL& pd) {
  const uint32_t* ring = (const uint32_t*)(ring_all + rb);
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
      *(uint32_t*)(ring_all + and_or3(pos, 0xF00u, rb)) = (uint32_t)c[e];
      pos += c[e] < Q ? 256 : 0;
    }
    cnt = pos >> 8;
    const int ch = before >> 3;
    pend_store(pd, ent);
    if ((cnt >> 3) != ch && ch < 32) {
      const uint32_t* r = ring + (ch & 1) * 8 * 64;
#pragma unroll
      for (int j = 0; j < 8; ++j) pd.r[j] = r[j * 64];
      pd.ch = ch;
    }
  }
}

// ---- consumer: mlkem.hip encrypt_core_hs (MODE 0) with the matrix rows from the LDS ring
template <int T, int NP, int NB>
__device__ __forceinline__ void load_row(const char* ringb, uint32_t* fullc, uint32_t* freec, int r, int g, int L,
                                         PK8 an[KK]) {
  using Cf = FCfg<T, NP, NB>;
  wait_ge(&fullc[r % NB], (uint32_t)(NP * (r / NB + 1)));
#pragma unroll
  for (int j = 0; j < KK; ++j) {
    const uint2* p = (const uint2*)(ringb + ((r % NB) * Cf::RT + j * T + g) * ESTR + 24 * L);
    const uint2 a = p[0], b = p[1], c = p[2];
    an[j] = unpack12(U3{a.x, a.y, b.x}, U3{b.y, c.x, c.y});
  }
  signal(&freec[r % NB]);
}

template <int T, int NP, int NB>
__device__ __forceinline__ void enc_core_fused(size_t C, const uint64_t* __restrict__ prf,
                                               const uint8_t* __restrict__ ek_base, const uint8_t* __restrict__ m_base,
                                               uint8_t* __restrict__ ct, size_t hs, int r0, const char* ringb,
                                               uint32_t* fullc, uint32_t* freec, int g, int L, GroupLds& gl) {
  constexpr int K = KK, DU = P<K>::DU, DV = P<K>::DV;
  const uint8_t* ek = ek_base + hs * P<K>::PK;
  uint8_t* c = ct + hs * P<K>::CT;
  uint32_t diff = 0;
  BOp yb[K];
  {
    CbdRaw yr[K];
#pragma unroll
    for (int j = 0; j < K; ++j) yr[j] = cbd_load<P<K>::ETA1, 64>(prf, (size_t)j * C + hs, L);
#pragma unroll
    for (int j = 0; j < K; ++j) {
      PF16 f;
      cbd_f<P<K>::ETA1>(f, yr[j]);
      contig_to_stride_f(f, (float*)gl.poly, L);
      ntt_fwd_f<false>(f, (float*)gl.poly, L);
      yb[j] = make_bop_f(f, L);
    }
  }
  PK8 an[K];
  load_row<T, NP, NB>(ringb, fullc, freec, r0, g, L, an);
  CbdRaw er = cbd_load<P<K>::ETA2, 64>(prf, (size_t)K * C + hs, L);
  auto row = [&](int i, auto last_t) {
    constexpr bool LAST = decltype(last_t)::value;
    int acc[16];
#pragma unroll
    for (int t = 0; t < 16; ++t) acc[t] = 0;
#pragma unroll
    for (int j = 0; j < K; ++j) basemul_acc(acc, an[j], yb[j]);
    const CbdRaw ecur = er;
    if (!LAST) {
      load_row<T, NP, NB>(ringb, fullc, freec, r0 + i + 1, g, L, an);
    } else {
#pragma unroll
      for (int j = 0; j < K; ++j) {
        const uint2* e = (const uint2*)(ek + 384 * j + 24 * L);
        const uint2 a = e[0], b = e[1], cc = e[2];
        an[j].w[0] = a.x, an[j].w[1] = a.y, an[j].w[2] = b.x, an[j].w[3] = b.y, an[j].w[4] = cc.x, an[j].w[5] = cc.y;
      }
    }
    er = cbd_load<P<K>::ETA2, 64>(prf, (size_t)(K + i + 1) * C + hs, L);
    PF16 uf;
#pragma unroll
    for (int t = 0; t < 16; ++t) uf.v[t] = acc_to_f(acc[t]);
    ntt_inv_f(uf, (float*)gl.poly, L);
    stride_to_contig_f(uf, (float*)gl.poly, L);
    PF16 ef;
    cbd_f<P<K>::ETA2>(ef, ecur);
    P16 u;
#pragma unroll
    for (int t = 0; t < 16; ++t) u.v[t] = compress_f<DU>(uf.v[t] + ef.v[t]);
    pack_bits<DU>(u, gl, L);
    flush_bits<DU>(gl, c + 32 * DU * i, nullptr, diff, true, L);
  };
#pragma unroll 1
  for (int i = 0; i < K - 1; ++i) row(i, std::false_type{});
  row(K - 1, std::true_type{});
  int acc[16];
#pragma unroll
  for (int t = 0; t < 16; ++t) acc[t] = 0;
  bool bad = false;
#pragma unroll
  for (int j = 0; j < K; ++j) {
    const uint64_t a = ((uint64_t)an[j].w[1] << 32) | an[j].w[0], b = ((uint64_t)an[j].w[3] << 32) | an[j].w[2],
                   cc = ((uint64_t)an[j].w[5] << 32) | an[j].w[4];
    basemul_acc(acc, decode12_w(a, b, cc, bad), yb[j]);
  }
  PF16 vf;
#pragma unroll
  for (int t = 0; t < 16; ++t) vf.v[t] = acc_to_f(acc[t]);
  ntt_inv_f(vf, (float*)gl.poly, L);
  stride_to_contig_f(vf, (float*)gl.poly, L);
  PF16 ef;
  cbd_f<P<K>::ETA2>(ef, er);
  const uint8_t* m = m_base + hs * 32;
  const uint32_t mb = (uint32_t)m[2 * L] | ((uint32_t)m[2 * L + 1] << 8);
  P16 v;
#pragma unroll
  for (int t = 0; t < 16; ++t) {
    const float mu = ((mb >> t) & 1) ? (float)((Q + 1) / 2) : 0.0f;
    v.v[t] = compress_f<DV>(vf.v[t] + ef.v[t] + mu);
  }
  pack_bits<DV>(v, gl, L);
  flush_bits<DV>(gl, c + 32 * DU * K, nullptr, diff, true, L);
}

// MODE 0: the fused kernel; timing-only (wrong output) MODE 1: producers only (the consumer waves
// take each row-tile's hand-off and hand it back without reading it), MODE 2: consumers only (the
// producer waves hand over row-tiles without running SHAKE128)
template <int T, int NP, int NB, bool FIX4, int MODE = 0>
__global__ __launch_bounds__(64 * (NP + T / 4)) void k_fused(const uint64_t* __restrict__ rho,
                                                                    const uint64_t* __restrict__ prf, size_t C,
                                                                    const uint8_t* __restrict__ pk,
                                                                    const uint8_t* __restrict__ coins,
                                                                    uint8_t* __restrict__ ct, int ntiles) {
  using Cf = FCfg<T, NP, NB>;
  __shared__ __attribute__((aligned(16))) char ringb[Cf::RING];
  __shared__ __attribute__((aligned(16))) uint32_t crings[NP * 16 * 64];
  __shared__ GroupLds glds[T];
  __shared__ uint32_t fullc[NB], freec[NB];
  if (threadIdx.x < NB) fullc[threadIdx.x] = freec[threadIdx.x] = 0;
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const unsigned G = gridDim.x;
  if (wave < NP) {
    __builtin_amdgcn_s_setprio(2);
    const uint32_t rb = (uint32_t)(wave * 16 * 64 + lane) * 4;
    const int nrounds = ntiles * KK / Cf::RPR;
    const int k = 64 * wave + lane;
#pragma unroll 1
    for (int q = 0; q < nrounds; ++q) {
      const int r = q * Cf::RPR + k / Cf::RT, e = k % Cf::RT, j = e / T, hl = e % T;
      const int tile = r / KK, i = r % KK;
      const size_t hs = ((size_t)tile * G + blockIdx.x) * T + hl;
      char* ent = ringb + (r % NB) * Cf::RT * ESTR + e * ESTR;
      if constexpr (MODE == 2) {
#pragma unroll
        for (int x = 0; x < Cf::RPR; ++x) {
          const int rr = q * Cf::RPR + x;
          wait_ge(&freec[rr % NB], (uint32_t)(Cf::NCW * (rr / NB)));
        }
#pragma unroll
        for (int x = 0; x < Cf::RPR; ++x) signal(&fullc[(q * Cf::RPR + x) % NB]);
        continue;
      }
      KState s;
      xof_init(s, rho + hs * 4, i * KK + j, KK);
      int cnt = 0;
      PendL pd;
      keccak_f(s);
      // the round's buffers: their previous row-tiles read by every consumer wave
#pragma unroll
      for (int x = 0; x < Cf::RPR; ++x) {
        const int rr = q * Cf::RPR + x;
        wait_ge(&freec[rr % NB], (uint32_t)(Cf::NCW * (rr / NB)));
      }
      compact_l(s, (char*)crings, rb, cnt, ent, pd);
#pragma unroll 1
      for (int b = 1; b < 3; ++b) {
        keccak_f(s);
        compact_l(s, (char*)crings, rb, cnt, ent, pd);
      }
      if constexpr (FIX4) {
#pragma unroll 1
        for (int b = 3; b < MAX_XOF_BLOCKS && cnt < 256; ++b) {
          keccak_f(s);
          compact_l(s, (char*)crings, rb, cnt, ent, pd);
        }
      }
      pend_store(pd, ent);
#pragma unroll
      for (int x = 0; x < Cf::RPR; ++x) signal(&fullc[(q * Cf::RPR + x) % NB]);
    }
  } else {
    const int g = (wave - NP) * 4 + (lane >> 4), L = lane & 15;
    if constexpr (MODE == 1) {
#pragma unroll 1
      for (int r = 0; r < ntiles * KK; ++r) {
        wait_ge(&fullc[r % NB], (uint32_t)(NP * (r / NB + 1)));
        signal(&freec[r % NB]);
      }
      return;
    }
#pragma unroll 1
    for (int t = 0; t < ntiles; ++t) {
      const size_t hs = ((size_t)t * G + blockIdx.x) * T + g;
      enc_core_fused<T, NP, NB>(C, prf, pk, coins, ct, hs, t * KK, ringb, fullc, freec, g, L, glds[g]);
    }
  }
}

// the product's SampleNTT role with each 256-thread workgroup padded (dynamic LDS) to `per_cu` per CU
template <class R>
__global__ __launch_bounds__(256) void k_xof_occ(R r) {
  extern __shared__ __attribute__((aligned(16))) char dyn[];
  r.run(blockIdx.x, dyn);
}

__global__ void k_fill(uint8_t* p, size_t nbytes, uint64_t seed) {  // synthetic keys / coins
  const size_t w = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (w * 8 >= nbytes) return;
  uint64_t x = (w + 1) * 0x9E3779B97F4A7C15ull ^ seed;
  x ^= x >> 31, x *= 0xBF58476D1CE4E5B9ull, x ^= x >> 29, x *= 0x94D049BB133111EBull, x ^= x >> 32;
  ((uint64_t*)p)[w] = x;
}
__global__ void k_rowdiff(const uint8_t* a, const uint8_t* b, size_t n, size_t len, uint8_t* flag) {
  const size_t h = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (h >= n) return;
  uint32_t d = 0;
  for (size_t x = 0; x < len; x += 8) d |= *(const uint64_t*)(a + h * len + x) != *(const uint64_t*)(b + h * len + x);
  flag[h] = (uint8_t)d;
}

template <int T_, int NP_, int NB_, bool F4_, int M_ = 0>
struct Tag {
  static constexpr int T = T_, NP = NP_, NB = NB_, M = M_;
  static constexpr bool F4 = F4_;
};

// argv[1] (optional): time only the variants whose name contains it (PMC passes)
int main(int argc, char** argv) {
  const std::string only = argc > 1 ? argv[1] : "";
  const size_t n = 1 << 20, C = n;
  const int PK = P<KK>::PK, CT = P<KK>::CT;
  uint8_t *pk, *coins, *ct_ref, *ct_f, *ss, *flag;
  int32_t* status;
  void* scratch;
  hipMalloc(&pk, n * PK);
  hipMalloc(&coins, n * 32);
  hipMalloc(&ct_ref, n * CT);
  hipMalloc(&ct_f, n * CT);
  hipMalloc(&ss, n * 32);
  hipMalloc(&status, n * 4);
  hipMalloc(&flag, n);
  hipMalloc(&scratch, scratch_words(KK, C) * 8);
  hipLaunchKernelGGL(k_fill, dim3((unsigned)((n * PK / 8 + 255) / 256)), dim3(256), 0, 0, pk, n * PK, 0x1234ull);
  hipLaunchKernelGGL(k_fill, dim3((unsigned)((n * 4 + 255) / 256)), dim3(256), 0, 0, coins, n * 32, 0x5678ull);
  Streams s;
  s.main = 0;
  s.serial = true;
  encaps_impl<KK>(n, ct_ref, ss, pk, coins, status, scratch, s);  // reference ct; leaves rho copy + PRF words
  hipDeviceSynchronize();
  const ScratchView v = carve(scratch, KK, C);
  uint32_t nfix = 0;
  hipMemcpy(&nfix, v.nfix, 4, hipMemcpyDeviceToHost);
  std::vector<uint32_t> fix(nfix);
  hipMemcpy(fix.data(), v.fix, 4 * (size_t)nfix, hipMemcpyDeviceToHost);
  std::set<size_t> fix_hs;
  for (uint32_t e : fix) fix_hs.insert(e % C);

  const RXof<KK, false> xr = xof_role<KK>((const uint8_t*)v.rho, n, C, v);
  const RXof<KK, true> fr = fix_role<KK>((const uint8_t*)v.rho, n, C, v);
  const RCore<KK, 0> core{n, C, v.xof, v.prf, pk, (size_t)PK, coins, (size_t)32, ct_ref, status, v.kprime, v.kbar,
                          nullptr, (unsigned)((n + GROUPS - 1) / GROUPS)};
  const unsigned G = 256;
  struct Var {
    std::string name;
    std::function<void()> launch;
  };
  std::vector<Var> vars;
  vars.push_back({"xof", [&] {
                    hipMemsetAsync(v.nfix, 0, 4, 0);
                    hipLaunchKernelGGL((k_role<RXof<KK, false>>), dim3(xr.nb), dim3(256), 0, 0, xr);
                  }});
  vars.push_back({"fix", [&] { hipLaunchKernelGGL((k_role<RXof<KK, true>>), dim3(fr.nb), dim3(256), 0, 0, fr); }});
  vars.push_back({"core", [&] { hipLaunchKernelGGL((k_role<RCore<KK, 0>>), dim3(core.nb), dim3(256), 0, 0, core); }});
  auto add_fused = [&](auto tag, const char* name) {
    using Tg = decltype(tag);
    constexpr int T = Tg::T, NP = Tg::NP, NB = Tg::NB, M = Tg::M;
    constexpr bool F4 = Tg::F4;
    const int ntiles = (int)(n / ((size_t)T * G));
    vars.push_back({name, [=] {
                      hipLaunchKernelGGL((k_fused<T, NP, NB, F4, M>), dim3(G), dim3(FCfg<T, NP, NB>::THREADS), 0, 0,
                                         (const uint64_t*)v.rho, (const uint64_t*)v.prf, C, pk, coins, ct_f, ntiles);
                    }});
  };
  add_fused(Tag<32, 3, 2, false>{}, "fused_t32_np3_nb2");
  add_fused(Tag<32, 3, 2, true>{}, "fused_t32_np3_nb2_fix4");
  add_fused(Tag<16, 3, 6, false>{}, "fused_t16_np3_nb6");
  add_fused(Tag<16, 3, 6, true>{}, "fused_t16_np3_nb6_fix4");
  add_fused(Tag<16, 3, 6, true, 1>{}, "timing_t16_np3_nb6_fix4_producers_only");
  add_fused(Tag<16, 3, 6, true, 2>{}, "timing_t16_np3_nb6_consumers_only");
  hipFuncSetAttribute((const void*)k_xof_occ<RXof<KK, false>>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  for (int per_cu = 1; per_cu <= 5; ++per_cu) {
    const size_t dyn = std::max<size_t>(XOF_LDS, (163840 / per_cu - 512) & ~(size_t)255);
    vars.push_back({"xof_" + std::to_string(per_cu) + "wg_per_cu", [=] {
                      hipMemsetAsync(v.nfix, 0, 4, 0);
                      hipLaunchKernelGGL((k_xof_occ<RXof<KK, false>>), dim3(xr.nb), dim3(256), dyn, 0, xr);
                    }});
  }
  if (!only.empty())
    vars.erase(std::remove_if(vars.begin(), vars.end(), [&](const Var& x) { return x.name.find(only) == std::string::npos; }),
               vars.end());
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int w = 0; w < 3; ++w)
    for (auto& x : vars) x.launch();
  hipError_t err = hipDeviceSynchronize();
  if (err != hipSuccess) {
    printf("{\"hip\": \"%s\"}\n", hipGetErrorString(err));
    return 1;
  }
  std::vector<std::vector<float>> t(vars.size());
  for (int r = 0; r < 7; ++r)
    for (size_t i = 0; i < vars.size(); ++i) {
      hipEventRecord(e0, 0);
      for (int k = 0; k < 3; ++k) vars[i].launch();
      hipEventRecord(e1, 0);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      t[i].push_back(ms / 3);
    }
  // parity of each fused variant against the product's ciphertexts
  printf("{\"alg\": \"ML-KEM-768\", \"handshakes\": %zu, \"fixup_entries\": %u, \"fixup_handshakes\": %zu, "
         "\"ms_per_2p20\": {",
         n, nfix, fix_hs.size());
  for (size_t i = 0; i < vars.size(); ++i) {
    auto v2 = t[i];
    std::sort(v2.begin(), v2.end());
    printf("%s\"%s\": %.4f", i ? ", " : "", vars[i].name.c_str(), v2[v2.size() / 2]);
  }
  printf("}, \"parity\": {");
  bool first = true;
  int rc = 0;
  for (size_t i = 0; i < vars.size(); ++i) {
    if (vars[i].name.rfind("fused", 0) != 0) continue;
    hipMemset(ct_f, 0, n * CT);
    vars[i].launch();
    hipLaunchKernelGGL(k_rowdiff, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, ct_f, ct_ref, n, (size_t)CT, flag);
    std::vector<uint8_t> f(n);
    hipMemcpy(f.data(), flag, n, hipMemcpyDeviceToHost);
    size_t bad = 0, bad_nonfix = 0;
    for (size_t h = 0; h < n; ++h)
      if (f[h]) ++bad, bad_nonfix += fix_hs.count(h) == 0;
    const bool fix4 = vars[i].name.find("fix4") != std::string::npos;
    if (bad_nonfix || (fix4 && bad)) rc = 1;
    printf("%s\"%s\": {\"rows_differ\": %zu, \"rows_differ_outside_fixup\": %zu}", first ? "" : ", ",
           vars[i].name.c_str(), bad, bad_nonfix);
    first = false;
  }
  err = hipDeviceSynchronize();
  printf("}, \"hip\": \"%s\"}\n", hipGetErrorString(err));
  return err == hipSuccess ? rc : 1;
}
