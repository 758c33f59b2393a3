// FrodoKEM-640/976/1344-SHAKE (round-3 specification) batched KeyGen / Encaps /
// Decaps for gfx950.
//
// Replaces liboqs's FrodoKEM behind OQS_KEM_keypair / encaps / decaps
// (quantum_resistant_p2p/vendor/oqs.py:318, 348, 372) for the variants
// FrodoKEMKeyExchange selects (quantum_resistant_p2p/crypto/key_exchange.py:332-343).
//
// Work per Encaps (640): Gen(A) = 640 rows x 8 SHAKE128 blocks = 5,120 Keccak
// permutations; S'A = 3.3 M multiply-adds mod 2^16.  Kernels:
//
//   k_fr_front_enc    lane / hs   pkh = H(pk); (seedSE || k) = H(pkh || mu)
//   k_fr_dec_m        wave / hs   M = C - B'S, mu' = Decode(M)               (VALU)
//   k_fr_g2_dec       lane / hs   (seedSE' || k') = H(pkh || mu')
//   k_fr_se_stream    lane / hs   SHAKE(0x96 || seedSE) raw words (123 perms, sequential)
//   k_fr_sample       thread / 4 words   CDF sampler -> S' (int8, zero-padded), E', E''
//   k_fr_gen_at       lane / row  Gen(A) row r -> balanced int8 limbs, written as
//                                  transposed byte planes T[c][r] via an LDS stage
//   k_fr_mm           wave / 16 cols    B' = S'A + E' on v_mfma_i32_16x16x64_i8:
//                                  A = 256*hi + lo (balanced int8 limbs), two i8 MFMAs per
//                                  K-step, int32 accumulation -> exact mod 2^16
//   k_fr_pack         wave / hs   V = S'B + E'', C = V + Encode(mu), Pack(B', C);
//                                  decaps: compare with ct, select k' or s (constant time)
//   k_fr_ss           lane / hs   ss = H(ct || k)
// KeyGen: k_fr_kg_front (seedA, SHAKE(0x5F || seedSE) stream), k_fr_sample,
// k_fr_kg_rows (lane / row: Gen(A) row and B = AS + E on VALU), k_fr_kg_pack.
#include "keccak.cuh"
#include "qrkem_internal.h"

namespace qrk {
namespace frodo {

typedef int v4i __attribute__((ext_vector_type(4)));

constexpr int NBAR = 8;
constexpr int SUB = 256;  // handshakes per Gen(A) / MFMA sub-chunk (A planes stay in the 256 MiB MALL for n = 640)

template <int N_>
struct FP {
  static constexpr int N = N_;
  static constexpr int LOGQ = N_ == 640 ? 15 : 16;
  static constexpr uint32_t QMASK = (1u << LOGQ) - 1;
  static constexpr int EB = N_ == 640 ? 2 : (N_ == 976 ? 3 : 4);  // bits extracted per coefficient
  static constexpr int SEC = N_ == 640 ? 16 : (N_ == 976 ? 24 : 32);
  static constexpr int RW = N_ == 640 ? 21 : 17;  // rate (words) of the hash SHAKE (128 vs 256)
  static constexpr int PK = 16 + LOGQ * N;
  static constexpr int CT = LOGQ * N + LOGQ * NBAR;
  static constexpr int SK = SEC + PK + 2 * N * NBAR + SEC;
  static constexpr int MU = EB * NBAR;  // bytes
  static constexpr int NP = (N + 127) / 128 * 128;  // padded row pitch of S' / A planes
  static constexpr int SE_WORDS = (2 * N + NBAR) * NBAR * 2 / 8;  // encaps sampler stream (u64)
  static constexpr int KG_WORDS = 2 * N * NBAR * 2 / 8;           // keygen sampler stream (u64)
  static constexpr int A_BLOCKS = (2 * N + 167) / 168;            // SHAKE128 blocks per row of A
};

template <int N>
__device__ __forceinline__ int cdf_sample(uint32_t r) {
  // CDF tables of the round-3 parameter sets (FrodoKEM spec, Table 3)
  constexpr uint16_t T640[12] = {4643, 13363, 20579, 25843, 29227, 31145, 32103, 32525, 32689, 32745, 32762, 32766};
  constexpr uint16_t T976[10] = {5638, 15915, 23689, 28571, 31116, 32217, 32613, 32731, 32760, 32766};
  constexpr uint16_t T1344[6] = {9142, 23462, 30338, 32361, 32725, 32765};
  const int prnd = (int)((r & 0xFFFF) >> 1);
  int s = 0;
  if constexpr (N == 640) {
#pragma unroll
    for (int t = 0; t < 12; ++t) s += (int)T640[t] < prnd;
  } else if constexpr (N == 976) {
#pragma unroll
    for (int t = 0; t < 10; ++t) s += (int)T976[t] < prnd;
  } else {
#pragma unroll
    for (int t = 0; t < 6; ++t) s += (int)T1344[t] < prnd;
  }
  return (r & 1) ? -s : s;
}

__device__ __forceinline__ size_t tidx(size_t hs, int w, int W) {
  return ((hs >> 6) * (size_t)W + (size_t)w) * 64 + (hs & 63);
}

// ---------------------------------------------------------------- scratch
template <int N>
struct View {
  uint64_t* raw;   // sampler stream, tiled [C/64][W][64]
  int8_t* sp8;     // S' (or S^T for KeyGen) int8 [C][8][NP], zero padded
  int16_t* ep16;   // E' [C][8][N]   (KeyGen: E [C][N][8])
  int16_t* epp16;  // E'' [C][64]
  uint16_t* bp16;  // B' = S'A + E' masked [C][8][N]   (KeyGen: B [C][N][8])
  uint64_t* seeds; // per hs 16 u64: seedSE | k | pkh | mu'  (4 x 32 B)
  uint64_t* kk;    // per hs 4 u64: key fed to the final hash
  uint8_t* tlo;    // A planes [SUB][N][NP] (lo limb), transposed: T[c][r] = limb(A[r][c])
  uint8_t* thi;
};

inline size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

template <int N>
size_t scratch_bytes_t(size_t C) {
  using P = FP<N>;
  const size_t W = (size_t)(P::SE_WORDS > P::KG_WORDS ? P::SE_WORDS : P::KG_WORDS);
  return al256(C * W * 8) + al256(C * 8 * P::NP) + al256(C * 8 * N * 2) + al256(C * 64 * 2) + al256(C * 8 * N * 2) +
         al256(C * 128) + al256(C * 32) + 2 * al256((size_t)SUB * N * P::NP);
}

template <int N>
View<N> carve(void* base, size_t C) {
  using P = FP<N>;
  const size_t W = (size_t)(P::SE_WORDS > P::KG_WORDS ? P::SE_WORDS : P::KG_WORDS);
  uint8_t* p = (uint8_t*)base;
  View<N> v;
  v.raw = (uint64_t*)p;
  p += al256(C * W * 8);
  v.sp8 = (int8_t*)p;
  p += al256(C * 8 * P::NP);
  v.ep16 = (int16_t*)p;
  p += al256(C * 8 * N * 2);
  v.epp16 = (int16_t*)p;
  p += al256(C * 64 * 2);
  v.bp16 = (uint16_t*)p;
  p += al256(C * 8 * N * 2);
  v.seeds = (uint64_t*)p;
  p += al256(C * 128);
  v.kk = (uint64_t*)p;
  p += al256(C * 32);
  v.tlo = p;
  p += al256((size_t)SUB * N * P::NP);
  v.thi = p;
  return v;
}

// absorb a short message of NB bytes (NB <= 8*RW - 1) held in words w[] (little-endian)
template <int RW, int NW>
__device__ __forceinline__ void absorb_short(KState& s, const uint64_t* w, int nbytes) {
#pragma unroll
  for (int i = 0; i < NW; ++i) kxor(s, i, w[i]);
  // domain byte 0x1F at byte nbytes (caller guarantees nbytes < 8*RW)
  const int wi = nbytes >> 3, sh = 8 * (nbytes & 7);
#pragma unroll
  for (int i = 0; i <= NW; ++i)
    if (i == wi) kxor(s, i, (uint64_t)DS_SHAKE << sh);
  s.a[RW - 1].hi ^= 0x80000000u;
  keccak_f(s);
}

// squeeze W words of an already-absorbed sponge into the tiled raw stream of hs
template <int RW>
__device__ __forceinline__ void squeeze_tiled(KState& s, uint64_t* raw, size_t hs, int W, int RAWW) {
  int w = 0;
#pragma unroll 1
  while (true) {
#pragma unroll
    for (int i = 0; i < RW; ++i)
      if (w + i < W) raw[tidx(hs, w + i, RAWW)] = kword(s, i);
    w += RW;
    if (w >= W) break;
    keccak_f(s);
  }
}

// ---------------------------------------------------------------- Encaps front: pkh, G2
template <int N>
__global__ __launch_bounds__(256) void k_fr_front_enc(const uint8_t* __restrict__ pk, const uint8_t* __restrict__ mu,
                                                      size_t n, uint64_t* __restrict__ seeds) {
  using P = FP<N>;
  const size_t hs = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (hs >= n) return;
  const uint64_t* pkw = (const uint64_t*)(pk + hs * P::PK);
  KState s;
  kzero(s);
  absorb_words<P::RW, P::PK / 8, DS_SHAKE>(s, [&](int w) { return pkw[w]; });
  uint64_t in[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // pkh || mu: SEC + MU <= 64 bytes
#pragma unroll
  for (int w = 0; w < P::SEC / 8; ++w) in[w] = kword(s, w);
  const uint64_t* muw = (const uint64_t*)(mu + hs * P::MU);
#pragma unroll
  for (int w = 0; w < P::MU / 8; ++w) in[P::SEC / 8 + w] = muw[w];
  uint64_t* sd = seeds + hs * 16;
#pragma unroll
  for (int w = 0; w < P::SEC / 8; ++w) sd[8 + w] = in[w];  // pkh
  kzero(s);
  absorb_short<P::RW, 8>(s, in, P::SEC + P::MU);
#pragma unroll
  for (int w = 0; w < 2 * P::SEC / 8; ++w) sd[w] = kword(s, w);  // seedSE || k
}

// Decaps: (seedSE' || k') = H(pkh || mu'), pkh from sk, mu' from seeds[12..]
template <int N>
__global__ __launch_bounds__(256) void k_fr_g2_dec(const uint8_t* __restrict__ sk, size_t n,
                                                   uint64_t* __restrict__ seeds) {
  using P = FP<N>;
  const size_t hs = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (hs >= n) return;
  const uint64_t* pkh = (const uint64_t*)(sk + hs * P::SK + P::SEC + P::PK + 2 * N * NBAR);
  uint64_t* sd = seeds + hs * 16;
  uint64_t in[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
  for (int w = 0; w < P::SEC / 8; ++w) in[w] = pkh[w];
#pragma unroll
  for (int w = 0; w < P::MU / 8; ++w) in[P::SEC / 8 + w] = sd[12 + w];
  KState s;
  kzero(s);
  absorb_short<P::RW, 8>(s, in, P::SEC + P::MU);
#pragma unroll
  for (int w = 0; w < 2 * P::SEC / 8; ++w) sd[w] = kword(s, w);
}

// SHAKE(domain || seedSE) sampler stream, W words, one lane per handshake
template <int N>
__global__ __launch_bounds__(256) void k_fr_se_stream(const uint64_t* __restrict__ seeds, size_t n, int domain,
                                                      int W, int RAWW, uint64_t* __restrict__ raw) {
  using P = FP<N>;
  const size_t hs = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (hs >= n) return;
  const uint64_t* sd = seeds + hs * 16;
  uint64_t in[5] = {0, 0, 0, 0, 0};  // domain byte || seedSE (SEC bytes): shift by one byte
  uint64_t prev = (uint64_t)domain;
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    const uint64_t x = w < P::SEC / 8 ? sd[w] : 0;
    in[w] = prev | (x << 8);
    prev = x >> 56;
  }
  in[4] = prev;
  KState s;
  kzero(s);
  absorb_short<P::RW, 5>(s, in, 1 + P::SEC);
  squeeze_tiled<P::RW>(s, raw, hs, W, RAWW);
}

// CDF sampler over the raw stream.  Encaps (KG=false): words -> S' (8N, int8 [8][NP]),
// E' (8N, int16 [8][N]), E'' (64).  KeyGen (KG=true): S^T (8N -> int8 [8][NP]) and E (8N, int16 [N][8]).
template <int N, bool KG>
__global__ __launch_bounds__(256) void k_fr_sample(const uint64_t* __restrict__ raw, size_t n, int RAWW,
                                                   int8_t* __restrict__ sp8, int16_t* __restrict__ ep16,
                                                   int16_t* __restrict__ epp16) {
  using P = FP<N>;
  constexpr int NV = KG ? 2 * N * NBAR : (2 * N + NBAR) * NBAR;  // 16-bit samples per hs
  constexpr int NW = NV / 4;
  const size_t t = (size_t)blockIdx.x * 256 + threadIdx.x;  // one u64 = 4 samples
  const size_t hs = t / NW;
  const int w = (int)(t % NW);
  if (hs >= n) return;
  const uint64_t x = raw[tidx(hs, w, RAWW)];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int idx = 4 * w + e;
    const int v = cdf_sample<N>((uint32_t)(x >> (16 * e)) & 0xFFFF);
    if (idx < NBAR * N) {
      const int k = idx / N, j = idx % N;
      sp8[(hs * NBAR + k) * P::NP + j] = (int8_t)v;
    } else if (idx < 2 * NBAR * N) {
      ep16[hs * NBAR * N + (idx - NBAR * N)] = (int16_t)v;
    } else {
      epp16[hs * 64 + (idx - 2 * NBAR * N)] = (int16_t)v;
    }
  }
  // zero the K padding of S' rows once per hs (pad columns N..NP)
  if (w < NBAR && P::NP > N) {
    for (int j = N; j < P::NP; ++j) sp8[(hs * NBAR + w) * P::NP + j] = 0;
  }
}

// balanced limbs of a 16-bit value a: a == 256*hi + lo (mod 2^16), lo, hi in [-128, 127]
__device__ __forceinline__ uint32_t limb_encode(uint32_t a) {
  return ((a + 128u) & 0xFF00u) | (a & 0xFFu);  // byte0 = lo (two's complement), byte1 = hi
}

// Gen(A) (SHAKE variant): row r of handshake hs = SHAKE128(LE16(r) || seedA), 2N bytes.
// Each 128-lane workgroup owns 128 consecutive rows of one handshake; per squeezed block
// the rows' 84 limb-encoded values are staged in LDS [84][128] and written out as
// transposed byte planes T_lo/T_hi[hs][c][r] with 16-byte stores (16 rows per store).
template <int N>
__global__ __launch_bounds__(128) void k_fr_gen_at(const uint8_t* __restrict__ seed_base, size_t seed_stride,
                                                   size_t hs0, size_t nsub, uint8_t* __restrict__ tlo,
                                                   uint8_t* __restrict__ thi) {
  using P = FP<N>;
  constexpr int WGS_PER_HS = P::NP / 128;
  __shared__ uint16_t st[84 * 128];
  const size_t h = blockIdx.x / WGS_PER_HS;  // handshake within the sub-chunk
  const int r0 = (int)(blockIdx.x % WGS_PER_HS) * 128;
  if (h >= nsub) return;
  const int r = r0 + threadIdx.x;
  const bool live = r < N;
  const uint8_t* sa = seed_base + (hs0 + h) * seed_stride;
  uint64_t in[3];
  {
    const uint64_t s0 = ((const uint64_t*)sa)[0], s1 = ((const uint64_t*)sa)[1];
    in[0] = (uint64_t)(r & 0xFFFF) | (s0 << 16);
    in[1] = (s0 >> 48) | (s1 << 16);
    in[2] = s1 >> 48;
  }
  KState s;
  kzero(s);
  absorb_short<21, 3>(s, in, 18);
  uint8_t* plo = tlo + h * (size_t)N * P::NP;
  uint8_t* phi = thi + h * (size_t)N * P::NP;
#pragma unroll 1
  for (int b = 0; b < P::A_BLOCKS; ++b) {
    if (b) keccak_f(s);
    const int c0 = 84 * b;
    const int nc = (N - c0) < 84 ? (N - c0) : 84;
#pragma unroll
    for (int w = 0; w < 21; ++w) {
      const uint32_t lo = s.a[w].lo, hi = s.a[w].hi;
      const uint32_t v[4] = {lo & 0xFFFF, lo >> 16, hi & 0xFFFF, hi >> 16};
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (4 * w + e < nc) st[(4 * w + e) * 128 + threadIdx.x] = live ? (uint16_t)limb_encode(v[e]) : 0;
    }
    __syncthreads();
    // nc columns x 8 groups of 16 rows
    for (int task = threadIdx.x; task < nc * 8; task += 128) {
      const int c = task >> 3, g = task & 7;
      const uint4 a = *(const uint4*)&st[c * 128 + 16 * g];
      const uint4 bb = *(const uint4*)&st[c * 128 + 16 * g + 8];
      // even bytes -> lo plane, odd bytes -> hi plane
      const uint32_t w8[8] = {a.x, a.y, a.z, a.w, bb.x, bb.y, bb.z, bb.w};
      uint32_t ol[4], oh[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        ol[q] = __builtin_amdgcn_perm(w8[2 * q + 1], w8[2 * q], 0x06040200u);
        oh[q] = __builtin_amdgcn_perm(w8[2 * q + 1], w8[2 * q], 0x07050301u);
      }
      const size_t off = (size_t)(c0 + c) * P::NP + r0 + 16 * g;
      *(uint4*)(plo + off) = make_uint4(ol[0], ol[1], ol[2], ol[3]);
      *(uint4*)(phi + off) = make_uint4(oh[0], oh[1], oh[2], oh[3]);
    }
    __syncthreads();
  }
}

// B'[k][c] = (sum_r S'[k][r] A[r][c] + E'[k][c]) mod q on i8 MFMA.
// D(16x16) = X(16x64) . Y(64x16) with m = c (16 columns of A), n = k (8 used),
// K = r:  X[c][r] = T[c][r] (limb planes), Y[r][k] = S'[k][r].  Lane l holds
// m/n index l & 15 and K slice 16*(l >> 4) .. +15 of both operands (a consistent
// pairing of the contraction index, so the result is independent of the
// hardware's internal K order); D: col = l & 15, row = 4*(l >> 4) + reg.
template <int N>
__global__ __launch_bounds__(256) void k_fr_mm(size_t hs0, size_t nsub, const uint8_t* __restrict__ tlo,
                                               const uint8_t* __restrict__ thi, const int8_t* __restrict__ sp8,
                                               const int16_t* __restrict__ ep16, uint16_t* __restrict__ bp16) {
  using P = FP<N>;
  constexpr int TILES = N / 16;
  constexpr int WG_PER_HS = (TILES + 3) / 4;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const size_t h = blockIdx.x / WG_PER_HS;
  const int tile = (int)(blockIdx.x % WG_PER_HS) * 4 + wv;
  if (h >= nsub || tile >= TILES) return;
  const size_t hs = hs0 + h;
  const int c0 = tile * 16;
  const int m = lane & 15, ks = 16 * (lane >> 4);
  const uint8_t* xl = tlo + h * (size_t)N * P::NP + (size_t)(c0 + m) * P::NP + ks;
  const uint8_t* xh = thi + h * (size_t)N * P::NP + (size_t)(c0 + m) * P::NP + ks;
  const bool kv = m < NBAR;
  const int8_t* yp = sp8 + (hs * NBAR + (kv ? m : 0)) * P::NP + ks;
  v4i acc_lo = {0, 0, 0, 0}, acc_hi = {0, 0, 0, 0};
#pragma unroll 2
  for (int r0 = 0; r0 < P::NP; r0 += 64) {
    const v4i a_lo = *(const v4i*)(xl + r0);
    const v4i a_hi = *(const v4i*)(xh + r0);
    v4i y = *(const v4i*)(yp + r0);
    if (!kv) y = v4i{0, 0, 0, 0};
    acc_lo = __builtin_amdgcn_mfma_i32_16x16x64_i8(a_lo, y, acc_lo, 0, 0, 0);
    acc_hi = __builtin_amdgcn_mfma_i32_16x16x64_i8(a_hi, y, acc_hi, 0, 0, 0);
  }
  if (kv) {
    const int k = m;
#pragma unroll
    for (int reg = 0; reg < 4; ++reg) {
      const int c = c0 + 4 * (lane >> 4) + reg;
      const uint32_t v = (uint32_t)(acc_lo[reg] + 256 * acc_hi[reg]) + (uint32_t)ep16[(hs * NBAR + k) * N + c];
      bp16[(hs * NBAR + k) * N + c] = (uint16_t)(v & P::QMASK);
    }
  }
}

// LOGQ-bit MSB-first bit-field reads / writes
template <int LOGQ>
__device__ __forceinline__ uint32_t unpack_at(const uint8_t* p, size_t idx) {
  const size_t bit = idx * LOGQ;
  const uint8_t* b = p + (bit >> 3);
  // the third byte is touched only when the field reaches it (no read past the packed array)
  const bool third = (int)(bit & 7) + LOGQ > 16;
  const uint32_t w = ((uint32_t)b[0] << 16) | ((uint32_t)b[1] << 8) | (third ? (uint32_t)b[2] : 0u);
  const int sh = 24 - (int)(bit & 7) - LOGQ;
  return (w >> sh) & ((1u << LOGQ) - 1);
}

// Pack cnt values (MSB-first, LOGQ bits each) starting at a byte-aligned bit offset.
template <int LOGQ, typename Get>
__device__ __forceinline__ void pack_run(uint8_t* dst, int cnt, Get get) {
  uint64_t acc = 0;
  int bits = 0, o = 0;
  for (int i = 0; i < cnt; ++i) {
    acc = (acc << LOGQ) | (get(i) & ((1u << LOGQ) - 1));
    bits += LOGQ;
    while (bits >= 8) {
      dst[o++] = (uint8_t)(acc >> (bits - 8));
      bits -= 8;
    }
  }
}

__device__ __forceinline__ uint32_t wave_or(uint32_t x) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) x |= __shfl_xor(x, d, 64);
  return x;
}

// V = S'B + E'', C = V + Encode(mu) (mod q); Pack(B') || Pack(C) -> out.
// MODE 0 (encaps): out = ct, kk = k.  MODE 1 (decaps): ct' is packed into LDS,
// compared with ct and select kk = (ct == ct') ? k' : s in constant time.
template <int N, int MODE>
__global__ __launch_bounds__(64) void k_fr_pack(size_t n, const uint8_t* __restrict__ pk_base, size_t pk_stride,
                                                const int8_t* __restrict__ sp8, const int16_t* __restrict__ epp16,
                                                const uint16_t* __restrict__ bp16, const uint64_t* __restrict__ seeds,
                                                const uint8_t* __restrict__ mu_base, size_t mu_stride,
                                                uint8_t* __restrict__ out, const uint8_t* __restrict__ ct_in,
                                                const uint8_t* __restrict__ s_base, size_t s_stride,
                                                uint64_t* __restrict__ kk) {
  using P = FP<N>;
  const size_t hs = blockIdx.x;
  if (hs >= n) return;
  const int l = threadIdx.x;
  const uint8_t* pkb = pk_base + hs * pk_stride + 16;  // packed B (N x 8)
  // ---- V[k][i] for lane (k = l >> 3, i = l & 7)
  const int k = l >> 3, i = l & 7;
  const int8_t* sp = sp8 + (hs * NBAR + k) * P::NP;
  uint32_t acc = (uint32_t)(int32_t)epp16[hs * 64 + l];
  for (int j = 0; j < N; ++j) acc += (uint32_t)((int32_t)sp[j] * (int32_t)unpack_at<P::LOGQ>(pkb, (size_t)j * NBAR + i));
  // Encode(mu): EB bits of mu at bit position EB*(8k + i)
  __shared__ uint8_t cbuf[MODE ? P::CT : 1];  // decaps: re-encryption ciphertext stays on chip
  const uint8_t* mu = mu_base + hs * mu_stride;
  const int bit0 = P::EB * l;
  uint32_t mv = 0;
#pragma unroll
  for (int b = 0; b < P::EB; ++b) mv |= (uint32_t)((mu[(bit0 + b) >> 3] >> ((bit0 + b) & 7)) & 1) << b;
  const uint32_t cval = (acc + (mv << (P::LOGQ - P::EB))) & P::QMASK;
  uint8_t* o = MODE ? cbuf : out + hs * P::CT;
  // ---- Pack B' (8N values, [k][c] row-major): lane l packs values [l*N/8, (l+1)*N/8)
  constexpr int PER = NBAR * N / 64;  // values per lane; PER*LOGQ is a multiple of 8
  const uint16_t* bp = bp16 + hs * NBAR * N;
  pack_run<P::LOGQ>(o + (size_t)l * PER * P::LOGQ / 8, PER, [&](int t) { return (uint32_t)bp[l * PER + t]; });
  // ---- Pack C (64 values): lanes 0..7 pack 8 values each (8*LOGQ bits = LOGQ bytes)
  __shared__ uint32_t cv[64];
  cv[l] = cval;
  __syncthreads();
  if (l < 8) pack_run<P::LOGQ>(o + P::LOGQ * N + l * P::LOGQ, 8, [&](int t) { return cv[8 * l + t]; });
  __syncthreads();
  const uint64_t* sd = seeds + hs * 16;
  if (MODE == 0) {
    if (l < P::SEC / 8) kk[hs * 4 + l] = sd[P::SEC / 8 + l];
    return;
  }
  // ---- decaps: constant-time compare of ct' with ct, select k' or s
  uint32_t diff = 0;
  const uint8_t* c1 = ct_in + hs * P::CT;
  for (int b = l; b < P::CT; b += 64) diff |= (uint32_t)(o[b] ^ c1[b]);
  diff = wave_or(diff);
  const uint64_t mask = (uint64_t)0 - (uint64_t)(diff == 0);  // computed without a branch on diff
  if (l < P::SEC / 8) {
    const uint64_t kp = sd[P::SEC / 8 + l];
    const uint64_t sv = ((const uint64_t*)(s_base + hs * s_stride))[l];
    kk[hs * 4 + l] = (kp & mask) | (sv & ~mask);
  }
}

// ss = H(ct || kk)
template <int N>
__global__ __launch_bounds__(256) void k_fr_ss(const uint8_t* __restrict__ ct, size_t n,
                                               const uint64_t* __restrict__ kk, uint8_t* __restrict__ ss) {
  using P = FP<N>;
  const size_t hs = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (hs >= n) return;
  const uint64_t* c = (const uint64_t*)(ct + hs * P::CT);
  const uint64_t* kw = kk + hs * 4;
  constexpr int CW = P::CT / 8;
  KState s;
  kzero(s);
  absorb_words<P::RW, CW + P::SEC / 8, DS_SHAKE>(s, [&](int w) { return w < CW ? c[w] : kw[w - CW]; });
  uint64_t* o = (uint64_t*)(ss + hs * P::SEC);
#pragma unroll
  for (int w = 0; w < P::SEC / 8; ++w) o[w] = kword(s, w);
}

// Decaps: M = C - B'S, mu' = Decode(M) -> seeds[12..]  (one wave per handshake)
template <int N>
__global__ __launch_bounds__(64) void k_fr_dec_m(size_t n, const uint8_t* __restrict__ ct,
                                                 const uint8_t* __restrict__ sk, uint64_t* __restrict__ seeds) {
  using P = FP<N>;
  const size_t hs = blockIdx.x;
  if (hs >= n) return;
  const int l = threadIdx.x, i = l >> 3, k = l & 7;  // M[i][k]
  const uint8_t* c = ct + hs * P::CT;
  const uint8_t* st = sk + hs * P::SK + P::SEC + P::PK;  // S^T int16 LE [8][N]
  uint32_t acc = 0;
  for (int j = 0; j < N; ++j) {
    const int32_t sv = (int16_t)((uint16_t)st[2 * (k * N + j)] | ((uint16_t)st[2 * (k * N + j) + 1] << 8));
    acc += (uint32_t)((int32_t)unpack_at<P::LOGQ>(c, (size_t)i * N + j) * sv);
  }
  const uint32_t cv = unpack_at<P::LOGQ>(c + P::LOGQ * N, (size_t)l);
  const uint32_t mval = (cv - acc) & P::QMASK;
  const uint32_t t = ((mval + (1u << (P::LOGQ - P::EB - 1))) >> (P::LOGQ - P::EB)) & ((1u << P::EB) - 1);
  // assemble EB*64 bits, lane l contributes bits [EB*l, EB*l + EB)
  uint64_t* mu = seeds + hs * 16 + 12;
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    uint64_t part = 0;
    const int b = P::EB * l - 64 * w;
    if (b >= 0 && b < 64) part = (uint64_t)t << b;
    else if (b < 0 && b + P::EB > 0) part = (uint64_t)t >> (-b);
    uint32_t lo = (uint32_t)part, hi = (uint32_t)(part >> 32);
    lo = wave_or(lo);
    hi = wave_or(hi);
    if (l == 0 && w < (P::MU + 7) / 8) mu[w] = ((uint64_t)hi << 32) | lo;
  }
}

// ---------------------------------------------------------------- KeyGen
// seedA = H(z, 16) -> pk[0..16) and sk's pk copy; SHAKE(0x5F || seedSE) stream -> raw
template <int N>
__global__ __launch_bounds__(256) void k_fr_kg_front(const uint8_t* __restrict__ coins, size_t n,
                                                     uint8_t* __restrict__ pk, uint8_t* __restrict__ sk,
                                                     uint64_t* __restrict__ seeds) {
  using P = FP<N>;
  const size_t hs = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (hs >= n) return;
  const uint8_t* cz = coins + hs * (2 * P::SEC + 16);
  const uint64_t* cw = (const uint64_t*)cz;  // s || seedSE || z (8-byte aligned: coins stride multiple of 8)
  uint64_t z[2] = {cw[2 * P::SEC / 8], cw[2 * P::SEC / 8 + 1]};
  KState s;
  kzero(s);
  absorb_short<P::RW, 2>(s, z, 16);
  uint64_t* pka = (uint64_t*)(pk + hs * P::PK);
  uint64_t* ska = (uint64_t*)(sk + hs * P::SK + P::SEC);  // SEC is a multiple of 8
  pka[0] = kword(s, 0);
  pka[1] = kword(s, 1);
  ska[0] = kword(s, 0);
  ska[1] = kword(s, 1);
  uint64_t* sd = seeds + hs * 16;
#pragma unroll
  for (int w = 0; w < P::SEC / 8; ++w) {
    sd[w] = cw[P::SEC / 8 + w];                           // seedSE
    ((uint64_t*)(sk + hs * P::SK))[w] = cw[w];            // s
  }
}

// B = A S + E (mod q) on VALU: lane r generates row r of A and dots it with the
// 8 rows of S^T (staged in LDS).  KeyGen is not on the timed path.
template <int N>
__global__ __launch_bounds__(128) void k_fr_kg_rows(const uint8_t* __restrict__ pk, size_t n,
                                                    const int8_t* __restrict__ sp8, const int16_t* __restrict__ e16,
                                                    uint16_t* __restrict__ bmat) {
  using P = FP<N>;
  constexpr int WGS_PER_HS = P::NP / 128;
  __shared__ int8_t st[NBAR * P::NP];
  const size_t hs = blockIdx.x / WGS_PER_HS;
  if (hs >= n) return;
  const int r = (int)(blockIdx.x % WGS_PER_HS) * 128 + threadIdx.x;
  for (int t = threadIdx.x; t < NBAR * P::NP; t += 128) st[t] = sp8[hs * NBAR * P::NP + t];
  __syncthreads();
  if (r >= N) return;
  const uint8_t* sa = pk + hs * P::PK;
  uint64_t in[3];
  {
    const uint64_t s0 = ((const uint64_t*)sa)[0], s1 = ((const uint64_t*)sa)[1];
    in[0] = (uint64_t)(r & 0xFFFF) | (s0 << 16);
    in[1] = (s0 >> 48) | (s1 << 16);
    in[2] = s1 >> 48;
  }
  KState s;
  kzero(s);
  absorb_short<21, 3>(s, in, 18);
  uint32_t acc[NBAR];
#pragma unroll
  for (int k = 0; k < NBAR; ++k) acc[k] = (uint32_t)(int32_t)e16[(hs * N + r) * NBAR + k];
#pragma unroll 1
  for (int b = 0; b < P::A_BLOCKS; ++b) {
    if (b) keccak_f(s);
    const int c0 = 84 * b;
#pragma unroll
    for (int w = 0; w < 21; ++w) {
      const uint32_t lo = s.a[w].lo, hi = s.a[w].hi;
      const uint32_t v[4] = {lo & 0xFFFF, lo >> 16, hi & 0xFFFF, hi >> 16};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int c = c0 + 4 * w + e;
        if (c < N) {
#pragma unroll
          for (int k = 0; k < NBAR; ++k) acc[k] += v[e] * (uint32_t)(int32_t)st[k * P::NP + c];
        }
      }
    }
  }
#pragma unroll
  for (int k = 0; k < NBAR; ++k) bmat[(hs * N + r) * NBAR + k] = (uint16_t)(acc[k] & P::QMASK);
}

// pk = seedA || Pack(B);  sk = s || pk || S^T (int16 LE) || pkh   (one wave per handshake;
// pkh is hashed by k_fr_kg_pkh afterwards)
template <int N>
__global__ __launch_bounds__(64) void k_fr_kg_pack(size_t n, const uint16_t* __restrict__ bmat,
                                                   const int8_t* __restrict__ sp8, uint8_t* __restrict__ pk,
                                                   uint8_t* __restrict__ sk) {
  using P = FP<N>;
  const size_t hs = blockIdx.x;
  if (hs >= n) return;
  const int l = threadIdx.x;
  constexpr int PER = NBAR * N / 64;
  uint8_t* pkb = pk + hs * P::PK + 16;
  const uint16_t* bm = bmat + hs * N * NBAR;
  pack_run<P::LOGQ>(pkb + (size_t)l * PER * P::LOGQ / 8, PER, [&](int t) { return (uint32_t)bm[l * PER + t]; });
  __syncthreads();
  // copy pk[16..] into sk, S^T as int16 LE
  uint8_t* skp = sk + hs * P::SK + P::SEC;
  for (int b = 16 + l; b < P::PK; b += 64) skp[b] = pk[hs * P::PK + b];
  uint8_t* sts = sk + hs * P::SK + P::SEC + P::PK;
  for (int t = l; t < NBAR * N; t += 64) {
    const int k = t / N, j = t % N;
    const int16_t v = sp8[(hs * NBAR + k) * P::NP + j];
    sts[2 * t] = (uint8_t)v;
    sts[2 * t + 1] = (uint8_t)((uint16_t)v >> 8);
  }
}

template <int N>
__global__ __launch_bounds__(256) void k_fr_kg_pkh(const uint8_t* __restrict__ pk, size_t n, uint8_t* __restrict__ sk) {
  using P = FP<N>;
  const size_t hs = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (hs >= n) return;
  const uint64_t* pkw = (const uint64_t*)(pk + hs * P::PK);
  KState s;
  kzero(s);
  absorb_words<P::RW, P::PK / 8, DS_SHAKE>(s, [&](int w) { return pkw[w]; });
  uint64_t* o = (uint64_t*)(sk + hs * P::SK + P::SEC + P::PK + 2 * N * NBAR);
#pragma unroll
  for (int w = 0; w < P::SEC / 8; ++w) o[w] = kword(s, w);
}

// ---------------------------------------------------------------- launchers
inline unsigned blocks_for(size_t t, int per = 256) { return (unsigned)((t + per - 1) / per); }
inline size_t round64(size_t x) { return (x + 63) & ~(size_t)63; }

// S'A + E' for every handshake of the chunk, SUB handshakes at a time
template <int N>
void launch_sa(const View<N>& v, const uint8_t* seed_base, size_t seed_stride, size_t n, hipStream_t st) {
  using P = FP<N>;
  for (size_t h0 = 0; h0 < n; h0 += SUB) {
    const size_t m = n - h0 < (size_t)SUB ? n - h0 : (size_t)SUB;
    QRK_LAUNCH("k_fr_gen_at", st, k_fr_gen_at<N>, dim3((unsigned)(m * (P::NP / 128))), dim3(128), 0, st, seed_base,
               seed_stride, h0, m, v.tlo, v.thi);
    QRK_LAUNCH("k_fr_mm", st, k_fr_mm<N>, dim3((unsigned)(m * ((N / 16 + 3) / 4))), dim3(256), 0, st, h0, m, v.tlo,
               v.thi, v.sp8, v.ep16, v.bp16);
  }
}

template <int N>
hipError_t encaps_t(size_t n, uint8_t* ct, uint8_t* ss, const uint8_t* pk, const uint8_t* mu, void* scratch,
                    hipStream_t st) {
  using P = FP<N>;
  const size_t C = round64(n);
  View<N> v = carve<N>(scratch, C);
  QRK_LAUNCH("k_fr_front_enc", st, k_fr_front_enc<N>, dim3(blocks_for(n)), dim3(256), 0, st, pk, mu, n, v.seeds);
  QRK_LAUNCH("k_fr_se_stream", st, k_fr_se_stream<N>, dim3(blocks_for(n)), dim3(256), 0, st, v.seeds, n, 0x96,
             P::SE_WORDS, P::SE_WORDS, v.raw);
  QRK_LAUNCH("k_fr_sample", st, (k_fr_sample<N, false>), dim3(blocks_for(n * (P::SE_WORDS))), dim3(256), 0, st,
             v.raw, n, P::SE_WORDS, v.sp8, v.ep16, v.epp16);
  launch_sa<N>(v, pk, P::PK, n, st);
  QRK_LAUNCH("k_fr_pack", st, (k_fr_pack<N, 0>), dim3((unsigned)n), dim3(64), 0, st, n, pk, (size_t)P::PK, v.sp8,
             v.epp16, v.bp16, v.seeds, mu, (size_t)P::MU, ct, nullptr, nullptr, (size_t)0, v.kk);
  QRK_LAUNCH("k_fr_ss", st, k_fr_ss<N>, dim3(blocks_for(n)), dim3(256), 0, st, ct, n, v.kk, ss);
  return hipGetLastError();
}

template <int N>
hipError_t decaps_t(size_t n, uint8_t* ss, const uint8_t* ct, const uint8_t* sk, void* scratch, hipStream_t st) {
  using P = FP<N>;
  const size_t C = round64(n);
  View<N> v = carve<N>(scratch, C);
  const uint8_t* pk_in_sk = sk + P::SEC;
  QRK_LAUNCH("k_fr_dec_m", st, k_fr_dec_m<N>, dim3((unsigned)n), dim3(64), 0, st, n, ct, sk, v.seeds);
  QRK_LAUNCH("k_fr_g2_dec", st, k_fr_g2_dec<N>, dim3(blocks_for(n)), dim3(256), 0, st, sk, n, v.seeds);
  QRK_LAUNCH("k_fr_se_stream", st, k_fr_se_stream<N>, dim3(blocks_for(n)), dim3(256), 0, st, v.seeds, n, 0x96,
             P::SE_WORDS, P::SE_WORDS, v.raw);
  QRK_LAUNCH("k_fr_sample", st, (k_fr_sample<N, false>), dim3(blocks_for(n * (P::SE_WORDS))), dim3(256), 0, st,
             v.raw, n, P::SE_WORDS, v.sp8, v.ep16, v.epp16);
  launch_sa<N>(v, pk_in_sk, P::SK, n, st);
  QRK_LAUNCH("k_fr_pack", st, (k_fr_pack<N, 1>), dim3((unsigned)n), dim3(64), 0, st, n, pk_in_sk, (size_t)P::SK,
             v.sp8, v.epp16, v.bp16, v.seeds, (const uint8_t*)(v.seeds + 12), (size_t)128, nullptr, ct, sk,
             (size_t)P::SK, v.kk);
  QRK_LAUNCH("k_fr_ss", st, k_fr_ss<N>, dim3(blocks_for(n)), dim3(256), 0, st, ct, n, v.kk, ss);
  return hipGetLastError();
}

template <int N>
hipError_t keypair_t(size_t n, uint8_t* pk, uint8_t* sk, const uint8_t* coins, void* scratch, hipStream_t st) {
  using P = FP<N>;
  const size_t C = round64(n);
  View<N> v = carve<N>(scratch, C);
  QRK_LAUNCH("k_fr_kg_front", st, k_fr_kg_front<N>, dim3(blocks_for(n)), dim3(256), 0, st, coins, n, pk, sk,
             v.seeds);
  QRK_LAUNCH("k_fr_se_stream", st, k_fr_se_stream<N>, dim3(blocks_for(n)), dim3(256), 0, st, v.seeds, n, 0x5F,
             P::KG_WORDS, P::KG_WORDS, v.raw);
  // S^T -> sp8 ([8][NP] int8), E -> ep16 as [N][8]
  QRK_LAUNCH("k_fr_sample", st, (k_fr_sample<N, true>), dim3(blocks_for(n * (P::KG_WORDS))), dim3(256), 0, st,
             v.raw, n, P::KG_WORDS, v.sp8, v.ep16, v.epp16);
  QRK_LAUNCH("k_fr_kg_rows", st, k_fr_kg_rows<N>, dim3((unsigned)(n * (P::NP / 128))), dim3(128), 0, st, pk, n,
             v.sp8, v.ep16, v.bp16);
  QRK_LAUNCH("k_fr_kg_pack", st, k_fr_kg_pack<N>, dim3((unsigned)n), dim3(64), 0, st, n, v.bp16, v.sp8, pk, sk);
  QRK_LAUNCH("k_fr_kg_pkh", st, k_fr_kg_pkh<N>, dim3(blocks_for(n)), dim3(256), 0, st, pk, n, sk);
  return hipGetLastError();
}

}  // namespace frodo

size_t frodo_scratch_bytes(const AlgInfo& a, size_t chunk) {
  const size_t C = frodo::round64(chunk);
  switch (a.k) {
    case 640: return frodo::scratch_bytes_t<640>(C);
    case 976: return frodo::scratch_bytes_t<976>(C);
    case 1344: return frodo::scratch_bytes_t<1344>(C);
  }
  return 0;
}

#define QRK_FRODO_DISPATCH(CALL)                       \
  switch (a.k) {                                       \
    case 640: return frodo::CALL<640>;                 \
    case 976: return frodo::CALL<976>;                 \
    case 1344: return frodo::CALL<1344>;               \
  }                                                    \
  return hipErrorInvalidValue

hipError_t frodo_keypair(const AlgInfo& a, size_t n, uint8_t* pk, uint8_t* sk, const uint8_t* coins, void* scratch,
                         const Streams& s) {
  if (n == 0) return hipSuccess;
  if (a.aes) return hipErrorNotSupported;
  switch (a.k) {
    case 640: return frodo::keypair_t<640>(n, pk, sk, coins, scratch, s.main);
    case 976: return frodo::keypair_t<976>(n, pk, sk, coins, scratch, s.main);
    case 1344: return frodo::keypair_t<1344>(n, pk, sk, coins, scratch, s.main);
  }
  return hipErrorInvalidValue;
}

hipError_t frodo_encaps(const AlgInfo& a, size_t n, uint8_t* ct, uint8_t* ss, const uint8_t* pk, const uint8_t* coins,
                        void* scratch, const Streams& s) {
  if (n == 0) return hipSuccess;
  if (a.aes) return hipErrorNotSupported;
  switch (a.k) {
    case 640: return frodo::encaps_t<640>(n, ct, ss, pk, coins, scratch, s.main);
    case 976: return frodo::encaps_t<976>(n, ct, ss, pk, coins, scratch, s.main);
    case 1344: return frodo::encaps_t<1344>(n, ct, ss, pk, coins, scratch, s.main);
  }
  return hipErrorInvalidValue;
}

hipError_t frodo_decaps(const AlgInfo& a, size_t n, uint8_t* ss, const uint8_t* ct, const uint8_t* sk, void* scratch,
                        const Streams& s) {
  if (n == 0) return hipSuccess;
  if (a.aes) return hipErrorNotSupported;
  switch (a.k) {
    case 640: return frodo::decaps_t<640>(n, ss, ct, sk, scratch, s.main);
    case 976: return frodo::decaps_t<976>(n, ss, ct, sk, scratch, s.main);
    case 1344: return frodo::decaps_t<1344>(n, ss, ct, sk, scratch, s.main);
  }
  return hipErrorInvalidValue;
}

}  // namespace qrk
