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
//   k_fr_dec_m        256 / hs    M = C - B'S (B', S^T staged in LDS), mu' = Decode(M)
//   k_fr_g2_dec       lane / hs   (seedSE' || k') = H(pkh || mu')
//   k_fr_se_stream    lane / hs   SHAKE(0x96 || seedSE) raw words (123 perms, sequential)
//   k_fr_sample       thread / 4 words   CDF sampler -> S' (int8, zero-padded), E', E''
//   k_fr_gen_mm       wave / 64 rows   Gen(A) (lane = row, SHAKE128) fused with S'A on
//                                  v_mfma_i32_16x16x64_i8: each squeezed block's 84 columns
//                                  are split into balanced int8 limbs (A = 256*hi + lo) in
//                                  LDS and contracted over the wave's 64 rows (two i8 MFMAs
//                                  per 16 columns, int32 accumulation, exact mod 2^16);
//                                  per-wave u16 partial sums of S'A go to scratch
//   k_fr_pack         256 / hs    B' = sum(partials) + E', V = S'B + E'', C = V + Encode(mu),
//                                  Pack(B', C) staged in LDS; encaps: coalesced ct store;
//                                  decaps: compare with ct, select k' or s (constant time)
//   k_fr_ss           lane / hs   ss = H(ct || k)
// KeyGen: k_fr_kg_front (seedA, SHAKE(0x5F || seedSE) stream), k_fr_sample, B = AS + E fused with
// Gen(A) (SHAKE: k_fr_kg_mm on i8 MFMA; AES: k_fr_kg_rows_aes, lane / row on VALU), k_fr_kg_pack.
// AES Gen(A): k_fr_aes_prep + k_fr_gen_mv_aes (column-major, S'A on v_pk_mad_u16).
#include "aes.cuh"
#include "keccak.cuh"
#include "keccak_coop.cuh"
#include "qrkem_internal.h"

namespace qrk {
namespace frodo {

typedef int v4i __attribute__((ext_vector_type(4)));

constexpr int NBAR = 8;
// KeyGen B = AS + E for FrodoKEM-SHAKE: 1 = fused Gen(A) + i8 MFMA (k_fr_kg_mm), 0 = VALU rows
constexpr int ST_PITCH = 72;  // LDS pitch (u16) of one column of a 64-row A block: 144 B -> conflict-free 16-B reads

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
  static constexpr int NP = (N + 127) / 128 * 128;  // padded row pitch of S' (>= 64 * NWV, zero padded)
  static constexpr int NWV = (N + 63) / 64;         // 64-row waves of Gen(A) per handshake
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
  uint16_t* part;  // per-wave partial S'A (u16, mod 2^16) [C][NWV][8][N]; KeyGen: B [C][N][8]
  uint64_t* seeds; // per hs 16 u64: seedSE | k | pkh | mu'  (4 x 32 B)
  uint64_t* kk;    // per hs 4 u64: key fed to the final hash
  uint32_t* aesp;  // FrodoKEM-AES: per hs aes::prep_words<N>() words (round keys, round-2 parts)
};

inline size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }

template <int N>
size_t scratch_bytes_t(size_t C) {
  using P = FP<N>;
  const size_t W = (size_t)(P::SE_WORDS > P::KG_WORDS ? P::SE_WORDS : P::KG_WORDS);
  return al256(C * W * 8) + al256(C * 8 * P::NP + 256) + al256(C * 8 * N * 2) + al256(C * 64 * 2) +
         al256(C * P::NWV * 8 * N * 2) + al256(C * 128) + al256(C * 32) + al256(C * aes::prep_words<N>() * 4);
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
  p += al256(C * 8 * P::NP + 256);  // + slack: k_fr_kg_mm reads up to 128 B past a row
  v.ep16 = (int16_t*)p;
  p += al256(C * 8 * N * 2);
  v.epp16 = (int16_t*)p;
  p += al256(C * 64 * 2);
  v.part = (uint16_t*)p;
  p += al256(C * P::NWV * 8 * N * 2);
  v.seeds = (uint64_t*)p;
  p += al256(C * 128);
  v.kk = (uint64_t*)p;
  p += al256(C * 32);
  v.aesp = (uint32_t*)p;
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

// One thread per (hs, word) in handshake order: strided reads, stores contiguous across the wave
// (following the tiled stream layout instead ran 1.68-1.72 against 1.40 ms at FrodoKEM-640 2^16,
// profiles/r2/ab_fr_sample_tiled_rejected.jsonl: the scattered stores cost more than the reads).
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

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

// +128 on both 16-bit halves (v_pk_add_u16).  Balanced limbs of a 16-bit value a:
// lo = a & 0xFF and hi = ((a + 128) >> 8) & 0xFF, read as int8, satisfy a == 256*hi + lo (mod 2^16).
__device__ __forceinline__ uint32_t add80(uint32_t x) {
  const u16x2 t = __builtin_bit_cast(u16x2, x) + (u16x2){0x80, 0x80};
  return __builtin_bit_cast(uint32_t, t);
}

// Gen(A) fused with S'A.  Row r of handshake hs = SHAKE128(LE16(r) || seedA) (2N bytes,
// little-endian u16).  One wave owns 64 consecutive rows (lane = row) of one handshake;
// per squeezed SHAKE128 block its 84 columns are limb-encoded into LDS as [c][r] and
// contracted over the wave's rows on i8 MFMA:
//   D(16x16) = X(16x64) . Y(64x16),  m = column c (16 per tile), n = k (8 used), K = row r,
//   X[c][r] = limb(A[r][c]) from LDS, Y[r][k] = S'[k][r] (fixed per wave, kept in registers).
// Lane l supplies m/n = l & 15 and the K slice 16*(l >> 4) .. +15 of both operands (the same
// pairing of contraction indices in X and Y, so the result does not depend on the hardware's
// order inside a fragment); D: col = l & 15 (k), row = 4*(l >> 4) + reg (c).
// The wave's partial sum lo + 256*hi (mod 2^16) of 4 consecutive columns is one 8-byte store.
template <int N>
__global__ __launch_bounds__(64) void k_fr_gen_mm(const uint8_t* __restrict__ seed_base, size_t seed_stride, size_t n,
                                                  const int8_t* __restrict__ sp8, uint16_t* __restrict__ part) {
  using P = FP<N>;
  __shared__ __attribute__((aligned(16))) uint16_t st[96 * ST_PITCH];
  const size_t hs = blockIdx.x / P::NWV;
  const int wv = (int)(blockIdx.x % P::NWV);
  if (hs >= n) return;
  const int lane = threadIdx.x;
  const int r = wv * 64 + lane;
  const int kq = lane & 15, ks = 16 * (lane >> 4);
  v4i y = {0, 0, 0, 0};
  if (kq < NBAR) y = *(const v4i*)(sp8 + (hs * NBAR + kq) * P::NP + wv * 64 + ks);  // zero past row N
  const uint8_t* sa = seed_base + hs * seed_stride;
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
  uint16_t* prt = part + (hs * P::NWV + wv) * NBAR * N;
#pragma unroll 1
  for (int b = 0; b < P::A_BLOCKS; ++b) {
    if (b) keccak_f(s);
    const int c0 = 84 * b;
    const int nc = (N - c0) < 84 ? (N - c0) : 84;  // a multiple of 4 for every parameter set
#pragma unroll
    for (int w = 0; w < 21; ++w) {
      const uint32_t lo = s.a[w].lo, hi = s.a[w].hi;
      // two values per dword: limb lo = low byte of the value, limb hi = high byte of
      // (value + 128) (packed 16-bit add, no carry between the halves):
      // al = [lo0 | hi0 << 8 | lo1 << 16 | hi1 << 24] for values 4w, 4w+1
      const uint32_t al = __builtin_amdgcn_perm(add80(lo), lo, 0x07020500u);
      const uint32_t ah = __builtin_amdgcn_perm(add80(hi), hi, 0x07020500u);
      if (4 * w < nc) {
        st[(4 * w + 0) * ST_PITCH + lane] = (uint16_t)al;
        st[(4 * w + 1) * ST_PITCH + lane] = (uint16_t)(al >> 16);
        st[(4 * w + 2) * ST_PITCH + lane] = (uint16_t)ah;
        st[(4 * w + 3) * ST_PITCH + lane] = (uint16_t)(ah >> 16);
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int ntile = (nc + 15) >> 4;
#pragma unroll
    for (int t = 0; t < 6; ++t) {
      if (t < ntile) {
        const uint16_t* src = st + (16 * t + kq) * ST_PITCH + ks;
        const uint4 a0 = *(const uint4*)src;        // rows ks .. ks+7
        const uint4 a1 = *(const uint4*)(src + 8);  // rows ks+8 .. ks+15
        const uint32_t w8[8] = {a0.x, a0.y, a0.z, a0.w, a1.x, a1.y, a1.z, a1.w};
        v4i xl, xh;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          xl[q] = (int)__builtin_amdgcn_perm(w8[2 * q + 1], w8[2 * q], 0x06040200u);
          xh[q] = (int)__builtin_amdgcn_perm(w8[2 * q + 1], w8[2 * q], 0x07050301u);
        }
        const v4i z = {0, 0, 0, 0};
        const v4i dl = __builtin_amdgcn_mfma_i32_16x16x64_i8(xl, y, z, 0, 0, 0);
        const v4i dh = __builtin_amdgcn_mfma_i32_16x16x64_i8(xh, y, z, 0, 0, 0);
        const int cl = 16 * t + 4 * (lane >> 4);
        if (kq < NBAR && cl < nc) {
          uint32_t v[4];
#pragma unroll
          for (int g = 0; g < 4; ++g) v[g] = ((uint32_t)dl[g] + ((uint32_t)dh[g] << 8)) & 0xFFFFu;
          *(uint2*)(prt + kq * N + c0 + cl) = make_uint2(v[0] | (v[1] << 16), v[2] | (v[3] << 16));
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
}

// ---------------------------------------------------------------- FrodoKEM-AES Gen(A)
// Per handshake (lane per (hs, column block jb)): round keys of seedA, the round-1
// constants and the uniform round-2 part of column block jb (aes.cuh).  seedA at
// seed_base + hs * seed_stride (pk, or the pk copy inside sk).
// ROWS: NB + N threads per handshake, the last N of which store the per-row parts (prep_rowp) for
// the column-major Gen(A) kernel k_fr_gen_mv_aes.
template <int N, bool ROWS = false>
__global__ __launch_bounds__(256) void k_fr_aes_prep(const uint8_t* __restrict__ seed_base, size_t seed_stride,
                                                     size_t n, uint32_t* __restrict__ prep) {
  using namespace aes;
  constexpr int NB = N / 8, W = prep_words<N>(), TPH = ROWS ? NB + N : NB;
  const size_t t = (size_t)blockIdx.x * 256 + threadIdx.x;
  const size_t hs = t / TPH;
  const int jb = (int)(t % TPH);
  if (hs >= n) return;
  const uint32_t* sa = (const uint32_t*)(seed_base + hs * seed_stride);
  const uint32_t key[4] = {sa[0], sa[1], sa[2], sa[3]};
  uint32_t rk[44];
  expand_key(key, rk);
  const uint32_t r1 = rk[1], r2 = rk[2], r3 = rk[3];
  // round-1 output columns with the (i, j)-dependent byte left out (see aes.cuh)
  const uint32_t C0 = Tg(1, B(r1, 1)) ^ Tg(2, B(r2, 2)) ^ Tg(3, B(r3, 3)) ^ rk[4];
  const uint32_t C1 = Tg(0, B(r1, 0)) ^ Tg(1, B(r2, 1)) ^ Tg(2, B(r3, 2)) ^ rk[5];
  const uint32_t C2 = Tg(0, B(r2, 0)) ^ Tg(1, B(r3, 1)) ^ Tg(3, B(r1, 3)) ^ rk[6];
  const uint32_t C3 = Tg(0, B(r3, 0)) ^ Tg(2, B(r1, 2)) ^ Tg(3, B(r2, 3)) ^ rk[7];
  uint32_t* o = prep + hs * W;
  if (ROWS && jb >= NB) {
    uint32_t lp[4];
    row_part_g(rk[0], C0, C3, (uint32_t)(jb - NB), lp);
    *(uint4*)(o + prep_rowp<N>() + 4 * (jb - NB)) = make_uint4(lp[0], lp[1], lp[2], lp[3]);
    return;
  }
  if (jb == 0) {
#pragma unroll
    for (int i = 0; i < 44; ++i) o[i] = rk[i];
    o[44] = C0, o[45] = C3, o[46] = C1, o[47] = C2;
  }
  const uint32_t j = 8u * (uint32_t)jb, k = rk[0];
  const uint32_t y1 = Tg(3, ((j >> 8) ^ (k >> 24)) & 0xFF) ^ C1;  // column 1 after round 1
  const uint32_t y2 = Tg(2, (j ^ (k >> 16)) & 0xFF) ^ C2;         // column 2 after round 1
  uint32_t* u = o + PREP_HDR + 4 * jb;
  u[0] = Tg(1, B(y1, 1)) ^ Tg(2, B(y2, 2)) ^ rk[8];
  u[1] = Tg(0, B(y1, 0)) ^ Tg(1, B(y2, 1)) ^ rk[9];
  u[2] = Tg(0, B(y2, 0)) ^ Tg(3, B(y1, 3)) ^ rk[10];
  u[3] = Tg(2, B(y1, 2)) ^ Tg(3, B(y2, 3)) ^ rk[11];
}

// Gen(A) with AES-128 fused with S'A on the VALU, column-major: one lane owns column block jb (8
// columns of A) of one handshake and walks the rows i of its row range, two AES blocks in flight;
// after round 2 a block's state is rowpart(i) ^ colpart(jb) (aes.cuh), so the lane keeps its
// colpart in registers and reads the row parts (prep_rowp) and the S' pairs of row i
// (S'[2q][i] | S'[2q+1][i] << 16, k_fr_kg_spairs) as it goes.  Each A value is multiplied into
// the 8 outputs B'[k][8 jb + c] with 4 v_pk_mad_u16 (mod 2^16 is all Encaps needs: q | 2^16), so
// the lane ends with whole sums for its columns -- no LDS staging beside the T-table (the kernel is
// bound by the table lookups on the CU's LDS, where an i8-MFMA variant's operand staging added
// ~12 % more LDS instructions (rejected by A/B in round 3) while the four SIMDs have VALU to
// spare), and no per-wave partial sums.
// fr_mv_r<N>() row ranges per column block keep every handshake's lanes whole waves (waves never span
// two handshakes, so round keys and S' pairs are scalar loads): 640: 80 x 4 = 320 lanes, 976: 122
// (+ 6 idle) = 128, 1344: 168 x 8 = 1344.  Output: R partial sums [hs][R][8][N], added by k_fr_pack.
template <int N>
constexpr int fr_mv_r() { return N == 640 ? 4 : (N == 976 ? 1 : 8); }
template <int N>
constexpr int fr_mv_lph() { return ((N / 8) * fr_mv_r<N>() + 63) / 64 * 64; }  // lanes per handshake
template <int N>
__global__ __launch_bounds__(1024) void k_fr_gen_mv_aes(const uint32_t* __restrict__ prep, size_t n,
                                                        const uint32_t* __restrict__ spair, uint16_t* __restrict__ part) {
  constexpr int NB = N / 8, R = fr_mv_r<N>(), LPH = fr_mv_lph<N>(), RN = N / R;
  static_assert(RN % 2 == 0, "row pairs");
  __shared__ __attribute__((aligned(16))) uint32_t tab[256 * 64];  // T0 | T2 interleaved per entry
  aes::fill_lds2(tab, threadIdx.x, 1024);
  __syncthreads();
  const size_t gl = (size_t)blockIdx.x * 1024 + threadIdx.x;
  const uint32_t hs = __builtin_amdgcn_readfirstlane((uint32_t)(gl / LPH));  // whole waves per handshake
  const int l = (int)(gl % LPH);
  if (hs >= n || l >= NB * R) return;
  const int r = l / NB, jb = l % NB;
  const uint32_t* hp = prep + (size_t)hs * aes::prep_words<N>();
  const uint32_t* rowp = hp + aes::prep_rowp<N>();
  const uint32_t* sp = spair + (size_t)hs * N * 4;
  const int lane = threadIdx.x & 63;
  const aes::Lds2 L{(const char*)tab, (uint32_t)(lane & 31) * 4u, 128u + (uint32_t)(lane & 31) * 4u};
  const uint4 cu = *(const uint4*)(hp + aes::PREP_HDR + 4 * jb);
  u16x2 acc[8][4];
#pragma unroll
  for (int c = 0; c < 8; ++c)
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[c][q] = (u16x2){0, 0};
#pragma unroll 1
  for (int i = r * RN; i < (r + 1) * RN; i += 2) {
    const uint4 a = *(const uint4*)(rowp + 4 * i), b = *(const uint4*)(rowp + 4 * i + 4);
    uint32_t z[4] = {a.x ^ cu.x, a.y ^ cu.y, a.z ^ cu.z, a.w ^ cu.w};
    uint32_t w[4] = {b.x ^ cu.x, b.y ^ cu.y, b.z ^ cu.z, b.w ^ cu.w};
    aes::rounds_3_10_x2(L, z, w, hp);
    const uint32_t* s0 = sp + 4 * i;  // S' pairs of rows i, i + 1 (uniform: scalar loads)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const uint32_t* x = h ? w : z;
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const uint32_t v = x[c >> 1];
        const u16x2 vv = __builtin_bit_cast(u16x2, __builtin_amdgcn_perm(v, v, (c & 1) ? 0x03020302u : 0x01000100u));
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[c][q] = vv * __builtin_bit_cast(u16x2, s0[4 * h + q]) + acc[c][q];
      }
    }
  }
  // B'[k][8 jb + c] (partial over the row range r): 8 values per k as one 16-byte store
  uint16_t* prt = part + ((size_t)hs * R + r) * NBAR * N + 8 * jb;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    uint32_t lo[4], hi[4];  // rows k = 2q (low halves) and 2q + 1 (high halves), columns c = 0..7
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const uint32_t a0 = __builtin_bit_cast(uint32_t, acc[2 * e][q]), a1 = __builtin_bit_cast(uint32_t, acc[2 * e + 1][q]);
      lo[e] = __builtin_amdgcn_perm(a1, a0, 0x05040100u);
      hi[e] = __builtin_amdgcn_perm(a1, a0, 0x07060302u);
    }
    *(uint4*)(prt + (2 * q) * N) = make_uint4(lo[0], lo[1], lo[2], lo[3]);
    *(uint4*)(prt + (2 * q + 1) * N) = make_uint4(hi[0], hi[1], hi[2], hi[3]);
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

// 8 LOGQ-bit values, MSB first, in LOGQ bytes (a group never straddles a byte boundary)
template <int LOGQ>
__device__ __forceinline__ void unpack8(const uint8_t* p, uint32_t v[8]) {
  unsigned __int128 x = 0;
#pragma unroll
  for (int b = 0; b < LOGQ; ++b) x = (x << 8) | p[b];
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = (uint32_t)(x >> ((7 - i) * LOGQ)) & ((1u << LOGQ) - 1);
}

template <int LOGQ>
__device__ __forceinline__ void pack8(const uint32_t v[8], uint8_t* p) {
  unsigned __int128 x = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) x = (x << LOGQ) | (v[i] & ((1u << LOGQ) - 1));
#pragma unroll
  for (int b = 0; b < LOGQ; ++b) p[b] = (uint8_t)(x >> (8 * (LOGQ - 1 - b)));
}

__device__ __forceinline__ uint32_t wave_or(uint32_t x) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) x |= __shfl_xor(x, d, 64);
  return x;
}

// B' = (sum of the NWV partial S'A + E') mod q; V = S'B + E''; C = V + Encode(mu) (mod q);
// ct = Pack(B') || Pack(C), staged in LDS.  One 256-thread workgroup per handshake.
// MODE 0 (encaps): ct is stored with coalesced 8-byte stores, kk = k.
// MODE 1 (decaps): ct' stays in LDS, is compared with the received ct, and
// kk = (ct == ct') ? k' : s is selected in constant time.
template <int N, int MODE, int NPART = FP<N>::NWV>
__global__ __launch_bounds__(256) void k_fr_pack(size_t n, const uint8_t* __restrict__ pk_base, size_t pk_stride,
                                                 const int8_t* __restrict__ sp8, const int16_t* __restrict__ ep16,
                                                 const int16_t* __restrict__ epp16, const uint16_t* __restrict__ part,
                                                 const uint64_t* __restrict__ seeds, const uint8_t* __restrict__ mu_base,
                                                 size_t mu_stride, uint8_t* __restrict__ ct_out,
                                                 const uint8_t* __restrict__ ct_in, const uint8_t* __restrict__ s_base,
                                                 size_t s_stride, uint64_t* __restrict__ kk) {
  using P = FP<N>;
  constexpr int CTW = P::CT / 8;
  __shared__ __attribute__((aligned(16))) uint16_t bsh[N * NBAR];  // B [j][i]
  __shared__ __attribute__((aligned(16))) uint8_t cbuf[(P::CT + 15) / 16 * 16];
  __shared__ uint32_t red[256];
  __shared__ uint32_t cv[64];
  const size_t hs = blockIdx.x;
  if (hs >= n) return;
  const int t = threadIdx.x;
  // 1. unpack B (N rows of 8 values = one LOGQ-byte group each)
  const uint8_t* pkb = pk_base + hs * pk_stride + 16;
  for (int g = t; g < N; g += 256) {
    uint32_t v[8];
    unpack8<P::LOGQ>(pkb + g * P::LOGQ, v);
    *(uint4*)&bsh[g * 8] = make_uint4(v[0] | (v[1] << 16), v[2] | (v[3] << 16), v[4] | (v[5] << 16), v[6] | (v[7] << 16));
  }
  // 2. B' groups: partial sums (u16 pairs, lane-wise adds) + E', masked, packed into LDS
  const uint16_t* pp = part + hs * NPART * NBAR * N;
  const int16_t* ep = ep16 + hs * NBAR * N;
  for (int g = t; g < N; g += 256) {
    uint32_t lo[4], hi[4];
    {
      const uint4 e0 = *(const uint4*)(ep + 8 * g);
      const uint32_t e[4] = {e0.x, e0.y, e0.z, e0.w};
#pragma unroll
      for (int q = 0; q < 4; ++q) lo[q] = e[q] & 0xFFFF, hi[q] = e[q] >> 16;
    }
#pragma unroll 4
    for (int w = 0; w < NPART; ++w) {
      const uint4 x = *(const uint4*)(pp + (size_t)w * NBAR * N + 8 * g);
      const uint32_t xs[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
      for (int q = 0; q < 4; ++q) lo[q] += xs[q] & 0xFFFF, hi[q] += xs[q] >> 16;
    }
    uint32_t v[8];
#pragma unroll
    for (int q = 0; q < 4; ++q) v[2 * q] = lo[q], v[2 * q + 1] = hi[q];
    pack8<P::LOGQ>(v, cbuf + g * P::LOGQ);
  }
  __syncthreads();
  // 3. V[k][i] = sum_j S'[k][j] B[j][i]: thread (k, i) x quarter of j
  {
    const int p = t & 63, k = p >> 3, i = p & 7, qj = t >> 6;
    constexpr int JQ = N / 4;  // a multiple of 4
    const int8_t* sp = sp8 + (hs * NBAR + k) * P::NP + qj * JQ;
    const uint16_t* bc = bsh + qj * JQ * NBAR + i;
    uint32_t acc = 0;
#pragma unroll 4
    for (int j = 0; j < JQ; j += 4) {
      const uint32_t s4 = *(const uint32_t*)(sp + j);
#pragma unroll
      for (int e = 0; e < 4; ++e) acc += (uint32_t)((int32_t)(int8_t)(s4 >> (8 * e)) * (int32_t)bc[(j + e) * NBAR]);
    }
    red[t] = acc;
  }
  __syncthreads();
  if (t < 64) {
    // Encode(mu): value t takes EB bits of mu at bit EB*t (little-endian bit order)
    const uint8_t* mu = mu_base + hs * mu_stride;
    const int bit0 = P::EB * t;
    uint32_t mv = 0;
#pragma unroll
    for (int b = 0; b < P::EB; ++b) mv |= (uint32_t)((mu[(bit0 + b) >> 3] >> ((bit0 + b) & 7)) & 1) << b;
    const uint32_t v = red[t] + red[t + 64] + red[t + 128] + red[t + 192] + (uint32_t)(int32_t)epp16[hs * 64 + t];
    cv[t] = (v + (mv << (P::LOGQ - P::EB))) & P::QMASK;
  }
  __syncthreads();
  if (t < 8) {
    uint32_t v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = cv[8 * t + e];
    pack8<P::LOGQ>(v, cbuf + P::LOGQ * N + t * P::LOGQ);
  }
  __syncthreads();
  const uint64_t* cb = (const uint64_t*)cbuf;
  const uint64_t* sd = seeds + hs * 16;
  if (MODE == 0) {
    uint64_t* o = (uint64_t*)(ct_out + hs * P::CT);
    for (int x = t; x < CTW; x += 256) o[x] = cb[x];
    if (t < P::SEC / 8) kk[hs * 4 + t] = sd[P::SEC / 8 + t];
    return;
  }
  // 4. decaps: constant-time compare of ct' (LDS) with ct, select k' or s
  const uint64_t* c1 = (const uint64_t*)(ct_in + hs * P::CT);
  uint64_t d = 0;
  for (int x = t; x < CTW; x += 256) d |= cb[x] ^ c1[x];
  uint32_t diff = wave_or((uint32_t)d | (uint32_t)(d >> 32));
  __syncthreads();
  if ((t & 63) == 0) red[t >> 6] = diff;
  __syncthreads();
  diff = red[0] | red[1] | red[2] | red[3];
  const uint64_t mask = (uint64_t)0 - (uint64_t)(diff == 0);
  if (t < P::SEC / 8) {
    const uint64_t kp = sd[P::SEC / 8 + t];
    const uint64_t sv = ((const uint64_t*)(s_base + hs * s_stride))[t];
    kk[hs * 4 + t] = (kp & mask) | (sv & ~mask);
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

// Decaps: M = C - B'S, mu' = Decode(M) -> seeds[12..].  One 256-thread workgroup per
// handshake: B' (from ct) and S^T (from sk) are staged in LDS with a padded pitch (rows land
// on distinct banks), thread (i, k) x quarter of j accumulates, LDS reduction, wave 0 decodes.
template <int N>
__global__ __launch_bounds__(256) void k_fr_dec_m(size_t n, const uint8_t* __restrict__ ct,
                                                  const uint8_t* __restrict__ sk, uint64_t* __restrict__ seeds) {
  using P = FP<N>;
  constexpr int PIT = N + 8;
  __shared__ __attribute__((aligned(16))) uint16_t bq[NBAR * PIT];
  __shared__ __attribute__((aligned(16))) uint16_t sq[NBAR * PIT];
  __shared__ uint32_t red[256];
  const size_t hs = blockIdx.x;
  if (hs >= n) return;
  const int t = threadIdx.x;
  const uint8_t* c = ct + hs * P::CT;
  for (int g = t; g < N; g += 256) {  // B' group g = flat values 8g .. 8g+7 = row i, columns j .. j+7
    uint32_t v[8];
    unpack8<P::LOGQ>(c + g * P::LOGQ, v);
    const int i = (8 * g) / N, j = (8 * g) % N;
    *(uint4*)&bq[i * PIT + j] =
        make_uint4(v[0] | (v[1] << 16), v[2] | (v[3] << 16), v[4] | (v[5] << 16), v[6] | (v[7] << 16));
  }
  const uint64_t* sts = (const uint64_t*)(sk + hs * P::SK + P::SEC + P::PK);  // S^T int16 LE [8][N], 8-B aligned
  for (int g = t; g < N; g += 256) {
    const int k = (8 * g) / N, j = (8 * g) % N;
    *(uint2*)&sq[k * PIT + j] = *(const uint2*)&sts[2 * g];
    *(uint2*)&sq[k * PIT + j + 4] = *(const uint2*)&sts[2 * g + 1];
  }
  __syncthreads();
  {
    const int p = t & 63, i = p >> 3, k = p & 7, qj = t >> 6;
    constexpr int JQ = N / 4;
    const uint32_t* b2 = (const uint32_t*)&bq[i * PIT + qj * JQ];
    const uint32_t* s2 = (const uint32_t*)&sq[k * PIT + qj * JQ];
    uint32_t acc = 0;
#pragma unroll 4
    for (int j = 0; j < JQ / 2; ++j) {
      const uint32_t bb = b2[j], ss = s2[j];
      acc += (bb & 0xFFFF) * (uint32_t)(int32_t)(int16_t)(ss & 0xFFFF);
      acc += (bb >> 16) * (uint32_t)(int32_t)(int16_t)(ss >> 16);
    }
    red[t] = acc;
  }
  __syncthreads();
  if (t >= 64) return;
  const uint32_t acc = red[t] + red[t + 64] + red[t + 128] + red[t + 192];
  const uint32_t cval = unpack_at<P::LOGQ>(c + P::LOGQ * N, (size_t)t);
  const uint32_t mval = (cval - acc) & P::QMASK;
  const uint32_t dv = ((mval + (1u << (P::LOGQ - P::EB - 1))) >> (P::LOGQ - P::EB)) & ((1u << P::EB) - 1);
  // assemble EB*64 bits: value t contributes bits [EB*t, EB*t + EB)
  uint64_t* mu = seeds + hs * 16 + 12;
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    uint64_t part = 0;
    const int b = P::EB * t - 64 * w;
    if (b >= 0 && b < 64) part = (uint64_t)dv << b;
    else if (b < 0 && b + P::EB > 0) part = (uint64_t)dv >> (-b);
    const uint32_t lo = wave_or((uint32_t)part), hi = wave_or((uint32_t)(part >> 32));
    if (t == 0 && w < (P::MU + 7) / 8) mu[w] = ((uint64_t)hi << 32) | lo;
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

// KeyGen: column c of S as four u16 pairs (S[c][0] | S[c][1] << 16, ...), so the
// rows kernel multiplies one A value into all 8 accumulators with 4 v_pk_mad_u16 (mod 2^16 is
// all KeyGen needs: q | 2^16).  Written over the consumed sampler stream.
template <int N>
__global__ __launch_bounds__(256) void k_fr_kg_spairs(size_t n, const int8_t* __restrict__ sp8,
                                                      uint32_t* __restrict__ spair) {
  using P = FP<N>;
  const size_t t = (size_t)blockIdx.x * 256 + threadIdx.x;
  const size_t hs = t / N;
  const int c = (int)(t % N);
  if (hs >= n) return;
  const int8_t* s = sp8 + hs * NBAR * P::NP + c;
  uint4 o;
  o.x = (uint32_t)(uint16_t)(int16_t)s[0 * P::NP] | (uint32_t)(uint16_t)(int16_t)s[1 * P::NP] << 16;
  o.y = (uint32_t)(uint16_t)(int16_t)s[2 * P::NP] | (uint32_t)(uint16_t)(int16_t)s[3 * P::NP] << 16;
  o.z = (uint32_t)(uint16_t)(int16_t)s[4 * P::NP] | (uint32_t)(uint16_t)(int16_t)s[5 * P::NP] << 16;
  o.w = (uint32_t)(uint16_t)(int16_t)s[6 * P::NP] | (uint32_t)(uint16_t)(int16_t)s[7 * P::NP] << 16;
  ((uint4*)spair)[hs * N + c] = o;
}

// KeyGen B = A S + E (mod 2^16), Gen(A) fused with the product on i8 MFMA (SHAKE128 A).
// One wave owns 64 consecutive rows of one handshake (lane = row r squeezes row r of A).
// Each SHAKE128 block's 84 columns go to LDS row-major, one byte per (row, column) and limb
// (balanced limbs: lo = a & 0xFF, hi = ((a + 128) >> 8) & 0xFF, a == 256 hi + lo mod 2^16),
// and are contracted over the columns:
//   D(16x16) = X(16 rows x 64 cols) . Y(64 cols x 16),  X[r][c] = limb(A[r][c]),
//   Y[c][k] = S[c][k] (k < 8 used; S^T rows from sp8),
// four 16-row tiles x two 64-column halves (the second half holds columns 64..83, the rest of
// the stage is zero) x two limbs = 16 MFMAs per block, i32 accumulation over all N columns
// (|acc| <= N * 128 * 12 < 2^31).  Lane l supplies the same K slice 16 (l >> 4) .. +15 of X
// and Y, so the hardware's order inside a fragment does not matter.  B = lo + 256 hi + E.
// LDS row pitch (bytes): 25 dwords (odd, so the 64 lanes' dword writes hit distinct banks),
// holding the block's 84 columns and 16 zero columns; the second K half's slices past column
// 96 are zero registers, not LDS
constexpr int KG_RP = 100;
template <int N>
__global__ __launch_bounds__(64) void k_fr_kg_mm(const uint8_t* __restrict__ pk, size_t n,
                                                 const int8_t* __restrict__ sp8, const int16_t* __restrict__ e16,
                                                 uint16_t* __restrict__ bmat) {
  using P = FP<N>;
  __shared__ __attribute__((aligned(16))) uint8_t st[2][64 * KG_RP];
  const size_t hs = blockIdx.x / P::NWV;
  const int wv = (int)(blockIdx.x % P::NWV);
  if (hs >= n) return;
  const int lane = threadIdx.x;
  const int r = wv * 64 + lane;
  const int kq = lane & 15, ks = 16 * (lane >> 4);
  // zero the stage once: columns 84..99 of every row stay zero
  for (int i = lane; i < 2 * 64 * KG_RP / 4; i += 64) ((uint32_t*)st)[i] = 0u;
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
  const int8_t* sk = sp8 + (hs * NBAR + (kq & 7)) * P::NP;  // S^T row kq (k < 8)
  v4i acc[4][2];
#pragma unroll
  for (int t = 0; t < 4; ++t) acc[t][0] = acc[t][1] = (v4i){0, 0, 0, 0};
  uint32_t* row_lo = (uint32_t*)(st[0] + lane * KG_RP);
  uint32_t* row_hi = (uint32_t*)(st[1] + lane * KG_RP);
#pragma unroll 1
  for (int b = 0; b < P::A_BLOCKS; ++b) {
    if (b) keccak_f(s);
    const int c0 = 84 * b;
    const int nc = (N - c0) < 84 ? (N - c0) : 84;  // a multiple of 4 for every parameter set
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int w = 0; w < 21; ++w) {
      // values 4w .. 4w+3 of this row: lo limbs -> one dword, hi limbs -> one dword
      const uint32_t lo = s.a[w].lo, hi = s.a[w].hi;
      const uint32_t lo80 = add80(lo), hi80 = add80(hi);
      const bool ok = 4 * w < nc && r < N;  // columns past the row's end and rows past N: zero
      row_lo[w] = ok ? __builtin_amdgcn_perm(hi, lo, 0x06040200u) : 0u;
      row_hi[w] = ok ? __builtin_amdgcn_perm(hi80, lo80, 0x07050301u) : 0u;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // Y: S^T row (kq & 7) at this lane's 16 columns of each K half, loaded without conditions
    // (columns past N read zero padding, the next row or the scratch slack after sp8 -- all
    // paired with zero X; lanes kq >= 8 feed output columns that are discarded)
    const v4i y0 = *(const v4i*)(sk + c0 + ks), y1 = *(const v4i*)(sk + c0 + 64 + ks);
    // X slices reaching past column 99 of the stage (64 + ks >= 96) read the zero columns
    // 84..99 instead (a slice that crossed the pitch would read the next row)
    const int xo1 = (64 + ks + 16 <= KG_RP) ? 64 + ks : 84;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int off = (16 * t + kq) * KG_RP + (h ? xo1 : ks);
        v4i xl, xh;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          xl[q] = *(const int*)(st[0] + off + 4 * q);
          xh[q] = *(const int*)(st[1] + off + 4 * q);
        }
        acc[t][0] = __builtin_amdgcn_mfma_i32_16x16x64_i8(xl, h ? y1 : y0, acc[t][0], 0, 0, 0);
        acc[t][1] = __builtin_amdgcn_mfma_i32_16x16x64_i8(xh, h ? y1 : y0, acc[t][1], 0, 0, 0);
      }
    }
  }
  // D[m][n]: m = row 16 t + 4 (lane >> 4) + g, n = k = lane & 15
  if (kq < NBAR) {
#pragma unroll
    for (int t = 0; t < 4; ++t) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int rr = wv * 64 + 16 * t + 4 * (lane >> 4) + g;
        if (rr < N) {
          const size_t o = ((size_t)hs * N + rr) * NBAR + kq;
          const uint32_t v = (uint32_t)acc[t][0][g] + ((uint32_t)acc[t][1][g] << 8) + (uint32_t)(int)e16[o];
          bmat[o] = (uint16_t)(v & P::QMASK);
        }
      }
    }
  }
}

// Workgroup size of the AES KeyGen rows kernel: all rows of a handshake in as few
// workgroups as possible (at most 1024 threads), whole waves.
template <int N>
constexpr int kg_wgs() { return (N + 1023) / 1024; }
template <int N>
constexpr int kg_threads() { return ((N + kg_wgs<N>() - 1) / kg_wgs<N>() + 63) / 64 * 64; }

// FrodoKEM-AES KeyGen rows: B = A S + E (mod 2^16), lane = row, A from AES-128 with the
// two-table LDS T-table layout (aes.cuh, two blocks per iteration), S from the uniform
// pair table (scalar loads), 4 packed 16-bit multiply-adds per A value.  Not on the timed path
// of encaps/decaps, but twice per exchange in the handshake driver.
template <int N>
__global__ __launch_bounds__(kg_threads<N>()) void k_fr_kg_rows_aes(const uint32_t* __restrict__ prep, size_t n,
                                                                    const uint32_t* __restrict__ spair,
                                                                    const int16_t* __restrict__ e16,
                                                                    uint16_t* __restrict__ bmat) {
  using P = FP<N>;
  constexpr int T = kg_threads<N>();
  __shared__ __attribute__((aligned(16))) uint32_t tab[256 * 64];
  const uint32_t hs = __builtin_amdgcn_readfirstlane(blockIdx.x / kg_wgs<N>());
  if (hs >= n) return;
  const int r = (int)(blockIdx.x % kg_wgs<N>()) * T + threadIdx.x;
  aes::fill_lds2(tab, threadIdx.x, T);
  __syncthreads();
  if (r >= N) return;
  const uint32_t* hp = prep + (size_t)hs * aes::prep_words<N>();
  const aes::Lds2 L{(const char*)tab, (uint32_t)(threadIdx.x & 31) * 4u, 128u + (uint32_t)(threadIdx.x & 31) * 4u};
  uint32_t lp[4];
  aes::row_part(L, hp, (uint32_t)r, lp);
  u16x2 acc[4];
  {
    const uint4 e = *(const uint4*)(e16 + ((size_t)hs * N + r) * NBAR);  // E[r][0..7], int16 LE
    acc[0] = __builtin_bit_cast(u16x2, e.x), acc[1] = __builtin_bit_cast(u16x2, e.y);
    acc[2] = __builtin_bit_cast(u16x2, e.z), acc[3] = __builtin_bit_cast(u16x2, e.w);
  }
  const uint32_t* sp = spair + (size_t)hs * N * 4;
#pragma unroll 1
  for (int jb = 0; jb < N / 8; jb += 2) {
    const uint32_t* u = hp + aes::PREP_HDR + 4 * jb;
    uint32_t z[4] = {lp[0] ^ u[0], lp[1] ^ u[1], lp[2] ^ u[2], lp[3] ^ u[3]};
    uint32_t w[4] = {lp[0] ^ u[4], lp[1] ^ u[5], lp[2] ^ u[6], lp[3] ^ u[7]};
    aes::rounds_3_10_x2(L, z, w, hp);
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const uint32_t x = e < 8 ? z[e >> 1] : w[(e - 8) >> 1];
      const u16x2 vv = __builtin_bit_cast(u16x2, __builtin_amdgcn_perm(x, x, (e & 1) ? 0x03020302u : 0x01000100u));
      const uint32_t* s4 = sp + (size_t)(8 * jb + e) * 4;
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[q] = vv * __builtin_bit_cast(u16x2, s4[q]) + acc[q];
    }
  }
  const uint32_t m = P::QMASK | (P::QMASK << 16);
  *(uint4*)(bmat + ((size_t)hs * N + r) * NBAR) =
      make_uint4(__builtin_bit_cast(uint32_t, acc[0]) & m, __builtin_bit_cast(uint32_t, acc[1]) & m,
                 __builtin_bit_cast(uint32_t, acc[2]) & m, __builtin_bit_cast(uint32_t, acc[3]) & m);
}

// pk = seedA || Pack(B);  sk = s || pk || S^T (int16 LE) || pkh.  One 256-thread workgroup
// per handshake; packed B is staged in LDS and copied out with 8-byte stores (pkh is hashed
// by k_fr_kg_pkh afterwards; seedA and s were written by k_fr_kg_front).
template <int N>
__global__ __launch_bounds__(256) void k_fr_kg_pack(size_t n, const uint16_t* __restrict__ bmat,
                                                    const int8_t* __restrict__ sp8, uint8_t* __restrict__ pk,
                                                    uint8_t* __restrict__ sk) {
  using P = FP<N>;
  __shared__ __attribute__((aligned(16))) uint8_t pbuf[(P::PK + 15) / 16 * 16];
  const size_t hs = blockIdx.x;
  if (hs >= n) return;
  const int t = threadIdx.x;
  const uint16_t* bm = bmat + hs * N * NBAR;
  if (t < 2) ((uint64_t*)pbuf)[t] = ((const uint64_t*)(pk + hs * P::PK))[t];  // seedA
  for (int g = t; g < N; g += 256) {
    const uint4 x = *(const uint4*)(bm + 8 * g);
    const uint32_t v[8] = {x.x & 0xFFFF, x.x >> 16, x.y & 0xFFFF, x.y >> 16,
                           x.z & 0xFFFF, x.z >> 16, x.w & 0xFFFF, x.w >> 16};
    pack8<P::LOGQ>(v, pbuf + 16 + g * P::LOGQ);
  }
  __syncthreads();
  uint64_t* po = (uint64_t*)(pk + hs * P::PK);
  uint64_t* so = (uint64_t*)(sk + hs * P::SK + P::SEC);
  const uint64_t* pb = (const uint64_t*)pbuf;
  for (int x = t; x < P::PK / 8; x += 256) {
    const uint64_t w = pb[x];
    if (x >= 2) po[x] = w;
    so[x] = w;
  }
  uint64_t* sto = (uint64_t*)(sk + hs * P::SK + P::SEC + P::PK);
  for (int g = t; g < N; g += 256) {  // 8 S^T entries -> 16 bytes of int16 LE
    const int k = (8 * g) / N, j = (8 * g) % N;
    const uint2 raw = *(const uint2*)(sp8 + (hs * NBAR + k) * P::NP + j);
    const uint32_t b8[2] = {raw.x, raw.y};
    uint64_t o[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      uint64_t acc = 0;
#pragma unroll
      for (int e = 0; e < 4; ++e) acc |= (uint64_t)(uint16_t)(int16_t)(int8_t)(b8[h] >> (8 * e)) << (16 * e);
      o[h] = acc;
    }
    sto[2 * g] = o[0];
    sto[2 * g + 1] = o[1];
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

// ---------------------------------------------------------------- small batches: wave-cooperative sponges
// For a handful of handshakes (the reference's one-call-per-handshake pattern) the lane-per-hs
// sponge kernels above are latency-bound: one lane runs H(pk) (58 / 94 / 129 permutations), the
// SE stream (123 / 231 / 318) and ss = H(ct || k) in sequence at ~9 us per permutation on a wave
// that is alone on its SIMD.  Below QRK_FR_COOP_MAX handshakes these four sponges run one state
// per wave (keccak_coop.cuh, ~2.7 us per permutation) with identical outputs.
#ifndef QRK_FR_COOP_MAX
#define QRK_FR_COOP_MAX 256
#endif

// H(pk) of the hs's pk as the wave's state (coop lanes idx < SEC/8 hold pkh)
template <int N>
__device__ __forceinline__ CState pkh_coop(const uint8_t* __restrict__ pk_row, const Coop& c) {
  using P = FP<N>;
  const uint64_t* pkw = (const uint64_t*)pk_row;
  CState s;
  coop_absorb<P::RW, P::PK / 8, DS_SHAKE>(s, c, [&](int w) { return pkw[w]; });
  return s;
}

template <int N>
__global__ __launch_bounds__(64) void k_fr_front_enc_c(const uint8_t* __restrict__ pk, const uint8_t* __restrict__ mu,
                                                       size_t n, uint64_t* __restrict__ seeds) {
  using P = FP<N>;
  constexpr int PW = P::SEC / 8, GW = (P::SEC + P::MU) / 8;
  static_assert((P::SEC + P::MU) % 8 == 0 && GW < P::RW, "pkh || mu is whole words of one block");
  const size_t hs = blockIdx.x;
  if (hs >= n) return;
  const Coop c = coop_init();
  const int i = c.idx;
  const bool canon = coop_canon(c);
  const CState h = pkh_coop<N>(pk + hs * P::PK, c);
  const uint64_t* muw = (const uint64_t*)(mu + hs * P::MU);
  uint64_t* sd = seeds + hs * 16;
  CState g;  // (seedSE || k) = H(pkh || mu): each pkh word stays on its lane
  if (i >= 0 && i < PW) {
    cs_xor(g, cs_word(h));
    if (canon) sd[8 + i] = cs_word(h);
  }
  if (i >= PW && i < GW) cs_xor(g, muw[i - PW]);
  if (i == GW) g.lo ^= DS_SHAKE;
  if (i == P::RW - 1) g.hi ^= 0x80000000u;
  g = kf_coop(g, c);
  if (canon && i < 2 * PW) sd[i] = cs_word(g);
}

template <int N>
__global__ __launch_bounds__(64) void k_fr_se_stream_c(const uint64_t* __restrict__ seeds, size_t n, int domain, int W,
                                                       int RAWW, uint64_t* __restrict__ raw) {
  using P = FP<N>;
  const size_t hs = blockIdx.x;
  if (hs >= n) return;
  const Coop c = coop_init();
  const int i = c.idx;
  const bool canon = coop_canon(c);
  const uint64_t* sd = seeds + hs * 16;
  // word i of domain || seedSE: the seed shifted up by one byte
  CState s;
  if (i >= 0 && i < 5) {
    const uint64_t cur = i < P::SEC / 8 ? sd[i] : 0;
    const uint64_t prv = i == 0 ? (uint64_t)domain : (i - 1 < P::SEC / 8 ? sd[i - 1] >> 56 : 0);
    cs_xor(s, prv | (cur << 8));
  }
  if (i == (1 + P::SEC) / 8) cs_xor(s, (uint64_t)DS_SHAKE << (8 * ((1 + P::SEC) % 8)));
  if (i == P::RW - 1) s.hi ^= 0x80000000u;
  s = kf_coop(s, c);
  coop_squeeze<P::RW>(s, c, W, [&](int w, uint64_t v) {
    if (canon) raw[tidx(hs, w, RAWW)] = v;
  });
}

template <int N>
__global__ __launch_bounds__(64) void k_fr_ss_c(const uint8_t* __restrict__ ct, size_t n,
                                                const uint64_t* __restrict__ kk, uint8_t* __restrict__ ss) {
  using P = FP<N>;
  constexpr int CW = P::CT / 8;
  const size_t hs = blockIdx.x;
  if (hs >= n) return;
  const Coop c = coop_init();
  const uint64_t* cw = (const uint64_t*)(ct + hs * P::CT);
  const uint64_t* kw = kk + hs * 4;
  CState s;
  coop_absorb<P::RW, CW + P::SEC / 8, DS_SHAKE>(s, c, [&](int w) { return w < CW ? cw[w] : kw[w - CW]; });
  if (coop_canon(c) && c.idx < P::SEC / 8) ((uint64_t*)(ss + hs * P::SEC))[c.idx] = cs_word(s);
}

template <int N>
__global__ __launch_bounds__(64) void k_fr_kg_pkh_c(const uint8_t* __restrict__ pk, size_t n, uint8_t* __restrict__ sk) {
  using P = FP<N>;
  const size_t hs = blockIdx.x;
  if (hs >= n) return;
  const Coop c = coop_init();
  const CState h = pkh_coop<N>(pk + hs * P::PK, c);
  uint64_t* o = (uint64_t*)(sk + hs * P::SK + P::SEC + P::PK + 2 * N * NBAR);
  if (coop_canon(c) && c.idx < P::SEC / 8) o[c.idx] = cs_word(h);
}

// ---------------------------------------------------------------- launchers
inline unsigned blocks_for(size_t t, int per = 256) { return (unsigned)((t + per - 1) / per); }
inline size_t round64(size_t x) { return (x + 63) & ~(size_t)63; }

inline bool coop_path(size_t n) { return n <= QRK_FR_COOP_MAX; }

// SHAKE(domain || seedSE) sampler stream of W words per handshake
template <int N>
void launch_se(const View<N>& v, size_t n, int domain, int W, hipStream_t st) {
  if (coop_path(n))
    QRK_LAUNCH("k_fr_se_stream", st, k_fr_se_stream_c<N>, dim3((unsigned)n), dim3(64), 0, st, v.seeds, n, domain, W, W,
               v.raw);
  else
    QRK_LAUNCH("k_fr_se_stream", st, k_fr_se_stream<N>, dim3(blocks_for(n)), dim3(256), 0, st, v.seeds, n, domain, W,
               W, v.raw);
}

// ss = H(ct || kk)
template <int N>
void launch_ss(const uint8_t* ct, size_t n, const View<N>& v, uint8_t* ss, hipStream_t st) {
  if (coop_path(n))
    QRK_LAUNCH("k_fr_ss", st, k_fr_ss_c<N>, dim3((unsigned)n), dim3(64), 0, st, ct, n, v.kk, ss);
  else
    QRK_LAUNCH("k_fr_ss", st, k_fr_ss<N>, dim3(blocks_for(n)), dim3(256), 0, st, ct, n, v.kk, ss);
}

// partial sums of S'A per handshake that k_fr_pack adds: one per 64-row wave (the SHAKE MFMA
// kernel), or the column-major AES kernel's row ranges
template <int N, bool AES>
constexpr int fr_npart() { return AES ? fr_mv_r<N>() : FP<N>::NWV; }

// partial sums of S'A for every handshake of the chunk (Gen(A) fused)
template <int N, bool AES>
void launch_sa(const View<N>& v, const uint8_t* seed_base, size_t seed_stride, size_t n, hipStream_t st) {
  if constexpr (AES) {
    uint32_t* spair = (uint32_t*)v.raw;  // the sampler stream is consumed by now
    QRK_LAUNCH("k_fr_kg_spairs", st, k_fr_kg_spairs<N>, dim3(blocks_for(n * N)), dim3(256), 0, st, n, v.sp8, spair);
    QRK_LAUNCH("k_fr_aes_prep", st, (k_fr_aes_prep<N, true>), dim3(blocks_for(n * (N / 8 + N))), dim3(256), 0, st,
               seed_base, seed_stride, n, v.aesp);
    QRK_LAUNCH("k_fr_gen_mv_aes", st, k_fr_gen_mv_aes<N>, dim3(blocks_for(n * fr_mv_lph<N>(), 1024)), dim3(1024), 0,
               st, v.aesp, n, spair, v.part);
  } else {
    QRK_LAUNCH("k_fr_gen_mm", st, k_fr_gen_mm<N>, dim3((unsigned)(n * FP<N>::NWV)), dim3(64), 0, st, seed_base,
               seed_stride, n, v.sp8, v.part);
  }
}

template <int N, bool AES>
hipError_t encaps_t(size_t n, uint8_t* ct, uint8_t* ss, const uint8_t* pk, const uint8_t* mu, void* scratch,
                    hipStream_t st) {
  using P = FP<N>;
  const size_t C = round64(n);
  View<N> v = carve<N>(scratch, C);
  if (coop_path(n)) {
    QRK_LAUNCH("k_fr_front_enc", st, k_fr_front_enc_c<N>, dim3((unsigned)n), dim3(64), 0, st, pk, mu, n, v.seeds);
  } else {
    QRK_LAUNCH("k_fr_front_enc", st, k_fr_front_enc<N>, dim3(blocks_for(n)), dim3(256), 0, st, pk, mu, n, v.seeds);
  }
  launch_se<N>(v, n, 0x96, P::SE_WORDS, st);
  QRK_LAUNCH("k_fr_sample", st, (k_fr_sample<N, false>), dim3(blocks_for(round64(n) * (P::SE_WORDS))), dim3(256), 0, st,
             v.raw, n, P::SE_WORDS, v.sp8, v.ep16, v.epp16);
  launch_sa<N, AES>(v, pk, P::PK, n, st);
  QRK_LAUNCH("k_fr_pack", st, (k_fr_pack<N, 0, fr_npart<N, AES>()>), dim3((unsigned)n), dim3(256), 0, st, n, pk, (size_t)P::PK, v.sp8,
             v.ep16, v.epp16, v.part, v.seeds, mu, (size_t)P::MU, ct, nullptr, nullptr, (size_t)0, v.kk);
  launch_ss<N>(ct, n, v, ss, st);
  return hipGetLastError();
}

template <int N, bool AES>
hipError_t decaps_t(size_t n, uint8_t* ss, const uint8_t* ct, const uint8_t* sk, void* scratch, hipStream_t st) {
  using P = FP<N>;
  const size_t C = round64(n);
  View<N> v = carve<N>(scratch, C);
  const uint8_t* pk_in_sk = sk + P::SEC;
  QRK_LAUNCH("k_fr_dec_m", st, k_fr_dec_m<N>, dim3((unsigned)n), dim3(256), 0, st, n, ct, sk, v.seeds);
  QRK_LAUNCH("k_fr_g2_dec", st, k_fr_g2_dec<N>, dim3(blocks_for(n)), dim3(256), 0, st, sk, n, v.seeds);
  launch_se<N>(v, n, 0x96, P::SE_WORDS, st);
  QRK_LAUNCH("k_fr_sample", st, (k_fr_sample<N, false>), dim3(blocks_for(round64(n) * (P::SE_WORDS))), dim3(256), 0, st,
             v.raw, n, P::SE_WORDS, v.sp8, v.ep16, v.epp16);
  launch_sa<N, AES>(v, pk_in_sk, P::SK, n, st);
  QRK_LAUNCH("k_fr_pack", st, (k_fr_pack<N, 1, fr_npart<N, AES>()>), dim3((unsigned)n), dim3(256), 0, st, n, pk_in_sk, (size_t)P::SK,
             v.sp8, v.ep16, v.epp16, v.part, v.seeds, (const uint8_t*)(v.seeds + 12), (size_t)128, nullptr, ct, sk,
             (size_t)P::SK, v.kk);
  launch_ss<N>(ct, n, v, ss, st);
  return hipGetLastError();
}

template <int N, bool AES>
hipError_t keypair_t(size_t n, uint8_t* pk, uint8_t* sk, const uint8_t* coins, void* scratch, hipStream_t st) {
  using P = FP<N>;
  const size_t C = round64(n);
  View<N> v = carve<N>(scratch, C);
  QRK_LAUNCH("k_fr_kg_front", st, k_fr_kg_front<N>, dim3(blocks_for(n)), dim3(256), 0, st, coins, n, pk, sk,
             v.seeds);
  launch_se<N>(v, n, 0x5F, P::KG_WORDS, st);
  // S^T -> sp8 ([8][NP] int8), E -> ep16 as [N][8]
  QRK_LAUNCH("k_fr_sample", st, (k_fr_sample<N, true>), dim3(blocks_for(round64(n) * (P::KG_WORDS))), dim3(256), 0, st,
             v.raw, n, P::KG_WORDS, v.sp8, v.ep16, v.epp16);
  if constexpr (AES) {
    uint32_t* spair = (uint32_t*)v.raw;  // the sampler stream is consumed by now
    QRK_LAUNCH("k_fr_kg_spairs", st, k_fr_kg_spairs<N>, dim3(blocks_for(n * N)), dim3(256), 0, st, n, v.sp8, spair);
    QRK_LAUNCH("k_fr_aes_prep", st, k_fr_aes_prep<N>, dim3(blocks_for(n * (N / 8))), dim3(256), 0, st, pk,
               (size_t)P::PK, n, v.aesp);
    QRK_LAUNCH("k_fr_kg_rows_aes", st, k_fr_kg_rows_aes<N>, dim3((unsigned)(n * kg_wgs<N>())), dim3(kg_threads<N>()),
               0, st, v.aesp, n, spair, v.ep16, v.part);
  } else {
    QRK_LAUNCH("k_fr_kg_mm", st, k_fr_kg_mm<N>, dim3((unsigned)(n * P::NWV)), dim3(64), 0, st, pk, n, v.sp8, v.ep16,
               v.part);
  }
  QRK_LAUNCH("k_fr_kg_pack", st, k_fr_kg_pack<N>, dim3((unsigned)n), dim3(256), 0, st, n, v.part, v.sp8, pk, sk);
  if (coop_path(n))
    QRK_LAUNCH("k_fr_kg_pkh", st, k_fr_kg_pkh_c<N>, dim3((unsigned)n), dim3(64), 0, st, pk, n, sk);
  else
    QRK_LAUNCH("k_fr_kg_pkh", st, k_fr_kg_pkh<N>, dim3(blocks_for(n)), dim3(256), 0, st, pk, n, sk);
  return hipGetLastError();
}

template <int N>
hipError_t cleanse_t(size_t n, void* scratch, hipStream_t st) {
  const size_t C = round64(n);
  const View<N> v = carve<N>(scratch, C);
  return hipMemsetAsync(v.seeds, 0, (size_t)((uint8_t*)v.aesp - (uint8_t*)v.seeds), st);  // seeds | kk
}

}  // namespace frodo

hipError_t frodo_cleanse(const AlgInfo& a, size_t n, void* scratch, hipStream_t st) {
  if (n == 0) return hipSuccess;
  switch (a.k) {
    case 640: return frodo::cleanse_t<640>(n, scratch, st);
    case 976: return frodo::cleanse_t<976>(n, scratch, st);
    case 1344: return frodo::cleanse_t<1344>(n, scratch, st);
  }
  return hipErrorInvalidValue;
}

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
  switch (a.k * 2 + (a.aes ? 1 : 0)) {
    case 1280: return frodo::keypair_t<640, false>(n, pk, sk, coins, scratch, s.main);
    case 1281: return frodo::keypair_t<640, true>(n, pk, sk, coins, scratch, s.main);
    case 1952: return frodo::keypair_t<976, false>(n, pk, sk, coins, scratch, s.main);
    case 1953: return frodo::keypair_t<976, true>(n, pk, sk, coins, scratch, s.main);
    case 2688: return frodo::keypair_t<1344, false>(n, pk, sk, coins, scratch, s.main);
    case 2689: return frodo::keypair_t<1344, true>(n, pk, sk, coins, scratch, s.main);
  }
  return hipErrorInvalidValue;
}

hipError_t frodo_encaps(const AlgInfo& a, size_t n, uint8_t* ct, uint8_t* ss, const uint8_t* pk, const uint8_t* coins,
                        void* scratch, const Streams& s) {
  if (n == 0) return hipSuccess;
  switch (a.k * 2 + (a.aes ? 1 : 0)) {
    case 1280: return frodo::encaps_t<640, false>(n, ct, ss, pk, coins, scratch, s.main);
    case 1281: return frodo::encaps_t<640, true>(n, ct, ss, pk, coins, scratch, s.main);
    case 1952: return frodo::encaps_t<976, false>(n, ct, ss, pk, coins, scratch, s.main);
    case 1953: return frodo::encaps_t<976, true>(n, ct, ss, pk, coins, scratch, s.main);
    case 2688: return frodo::encaps_t<1344, false>(n, ct, ss, pk, coins, scratch, s.main);
    case 2689: return frodo::encaps_t<1344, true>(n, ct, ss, pk, coins, scratch, s.main);
  }
  return hipErrorInvalidValue;
}

hipError_t frodo_decaps(const AlgInfo& a, size_t n, uint8_t* ss, const uint8_t* ct, const uint8_t* sk, void* scratch,
                        const Streams& s) {
  if (n == 0) return hipSuccess;
  switch (a.k * 2 + (a.aes ? 1 : 0)) {
    case 1280: return frodo::decaps_t<640, false>(n, ss, ct, sk, scratch, s.main);
    case 1281: return frodo::decaps_t<640, true>(n, ss, ct, sk, scratch, s.main);
    case 1952: return frodo::decaps_t<976, false>(n, ss, ct, sk, scratch, s.main);
    case 1953: return frodo::decaps_t<976, true>(n, ss, ct, sk, scratch, s.main);
    case 2688: return frodo::decaps_t<1344, false>(n, ss, ct, sk, scratch, s.main);
    case 2689: return frodo::decaps_t<1344, true>(n, ss, ct, sk, scratch, s.main);
  }
  return hipErrorInvalidValue;
}

}  // namespace qrk
