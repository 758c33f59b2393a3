// AES-128 (FIPS 197) for FrodoKEM-*-AES Gen(A) on gfx950.
//
// FrodoKEM-AES (round-3 spec, Gen(A) with AES128): A[i][j..j+7] = the 8 little-endian
// u16 of AES128_seedA(LE16(i) || LE16(j) || 0^96) for j = 0, 8, ..., n-8.  The reference
// reaches this through liboqs (quantum_resistant_p2p/vendor/oqs.py:318, 348, 372) for the
// variants FrodoKEMKeyExchange selects by default (use_aes=True,
// quantum_resistant_p2p/crypto/key_exchange.py:319, 332-343).
//
// Encryption uses one T-table T0 (SubBytes + MixColumns of one state byte) held in LDS
// replicated 32 times (entry x of lane l at dword 32x + (l & 31)): a ds_read_b32 wave
// access is two 32-lane groups on 32 banks, so every lane reads its own bank whatever the
// indices -- no bank conflicts.  T1..T3 are byte rotations of T0 (v_alignbit).
// State words are little-endian columns (byte r of word c = state[r][c]).
//
// Gen(A) structure exploited (per handshake, i = row of the lane, j = block column,
// uniform across the wave): after AddRoundKey only column 0 depends on (i, j); after
// round 1 columns 0 and 3 depend only on i and columns 1 and 2 only on j; after round 2
// every column is  lane_part(i) ^ uniform_part(j).  Rounds 1-2 therefore cost nothing
// per block: the per-row part is computed once per lane and the per-column-block part
// once per handshake (k_fr_aes_prep) and read with scalar loads.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace qrk {
namespace aes {

constexpr uint8_t gmul2(uint8_t x) { return (uint8_t)((x << 1) ^ ((x & 0x80) ? 0x1B : 0)); }
constexpr uint8_t gmul(uint8_t a, uint8_t b) {
  uint8_t r = 0;
  for (int i = 0; i < 8; ++i) {
    if (b & 1) r ^= a;
    a = gmul2(a);
    b >>= 1;
  }
  return r;
}
constexpr uint8_t ginv(uint8_t x) {  // x^254 in GF(2^8), square-and-multiply
  uint8_t r = 1, b = x;
  for (int e = 254; e; e >>= 1) {
    if (e & 1) r = gmul(r, b);
    b = gmul(b, b);
  }
  return r;
}
constexpr uint8_t rotl8(uint8_t x, int s) { return (uint8_t)((x << s) | (x >> (8 - s))); }
constexpr uint8_t sbox_of(int x) {  // FIPS 197 section 5.1.1: inverse, then the affine map
  const uint8_t b = ginv((uint8_t)x);
  return (uint8_t)(b ^ rotl8(b, 1) ^ rotl8(b, 2) ^ rotl8(b, 3) ^ rotl8(b, 4) ^ 0x63);
}
struct Tables {
  uint8_t s[256];
  uint32_t t0[256];  // 2s | s << 8 | s << 16 | 3s << 24: column contribution of state row 0
};
constexpr Tables make_tables() {
  Tables t{};
  for (int x = 0; x < 256; ++x) {
    const uint8_t s = sbox_of(x);
    t.s[x] = s;
    t.t0[x] = (uint32_t)gmul2(s) | (uint32_t)s << 8 | (uint32_t)s << 16 | (uint32_t)(gmul2(s) ^ s) << 24;
  }
  return t;
}
constexpr Tables TABC = make_tables();
__constant__ static const Tables TAB = TABC;

__device__ __forceinline__ uint32_t rot8(uint32_t x) { return __builtin_amdgcn_alignbit(x, x, 24); }
__device__ __forceinline__ uint32_t rot16(uint32_t x) { return __builtin_amdgcn_alignbit(x, x, 16); }
__device__ __forceinline__ uint32_t rot24(uint32_t x) { return __builtin_amdgcn_alignbit(x, x, 8); }
__device__ __forceinline__ uint32_t B(uint32_t w, int r) { return (w >> (8 * r)) & 0xFF; }

// ---- global-memory (constant table) forms, for the per-handshake prep
__device__ __forceinline__ uint32_t Tg(int k, uint32_t x) {
  const uint32_t t = TAB.t0[x];
  return k == 0 ? t : k == 1 ? rot8(t) : k == 2 ? rot16(t) : rot24(t);
}
// FIPS 197 section 5.2, little-endian words: RotWord = rotate right by 8, Rcon in byte 0.
__device__ __forceinline__ void expand_key(const uint32_t key[4], uint32_t rk[44]) {
  uint32_t rc = 1;
#pragma unroll
  for (int i = 0; i < 4; ++i) rk[i] = key[i];
#pragma unroll
  for (int i = 4; i < 44; ++i) {
    uint32_t t = rk[i - 1];
    if (i % 4 == 0) {
      t = __builtin_amdgcn_alignbit(t, t, 8);
      t = (uint32_t)TAB.s[B(t, 0)] | (uint32_t)TAB.s[B(t, 1)] << 8 | (uint32_t)TAB.s[B(t, 2)] << 16 |
          (uint32_t)TAB.s[B(t, 3)] << 24;
      t ^= rc;
      rc = (rc << 1) ^ ((rc & 0x80) ? 0x11B : 0);
    }
    rk[i] = rk[i - 4] ^ t;
  }
}

// Per-handshake Gen(A) data (u32 words), computed by k_fr_aes_prep:
//   [0..44)  round keys rk0..rk10
//   [44..48) C0, C3 (round-1 constants of the per-row columns), C1, C2 (per-block columns)
//   [48 + 4 jb .. +4) uniform part of the round-2 output for column block j = 8 jb
//   [ROWP + 4 i .. +4) per-row part of the round-2 output for row i (the column-major Gen(A) kernel,
//                      where the column block is the lane's and the row the loop's)
constexpr int PREP_HDR = 48;
template <int N>
constexpr int prep_rowp() { return PREP_HDR + 4 * (N / 8); }
template <int N>
constexpr int prep_words() { return prep_rowp<N>() + 4 * N; }

// ---- LDS-replicated T-table lookups (entry x at byte 256 x; lane slot s = lane & 31).
// Two replicated tables, T0 and T2 = rot16(T0), interleaved in one 64 KiB array: the 256 B
// row of entry x holds T0[x] replicated 32 times (bytes 0-127) then T2[x] replicated 32 times
// (bytes 128-255).  Lane slot s reads byte offset 256 x + 4 s (T0) or 256 x + 128 + 4 s (T2),
// i.e. (byte r of the state word) << 8 | tl -- one v_perm_b32 per lookup, where the
// single-table layout needs a shift and a v_and_or_b32.  A full-round column needs one
// rotation instead of three, because rotation distributes over XOR:
//   T0[a] ^ T1[b] ^ T2[c] ^ T3[d] = (T0[a] ^ T2[c]) ^ rot8(T0[b] ^ T2[d]).
struct Lds2 {
  const char* base;
  uint32_t tl0, tl2;  // 4 s and 128 + 4 s
  __device__ __forceinline__ static uint32_t addr(uint32_t w, int r, uint32_t tl) {
    return __builtin_amdgcn_perm(w, tl, 0x0C0C0000u | ((uint32_t)(4 + r) << 8));
  }
  __device__ __forceinline__ uint32_t t0(uint32_t w, int r) const {
    return *(const uint32_t*)(base + addr(w, r, tl0));
  }
  __device__ __forceinline__ uint32_t t2(uint32_t w, int r) const {
    return *(const uint32_t*)(base + addr(w, r, tl2));
  }
  // T_k[byte r of w] (generic form, used once per row)
  __device__ __forceinline__ uint32_t t(int k, uint32_t w, int r) const {
    return k == 0 ? t0(w, r) : k == 1 ? rot8(t0(w, r)) : k == 2 ? t2(w, r) : rot8(t2(w, r));
  }
};
__device__ __forceinline__ void fill_lds2(uint32_t* tab, int tid, int nthreads) {
  for (int e = tid; e < 256 * 64; e += nthreads) {
    const uint32_t v = TAB.t0[e >> 6];
    tab[e] = (e & 32) ? rot16(v) : v;
  }
}
__device__ __forceinline__ void round_full2(const Lds2& L, uint32_t s[4], const uint32_t* rk) {
  uint32_t o[4];
#pragma unroll
  for (int c = 0; c < 4; ++c)
    o[c] = L.t0(s[c], 0) ^ L.t2(s[(c + 2) & 3], 2) ^ rot8(L.t0(s[(c + 1) & 3], 1) ^ L.t2(s[(c + 3) & 3], 3)) ^ rk[c];
#pragma unroll
  for (int c = 0; c < 4; ++c) s[c] = o[c];
}
// Final round: S-box bytes sit in byte 1 of T0; two v_perm_b32 gather them.
__device__ __forceinline__ void round_last2(const Lds2& L, uint32_t s[4], const uint32_t* rk) {
  uint32_t o[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const uint32_t a = L.t0(s[c], 0), b = L.t0(s[(c + 1) & 3], 1), d = L.t0(s[(c + 2) & 3], 2),
                   e = L.t0(s[(c + 3) & 3], 3);
    const uint32_t lo = __builtin_amdgcn_perm(b, a, 0x0C0C0501u);  // [a.b1, b.b1, 0, 0]
    const uint32_t hi = __builtin_amdgcn_perm(e, d, 0x05010C0Cu);  // [0, 0, d.b1, e.b1]
    o[c] = (lo | hi) ^ rk[c];
  }
#pragma unroll
  for (int c = 0; c < 4; ++c) s[c] = o[c];
}
__device__ __forceinline__ void rounds_3_10_x2(const Lds2& L, uint32_t z[4], uint32_t w[4], const uint32_t* rk) {
#pragma unroll
  for (int r = 3; r < 10; ++r) {
    round_full2(L, z, rk + 4 * r);
    round_full2(L, w, rk + 4 * r);
  }
  round_last2(L, z, rk + 40);
  round_last2(L, w, rk + 40);
}

// row_part below from the constant-memory table (the prep kernel, no LDS table): k = rk0 word 0,
// c0 / c3 = the round-1 constants the prep header stores at [44] / [45]
__device__ __forceinline__ void row_part_g(uint32_t k, uint32_t c0, uint32_t c3, uint32_t i, uint32_t lp[4]) {
  const uint32_t y0 = Tg(0, (i ^ k) & 0xFF) ^ c0;
  const uint32_t y3 = Tg(1, ((i >> 8) ^ (k >> 8)) & 0xFF) ^ c3;
  lp[0] = Tg(0, B(y0, 0)) ^ Tg(3, B(y3, 3));
  lp[1] = Tg(2, B(y3, 2)) ^ Tg(3, B(y0, 3));
  lp[2] = Tg(1, B(y3, 1)) ^ Tg(2, B(y0, 2));
  lp[3] = Tg(0, B(y3, 0)) ^ Tg(1, B(y0, 1));
}

// Per-row part of the round-2 output for row i (prep header at hp, uniform).
template <class LT>
__device__ __forceinline__ void row_part(const LT& L, const uint32_t* hp, uint32_t i, uint32_t lp[4]) {
  const uint32_t k = hp[0];  // rk0 word 0 = k0 | k1 << 8 | ...
  const uint32_t y0 = L.t(0, (i ^ k) & 0xFF, 0) ^ hp[44];
  const uint32_t y3 = L.t(1, ((i >> 8) ^ (k >> 8)) << 8, 1) ^ hp[45];
  lp[0] = L.t(0, y0, 0) ^ L.t(3, y3, 3);
  lp[1] = L.t(2, y3, 2) ^ L.t(3, y0, 3);
  lp[2] = L.t(1, y3, 1) ^ L.t(2, y0, 2);
  lp[3] = L.t(0, y3, 0) ^ L.t(1, y0, 1);
}

}  // namespace aes
}  // namespace qrk
