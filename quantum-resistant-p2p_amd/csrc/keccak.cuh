// Device Keccak-f[1600] for gfx950: one sponge state per lane.
//
// The 25 64-bit lanes are held as 50 VGPRs (lo/hi 32-bit halves).  Per round:
//   theta   : 20 v_bitop3 (column parity, XOR3) + 10 v_alignbit (rot-1)
//             + 50 v_bitop3 (a ^ C[x-1] ^ rot(C[x+1]) fused as one XOR3 per half)
//   rho/pi  : 48 v_alignbit/v_perm (funnel-shift rotates; pi is register renaming)
//   chi     : 50 v_bitop3 (a ^ (~b & c), selected by the compiler)
//   iota    : 2 v_xor
// = 180 VALU instructions per round, 4320 per permutation, no moves; 58 of them (the rotations)
// issue at half rate on gfx950, and so do the 64-bit shifts that could replace them
// (tools/rot64_probe.hip).  Two rounds per loop iteration (45.3 against 44.2 Top/s at one,
// profiles/r2/rot64_unroll_probe.json).
// XOR3 is emitted through inline asm because hipcc (ROCm 7.2) splits
// __builtin_amdgcn_bitop3_b32(...,0x96) back into two v_xor_b32.
//
// Replaces the Keccak inside liboqs that the reference reaches through
// quantum_resistant_p2p/vendor/oqs.py:318,348,372 (OQS_KEM_keypair/encaps/decaps).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace qrk {

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  uint32_t r;
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}


struct u2 {
  uint32_t lo, hi;
};

// 64-bit rotation as two funnel shifts.  (One 64-bit shift + one 32-bit shift + OR is no cheaper:
// the 64-bit shifts issue at half rate too, 38.7 against 44.1 Top/s, profiles/r2/rot64_probe.json.)

template <int N>
__device__ __forceinline__ u2 rol(u2 x) {
  if constexpr (N == 0) {
    return x;
  } else if constexpr (N == 32) {
    return {x.hi, x.lo};
  } else if constexpr (N < 32) {
    return {__builtin_amdgcn_alignbit(x.lo, x.hi, 32 - N), __builtin_amdgcn_alignbit(x.hi, x.lo, 32 - N)};
  } else {
    return {__builtin_amdgcn_alignbit(x.hi, x.lo, 64 - N), __builtin_amdgcn_alignbit(x.lo, x.hi, 64 - N)};
  }
}

__constant__ static const uint32_t KRC_LO[24] = {
    0x00000001u, 0x00008082u, 0x0000808au, 0x80008000u, 0x0000808bu, 0x80000001u,
    0x80008081u, 0x00008009u, 0x0000008au, 0x00000088u, 0x80008009u, 0x8000000au,
    0x8000808bu, 0x0000008bu, 0x00008089u, 0x00008003u, 0x00008002u, 0x00000080u,
    0x0000800au, 0x8000000au, 0x80008081u, 0x00008080u, 0x80000001u, 0x80008008u};
__constant__ static const uint32_t KRC_HI[24] = {
    0x00000000u, 0x00000000u, 0x80000000u, 0x80000000u, 0x00000000u, 0x00000000u,
    0x80000000u, 0x80000000u, 0x00000000u, 0x00000000u, 0x00000000u, 0x00000000u,
    0x00000000u, 0x80000000u, 0x80000000u, 0x80000000u, 0x80000000u, 0x80000000u,
    0x00000000u, 0x80000000u, 0x80000000u, 0x80000000u, 0x00000000u, 0x80000000u};

// Sponge state: lane (x, y) of FIPS 202 at index x + 5y.  Only ever indexed
// with compile-time constants (fully unrolled loops) so it stays in VGPRs.
struct KState {
  u2 a[25];
};

__device__ __forceinline__ void kzero(KState& s) {
#pragma unroll
  for (int i = 0; i < 25; ++i) s.a[i] = {0u, 0u};
}

// U rounds per loop iteration (24 = fully unrolled)
template <int U = 2>
__device__ __forceinline__ void keccak_fu(KState& s) {
#pragma unroll U
  for (int r = 0; r < 24; ++r) {
    u2 C[5], R[5], B[25];
#pragma unroll
    for (int x = 0; x < 5; ++x) {
      C[x].lo = xor3(xor3(s.a[x].lo, s.a[x + 5].lo, s.a[x + 10].lo), s.a[x + 15].lo, s.a[x + 20].lo);
      C[x].hi = xor3(xor3(s.a[x].hi, s.a[x + 5].hi, s.a[x + 10].hi), s.a[x + 15].hi, s.a[x + 20].hi);
    }
#pragma unroll
    for (int x = 0; x < 5; ++x) R[x] = rol<1>(C[x]);
#pragma unroll
    for (int i = 0; i < 25; ++i) {
      const int x = i % 5;
      s.a[i].lo = xor3(s.a[i].lo, C[(x + 4) % 5].lo, R[(x + 1) % 5].lo);
      s.a[i].hi = xor3(s.a[i].hi, C[(x + 4) % 5].hi, R[(x + 1) % 5].hi);
    }
    // rho + pi: B[y + 5*((2x + 3y) % 5)] = rot(A[x + 5y], r[x][y])
    B[0] = s.a[0];
    B[10] = rol<1>(s.a[1]);
    B[20] = rol<62>(s.a[2]);
    B[5] = rol<28>(s.a[3]);
    B[15] = rol<27>(s.a[4]);
    B[16] = rol<36>(s.a[5]);
    B[1] = rol<44>(s.a[6]);
    B[11] = rol<6>(s.a[7]);
    B[21] = rol<55>(s.a[8]);
    B[6] = rol<20>(s.a[9]);
    B[7] = rol<3>(s.a[10]);
    B[17] = rol<10>(s.a[11]);
    B[2] = rol<43>(s.a[12]);
    B[12] = rol<25>(s.a[13]);
    B[22] = rol<39>(s.a[14]);
    B[23] = rol<41>(s.a[15]);
    B[8] = rol<45>(s.a[16]);
    B[18] = rol<15>(s.a[17]);
    B[3] = rol<21>(s.a[18]);
    B[13] = rol<8>(s.a[19]);
    B[14] = rol<18>(s.a[20]);
    B[24] = rol<2>(s.a[21]);
    B[9] = rol<61>(s.a[22]);
    B[19] = rol<56>(s.a[23]);
    B[4] = rol<14>(s.a[24]);
#pragma unroll
    for (int y = 0; y < 5; ++y)
#pragma unroll
      for (int x = 0; x < 5; ++x) {
        const u2 b0 = B[x + 5 * y], b1 = B[(x + 1) % 5 + 5 * y], b2 = B[(x + 2) % 5 + 5 * y];
        s.a[x + 5 * y].lo = b0.lo ^ (~b1.lo & b2.lo);
        s.a[x + 5 * y].hi = b0.hi ^ (~b1.hi & b2.hi);
      }
    s.a[0].lo ^= KRC_LO[r];
    s.a[0].hi ^= KRC_HI[r];
  }
}
__device__ __forceinline__ void keccak_f(KState& s) { keccak_fu<2>(s); }

__device__ __forceinline__ void kxor(KState& s, int i, uint64_t w) {
  // i must be a compile-time constant after inlining
  s.a[i].lo ^= (uint32_t)w;
  s.a[i].hi ^= (uint32_t)(w >> 32);
}

__device__ __forceinline__ uint64_t kword(const KState& s, int i) {
  return ((uint64_t)s.a[i].hi << 32) | s.a[i].lo;
}

// Absorb a message of NW 64-bit words (little-endian) produced by `ld(w)`,
// then pad with domain byte DS at byte offset 8*NW.  RW = rate in words.
// NW is a compile-time constant so every state index is static.
// PF: the next block's words are loaded into registers before the current block's permutation
// runs, so global-load latency hides behind the 24 rounds (2 x RW VGPRs).  Without PF each block's
// words are loaded when absorbed: fewer VGPRs, which is what matters where the sponge shares a
// multi-role launch with SampleNTT (the launch's VGPR budget is the larger role's): the ML-KEM
// Encaps front and J(z || c) drop from 127 / 130 to 82 / 87 VGPRs and their launches run
// SampleNTT at 5 waves / SIMD (2^16 handshakes +2.2 %, 2^20 unchanged,
// profiles/r4/schedule_ab/abx_*_absorb_noprefetch.jsonl).  Alone, prefetching was no slower for
// ML-KEM and faster for the FrodoKEM H(pk) and ss kernels (profiles/r2/ab_absorb_prefetch.jsonl).
template <int RW, int NW, uint32_t DS, bool PF = true, typename Loader>
__device__ __forceinline__ void absorb_words(KState& s, Loader ld) {
  constexpr int NFULL = NW / RW;
  constexpr int TAIL = NW % RW;
  if constexpr (!PF) {
#pragma unroll 1
    for (int b = 0; b < NFULL; ++b) {
#pragma unroll
      for (int w = 0; w < RW; ++w) kxor(s, w, ld(b * RW + w));
      keccak_f(s);
    }
#pragma unroll
    for (int w = 0; w < TAIL; ++w) kxor(s, w, ld(NFULL * RW + w));
    s.a[TAIL].lo ^= DS;
    s.a[RW - 1].hi ^= 0x80000000u;
    keccak_f(s);
    return;
  }
  uint64_t nxt[RW];
#pragma unroll
  for (int w = 0; w < RW; ++w) nxt[w] = (NFULL > 0 || w < TAIL) ? ld(w) : 0;
#pragma unroll 1
  for (int b = 0; b < NFULL; ++b) {
#pragma unroll
    for (int w = 0; w < RW; ++w) kxor(s, w, nxt[w]);
    const int nb = (b + 1) * RW;
#pragma unroll
    for (int w = 0; w < RW; ++w) nxt[w] = (b + 1 < NFULL || w < TAIL) ? ld(nb + w) : 0;
    keccak_f(s);
  }
#pragma unroll
  for (int w = 0; w < TAIL; ++w) kxor(s, w, nxt[w]);
  s.a[TAIL].lo ^= DS;
  s.a[RW - 1].hi ^= 0x80000000u;
  keccak_f(s);
}

constexpr uint32_t DS_SHA3 = 0x06u;
constexpr uint32_t DS_SHAKE = 0x1Fu;
constexpr int RW_SHAKE128 = 21;
constexpr int RW_SHAKE256 = 17;
constexpr int RW_SHA3_256 = 17;
constexpr int RW_SHA3_512 = 9;

}  // namespace qrk
