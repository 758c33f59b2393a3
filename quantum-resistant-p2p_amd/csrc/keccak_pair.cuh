// Keccak-f[1600] on a lane pair, for sponges whose latency, not throughput, bounds a launch.
//
// Lane 2p holds the low 32 bits of all 25 state words, lane 2p + 1 the high 32 bits.  Column parity,
// theta's XOR, chi and iota are bitwise and stay in the lane; pi is register renaming as in the
// lane-per-state form (keccak.cuh).  A 64-bit rotation needs both halves: each lane takes its
// partner's half by one DPP quad_perm [1,0,3,2] and keeps one funnel shift, the same instruction for
// both lanes (new half = alignbit(own, partner, 32 - r) for r < 32, alignbit(partner, own, 64 - r)
// for r > 32).  Per round and lane: 10 XOR3 (parity) + 5 DPP + 5 funnel shifts (rot-1 of C) + 25 XOR3
// (theta) + 24 DPP + 24 funnel shifts (rho) + 25 bitop3 (chi) + 2 (iota) = 120 instructions, 29 of
// them half-rate, against 180 (58 half-rate) for one lane holding the whole state: a chain of sponge
// permutations finishes ~1.5x sooner on two lanes at 1.3x the issue slots per state.  Used for the
// ML-KEM batched Encaps front (H(ek) + G) and Decaps' G(m' || h) at chunks of at most 2^15
// handshakes, where one lane-per-handshake wave per SIMD was the critical path of the launch
// (DESIGN.md section 4, round 5).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "keccak.cuh"

namespace qrk {

struct PState {
  uint32_t a[25];  // this lane's half (low: even lane, high: odd lane) of state word x + 5y
};

__device__ __forceinline__ void pzero(PState& s) {
#pragma unroll
  for (int i = 0; i < 25; ++i) s.a[i] = 0u;
}

// the partner lane's value (lane l ^ 1): DPP quad_perm [1, 0, 3, 2]
__device__ __forceinline__ uint32_t pswap(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, true);
}

template <int N>
__device__ __forceinline__ uint32_t prol(uint32_t own, uint32_t other) {
  static_assert(N != 32, "no rotation by 32 in Keccak");
  if constexpr (N == 0)
    return own;
  else if constexpr (N < 32)
    return __builtin_amdgcn_alignbit(own, other, 32 - N);
  else
    return __builtin_amdgcn_alignbit(other, own, 64 - N);
}

// hm: all-ones on the high-half lane of the pair, zero on the low-half lane
__device__ __forceinline__ void keccak_pair(PState& s, uint32_t hm) {
#pragma unroll 2
  for (int r = 0; r < 24; ++r) {
    uint32_t C[5], R[5], B[25];
#pragma unroll
    for (int x = 0; x < 5; ++x) C[x] = xor3(xor3(s.a[x], s.a[x + 5], s.a[x + 10]), s.a[x + 15], s.a[x + 20]);
#pragma unroll
    for (int x = 0; x < 5; ++x) R[x] = prol<1>(C[x], pswap(C[x]));
#pragma unroll
    for (int i = 0; i < 25; ++i) s.a[i] = xor3(s.a[i], C[(i % 5 + 4) % 5], R[(i % 5 + 1) % 5]);
    // rho + pi: B[y + 5((2x + 3y) % 5)] = rot(A[x + 5y], r[x][y])
    B[0] = s.a[0];
    B[10] = prol<1>(s.a[1], pswap(s.a[1]));
    B[20] = prol<62>(s.a[2], pswap(s.a[2]));
    B[5] = prol<28>(s.a[3], pswap(s.a[3]));
    B[15] = prol<27>(s.a[4], pswap(s.a[4]));
    B[16] = prol<36>(s.a[5], pswap(s.a[5]));
    B[1] = prol<44>(s.a[6], pswap(s.a[6]));
    B[11] = prol<6>(s.a[7], pswap(s.a[7]));
    B[21] = prol<55>(s.a[8], pswap(s.a[8]));
    B[6] = prol<20>(s.a[9], pswap(s.a[9]));
    B[7] = prol<3>(s.a[10], pswap(s.a[10]));
    B[17] = prol<10>(s.a[11], pswap(s.a[11]));
    B[2] = prol<43>(s.a[12], pswap(s.a[12]));
    B[12] = prol<25>(s.a[13], pswap(s.a[13]));
    B[22] = prol<39>(s.a[14], pswap(s.a[14]));
    B[23] = prol<41>(s.a[15], pswap(s.a[15]));
    B[8] = prol<45>(s.a[16], pswap(s.a[16]));
    B[18] = prol<15>(s.a[17], pswap(s.a[17]));
    B[3] = prol<21>(s.a[18], pswap(s.a[18]));
    B[13] = prol<8>(s.a[19], pswap(s.a[19]));
    B[14] = prol<18>(s.a[20], pswap(s.a[20]));
    B[24] = prol<2>(s.a[21], pswap(s.a[21]));
    B[9] = prol<61>(s.a[22], pswap(s.a[22]));
    B[19] = prol<56>(s.a[23], pswap(s.a[23]));
    B[4] = prol<14>(s.a[24], pswap(s.a[24]));
#pragma unroll
    for (int y = 0; y < 5; ++y)
#pragma unroll
      for (int x = 0; x < 5; ++x)
        s.a[x + 5 * y] = B[x + 5 * y] ^ (~B[(x + 1) % 5 + 5 * y] & B[(x + 2) % 5 + 5 * y]);
    s.a[0] ^= (KRC_HI[r] & hm) | (KRC_LO[r] & ~hm);
  }
}

// Absorb NW 64-bit message words (ld32(w): this lane's 32-bit half of word w), padded with domain
// byte DS at byte 8 NW; RW = rate in words.  Every lane of the wave calls it.
template <int RW, int NW, uint32_t DS, typename Loader>
__device__ __forceinline__ void pabsorb(PState& s, uint32_t hm, Loader ld32) {
  constexpr int NFULL = NW / RW, TAIL = NW % RW;
#pragma unroll 1
  for (int b = 0; b < NFULL; ++b) {
#pragma unroll
    for (int w = 0; w < RW; ++w) s.a[w] ^= ld32(b * RW + w);
    keccak_pair(s, hm);
  }
#pragma unroll
  for (int w = 0; w < TAIL; ++w) s.a[w] ^= ld32(NFULL * RW + w);
  s.a[TAIL] ^= DS & ~hm;
  s.a[RW - 1] ^= 0x80000000u & hm;
  keccak_pair(s, hm);
}

}  // namespace qrk
