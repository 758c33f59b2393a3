// Wave-cooperative Keccak-f[1600] for gfx950: one sponge state spread over one wave.
//
// Used where one handshake's sponge chain is the critical path (the single-shot kernels: H(ek),
// J(z || c), G, the PRFs and SampleNTT of one handshake), not for batches, where one state per
// lane (keccak.cuh) keeps every lane busy.  One wave64 issues one VALU instruction per 4 cycles,
// so the 4320-instruction lane-per-state permutation costs about 9 us on a single wave; spread
// over the lanes it costs ~20 VALU + 10 lane permutes per round.
//
// Layout: lane y + 8x holds A[x][y] (FIPS 202 lane (x, y)) as a lo/hi pair.  Lanes with x >= 5
// or y >= 5 hold zero for the whole permutation.  Per round:
//   theta : column parity = XOR over the 8 lanes of group x: three DPP steps (quad_perm 1032,
//           quad_perm 2301, row_half_mirror) per half; C[x-1], C[x+1] fetched with ds_bpermute
//   rho   : per-lane rotation (pre-swap of the halves + two v_alignbit with a per-lane shift)
//   pi+chi: each lane gathers its three chi inputs B[X][Y], B[X+1][Y], B[X+2][Y] straight from
//           the lanes pi moves them from (ds_bpermute), then a ^ (~b & c)
//   iota  : lane 0 only (round constant masked by a lane-0 mask)
// Idle lanes point every permute at lane 40 (x = 5: always zero), so they stay zero.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "keccak.cuh"

namespace qrk {

struct Coop {
  int idx;          // state index x + 5y of this lane, or -1 for an idle lane
  int a_m1, a_p1;   // ds_bpermute byte addresses of C[x-1], C[x+1]
  int g0, g1, g2;   // ... of the chi inputs B[X][Y], B[X+1][Y], B[X+2][Y]
  uint32_t shift;   // rho: v_alignbit shift (32 - r mod 32) mod 32
  bool swap;        // rho: swap the halves first
  uint32_t m0;      // all-ones on lane 0 (iota)
};

__device__ __forceinline__ int coop_lane_of(int i) { return (i / 5) + 8 * (i % 5); }  // i = x + 5y -> y + 8x

__device__ __forceinline__ Coop coop_init() {
  // rotation offsets r[x + 5y] (FIPS 202 Table 2)
  constexpr uint8_t RHO[25] = {0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43, 25, 39, 41, 45, 15, 21, 8, 18, 2, 61, 56, 14};
  Coop c;
  const int l = threadIdx.x & 63, x = l >> 3, y = l & 7;
  const bool v = x < 5 && y < 5;
  constexpr int Z = 40;
  c.idx = v ? x + 5 * y : -1;
  c.a_m1 = 4 * (v ? y + 8 * ((x + 4) % 5) : Z);
  c.a_p1 = 4 * (v ? y + 8 * ((x + 1) % 5) : Z);
  // B[X][Y] = rot(A[x][y]) with (X, Y) = (y, 2x + 3y): the source of B[X'][Y] is (3Y + X', X')
  const int X0 = x, X1 = (x + 1) % 5, X2 = (x + 2) % 5, Y = y;
  c.g0 = 4 * (v ? X0 + 8 * ((3 * Y + X0) % 5) : Z);
  c.g1 = 4 * (v ? X1 + 8 * ((3 * Y + X1) % 5) : Z);
  c.g2 = 4 * (v ? X2 + 8 * ((3 * Y + X2) % 5) : Z);
  const int r = v ? RHO[x + 5 * y] : 0;
  const int n = r & 31;
  c.shift = (uint32_t)((32 - n) & 31);
  c.swap = (r >= 32) != (n == 0);  // alignbit by 0 returns the low operand: r = 0 needs the swap
  c.m0 = l == 0 ? 0xFFFFFFFFu : 0u;
  return c;
}

__device__ __forceinline__ uint32_t dpp_q1032(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);
}
__device__ __forceinline__ uint32_t dpp_q2301(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);
}
__device__ __forceinline__ uint32_t dpp_half_mirror(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, false);
}
__device__ __forceinline__ uint32_t bperm(int addr, uint32_t v) { return (uint32_t)__builtin_amdgcn_ds_bpermute(addr, (int)v); }

// 24 rounds on the wave's state (lo, hi of this lane's A[x][y]); every lane of the wave calls it.
#ifndef QRK_COOP_UNROLL
#define QRK_COOP_UNROLL 24  // fully unrolled: 6.6k cycles per permutation against 8.7k rolled (tools/coop_ab.sh)
#endif
__device__ __forceinline__ void keccak_f_coop(uint32_t& lo, uint32_t& hi, const Coop& c) {
#pragma unroll QRK_COOP_UNROLL
  for (int r = 0; r < 24; ++r) {
    uint32_t cl = lo, ch = hi;
    cl ^= dpp_q1032(cl);
    ch ^= dpp_q1032(ch);
    cl ^= dpp_q2301(cl);
    ch ^= dpp_q2301(ch);
    cl ^= dpp_half_mirror(cl);
    ch ^= dpp_half_mirror(ch);
    const uint32_t ml = bperm(c.a_m1, cl), mh = bperm(c.a_m1, ch);
    const uint32_t pl = bperm(c.a_p1, cl), ph = bperm(c.a_p1, ch);
    lo = xor3(lo, ml, __builtin_amdgcn_alignbit(pl, ph, 31));
    hi = xor3(hi, mh, __builtin_amdgcn_alignbit(ph, pl, 31));
    const uint32_t sl = c.swap ? hi : lo, sh = c.swap ? lo : hi;
    lo = __builtin_amdgcn_alignbit(sl, sh, c.shift);
    hi = __builtin_amdgcn_alignbit(sh, sl, c.shift);
    const uint32_t b0l = bperm(c.g0, lo), b0h = bperm(c.g0, hi);
    const uint32_t b1l = bperm(c.g1, lo), b1h = bperm(c.g1, hi);
    const uint32_t b2l = bperm(c.g2, lo), b2h = bperm(c.g2, hi);
    lo = (b0l ^ (~b1l & b2l)) ^ (KRC_LO[r] & c.m0);
    hi = (b0h ^ (~b1h & b2h)) ^ (KRC_HI[r] & c.m0);
  }
}

}  // namespace qrk
