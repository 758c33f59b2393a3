// Wave-cooperative Keccak-f[1600] for gfx950: one sponge state spread over one wave.
//
// Used where one handshake's sponge chain is the critical path (the ML-KEM single-shot kernels:
// H(ek), J(z || c), G, the PRFs and SampleNTT of one handshake; the FrodoKEM / HQC long sponges
// below 256 handshakes: H(pk), the SE stream, ss, the seedexpanders and the K hash), not for large
// batches, where one state per lane (keccak.cuh) keeps every lane busy.  One wave64 issues one VALU instruction per 4 cycles,
// so the 4320-instruction lane-per-state permutation costs about 9 us on a single wave; spread
// over the lanes it costs ~20 VALU + 10 lane permutes per round.
//
// Layout (v2): row y of the state in lanes 8y .. 8y + 7, lane 8y + s holding column
// (s + 4) mod 5 -- columns 0-4 at slots 1-5 plus replicas of columns 4, 0, 1 at slots 0, 6, 7 --
// as a lo/hi pair; lanes 40-63 are idle.  Per round:
//   theta : column parity = XOR over the rows: DPP row_ror:8, then v_permlane16_swap and
//           v_permlane32_swap butterflies; C[x-1] / C[x+1] are the neighbouring slots (DPP
//           row_shr:1 / row_shl:1), so theta needs no LDS round trip
//   rho   : per-lane rotation (pre-swap of the halves + two v_alignbit with a per-lane shift)
//   pi+chi: every slot (replicas too) gathers its three chi inputs B[X][Y], B[X+1][Y], B[X+2][Y]
//           straight from the canonical lanes pi moves them from (ds_bpermute), then a ^ (~b & c)
//   iota  : the (0, 0) lane and its replica
// Replicas absorb the same message words as their canonical lane, so they mirror it at every
// round start.  v1 (QRK_COOP_V1=1, default): lane y + 8x, column parity by DPP quad/half-mirror
// steps and C[x -/+ 1] by ds_bpermute (two LDS round trips per round); lanes outside the 5 x 5
// block stay zero (their permutes read lane 40).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "keccak.cuh"

namespace qrk {

// v2 (default) against v1 (QRK_COOP_V1=1): alone on a CU both cost ~6.6k cycles per permutation
// (profiles/r2/keccak_coop_v1_v2.txt), but beside the SampleNTT waves of a single-shot kernel v2's
// fewer ds_bpermutes (the LDS crossbar is shared by the CU's waves) take ML-KEM-768 Encaps' H(ek) + G
// chain from 37.2 to 33.2 us (profiles/r2/single_shot_trace_coop_ab.json).
// QRK_COOP_CHI_DPP=1 (v2 only, default): chi's B[X+1], B[X+2] from the neighbouring slots by DPP (2
// ds_bpermute per round instead of 6; slots 6, 7 refreshed from 1, 2 after the round): 6477 against
// 6218 cycles alone, but the chain 31.6 -> 30.6 us and SampleNTT 12.1 -> 9.8 us inside the kernel.
#ifndef QRK_COOP_V1
#define QRK_COOP_V1 0
#endif
#ifndef QRK_COOP_CHI_DPP
#define QRK_COOP_CHI_DPP 1
#endif

struct Coop {
  int idx;          // state index x + 5y held by this lane (replica lanes too), or -1 for an idle lane
  int a_m1, a_p1;   // v1: ds_bpermute byte addresses of C[x-1], C[x+1]
  int g0, g1, g2;   // ds_bpermute byte addresses of the chi inputs B[X][Y], B[X+1][Y], B[X+2][Y]
  uint32_t shift;   // rho: v_alignbit shift (32 - r mod 32) mod 32
  bool swap;        // rho: swap the halves first
  uint32_t m0;      // all-ones where iota applies (lane (0, 0) and its replica)
  uint32_t live;    // v2: all-ones on the 40 state lanes (the column parity ignores the rest)
  bool hi_slots;    // v2 + QRK_COOP_CHI_DPP: slots 6, 7 (refreshed from slots 1, 2)
};

#if QRK_COOP_V1
__device__ __forceinline__ int coop_lane_of(int i) { return (i / 5) + 8 * (i % 5); }  // i = x + 5y -> y + 8x
#else
// v2: lane s + 8y (slot s = 0..7 of row y) holds column x(s) = (s + 4) mod 5: columns 0-4 at slots
// 1-5 (canonical), replicas of columns 4, 0, 1 at slots 0, 6, 7, so C[x-1] and C[x+1] of every
// canonical slot are the neighbouring lanes of the same 16-lane row (DPP row_shr:1 / row_shl:1).
__device__ __forceinline__ int coop_lane_of(int i) { return (i % 5) + 1 + 8 * (i / 5); }  // canonical lane of x + 5y
#endif

__device__ __forceinline__ Coop coop_init() {
  // rotation offsets r[x + 5y] (FIPS 202 Table 2)
  constexpr uint8_t RHO[25] = {0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43, 25, 39, 41, 45, 15, 21, 8, 18, 2, 61, 56, 14};
  Coop c;
  const int l = threadIdx.x & 63;
#if QRK_COOP_V1
  const int x = l >> 3, y = l & 7;
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
  c.live = v ? 0xFFFFFFFFu : 0u;
  c.m0 = l == 0 ? 0xFFFFFFFFu : 0u;
#else
  const int sl = l & 7, y = l >> 3;
  const bool v = y < 5;
  const int x = (sl + 4) % 5;
  c.idx = v ? x + 5 * y : -1;
  c.a_m1 = c.a_p1 = 0;
  auto lane_xy = [](int xx, int yy) { return 4 * (xx + 1 + 8 * yy); };
  const int X0 = x, X1 = (x + 1) % 5, X2 = (x + 2) % 5, Y = y;
  c.g0 = v ? lane_xy((3 * Y + X0) % 5, X0) : 4 * l;
  c.g1 = v ? lane_xy((3 * Y + X1) % 5, X1) : 4 * l;
  c.g2 = v ? lane_xy((3 * Y + X2) % 5, X2) : 4 * l;
  c.live = v ? 0xFFFFFFFFu : 0u;
#if QRK_COOP_CHI_DPP
  c.m0 = (v && sl == 1 && y == 0) ? 0xFFFFFFFFu : 0u;  // the replica at slot 6 is refreshed from slot 1
#else
  c.m0 = (v && x == 0 && y == 0) ? 0xFFFFFFFFu : 0u;
#endif
  c.hi_slots = sl >= 6;
#endif
  const int r = v ? RHO[x + 5 * y] : 0;
  const int n = r & 31;
  c.shift = (uint32_t)((32 - n) & 31);
  c.swap = (r >= 32) != (n == 0);  // alignbit by 0 returns the low operand: r = 0 needs the swap
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
__device__ __forceinline__ uint32_t dpp_ror8(uint32_t v) {  // lane l <- lane (l + 8) mod 16 of its row
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x128, 0xF, 0xF, true);
}
__device__ __forceinline__ uint32_t dpp_shr1(uint32_t v) {  // lane l <- lane l - 1 (same row)
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x111, 0xF, 0xF, true);
}
__device__ __forceinline__ uint32_t dpp_shl1(uint32_t v) {  // lane l <- lane l + 1 (same row)
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x101, 0xF, 0xF, true);
}
// XOR of lane l and lane l ^ 16 / l ^ 32 (gfx950 v_permlane16_swap / v_permlane32_swap)
__device__ __forceinline__ uint32_t xor_swap16(uint32_t v) {
  const auto p = __builtin_amdgcn_permlane16_swap(v, v, false, false);
  return p[0] ^ p[1];
}
__device__ __forceinline__ uint32_t xor_swap32(uint32_t v) {
  const auto p = __builtin_amdgcn_permlane32_swap(v, v, false, false);
  return p[0] ^ p[1];
}
__device__ __forceinline__ uint32_t dpp_shl2(uint32_t v) {  // lane l <- lane l + 2 (same row)
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x102, 0xF, 0xF, true);
}
__device__ __forceinline__ uint32_t dpp_shr5(uint32_t v) {  // lane l <- lane l - 5 (same row)
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x115, 0xF, 0xF, true);
}
__device__ __forceinline__ uint32_t bperm(int addr, uint32_t v) { return (uint32_t)__builtin_amdgcn_ds_bpermute(addr, (int)v); }

// 24 rounds on the wave's state (lo, hi of this lane's A[x][y]); every lane of the wave calls it.
#ifndef QRK_COOP_UNROLL
#define QRK_COOP_UNROLL 24  // fully unrolled: 6.6k cycles per permutation against 8.7k rolled (tools/coop_ab.sh)
#endif
__device__ __forceinline__ void keccak_f_coop(uint32_t& lo, uint32_t& hi, const Coop& c) {
#pragma unroll QRK_COOP_UNROLL
  for (int r = 0; r < 24; ++r) {
#if QRK_COOP_V1
    uint32_t cl = lo, ch = hi;
    cl ^= dpp_q1032(cl);
    ch ^= dpp_q1032(ch);
    cl ^= dpp_q2301(cl);
    ch ^= dpp_q2301(ch);
    cl ^= dpp_half_mirror(cl);
    ch ^= dpp_half_mirror(ch);
    const uint32_t ml = bperm(c.a_m1, cl), mh = bperm(c.a_m1, ch);
    const uint32_t pl = bperm(c.a_p1, cl), ph = bperm(c.a_p1, ch);
#else
    // column parity over the 8 rows (rows 5-7 and idle lanes masked): pairs within a 16-lane
    // row (DPP row_ror:8), then across rows (permlane swaps); every lane ends with C[x(s)]
    uint32_t cl = lo & c.live, ch = hi & c.live;
    cl ^= dpp_ror8(cl);
    ch ^= dpp_ror8(ch);
    // lo and hi share the cross-row butterflies: swap16(cl, ch) leaves rows 0/2 with lo pair sums
    // and rows 1/3 with hi pair sums; swap32 completes them; a last swap16 hands every lane both
    {
      const auto p = __builtin_amdgcn_permlane16_swap(cl, ch, false, false);
      const uint32_t t = p[0] ^ p[1];
      const auto q = __builtin_amdgcn_permlane32_swap(t, t, false, false);
      const uint32_t u = q[0] ^ q[1];
      const auto w = __builtin_amdgcn_permlane16_swap(u, u, false, false);
      cl = w[0];
      ch = w[1];
    }
    const uint32_t ml = dpp_shr1(cl), mh = dpp_shr1(ch);
    const uint32_t pl = dpp_shl1(cl), ph = dpp_shl1(ch);
#endif
    lo = xor3(lo, ml, __builtin_amdgcn_alignbit(pl, ph, 31));
    hi = xor3(hi, mh, __builtin_amdgcn_alignbit(ph, pl, 31));
    const uint32_t sl = c.swap ? hi : lo, sh = c.swap ? lo : hi;
    lo = __builtin_amdgcn_alignbit(sl, sh, c.shift);
    hi = __builtin_amdgcn_alignbit(sh, sl, c.shift);
#if !QRK_COOP_V1 && QRK_COOP_CHI_DPP
    const uint32_t b0l = bperm(c.g0, lo), b0h = bperm(c.g0, hi);
    const uint32_t b1l = dpp_shl1(b0l), b1h = dpp_shl1(b0h);
    const uint32_t b2l = dpp_shl2(b0l), b2h = dpp_shl2(b0h);
    lo = (b0l ^ (~b1l & b2l)) ^ (KRC_LO[r] & c.m0);
    hi = (b0h ^ (~b1h & b2h)) ^ (KRC_HI[r] & c.m0);
    const uint32_t rl = dpp_shr5(lo), rh = dpp_shr5(hi);
    lo = c.hi_slots ? rl : lo;
    hi = c.hi_slots ? rh : hi;
#else
    const uint32_t b0l = bperm(c.g0, lo), b0h = bperm(c.g0, hi);
    const uint32_t b1l = bperm(c.g1, lo), b1h = bperm(c.g1, hi);
    const uint32_t b2l = bperm(c.g2, lo), b2h = bperm(c.g2, hi);
    lo = (b0l ^ (~b1l & b2l)) ^ (KRC_LO[r] & c.m0);
    hi = (b0h ^ (~b1h & b2h)) ^ (KRC_HI[r] & c.m0);
#endif
  }
}

// One sponge state spread over the wave: this lane's 64-bit word (index Coop::idx).
struct CState {
  uint32_t lo = 0, hi = 0;
};
__device__ __forceinline__ void cs_xor(CState& s, uint64_t w) {
  s.lo ^= (uint32_t)w;
  s.hi ^= (uint32_t)(w >> 32);
}
__device__ __forceinline__ uint64_t cs_word(const CState& s) { return ((uint64_t)s.hi << 32) | s.lo; }
// word w (per lane) of the state, fetched from the lane that holds it
__device__ __forceinline__ uint64_t cs_get(const CState& s, int w) {
  const int a = 4 * coop_lane_of(w);
  return ((uint64_t)bperm(a, s.hi) << 32) | bperm(a, s.lo);
}
// the permutation as a call (one copy of the unrolled rounds per kernel, not one per call site);
// QRK_COOP_CALL=0 inlines it at every call site
#ifndef QRK_COOP_CALL
#define QRK_COOP_CALL 1
#endif
#if QRK_COOP_CALL
static __device__ __noinline__
#else
__device__ __forceinline__
#endif
CState kf_coop(CState s, Coop c) {
  keccak_f_coop(s.lo, s.hi, c);
  return s;
}

// Sponge absorb of NW message words ld(0..NW-1) at rate RW, padded with domain byte DS; the
// lanes holding state words 0..RW-1 each load their word of the next block before the current
// block's permutation.
template <int RW, int NW, uint32_t DS, typename Loader>
__device__ __forceinline__ void coop_absorb(CState& s, const Coop& c, Loader ld) {
  constexpr int NFULL = NW / RW, TAIL = NW % RW;
  const int i = c.idx;
  const bool rl = i >= 0 && i < RW;
  uint64_t nxt = (rl && (NFULL > 0 || i < TAIL)) ? ld(i) : 0;
#pragma unroll 1
  for (int b = 0; b < NFULL; ++b) {
    cs_xor(s, nxt);
    nxt = (rl && (b + 1 < NFULL || i < TAIL)) ? ld((b + 1) * RW + i) : 0;
    s = kf_coop(s, c);
  }
  cs_xor(s, nxt);
  if (i == TAIL) s.lo ^= DS;
  if (i == RW - 1) s.hi ^= 0x80000000u;
  s = kf_coop(s, c);
}


// the lane that owns state word c.idx (replica lanes mirror it and must not write outputs twice)
__device__ __forceinline__ bool coop_canon(const Coop& c) {
  return c.idx >= 0 && (int)(threadIdx.x & 63) == coop_lane_of(c.idx);
}

// Squeeze NW words of an absorbed sponge: word w goes to out(w, value) on the lane that holds
// it (lanes idx < RW of each block), permuting between blocks.
template <int RW, typename Store>
__device__ __forceinline__ void coop_squeeze(CState& s, const Coop& c, int NW, Store out) {
  const int i = c.idx;
  const bool rl = i >= 0 && i < RW;
  int w = 0;
#pragma unroll 1
  while (true) {
    if (rl && w + i < NW) out(w + i, cs_word(s));
    w += RW;
    if (w >= NW) break;
    s = kf_coop(s, c);
  }
}

}  // namespace qrk
