// Wave-cooperative Keccak-f[1600] for gfx950: one sponge state spread over one wave.
//
// Used where one handshake's sponge chain is the critical path (the ML-KEM single-shot kernels:
// H(ek), J(z || c), G, the PRFs and SampleNTT of one handshake; the FrodoKEM / HQC long sponges
// below 256 handshakes: H(pk), the SE stream, ss, the seedexpanders and the K hash), not for large
// batches, where one state per lane (keccak.cuh) keeps every lane busy.  One wave64 issues one VALU instruction per 4 cycles,
// so the 4320-instruction lane-per-state permutation costs about 9 us on a single wave; spread
// over the lanes it costs ~20 VALU + 10 lane permutes per round.
//
// Layout: row y of the state in lanes 8y .. 8y + 7, lane 8y + s holding column
// (s + 4) mod 5 -- columns 0-4 at slots 1-5 plus replicas of columns 4, 0, 1 at slots 0, 6, 7 --
// as a lo/hi pair; lanes 40-47, 48-55 and 56-63 mirror row 4.  Per round:
//   theta : column parity = XOR over the rows: DPP row_ror:8, then v_permlane16_swap and
//           v_permlane32_swap butterflies; C[x-1] / C[x+1] are the neighbouring slots (DPP
//           row_shr:1 / row_shl:1), so theta needs no LDS round trip
//   rho   : per-lane rotation (pre-swap of the halves + two v_alignbit with a per-lane shift)
//   pi+chi: every slot (replicas too) gathers its three chi inputs B[X][Y], B[X+1][Y], B[X+2][Y]
//           straight from the canonical lanes pi moves them from (ds_bpermute), then a ^ (~b & c)
//   iota  : the (0, 0) lane and its replica
// Replicas absorb the same message words as their canonical lane, so they mirror it at every
// round start.  The three row-4 mirrors replace a column-parity mask: the first butterfly step
// leaves lanes 32-47 unpaired (row 4 twice) and pairs 48-55 with 56-63 (row 4 ^ row 4 = 0), so no
// lane needs masking and each round's chain is one instruction shorter: 6478 -> 6364 cycles per
// permutation alone, ML-KEM-768 single-shot calls -0.35 to -0.6 us
// (profiles/r4/single_shot/{coop_probe,latency}_mirror_rows_ab.*).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "keccak.cuh"

namespace qrk {

// This layout against the round-1 one (lane y + 8x, C[x -/+ 1] by ds_bpermute, two LDS round trips
// per round): alone on a CU both cost ~6.6k cycles per permutation (profiles/r2/keccak_coop_v1_v2.txt),
// but beside the SampleNTT waves of a single-shot kernel its fewer ds_bpermutes (the LDS crossbar is
// shared by the CU's waves) take ML-KEM-768 Encaps' H(ek) + G chain from 37.2 to 33.2 us
// (profiles/r2/single_shot_trace_coop_ab.json).  chi's B[X+1], B[X+2] come from the neighbouring
// slots by DPP (2 ds_bpermute per round instead of 6; slots 6, 7 refreshed from 1, 2 after the
// round): 6477 against 6218 cycles alone, but the chain 31.6 -> 30.6 us and SampleNTT 12.1 -> 9.8 us
// inside the kernel.

struct Coop {
  int idx;          // state index x + 5y held by this lane (replica lanes too)
  int a_m1, a_p1;   // zero (round-1 layout fields; kept so kf_coop's argument layout is unchanged)
  int g0, g1, g2;   // ds_bpermute byte addresses of the chi inputs B[X][Y], B[X+1][Y], B[X+2][Y]
  uint32_t shift;   // rho: v_alignbit shift (32 - r mod 32) mod 32
  bool swap;        // rho: swap the halves first
  uint32_t m0;      // all-ones where iota applies (lane (0, 0) and its replica)
  bool hi_slots;    // slots 6, 7 (refreshed from slots 1, 2)
  uint32_t hsm;     // all-ones on slots 6, 7
};

// v2: lane s + 8y (slot s = 0..7 of row y) holds column x(s) = (s + 4) mod 5: columns 0-4 at slots
// 1-5 (canonical), replicas of columns 4, 0, 1 at slots 0, 6, 7, so C[x-1] and C[x+1] of every
// canonical slot are the neighbouring lanes of the same 16-lane row (DPP row_shr:1 / row_shl:1).
__device__ __forceinline__ int coop_lane_of(int i) { return (i % 5) + 1 + 8 * (i / 5); }  // canonical lane of x + 5y

__device__ __forceinline__ Coop coop_init() {
  // rotation offsets r[x + 5y] (FIPS 202 Table 2)
  constexpr uint8_t RHO[25] = {0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43, 25, 39, 41, 45, 15, 21, 8, 18, 2, 61, 56, 14};
  Coop c;
  const int l = threadIdx.x & 63;
  const int sl = l & 7, y = (l >> 3) < 4 ? (l >> 3) : 4;  // lanes 40-63: three mirrors of row 4
  const int x = (sl + 4) % 5;
  c.idx = x + 5 * y;
  c.a_m1 = c.a_p1 = 0;
  auto lane_xy = [](int xx, int yy) { return 4 * (xx + 1 + 8 * yy); };
  const int X0 = x, X1 = (x + 1) % 5, X2 = (x + 2) % 5, Y = y;
  c.g0 = lane_xy((3 * Y + X0) % 5, X0);
  c.g1 = lane_xy((3 * Y + X1) % 5, X1);
  c.g2 = lane_xy((3 * Y + X2) % 5, X2);
  c.m0 = (sl == 1 && y == 0) ? 0xFFFFFFFFu : 0u;  // the replica at slot 6 is refreshed from slot 1
  c.hi_slots = sl >= 6;
  c.hsm = sl >= 6 ? 0xFFFFFFFFu : 0u;
  const int r = RHO[x + 5 * y];
  const int n = r & 31;
  c.shift = (uint32_t)((32 - n) & 31);
  c.swap = (r >= 32) != (n == 0);  // alignbit by 0 returns the low operand: r = 0 needs the swap
  return c;
}

__device__ __forceinline__ uint32_t dpp_shr1(uint32_t v) {  // lane l <- lane l - 1 (same row)
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x111, 0xF, 0xF, true);
}
__device__ __forceinline__ uint32_t dpp_shl1(uint32_t v) {  // lane l <- lane l + 1 (same row)
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x101, 0xF, 0xF, true);
}
__device__ __forceinline__ uint32_t dpp_shl2(uint32_t v) {  // lane l <- lane l + 2 (same row)
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x102, 0xF, 0xF, true);
}
__device__ __forceinline__ uint32_t dpp_shr5(uint32_t v) {  // lane l <- lane l - 5 (same row)
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x115, 0xF, 0xF, true);
}
// a DPP shift (CTRL) with the 16-lane rows whose ROWS bit is clear left at 0 (0x128: row_ror:8)
template <int CTRL, int ROWS>
__device__ __forceinline__ uint32_t dpp_rows(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROWS, 0xF, true);
}
__device__ __forceinline__ uint32_t bperm(int addr, uint32_t v) { return (uint32_t)__builtin_amdgcn_ds_bpermute(addr, (int)v); }

// 24 rounds on the wave's state (lo, hi of this lane's A[x][y]); every lane of the wave calls it.
__device__ __forceinline__ void keccak_f_coop(uint32_t& lo, uint32_t& hi, const Coop& c) {
  // sl_ / sh_: copies of lo / hi that the first butterfly step overwrites in place (the next
  // round's come out of the slot refresh as a v_bitop3 select beside the v_cndmask one)
  uint32_t sl_ = lo, sh_ = hi;
#pragma unroll 24
  for (int r = 0; r < 24; ++r) {
    // column parity over the rows: pairs within a 16-lane row (DPP row_ror:8) for rows 0-3, while
    // lanes 32-47 keep row 4 (16-lane row 2 masked) and lanes 48-63 (two copies of row 4) cancel
    // to zero; then across rows (permlane swaps); every lane ends with C[x(s)]
    uint32_t cl = sl_ ^ dpp_rows<0x128, 0xB>(sl_), ch = sh_ ^ dpp_rows<0x128, 0xB>(sh_);
    // lo and hi share the cross-row butterflies: swap16(cl, ch) leaves rows 0/2 with lo pair sums
    // and rows 1/3 with hi pair sums; swap32 completes them; a last swap16 hands every lane both.
    // Each swap takes two registers holding the same sum: the second copy is a v_bitop3 XOR
    // (which the compiler does not merge with the v_xor) instead of a v_mov after it -- same
    // latency alone, but 2 fewer dependent instructions per round cut the ML-KEM-768 single-shot
    // kernels by ~1.1 us (profiles/r4/single_shot/latency_butterfly_mov_vs_bitop3.jsonl)
    {
      const auto p = __builtin_amdgcn_permlane16_swap(cl, ch, false, false);
      const uint32_t t = p[0] ^ p[1], t2 = __builtin_amdgcn_bitop3_b32(p[0], p[1], p[1], 0x3C);
      const auto q = __builtin_amdgcn_permlane32_swap(t, t2, false, false);
      const uint32_t u = q[0] ^ q[1], u2 = __builtin_amdgcn_bitop3_b32(q[0], q[1], q[1], 0x3C);
      const auto w = __builtin_amdgcn_permlane16_swap(u, u2, false, false);
      cl = w[0];
      ch = w[1];
    }
    const uint32_t ml = dpp_shr1(cl), mh = dpp_shr1(ch);
    const uint32_t pl = dpp_shl1(cl), ph = dpp_shl1(ch);
    lo = xor3(lo, ml, __builtin_amdgcn_alignbit(pl, ph, 31));
    hi = xor3(hi, mh, __builtin_amdgcn_alignbit(ph, pl, 31));
    const uint32_t sl = c.swap ? hi : lo, sh = c.swap ? lo : hi;
    lo = __builtin_amdgcn_alignbit(sl, sh, c.shift);
    hi = __builtin_amdgcn_alignbit(sh, sl, c.shift);
    const uint32_t b0l = bperm(c.g0, lo), b0h = bperm(c.g0, hi);
    const uint32_t b1l = dpp_shl1(b0l), b1h = dpp_shl1(b0h);
    const uint32_t b2l = dpp_shl2(b0l), b2h = dpp_shl2(b0h);
    lo = (b0l ^ (~b1l & b2l)) ^ (KRC_LO[r] & c.m0);
    hi = (b0h ^ (~b1h & b2h)) ^ (KRC_HI[r] & c.m0);
    const uint32_t rl = dpp_shr5(lo), rh = dpp_shr5(hi);
    sl_ = __builtin_amdgcn_bitop3_b32(c.hsm, rl, lo, 0xCA);  // hsm ? rl : lo
    sh_ = __builtin_amdgcn_bitop3_b32(c.hsm, rh, hi, 0xCA);
    lo = c.hi_slots ? rl : lo;
    hi = c.hi_slots ? rh : hi;
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
// The permutation inlined at every call site.  As a call (one copy per kernel) every entry began
// with s_waitcnt vmcnt(0) lgkmcnt(0), which waited for the caller's outstanding stores and
// prefetch loads before the first round; inlined, the waits sit at the uses: ML-KEM-768 OQS
// keypair / encaps / decaps 56.6 / 55.4 / 44.2 -> 54.2 / 53.8 / 42.9 us, FrodoKEM-640-AES
// single calls -6 % (profiles/r4/single_shot/*_coop_call_vs_inline.jsonl).
static __device__ __forceinline__
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
