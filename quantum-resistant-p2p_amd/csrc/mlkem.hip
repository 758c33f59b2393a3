// ML-KEM-512/768/1024 (FIPS 203) batched KeyGen / Encaps / Decaps for gfx950.
//
// Replaces, for N handshakes at once, the liboqs calls the reference makes one
// at a time: OQS_KEM_keypair / OQS_KEM_encaps / OQS_KEM_decaps
// (quantum_resistant_p2p/vendor/oqs.py:318, :348, :372), reached from
// MLKEMKeyExchange.generate_keypair / encapsulate / decapsulate
// (quantum_resistant_p2p/crypto/key_exchange.py:125-186).
//
// Decomposition (DESIGN.md "Kernels"): every handshake is split into
// independent Keccak instances, each run by one lane, and polynomial stages,
// each run by a 16-lane group per handshake.
//
//   front / J / G  lane / handshake   H(ek), G(.), J(z||c)            (SHA3 / SHAKE256)
//   PRFs           lane / (nonce, hs)  PRF_eta(seed, N) raw bytes     (SHAKE256)
//   SampleNTT      lane / (x, y, hs)   3 SHAKE128 blocks, compacted to 12-bit chunks in the
//                                      producer; the ~0.7 % of entries that need a 4th block
//                                      go on a fix-up list (lane or wave per entry)
//   keygen / encrypt / decrypt cores
//                  16 lanes / hs       CBD, NTT, basemul, invNTT, compress/encode,
//                                      FO re-encrypt compare + implicit rejection
//
// Independent stages of one operation share multi-role launches (k_multi, roles in grid order,
// every kernel on the caller's stream); n <= 1024 runs one-launch kernels with wave-cooperative
// sponges instead (the reference's one-call-per-handshake pattern).  Keccak output goes to device
// scratch in a 64-instance tiled SoA layout (word w of instance i at ((i/64)*W + w)*64 + i%64):
// every lane-per-instance store is a fully coalesced 512-byte wave store.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "keccak.cuh"
#include "keccak_coop.cuh"
#include "keccak_pair.cuh"
#include "qrkem_internal.h"

namespace qrk {
namespace mlkem {

constexpr int Q = 3329;
// The batched SampleNTT output holds 12-bit coefficients (384 B per matrix entry, 8 per 12-byte
// chunk) rather than int16 (512 B): the encrypt core waits on memory, not on the VALU (SQ wait_any
// 0.28-0.35 after the round-3 arithmetic cut its VALU instructions 20 % with no change in time), and
// the matrix is 58 % of its HBM reads.
constexpr int XOF_W = 48;    // u64 words per matrix entry in scratch
constexpr int PRF_W = 24;    // up to 192 B of PRF output (eta = 3)

// ---------------------------------------------------------------- tables
constexpr int powq(int b, int e) {
  long r = 1;
  for (int i = 0; i < e; ++i) r = (r * b) % Q;
  return (int)r;
}
constexpr int br7(int i) {
  int r = 0;
  for (int b = 0; b < 7; ++b) r |= ((i >> b) & 1) << (6 - b);
  return r;
}
constexpr int centered(long x) {
  x %= Q;
  if (x < 0) x += Q;
  return (int)(x > Q / 2 ? x - Q : x);
}

// Plain-domain twiddles as fp32 (centered integers, exact): the NTTs run in fp32.  zq is z
// divided by q (rounded to fp32) for the three-FMA modular product below.
struct TablesF {
  float z[128];  // zeta^br7(i) mod q
  float g[128];  // gamma_i = zeta^(2 br7(i) + 1) mod q
  float zq[128];
};
constexpr TablesF make_tables_f() {
  TablesF t{};
  for (int i = 0; i < 128; ++i) {
    t.z[i] = (float)centered(powq(17, br7(i)));
    t.g[i] = (float)centered(powq(17, 2 * br7(i) + 1));
    t.zq[i] = (float)((double)t.z[i] / 3329.0);
  }
  return t;
}
constexpr TablesF TABFC = make_tables_f();
__constant__ TablesF TABFD = make_tables_f();
constexpr float INV128F = (float)centered(3303);  // 128^-1 mod q (plain domain) = -26
// zeta_1 * 128^-1: the inverse NTT's last layer folds the 128^-1 scaling into its twiddle
constexpr float Z1INV128F = (float)centered((long)powq(17, br7(1)) * 3303);

// ---------------------------------------------------------------- arithmetic
// x < 0 ? -1 : 0 as one v_ashrrev_i32 (inline asm, so the compiler keeps the mask arithmetic
// instead of turning it back into v_cmp + v_cndmask_e64, whose SGPR lane mask costs a VOP3
// issue and hazard wait states)
__device__ __forceinline__ int sign_mask(int x) {
  int r;
  asm("v_ashrrev_i32 %0, 31, %1" : "=v"(r) : "v"(x));
  return r;
}
// ---- fp32 modular arithmetic (every value is an exact integer below 2^24)
// MAGIC = 1.5 * 2^23: x + MAGIC rounds x to an integer (round-to-nearest-even), and
// for |x| < 2^22 the bit pattern of x + MAGIC is 0x4B400000 + x, so its low 16 bits
// are x as int16.  All ops below are full-rate on gfx950 (v_mul/v_add/v_fmaak/v_fmamk
// _f32), unlike the 24/32-bit integer multiplies (half rate).
constexpr float QF = 3329.0f;
constexpr float QINVF = 1.0f / 3329.0f;
constexpr float MAGIC = 12582912.0f;
// p - t q.  (Forcing v_fmamk_f32 with a literal -q through inline asm, in place of the v_fmac_f32
// the compiler picks at ~0.65 of the full rate, made the cores 7-10 % slower: hazard s_nops and
// lost v_pk_fma_f32 pairing, profiles/r3/ab_fmamk_rejected_and_wrap_probe.jsonl.)
__device__ __forceinline__ float fms_q(float t, float p) {  // p - t q
  return __builtin_fmaf(t, -QF, p);
}
// The modular product / reduction as three FMAs with MAGIC folded into the constants (below), where
// the round-2 form spent a product, a rounding FMA, the MAGIC subtraction and an FMA.
// MAGIC * q = 9987 * 2^22, exact in fp32
constexpr float MQF = MAGIC * QF;
// x mod q, centered: |result| <= 1665 for |x| < 2^24 (|x / q - rint| <= 1/2 + 3e-4)
// Three-FMA form: k = x/q + MAGIC rounds to MAGIC + kint (the binade [2^23, 2^24) has ulp 1);
// fma(k, -q, MAGIC q) = -q kint exactly (|q kint| < 2^24 for |x| <= 1.677e7); x + that is exact.
__device__ __forceinline__ float reduce_f(float x) {
  const float k = __builtin_fmaf(x, QINVF, MAGIC);
  return x + __builtin_fmaf(k, -QF, MQF);
}
// x * z mod q, centered, exact when |x * z| < 2^24 (for |z| <= 1664: |x| < 10082).
// zq = fl(z / q).  Three FMAs: k = MAGIC + round(x zq) (|x zq - x z / q| < 3e-4, so the
// result stays within q/2 + 1), n = -q round(.) exactly, then x z + n with one rounding of an
// exact integer below 2^24.  The round-2 form spent a product, the MAGIC
// subtraction and a three-VGPR fmac (0.65 of the full rate, profiles/r1/valu_peak_r1b.json).
__device__ __forceinline__ float modmul_f(float x, float z, float zq) {
  const float k = __builtin_fmaf(x, zq, MAGIC);
  return __builtin_fmaf(x, z, __builtin_fmaf(k, -QF, MQF));
}
// The same product for lane-indexed twiddles (the NTT layers after the transpose, basemul gamma)
// stays on the round-2 form: its single constant per twiddle holds fewer live registers than z
// and z / q together.  The three-FMA form there (z / q from a table or from z * (1/q)) cost the
// encrypt core a wave per SIMD (170 VGPRs: 2.64 against 2.29 ms per 2^20 launch) and the decrypt
// core one too (106 against 91 VGPRs: 0.95 against 0.90 ms), profiles/r3/ab_core_arith_*.jsonl.
__device__ __forceinline__ float modmul_lf(float x, float z) {
  const float p = x * z;
  const float t = __builtin_fmaf(p, QINVF, MAGIC) - MAGIC;
  return fms_q(t, p);
}
__device__ __forceinline__ float i2f(int x) {  // |x| < 2^22
  return __int_as_float(0x4B400000 + x) - MAGIC;
}
__device__ __forceinline__ int f2i(float x) {  // exact integer, |x| < 2^22
  return __float_as_int(x + MAGIC) - 0x4B400000;
}
__device__ __forceinline__ uint32_t f2bits(float x) {  // low 16 bits = x as int16
  return __float_as_uint(x + MAGIC);
}
// canonical [0, q) integer of an exact fp32 integer
__device__ __forceinline__ int canon_f(float x) {
  const int r = f2i(reduce_f(x));
  return r + (sign_mask(r) & Q);
}
// basemul accumulator (|acc| < 2^31) -> centered residue: acc = hi 2^16 + lo with
// 2^16 = -1044 (mod q), |hi * 1044 + lo| < 5.1e6 (exact), then one reduction
// With HI = MAGIC + hi and LO = MAGIC + lo as bit patterns (no MAGIC subtractions),
// fma(HI, -1044, 1043 MAGIC) = -MAGIC - 1044 hi is an exact integer below 2^24 (|hi| < 2^11) and
// adding LO leaves lo - 1044 hi exactly: two full-rate ops where the round-2 form spent two
// subtractions and a three-VGPR fmac.
__device__ __forceinline__ float acc_to_f(int acc) {
  const float hi = __int_as_float(0x4B400000 + (acc >> 16)), lo = __int_as_float(0x4B400000 | (acc & 0xFFFF));
  return reduce_f(__builtin_fmaf(hi, -1044.0f, 1043.0f * MAGIC) + lo);
}

// Compress_d(x) = round(2^d x / q) mod 2^d for x in [0, q): exact via 24-bit mulhi
template <int D>
__device__ __forceinline__ int compress(int x) {
  const uint32_t y = ((uint32_t)x << D) + (Q / 2);
  return (int)(__umulhi(y, 1290168u) & ((1u << D) - 1));
}
// Compress_d of any exact fp32 integer v congruent to x mod q, |v| <= 4091 (no reduction first):
// fma(v, fl(2^d / q), MAGIC) rounds v 2^d / q to an integer whose low d bits are
// round(x 2^d / q) mod 2^d (adding q to v adds 2^d).  Correct rounding: v 2^(d+1) is even and
// (2k + 1) q odd, so v 2^d / q is at least 1 / (2q) = 1.5e-4 from every half-integer, and the
// constant's relative error 2^-24 moves it by at most 2517 * 2^-24 < 1.5e-4 for
// |v 2^d / q| <= 2517.  Two full-rate ops where canon_f + compress spent about twelve.
template <int D>
__device__ __forceinline__ int compress_f(float v) {
  constexpr float C = (float)((double)(1 << D) / 3329.0);
  return (int)(__float_as_uint(__builtin_fmaf(v, C, MAGIC)) & ((1u << D) - 1));
}
template <int D>
__device__ __forceinline__ int decompress(int y) {
  return (int)(((uint32_t)Q * (uint32_t)y + (1u << (D - 1))) >> D);
}

// Tiled scratch layouts: word w of instance i at ((i / TW) W + w) TW + i % TW -- TW = 64 for the
// batched kernels (one coalesced wave store per word), 16 for the small path's LDS copies.
template <int TW = 64>
__device__ __forceinline__ size_t tidx(size_t inst, int w, int W) {
  return ((inst / TW) * (size_t)W + (size_t)w) * TW + (inst % TW);
}

// 16-lane group synchronisation: a group never spans two waves, so ordering
// LDS traffic inside the wave is enough.
__device__ __forceinline__ void gsync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// 8 consecutive 12-bit fields of the little-endian 96-bit string w0|w1|w2
__device__ __forceinline__ void split12(uint32_t w0, uint32_t w1, uint32_t w2, int c[8]) {
  c[0] = (int)(w0 & 0xFFF);
  c[1] = (int)((w0 >> 12) & 0xFFF);
  c[2] = (int)(__builtin_amdgcn_alignbit(w1, w0, 24) & 0xFFF);
  c[3] = (int)((w1 >> 4) & 0xFFF);
  c[4] = (int)((w1 >> 16) & 0xFFF);
  c[5] = (int)(__builtin_amdgcn_alignbit(w2, w1, 28) & 0xFFF);
  c[6] = (int)((w2 >> 8) & 0xFFF);
  c[7] = (int)(w2 >> 20);
}

// ============================================================ lane-per-instance Keccak kernels

// SampleNTT (FIPS 203 Alg. 7), one lane per matrix entry: SHAKE128(rho || x || y)
// squeezed block by block until 256 values < q have been accepted (3 blocks
// with probability ~0.993, rarely 4).  Compaction happens in the producer:
// every candidate is written to a 16-entry per-lane LDS ring at the running
// count (a rejected one is simply overwritten by the next), and each completed
// 8-coefficient chunk is flushed as one 16-byte store.  The ring is
// lane-interleaved (entry i of lane l at dword i*64 + l of the wave's ring), so
// every lane always hits its own LDS bank: the random per-lane write offsets
// never conflict.  Output: 256 int16 coefficients per entry in a 64-entry tiled
// layout of 12-bit chunks (see XUnit below), so the consumer reads them without any
// parsing.  inst = (x*K + y) * C + hs.
constexpr int MAX_XOF_BLOCKS = 16;

// Rejected SampleNTT acceptance forms (A/B on one box, no faster than v_cmp + v_cndmask): a sign
// mask (three full-rate ops, profiles/r2/ab_xof_signmask_rejected.jsonl) and a shifted difference
// advancing the ring position by (c - q) >> 23 (profiles/r2/ab_xof_acc_rejected.jsonl).

// (a & m) | b as one v_bitop3_b32 (truth table 0xEA): full rate on gfx950, where
// v_and_or_b32 issues at half rate (profiles/r1/valu_peak_r1b.json)
__device__ __forceinline__ uint32_t and_or3(uint32_t a, uint32_t m, uint32_t b) {
  uint32_t r;
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0xea" : "=v"(r) : "v"(a), "s"(m), "v"(b));
  return r;
}

// Compact one squeezed SHAKE128 block (112 candidates) into the lane's ring,
// flushing completed 8-coefficient chunks to dst.
// `rb` = byte offset of the lane's ring column inside ring_all (wave * 4096 + lane * 4): bits
// 8-11 are zero, so an entry address is one v_bitop3_b32, (pos & 0xF00) | rb, with the static
// LDS base folded into the ds_write offset.
// A completed chunk's 8 ring entries are read when it completes and packed + stored one triplet
// later (or after the block), so the LDS read latency is not waited for on the spot (-1.5 %,
// profiles/r2/ab_xof_pipe_flush.jsonl).
// One 8-coefficient chunk of the batched SampleNTT output: 12 bytes of 12-bit fields.
struct U3 {
  uint32_t x, y, z;
};
// Tile units of two consecutive chunks (24 B): chunk pair p of entry i at ((i / TW) 16 + p) TW +
// i % TW, so a consumer lane's 16 coefficients are 24 contiguous bytes (one load pair instead of
// two 12-byte loads 768 B apart).  A/B on one box, four interleaved pairs
// (profiles/r3/final/ab_pair24.jsonl): encrypt core 1.97 -> 1.88 ms, fix-up 0.160 -> 0.103 ms per
// 2^20 launch, k_xof unchanged.
struct U6 {
  U3 h[2];
};
typedef U3 XChunk;
typedef U6 XUnit;
constexpr int XUNITS = 16;  // units per entry
// an entry's first unit, and chunk ch of it
template <int TW>
__device__ __forceinline__ XUnit* xent(XUnit* out, size_t inst) {
  return out + (inst / TW) * XUNITS * TW + (inst % TW);
}
template <int TW>
__device__ __forceinline__ XChunk* xc(XUnit* ent, int ch) {
  return &ent[(ch >> 1) * TW].h[ch & 1];
}
// r[j]: the chunk's coefficients (< 2^12, from the ring)
__device__ __forceinline__ void chunk_store(XChunk* dst, const uint32_t r[8]) {
  U3 w;
  w.x = r[0] | (r[1] << 12) | (r[2] << 24);
  w.y = (r[2] >> 8) | (r[3] << 4) | (r[4] << 16) | (r[5] << 28);
  w.z = (r[5] >> 4) | (r[6] << 8) | (r[7] << 20);
  *dst = w;
}
struct XofPend {
  uint32_t r[8];  // the chunk's ring entries, in order
  int ch = -1;    // its chunk index, -1: nothing pending
};
template <int TW = 64>
__device__ __forceinline__ void xof_pend_store(XofPend& pd, XUnit* dst) {
  if (pd.ch >= 0) {
    chunk_store(xc<TW>(dst, pd.ch), pd.r);
    pd.ch = -1;
  }
}

template <int TW = 64>
__device__ __forceinline__ void compact_block(const KState& s, char* ring_all, uint32_t rb, int& cnt, XUnit* dst,
                                              XofPend& pd) {
  const uint32_t* ring = (const uint32_t*)(ring_all + rb);
#pragma unroll
  for (int t = 0; t < 14; ++t) {  // 42 dwords = 14 triplets of 8 twelve-bit candidates
    uint32_t d[3];
#pragma unroll
    for (int e = 0; e < 3; ++e) {
      const int di = 3 * t + e;
      d[e] = (di & 1) ? s.a[di >> 1].hi : s.a[di >> 1].lo;
    }
    int c[8];
    split12(d[0], d[1], d[2], c);
    const int before = cnt;
    // cnt kept pre-scaled by 256 (the byte stride of one ring entry): per candidate
    // one and + add for the address and cmp + cndmask + add for the count
    int pos = cnt << 8;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      *(uint32_t*)(ring_all + and_or3(pos, 0xF00u, rb)) = (uint32_t)c[e];
      pos += c[e] < Q ? 256 : 0;
    }
    cnt = pos >> 8;
    const int ch = before >> 3;
    // the chunk completed one triplet ago: its ring reads were issued then, so they have
    // landed by now (a wave's LDS instructions execute in issue order, so the reads saw the
    // chunk before this triplet's writes could reuse its slots)
    xof_pend_store<TW>(pd, dst);
    if ((cnt >> 3) != ch && ch < 32) {
      const uint32_t* r = ring + (ch & 1) * 8 * 64;
#pragma unroll
      for (int j = 0; j < 8; ++j) pd.r[j] = r[j * 64];
      pd.ch = ch;
    }
  }
}


// Fix-up entries are recomputed from scratch.  (Resume records -- the sponge state, count and
// partial chunk saved after the 3rd block, so the fix-up needs one more permutation -- cut the
// fix-up from 0.35 to 0.25 ms but slowed k_xof 1.8 %: no net gain, profiles/r2/ab_xof_resume.jsonl.)
// Tile width 64 makes k_xof's stores one contiguous KB per wave; width 1 (each entry contiguous)
// sped the encrypt core up 4 % but slowed k_xof's scattered stores 4-8 % (net -2 %,
// profiles/r2/ab_xof_tile_width.jsonl).
constexpr int XTW = 64;

__device__ __forceinline__ void xof_init(KState& s, const uint64_t* __restrict__ rho, int xy, int K) {
  kzero(s);
#pragma unroll
  for (int w = 0; w < 4; ++w) kxor(s, w, rho[w]);
  s.a[4].lo ^= (uint32_t)(xy / K) | ((uint32_t)(xy % K) << 8) | (DS_SHAKE << 16);
  s.a[RW_SHAKE128 - 1].hi ^= 0x80000000u;
}

// squeeze + compact blocks: exactly NB of them (ALL = false), or until 256 values (ALL = true)
template <bool ALL, int NB, int TW = 64>
__device__ __forceinline__ void xof_blocks(KState& s, int& cnt, XUnit* __restrict__ dst, char* ring_all, uint32_t rb) {
  XofPend pd;
#pragma unroll 1
  for (int b = 0; b < NB && (!ALL || cnt < 256); ++b) {
    keccak_f(s);
    compact_block<TW>(s, ring_all, rb, cnt, dst, pd);
  }
  xof_pend_store<TW>(pd, dst);
}

// One SampleNTT entry inst = (x K + y) C + hs from scratch: SHAKE128(rho || x || y), ALL = false:
// exactly 3 blocks (returns the count, < 256 when a 4th block is needed); ALL = true: as many
// blocks as it takes.  rb = this lane's ring column (see compact_block).
template <int K, bool ALL, int TW = 64>
__device__ __forceinline__ int xof_entry(const uint64_t* __restrict__ rho, int xy, size_t inst, XUnit* __restrict__ out,
                                         char* ring_all, uint32_t rb) {
  XUnit* dst = xent<TW>(out, inst);
  KState s;
  xof_init(s, rho, xy, K);
  int cnt = 0;
  xof_blocks<ALL, ALL ? MAX_XOF_BLOCKS : 3, TW>(s, cnt, dst, ring_all, rb);
  return cnt;
}

// FIX == false: every entry squeezes exactly 3 blocks (uniform across the wave); the ~0.7 % that
// still lack 256 values go on the fix-up list.
// FIX == true: one lane per slot completes the entry (rewriting identical chunks on the
// from-scratch path), so the rare 4th block never idles a whole wave.
template <int K, bool FIX>
struct XofArgs {
  const uint8_t* rho_base;
  size_t rho_stride, n, C;
  XUnit* out;
  uint32_t *fix, *nfix;  // the fix-up list and its counter
  uint32_t* zero_next;   // main pass (chunks <= DIRECT_RHO_MAX): the counter the next call counts into
};
// block vb of nvb (FIX: the grid-stride walk over the list uses nvb)
template <int K, bool FIX>
__device__ __forceinline__ void xof_body(const XofArgs<K, FIX>& a, unsigned vb, unsigned nvb, uint32_t* ring_all) {
  const uint32_t rb = ((threadIdx.x >> 6) * 16 * 64 + (threadIdx.x & 63)) * 4;  // ring_all: [wave][16][64]
  char* ring = (char*)ring_all;
  if constexpr (!FIX) {
    if (vb == 0 && threadIdx.x == 0 && a.zero_next) *a.zero_next = 0u;
    const size_t e = (size_t)vb * 256 + threadIdx.x, hs = e % a.C;
    if (e >= (size_t)K * K * a.C || hs >= a.n) return;
    const int xy = (int)(e / a.C);
    const size_t inst = (size_t)xy * a.C + hs;
    KState s;
    xof_init(s, (const uint64_t*)(a.rho_base + hs * a.rho_stride), xy, K);
    int cnt = 0;
    xof_blocks<false, 3, XTW>(s, cnt, xent<XTW>(a.out, inst), ring, rb);
    if (cnt < 256) a.fix[atomicAdd(a.nfix, 1u)] = (uint32_t)inst;
  } else {
    const size_t stride = (size_t)nvb * 256, limit = (size_t)*a.nfix;
#pragma unroll 1
    for (size_t r = (size_t)vb * 256 + threadIdx.x; r < limit; r += stride) {
      const size_t inst = a.fix[r];
      xof_entry<K, true, XTW>((const uint64_t*)(a.rho_base + (inst % a.C) * a.rho_stride), (int)(inst / a.C), inst,
                              a.out, ring, rb);
    }
  }
}
constexpr int XOF_LDS = 4 * 16 * 64 * 4;  // the 256-thread block's compaction rings

// PRF producer: SHAKE256(seed || N) -> 64*eta bytes; inst = N * C + hs.
// eta = (N < eta1_upto) ? ETA1 : ETA2.
template <int ETA1, int ETA2, int TW = 64>
__device__ __forceinline__ void prf_inst(const uint64_t* __restrict__ seed, int N, size_t inst, int eta1_upto,
                                         uint64_t* __restrict__ prf) {
  const int eta = N < eta1_upto ? ETA1 : ETA2;
  KState s;
  kzero(s);
#pragma unroll
  for (int w = 0; w < 4; ++w) kxor(s, w, seed[w]);
  s.a[4].lo ^= (uint32_t)N | (DS_SHAKE << 8);
  s.a[RW_SHAKE256 - 1].hi ^= 0x80000000u;
  keccak_f(s);
  if (eta == 2) {
#pragma unroll
    for (int w = 0; w < 16; ++w) prf[tidx<TW>(inst, w, PRF_W)] = kword(s, w);
  } else {
#pragma unroll
    for (int w = 0; w < 17; ++w) prf[tidx<TW>(inst, w, PRF_W)] = kword(s, w);
    keccak_f(s);
#pragma unroll
    for (int w = 0; w < 7; ++w) prf[tidx<TW>(inst, 17 + w, PRF_W)] = kword(s, w);
  }
}


template <int K>
struct P {
  static constexpr int ETA1 = (K == 2) ? 3 : 2;
  static constexpr int ETA2 = 2;
  static constexpr int DU = (K == 4) ? 11 : 10;
  static constexpr int DV = (K == 4) ? 5 : 4;
  static constexpr int PK = 384 * K + 32;
  static constexpr int SK = 768 * K + 96;
  static constexpr int CT = 32 * (DU * K + DV);
};

// KeyGen front: (rho, sigma) = G(d || k).  rho -> pk[384k..] and dk's ek copy; sigma -> seeds.
template <int K>
__device__ __forceinline__ void front_keygen_hs(const uint8_t* __restrict__ coins, size_t hs, uint8_t* __restrict__ pk,
                                                uint8_t* __restrict__ sk, uint64_t* __restrict__ seeds,
                                                uint64_t* __restrict__ rho) {
  const uint64_t* d = (const uint64_t*)(coins + hs * 64);
  KState s;
  kzero(s);
#pragma unroll
  for (int w = 0; w < 4; ++w) kxor(s, w, d[w]);
  s.a[4].lo ^= (uint32_t)K | (DS_SHA3 << 8);
  s.a[RW_SHA3_512 - 1].hi ^= 0x80000000u;
  keccak_f(s);
  uint64_t* rho_pk = (uint64_t*)(pk + hs * P<K>::PK + 384 * K);
  uint64_t* rho_sk = (uint64_t*)(sk + hs * P<K>::SK + 768 * K);
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    rho_pk[w] = kword(s, w);
    rho_sk[w] = kword(s, w);
    seeds[hs * 4 + w] = kword(s, 4 + w);
    if (rho) rho[hs * 4 + w] = kword(s, w);
  }
}
template <int K>
__global__ __launch_bounds__(256) void k_front_keygen(const uint8_t* __restrict__ coins, size_t n,
                                                      uint8_t* __restrict__ pk, uint8_t* __restrict__ sk,
                                                      uint64_t* __restrict__ seeds, uint64_t* __restrict__ rho,
                                                      uint32_t* __restrict__ nfix) {
  const size_t hs = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (hs == 0) *nfix = 0;  // the SampleNTT fix-up counter (no memset launch)
  if (hs < n) front_keygen_hs<K>(coins, hs, pk, sk, seeds, rho);
}

// KeyGen back: dk = dk_pke || ek || H(ek) || z  (ek already copied by the core kernel)
template <int K>
__device__ __forceinline__ void back_keygen_hs(const uint8_t* __restrict__ coins, size_t hs,
                                               const uint8_t* __restrict__ pk, uint8_t* __restrict__ sk) {
  const uint64_t* ek = (const uint64_t*)(pk + hs * P<K>::PK);
  KState s;
  kzero(s);
  absorb_words<RW_SHA3_256, P<K>::PK / 8, DS_SHA3>(s, [&](int w) { return ek[w]; });
  uint64_t* tail = (uint64_t*)(sk + hs * P<K>::SK + 768 * K + 32);
  const uint64_t* z = (const uint64_t*)(coins + hs * 64 + 32);
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    tail[w] = kword(s, w);
    tail[4 + w] = z[w];
  }
}
template <int K>
__global__ __launch_bounds__(256) void k_back_keygen(const uint8_t* __restrict__ coins, size_t n,
                                                     const uint8_t* __restrict__ pk, uint8_t* __restrict__ sk) {
  const size_t hs = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (hs < n) back_keygen_hs<K>(coins, hs, pk, sk);
}

// Encaps front: (K, r) = G(m || H(ek)); K -> ss, r -> seeds
template <int K>
__device__ __forceinline__ void front_encaps_hs(const uint8_t* __restrict__ pk, const uint8_t* __restrict__ coins,
                                                size_t hs, uint8_t* __restrict__ ss, uint64_t* __restrict__ seeds) {
  const uint64_t* ek = (const uint64_t*)(pk + hs * P<K>::PK);
  KState s;
  kzero(s);
  absorb_words<RW_SHA3_256, P<K>::PK / 8, DS_SHA3, false>(s, [&](int w) { return ek[w]; });
  uint64_t h[4];
#pragma unroll
  for (int w = 0; w < 4; ++w) h[w] = kword(s, w);
  const uint64_t* m = (const uint64_t*)(coins + hs * 32);
  kzero(s);
  absorb_words<RW_SHA3_512, 8, DS_SHA3>(s, [&](int w) { return w < 4 ? m[w] : h[w - 4]; });
  uint64_t* K_out = (uint64_t*)(ss + hs * 32);
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    K_out[w] = kword(s, w);
    seeds[hs * 4 + w] = kword(s, 4 + w);
  }
}

// Decaps front: (K', r') = G(m' || h), Kbar = J(z || c)
template <int K>
__device__ __forceinline__ void g_decaps_hs(const uint8_t* __restrict__ sk, const uint64_t* __restrict__ mprime,
                                            size_t hs, uint64_t* __restrict__ seeds, uint64_t* __restrict__ kprime) {
  const uint64_t* h = (const uint64_t*)(sk + hs * P<K>::SK + 768 * K + 32);
  const uint64_t* m = mprime + hs * 4;
  KState s;
  kzero(s);
  absorb_words<RW_SHA3_512, 8, DS_SHA3>(s, [&](int w) { return w < 4 ? m[w] : h[w - 4]; });
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    kprime[hs * 4 + w] = kword(s, w);
    seeds[hs * 4 + w] = kword(s, 4 + w);
  }
}
template <int K>
__device__ __forceinline__ void j_decaps_hs(const uint8_t* __restrict__ ct, const uint8_t* __restrict__ sk, size_t hs,
                                            uint64_t* __restrict__ kbar) {
  const uint64_t* z = (const uint64_t*)(sk + hs * P<K>::SK + 768 * K + 64);
  const uint64_t* c = (const uint64_t*)(ct + hs * P<K>::CT);
  KState s;
  kzero(s);
  absorb_words<RW_SHAKE256, 4 + P<K>::CT / 8, DS_SHAKE, false>(s, [&](int w) { return w < 4 ? z[w] : c[w - 4]; });
#pragma unroll
  for (int w = 0; w < 4; ++w) kbar[hs * 4 + w] = kword(s, w);
}

// The Encaps front and G(m' || h) on a lane pair (keccak_pair.cuh: the even lane holds the low
// halves of the state words, the odd lane the high halves) for chunks of at most QRK_PAIR_FRONT_MAX
// handshakes: there the front's lane-per-handshake waves (one per SIMD at 2^14 handshakes) are the
// critical path of their launch (2^14: +8.8 %, 2^15: +1.5 %, profiles/r5/pair_fronts/).  (J on pairs
// lost: see decaps_impl.)  `half` = lane & 1, hm = all-ones on the odd lane.
template <int K>
__device__ __forceinline__ void front_encaps_pair(const uint8_t* __restrict__ pk, const uint8_t* __restrict__ coins,
                                                  size_t hs, int half, uint32_t hm, uint8_t* __restrict__ ss,
                                                  uint64_t* __restrict__ seeds) {
  const uint32_t* ek = (const uint32_t*)(pk + hs * P<K>::PK);
  PState s;
  pzero(s);
  pabsorb<RW_SHA3_256, P<K>::PK / 8, DS_SHA3>(s, hm, [&](int w) { return ek[2 * w + half]; });
  uint32_t h[4];
#pragma unroll
  for (int w = 0; w < 4; ++w) h[w] = s.a[w];
  const uint32_t* m = (const uint32_t*)(coins + hs * 32);
  pzero(s);
  pabsorb<RW_SHA3_512, 8, DS_SHA3>(s, hm, [&](int w) { return w < 4 ? m[2 * w + half] : h[w - 4]; });
  uint32_t* k_out = (uint32_t*)(ss + hs * 32);
  uint32_t* r_out = (uint32_t*)(seeds + hs * 4);
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    k_out[2 * w + half] = s.a[w];
    r_out[2 * w + half] = s.a[4 + w];
  }
}
template <int K>
__device__ __forceinline__ void g_decaps_pair(const uint8_t* __restrict__ sk, const uint64_t* __restrict__ mprime,
                                              size_t hs, int half, uint32_t hm, uint64_t* __restrict__ seeds,
                                              uint64_t* __restrict__ kprime) {
  const uint32_t* h = (const uint32_t*)(sk + hs * P<K>::SK + 768 * K + 32);
  const uint32_t* m = (const uint32_t*)(mprime + hs * 4);
  PState s;
  pzero(s);
  pabsorb<RW_SHA3_512, 8, DS_SHA3>(s, hm, [&](int w) { return w < 4 ? m[2 * w + half] : h[2 * (w - 4) + half]; });
  uint32_t* kp = (uint32_t*)(kprime + hs * 4);
  uint32_t* sd = (uint32_t*)(seeds + hs * 4);
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    kp[2 * w + half] = s.a[w];
    sd[2 * w + half] = s.a[4 + w];
  }
}

// ============================================================ 16-lane polynomial groups

struct P16 {
  int v[16];
};

// Per-group LDS: a padded 272-dword polynomial image (index j -> j + j/16, so both
// the stride image [L + 16m] and the contiguous image [16L + t] are conflict-free)
// plus 84 words of byte staging (raw XOF blocks, bit-packed encodings).
constexpr int PBUF = 272;
// 44 words of byte staging hold the largest packed polynomial (du = 11: 352 bytes).  The
// group stride is 368 dwords = 16 (mod 32): the two 16-lane groups that share a ds_* bank
// half (lanes 0-31 / 32-63) then use disjoint bank sets for every access pattern above.
constexpr int RAWW = 44;
// (Aliasing the byte staging onto the polynomial image -- 1088 B per group instead of 1472 -- was
// only needed by the rejected LDS-DMA matrix prefetch)
struct GroupLds {
  int poly[PBUF];
  uint64_t raw[RAWW];
  int pad[8];
};
static_assert(sizeof(GroupLds) / 4 % 32 == 16, "group stride must be 16 mod 32 dwords");
constexpr int GROUPS = 16;  // 256 threads

// ---- fp32 NTTs (plain domain).  Same data movement as the integer versions above.
struct PF16 {
  float v[16];
};

__device__ __forceinline__ void stride_to_contig_f(PF16& p, float* buf, int L) {
#pragma unroll
  for (int m = 0; m < 16; ++m) buf[L + 17 * m] = p.v[m];
  gsync();
#pragma unroll
  for (int t = 0; t < 16; ++t) p.v[t] = buf[17 * L + t];
  gsync();
}
__device__ __forceinline__ void contig_to_stride_f(PF16& p, float* buf, int L) {
#pragma unroll
  for (int t = 0; t < 16; ++t) buf[17 * L + t] = p.v[t];
  gsync();
#pragma unroll
  for (int m = 0; m < 16; ++m) p.v[m] = buf[L + 17 * m];
  gsync();
}

// FIPS 203 Alg. 9 in fp32.  In: stride layout (v[m] = f[L+16m]), |f| <= B0.
// Out: contiguous layout (v[t] = f[16L+t]).  Each layer adds at most 1665 to the
// bound and a layer's twiddle products must stay below 2^24 (|input| < 10082):
// B0 <= 3 (CBD) -> 3 + 6 * 1665 = 9993 before the last layer, output <= 11658.
// MIDRED (inputs up to q, e.g. decompressed u): reduce everything after layer 4;
// output <= 4 * 1665.
template <bool MIDRED>
__device__ __forceinline__ void ntt_fwd_f(PF16& p, float* buf, int L) {
#pragma unroll
  for (int lg = 0; lg < 4; ++lg) {
    const int step = 8 >> lg;
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      if (((m / step) & 1) == 0) {
        const int zi = (1 << lg) + m / (2 * step);
        const float t = modmul_f(p.v[m + step], TABFC.z[zi], TABFC.zq[zi]);
        p.v[m + step] = p.v[m] - t;
        p.v[m] = p.v[m] + t;
      }
    }
  }
  if (MIDRED) {
#pragma unroll
    for (int m = 0; m < 16; ++m) p.v[m] = reduce_f(p.v[m]);
  }
  stride_to_contig_f(p, buf, L);
  {
    const float z = TABFD.z[16 + L];
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const float u = modmul_lf(p.v[t + 8], z);
      p.v[t + 8] = p.v[t] - u;
      p.v[t] = p.v[t] + u;
    }
  }
  {
    const float z0 = TABFD.z[32 + 2 * L], z1 = TABFD.z[33 + 2 * L];
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      if (((t >> 2) & 1) == 0) {
        const float u = modmul_lf(p.v[t + 4], t < 8 ? z0 : z1);
        p.v[t + 4] = p.v[t] - u;
        p.v[t] = p.v[t] + u;
      }
    }
  }
  {
    float z[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) z[s] = TABFD.z[64 + 4 * L + s];
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      if (((t >> 1) & 1) == 0) {
        const float u = modmul_lf(p.v[t + 2], z[t >> 2]);
        p.v[t + 2] = p.v[t] - u;
        p.v[t] = p.v[t] + u;
      }
    }
  }
}

// FIPS 203 Alg. 10 in fp32 (including the 128^-1 scaling).  In: contiguous, |f| <= 1665.
// Out: stride layout, |f| <= 1665.  Gentleman-Sande sums double per layer; the sums of
// every second layer are reduced, so |y - x| <= 6660 at every twiddle product.  The last
// layer folds the scaling in: x + y times 128^-1 = -26 and y - x times
// zeta_1 128^-1, instead of a separate product for all 16 outputs.
__device__ __forceinline__ void ntt_inv_f(PF16& p, float* buf, int L) {
  {
    float z[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) z[s] = TABFD.z[127 - 4 * L - s];
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      if (((t >> 1) & 1) == 0) {
        const float x = p.v[t], y = p.v[t + 2];
        p.v[t] = x + y;
        p.v[t + 2] = modmul_lf(y - x, z[t >> 2]);
      }
    }
  }
  {
    const float z0 = TABFD.z[63 - 2 * L], z1 = TABFD.z[62 - 2 * L];
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      if (((t >> 2) & 1) == 0) {
        const float x = p.v[t], y = p.v[t + 4];
        p.v[t] = reduce_f(x + y);
        p.v[t + 4] = modmul_lf(y - x, t < 8 ? z0 : z1);
      }
    }
  }
  {
    const float z = TABFD.z[31 - L];
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const float x = p.v[t], y = p.v[t + 8];
      p.v[t] = x + y;
      p.v[t + 8] = modmul_lf(y - x, z);
    }
  }
  contig_to_stride_f(p, buf, L);
#pragma unroll
  for (int lg = 3; lg >= (1 ? 1 : 0); --lg) {
    const int step = 8 >> lg;
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      if (((m / step) & 1) == 0) {
        const int zi = (2 << lg) - 1 - m / (2 * step);
        const float x = p.v[m], y = p.v[m + step];
        p.v[m] = ((lg & 1) == 1) ? reduce_f(x + y) : x + y;  // layers 4 and 6 reduce their sums
        p.v[m + step] = modmul_f(y - x, TABFC.z[zi], TABFC.zq[zi]);
      }
    }
  }
  // layer 7 (step 8, zeta_1) with the scaling: |x + y|, |y - x| <= 2 * 6660, far inside the
  // modmul_f bound for the small factors
#pragma unroll
  for (int m = 0; m < 8; ++m) {
    const float x = p.v[m], y = p.v[m + 8];
    p.v[m] = modmul_f(x + y, INV128F, (float)(INV128F / 3329.0));
    p.v[m + 8] = modmul_f(y - x, Z1INV128F, (float)(Z1INV128F / 3329.0));
  }
}

// ---- base-case multiplication (FIPS 203 Alg. 11/12) on packed int16 pairs
// A coefficient pair (a0, a1) lives in one dword (lo, hi) -- exactly the
// producer's sampled layout.  For the other operand b we precompute
//   B0 = (b0, b1*gamma)   and   B1 = (b1, b0)
// so that  c0 = a0 b0 + a1 b1 gamma = dot2(A, B0),  c1 = a0 b1 + a1 b0 = dot2(A, B1):
// two v_dot2c_i32_i16 per pair, accumulated unreduced over the k terms.
typedef short v2s __attribute__((ext_vector_type(2)));

struct PK8 {  // 16 coefficients as 8 packed int16 pairs (contiguous layout)
  uint32_t w[8];
};
struct BOp {  // basemul right operand
  uint32_t b0[8], b1[8];
};

__device__ __forceinline__ uint32_t pack16(int lo, int hi) {
  return __builtin_amdgcn_perm((uint32_t)hi, (uint32_t)lo, 0x05040100u);
}

// From an fp32 NTT output (|b| <= 11658, fits int16): B0 = (b0, b1 gamma mod q),
// B1 = (b1, b0).  b1 is reduced before the gamma product to keep it below 2^24.
__device__ __forceinline__ BOp make_bop_f(const PF16& b, int L) {
  BOp r;
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const uint32_t e0 = f2bits(b.v[2 * u]), e1 = f2bits(b.v[2 * u + 1]);
    const uint32_t g = f2bits(modmul_lf(reduce_f(b.v[2 * u + 1]), TABFD.g[8 * L + u]));
    r.b0[u] = pack16((int)e0, (int)g);
    r.b1[u] = pack16((int)e1, (int)e0);
  }
  return r;
}

__device__ __forceinline__ int dot2(uint32_t a, uint32_t b, int c) {
  return __builtin_amdgcn_sdot2(__builtin_bit_cast(v2s, a), __builtin_bit_cast(v2s, b), c, false);
}

// acc += a o b  (a in [0, q), b centered; |acc| stays < 2^27 for k <= 4)
__device__ __forceinline__ void basemul_acc(int acc[16], const PK8& a, const BOp& b) {
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    acc[2 * u] = dot2(a.w[u], b.b0[u], acc[2 * u]);
    acc[2 * u + 1] = dot2(a.w[u], b.b1[u], acc[2 * u + 1]);
  }
}

// Split CBD: the PRF words are loaded first (so a caller can prefetch them one
// stage ahead) and expanded straight to fp32.
struct CbdRaw {
  uint32_t d[3];
};
template <int ETA, int TW = 64>
__device__ __forceinline__ CbdRaw cbd_load(const uint64_t* __restrict__ prf, size_t inst, int L) {
  CbdRaw r;
  if constexpr (ETA == 2) {
    const uint64_t w = prf[tidx<TW>(inst, L, PRF_W)];
    r.d[0] = (uint32_t)w, r.d[1] = (uint32_t)(w >> 32), r.d[2] = 0;
  } else {
    const int wi = (3 * L) >> 1;
    const uint64_t a = prf[tidx<TW>(inst, wi, PRF_W)], b = prf[tidx<TW>(inst, wi + 1, PRF_W)];
    const bool odd = L & 1;
    r.d[0] = odd ? (uint32_t)(a >> 32) : (uint32_t)a;
    r.d[1] = odd ? (uint32_t)b : (uint32_t)(a >> 32);
    r.d[2] = odd ? (uint32_t)(b >> 32) : (uint32_t)b;
  }
  return r;
}
// eta = 2 in SWAR form: per nibble (a0 a1 b0 b1), x holds a0+a1 and b0+b1 in two bit
// pairs, y = (a0+a1) + 4 - (b0+b1) per nibble (no borrow), coefficient = nibble - 4,
// built as an fp32 directly (0x4B400000 | nibble is 2^23 * 1.5 + nibble).
template <int ETA>
__device__ __forceinline__ void cbd_f(PF16& p, const CbdRaw& r) {
  if constexpr (ETA == 2) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const uint32_t d = r.d[h];
      const uint32_t x = (d & 0x55555555u) + ((d >> 1) & 0x55555555u);
      const uint32_t y = (x & 0x33333333u) + 0x44444444u - ((x >> 2) & 0x33333333u);
#pragma unroll
      for (int t = 0; t < 8; ++t)
        p.v[8 * h + t] = __uint_as_float(((y >> (4 * t)) & 0xFu) | 0x4B400000u) - (MAGIC + 4.0f);
    }
  } else {
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      const int bit = 6 * t, i = bit >> 5, sh = bit & 31;
      uint32_t f = r.d[i] >> sh;
      if (sh + 6 > 32) f |= r.d[i + 1] << (32 - sh);
      f &= 0x3F;
      p.v[t] = i2f((int)__popc(f & 7u) - (int)__popc(f & 0x38u));
    }
  }
}

// A group's 16*D*2 bytes at src (4-byte aligned) as this lane's share of dwords (L, L + 16, ...),
// loaded ahead of load_bits_r; DL <= D reads a shorter (DL-bit) encoding into the same shape.
template <int D>
struct RawW {
  uint32_t w[(8 * D + 15) / 16];
};
template <int D, int DL = D>
__device__ __forceinline__ RawW<D> raw_load(const uint8_t* __restrict__ src, int L) {
  RawW<D> r;
  const uint32_t* s32 = (const uint32_t*)src;
#pragma unroll
  for (int i = 0; i < (8 * D + 15) / 16; ++i) {
    const int idx = L + 16 * i;
    r.w[i] = idx < 8 * DL ? s32[idx] : 0u;
  }
  return r;
}
// Group-cooperative stage of 16*D*2 bytes (already loaded, raw_load) into the raw stage, then lane
// L unpacks its 16 D-bit fields (bits 16*D*L ...).
template <int D, int DX>
__device__ __forceinline__ void load_bits_r(P16& p, const RawW<DX>& r, GroupLds& g, int L) {
  constexpr int NDW = 8 * D;  // dwords for 256 D-bit values
  uint32_t* st = (uint32_t*)g.raw;
#pragma unroll
  for (int i = 0; i < (NDW + 15) / 16; ++i) {
    const int idx = L + 16 * i;
    if (idx < NDW) st[idx] = r.w[i];
  }
  gsync();
  // this lane's 2D bytes start at byte 2*D*L
  const int b0 = 2 * D * L;
  uint32_t w[8];
  const uint16_t* st16 = (const uint16_t*)g.raw;
#pragma unroll
  for (int j = 0; j < D; ++j) {
    // assemble dwords from halfwords (2D bytes = D halfwords)
    const uint32_t h = st16[(b0 >> 1) + j];
    if (j & 1)
      w[j >> 1] |= h << 16;
    else
      w[j >> 1] = h;
  }
#pragma unroll
  for (int t = 0; t < 16; ++t) {
    const int bit = D * t;
    const int i = bit >> 5, sh = bit & 31;
    uint32_t v = w[i] >> sh;
    if (sh + D > 32) v |= w[i + 1] << (32 - sh);
    p.v[t] = (int)(v & ((1u << D) - 1));
  }
  gsync();
}
template <int D>
__device__ __forceinline__ void load_bits(P16& p, const uint8_t* __restrict__ src, GroupLds& g, int L) {
  load_bits_r<D>(p, raw_load<D>(src, L), g, L);
}

// Pack lane L's 16 D-bit fields into the raw stage at byte 2*D*L (whole group: 32*D bytes).
template <int D>
__device__ __forceinline__ void pack_bits(const P16& p, GroupLds& g, int L) {
  uint32_t w[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) w[i] = 0;
#pragma unroll
  for (int t = 0; t < 16; ++t) {
    const int bit = D * t;
    const int i = bit >> 5, sh = bit & 31;
    const uint32_t v = (uint32_t)p.v[t];
    w[i] |= v << sh;
    if (sh + D > 32) w[i + 1] |= v >> (32 - sh);
  }
  uint16_t* st16 = (uint16_t*)g.raw;
  const int h0 = D * L;
#pragma unroll
  for (int j = 0; j < D; ++j) st16[h0 + j] = (uint16_t)(w[j >> 1] >> (16 * (j & 1)));
  gsync();
}

// Store the packed stage (8*D dwords) to dst; or, when cmp != nullptr, OR the
// XOR with cmp into diff instead (Decaps re-encryption compare).
template <int D>
__device__ __forceinline__ void flush_bits(GroupLds& g, uint8_t* dst, const uint8_t* cmp, uint32_t& diff,
                                           bool active, int L) {
  constexpr int NDW = 8 * D;
  const uint32_t* st = (const uint32_t*)g.raw;
#pragma unroll
  for (int i = 0; i < (NDW + 15) / 16; ++i) {
    const int idx = L + 16 * i;
    if (idx < NDW) {
      const uint32_t v = st[idx];
      if (cmp)
        diff |= v ^ ((const uint32_t*)cmp)[idx];
      else if (active)
        ((uint32_t*)dst)[idx] = v;
    }
  }
  gsync();
}

// Decaps compare with the received ciphertext words loaded ahead of time (cmp_load):
// the global-load latency hides behind the row's NTT work instead of stalling the flush.
template <int D>
struct CmpWords {
  uint32_t w[(8 * D + 15) / 16];
};
template <int D>
__device__ __forceinline__ CmpWords<D> cmp_load(const uint8_t* cmp, int L) {
  CmpWords<D> r;
#pragma unroll
  for (int i = 0; i < (8 * D + 15) / 16; ++i) {
    const int idx = L + 16 * i;
    r.w[i] = idx < 8 * D ? ((const uint32_t*)cmp)[idx] : 0u;
  }
  return r;
}
template <int D>
__device__ __forceinline__ void flush_cmp(GroupLds& g, const CmpWords<D>& c, uint32_t& diff, int L) {
  const uint32_t* st = (const uint32_t*)g.raw;
#pragma unroll
  for (int i = 0; i < (8 * D + 15) / 16; ++i) {
    const int idx = L + 16 * i;
    if (idx < 8 * D) diff |= st[idx] ^ c.w[i];
  }
  gsync();
}

// SampleNTT consumer: lane L loads coefficients 16L..16L+15 (chunks 2L, 2L+1)
// of the producer's compacted output -- contiguous layout, no parsing.
// The batched producer's 12-bit chunks, spread back to int16 pairs: a pair is 24
// consecutive bits x, (x & 0xFFF) | (x << 4 & 0x0FFF0000) -- about 3 VALU per pair.
__device__ __forceinline__ PK8 unpack12(const U3& u, const U3& v) {
  const uint32_t w[6] = {u.x, u.y, u.z, v.x, v.y, v.z};
  PK8 r;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const uint32_t a = w[3 * h], b = w[3 * h + 1], c = w[3 * h + 2];
    const uint32_t x[4] = {a, __builtin_amdgcn_alignbit(b, a, 24), __builtin_amdgcn_alignbit(c, b, 16), c >> 8};
#pragma unroll
    for (int k = 0; k < 4; ++k) r.w[4 * h + k] = (x[k] & 0xFFFu) | ((x[k] << 4) & 0x0FFF0000u);
  }
  return r;
}
template <int TW = 64, bool P12 = false>
__device__ __forceinline__ PK8 load_sampled(const void* __restrict__ xs_, size_t inst, int L) {
  if constexpr (P12) {
    const XUnit* base = xent<TW>((XUnit*)xs_, inst);
    const U6 u = base[L * TW];
    return unpack12(u.h[0], u.h[1]);
  } else {
    const uint4* base = (const uint4*)xs_ + (inst / TW) * 32 * TW + (inst % TW);
    const uint4 u = base[(2 * L) * TW], v = base[(2 * L + 1) * TW];
    return PK8{{u.x, u.y, u.z, u.w, v.x, v.y, v.z, v.w}};
  }
}
// the batched cores' view of the SampleNTT output
#define LOAD_XOF(TW_, inst) load_sampled<(TW_) == 64 ? XTW : (TW_), (TW_) == 64>(xof, (inst), L)

// ByteDecode_12 (reduced mod q) of a 384-byte NTT-domain polynomial into packed
// pairs; `bad` collects the FIPS 203 section 7.2 modulus-check failure.
__device__ __forceinline__ PK8 decode12_w(uint64_t a, uint64_t b, uint64_t c, bool& bad);
__device__ __forceinline__ PK8 decode12(const uint8_t* __restrict__ src, bool& bad, int L) {
  const uint64_t* s = (const uint64_t*)(src + 24 * L);
  return decode12_w(s[0], s[1], s[2], bad);
}
// ByteDecode_12 of this lane's 24 bytes already in registers (a, b, c little-endian)
__device__ __forceinline__ PK8 decode12_w(uint64_t a, uint64_t b, uint64_t c, bool& bad) {
  int v[16];
  split12((uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, v);
  split12((uint32_t)(b >> 32), (uint32_t)c, (uint32_t)(c >> 32), v + 8);
  PK8 r;
  // unsigned min(v, v - q) is v mod q for v < 2q (v - q wraps when v < q); the largest
  // coefficient decides the modulus check (two full-rate ops and one max, no lane masks)
  uint32_t mx = 0;
#pragma unroll
  for (int t = 0; t < 16; ++t) {
    const uint32_t u = (uint32_t)v[t];
    mx = u > mx ? u : mx;
    v[t] = (int)__builtin_elementwise_min(u, u - (uint32_t)Q);
  }
  bad |= mx >= (uint32_t)Q;
#pragma unroll
  for (int u = 0; u < 8; ++u) r.w[u] = pack16(v[2 * u], v[2 * u + 1]);
  return r;
}

__device__ __forceinline__ void encode12(const P16& p, uint8_t* dst, int L) {
  uint32_t w[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) w[i] = 0;
#pragma unroll
  for (int t = 0; t < 16; ++t) {
    const int bit = 12 * t, i = bit >> 5, sh = bit & 31;
    const uint32_t v = (uint32_t)p.v[t];
    w[i] |= v << sh;
    if (sh + 12 > 32) w[i + 1] |= v >> (32 - sh);
  }
  uint64_t* d = (uint64_t*)(dst + 24 * L);
  d[0] = ((uint64_t)w[1] << 32) | w[0];
  d[1] = ((uint64_t)w[3] << 32) | w[2];
  d[2] = ((uint64_t)w[5] << 32) | w[4];
}

__device__ __forceinline__ uint32_t group_or(uint32_t x) {
#pragma unroll
  for (int d = 1; d < 16; d <<= 1) x |= __shfl_xor(x, d, 16);
  return x;
}

// Scratch carve-up for a chunk of C handshakes
struct ScratchView {
  uint64_t *xof, *prf, *seeds, *mprime, *kprime, *kbar;
  uint32_t *fix, *nfix;  // SampleNTT fix-up list (entries needing > 3 blocks, capacity K^2 C), its counter
  uint64_t* rho;         // every handshake's rho, 32 B apart (k_rho_copy)
};
__host__ __device__ inline size_t scratch_words(int K, size_t C) {
  return (size_t)K * K * C * XOF_W + (size_t)(2 * K + 1) * C * PRF_W + 16 * C + ((size_t)K * K * C + 16) / 2 + 4 +
         4 * C;
}
inline ScratchView carve(void* base, int K, size_t C) {
  ScratchView v;
  uint64_t* p = (uint64_t*)base;
  v.xof = p;
  p += (size_t)K * K * C * XOF_W;
  v.prf = p;
  p += (size_t)(2 * K + 1) * C * PRF_W;
  v.seeds = p;
  p += 4 * C;
  v.mprime = p;
  p += 4 * C;
  v.kprime = p;
  p += 4 * C;
  v.kbar = p;
  p += 4 * C;
  v.nfix = (uint32_t*)p;
  v.fix = v.nfix + 16;
  p += ((size_t)K * K * C + 16) / 2 + 4;
  v.rho = p;
  return v;
}

// k_xof reads rho from a compact copy (32 B per handshake) instead of the
// keys themselves.  Its K^2 lanes per handshake sit in K^2 different waves, and each wave's 64
// rho reads at the key stride (1184 B for ML-KEM-768) touch 64 cache lines: rocprofv3 counts
// 1.2 GB of reads per 2^20-handshake k_xof launch for 33 MB of rho
// (profiles/r3/rocprof_mlkem768_b20_r3b.json).  The copy is one 32-B read per handshake.
// It also zeroes the SampleNTT fix-up counter the next kernel counts into (no memset launch).
__global__ __launch_bounds__(256) void k_rho_copy(const uint8_t* __restrict__ base, size_t stride, size_t n,
                                                  uint64_t* __restrict__ out, uint32_t* __restrict__ nfix) {
  const size_t t = (size_t)blockIdx.x * 256 + threadIdx.x;  // one thread per word
  if (t == 0) *nfix = 0;
  if (t >= 4 * n) return;
  out[t] = ((const uint64_t*)(base + (t >> 2) * stride))[t & 3];
}

// ------------------------------------------------------------ single-shot phase trace (tools only)
// -DQRK_SS_TRACE=1 (a tools/build_variant.sh build): the single-shot kernels stamp the 100 MHz
// wall clock at phase boundaries into g_ss_trace; qrk_dbg_ss_trace() copies it out.
#ifndef QRK_SS_TRACE
#define QRK_SS_TRACE 0
#endif
#if QRK_SS_TRACE
__device__ unsigned long long g_ss_trace[32];
#define SS_MARK(cond, i)                                      \
  do {                                                        \
    if (cond) g_ss_trace[i] = wall_clock64();                 \
  } while (0)
#define SS_CLK(cond, i)                                       \
  do {                                                        \
    if (cond) g_ss_trace[i] = clock64();                      \
  } while (0)
#else
#define SS_CLK(cond, i) \
  do {                  \
  } while (0)
#define SS_MARK(cond, i) \
  do {                   \
  } while (0)
#endif

// ------------------------------------------------------------ KeyGen core
// s_hat = NTT(CBD(PRF(sigma, j))), e_hat = NTT(CBD(PRF(sigma, k+i))),
// t_hat_i = sum_j A[i][j] o s_hat_j + e_hat_i   (A[i][j] = SampleNTT(rho || j || i))
template <int K>
__device__ __forceinline__ void keygen_core_hs(size_t n, size_t C, const uint64_t* __restrict__ xof,
                                                     const uint64_t* __restrict__ prf, uint8_t* __restrict__ pk,
                                                     uint8_t* __restrict__ sk, size_t hs_raw, int L, GroupLds& g) {
  const bool active = hs_raw < n;
  const size_t hs = active ? hs_raw : n - 1;  // index in the chunk
  uint8_t* ek = pk + hs * P<K>::PK;
  uint8_t* dk = sk + hs * P<K>::SK;
  BOp sb[K];
  {
    CbdRaw sr[K];  // every s_j's CBD words issued before the first NTT
#pragma unroll
    for (int j = 0; j < K; ++j) sr[j] = cbd_load<P<K>::ETA1, 64>(prf, (size_t)j * C + hs, L);
#pragma unroll
    for (int j = 0; j < K; ++j) {
      PF16 f;
      cbd_f<P<K>::ETA1>(f, sr[j]);
      contig_to_stride_f(f, (float*)g.poly, L);
      ntt_fwd_f<false>(f, (float*)g.poly, L);
      sb[j] = make_bop_f(f, L);
      P16 t;
#pragma unroll
      for (int x = 0; x < 16; ++x) t.v[x] = canon_f(f.v[x]);
      if (active) encode12(t, dk + 384 * j, L);
    }
  }
  // row i's matrix entries and e_i's CBD words are loaded one row ahead
  PK8 an[K];
#pragma unroll
  for (int j = 0; j < K; ++j) an[j] = LOAD_XOF(64, (size_t)(j * K) * C + hs);
  CbdRaw er = cbd_load<P<K>::ETA1, 64>(prf, (size_t)K * C + hs, L);
#pragma unroll 1
  for (int i = 0; i < K; ++i) {
    int acc[16];
#pragma unroll
    for (int t = 0; t < 16; ++t) acc[t] = 0;
#pragma unroll
    for (int j = 0; j < K; ++j) basemul_acc(acc, an[j], sb[j]);
    const CbdRaw ecur = er;
    if (i + 1 < K) {
#pragma unroll
      for (int j = 0; j < K; ++j) an[j] = LOAD_XOF(64, (size_t)(j * K + i + 1) * C + hs);
      er = cbd_load<P<K>::ETA1, 64>(prf, (size_t)(K + i + 1) * C + hs, L);
    }
    PF16 ef;
    cbd_f<P<K>::ETA1>(ef, ecur);
    contig_to_stride_f(ef, (float*)g.poly, L);
    ntt_fwd_f<false>(ef, (float*)g.poly, L);
    P16 t;
#pragma unroll
    for (int x = 0; x < 16; ++x) t.v[x] = canon_f(acc_to_f(acc[x]) + ef.v[x]);
    if (active) {
      encode12(t, ek + 384 * i, L);
      encode12(t, dk + 384 * K + 384 * i, L);
    }
  }
}
template <int K>
__global__ __launch_bounds__(256) void k_keygen_core(size_t n, size_t C, const uint64_t* __restrict__ xof,
                                                     const uint64_t* __restrict__ prf, uint8_t* __restrict__ pk,
                                                     uint8_t* __restrict__ sk) {
  __shared__ GroupLds lds[GROUPS];
  const int gi = threadIdx.x >> 4;
  keygen_core_hs<K>(n, C, xof, prf, pk, sk, (size_t)blockIdx.x * GROUPS + gi, threadIdx.x & 15, lds[gi]);
}

// ------------------------------------------------------------ K-PKE.Encrypt core
// MODE 0 (encaps): write c.  MODE 1 (decaps): compare c' with the input c and
// select K' or Kbar in constant time (FIPS 203 Alg. 18 lines 9-11).
template <int K, int MODE>
__device__ __forceinline__ void encrypt_core_hs(size_t n, size_t C, const uint64_t* __restrict__ xof,
                                                      const uint64_t* __restrict__ prf,
                                                      const uint8_t* __restrict__ ek_base, size_t ek_stride,
                                                      const uint8_t* __restrict__ m_base, size_t m_stride,
                                                      uint8_t* __restrict__ ct, int32_t* __restrict__ status,
                                                      const uint64_t* __restrict__ kprime,
                                                      const uint64_t* __restrict__ kbar, uint8_t* __restrict__ ss, size_t hs_raw, int L, GroupLds& g) {
  constexpr int DU = P<K>::DU, DV = P<K>::DV;
  const bool active = hs_raw < n;
  const size_t hs = active ? hs_raw : n - 1;  // index in the chunk
  const uint8_t* ek = ek_base + hs * ek_stride;
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
      contig_to_stride_f(f, (float*)g.poly, L);
      ntt_fwd_f<false>(f, (float*)g.poly, L);
      yb[j] = make_bop_f(f, L);
    }
  }
  // u_i = NTT^-1(sum_j A[j][i] o y_j) + e1_i ;  A[j][i] = SampleNTT(rho || i || j).
  // Row i+1's matrix entries and the next CBD words are loaded one row ahead (latency hidden
  // inside the wave; loading each entry as the basemul needs it, at 4 waves / SIMD, was slower).
  // Issuing the first row's entries before the K NTT(y_j) instead was 3 % slower
  // (profiles/r3/ab_core_arith_c.jsonl).
  PK8 an[K];
#pragma unroll
  for (int j = 0; j < K; ++j) an[j] = LOAD_XOF(64, (size_t)j * C + hs);
  CbdRaw er = cbd_load<P<K>::ETA2, 64>(prf, (size_t)K * C + hs, L);
  // one u-row; LAST: the final row (peeled, so its prefetch is t_hat's words: the core waited on
  // memory 25-29 % of its wave time before, profiles/r2/sq_mlkem768_b20_r2b.txt)
  auto row = [&](int i, auto last_t) {
    constexpr bool LAST = decltype(last_t)::value;
    int acc[16];
#pragma unroll
    for (int t = 0; t < 16; ++t) acc[t] = 0;
#pragma unroll
    for (int j = 0; j < K; ++j) basemul_acc(acc, an[j], yb[j]);
    const CbdRaw ecur = er;
    if (!LAST) {
      if (i + 1 < K) {
#pragma unroll
        for (int j = 0; j < K; ++j) an[j] = LOAD_XOF(64, (size_t)((i + 1) * K + j) * C + hs);
      }
    } else {
      // last row: the matrix registers are free, so t_hat's 24 bytes per lane and row (for v
      // below) are loaded into them here, one row's NTT^-1 ahead of their use
#pragma unroll
      for (int j = 0; j < K; ++j) {
        const uint2* e = (const uint2*)(ek + 384 * j + 24 * L);
        const uint2 a = e[0], b = e[1], c = e[2];
        an[j].w[0] = a.x, an[j].w[1] = a.y, an[j].w[2] = b.x, an[j].w[3] = b.y, an[j].w[4] = c.x, an[j].w[5] = c.y;
      }
    }
    er = cbd_load<P<K>::ETA2, 64>(prf, (size_t)(K + i + 1) * C + hs, L);  // e1_{i+1}, or e2 after the last row
    PF16 uf;
#pragma unroll
    for (int t = 0; t < 16; ++t) uf.v[t] = acc_to_f(acc[t]);
    ntt_inv_f(uf, (float*)g.poly, L);
    CmpWords<DU> cw;
    if (MODE) cw = cmp_load<DU>(c + 32 * DU * i, L);
    stride_to_contig_f(uf, (float*)g.poly, L);
    PF16 ef;
    cbd_f<P<K>::ETA2>(ef, ecur);
    P16 u;
#pragma unroll
    for (int t = 0; t < 16; ++t) u.v[t] = compress_f<DU>(uf.v[t] + ef.v[t]);
    pack_bits<DU>(u, g, L);
    if (MODE)
      flush_cmp<DU>(g, cw, diff, L);
    else
      flush_bits<DU>(g, c + 32 * DU * i, nullptr, diff, active, L);
  };
#pragma unroll 1
  for (int i = 0; i < K - 1; ++i) row(i, std::false_type{});
  row(K - 1, std::true_type{});
  // v = NTT^-1(t_hat^T o y_hat) + e2 + Decompress_1(m)
  {
    int acc[16];
#pragma unroll
    for (int t = 0; t < 16; ++t) acc[t] = 0;
    bool bad = false;
#pragma unroll
    for (int j = 0; j < K; ++j) {
      uint32_t w[6];
#pragma unroll
      for (int t = 0; t < 6; ++t) w[t] = an[j].w[t];
      const uint64_t a = ((uint64_t)w[1] << 32) | w[0], b = ((uint64_t)w[3] << 32) | w[2],
                     c = ((uint64_t)w[5] << 32) | w[4];
      basemul_acc(acc, decode12_w(a, b, c, bad), yb[j]);
    }
    PF16 vf;
#pragma unroll
    for (int t = 0; t < 16; ++t) vf.v[t] = acc_to_f(acc[t]);
    ntt_inv_f(vf, (float*)g.poly, L);
    stride_to_contig_f(vf, (float*)g.poly, L);
    PF16 ef;
    cbd_f<P<K>::ETA2>(ef, er);  // e2
    const uint8_t* m = m_base + hs * m_stride;
    const uint32_t mb = (uint32_t)m[2 * L] | ((uint32_t)m[2 * L + 1] << 8);
    P16 v;
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      const float mu = ((mb >> t) & 1) ? (float)((Q + 1) / 2) : 0.0f;
      v.v[t] = compress_f<DV>(vf.v[t] + ef.v[t] + mu);
    }
    pack_bits<DV>(v, g, L);
    flush_bits<DV>(g, c + 32 * DU * K, MODE ? c + 32 * DU * K : nullptr, diff, active, L);
    if (MODE == 0 && status) {
      const uint32_t anybad = group_or(bad ? 1u : 0u);
      if (active && L == 0) status[hs] = anybad ? -1 : 0;
    }
  }
  if (MODE == 1) {
    // constant-time select: ss = (c == c') ? K' : Kbar
    const uint32_t d = group_or(diff);
    const uint32_t mask = (uint32_t)(((uint64_t)d - 1u) >> 32);  // all-ones iff d == 0, no branch
    if (L < 8) {
      const uint32_t kp = ((const uint32_t*)(kprime + hs * 4))[L];
      const uint32_t kb = ((const uint32_t*)(kbar + hs * 4))[L];
      if (active) ((uint32_t*)(ss + hs * 32))[L] = (kp & mask) | (kb & ~mask);
    }
  }
}
// ------------------------------------------------------------ K-PKE.Decrypt core
template <int K, int TW = 64>
__device__ __forceinline__ void decrypt_core_hs(size_t n, const uint8_t* __restrict__ ct,
                                                      const uint8_t* __restrict__ sk, uint64_t* __restrict__ mprime, size_t hs_raw, int L, GroupLds& g) {
  constexpr int DU = P<K>::DU, DV = P<K>::DV;
  const bool active = hs_raw < n;
  const size_t hs = active ? hs_raw : n - 1;
  const uint8_t* c = ct + (TW == 64 ? hs : 0) * P<K>::CT;  // the small path passes LDS copies
  const uint8_t* dk = sk + (TW == 64 ? hs : 0) * P<K>::SK;
  int acc[16];
#pragma unroll
  for (int t = 0; t < 16; ++t) acc[t] = 0;
  bool bad = false;
#pragma unroll 1
  for (int j = 0; j < K; ++j) {
    // s_hat_j's 24 bytes per lane, issued before the NTT that precedes their use
    const uint2* e = (const uint2*)(dk + 384 * j + 24 * L);
    const uint2 da = e[0], db = e[1], dc = e[2];
    P16 u;
    load_bits<DU>(u, c + 32 * DU * j, g, L);
    PF16 uf;
#pragma unroll
    for (int t = 0; t < 16; ++t) uf.v[t] = i2f(decompress<DU>(u.v[t]));
    contig_to_stride_f(uf, (float*)g.poly, L);
    ntt_fwd_f<true>(uf, (float*)g.poly, L);
    basemul_acc(acc,
                decode12_w(((uint64_t)da.y << 32) | da.x, ((uint64_t)db.y << 32) | db.x, ((uint64_t)dc.y << 32) | dc.x, bad),
                make_bop_f(uf, L));
  }
  PF16 w;
#pragma unroll
  for (int t = 0; t < 16; ++t) w.v[t] = acc_to_f(acc[t]);
  ntt_inv_f(w, (float*)g.poly, L);
  stride_to_contig_f(w, (float*)g.poly, L);
  P16 v;
  load_bits<DV>(v, c + 32 * DU * K, g, L);
  uint32_t bits = 0;
#pragma unroll
  for (int t = 0; t < 16; ++t) {
    bits |= (uint32_t)compress_f<1>(i2f(decompress<DV>(v.v[t])) - w.v[t]) << t;
  }
  if (active) ((uint16_t*)(mprime + (TW == 64 ? hs : 0) * 4))[L] = (uint16_t)bits;
}

// ============================================================ small batches: one launch per operation
// The reference calls one KeyGen / Encaps / Decaps at a time (key_exchange.py:133, 156, 179):
// there the batched schedule's per-kernel launches dominate, and one handshake's sponge chain is
// the critical path.  For small n one 512-thread workgroup per handshake runs the whole operation
// in a single launch, every sponge wave-cooperative (keccak_coop.cuh, one state per wave):
//   encaps: wave 0 H(ek) then G(m || h);    waves 1-7 the K^2 SampleNTT entries
//   decaps: wave 0 Decrypt then G(m' || h); wave 1 J(z || c);  waves 2-7 SampleNTT
//   keygen: wave 0 G(d || k), then PRFs and SampleNTT over all waves, the core, H(ek)
// then the 2K+1 (2K) PRFs, one per wave, and the 16-lane polynomial core.  SampleNTT entries, PRF
// outputs and the decaps intermediates stay in LDS (the batched layouts at tile width 16, C = 1).
// One launch per operation wins up to 1024 handshakes (ML-KEM-768 encaps+decaps 249 against 346 us
// at 1024, 466 against 396 at 2048: profiles/r2/small_crossover.json)
#ifndef QRK_SMALL_MAX
#define QRK_SMALL_MAX 1024
#endif
constexpr int ONE_WAVES = 12;  // Encaps / Decaps: 3 waves per SIMD, the 16-lane cores fit in 170 VGPRs
constexpr int KG_WAVES = 16;
constexpr int MAX_ONE_WAVES = KG_WAVES > ONE_WAVES ? KG_WAVES : ONE_WAVES;

// ordering between lanes of one wave across phases: a workgroup-scope release / acquire around
// a wave barrier
__device__ __forceinline__ void wave_phase() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// SampleNTT entry e = x K + y (FIPS 203 Alg. 7) on one wave: SHAKE128(rho || x || y) squeezed
// block by block; each block's 56 byte triples are parsed by lanes 0-55 (two candidates each)
// and the accepted ones placed by ballot prefix counts, so the wave keeps FIPS order:
// place(j, value) for coefficient j.  pbuf: this wave's 44-dword LDS parse buffer.  after_block(cnt):
// called with the running count of accepted values once a block's values are placed.
struct NoHook {
  __device__ __forceinline__ void operator()(int) const {}
};
template <int K, typename Place, typename Hook = NoHook>
__device__ __forceinline__ void xof_coop_place(const uint64_t* __restrict__ rho, int e, uint32_t* __restrict__ pbuf,
                                               const Coop& c, Place place, Hook after_block = Hook()) {
  const int i = c.idx, lane = threadIdx.x & 63;
  CState s;
  if (i >= 0 && i < 4) cs_xor(s, rho[i]);
  if (i == 4) s.lo ^= (uint32_t)(e / K) | ((uint32_t)(e % K) << 8) | (DS_SHAKE << 16);
  if (i == RW_SHAKE128 - 1) s.hi ^= 0x80000000u;
  int cnt = 0;
#pragma unroll 1
  while (cnt < 256) {  // wave-uniform
    s = kf_coop(s, c);
    if (i >= 0 && i < RW_SHAKE128) {
      pbuf[2 * i] = s.lo;
      pbuf[2 * i + 1] = s.hi;
    }
    wave_phase();
    uint32_t d1 = Q, d2 = Q;
    if (lane < 56) {
      const int b = 3 * lane;
      const uint32_t v = __builtin_amdgcn_alignbit(pbuf[(b >> 2) + 1], pbuf[b >> 2], 8 * (b & 3));
      d1 = v & 0xFFF;
      d2 = (v >> 12) & 0xFFF;
    }
    const bool a1 = d1 < (uint32_t)Q, a2 = d2 < (uint32_t)Q;
    const uint64_t m1 = __ballot(a1), m2 = __ballot(a2);
    const int pre = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m1 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m1, 0)) +
                    (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m2 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m2, 0));
    const int p1 = cnt + pre, p2 = p1 + (a1 ? 1 : 0);
    if (a1 && p1 < 256) place(p1, d1);
    if (a2 && p2 < 256) place(p2, d2);
    cnt += __popcll(m1) + __popcll(m2);
    wave_phase();  // this block's parse reads are done before the next block's pbuf writes
    after_block(cnt);
  }
}
// ... into the single-shot layout: coefficient j of entry e at int16 index ((j / 8) 16 + e) 8 + j % 8
// of xs16 (the k_xof layout at tile width 16)
template <int K>
__device__ __forceinline__ void xof_coop(const uint64_t* __restrict__ rho, int e, uint16_t* __restrict__ xs16,
                                         uint32_t* __restrict__ pbuf, const Coop& c) {
  xof_coop_place<K>(rho, e, pbuf, c,
                    [&](int j, uint32_t d) { xs16[(((j >> 3) * 16 + e) << 3) + (j & 7)] = (uint16_t)d; });
}
// ... into the batched layout (the SampleNTT fix-up for small chunks, one wave per listed entry
// inst = xy C + hs): the 256 values in FIPS order in the wave's LDS buffer cb, then lanes 0-31
// pack one 8-coefficient chunk each into the entry's 12-bit tiles, as k_xof would have
template <int K>
__device__ __forceinline__ void xof_fix_coop(const uint8_t* __restrict__ rho_base, size_t rho_stride, size_t C,
                                             uint32_t inst, XUnit* __restrict__ out, uint16_t* __restrict__ cb,
                                             uint32_t* __restrict__ pbuf, const Coop& c) {
  const size_t hs = inst % C;
  xof_coop_place<K>((const uint64_t*)(rho_base + hs * rho_stride), (int)(inst / C), pbuf, c,
                    [&](int j, uint32_t d) { cb[j] = (uint16_t)d; });
  const int lane = threadIdx.x & 63;
  if (lane < 32) {
    uint32_t r[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = cb[8 * lane + j];
    chunk_store(xc<XTW>(xent<XTW>(out, inst), lane), r);
  }
  wave_phase();  // cb is read before the next entry's values are placed
}

// PRF instance N on one wave: SHAKE256(seed || N) -> 64 eta bytes; word w at ps[w 16 + N].
template <int ETA>
__device__ __forceinline__ void prf_coop(const uint64_t* __restrict__ seed, int N, uint64_t* __restrict__ ps,
                                         const Coop& c) {
  const int i = c.idx;
  CState s;
  if (i >= 0 && i < 4) cs_xor(s, seed[i]);
  if (i == 4) s.lo ^= (uint32_t)N | (DS_SHAKE << 8);
  if (i == RW_SHAKE256 - 1) s.hi ^= 0x80000000u;
  s = kf_coop(s, c);
  if (ETA == 2) {
    if (i >= 0 && i < 16) ps[i * 16 + N] = cs_word(s);
  } else {
    if (i >= 0 && i < 17) ps[i * 16 + N] = cs_word(s);
    s = kf_coop(s, c);
    if (i >= 0 && i < 7) ps[(17 + i) * 16 + N] = cs_word(s);
  }
}

struct OneLds {
  uint4 xs[32 * 16];             // SampleNTT entries (K^2 <= 16)
  uint64_t ps[PRF_W * 16];       // PRF outputs (2K + 1 <= 9)
  uint32_t bop[4][16][16];       // NTT(y_j) / NTT(s_j) as basemul operands: word w of lane L at [j][w][L]
  float ef[4][16][16];           // KeyGen: NTT(e_i), coefficient t of lane L at [i][t][L]
  uint32_t pbuf[MAX_ONE_WAVES][44];  // per-wave SampleNTT parse buffers
  uint64_t io[600];              // the handshake's inputs (Encaps ek | m, Decaps c | dk; KeyGen ek)
  uint64_t seed[4], mp[4], kp[4], kb[4];
  uint32_t diff[8];              // Decaps compare: per worker group
  int flag_seed, flag_kb, n_ready, n_xof, n_done;
  GroupLds g[8];                 // 16-lane groups: PRF instance N's NTT uses g[N]; rows g[0..K-1], v g[4], Decrypt g[5]
};

// Zero the workgroup's LDS copy of the key material before it exits (LDS is not cleared between
// workgroups); every thread of the workgroup calls it.  With a completion flag (single-shot host
// calls) the outputs are first made visible at system scope, then the flag is stored.
__device__ __forceinline__ void wipe_one(OneLds& sl, uint32_t* done, uint32_t ticket) {
  const int nthreads = (int)blockDim.x;
  if (done) __threadfence_system();
  __syncthreads();
  if (done && threadIdx.x == 0) __hip_atomic_store(done, ticket, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  uint4* w = (uint4*)&sl;
  for (int x = threadIdx.x; x < (int)(sizeof(OneLds) / 16); x += nthreads) w[x] = make_uint4(0, 0, 0, 0);
}

// Cross-wave flags (Decaps, where the J chain must not hold a workgroup barrier): a wave's LDS
// writes are released before it bumps a counter; readers spin with an acquiring load.
__device__ __forceinline__ void one_signal(int* p) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_add(p, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void one_wait(int* p, int target) {
  while (__hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < target) __builtin_amdgcn_s_sleep(1);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// Copy one handshake's inputs (host-mapped or device memory) into LDS in one parallel burst: the
// zero-copy single-shot calls then pay one PCIe round trip instead of one per dependent load.
__device__ __forceinline__ void stage_in(uint64_t* __restrict__ dst, const uint64_t* __restrict__ src, int words) {
  for (int w = threadIdx.x; w < words; w += (int)blockDim.x) dst[w] = src[w];
}

__device__ __forceinline__ void bop_store(OneLds& sl, int j, const BOp& b, int L) {
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    sl.bop[j][u][L] = b.b0[u];
    sl.bop[j][8 + u][L] = b.b1[u];
  }
}
__device__ __forceinline__ BOp bop_load(const OneLds& sl, int j, int L) {
  BOp b;
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    b.b0[u] = sl.bop[j][u][L];
    b.b1[u] = sl.bop[j][8 + u][L];
  }
  return b;
}

// PRF instance N (one wave), then for the secret vector (N < nvec) its NTT on lanes 0-15 into
// the shared basemul operands (KeyGen also writes NTT(s_j) to dk; KG: NTT(e_i) kept as fp32).
template <int K, bool KG>
__device__ __forceinline__ void prf_ntt_one(OneLds& sl, int N, uint8_t* __restrict__ dk, const Coop& c) {
  constexpr int ETA_V = P<K>::ETA1, ETA_E = KG ? P<K>::ETA1 : P<K>::ETA2;
  if (N < K)
    prf_coop<ETA_V>(sl.seed, N, sl.ps, c);
  else
    prf_coop<ETA_E>(sl.seed, N, sl.ps, c);
  const int L = threadIdx.x & 63;
  if (L < 16 && (N < K || KG)) {
    wave_phase();
    PF16 f;
    cbd_f<ETA_V>(f, cbd_load<ETA_V, 16>(sl.ps, (size_t)N, L));
    GroupLds& g = sl.g[N];  // N < 2K <= 8 (KeyGen), N < K otherwise
    contig_to_stride_f(f, (float*)g.poly, L);
    ntt_fwd_f<false>(f, (float*)g.poly, L);
    if (N < K) {
      bop_store(sl, N, make_bop_f(f, L), L);
      if (KG) {
        P16 t;
#pragma unroll
        for (int x = 0; x < 16; ++x) t.v[x] = canon_f(f.v[x]);
        encode12(t, dk + 384 * N, L);
      }
    } else {
#pragma unroll
      for (int x = 0; x < 16; ++x) sl.ef[N - K][x][L] = f.v[x];
    }
  }
}

// u_i = Compress_du(NTT^-1(sum_j A[i][j]^T o y_j) + e1_i) on one 16-lane group: written to c (MODE
// 0) or compared with it into diff (MODE 1).
template <int K, int MODE>
__device__ __forceinline__ void enc_row_one(const OneLds& sl, int i, uint8_t* __restrict__ c, uint32_t& diff,
                                            GroupLds& g, int L) {
  constexpr int DU = P<K>::DU;
  int acc[16];
#pragma unroll
  for (int t = 0; t < 16; ++t) acc[t] = 0;
#pragma unroll
  for (int j = 0; j < K; ++j) basemul_acc(acc, load_sampled<16>(sl.xs, (size_t)(i * K + j), L), bop_load(sl, j, L));
  const CbdRaw er = cbd_load<P<K>::ETA2, 16>(sl.ps, (size_t)(K + i), L);
  CmpWords<DU> cw;
  if (MODE) cw = cmp_load<DU>(c + 32 * DU * i, L);
  PF16 uf;
#pragma unroll
  for (int t = 0; t < 16; ++t) uf.v[t] = acc_to_f(acc[t]);
  ntt_inv_f(uf, (float*)g.poly, L);
  stride_to_contig_f(uf, (float*)g.poly, L);
  PF16 ef;
  cbd_f<P<K>::ETA2>(ef, er);
  P16 u;
#pragma unroll
  for (int t = 0; t < 16; ++t) u.v[t] = compress_f<DU>(uf.v[t] + ef.v[t]);
  pack_bits<DU>(u, g, L);
  if (MODE)
    flush_cmp<DU>(g, cw, diff, L);
  else
    flush_bits<DU>(g, c + 32 * DU * i, nullptr, diff, true, L);
}

// v = Compress_dv(NTT^-1(t_hat^T o y_hat) + e2 + Decompress_1(m)) on one 16-lane group; returns
// the FIPS 203 modulus-check failure of ek (Encaps status).
template <int K, int MODE>
__device__ __forceinline__ bool enc_v_one(const OneLds& sl, const uint8_t* __restrict__ ek, const uint8_t* __restrict__ m,
                                          uint8_t* __restrict__ c, uint32_t& diff, GroupLds& g, int L) {
  constexpr int DU = P<K>::DU, DV = P<K>::DV;
  int acc[16];
#pragma unroll
  for (int t = 0; t < 16; ++t) acc[t] = 0;
  bool bad = false;
#pragma unroll
  for (int j = 0; j < K; ++j) basemul_acc(acc, decode12(ek + 384 * j, bad, L), bop_load(sl, j, L));
  const CbdRaw er = cbd_load<P<K>::ETA2, 16>(sl.ps, (size_t)(2 * K), L);
  const uint32_t mb = (uint32_t)m[2 * L] | ((uint32_t)m[2 * L + 1] << 8);
  PF16 vf;
#pragma unroll
  for (int t = 0; t < 16; ++t) vf.v[t] = acc_to_f(acc[t]);
  ntt_inv_f(vf, (float*)g.poly, L);
  stride_to_contig_f(vf, (float*)g.poly, L);
  PF16 ef;
  cbd_f<P<K>::ETA2>(ef, er);
  P16 v;
#pragma unroll
  for (int t = 0; t < 16; ++t) {
    const float mu = ((mb >> t) & 1) ? (float)((Q + 1) / 2) : 0.0f;
    v.v[t] = compress_f<DV>(vf.v[t] + ef.v[t] + mu);
  }
  pack_bits<DV>(v, g, L);
  flush_bits<DV>(g, c + 32 * DU * K, MODE ? c + 32 * DU * K : nullptr, diff, true, L);
  return group_or(bad ? 1u : 0u) != 0;
}

// The public input of a single-shot host call (n == 1) passed by value, so the kernel does not read
// it over PCIe before H(ek); the secret inputs (the coins m here, dk for Decaps, d || z for KeyGen)
// stay in the pinned mirror, which the host wipes after the call: the HIP runtime's kernel-argument
// pool is never wiped.
template <int K>
struct EncIn {
  uint64_t pk[P<K>::PK / 8];
};
template <int K>
__global__ __launch_bounds__(64 * ONE_WAVES) void k_encaps_one(size_t n, const uint8_t* __restrict__ pk,
                                                                const uint8_t* __restrict__ coins, EncIn<K> in,
                                                                uint8_t* __restrict__ ct,
                                                                uint8_t* __restrict__ ss, int32_t* __restrict__ status,
                                                                uint32_t* done, uint32_t ticket) {
  __shared__ __attribute__((aligned(16))) OneLds sl;
  const size_t hs = blockIdx.x;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const Coop c = coop_init();
  const int i = c.idx;
  constexpr int EKW = P<K>::PK / 8;
  SS_MARK(threadIdx.x == 0, 0);
  SS_CLK(threadIdx.x == 0, 20);
  // ek from memory, or (pk == nullptr: n == 1 host calls) from the kernel argument; m from memory
  stage_in(sl.io, pk ? (const uint64_t*)(pk + hs * P<K>::PK) : in.pk, EKW);
  stage_in(sl.io + EKW, (const uint64_t*)(coins + hs * 32), 4);
  __syncthreads();
  const uint64_t* ek = sl.io;
  if (wave == 0) {  // (K, r) = G(m || H(ek)): the critical chain
    __builtin_amdgcn_s_setprio(3);
    CState s;
    coop_absorb<RW_SHA3_256, P<K>::PK / 8, DS_SHA3>(s, c, [&](int w) { return ek[w]; });
    const uint64_t h = cs_get(s, (i >= 4 && i < 8) ? i - 4 : 0);
    const uint64_t* m = sl.io + EKW;
    CState g;
    if (i >= 0 && i < 4) cs_xor(g, m[i]);
    if (i >= 4 && i < 8) cs_xor(g, h);
    if (i == 8) {
      g.lo ^= DS_SHA3;
      g.hi ^= 0x80000000u;
    }
    g = kf_coop(g, c);
    if (i >= 0 && i < 4) ((uint64_t*)(ss + hs * 32))[i] = cs_word(g);
    if (i >= 4 && i < 8) sl.seed[i - 4] = cs_word(g);
    __builtin_amdgcn_s_setprio(0);
    SS_MARK(threadIdx.x == 0, 1);
    SS_CLK(threadIdx.x == 0, 21);
  } else {
#pragma unroll 1
    for (int e = wave - 1; e < K * K; e += ONE_WAVES - 1)
      xof_coop<K>(ek + 48 * K, e, (uint16_t*)sl.xs, sl.pbuf[wave], c);
    SS_MARK(threadIdx.x == 64, 3);
  }
  __syncthreads();
  if (wave < 2 * K + 1) prf_ntt_one<K, false>(sl, wave, nullptr, c);  // PRF(r, N), NTT(y_N)
  SS_MARK(threadIdx.x == 0, 2);
  __syncthreads();
  SS_MARK(threadIdx.x == 0, 4);
  uint8_t* cc = ct + hs * P<K>::CT;
  uint32_t diff = 0;
  if (wave == 0 && (lane >> 4) < K) {
    enc_row_one<K, 0>(sl, lane >> 4, cc, diff, sl.g[lane >> 4], lane & 15);
  } else if (wave == 1 && lane < 16) {
    const bool bad = enc_v_one<K, 0>(sl, (const uint8_t*)ek, (const uint8_t*)(sl.io + EKW), cc, diff, sl.g[4], lane);
    if (status && lane == 0) status[hs] = bad ? -1 : 0;
  }
  SS_MARK(threadIdx.x == 0, 7);
  wipe_one(sl, done, ticket);
}

// the ciphertext of a single-shot host call passed by value (<= 1568 B); dk stays in the pinned mirror
template <int K>
struct DecIn {
  uint64_t ct[P<K>::CT / 8];
};
template <int K>
__global__ __launch_bounds__(64 * ONE_WAVES) void k_decaps_one(size_t n, const uint8_t* __restrict__ ct,
                                                                const uint8_t* __restrict__ sk, DecIn<K> in,
                                                                uint8_t* __restrict__ ss,
                                                                uint32_t* done, uint32_t ticket) {
  __shared__ __attribute__((aligned(16))) OneLds sl;
  const size_t hs = blockIdx.x;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const Coop c = coop_init();
  const int i = c.idx;
  constexpr int CTW = P<K>::CT / 8, SKW = P<K>::SK / 8;
  // c from memory, or (ct == nullptr: n == 1 host calls) from the kernel argument; dk from memory
  stage_in(sl.io, ct ? (const uint64_t*)(ct + hs * P<K>::CT) : in.ct, CTW);
  stage_in(sl.io + CTW, (const uint64_t*)(sk + hs * P<K>::SK), SKW);
  uint8_t* cc = (uint8_t*)sl.io;                   // the received ciphertext (LDS copy)
  const uint8_t* dk = (const uint8_t*)(sl.io + CTW);  // dk (LDS copy)
  constexpr int XW = ONE_WAVES - 3;  // SampleNTT waves 2 .. ONE_WAVES - 2; the last wave computes v
  if (threadIdx.x == 0) sl.flag_seed = sl.flag_kb = sl.n_ready = sl.n_xof = sl.n_done = 0;
  __syncthreads();
  SS_MARK(threadIdx.x == 0, 0);
  if (wave == 0) {  // m' = Decrypt(c), (K', r') = G(m' || h), PRF(r', 0), then the u rows and the select
    if (lane < 16) decrypt_core_hs<K, 16>(n, cc, dk, sl.mp, hs, lane, sl.g[5]);
    SS_MARK(lane == 0, 8);
    wave_phase();
    const uint64_t* h = (const uint64_t*)(dk + 768 * K + 32);
    CState g;
    if (i >= 0 && i < 4) cs_xor(g, sl.mp[i]);
    if (i >= 4 && i < 8) cs_xor(g, h[i - 4]);
    if (i == 8) {
      g.lo ^= DS_SHA3;
      g.hi ^= 0x80000000u;
    }
    g = kf_coop(g, c);
    if (i >= 0 && i < 4) sl.kp[i] = cs_word(g);
    if (i >= 4 && i < 8) sl.seed[i - 4] = cs_word(g);
    one_signal(&sl.flag_seed);
    SS_MARK(lane == 0, 9);
    prf_ntt_one<K, false>(sl, 0, nullptr, c);
    one_signal(&sl.n_ready);
    one_wait(&sl.n_ready, 2 * K + 1);
    one_wait(&sl.n_xof, K * K);
    SS_MARK(lane == 0, 4);
    uint32_t diff = 0;
    if ((lane >> 4) < K) enc_row_one<K, 1>(sl, lane >> 4, cc, diff, sl.g[lane >> 4], lane & 15);
    diff = group_or(diff);
    if ((lane & 15) == 0 && (lane >> 4) < K) sl.diff[lane >> 4] = diff;
    one_wait(&sl.n_done, 1);   // v
    one_wait(&sl.flag_kb, 1);  // Kbar
    SS_MARK(lane == 0, 6);
    if (lane < 8) {  // constant-time select: ss = (c == c') ? K' : Kbar
      uint32_t d = sl.diff[4];
#pragma unroll
      for (int r = 0; r < K; ++r) d |= sl.diff[r];
      const uint32_t mask = (uint32_t)(((uint64_t)d - 1u) >> 32);  // all-ones iff d == 0, no branch
      const uint32_t kp = ((const uint32_t*)sl.kp)[lane], kb = ((const uint32_t*)sl.kb)[lane];
      ((uint32_t*)(ss + hs * 32))[lane] = (kp & mask) | (kb & ~mask);
    }
    SS_MARK(lane == 0, 7);
  } else if (wave == 1) {  // Kbar = J(z || c) beside everything else
    __builtin_amdgcn_s_setprio(3);
    const uint64_t* z = (const uint64_t*)(dk + 768 * K + 64);
    const uint64_t* cw = (const uint64_t*)cc;
    CState s;
    coop_absorb<RW_SHAKE256, 4 + P<K>::CT / 8, DS_SHAKE>(s, c, [&](int w) { return w < 4 ? z[w] : cw[w - 4]; });
    if (i >= 0 && i < 4) sl.kb[i] = cs_word(s);
    __builtin_amdgcn_s_setprio(0);
    one_signal(&sl.flag_kb);
    SS_MARK(lane == 0, 11);
  } else if (wave < ONE_WAVES - 1) {  // SampleNTT, then PRF(r', N) for N = wave - 1
#pragma unroll 1
    for (int e = wave - 2; e < K * K; e += XW) {
      xof_coop<K>((const uint64_t*)(dk + 768 * K), e, (uint16_t*)sl.xs, sl.pbuf[wave], c);
      one_signal(&sl.n_xof);
    }
    SS_MARK(lane == 0 && wave == 2, 12);
    const int N = wave - 1;
    if (N < 2 * K + 1) {
      one_wait(&sl.flag_seed, 1);
      prf_ntt_one<K, false>(sl, N, nullptr, c);
      one_signal(&sl.n_ready);
    }
    SS_MARK(lane == 0 && wave == 2, 10);
  } else {  // v
    one_wait(&sl.n_ready, 2 * K + 1);
    if (lane < 16) {
      uint32_t diff = 0;
      enc_v_one<K, 1>(sl, dk + 384 * K, (const uint8_t*)sl.mp, cc, diff, sl.g[4], lane);
      diff = group_or(diff);
      if (lane == 0) sl.diff[4] = diff;
    }
    one_signal(&sl.n_done);
  }
  wipe_one(sl, done, ticket);
}

template <int K>
__global__ __launch_bounds__(64 * KG_WAVES) void k_keygen_one(size_t n, const uint8_t* __restrict__ coins,
                                                                uint8_t* __restrict__ pk, uint8_t* __restrict__ sk,
                                                                uint32_t* done, uint32_t ticket) {
  __shared__ __attribute__((aligned(16))) OneLds sl;
  const size_t hs = blockIdx.x;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const Coop c = coop_init();
  const int i = c.idx;
  uint8_t* ek = pk + hs * P<K>::PK;
  uint8_t* dk = sk + hs * P<K>::SK;
  SS_MARK(threadIdx.x == 0, 0);
  // z (dk's last 32 bytes) is loaded with d: the coins row may be host memory (single-shot calls),
  // and a load after H(ek) put one more PCIe round trip on the critical path
  const uint64_t zw = (wave == 0 && i >= 0 && i < 4) ? ((const uint64_t*)(coins + hs * 64 + 32))[i] : 0;
  if (wave == 0) {  // (rho, sigma) = G(d || k)
    const uint64_t* d = (const uint64_t*)(coins + hs * 64);
    CState g;
    if (i >= 0 && i < 4) cs_xor(g, d[i]);
    if (i == 4) g.lo ^= (uint32_t)K | (DS_SHA3 << 8);
    if (i == RW_SHA3_512 - 1) g.hi ^= 0x80000000u;
    g = kf_coop(g, c);
    if (i >= 0 && i < 4) {
      ((uint64_t*)(ek + 384 * K))[i] = cs_word(g);
      ((uint64_t*)(dk + 768 * K))[i] = cs_word(g);
      sl.kp[i] = cs_word(g);  // rho for SampleNTT
      sl.io[48 * K + i] = cs_word(g);  // ek's LDS copy (hashed below)
    }
    if (i >= 4 && i < 8) sl.seed[i - 4] = cs_word(g);
    SS_MARK(threadIdx.x == 0, 13);
  }
  __syncthreads();
#pragma unroll 1
  for (int it = wave; it < 2 * K + K * K; it += KG_WAVES) {  // the 2K PRFs (+ NTTs) first, then SampleNTT
    if (it < 2 * K)
      prf_ntt_one<K, true>(sl, it, dk, c);
    else
      xof_coop<K>(sl.kp, it - 2 * K, (uint16_t*)sl.xs, sl.pbuf[wave], c);
  }
  SS_MARK(threadIdx.x == 0, 14);
  __syncthreads();
  SS_MARK(threadIdx.x == 0, 4);
  if (wave == 0 && (lane >> 4) < K) {  // t_hat_i = sum_j A[i][j] o s_hat_j + e_hat_i, one group per row
    const int r = lane >> 4, L = lane & 15;
    int acc[16];
#pragma unroll
    for (int t = 0; t < 16; ++t) acc[t] = 0;
#pragma unroll
    for (int j = 0; j < K; ++j) basemul_acc(acc, load_sampled<16>(sl.xs, (size_t)(j * K + r), L), bop_load(sl, j, L));
    P16 t;
#pragma unroll
    for (int x = 0; x < 16; ++x) t.v[x] = canon_f(acc_to_f(acc[x]) + sl.ef[r][x][L]);
    encode12(t, ek + 384 * r, L);
    encode12(t, dk + 384 * K + 384 * r, L);
    encode12(t, (uint8_t*)sl.io + 384 * r, L);
  }
  SS_MARK(threadIdx.x == 0, 16);
  __syncthreads();
  if (wave == 0) {  // dk tail: H(ek) || z
    const uint64_t* ekw = sl.io;
    CState s;
    coop_absorb<RW_SHA3_256, P<K>::PK / 8, DS_SHA3>(s, c, [&](int w) { return ekw[w]; });
    uint64_t* tail = (uint64_t*)(dk + 768 * K + 32);
    if (i >= 0 && i < 4) {
      tail[i] = cs_word(s);
      tail[4 + i] = zw;
    }
    SS_MARK(threadIdx.x == 0, 17);
  }
  wipe_one(sl, done, ticket);
}

// ------------------------------------------------------------ single-shot KeyGen over K^2 + 2K workgroups
// k_keygen_one runs the 2K PRFs and K^2 SampleNTT entries of one handshake as 15 waves (ML-KEM-768)
// of one workgroup: their cooperative permutations share one CU and take ~2x their isolated time
// (phase trace: 18.8 us for 3 + 1 sequential permutations, profiles/r2/single_shot_trace_final.json).
// For n <= QRK_KG_MULTI_MAX the items get a one-wave workgroup each, on different CUs: every
// workgroup runs G(d || k) itself (one permutation, no cross-workgroup wait), then its item, writes
// the result to the context scratch (MkScr) and counts itself in with a device-scope fence and an
// atomic add; the workgroup that arrives last computes t_hat on four 16-lane groups, hashes ek
// (H(ek), 9 permutations at ML-KEM-768) and wipes the scratch and its counter.  No workgroup waits
// for another (the last one simply finds everything published), so nothing can spin.
#ifndef QRK_KG_MULTI_MAX
#define QRK_KG_MULTI_MAX 16
#endif
// 1 (default): host-pointer KeyGen calls of n <= QRK_KG_MULTI_MAX run k_keygen_pipe (H(ek) pipelined
// with SampleNTT, below; 37.5 against 41.6 us per kernel, profiles/r5/single_shot/), which reports a
// lost hand-off through the call's error word (Streams::kg_err); device-pointer calls, which have no
// host-visible error word, keep k_keygen_multi (no cross-workgroup waits, so nothing to time out).
// 0: k_keygen_multi everywhere (A/B builds: tools/build_variant.sh ... -DQRK_KG_PIPE=0).
#ifndef QRK_KG_PIPE
#define QRK_KG_PIPE 1
#endif
struct MkScr {
  uint4 xs[32 * 16];        // SampleNTT entries, load_sampled<16> layout (K^2 <= 16)
  uint32_t bop[4][16][16];  // NTT(s_j) basemul operands, word w of lane L at [j][w][L]
  float ef[4][16][16];      // NTT(e_i), coefficient t of lane L at [i][t][L]
};
struct MkLds {
  uint64_t ps[PRF_W * 16];
  uint32_t pbuf[44];
  uint64_t rho[4], sigma[4];
  uint64_t io[200];  // ek (KeyGen's LDS copy for H(ek)): 1568 B at K = 4
  GroupLds g[4];
  int last;
};
__device__ __forceinline__ void mk_wipe_lds(MkLds& sl) {
  __syncthreads();
  uint4* w = (uint4*)&sl;
  for (int x = threadIdx.x; x < (int)(sizeof(MkLds) / 16); x += (int)blockDim.x) w[x] = make_uint4(0, 0, 0, 0);
}

template <int K>
__global__ __launch_bounds__(64) void k_keygen_multi(size_t n, const uint8_t* __restrict__ coins,
                                                     uint8_t* __restrict__ pk, uint8_t* __restrict__ sk,
                                                     MkScr* __restrict__ scr_all, uint32_t* __restrict__ cnt,
                                                     uint32_t* done, uint32_t ticket) {
  constexpr int NI = 2 * K + K * K;
  __shared__ __attribute__((aligned(16))) MkLds sl;
  const size_t hs = blockIdx.x / NI;
  const int item = (int)(blockIdx.x % NI);
  const int lane = threadIdx.x;
  const Coop c = coop_init();
  const int i = c.idx;
  MkScr& scr = scr_all[hs];
  uint8_t* ek = pk + hs * P<K>::PK;
  uint8_t* dk = sk + hs * P<K>::SK;
  // the coins row (secret: always memory, never a kernel argument); z for dk's tail is loaded with d
  // rather than after H(ek) in the last workgroup
  const uint64_t* cw = (const uint64_t*)(coins + hs * 64);
  const uint64_t zw = (i >= 0 && i < 4) ? cw[4 + i] : 0;
  SS_MARK(blockIdx.x == 0 && lane == 0, 0);
  SS_MARK(blockIdx.x == NI - 1 && lane == 0, 14);
  {  // (rho, sigma) = G(d || k), in every workgroup
    const uint64_t* d = cw;
    CState g;
    if (i >= 0 && i < 4) cs_xor(g, d[i]);
    if (i == 4) g.lo ^= (uint32_t)K | (DS_SHA3 << 8);
    if (i == RW_SHA3_512 - 1) g.hi ^= 0x80000000u;
    g = kf_coop(g, c);
    if (i >= 0 && i < 4 && coop_canon(c)) sl.rho[i] = cs_word(g);
    if (i >= 4 && i < 8 && coop_canon(c)) sl.sigma[i - 4] = cs_word(g);
    wave_phase();
    SS_MARK(blockIdx.x == 0 && lane == 0, 13);
  }
  if (item < 2 * K) {  // PRF(sigma, item) -> CBD -> NTT: s_item (operand + dk) or e_(item - K)
    prf_coop<P<K>::ETA1>(sl.sigma, item, sl.ps, c);
    wave_phase();
    if (lane < 16) {
      PF16 f;
      cbd_f<P<K>::ETA1>(f, cbd_load<P<K>::ETA1, 16>(sl.ps, (size_t)item, lane));
      contig_to_stride_f(f, (float*)sl.g[0].poly, lane);
      ntt_fwd_f<false>(f, (float*)sl.g[0].poly, lane);
      if (item < K) {
        const BOp b = make_bop_f(f, lane);
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          scr.bop[item][u][lane] = b.b0[u];
          scr.bop[item][8 + u][lane] = b.b1[u];
        }
        P16 t;
#pragma unroll
        for (int x = 0; x < 16; ++x) t.v[x] = canon_f(f.v[x]);
        encode12(t, dk + 384 * item, lane);
      } else {
#pragma unroll
        for (int x = 0; x < 16; ++x) scr.ef[item - K][x][lane] = f.v[x];
      }
    }
  } else {  // SampleNTT entry e = x K + y straight into the scratch
    xof_coop<K>(sl.rho, item - 2 * K, (uint16_t*)scr.xs, sl.pbuf, c);
    SS_MARK(item == 2 * K && lane == 0, 15);
  }
  // publish, then count in: the last of the NI workgroups of this handshake finishes it.  With a
  // host-visible completion flag (n == 1, zero-copy pinned outputs) every workgroup's dk stores are
  // released at system scope before it counts in, so the host-side ordering does not rest on
  // agent -> system release transitivity across the XCDs' L2s.
  if (done)
    __threadfence_system();
  else
    __threadfence();
  __syncthreads();
  if (lane == 0) sl.last = (int)(atomicAdd(&cnt[hs], 1u) == (uint32_t)(NI - 1));
  __syncthreads();
  if (!sl.last) {
    mk_wipe_lds(sl);
    return;
  }
  __threadfence();  // acquire: the other workgroups' stores are visible past the counter
  SS_MARK(lane == 0, 4);
  if ((lane >> 4) < K) {  // t_hat_r = sum_j A[r][j] o s_hat_j + e_hat_r, one 16-lane group per row
    const int r = lane >> 4, L = lane & 15;
    int acc[16];
#pragma unroll
    for (int t = 0; t < 16; ++t) acc[t] = 0;
#pragma unroll
    for (int j = 0; j < K; ++j) {
      BOp b;
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        b.b0[u] = scr.bop[j][u][L];
        b.b1[u] = scr.bop[j][8 + u][L];
      }
      basemul_acc(acc, load_sampled<16>(scr.xs, (size_t)(j * K + r), L), b);
    }
    P16 t;
#pragma unroll
    for (int x = 0; x < 16; ++x) t.v[x] = canon_f(acc_to_f(acc[x]) + scr.ef[r][x][L]);
    encode12(t, ek + 384 * r, L);
    encode12(t, dk + 384 * K + 384 * r, L);
    encode12(t, (uint8_t*)sl.io + 384 * r, L);
  }
  if (lane < 4) {
    ((uint64_t*)(ek + 384 * K))[lane] = sl.rho[lane];
    ((uint64_t*)(dk + 768 * K))[lane] = sl.rho[lane];
    sl.io[48 * K + lane] = sl.rho[lane];
  }
  wave_phase();
  SS_MARK(lane == 0, 16);
  {  // dk tail: H(ek) || z
    CState s;
    coop_absorb<RW_SHA3_256, P<K>::PK / 8, DS_SHA3>(s, c, [&](int w) { return sl.io[w]; });
    uint64_t* tail = (uint64_t*)(dk + 768 * K + 32);
    if (i >= 0 && i < 4 && coop_canon(c)) {
      tail[i] = cs_word(s);
      tail[4 + i] = zw;
    }
    SS_MARK(lane == 0, 17);
  }
  // wipe the handshake's scratch (s_hat, e_hat, A) and reset its counter for the next call (wiping
  // it before H(ek) instead delays H by 0.9 us and saves 0.4 us after it:
  // profiles/r4/single_shot/keygen_trace_*.json)
  {
    uint4* w = (uint4*)&scr;
    for (int x = lane; x < (int)(sizeof(MkScr) / 16); x += 64) w[x] = make_uint4(0, 0, 0, 0);
  }
  if (lane == 0) atomicSub(&cnt[hs], (uint32_t)NI);
  if (done) __threadfence_system();
  mk_wipe_lds(sl);
  SS_MARK(lane == 0, 18);
  if (done && lane == 0) {
    // n == 1: the only handshake; the flag means every output is visible to the host
    __hip_atomic_store(done, ticket, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// ------------------------------------------------------------ single-shot KeyGen, H(ek) pipelined
// k_keygen_multi's critical path is G, three SampleNTT blocks, the count-in, t_hat, then the nine
// permutations of H(ek) = SHA3-256(t_hat || rho): 13 sequential cooperative permutations.  H(ek)
// absorbs t_hat_0 first, and t_hat_0's coefficient c needs only coefficient c of the row-0 entries
// A[0][j], which SampleNTT emits in FIPS order: so H's first blocks can run while SampleNTT still
// squeezes.  k_keygen_pipe, per handshake, 3K workgroups of K + 2 waves:
//   PRF items (2K, one wave busy): G, PRF(sigma, N), CBD, NTT -> NTT(s_j) basemul operands or
//     NTT(e_i) into the scratch, published to the others (write-through sc1 stores, a drained wave,
//     then an sc1 flag store: MI355X_MICROARCH.md "Valid forms", table row 1); dk's s_hat bytes
//   row r = 1 .. K-1 (K waves): G and SampleNTT A[r][j] (wave j), then t_hat_r, published the same
//     way; ek / dk's t_hat_r bytes
//   row 0 = the collector (K + 2 waves): waves 0 .. K-1 G and SampleNTT A[0][j], bumping an LDS count
//     after every block; wave K computes t_hat_0 in three ranges of coefficient pairs as soon as
//     every A[0][j] has emitted them (H(ek) blocks 0, 1 and 2 need t_hat_0 bytes < 136, < 272, all),
//     then copies t_hat_1 .. t_hat_{K-1} in from the row workgroups; wave K + 1 computes G itself
//     and absorbs ek block by block as its bytes arrive
// The critical path becomes G, SampleNTT's first two blocks (one block yields ~91 coefficients,
// H's block 0 needs 92), then the nine H(ek) permutations: 11 permutations.
// Hand-offs (MI355X_MICROARCH.md "Valid forms", the Consumer bullet with the acquire kept): the
// producer wave stores every payload byte with sc1 stores, waits vmcnt(0), then one lane stores the
// flag (sc1); the consumer wave polls the flag with relaxed sc1 loads, then ONE agent-scope acquire
// (buffer_inv sc1 + vmcnt(0): the CU's L1 may hold a stale line, the producer may sit on another
// XCD), then loads the payload in that same wave.
// Failure semantics: every wait is a bounded spin (KG_SPIN_TICKS).  A wait that expires marks its
// workgroup in error; a workgroup's outputs-done flag carries it (2 instead of 1); the collector,
// which waits for every other workgroup's flag, stores 1 into the call's error word (host-mapped,
// Streams::kg_err) before the completion ticket when any wait of the handshake expired, and the host
// returns OQS_ERROR for the call, re-zeroes the flag words (a straggler may set one after the
// collector's reset) and wipes the scratch.  The collector waits until every other workgroup has
// published its host outputs (system-scope release before the flag when the outputs are host
// memory), wipes the secret scratch (s_hat, e_hat), resets the flags and stores the ticket.
struct PipeScr {
  uint32_t bop[4][16][16];  // NTT(s_j) basemul operands, word w of lane L at [j][w][L] (secret)
  float ef[4][16][16];      // NTT(e_i), coefficient t of lane L at [i][t][L] (secret)
  uint32_t th[4][96];       // t_hat_r as ek bytes, rows 1 .. K-1 (public)
};
// flag words per handshake (ctx->kg_cnt, zeroed at allocation, reset by the collector):
// [N] PRF item N published, [8 + r] t_hat_r published, [16 + w] workgroup w's outputs written
constexpr int KG_FLAGS = 32;
struct PipeLds {
  uint4 xs[32 * 4];        // the workgroup's K <= 4 entries, load_sampled<4> layout
  uint32_t pbuf[4][44];    // SampleNTT parse buffers
  uint32_t bop[4][16][16];  // collector: the NTT(s_j) operands
  float ef[16][16];        // collector: NTT(e_0)
  uint64_t io[200];        // collector: ek (1568 B at K = 4)
  uint64_t rho[4][4];      // per SampleNTT wave
  uint64_t ps[PRF_W * 16];  // PRF items
  uint64_t sigma[4];
  GroupLds g;
  int prog[4], io_ready;
  int err;  // a bounded wait of this workgroup expired
};
typedef __attribute__((address_space(1))) uint32_t gu32;
typedef __attribute__((address_space(1))) uint64_t gu64;
__device__ __forceinline__ void st_sc1(uint32_t* p, uint32_t v) {
  __hip_atomic_store((gu32*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t ld_sc1(const uint32_t* p) {
  return __hip_atomic_load((gu32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// bounded spins (50 ms of the 100 MHz wall clock): a lost hand-off ends the kernel (and reports
// itself through the error word) instead of hanging the GPU
constexpr uint64_t KG_SPIN_TICKS = 5000000;
// one wave polls flag words (relaxed sc1 loads, all of them issued per pass) until every one is
// nonzero or the spin expires (returns false); *orv = OR of the values last read.  ACQ: the payload
// loads that follow in this wave are ordered by one agent-scope acquire (invalidates this CU's L1;
// its vmcnt(0) waits for the invalidate); without ACQ no payload is read after the poll.
template <int NF, bool ACQ>
__device__ __forceinline__ bool kg_wait_flags(const uint32_t* const (&f)[NF], uint32_t* orv = nullptr) {
  const uint64_t t0 = wall_clock64();
  bool all;
  uint32_t o;
  for (;;) {
    uint32_t v[NF];
#pragma unroll
    for (int k = 0; k < NF; ++k) v[k] = ld_sc1(f[k]);
    all = true;
    o = 0u;
#pragma unroll
    for (int k = 0; k < NF; ++k) all = all && v[k] != 0u, o |= v[k];
    if (all || wall_clock64() - t0 >= KG_SPIN_TICKS) break;
    __builtin_amdgcn_s_sleep(1);
  }
  if (ACQ) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  if (orv) *orv = o;
  return all;
}
__device__ __forceinline__ bool kg_wait_flag(const uint32_t* f) {
  const uint32_t* const a[1] = {f};
  return kg_wait_flags<1, true>(a);
}
// the storing wave's sc1 stores drained, then one lane stores the flag
__device__ __forceinline__ void kg_publish(uint32_t* f) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if ((threadIdx.x & 63) == 0) st_sc1(f, 1u);
}
__device__ __forceinline__ bool lds_wait_ge(const int* p, int v) {
  const uint64_t t0 = wall_clock64();
  bool ok;
  while (!(ok = __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) >= v) &&
         wall_clock64() - t0 < KG_SPIN_TICKS)
    __builtin_amdgcn_s_sleep(1);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  return ok;
}
// a wave whose bounded wait expired marks its workgroup in error (the whole wave stores the same 1)
__device__ __forceinline__ void kg_mark(PipeLds& sl, bool ok) {
  if (!ok) sl.err = 1;
}
__device__ __forceinline__ void lds_release_store(int* p, int v) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  if ((threadIdx.x & 63) == 0) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// (rho, sigma) = G(d || k) on one wave
__device__ __forceinline__ CState g_keygen_coop(const uint64_t* d, int K, const Coop& c) {
  const int i = c.idx;
  CState g;
  if (i >= 0 && i < 4) cs_xor(g, d[i]);
  if (i == 4) g.lo ^= (uint32_t)K | (DS_SHA3 << 8);
  if (i == RW_SHA3_512 - 1) g.hi ^= 0x80000000u;
  return kf_coop(g, c);
}
// SampleNTT A[r][j] = SampleNTT(rho || j || r) on wave j into slot j of the workgroup's entries
template <int K>
__device__ __forceinline__ void kg_pipe_sample(PipeLds& sl, const uint64_t* d, int r, int j, const Coop& c) {
  const CState g = g_keygen_coop(d, K, c);
  if (c.idx >= 0 && c.idx < 4 && coop_canon(c)) sl.rho[j][c.idx] = cs_word(g);
  wave_phase();
  uint16_t* xs16 = (uint16_t*)sl.xs;
  xof_coop_place<K>(
      sl.rho[j], j * K + r, sl.pbuf[j], c, [&](int q, uint32_t v) { xs16[(((q >> 3) * 4 + j) << 3) + (q & 7)] = (uint16_t)v; },
      [&](int cnt) {
        lds_release_store(&sl.prog[j], cnt < 256 ? cnt : 256);
        SS_MARK(r == 0 && j == 0 && (threadIdx.x & 63) == 0, cnt < 120 ? 10 : cnt < 210 ? 11 : 12);
      });
}
// The s_hat operands and e_hat_r from the PRF workgroups into LDS (one wave): it waits for their K + 1
// flags, then issues every 8-byte sc1 load before the first LDS store (one round trip, not one per load)
template <int K>
__device__ __forceinline__ void kg_load_ops(PipeLds& sl, const PipeScr& scr, const uint32_t* fl, int r) {
  const uint32_t* f[K + 1];
#pragma unroll
  for (int j = 0; j < K; ++j) f[j] = &fl[j];
  f[K] = &fl[K + r];
  kg_mark(sl, kg_wait_flags<K + 1, true>(f));
  const int lane = threadIdx.x & 63;
  constexpr int NB = K * 128 / 64, NE = 128 / 64;  // u64 words per lane
  uint64_t vb[NB], ve[NE];
  const uint64_t* sb = (const uint64_t*)&scr.bop[0][0][0];
  const uint64_t* se = (const uint64_t*)&scr.ef[r][0][0];
#pragma unroll
  for (int k = 0; k < NB; ++k) vb[k] = __hip_atomic_load((const gu64*)(sb + lane + 64 * k), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
  for (int k = 0; k < NE; ++k) ve[k] = __hip_atomic_load((const gu64*)(se + lane + 64 * k), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
  for (int k = 0; k < NB; ++k) ((uint64_t*)&sl.bop[0][0][0])[lane + 64 * k] = vb[k];
#pragma unroll
  for (int k = 0; k < NE; ++k) ((uint64_t*)&sl.ef[0][0])[lane + 64 * k] = ve[k];
  wave_phase();
}
// t_hat_r coefficient pair p (K-term basemul from the entries in LDS and the s_hat operands, + e_hat)
// as its three ek bytes
template <int K, typename BopAt, typename EfAt>
__device__ __forceinline__ uint32_t kg_pipe_pair(const PipeLds& sl, int p, BopAt bop_at, EfAt ef_at) {
  const int L = p >> 3, u = p & 7;
  int a0 = 0, a1 = 0;
#pragma unroll
  for (int j = 0; j < K; ++j) {
    const uint32_t a = ((const uint32_t*)sl.xs)[(((2 * p) >> 3) * 4 + j) * 4 + (p & 3)];
    a0 = dot2(a, bop_at(j, u, L), a0);
    a1 = dot2(a, bop_at(j, 8 + u, L), a1);
  }
  const uint32_t t0 = (uint32_t)canon_f(acc_to_f(a0) + ef_at(2 * u, L));
  const uint32_t t1 = (uint32_t)canon_f(acc_to_f(a1) + ef_at(2 * u + 1, L));
  return t0 | (t1 << 12);  // 24 bits, little-endian ek bytes 3p .. 3p + 2
}
// tests only (qrk_dbg_kg_late): the workgroup of role `late` (>= 0: PRF item N = role < 2K, or row
// r = role - 2K + 1) sleeps this long before it stores its payload and flags, past every consumer's
// and the collector's bounded wait
constexpr uint64_t KG_DBG_LATE_TICKS = 15000000;  // 150 ms
__device__ __forceinline__ void kg_dbg_sleep() {
  const uint64_t t0 = wall_clock64();
  while (wall_clock64() - t0 < KG_DBG_LATE_TICKS) __builtin_amdgcn_s_sleep(127);
}
template <int K>
__global__ __launch_bounds__(64 * (K + 2)) void k_keygen_pipe(size_t n, const uint8_t* __restrict__ coins,
                                                              uint8_t* __restrict__ pk, uint8_t* __restrict__ sk,
                                                              PipeScr* __restrict__ scr_all, uint32_t* __restrict__ flags,
                                                              uint32_t* done, uint32_t ticket, uint32_t* err, int late) {
  constexpr int NWG = 3 * K, PKB = P<K>::PK;
  __shared__ __attribute__((aligned(16))) PipeLds sl;
  const size_t hs = blockIdx.x / NWG;
  const int role = (int)(blockIdx.x % NWG);  // [0, 2K) PRF items, [2K, 3K - 1) rows 1 .. K-1, 3K - 1 the collector
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const Coop c = coop_init();
  const int i = c.idx;
  PipeScr& scr = scr_all[hs];
  uint32_t* fl = flags + hs * KG_FLAGS;
  uint8_t* ek = pk + hs * PKB;
  uint8_t* dk = sk + hs * P<K>::SK;
  const uint64_t* d = (const uint64_t*)(coins + hs * 64);
  // returns whether any wait of this workgroup expired, then wipes the LDS
  auto wipe_lds = [&] {
    __syncthreads();
    const int e = sl.err;
    __syncthreads();
    uint4* w = (uint4*)&sl;
    for (int x = threadIdx.x; x < (int)(sizeof(PipeLds) / 16); x += (int)blockDim.x) w[x] = make_uint4(0, 0, 0, 0);
    return e != 0;
  };
  // a non-collector workgroup's last act (after its LDS wipe): its host-memory outputs released at
  // system scope, then its flag, 2 when one of its waits expired (the collector's done ticket follows
  // every such flag)
  auto outputs_done = [&](int w, bool e) {
    if (done) __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      st_sc1(&fl[16 + w], e ? 2u : 1u);
    }
  };
  if (threadIdx.x < 4) sl.prog[threadIdx.x] = 0;
  if (threadIdx.x == 0) sl.io_ready = 0, sl.err = 0;
  __syncthreads();
  SS_MARK(role == NWG - 1 && threadIdx.x == 0, 0);
  if (role < 2 * K) {  // ------------------------------------------------ PRF item N = role
    const int N = role;
    if (wave == 0) {
      const CState g = g_keygen_coop(d, K, c);
      if (i >= 4 && i < 8 && coop_canon(c)) sl.sigma[i - 4] = cs_word(g);
      wave_phase();
      prf_coop<P<K>::ETA1>(sl.sigma, N, sl.ps, c);
      wave_phase();
      PF16 f;
      if (lane < 16) {
        cbd_f<P<K>::ETA1>(f, cbd_load<P<K>::ETA1, 16>(sl.ps, (size_t)N, lane));
        contig_to_stride_f(f, (float*)sl.g.poly, lane);
        ntt_fwd_f<false>(f, (float*)sl.g.poly, lane);
        if (role == late) kg_dbg_sleep();
        if (N < K) {
          const BOp b = make_bop_f(f, lane);
#pragma unroll
          for (int u = 0; u < 8; ++u) {
            st_sc1(&scr.bop[N][u][lane], b.b0[u]);
            st_sc1(&scr.bop[N][8 + u][lane], b.b1[u]);
          }
        } else {
#pragma unroll
          for (int x = 0; x < 16; ++x) st_sc1((uint32_t*)&scr.ef[N - K][x][lane], __float_as_uint(f.v[x]));
        }
      }
      kg_publish(&fl[N]);
      SS_MARK(N == 0 && lane == 0, 1);
      if (N < K && lane < 16) {
        P16 t;
#pragma unroll
        for (int x = 0; x < 16; ++x) t.v[x] = canon_f(f.v[x]);
        encode12(t, dk + 384 * N, lane);
      }
    }
    // sigma, the PRF output and NTT(s) / NTT(e): wiped before the flag that ends this workgroup
    const bool e = wipe_lds();
    outputs_done(N, e);
    return;
  }
  const int r = role < NWG - 1 ? role - 2 * K + 1 : 0;  // the matrix row of this workgroup
  if (wave < K) {  // ------------------------------------------------------ SampleNTT A[r][wave]
    kg_pipe_sample<K>(sl, d, r, wave, c);
    SS_MARK(r == 0 && wave == 0 && lane == 0, 2);
  }
  if (r > 0) {  // ---------------------------------------------------------- row r's t_hat
    if (wave == 0) {
      kg_load_ops<K>(sl, scr, fl, r);
#pragma unroll
      for (int j = 0; j < K; ++j) kg_mark(sl, lds_wait_ge(&sl.prog[j], 256));
      // lane l: pairs l and l + 64
      uint32_t tb[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int p = lane + 64 * h;
        tb[h] = kg_pipe_pair<K>(
            sl, p, [&](int j, int w, int L) { return sl.bop[j][w][L]; }, [&](int t, int L) { return sl.ef[t][L]; });
      }
      uint8_t* io8 = (uint8_t*)sl.io;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int p = lane + 64 * h;
        io8[3 * p] = (uint8_t)tb[h];
        io8[3 * p + 1] = (uint8_t)(tb[h] >> 8);
        io8[3 * p + 2] = (uint8_t)(tb[h] >> 16);
      }
      wave_phase();
      if (role == late) kg_dbg_sleep();
      const uint32_t* io32 = (const uint32_t*)sl.io;
      for (int w = lane; w < 96; w += 64) st_sc1(&scr.th[r][w], io32[w]);
      kg_publish(&fl[8 + r]);
      SS_MARK(r == 1 && lane == 0, 19);
      for (int w = lane; w < 96; w += 64) {
        ((uint32_t*)(ek + 384 * r))[w] = io32[w];
        ((uint32_t*)(dk + 384 * K + 384 * r))[w] = io32[w];
      }
    }
    const bool e = wipe_lds();  // the s_hat / e_hat copies: wiped before the flag that ends this workgroup
    outputs_done(2 * K + r - 1, e);
    return;
  }
  // ------------------------------------------------------------------------ the collector (row 0)
  uint8_t* io8 = (uint8_t*)sl.io;
  if (wave == K) {  // t_hat_0 pairs as A[0][j] fills, then the other rows' t_hat
    kg_load_ops<K>(sl, scr, fl, 0);
    SS_MARK(lane == 0, 22);
    // pair ranges whose bytes complete H(ek) blocks 0, 1, 2: pair p is ek bytes 3p .. 3p + 2
    constexpr int LIM[4] = {0, 46, 91, 128};
#pragma unroll 1
    for (int b = 0; b < 3; ++b) {
#pragma unroll
      for (int j = 0; j < K; ++j) kg_mark(sl, lds_wait_ge(&sl.prog[j], 2 * LIM[b + 1]));
      const int p = LIM[b] + lane;
      if (p < LIM[b + 1]) {
        const uint32_t t = kg_pipe_pair<K>(
            sl, p, [&](int j, int w, int L) { return sl.bop[j][w][L]; }, [&](int t, int L) { return sl.ef[t][L]; });
        io8[3 * p] = (uint8_t)t;
        io8[3 * p + 1] = (uint8_t)(t >> 8);
        io8[3 * p + 2] = (uint8_t)(t >> 16);
      }
      lds_release_store(&sl.io_ready, 3 * LIM[b + 1]);
    }
    SS_MARK(lane == 0, 3);
    const uint32_t* io32 = (const uint32_t*)sl.io;
    for (int w = lane; w < 96; w += 64) {
      ((uint32_t*)ek)[w] = io32[w];
      ((uint32_t*)(dk + 384 * K))[w] = io32[w];
    }
    for (int rr = 1; rr < K; ++rr) {
      kg_mark(sl, kg_wait_flag(&fl[8 + rr]));
      const uint64_t* st = (const uint64_t*)&scr.th[rr][0];
      uint64_t v = 0;
      if (lane < 48) v = __hip_atomic_load((const gu64*)(st + lane), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (lane < 48) sl.io[48 * rr + lane] = v;
      lds_release_store(&sl.io_ready, 384 * (rr + 1));
    }
    SS_MARK(lane == 0, 5);
  } else if (wave == K + 1) {  // H(ek), block by block as ek's bytes arrive
    __builtin_amdgcn_s_setprio(3);
    const uint64_t zw = (i >= 0 && i < 4) ? d[4 + i] : 0;
    SS_MARK(lane == 0, 7);
    constexpr int RW = RW_SHA3_256, NW = PKB / 8, NFULL = NW / RW, TAIL = NW % RW;
    const bool rl = i >= 0 && i < RW;
    CState s;
#pragma unroll 1
    for (int b = 0; b < NFULL; ++b) {
      const int need = 8 * RW * (b + 1) < 384 * K ? 8 * RW * (b + 1) : 384 * K;
      kg_mark(sl, lds_wait_ge(&sl.io_ready, need));
      SS_MARK(lane == 0 && b < 4, 8 + (b == 0 ? 0 : b == 1 ? 5 : b == 2 ? 1 : 6));
      if (rl) cs_xor(s, sl.io[b * RW + i]);
      s = kf_coop(s, c);
    }
    // rho (ek's last 32 bytes, in the final partial block for every K) from SampleNTT wave 0's copy
    // of G's output: wave 0 wrote it before its first progress release, which the t_hat wave acquired
    // before it released io_ready (this wave computes no G of its own: one cooperative permutation
    // fewer beside the SampleNTT waves)
    kg_mark(sl, lds_wait_ge(&sl.io_ready, 384 * K));
    if (i >= 0 && i < 4 && coop_canon(c)) {
      const uint64_t rw = sl.rho[0][i];
      sl.io[48 * K + i] = rw;
      ((uint64_t*)(ek + 384 * K))[i] = rw;
      ((uint64_t*)(dk + 768 * K))[i] = rw;
    }
    wave_phase();
    if (rl && i < TAIL) cs_xor(s, sl.io[NFULL * RW + i]);
    if (i == TAIL) s.lo ^= DS_SHA3;
    if (i == RW - 1) s.hi ^= 0x80000000u;
    s = kf_coop(s, c);
    if (i >= 0 && i < 4 && coop_canon(c)) {
      uint64_t* tail = (uint64_t*)(dk + 768 * K + 32);
      tail[i] = cs_word(s);
      tail[4 + i] = zw;
    }
    __builtin_amdgcn_s_setprio(0);
    SS_MARK(lane == 0, 4);
  }
  // Completion, in key-hygiene order: this workgroup's outputs released; its LDS (which holds copies
  // of s_hat and e_hat_0) wiped; every other workgroup's outputs (and its last scratch / flag
  // access) done; the secret scratch (s_hat, e_hat) wiped and the flags reset; those stores drained;
  // the error word set if any wait of this handshake expired; and only then the completion ticket
  // stored for the host -- the ticket is the kernel's last act.
  if (done) __threadfence_system();
  const bool own_err = wipe_lds();
  __syncthreads();
  if (wave == 0) {
    const uint32_t* of[NWG - 1];
#pragma unroll
    for (int w = 0; w < NWG - 1; ++w) of[w] = &fl[16 + w];
    uint32_t seen = 0u;
    const bool all = kg_wait_flags<NWG - 1, false>(of, &seen);  // no payload read after it
    uint4* sw = (uint4*)&scr;
    for (int x = lane; x < (int)(offsetof(PipeScr, th) / 16); x += 64) sw[x] = make_uint4(0, 0, 0, 0);
    if (lane < KG_FLAGS) st_sc1(&fl[lane], 0u);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    SS_MARK(lane == 0, 6);
    if (lane == 0 && (own_err || !all || (seen & 2u)))
      __hip_atomic_store(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (done && lane == 0) __hip_atomic_store(done, ticket, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// ============================================================ multi-role launches
// Every kernel of a call runs on the caller's stream.  Kernels of one operation that do not depend
// on each other share one launch instead of running on side streams: a multi-role kernel
// (k_multi<A, B, ...>) whose first nb_A workgroups run role A, the next nb_B role B, and so on.
// The dispatcher hands out workgroups in grid order, so the first role is resident from the start
// and the later roles fill the CUs around it and after it.  The first role is the latency-bound
// one: a lane-per-handshake sponge (one wave per SIMD at 2^16 handshakes) or the SampleNTT fix-up
// (~0.7 % of the entries, 4+ sequential permutations per lane), and the throughput-bound
// SampleNTT / PRF waves behind it keep the chip full while it runs (tools/fuse_probe.hip,
// profiles/r4/schedule_probe/: at 2^16 Encaps 0.518 -> 0.475 ms, Decaps 0.598 -> 0.535 ms per
// call).  A role must not use workgroup barriers (its workgroups may share a CU with another
// role's) -- the roles below synchronise at most within a wave.
template <int K, bool FIX>
struct RXof {  // SampleNTT, lane / matrix entry (FIX: the fix-up list, grid-stride over nb blocks)
  static constexpr int LDS = XOF_LDS, WPE = 1;
  XofArgs<K, FIX> a;
  unsigned nb;
  __device__ __forceinline__ void run(unsigned vb, char* lds) const { xof_body<K, FIX>(a, vb, nb, (uint32_t*)lds); }
};
// The fix-up list on one wave per entry (small chunks): the wave-cooperative sponge (~2.7 us per
// permutation) instead of one lane's (~9 us on a lone wave), so the 4+ dependent permutations of an
// entry stop being the critical path of the launch
template <int K>
struct RXofFixCoop {
  static constexpr int WAVE_LDS = 512 + 44 * 4;  // 256 placed values (u16) + the parse buffer
  static constexpr int LDS = 4 * WAVE_LDS, WPE = 1;
  XofArgs<K, true> a;
  unsigned nb;
  __device__ __forceinline__ void run(unsigned vb, char* lds) const {
    const int wave = threadIdx.x >> 6;
    char* w = lds + wave * WAVE_LDS;
    const Coop c = coop_init();
    const uint32_t limit = *a.nfix;
#pragma unroll 1
    for (uint32_t r = vb * 4 + wave; r < limit; r += nb * 4)  // wave-uniform
      xof_fix_coop<K>(a.rho_base, a.rho_stride, a.C, a.fix[r], a.out, (uint16_t*)w, (uint32_t*)(w + 512), c);
  }
};
template <int K>
struct RFrontEnc {  // (K, r) = G(m || H(ek)), lane / handshake
  static constexpr int LDS = 0, WPE = 1;
  const uint8_t *pk, *coins;
  size_t n;
  uint8_t* ss;
  uint64_t* seeds;
  unsigned nb;
  __device__ __forceinline__ void run(unsigned vb, char*) const {
    const size_t hs = (size_t)vb * 256 + threadIdx.x;
    if (hs < n) front_encaps_hs<K>(pk, coins, hs, ss, seeds);
  }
};
template <int K>
struct RJDec {  // Kbar = J(z || c), lane / handshake: needs only the inputs
  static constexpr int LDS = 0, WPE = 1;
  const uint8_t *ct, *sk;
  size_t n;
  uint64_t* kbar;
  unsigned nb;
  __device__ __forceinline__ void run(unsigned vb, char*) const {
    const size_t hs = (size_t)vb * 256 + threadIdx.x;
    if (hs < n) j_decaps_hs<K>(ct, sk, hs, kbar);
  }
};
// lane-pair forms of two sponge roles (keccak_pair.cuh), 128 handshakes per workgroup
#ifndef QRK_PAIR_FRONT_MAX
#define QRK_PAIR_FRONT_MAX (1 << 15)
#endif
struct PairLane {
  size_t hs;
  int half;
  uint32_t hm;
};
__device__ __forceinline__ PairLane pair_lane(unsigned vb) {
  const size_t t = (size_t)vb * 256 + threadIdx.x;
  const int half = (int)(t & 1);
  return {t >> 1, half, half ? 0xFFFFFFFFu : 0u};
}
template <int K>
struct RFrontEncPair {
  static constexpr int LDS = 0, WPE = 1;
  const uint8_t *pk, *coins;
  size_t n;
  uint8_t* ss;
  uint64_t* seeds;
  unsigned nb;
  __device__ __forceinline__ void run(unsigned vb, char*) const {
    const PairLane p = pair_lane(vb);
    if (p.hs < n) front_encaps_pair<K>(pk, coins, p.hs, p.half, p.hm, ss, seeds);
  }
};
template <int K>
struct RGDecPair {
  static constexpr int LDS = 0, WPE = 1;
  const uint8_t* sk;
  const uint64_t* mprime;
  size_t n;
  uint64_t *seeds, *kprime;
  unsigned nb;
  __device__ __forceinline__ void run(unsigned vb, char*) const {
    const PairLane p = pair_lane(vb);
    if (p.hs < n) g_decaps_pair<K>(sk, mprime, p.hs, p.half, p.hm, seeds, kprime);
  }
};
template <int K>
struct RGDec {  // (K', r') = G(m' || h), lane / handshake
  static constexpr int LDS = 0, WPE = 1;
  const uint8_t* sk;
  const uint64_t* mprime;
  size_t n;
  uint64_t *seeds, *kprime;
  unsigned nb;
  __device__ __forceinline__ void run(unsigned vb, char*) const {
    const size_t hs = (size_t)vb * 256 + threadIdx.x;
    if (hs < n) g_decaps_hs<K>(sk, mprime, hs, seeds, kprime);
  }
};
template <int ETA1, int ETA2>
struct RPrf {  // PRF_eta(seed, N), lane / (N, handshake)
  static constexpr int LDS = 0, WPE = 1;
  const uint64_t* seeds;
  size_t n, C;
  int nprf, eta1_upto;
  uint64_t* prf;
  unsigned nb;
  __device__ __forceinline__ void run(unsigned vb, char*) const {
    const size_t inst = (size_t)vb * 256 + threadIdx.x;
    if (inst >= (size_t)nprf * C || inst % C >= n) return;
    prf_inst<ETA1, ETA2>(seeds + (inst % C) * 4, (int)(inst / C), inst, eta1_upto, prf);
  }
};
template <int K>
struct RDecrypt {  // m' = K-PKE.Decrypt(dk, c), 16 lanes / handshake
  static constexpr int LDS = GROUPS * (int)sizeof(GroupLds), WPE = 1;
  size_t n;
  const uint8_t *ct, *sk;
  uint64_t* mprime;
  unsigned nb;
  __device__ __forceinline__ void run(unsigned vb, char* lds) const {
    const int gi = threadIdx.x >> 4;
    decrypt_core_hs<K>(n, ct, sk, mprime, (size_t)vb * GROUPS + gi, threadIdx.x & 15, ((GroupLds*)lds)[gi]);
  }
};

// Waves per SIMD the core is compiled for: 3 (<= 168 VGPRs).  ML-KEM-1024's Decaps core spills at
// 168 (16 B) and takes a scratch allocation that slowed the launch after it, so it keeps its 176
// VGPRs (2 waves); its Encaps core fits 168 without spilling: 3.05 -> 2.77 ms per 2^20 core launch
// (both cores at 3 waves, profiles/r6/core4/).
template <int K, int MODE>
struct RCore {  // K-PKE.Encrypt (MODE 1: the Decaps re-encryption, compare and select), 16 lanes / hs
  static constexpr int LDS = GROUPS * (int)sizeof(GroupLds), WPE = (K == 4 && MODE == 1) ? 1 : 3;
  size_t n, C;
  const uint64_t *xof, *prf;
  const uint8_t* ek;
  size_t ek_stride;
  const uint8_t* m_base;
  size_t m_stride;
  uint8_t* ct;
  int32_t* status;
  const uint64_t *kprime, *kbar;
  uint8_t* ss;
  unsigned nb;
  __device__ __forceinline__ void run(unsigned vb, char* lds) const {
    const int gi = threadIdx.x >> 4;
    encrypt_core_hs<K, MODE>(n, C, xof, prf, ek, ek_stride, m_base, m_stride, ct, status, kprime, kbar, ss,
                             (size_t)vb * GROUPS + gi, threadIdx.x & 15, ((GroupLds*)lds)[gi]);
  }
};

constexpr int max_of(int a, int b) { return a > b ? a : b; }
template <class... R>
struct Roles {
  static constexpr int LDS = 0, WPE = 1;
};
template <class R0, class... R>
struct Roles<R0, R...> {
  static constexpr int LDS = max_of(R0::LDS, Roles<R...>::LDS), WPE = max_of(R0::WPE, Roles<R...>::WPE);
};
// roles in grid order: workgroup w runs role i with w - (nb_0 + ... + nb_{i-1}) as its block index
template <class... R>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(Roles<R...>::WPE))) void k_multi(R... r) {
  constexpr int L = Roles<R...>::LDS;
  __shared__ __attribute__((aligned(16))) char lds[L > 16 ? L : 16];
  unsigned w = blockIdx.x;
  bool ran = false;
  ((ran = ran || (w < r.nb ? (r.run(w, lds), true) : (w -= r.nb, false))), ...);
}
template <class R>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(R::WPE))) void k_role(R r) {
  constexpr int L = R::LDS;
  __shared__ __attribute__((aligned(16))) char lds[L > 16 ? L : 16];
  r.run(blockIdx.x, lds);
}

// ============================================================ host launchers

inline unsigned blocks_for(size_t threads) { return (unsigned)((threads + 255) / 256); }
inline size_t round64(size_t x) { return (x + 63) & ~(size_t)63; }

// independent kernels of one operation: one multi-role launch (roles in grid order), or (serial
// schedule) one launch each in that order -- the per-kernel timings in isolation.  `name` joins
// the kernel names with '+'.
template <class R>
void launch_one(const char* name, const R& r, const Streams& s) {
  if (r.nb) QRK_LAUNCH(name, s.main, k_role<R>, dim3(r.nb), dim3(256), 0, s.main, r);
}
template <class... R>
void launch_multi(const char* name, std::initializer_list<const char*> names, const Streams& s, const R&... r) {
  hipStream_t st = s.main;
  if (names.size() != sizeof...(R)) {  // one name per role (a launcher bug, not an input error)
    qrk_chk(hipErrorInvalidValue);
    return;
  }
  if (s.serial) {
    const char* const* nm = names.begin();
    (launch_one(*nm++, r, s), ...);
    return;
  }
  const unsigned nb = (0u + ... + r.nb);
  if (nb) QRK_LAUNCH(name, st, (k_multi<R...>), dim3(nb), dim3(256), 0, st, r...);
}

// SampleNTT roles for a chunk of C handshakes (n used): the main pass and its fix-up.  The fix-up
// covers fix-up rates up to 1/64 (~0.7 % expected) in a single pass, one lane per listed entry:
// it is latency-bound (4+ sequential permutations per lane), a second grid-stride pass would double it.
// Where SampleNTT reads rho and counts its fix-up entries: the compact copy in scratch and the
// scratch counter (k_rho_copy zeroes it), or -- chunks <= DIRECT_RHO_MAX -- rho in the keys
// themselves and one of the context's two fix-up counters (Streams::fixc), the main pass zeroing
// the other one for the next call: no k_rho_copy launch.
struct RhoSrc {
  const uint8_t* base;
  size_t stride;
  uint32_t *nfix, *zero_next;
};
template <int K>
RXof<K, false> xof_role(const RhoSrc& r, size_t n, size_t C, const ScratchView& v) {
  return {{r.base, r.stride, n, C, (XUnit*)v.xof, v.fix, r.nfix, r.zero_next}, blocks_for((size_t)K * K * C)};
}
template <int K>
RXof<K, true> fix_role(const RhoSrc& r, size_t n, size_t C, const ScratchView& v) {
  return {{r.base, r.stride, n, C, (XUnit*)v.xof, v.fix, r.nfix, nullptr},
          (unsigned)std::min<size_t>((size_t)K * K * C / (64 * 256) + 1, 4096)};
}
template <int K>
RXof<K, false> xof_role(const uint8_t* rho, size_t n, size_t C, const ScratchView& v) {
  return xof_role<K>(RhoSrc{rho, 32, v.nfix, nullptr}, n, C, v);
}
template <int K>
RXof<K, true> fix_role(const uint8_t* rho, size_t n, size_t C, const ScratchView& v) {
  return fix_role<K>(RhoSrc{rho, 32, v.nfix, nullptr}, n, C, v);
}
// chunks up to this size run the fix-up one wave per entry (RXofFixCoop): below it the
// lane-per-entry fix-up's latency shows past the PRFs it shares a launch with, above it the
// cooperative form's issue slots (~4x per entry) cost more.  Same-box A/Bs against the lane form
// (profiles/r4/schedule_ab/abx_2p1*_coop_fixup.jsonl): 2^13 +24.8 %, 2^14 +15.8 %, 2^15 +4.5 %,
// 2^16 -3.1 %, 2^17 -4.2 %.
constexpr size_t COOP_FIX_MAX = (size_t)1 << 15;
template <int K>
RXofFixCoop<K> fix_coop_role(const RhoSrc& r, size_t n, size_t C, const ScratchView& v) {
  return {{r.base, r.stride, n, C, (XUnit*)v.xof, v.fix, r.nfix, nullptr},
          (unsigned)std::min<size_t>((size_t)K * K * C / 256 + 1, 4096)};  // waves for 1/64 of the entries
}
// {SampleNTT fix-up, PRFs}: the fix-up's workgroups first (grid order)
template <int K, class Prf>
void launch_fix_prf(const RhoSrc& r, size_t n, size_t C, const ScratchView& v, const Prf& prf, const Streams& s) {
  if (C <= COOP_FIX_MAX)
    launch_multi("k_xof_fix+k_prf", {"k_xof_fix", "k_prf"}, s, fix_coop_role<K>(r, n, C, v), prf);
  else
    launch_multi("k_xof_fix+k_prf", {"k_xof_fix", "k_prf"}, s, fix_role<K>(r, n, C, v), prf);
}
template <int K, class Prf>
void launch_fix_prf(const uint8_t* rho, size_t n, size_t C, const ScratchView& v, const Prf& prf, const Streams& s) {
  launch_fix_prf<K>(RhoSrc{rho, 32, v.nfix, nullptr}, n, C, v, prf, s);
}

// Chunks up to this size read rho straight from the keys: there the k_rho_copy launch (~5 us,
// launch-bound) costs more than the strided rho reads it saves (64 cache lines per wave instead of
// 16; at 2^20 handshakes those reads were 1.2 GB per k_xof launch, see k_rho_copy).
constexpr size_t DIRECT_RHO_MAX = (size_t)1 << 15;
// Encaps / Decaps rho source for a chunk of C handshakes: keys_rho = the first key's rho.
// The fix-up counter pair is correct only because every batched ML-KEM Encaps / Decaps chunk reaches
// this function through run_batch (abi.cpp), the only code that sets Streams::fixc / fixp, and
// run_batch marks the pair dirty (both words re-zeroed before the next chunk) on any error after the
// parity flip below.  A new caller of mlkem_encaps / mlkem_decaps must keep both properties.
inline RhoSrc rho_source(const uint8_t* keys_rho, size_t key_stride, size_t n, size_t C, const ScratchView& v,
                         const Streams& s) {
  if (C <= DIRECT_RHO_MAX && s.fixc && s.fixp) {
    const int p = *s.fixp;
    *s.fixp = p ^ 1;  // the next call counts into the word this call's main pass zeroes
    if (g_dbg_fail_after_flip) qrk_chk(hipErrorLaunchFailure);  // tests only: a failure after the flip
    return {keys_rho, key_stride, s.fixc + p, s.fixc + (p ^ 1)};
  }
  // k_xof reads rho from the compact copy in scratch
  QRK_LAUNCH("k_rho_copy", s.main, k_rho_copy, dim3(blocks_for(4 * n)), dim3(256), 0, s.main, keys_rho, key_stride,
             n, v.rho, v.nfix);
  return {(const uint8_t*)v.rho, 32, v.nfix, nullptr};
}

// QRK_DEBUG_POISON (environment, tests / tools only): fill the sampled-matrix region with 0xFF
// before a batched Encaps / Decaps, so a read of an entry the call has not written shows up as a
// wrong result instead of reusing the previous call's identical matrix.
inline bool debug_poison() {
  static const bool on = std::getenv("QRK_DEBUG_POISON") != nullptr;
  return on;
}
template <int K>
void poison_xof(size_t C, const ScratchView& v, hipStream_t st) {
  if (debug_poison()) qrk_chk(hipMemsetAsync(v.xof, 0xFF, (size_t)K * K * C * XOF_W * 8, st));
}

// KeyGen: front (rho, sigma) -> SampleNTT -> {SampleNTT fix-up, PRFs} -> t_hat rows -> H(ek)
template <int K>
hipError_t keygen_impl(size_t n, uint8_t* pk, uint8_t* sk, const uint8_t* coins, void* scratch, const Streams& s) {
  const size_t C = round64(n);
  ScratchView v = carve(scratch, K, C);
  if (QRK_KG_PIPE && n <= QRK_KG_MULTI_MAX && s.kg_cnt && s.kg_err) {  // host-pointer calls
    QRK_LAUNCH("k_keygen_pipe", s.main, k_keygen_pipe<K>, dim3((unsigned)(n * 3 * K)), dim3(64 * (K + 2)), 0, s.main, n,
               coins, pk, sk, (PipeScr*)scratch, s.kg_cnt, n == 1 ? s.done : nullptr, s.ticket, s.kg_err,
               g_kg_dbg_late);
    return hipGetLastError();
  }
  if (n <= QRK_KG_MULTI_MAX && s.kg_cnt) {  // device-pointer calls (no error word), QRK_KG_PIPE=0 builds
    QRK_LAUNCH("k_keygen_multi", s.main, k_keygen_multi<K>, dim3((unsigned)(n * (2 * K + K * K))), dim3(64), 0,
               s.main, n, coins, pk, sk, (MkScr*)scratch, s.kg_cnt, n == 1 ? s.done : nullptr, s.ticket);
    return hipGetLastError();
  }
  if (n <= QRK_SMALL_MAX) {
    QRK_LAUNCH("k_keygen_one", s.main, k_keygen_one<K>, dim3((unsigned)n), dim3(64 * KG_WAVES), 0, s.main, n, coins,
               pk, sk, n == 1 ? s.done : nullptr, s.ticket);
    return hipGetLastError();
  }
  hipStream_t st = s.main;
  if (s.xof_keep) v.xof = s.xof_keep;  // the handshake driver keeps A_hat for the same party's Decaps
  QRK_LAUNCH("k_front_keygen", st, k_front_keygen<K>, dim3(blocks_for(n)), dim3(256), 0, st, coins, n, pk, sk,
             v.seeds, v.rho, v.nfix);
  const uint8_t* rho = (const uint8_t*)v.rho;
  launch_one("k_xof", xof_role<K>(rho, n, C, v), s);
  launch_fix_prf<K>(rho, n, C, v, RPrf<P<K>::ETA1, P<K>::ETA1>{v.seeds, n, C, 2 * K, 2 * K, v.prf, blocks_for(2 * K * C)},
                    s);
  QRK_LAUNCH("k_keygen_core", st, k_keygen_core<K>, dim3((unsigned)((n + GROUPS - 1) / GROUPS)), dim3(256), 0, st,
             n, C, v.xof, v.prf, pk, sk);
  QRK_LAUNCH("k_back_keygen", st, k_back_keygen<K>, dim3(blocks_for(n)), dim3(256), 0, st, coins, n, pk, sk);
  return hipGetLastError();
}

// Encaps: rho copy -> {G(m || H(ek)), SampleNTT} -> {SampleNTT fix-up, PRFs} -> K-PKE.Encrypt
template <int K>
hipError_t encaps_impl(size_t n, uint8_t* ct, uint8_t* ss, const uint8_t* pk, const uint8_t* coins,
                       int32_t* status, void* scratch, const Streams& s) {
  const size_t C = round64(n);
  ScratchView v = carve(scratch, K, C);
  if (n <= QRK_SMALL_MAX) {
    EncIn<K> in{};
    const bool by_value = n == 1 && s.host_in1;
    if (by_value) memcpy(in.pk, s.host_in1, sizeof(in.pk));
    QRK_LAUNCH("k_encaps_one", s.main, k_encaps_one<K>, dim3((unsigned)n), dim3(64 * ONE_WAVES), 0, s.main, n,
               by_value ? nullptr : pk, coins, in, ct, ss, status, n == 1 ? s.done : nullptr, s.ticket);
    return hipGetLastError();
  }
  hipStream_t st = s.main;
  poison_xof<K>(C, v, st);
  const RhoSrc rho = rho_source(pk + 384 * K, (size_t)P<K>::PK, n, C, v, s);
  if (g_launch_err != hipSuccess) return g_launch_err;  // nothing after a failed step
  const RFrontEnc<K> front{pk, coins, n, ss, v.seeds, blocks_for(n)};
  const RPrf<P<K>::ETA1, P<K>::ETA2> prf{v.seeds, n, C, 2 * K + 1, K, v.prf, blocks_for((2 * K + 1) * C)};
  const RCore<K, 0> core{n, C, v.xof, v.prf, pk, (size_t)P<K>::PK, coins, (size_t)32, ct, status, v.kprime, v.kbar,
                         nullptr, (unsigned)((n + GROUPS - 1) / GROUPS)};
  if (C <= QRK_PAIR_FRONT_MAX)
    launch_multi("k_front_encaps+k_xof", {"k_front_encaps", "k_xof"}, s,
                 RFrontEncPair<K>{pk, coins, n, ss, v.seeds, blocks_for(2 * n)}, xof_role<K>(rho, n, C, v));
  else
    launch_multi("k_front_encaps+k_xof", {"k_front_encaps", "k_xof"}, s, front, xof_role<K>(rho, n, C, v));
  launch_fix_prf<K>(rho, n, C, v, prf, s);
  launch_one("k_encrypt_core", core, s);
  return hipGetLastError();
}

// Decaps: rho copy -> {J(z || c), K-PKE.Decrypt, SampleNTT} -> G(m' || h) -> {SampleNTT fix-up, PRFs}
// -> re-encryption with the constant-time compare and select
template <int K>
hipError_t decaps_impl(size_t n, uint8_t* ss, const uint8_t* ct, const uint8_t* sk, void* scratch,
                       const Streams& s) {
  const size_t C = round64(n);
  ScratchView v = carve(scratch, K, C);
  if (n <= QRK_SMALL_MAX) {
    DecIn<K> in{};
    const bool by_value = n == 1 && s.host_in1;
    if (by_value) memcpy(in.ct, s.host_in1, sizeof(in.ct));
    QRK_LAUNCH("k_decaps_one", s.main, k_decaps_one<K>, dim3((unsigned)n), dim3(64 * ONE_WAVES), 0, s.main, n,
               by_value ? nullptr : ct, sk, in, ss, n == 1 ? s.done : nullptr, s.ticket);
    return hipGetLastError();
  }
  hipStream_t st = s.main;
  const unsigned gblocks = (unsigned)((n + GROUPS - 1) / GROUPS);
  const RDecrypt<K> dec{n, ct, sk, v.mprime, gblocks};
  const RJDec<K> jd{ct, sk, n, v.kbar, blocks_for(n)};
  const RGDec<K> gd{sk, v.mprime, n, v.seeds, v.kprime, blocks_for(n)};
  const RPrf<P<K>::ETA1, P<K>::ETA2> prf{v.seeds, n, C, 2 * K + 1, K, v.prf, blocks_for((2 * K + 1) * C)};
  if (s.xof_given) {  // A_hat from this party's KeyGen (handshake driver): no SampleNTT, no fix-up
    const RCore<K, 1> core{n, C, s.xof_given, v.prf, sk + 384 * K, (size_t)P<K>::SK, (const uint8_t*)v.mprime,
                           (size_t)32, const_cast<uint8_t*>(ct), nullptr, v.kprime, v.kbar, ss, gblocks};
    launch_multi("k_j_decaps+k_decrypt_core", {"k_j_decaps", "k_decrypt_core"}, s, jd, dec);
    if (C <= QRK_PAIR_FRONT_MAX)
      launch_one("k_g_decaps", RGDecPair<K>{sk, v.mprime, n, v.seeds, v.kprime, blocks_for(2 * n)}, s);
    else
      launch_one("k_g_decaps", gd, s);
    launch_one("k_prf", prf, s);
    launch_one("k_encrypt_core", core, s);
    return hipGetLastError();
  }
  poison_xof<K>(C, v, st);
  const RhoSrc rho = rho_source(sk + 768 * K, (size_t)P<K>::SK, n, C, v, s);
  if (g_launch_err != hipSuccess) return g_launch_err;  // nothing after a failed step
  const RCore<K, 1> core{n, C, v.xof, v.prf, sk + 384 * K, (size_t)P<K>::SK, (const uint8_t*)v.mprime, (size_t)32,
                         const_cast<uint8_t*>(ct), nullptr, v.kprime, v.kbar, ss, gblocks};
  // J stays one lane per handshake: at chunks <= 2^15 its launch, {J, decrypt core, SampleNTT}, is
  // throughput-bound, and J on lane pairs (1.3x the issue slots) ran it 105.3 -> 118.7 us at 2^14
  // (47.2e6 against 45.5e6 handshakes/s, profiles/r5/pair_fronts/abx_2p14_pairJ_noJ_off.jsonl); J split
  // over this launch and the next (its last two permutations beside the fix-up and the PRFs) took
  // 4 us off this launch and added 3-14 us to the next: no gain (profiles/r5/mid/)
  launch_multi("k_j_decaps+k_decrypt_core+k_xof", {"k_j_decaps", "k_decrypt_core", "k_xof"}, s, jd, dec,
               xof_role<K>(rho, n, C, v));
  if (C <= QRK_PAIR_FRONT_MAX)
    launch_one("k_g_decaps", RGDecPair<K>{sk, v.mprime, n, v.seeds, v.kprime, blocks_for(2 * n)}, s);
  else
    launch_one("k_g_decaps", gd, s);
  launch_fix_prf<K>(rho, n, C, v, prf, s);
  launch_one("k_encrypt_core", core, s);
  return hipGetLastError();
}

}  // namespace mlkem

size_t mlkem_scratch_bytes(const AlgInfo& a, size_t chunk) {
  // the multi-workgroup KeyGen (n <= QRK_KG_MULTI_MAX) keeps one MkScr (16 KiB) per handshake in
  // the scratch; every other path needs scratch_words (about 5.1 KB per ML-KEM-768 handshake)
  const size_t C = mlkem::round64(chunk);
  return std::max(mlkem::scratch_words(a.k, C) * 8,
                  std::min(C, (size_t)QRK_KG_MULTI_MAX) * std::max(sizeof(mlkem::MkScr), sizeof(mlkem::PipeScr)));
}
size_t mlkem_matrix_bytes(const AlgInfo& a, size_t chunk) {
  return (size_t)a.k * a.k * mlkem::round64(chunk) * mlkem::XOF_W * sizeof(uint64_t);
}
size_t mlkem_kg_flag_words() { return (size_t)QRK_KG_MULTI_MAX * mlkem::KG_FLAGS; }
size_t mlkem_kg_scratch_bytes() {
  return (size_t)QRK_KG_MULTI_MAX * std::max(sizeof(mlkem::MkScr), sizeof(mlkem::PipeScr));
}
int g_kg_dbg_late = -1;
int g_dbg_fail_after_flip = 0;

size_t mlkem_small_max() { return QRK_SMALL_MAX; }
size_t mlkem_kg_multi_max() { return QRK_KG_MULTI_MAX; }

void mlkem_records_span(const AlgInfo& a, size_t C, size_t* off, size_t* bytes) {
  // mlkem::carve: the sampled matrix, the PRF words, then seeds | m' | K' | Kbar (4 C words each)
  const size_t K = (size_t)a.k;
  *off = (K * K * C * mlkem::XOF_W + (2 * K + 1) * C * mlkem::PRF_W) * sizeof(uint64_t);
  *bytes = 16 * C * sizeof(uint64_t);
}

hipError_t mlkem_cleanse(const AlgInfo& a, size_t n, void* scratch, hipStream_t st) {
  // the one-launch kernels (n <= QRK_SMALL_MAX) keep their key material in LDS and wipe it
  if (n == 0 || n <= QRK_SMALL_MAX) return hipSuccess;
  const size_t C = mlkem::round64(n);
  const mlkem::ScratchView v = mlkem::carve(scratch, a.k, C);
  return hipMemsetAsync(v.seeds, 0, 16 * C * sizeof(uint64_t), st);  // seeds | mprime | kprime | kbar
}

hipError_t mlkem_keypair(const AlgInfo& a, size_t n, uint8_t* pk, uint8_t* sk, const uint8_t* coins, void* scratch,
                         const Streams& st) {
  if (n == 0) return hipSuccess;
  switch (a.k) {
    case 2: return mlkem::keygen_impl<2>(n, pk, sk, coins, scratch, st);
    case 3: return mlkem::keygen_impl<3>(n, pk, sk, coins, scratch, st);
    case 4: return mlkem::keygen_impl<4>(n, pk, sk, coins, scratch, st);
  }
  return hipErrorInvalidValue;
}

hipError_t mlkem_encaps(const AlgInfo& a, size_t n, uint8_t* ct, uint8_t* ss, const uint8_t* pk,
                        const uint8_t* coins, int32_t* status, void* scratch, const Streams& st) {
  if (n == 0) return hipSuccess;
  switch (a.k) {
    case 2: return mlkem::encaps_impl<2>(n, ct, ss, pk, coins, status, scratch, st);
    case 3: return mlkem::encaps_impl<3>(n, ct, ss, pk, coins, status, scratch, st);
    case 4: return mlkem::encaps_impl<4>(n, ct, ss, pk, coins, status, scratch, st);
  }
  return hipErrorInvalidValue;
}

hipError_t mlkem_decaps(const AlgInfo& a, size_t n, uint8_t* ss, const uint8_t* ct, const uint8_t* sk,
                        void* scratch, const Streams& st) {
  if (n == 0) return hipSuccess;
  switch (a.k) {
    case 2: return mlkem::decaps_impl<2>(n, ss, ct, sk, scratch, st);
    case 3: return mlkem::decaps_impl<3>(n, ss, ct, sk, scratch, st);
    case 4: return mlkem::decaps_impl<4>(n, ss, ct, sk, scratch, st);
  }
  return hipErrorInvalidValue;
}

}  // namespace qrk

#if QRK_SS_TRACE
extern "C" int qrk_dbg_ss_trace(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(qrk::mlkem::g_ss_trace), sizeof(qrk::mlkem::g_ss_trace)) == hipSuccess ? 0 : -1;
}
#endif
