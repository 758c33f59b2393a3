// HQC-128/192/256 (round-4 submission, version 2023-04-30) KeyGen / Encaps / Decaps for gfx950.
//
// Replaces liboqs's HQC behind OQS_KEM_keypair/encaps/decaps, which the reference reaches
// from HQCKeyExchange (quantum_resistant_p2p/crypto/key_exchange.py:189-309) through
// vendor/oqs.py:318,348,372.  Conventions are restated in oracle/py/hqc_spec.py.
//
// Kernels (C = chunk of handshakes):
//   k_hqc_kg_expand   lane / hs   SE(sk_seed) -> x, y random words; SE(pk_seed) -> h stream
//   k_hqc_enc_expand  lane / (stream, hs)   theta = G(m || pk[0:80] || salt); SE(theta) -> r1, r2, e words | SE(pk_seed) -> h
//   k_hqc_dec_expand  lane / hs   SE(sk_seed) -> x, y words (decryption uses y)
//   k_hqc_kg_mul      WG / hs     s = x + y h; pk = pk_seed || s; sk = sk_seed || sigma || pk
//   k_hqc_enc_mul     WG / hs     u = r1 + r2 h, v = C.encode(m) + r2 s + e (truncated); ct; K-hash message
//                                 (REENC: the same re-encryption inside Decaps, compared with the received ct)
//   k_hqc_decode      WG / hs     v - u y, duplicated RM(1,7) decoding (wave-wide Hadamard transform) -> symbols
//   k_hqc_rs          wave / hs   RS decoding (syndromes, Berlekamp-Massey, Chien, Forney) -> m'
//   k_hqc_hash        lane / hs   ss = SHAKE256(m || u || v || 0x05)
//
// The sparse-dense products in F2[X]/(X^n - 1) run one workgroup (256 threads) per handshake.
// The dense operand b is kept in LDS "doubled": D = b_raw ^ (clean(b) << n) as 32-bit words,
// so that bit p of X^k b is bit p + n - k of D and every output word is one funnel shift
// (v_alignbit) of two consecutive D words; the shift is uniform per position k.  Thread t owns
// WPT consecutive output words.  b_raw keeps the bits above X^(n-1) a malformed pk/ct carries,
// which reproduces the reference's single-fold reduction exactly (oracle/src/hqc.c mul_sparse).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "keccak.cuh"
#include "keccak_coop.cuh"
#include "qrkem_internal.h"

namespace qrk {
namespace hqc {

constexpr int SEED = 40, SALT = 16, SSB = 64;

// TPB threads per handshake in the workgroup kernels.  In the sparse-dense products the threads
// form PC = TPB / NBT position classes of NBT threads: thread t owns WPT consecutive output
// words (j0 = (t % NBT) * WPT) and the positions i = t / NBT (mod PC); the classes' partial sums
// are XOR-combined in LDS.  Fewer, longer per-position windows (WPT + 1 reads for WPT words) and
// a position chain PC times shorter per wave: the products are latency-bound
// (profiles/r1/sq_hqc128_b16.txt).  WPT odd, so a wave's windows fall on distinct LDS banks.
// (WPT, NBT): one-operand products (KeyGen, Decaps); (WPTE, NBTE): Encaps' two-operand product.
template <int N_, int N1_, int N2_, int W_, int WR_, int WE_, int K_, int DELTA_, int MULT_, int WPT_, int NBT_,
          int WPTE_, int NBTE_, int TPB_>
struct Params {
  static constexpr int N = N_, N1 = N1_, N2 = N2_, W = W_, WR = WR_, WE = WE_, K = K_, DELTA = DELTA_,
                       MULT = MULT_, WPT = WPT_, NBT = NBT_, WPTE = WPTE_, NBTE = NBTE_, TPB = TPB_;
  static constexpr int NB = (N + 7) / 8, VB = N1 * N2 / 8;
  static constexpr int NW32 = (N + 31) / 32, VW32 = VB / 4, N32 = N >> 5, NR = N & 31;
  static constexpr int NHW = (NB + 7) / 8;  // h stream words (the seedexpander squeezes 8-byte units)
  static constexpr int PK = SEED + NB, SK = SEED + K + PK, CT = NB + VB + SALT, KPC = 2 * SEED + K, ENC = K + SALT;
  static constexpr int RWW = (4 * W + 7) / 8, RWR = (4 * WR + 7) / 8, RWE = (4 * WE + 7) / 8;
  static constexpr int NWP = NBT * WPT > NBTE * WPTE ? NBT * WPT : NBTE * WPTE, NH2 = NWP + N32 + 2;
  static constexpr int MSGB = K + NB + VB, MW = (MSGB + 2 + 7) / 8;  // K-hash message || 0x05 || 0x1F, words
  static constexpr int MBW = ((SK > 8 * MW ? SK : 8 * MW) + 15) / 4;  // LDS byte buffer, words
  static constexpr int T2 = 2 * DELTA, WMAX = W > WR ? W : WR;
  static constexpr int ROW_KG = 2 * RWW + NHW, ROW_ENC = 2 * RWR + RWE + NHW;
  static constexpr int ROWW = ROW_ENC > ROW_KG ? ROW_ENC : ROW_KG;
  static_assert(NR != 0, "n is never a multiple of 32 for HQC");
  static_assert(T2 + 1 <= 64 && WMAX <= 192 && N1 <= 128, "lane mappings");
  static_assert(NBT * WPT >= NW32 && NBTE * WPTE >= NW32, "WPT too small");
  static_assert(WPT % 2 == 1 && NBT % 64 == 0 && TPB % NBT == 0 && WPTE % 2 == 1 && NBTE % 64 == 0 &&
                    TPB % NBTE == 0 && TPB >= 256,
                "bank-conflict-free windows; whole waves per position class; >= 4 waves");
};
template <int L> struct HQ;
// A/B on one box (2^16): HQC-128 (5, 128) for both beats (9, 64) + (5, 256); HQC-256 Encaps keeps
// one position class (5, 384) while its Decaps gains from three (15, 128) (profiles/r1/ab_hqc_prod.txt)
template <> struct HQ<128> : Params<17669, 46, 384, 66, 75, 75, 16, 15, 3, 5, 128, 5, 128, 256> {};
// Threads per handshake for HQC-192 / 256 (A/B on one box, profiles/r2/ab_hqc_tpb.jsonl): HQC-256
// runs 512 (3 workgroups x 8 waves per CU under its 52 KB of LDS, against 3 x 6 at 384): enc+dec
// 3.81e6 -> 4.18e6 /s; HQC-192 stays at 256 (384 / 512 with three-word windows: 8.4e6 -> 7.25e6;
// 384 with five-word windows, 35.7 KB of LDS: 6.2e6),
// and so does HQC-128 (512: 17.2e6 -> 15.0e6; it already holds the 32-wave limit at 256).
template <> struct HQ<192> : Params<35851, 56, 640, 100, 114, 114, 24, 16, 5, 9, 128, 5, 256, 256> {};
template <> struct HQ<256> : Params<57637, 90, 640, 131, 149, 149, 32, 29, 5, 15, 128, 5, 512, 512> {};

// ---------------------------------------------------------------- GF(2^8) = F2[x]/(x^8+x^4+x^3+x^2+1)
struct alignas(4) GfTabs {
  uint8_t exp[512];
  uint8_t log[256];
};
constexpr GfTabs make_gf() {
  GfTabs t{};
  unsigned x = 1;
  for (int i = 0; i < 255; ++i) {
    t.exp[i] = (uint8_t)x;
    t.log[x] = (uint8_t)i;
    x <<= 1;
    if (x & 0x100) x ^= 0x11D;
  }
  for (int i = 255; i < 512; ++i) t.exp[i] = t.exp[i - 255];
  return t;
}
constexpr GfTabs GFC = make_gf();
__constant__ GfTabs GF = GFC;

constexpr uint8_t cgmul(uint8_t a, uint8_t b) { return (a && b) ? GFC.exp[GFC.log[a] + GFC.log[b]] : 0; }

// Reed-Solomon parity as a linear map: parity(m) = sum_i m_i PAR[i][.], rows = parity of unit messages
// (the LFSR encoder of the spec is GF(2^8)-linear in m).  Stored as logarithms, 255 = zero.
template <int L>
struct RsTab {
  uint8_t lp[HQ<L>::K][HQ<L>::T2];
};
template <int L>
constexpr RsTab<L> make_rs() {
  using P = HQ<L>;
  uint8_t g[P::T2 + 1] = {};
  g[0] = 1;
  for (int i = 1; i <= P::T2; ++i) {  // g *= (x + alpha^i)
    const uint8_t a = GFC.exp[i];
    for (int j = i; j >= 1; --j) g[j] = (uint8_t)(g[j - 1] ^ cgmul(g[j], a));
    g[0] = cgmul(g[0], a);
  }
  RsTab<L> t{};
  for (int u = 0; u < P::K; ++u) {
    uint8_t msg[P::K] = {};
    msg[u] = 1;
    uint8_t cdw[P::T2] = {};
    for (int i = 0; i < P::K; ++i) {
      const uint8_t gate = (uint8_t)(msg[P::K - 1 - i] ^ cdw[P::T2 - 1]);
      for (int j = P::T2 - 1; j > 0; --j) cdw[j] = (uint8_t)(cdw[j - 1] ^ cgmul(gate, g[j]));
      cdw[0] = cgmul(gate, g[0]);
    }
    for (int j = 0; j < P::T2; ++j) t.lp[u][j] = cdw[j] ? GFC.log[cdw[j]] : 255;
  }
  return t;
}
constexpr RsTab<128> RS128 = make_rs<128>();
constexpr RsTab<192> RS192 = make_rs<192>();
constexpr RsTab<256> RS256 = make_rs<256>();
__constant__ RsTab<128> RSD128 = RS128;
__constant__ RsTab<192> RSD192 = RS192;
__constant__ RsTab<256> RSD256 = RS256;
template <int L>
__device__ __forceinline__ const RsTab<L>& rs_tab() {
  if constexpr (L == 128) return RSD128;
  else if constexpr (L == 192) return RSD192;
  else return RSD256;
}

struct Lgf {
  const uint8_t* e;  // exp[512] in LDS
  const uint8_t* l;  // log[256] in LDS
  __device__ __forceinline__ uint32_t mul(uint32_t a, uint32_t b) const {
    const uint32_t r = e[l[a] + l[b]];
    return (a && b) ? r : 0u;
  }
  __device__ __forceinline__ uint32_t inv(uint32_t a) const { return e[255 - l[a]]; }
};

// ---------------------------------------------------------------- small helpers
__device__ __forceinline__ uint32_t alignbit(uint32_t hi, uint32_t lo, uint32_t s) {
  return __builtin_amdgcn_alignbit(hi, lo, s);
}

// little-endian 8 bytes at an arbitrary address: aligned dword loads, each holding at least
// one byte of the field (so a load never leaves the page the field lies in)
__device__ __forceinline__ uint64_t ld64u(const uint8_t* p) {
  const uintptr_t a = (uintptr_t)p;
  const uint32_t* b = (const uint32_t*)(a & ~(uintptr_t)3);
  const uint32_t sh = (uint32_t)(a & 3) * 8;
  const uint32_t w0 = b[0], w1 = b[1];
  const uint32_t w2 = sh ? b[2] : 0u;
  return (uint64_t)alignbit(w1, w0, sh) | ((uint64_t)alignbit(w2, w1, sh) << 32);
}

// word j (little-endian) of the nbytes-long byte string at src (any alignment), bytes past the
// end read as 0: one or two aligned dword loads, each holding at least one byte of the string
__device__ __forceinline__ uint32_t ld32_masked(const uint8_t* src, int j, int nbytes) {
  const uintptr_t a = (uintptr_t)src + 4 * (uintptr_t)j;
  const uint32_t* b = (const uint32_t*)(a & ~(uintptr_t)3);
  const uint32_t sh = (uint32_t)(a & 3) * 8;
  const int valid = nbytes - 4 * j;  // >= 1
  const uint32_t w0 = b[0];
  const uint32_t w1 = (sh != 0 && valid > 4 - (int)(sh >> 3)) ? b[1] : 0u;
  const uint32_t w = sh ? alignbit(w1, w0, sh) : w0;
  return valid >= 4 ? w : (w & ((1u << (8 * valid)) - 1));
}

// one-block SHAKE256 over NWM words that already hold the message, domain byte and 0x1F pad
template <int NWM>
__device__ __forceinline__ void shake256_block(KState& s, const uint64_t (&w)[NWM]) {
  static_assert(NWM <= RW_SHAKE256, "one block");
  kzero(s);
#pragma unroll
  for (int i = 0; i < NWM; ++i) kxor(s, i, w[i]);
  s.a[RW_SHAKE256 - 1].hi ^= 0x80000000u;
  keccak_f(s);
}

// seedexpander(seed) = SHAKE256(seed || 0x02)
__device__ __forceinline__ void seedexp_init(KState& s, const uint64_t (&seed)[5]) {
  uint64_t w[6] = {seed[0], seed[1], seed[2], seed[3], seed[4], 0x02ull | (0x1Full << 8)};
  shake256_block<6>(s, w);
}

// squeeze NW words of a sponge into out[0..NW)
__device__ __forceinline__ void squeeze_words(KState& s, uint64_t* out, int NW) {
  int w = 0;
#pragma unroll 1
  while (true) {
#pragma unroll
    for (int i = 0; i < RW_SHAKE256; ++i)
      if (w + i < NW) out[w + i] = kword(s, i);
    w += RW_SHAKE256;
    if (w >= NW) break;
    keccak_f(s);
  }
}

// ---------------------------------------------------------------- lane / hs: seedexpander streams
// row: [x words RWW][y words RWW][h words NHW]
template <int L>
__global__ __launch_bounds__(256) void k_hqc_kg_expand(const uint8_t* __restrict__ coins, size_t n,
                                                       uint64_t* __restrict__ row) {
  using P = HQ<L>;
  const size_t hs = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (hs >= n) return;
  const uint8_t* c = coins + hs * P::KPC;
  uint64_t* r = row + hs * P::ROWW;
  uint64_t sd[5];
  KState s;
#pragma unroll
  for (int i = 0; i < 5; ++i) sd[i] = ld64u(c + 8 * i);
  seedexp_init(s, sd);
  squeeze_words(s, r, 2 * P::RWW);
#pragma unroll
  for (int i = 0; i < 5; ++i) sd[i] = ld64u(c + SEED + P::K + 8 * i);
  seedexp_init(s, sd);
  squeeze_words(s, r + 2 * P::RWW, P::NHW);
}

// row: [r1 RWR][r2 RWR][e RWE][h NHW].  m, pk, salt at arbitrary byte addresses (Encaps:
// coins / pk; Decaps re-encryption: m' / the pk inside sk / the salt inside ct).  Two independent
// sponges per handshake run on separate lanes (inst = stream * C + hs, C a multiple of 64, so a
// wave runs one kind): stream 0 theta = G(m || pk[0:80] || salt) then SE(theta) -> r1, r2, e;
// stream 1 SE(pk_seed) -> h.  Twice the lanes of a lane-per-handshake launch (latency-bound
// sponges at ~1 wave per SIMD for a 2^16 batch).
template <int L>
__global__ __launch_bounds__(256) void k_hqc_enc_expand(const uint8_t* __restrict__ m, size_t m_stride,
                                                        const uint8_t* __restrict__ pk, size_t pk_stride,
                                                        const uint8_t* __restrict__ salt, size_t salt_stride,
                                                        size_t n, size_t C, uint64_t* __restrict__ row) {
  using P = HQ<L>;
  constexpr int KW = P::K / 8, TW = KW + 10 + 2 + 1;  // m || pk[0:80] || salt || (0x03, 0x1F)
  const size_t inst = (size_t)blockIdx.x * 256 + threadIdx.x;
  const size_t hs = inst % C;
  const bool hstream = inst >= C;
  if (hs >= n || inst >= 2 * C) return;
  const uint8_t* pp = pk + hs * pk_stride;
  uint64_t* r = row + hs * P::ROWW;
  KState s;
  uint64_t sd[5];
  if (hstream) {
#pragma unroll
    for (int i = 0; i < 5; ++i) sd[i] = ld64u(pp + 8 * i);
    seedexp_init(s, sd);
    squeeze_words(s, r + 2 * P::RWR + P::RWE, P::NHW);
    return;
  }
  const uint8_t* mp = m + hs * m_stride;
  const uint8_t* sp = salt + hs * salt_stride;
  uint64_t w[TW];
#pragma unroll
  for (int i = 0; i < KW; ++i) w[i] = ld64u(mp + 8 * i);
#pragma unroll
  for (int i = 0; i < 10; ++i) w[KW + i] = ld64u(pp + 8 * i);
  w[KW + 10] = ld64u(sp);
  w[KW + 11] = ld64u(sp + 8);
  w[KW + 12] = 0x03ull | (0x1Full << 8);
  shake256_block<TW>(s, w);
#pragma unroll
  for (int i = 0; i < 5; ++i) sd[i] = kword(s, i);  // theta[0:40]
  seedexp_init(s, sd);
  squeeze_words(s, r, 2 * P::RWR + P::RWE);
}

// row: [x words RWW][y words RWW]
template <int L>
__global__ __launch_bounds__(256) void k_hqc_dec_expand(const uint8_t* __restrict__ sk, size_t n,
                                                        uint64_t* __restrict__ row) {
  using P = HQ<L>;
  const size_t hs = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (hs >= n) return;
  const uint8_t* k = sk + hs * P::SK;
  uint64_t sd[5];
#pragma unroll
  for (int i = 0; i < 5; ++i) sd[i] = ld64u(k + 8 * i);
  KState s;
  seedexp_init(s, sd);
  squeeze_words(s, row + hs * P::ROWW, 2 * P::RWW);
}

// ss = SHAKE256(msg) over MW padded words per hs (msg || 0x05 || 0x1F || 0*)
template <int L>
__global__ __launch_bounds__(256) void k_hqc_hash(const uint64_t* __restrict__ msg, size_t n, uint8_t* __restrict__ ss) {
  using P = HQ<L>;
  constexpr int RW = RW_SHAKE256, NFULL = (P::MW - 1) / RW, REM = P::MW - NFULL * RW;
  const size_t hs = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (hs >= n) return;
  const uint64_t* m = msg + hs * P::MW;
  KState s;
  kzero(s);
  uint64_t nxt[RW];
#pragma unroll
  for (int i = 0; i < RW; ++i) nxt[i] = (NFULL > 0 || i < REM) ? m[i] : 0;
#pragma unroll 1
  for (int b = 0; b < NFULL; ++b) {
#pragma unroll
    for (int i = 0; i < RW; ++i) kxor(s, i, nxt[i]);
    const int nb = (b + 1) * RW;
#pragma unroll
    for (int i = 0; i < RW; ++i) nxt[i] = (b + 1 < NFULL || i < REM) ? m[nb + i] : 0;
    keccak_f(s);
  }
#pragma unroll
  for (int i = 0; i < REM; ++i) kxor(s, i, nxt[i]);
  s.a[RW - 1].hi ^= 0x80000000u;
  keccak_f(s);
  uint64_t* o = (uint64_t*)(ss + hs * SSB);
#pragma unroll
  for (int i = 0; i < 8; ++i) o[i] = kword(s, i);
}

// ---------------------------------------------------------------- small batches: wave-cooperative sponges
// Below QRK_HQC_COOP_MAX handshakes the seedexpander streams and the K hash run one sponge state
// per wave (keccak_coop.cuh, ~2.7 us per permutation against ~9 us for a lane alone on its SIMD):
// the reference calls one handshake at a time, where the hash's 33 / 67 / 106 sequential
// permutations and the h stream are the critical path.  Same outputs as the lane kernels above.
#ifndef QRK_HQC_COOP_MAX
#define QRK_HQC_COOP_MAX 256
#endif

// seedexpander(seed) = SHAKE256(seed || 0x02) with the 40-byte seed at any alignment
__device__ __forceinline__ CState seedexp_coop(const uint8_t* __restrict__ seed, const Coop& c) {
  const int i = c.idx;
  CState s;
  if (i >= 0 && i < 5) cs_xor(s, ld64u(seed + 8 * i));
  if (i == 5) cs_xor(s, 0x02ull | (0x1Full << 8));
  if (i == RW_SHAKE256 - 1) s.hi ^= 0x80000000u;
  return kf_coop(s, c);
}
__device__ __forceinline__ void squeeze_coop(CState& s, const Coop& c, uint64_t* out, int NW) {
  const bool canon = coop_canon(c);
  coop_squeeze<RW_SHAKE256>(s, c, NW, [&](int w, uint64_t v) {
    if (canon) out[w] = v;
  });
}

// wave b < n: x, y of hs b; wave n + b: the h stream of hs b
template <int L>
__global__ __launch_bounds__(64) void k_hqc_kg_expand_c(const uint8_t* __restrict__ coins, size_t n,
                                                        uint64_t* __restrict__ row) {
  using P = HQ<L>;
  const size_t inst = blockIdx.x, hs = inst % n;
  const bool hstream = inst >= n;
  const Coop c = coop_init();
  const uint8_t* cb = coins + hs * P::KPC;
  uint64_t* r = row + hs * P::ROWW;
  CState s = seedexp_coop(hstream ? cb + SEED + P::K : cb, c);
  if (hstream)
    squeeze_coop(s, c, r + 2 * P::RWW, P::NHW);
  else
    squeeze_coop(s, c, r, 2 * P::RWW);
}

// wave b < n: theta = G(m || pk[0:80] || salt), then SE(theta) -> r1, r2, e of hs b;
// wave n + b: SE(pk_seed) -> h of hs b
template <int L>
__global__ __launch_bounds__(64) void k_hqc_enc_expand_c(const uint8_t* __restrict__ m, size_t m_stride,
                                                         const uint8_t* __restrict__ pk, size_t pk_stride,
                                                         const uint8_t* __restrict__ salt, size_t salt_stride,
                                                         size_t n, uint64_t* __restrict__ row) {
  using P = HQ<L>;
  constexpr int KW = P::K / 8, TW = KW + 10 + 2 + 1;  // m || pk[0:80] || salt || (0x03, 0x1F)
  static_assert(TW <= RW_SHAKE256, "one block");
  const size_t inst = blockIdx.x, hs = inst % n;
  const Coop c = coop_init();
  const int i = c.idx;
  const uint8_t* pp = pk + hs * pk_stride;
  uint64_t* r = row + hs * P::ROWW;
  if (inst >= n) {
    CState s = seedexp_coop(pp, c);
    squeeze_coop(s, c, r + 2 * P::RWR + P::RWE, P::NHW);
    return;
  }
  const uint8_t* mp = m + hs * m_stride;
  const uint8_t* sp = salt + hs * salt_stride;
  CState g;
  if (i >= 0 && i < KW) cs_xor(g, ld64u(mp + 8 * i));
  if (i >= KW && i < KW + 10) cs_xor(g, ld64u(pp + 8 * (i - KW)));
  if (i >= KW + 10 && i < KW + 12) cs_xor(g, ld64u(sp + 8 * (i - KW - 10)));
  if (i == KW + 12) cs_xor(g, 0x03ull | (0x1Full << 8));
  if (i == RW_SHAKE256 - 1) g.hi ^= 0x80000000u;
  g = kf_coop(g, c);
  // seedexpander(theta[0:40]): every theta word stays on its lane
  CState s;
  if (i >= 0 && i < 5) cs_xor(s, cs_word(g));
  if (i == 5) cs_xor(s, 0x02ull | (0x1Full << 8));
  if (i == RW_SHAKE256 - 1) s.hi ^= 0x80000000u;
  s = kf_coop(s, c);
  squeeze_coop(s, c, r, 2 * P::RWR + P::RWE);
}

template <int L>
__global__ __launch_bounds__(64) void k_hqc_dec_expand_c(const uint8_t* __restrict__ sk, size_t n,
                                                         uint64_t* __restrict__ row) {
  using P = HQ<L>;
  const size_t hs = blockIdx.x;
  if (hs >= n) return;
  const Coop c = coop_init();
  CState s = seedexp_coop(sk + hs * P::SK, c);
  squeeze_coop(s, c, row + hs * P::ROWW, 2 * P::RWW);
}

template <int L>
__global__ __launch_bounds__(64) void k_hqc_hash_c(const uint64_t* __restrict__ msg, size_t n, uint8_t* __restrict__ ss) {
  using P = HQ<L>;
  constexpr int RW = RW_SHAKE256, NFULL = (P::MW - 1) / RW, REM = P::MW - NFULL * RW;
  const size_t hs = blockIdx.x;
  if (hs >= n) return;
  const Coop c = coop_init();
  const int i = c.idx;
  const bool rl = i >= 0 && i < RW;
  const uint64_t* m = msg + hs * P::MW;
  CState s;
  uint64_t nxt = (rl && (NFULL > 0 || i < REM)) ? m[i] : 0;
#pragma unroll 1
  for (int b = 0; b < NFULL; ++b) {
    cs_xor(s, nxt);
    nxt = (rl && (b + 1 < NFULL || i < REM)) ? m[(b + 1) * RW + i] : 0;
    s = kf_coop(s, c);
  }
  cs_xor(s, nxt);
  if (i == RW - 1) s.hi ^= 0x80000000u;
  s = kf_coop(s, c);
  if (coop_canon(c) && i < 8) ((uint64_t*)(ss + hs * SSB))[i] = cs_word(s);
}

// ---------------------------------------------------------------- workgroup / hs helpers
// Thread index as seen by the workgroup helpers: threadIdx.x plus an opaque zero produced inside
// the caller's code (a volatile v_mov).  In the persistent handshake loop (k_hqc_enc_mul) the
// compiler would otherwise hoist every loop-invariant LDS address out of the loop and keep it
// live in a register (110-180 VGPRs, then spills under an occupancy bound); derived from this
// value, the addresses are recomputed per iteration (a few VALU ops) instead.
__device__ __forceinline__ int hq_tid() {
  int z;
  asm volatile("v_mov_b32 %0, 0" : "=v"(z));
  const int t = (int)threadIdx.x + z;
  __builtin_assume(t >= 0 && t < 1024);
  return t;
}

// support of a fixed-weight vector from its random words: s_i = i + floor(r_i (n - i) / 2^32)
template <int L>
__device__ __forceinline__ void supports_raw(const uint64_t* words, int weight, uint32_t* sup) {
  using P = HQ<L>;
  const uint32_t* r32 = (const uint32_t*)words;
  for (int i = hq_tid(); i < weight; i += P::TPB)
    sup[i] = (uint32_t)i + __umulhi(r32[i], (uint32_t)(P::N - i));
}

// The spec's duplicate removal (oracle/src/hqc.c fixed_weight): for i = w-2 .. 0, s_i := i when
// s_i equals some s_j with j > i (the current, possibly replaced, s_j).
// Duplicate removal of one vector of weight WT (<= 192) on one wave, element 64e + l in lane l's
// register v[e], no LDS round trips and no workgroup barriers (other waves work on their own
// vectors meanwhile).  The spec's loop has a closed form (tests/test_hqc_dedupe.py checks it and
// this wave restatement against the loop): s_i is replaced iff
//   s_j == s_i for some j > i   (the original values), or
//   i < s_i < w and s_{s_i} is replaced   (a chain through strictly increasing indices).
// The first term: every s_j broadcast once (v_readlane) and compared with all lanes (a ballot per
// register, masked to j > i, OR-ed into 64-bit lane masks); the chain: pointer jumping over
// (replaced, next) words gathered with ds_bpermute, ceil(log2 w) rounds.
// One v_readlane broadcast of s_j per j and a ballot per register.  The first term by lane rotations
// (63 rounds of ds_bpermute: HQC-128 enc_mul 0.976 vs 0.766 ms, profiles/r2/ab_hqc_dedupe_rot_rejected.jsonl
// -- the permutes compete with the products for the CU's LDS) or by broadcasts into per-lane VGPR
// accumulators (0.85 vs 0.77 ms, ab_hqc_dedupe_vreg_rejected.jsonl) was slower.
template <int WT>
__device__ __forceinline__ void dedupe_wave_cf(uint32_t* s) {
  constexpr int NE = (WT + 63) / 64;
  constexpr uint32_t NONE = 0xFFFFu, REP = 0x80000000u;
  constexpr int ROUNDS = 32 - __builtin_clz(WT - 1);
  static_assert(NE <= 3 && WT > 1, "weight");
  const int lane = hq_tid() & 63;
  uint32_t v[NE];
#pragma unroll
  for (int e = 0; e < NE; ++e) v[e] = (64 * e + lane < WT) ? s[64 * e + lane] : 0xFFFFFFFFu;
  uint64_t dup[NE] = {};
#pragma unroll
  for (int j = 1; j < WT; ++j) {
    const uint32_t sj = (uint32_t)__builtin_amdgcn_readlane((int)v[j >> 6], j & 63);
#pragma unroll
    for (int e = 0; e < NE; ++e) {
      if (64 * e >= j) continue;  // no i < j in this register
      uint64_t m = __ballot(v[e] == sj);
      if (64 * e + 64 > j) m &= (1ull << (j - 64 * e)) - 1;  // i < j
      dup[e] |= m;
    }
  }
  uint32_t x[NE];  // REP | next chain index (or NONE)
#pragma unroll
  for (int e = 0; e < NE; ++e) {
    const uint32_t i = 64 * e + lane;
    const uint32_t ptr = (v[e] > i && v[e] < (uint32_t)WT) ? v[e] : NONE;
    x[e] = ((dup[e] >> lane) & 1 ? REP : 0u) | ptr;
  }
#pragma unroll 1
  for (int r = 0; r < ROUNDS; ++r) {
    uint32_t y[NE];
#pragma unroll
    for (int e = 0; e < NE; ++e) {
      const uint32_t p = x[e] & NONE;
      const int src = 4 * (int)(p & 63);  // lane of element p (any lane when p == NONE)
      uint32_t g = 0;
#pragma unroll
      for (int f = 0; f < NE; ++f) {
        const uint32_t gf = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)x[f]);
        g = (p >> 6) == (uint32_t)f ? gf : g;
      }
      y[e] = p == NONE ? x[e] : ((x[e] & REP) | g);
    }
#pragma unroll
    for (int e = 0; e < NE; ++e) x[e] = y[e];
  }
#pragma unroll
  for (int e = 0; e < NE; ++e)
    if (64 * e + lane < WT) s[64 * e + lane] = (x[e] & REP) ? (uint32_t)(64 * e + lane) : v[e];
}

// The closed form on one wave.  A/B on one box (profiles/r2/ab_hqc_dedupe_staging.jsonl): HQC-128 /
// 256 enc+dec 17.26e6 / 3.76e6 (closed form, LDS staging) against 16.37e6 / 3.43e6 with round 1's
// workgroup-wide dedupe; the spec's serial loop, a workgroup-wide first term and a first term by
// lane rotations were slower or throughput-neutral (profiles/r2/ab_hqc_dedupe_*_rejected.jsonl).
template <int WT>
__device__ __forceinline__ void dedupe_wave(uint32_t* s) {
  dedupe_wave_cf<WT>(s);
}

// Raw words are staged in LDS first (building the doubled operands straight from global words, 3
// loads per word, was 2-3 % slower).

// doubled dense operand: D[q] = raw[q] ^ (clean << n)[q], raw words via rd(j) (0 outside [0, NW32)),
// clean = raw masked to n bits.  Written for q in [0, NH2).
template <int L, typename Rd>
__device__ __forceinline__ void build_doubled(uint32_t* D, Rd rd) {
  using P = HQ<L>;
  constexpr uint32_t TOPMASK = (1u << P::NR) - 1;
  auto clean = [&](int j) -> uint32_t {
    if (j < 0 || j >= P::NW32) return 0u;
    const uint32_t v = rd(j);
    return j == P::NW32 - 1 ? (v & TOPMASK) : v;
  };
  // every read first, then the stores: with a global-memory reader the thread's loads are all
  // in flight together (one round trip instead of one per output word)
  constexpr int QPT = (P::NH2 + P::TPB - 1) / P::TPB;
  const int tq = hq_tid();
  uint32_t d[QPT];
#pragma unroll
  for (int k = 0; k < QPT; ++k) {
    const int q = tq + k * P::TPB;
    uint32_t v = 0;
    if (q < P::NH2) {
      v = q < P::NW32 ? rd(q) : 0u;
      if (q >= P::N32) v ^= alignbit(clean(q - P::N32), clean(q - P::N32 - 1), 32 - P::NR);
    }
    d[k] = v;
  }
#pragma unroll
  for (int k = 0; k < QPT; ++k) {
    const int q = tq + k * P::TPB;
    if (q < P::NH2) D[q] = d[k];
  }
}

// Both doubled operands built in place from raw words staged at the front of D1 / D2
// (every thread reads first, one barrier, then the stores), so enc_mul needs no separate staging /
// message buffer and its LDS footprint drops by MBW words (more workgroups per CU for HQC-192/256).
template <int L>
__device__ __forceinline__ void build_doubled2_inplace(uint32_t* D1, uint32_t* D2) {
  using P = HQ<L>;
  constexpr uint32_t TOPMASK = (1u << P::NR) - 1;
  constexpr int QPT = (P::NH2 + P::TPB - 1) / P::TPB;
  const int tq = hq_tid();
  uint32_t a[QPT], b[QPT];
#pragma unroll
  for (int k = 0; k < QPT; ++k) {
    const int q = tq + k * P::TPB;
    uint32_t va = 0, vb = 0;
    if (q < P::NH2) {
      if (q < P::NW32) va = D1[q], vb = D2[q];
      if (q >= P::N32) {
        const int j1 = q - P::N32, j0 = j1 - 1;  // j1 < NW32 always; j0 may be -1
        uint32_t h1 = j1 < P::NW32 ? D1[j1] : 0u, s1 = j1 < P::NW32 ? D2[j1] : 0u;
        uint32_t h0 = j0 >= 0 ? D1[j0] : 0u, s0 = j0 >= 0 ? D2[j0] : 0u;
        if (j1 == P::NW32 - 1) h1 &= TOPMASK, s1 &= TOPMASK;
        if (j0 == P::NW32 - 1) h0 &= TOPMASK, s0 &= TOPMASK;
        va ^= alignbit(h1, h0, 32 - P::NR);
        vb ^= alignbit(s1, s0, 32 - P::NR);
      }
    }
    a[k] = va, b[k] = vb;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < QPT; ++k) {
    const int q = tq + k * P::TPB;
    if (q < P::NH2) D1[q] = a[k], D2[q] = b[k];
  }
}

// (Taking each window's last word from the neighbouring lane by DPP wave_shl:1 was slower: HQC-128
// enc_mul 0.818 vs 0.766 ms, HQC-256 6.18 vs 4.98 ms, profiles/r2/ab_hqc_dpp_win_rejected.jsonl.)
// acc[c] ^= word (j0 + c) of X^k D-operand for the positions k of sup in this thread's class
// (partial sums; prod_combine adds the classes)
template <int L, int NV, int WPT, int NBT>
__device__ __forceinline__ void sparse_dense(const uint32_t* sup, int weight, const uint32_t* const (&D)[NV],
                                             uint32_t (&acc)[NV][WPT]) {
  using P = HQ<L>;
  constexpr int PC = P::TPB / NBT;
  const int tt = hq_tid();
  const int j0 = (tt % NBT) * WPT;
  // one operand: unrolled so the next position's support read and window are in flight together;
  // two operands: not unrolled (both windows already in flight; keeps <= 64 VGPRs, 8 waves / SIMD)
  constexpr int UNR = NV == 1 ? 2 : 1;
#pragma unroll UNR
  for (int i = tt / NBT; i < weight; i += PC) {
    const uint32_t k = sup[i];
    const uint32_t e = (uint32_t)P::N - k;
    const int off = (int)(e >> 5) + j0;
    const uint32_t sh = e & 31;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      uint32_t w[WPT + 1];
#pragma unroll
      for (int c = 0; c <= WPT; ++c) w[c] = D[v][off + c];
#pragma unroll
      for (int c = 0; c < WPT; ++c) acc[v][c] ^= alignbit(w[c + 1], w[c], sh);
    }
  }
}

// out[v][j0 + c] = the product words: class 0 stores, the other classes XOR in after a barrier.
// Call with the operands no longer needed by any thread (out may alias them); `extra` runs in the
// XOR phase (further commutative updates of out).  Ends with a barrier.
template <int NV, int WPT, int NBT, typename Extra>
__device__ __forceinline__ void prod_combine(uint32_t* const (&out)[NV], const uint32_t (&acc)[NV][WPT], Extra extra) {
  const int tt = hq_tid();
  const int j0 = (tt % NBT) * WPT;
  const bool first = tt < NBT;
  if (first)
#pragma unroll
    for (int v = 0; v < NV; ++v)
#pragma unroll
      for (int q = 0; q < WPT; ++q) out[v][j0 + q] = acc[v][q];
  __syncthreads();
  if (!first)
#pragma unroll
    for (int v = 0; v < NV; ++v)
#pragma unroll
      for (int q = 0; q < WPT; ++q) atomicXor(&out[v][j0 + q], acc[v][q]);
  extra();
  __syncthreads();
}

// RM(1,7) codeword word q (0..3) of symbol b: bit j = b7 ^ <b0..6, j>
__device__ __forceinline__ uint32_t rm_word(uint32_t b, int q) {
  uint32_t w = 0u - (b >> 7 & 1);
  w ^= (0u - (b & 1)) & 0xaaaaaaaau;
  w ^= (0u - (b >> 1 & 1)) & 0xccccccccu;
  w ^= (0u - (b >> 2 & 1)) & 0xf0f0f0f0u;
  w ^= (0u - (b >> 3 & 1)) & 0xff00ff00u;
  w ^= (0u - (b >> 4 & 1)) & 0xffff0000u;
  w ^= (0u - (b >> 5 & 1)) & (0u - (uint32_t)(q & 1));
  w ^= (0u - (b >> 6 & 1)) & (0u - (uint32_t)(q >> 1 & 1));
  return w;
}

__device__ __forceinline__ uint32_t lds_u32_unaligned(const uint8_t* b, int off) {
  return (uint32_t)b[off] | (uint32_t)b[off + 1] << 8 | (uint32_t)b[off + 2] << 16 | (uint32_t)b[off + 3] << 24;
}
__device__ __forceinline__ void lds_store_u32_unaligned(uint8_t* b, int off, uint32_t v) {
  b[off] = (uint8_t)v;
  b[off + 1] = (uint8_t)(v >> 8);
  b[off + 2] = (uint8_t)(v >> 16);
  b[off + 3] = (uint8_t)(v >> 24);
}

__device__ __forceinline__ void fill_gf(uint8_t* e, uint8_t* l) {
  for (int i = threadIdx.x; i < 512; i += blockDim.x) e[i] = GF.exp[i];
  for (int i = threadIdx.x; i < 256; i += blockDim.x) l[i] = GF.log[i];
}

// ---------------------------------------------------------------- KeyGen: s = x + y h
template <int L>
__global__ __launch_bounds__(HQ<L>::TPB) __attribute__((amdgpu_waves_per_eu(1))) void k_hqc_kg_mul(size_t n, const uint64_t* __restrict__ row,
                                                    const uint8_t* __restrict__ coins, uint8_t* __restrict__ pk,
                                                    uint8_t* __restrict__ sk) {
  using P = HQ<L>;
  __shared__ uint32_t D[P::NH2];
  __shared__ uint32_t MB[P::MBW];
  __shared__ uint32_t SS[2 * P::WMAX];
  uint32_t* const SX = SS;
  uint32_t* const SY = SS + P::WMAX;
  const size_t hs = blockIdx.x;
  if (hs >= n) return;
  const int t = threadIdx.x;
  const uint64_t* rw = row + hs * P::ROWW;
  const uint8_t* c = coins + hs * P::KPC;
  uint8_t* mb = (uint8_t*)MB;
  const uint32_t* h32 = (const uint32_t*)(rw + 2 * P::RWW);
  build_doubled<L>(D, [&](int j) { return j == P::NW32 - 1 ? h32[j] & ((1u << P::NR) - 1) : h32[j]; });  // h: n bits
  supports_raw<L>(rw, P::W, SX);
  supports_raw<L>(rw + P::RWW, P::W, SY);
  // sk = sk_seed || sigma || pk_seed || s  (the coins' first 80 + K bytes, in order)
  for (int j = t; j < (P::KPC + 3) / 4; j += P::TPB) MB[j] = ld32_masked(c, j, P::KPC);
  __syncthreads();
  if (t < 64) dedupe_wave<P::W>(SX);
  else if (t < 128) dedupe_wave<P::W>(SY);
  __syncthreads();
  uint32_t acc[1][P::WPT] = {};
  const uint32_t* const Ds[1] = {D};
  sparse_dense<L, 1, P::WPT, P::NBT>(SY, P::W, Ds, acc);
  __syncthreads();  // D is reused as the output buffer
  uint32_t* const outs[1] = {D};
  prod_combine<1, P::WPT, P::NBT>(outs, acc, [&] {
    for (int i = t; i < P::W; i += P::TPB) atomicXor(&D[SX[i] >> 5], 1u << (SX[i] & 31));
  });
  constexpr int SOFF = (2 * SEED + P::K) / 4;  // s at byte 80 + K (a multiple of 4)
  for (int j = t; j < P::NW32; j += P::TPB) MB[SOFF + j] = j == P::NW32 - 1 ? (D[j] & ((1u << P::NR) - 1)) : D[j];
  __syncthreads();
  uint8_t* so = sk + hs * P::SK;
  uint8_t* po = pk + hs * P::PK;
#pragma unroll 8
  for (int b = t; b < P::SK; b += P::TPB) so[b] = mb[b];
#pragma unroll 8
  for (int b = t; b < P::PK; b += P::TPB) po[b] = mb[SEED + P::K + b];
}

// ---------------------------------------------------------------- phase trace (tools only)
// -DQRK_HQC_TRACE=1: workgroup QRK_HQC_TRACE_WG of k_hqc_enc_mul / k_hqc_decode stamps the 100 MHz
// wall clock at its phase boundaries (tools/hqc_trace.py reads them through qrk_dbg_hqc_trace).
#ifndef QRK_HQC_TRACE
#define QRK_HQC_TRACE 0
#endif
#ifndef QRK_HQC_TRACE_WG
#define QRK_HQC_TRACE_WG 30000
#endif
#if QRK_HQC_TRACE
__device__ unsigned long long g_hqc_trace[32];
#define HQ_MARK(i)                                                                 \
  do {                                                                             \
    if (blockIdx.x == QRK_HQC_TRACE_WG && threadIdx.x == 0) g_hqc_trace[i] = wall_clock64(); \
  } while (0)
#define HQ_MARK_T(i, tid)                                                          \
  do {                                                                             \
    if (blockIdx.x == QRK_HQC_TRACE_WG && threadIdx.x == (tid)) g_hqc_trace[i] = wall_clock64(); \
  } while (0)
#else
#define HQ_MARK_T(i, tid) \
  do {                    \
  } while (0)
#define HQ_MARK(i) \
  do {             \
  } while (0)
#endif

// ---------------------------------------------------------------- Encaps / re-encryption
// One workgroup per handshake.  (Persistent workgroups that prefetch the next handshake's global
// reads were slower, HQC-128 enc_mul 0.886 vs 0.761 ms, profiles/r2/ab_hqc_persist_rejected.jsonl:
// with 8 workgroups per CU the fresh workgroups' load phases already overlap the resident ones'
// work.)  The handshake's global reads are issued before any of them is used (enc_issue), so
// they are one round trip.

// word j of a byte string at any alignment, split in two halves: issue() starts the one or two
// aligned dword loads (no use of the data), finish() combines them -- ld32_masked across a gap
struct Ld32 {
  uint32_t w0, w1;
};
__device__ __forceinline__ Ld32 ld32_issue(const uint8_t* src, int j, int nbytes) {
  const uintptr_t a = (uintptr_t)src + 4 * (uintptr_t)j;
  const uint32_t* b = (const uint32_t*)(a & ~(uintptr_t)3);
  const uint32_t sh = (uint32_t)(a & 3) * 8;
  const int valid = nbytes - 4 * j;
  Ld32 r;
  r.w0 = b[0];
  r.w1 = (sh != 0 && valid > 4 - (int)(sh >> 3)) ? b[1] : 0u;
  return r;
}
__device__ __forceinline__ uint32_t ld32_finish(Ld32 r, uint32_t sh, int j, int nbytes) {
  const int valid = nbytes - 4 * j;
  const uint32_t w = sh ? alignbit(r.w1, r.w0, sh) : r.w0;
  return valid >= 4 ? w : (w & ((1u << (8 * valid)) - 1));
}

// one handshake's global reads for k_hqc_enc_mul, held in registers
template <int L, bool REENC>
struct EncIn {
  using P = HQ<L>;
  static constexpr int WA = (P::NW32 + P::TPB - 1) / P::TPB;
  uint32_t h[WA];
  Ld32 sw[WA];
  uint32_t q1, q2, qe, mm, ssh;
};

template <int L, bool REENC>
__device__ __forceinline__ void enc_issue(EncIn<L, REENC>& in, size_t hs, const uint64_t* __restrict__ row,
                                          const uint8_t* __restrict__ coins, const uint8_t* __restrict__ pk,
                                          const uint8_t* __restrict__ mp, const uint8_t* __restrict__ sk) {
  using P = HQ<L>;
  const int t = hq_tid();
  const uint64_t* rw = row + hs * P::ROWW;
  const uint8_t* spk = REENC ? sk + hs * P::SK + SEED + P::K : pk + hs * P::PK;  // the pk
  const uint32_t* h32 = (const uint32_t*)(rw + 2 * P::RWR + P::RWE);
  in.ssh = (uint32_t)(((uintptr_t)spk + SEED) & 3) * 8;
#pragma unroll
  for (int k = 0; k < EncIn<L, REENC>::WA; ++k) {
    const int j = t + k * P::TPB;
    in.h[k] = j < P::NW32 ? h32[j] : 0u;
    in.sw[k] = j < P::NW32 ? ld32_issue(spk + SEED, j, P::NB) : Ld32{0u, 0u};
  }
  const uint32_t* r32 = (const uint32_t*)rw;
  in.q1 = t < P::WR ? r32[t] : 0u;
  in.q2 = t < P::WR ? r32[2 * P::RWR + t] : 0u;
  in.qe = t < P::WE ? r32[4 * P::RWR + t] : 0u;
  in.mm = t < P::K ? (REENC ? mp[hs * 32 + t] : coins[hs * P::ENC + t]) : 0u;
}

// Encaps (REENC = false): m, salt from coins; s from pk; writes ct and the K-hash message rows.
// Decaps re-encryption (REENC = true): m' from mp; s and sigma from sk; compares (u', v') with the
// received ct; message = (m' if equal else sigma) || u || v of the received ct; status -1 if unequal.
// 8 waves per SIMD at HQC-128 as before the loop (<= 64 VGPRs; HQC-192/256 are held to 5 by their
// LDS): without the bound the compiler keeps loop-invariant values live across the handshake loop
template <int L, bool REENC>
__global__ __launch_bounds__(HQ<L>::TPB) __attribute__((amdgpu_waves_per_eu(L == 192 ? 7 : 8))) void k_hqc_enc_mul(size_t n, const uint64_t* __restrict__ row,
                                                     const uint8_t* __restrict__ coins, const uint8_t* __restrict__ pk,
                                                     uint8_t* __restrict__ ct_out, const uint8_t* __restrict__ mp,
                                                     const uint8_t* __restrict__ sk, const uint8_t* __restrict__ ct_in,
                                                     int32_t* __restrict__ status, uint64_t* __restrict__ msg) {
  using P = HQ<L>;
  // NOMB: the message is assembled over u (D1) once u has been read out (HQC-128 is wave-limited,
  // not LDS-limited, and keeps the separate buffer: the in-place path costs it a spill at 64 VGPRs)
  constexpr bool NOMB = L != 128;
  __shared__ __attribute__((aligned(16))) uint32_t D1[P::NH2];
  __shared__ uint32_t D2[P::NH2];
  __shared__ __attribute__((aligned(16))) uint32_t MBX[NOMB ? 4 : P::MBW];
  uint32_t* const MB = NOMB ? D1 : MBX;
  static_assert(!NOMB || (2 * P::MW <= P::NH2 && P::K / 4 + (P::NB + P::VB + 3) / 4 <= P::NH2), "message fits D1");
  static_assert(NOMB || 2 * P::NW32 <= P::MBW, "raw h and s words fit the message buffer");
  __shared__ uint32_t SS[3 * P::WMAX];
  uint32_t* const S1 = SS;
  uint32_t* const S2 = SS + P::WMAX;
  uint32_t* const SE = SS + 2 * P::WMAX;
  static_assert(P::WR == P::WE, "one dedupe over r1, r2, e");
  __shared__ __attribute__((aligned(4))) uint8_t GE[512], GL[256];
  __shared__ uint8_t SYM[128], MM[32];
  __shared__ uint32_t DIFF;
  size_t hs = blockIdx.x;
  if (hs >= n) return;
  uint8_t* mb = (uint8_t*)MB;
  const int t0 = threadIdx.x;
  if (t0 < 128) ((uint32_t*)GE)[t0] = ((const uint32_t*)GF.exp)[t0];
  if (t0 < 64) ((uint32_t*)GL)[t0] = ((const uint32_t*)GF.log)[t0];
  const size_t hstep = n;  // one handshake per workgroup: the loop body runs once
  EncIn<L, REENC> in;
  enc_issue<L, REENC>(in, hs, row, coins, pk, mp, sk);
#pragma unroll 1
  for (; hs < n; hs += hstep) {
    const int t = hq_tid(), wave = t >> 6, lane = t & 63;
    HQ_MARK(0 + 8 * REENC);
    // phase A: this handshake's reads (issued one iteration earlier) into LDS
#pragma unroll
    for (int k = 0; k < EncIn<L, REENC>::WA; ++k) {
      const int j = t + k * P::TPB;
      if (j < P::NW32) {
        uint32_t* const dst = NOMB ? D2 : MB;  // raw s, then raw h
        dst[j] = ld32_finish(in.sw[k], in.ssh, j, P::NB);
        (NOMB ? D1 : MB + P::NW32)[j] = j == P::NW32 - 1 ? in.h[k] & ((1u << P::NR) - 1) : in.h[k];
      }
    }
    if (t < P::WR) S1[t] = (uint32_t)t + __umulhi(in.q1, (uint32_t)(P::N - t));
    if (t < P::WR) S2[t] = (uint32_t)t + __umulhi(in.q2, (uint32_t)(P::N - t));
    if (t < P::WE) SE[t] = (uint32_t)t + __umulhi(in.qe, (uint32_t)(P::N - t));
    if (t < P::K) MM[t] = (uint8_t)in.mm;
    if (t == 0) DIFF = 0;
    __syncthreads();
    HQ_MARK(1 + 8 * REENC);
    // phase B: RS parity (wave 3), the three duplicate removals on waves 0-2
    if constexpr (NOMB) {
      build_doubled2_inplace<L>(D1, D2);
    } else {
      build_doubled<L>(D1, [&](int j) { return MB[P::NW32 + j]; });
      build_doubled<L>(D2, [&](int j) { return MB[j]; });
    }
    HQ_MARK_T(24 + 4 * REENC, 0);
    if (wave == 0) dedupe_wave<P::WR>(S1);
    HQ_MARK_T(25 + 4 * REENC, 0);
    if (wave == 1) dedupe_wave<P::WR>(S2);
    if (wave == 2) dedupe_wave<P::WE>(SE);
    if (wave == 3) {
      const RsTab<L>& rs = rs_tab<L>();
      if (lane < P::T2) {
        uint32_t par = 0;
#pragma unroll
        for (int i = 0; i < P::K; ++i) {
          const uint32_t mi = MM[i], lp = rs.lp[i][lane];
          const uint32_t pr = GE[GL[mi] + lp];
          par ^= (mi != 0 && lp != 255) ? pr : 0u;
        }
        SYM[lane] = (uint8_t)par;
      } else if (lane < P::T2 + P::K) {
        SYM[lane] = MM[lane - P::T2];
      }
      if (lane + 64 < P::N1) SYM[lane + 64] = MM[lane + 64 - P::T2];
    }
    HQ_MARK_T(26 + 4 * REENC, 192);
    __syncthreads();
    HQ_MARK(2 + 8 * REENC);
    // phase C: u = r2 h, v = r2 s (before r1 / e / codeword)
    uint32_t acc[2][P::WPTE] = {};
    const uint32_t* const Ds[2] = {D1, D2};
    sparse_dense<L, 2, P::WPTE, P::NBTE>(S2, P::WR, Ds, acc);
    HQ_MARK(3 + 8 * REENC);
    __syncthreads();
    HQ_MARK(4 + 8 * REENC);
    uint32_t* const outs[2] = {D1, D2};
    prod_combine<2, P::WPTE, P::NBTE>(outs, acc, [&] {
      for (int i = t; i < P::WR; i += P::TPB) atomicXor(&D1[S1[i] >> 5], 1u << (S1[i] & 31));
      for (int i = t; i < P::WE; i += P::TPB) atomicXor(&D2[SE[i] >> 5], 1u << (SE[i] & 31));
    });
    HQ_MARK(5 + 8 * REENC);
    constexpr uint32_t TOPMASK = (1u << P::NR) - 1;
    constexpr int UOFF = P::K / 4;  // u at message byte K
    auto vword = [&](int j) {       // v word j = (r2 s + e + codeword) word j
      const int sym = j / (4 * P::MULT);
      return D2[j] ^ rm_word(SYM[sym], j & 3);
    };
    // NOMB: u (in D1) out to registers before the message is built over it
    constexpr int UPT = (P::NW32 + P::TPB - 1) / P::TPB;
    uint32_t uw[UPT];
    if constexpr (NOMB) {
#pragma unroll
      for (int k = 0; k < UPT; ++k) {
        const int j = t + k * P::TPB;
        uw[k] = j < P::NW32 ? (j == P::NW32 - 1 ? (D1[j] & TOPMASK) : D1[j]) : 0u;
      }
      __syncthreads();
    }
    if constexpr (!REENC) {
      if constexpr (NOMB) {
#pragma unroll
        for (int k = 0; k < UPT; ++k) {
          const int j = t + k * P::TPB;
          if (j < P::NW32) MB[UOFF + j] = uw[k];
        }
      } else {
        for (int j = t; j < P::NW32; j += P::TPB) MB[UOFF + j] = j == P::NW32 - 1 ? (D1[j] & TOPMASK) : D1[j];
      }
      if (t < P::K) mb[t] = MM[t];
      __syncthreads();  // the last u word's spare bytes are v's first bytes
      for (int j = t; j < P::VW32; j += P::TPB) lds_store_u32_unaligned(mb, P::K + P::NB + 4 * j, vword(j));
    } else {
      // received u || v into the message area, then compare with the re-encryption
      const uint8_t* cin = ct_in + hs * P::CT;
      static_assert(P::K % 4 == 0, "u || v starts on a word");
      for (int j = t; j < (P::NB + P::VB + 3) / 4; j += P::TPB) MB[P::K / 4 + j] = ld32_masked(cin, j, P::NB + P::VB);
      __syncthreads();
      uint32_t diff = 0;
      constexpr int VALID = P::NB - 4 * (P::NW32 - 1);  // bytes of the last word that belong to u
      constexpr uint32_t BM = VALID >= 4 ? 0xFFFFFFFFu : ((1u << (8 * VALID)) - 1);
      if constexpr (NOMB) {
#pragma unroll
        for (int k = 0; k < UPT; ++k) {
          const int j = t + k * P::TPB;
          if (j < P::NW32) diff |= uw[k] ^ (j == P::NW32 - 1 ? MB[UOFF + j] & BM : MB[UOFF + j]);
        }
      } else {
        for (int j = t; j < P::NW32; j += P::TPB) {
          uint32_t u = D1[j], c = MB[UOFF + j];
          if (j == P::NW32 - 1) {
            u &= TOPMASK;
            c &= BM;
          }
          diff |= u ^ c;
        }
      }
      for (int j = t; j < P::VW32; j += P::TPB) diff |= vword(j) ^ lds_u32_unaligned(mb, P::K + P::NB + 4 * j);
      if (diff) atomicOr(&DIFF, 1u);
      __syncthreads();
      const bool ok = DIFF == 0;
      if (t < P::K) mb[t] = ok ? MM[t] : sk[hs * P::SK + SEED + t];
      if (t == 0) status[hs] = ok ? 0 : -1;
    }
    for (int b = P::MSGB + t; b < 8 * P::MW; b += P::TPB) mb[b] = b == P::MSGB ? 0x05 : (b == P::MSGB + 1 ? 0x1F : 0);
    __syncthreads();
    HQ_MARK(6 + 8 * REENC);
    // phase E: K-hash message rows (aligned words), ciphertext bytes
    const uint64_t* m64 = (const uint64_t*)MB;
    uint64_t* mo = msg + hs * P::MW;
    for (int w = t; w < P::MW; w += P::TPB) mo[w] = m64[w];
    if constexpr (!REENC) {
      uint8_t* co = ct_out + hs * P::CT;
#pragma unroll 8
      for (int b = t; b < P::NB + P::VB; b += P::TPB) co[b] = mb[P::K + b];
      if (t < SALT) co[P::NB + P::VB + t] = coins[hs * P::ENC + P::K + t];
    }
    HQ_MARK(7 + 8 * REENC);
    __syncthreads();  // the next iteration's staging overwrites MB, SS, MM
  }
}

// Hadamard butterfly on lane bit BIT for two symbols (x0 / x1 = positions l / l + 64):
// x = hi ? partner - x : x + partner, partner = the value of lane l ^ (1 << BIT).
// Partners without LDS: quad_perm DPP (bits 0, 1), row_shl/row_shr:4 under bank masks (bit 2),
// row_ror:8 (bit 3), v_permlane16_swap / v_permlane32_swap (bits 4, 5).  All lanes active.
template <int BIT>
__device__ __forceinline__ int lane_partner(int x, int lane) {
  if constexpr (BIT == 0) {
    return __builtin_amdgcn_update_dpp(0, x, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
  } else if constexpr (BIT == 1) {
    return __builtin_amdgcn_update_dpp(0, x, 0x4E, 0xF, 0xF, false);  // quad_perm [2,3,0,1]
  } else if constexpr (BIT == 2) {
    const int p = __builtin_amdgcn_update_dpp(x, x, 0x104, 0xF, 0x5, false);  // banks 0, 2: lane + 4
    return __builtin_amdgcn_update_dpp(p, x, 0x114, 0xF, 0xA, false);         // banks 1, 3: lane - 4
  } else if constexpr (BIT == 3) {
    return __builtin_amdgcn_update_dpp(0, x, 0x128, 0xF, 0xF, false);  // row_ror:8
  } else if constexpr (BIT == 4) {
    const auto r = __builtin_amdgcn_permlane16_swap((unsigned)x, (unsigned)x, false, false);
    return (int)(((lane >> 4) & 1) ? r[0] : r[1]);
  } else {
    const auto r = __builtin_amdgcn_permlane32_swap((unsigned)x, (unsigned)x, false, false);
    return (int)((lane >> 5) ? r[0] : r[1]);
  }
}
template <int BIT>
__device__ __forceinline__ void butterflies(int (&x0)[2], int (&x1)[2], int lane) {
  const bool hi = (lane >> BIT) & 1;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int p0 = lane_partner<BIT>(x0[u], lane), p1 = lane_partner<BIT>(x1[u], lane);
    x0[u] = hi ? p0 - x0[u] : x0[u] + p0;
    x1[u] = hi ? p1 - x1[u] : x1[u] + p1;
  }
}
// wave-uniform maximum (all lanes active): DPP within rows, then the four rows by v_readlane
__device__ __forceinline__ uint32_t max_wave(uint32_t k) {
  auto mx = [](uint32_t a, int b) { return a > (uint32_t)b ? a : (uint32_t)b; };
  k = mx(k, __builtin_amdgcn_update_dpp(0, (int)k, 0xB1, 0xF, 0xF, false));
  k = mx(k, __builtin_amdgcn_update_dpp(0, (int)k, 0x4E, 0xF, 0xF, false));
  k = mx(k, __builtin_amdgcn_update_dpp(0, (int)k, 0x141, 0xF, 0xF, false));  // row_half_mirror
  k = mx(k, __builtin_amdgcn_update_dpp(0, (int)k, 0x140, 0xF, 0xF, false));  // row_mirror
  const uint32_t a = (uint32_t)__builtin_amdgcn_readlane((int)k, 0), b = (uint32_t)__builtin_amdgcn_readlane((int)k, 16);
  const uint32_t c = (uint32_t)__builtin_amdgcn_readlane((int)k, 32), d = (uint32_t)__builtin_amdgcn_readlane((int)k, 48);
  const uint32_t ab = a > b ? a : b, cd = c > d ? c : d;
  return ab > cd ? ab : cd;
}

// ---------------------------------------------------------------- Decaps: m' = C.decode(v - u y)
// The combined product T reuses the u || v staging buffer (v is folded into the partial sums before
// the combine): one barrier more and NWP words less LDS per workgroup
template <int L>
__global__ __launch_bounds__(HQ<L>::TPB) __attribute__((amdgpu_waves_per_eu(L == 192 ? 8 : 1))) void k_hqc_decode(size_t n, const uint64_t* __restrict__ row,
                                                    const uint8_t* __restrict__ ct, uint8_t* __restrict__ syms,
                                                    size_t sym_stride) {
  using P = HQ<L>;
  __shared__ uint32_t D1[P::NH2];
  constexpr int MBD = (P::NB + P::VB + 8) / 4 + 1;
  __shared__ uint32_t MB[MBD > P::NWP ? MBD : P::NWP];
  uint32_t* const T = MB;
  __shared__ uint32_t SY[P::WMAX];
  __shared__ uint8_t SYM[128];
  const size_t hs = blockIdx.x;
  if (hs >= n) return;
  const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
  const uint64_t* rw = row + hs * P::ROWW;
  uint8_t* mb = (uint8_t*)MB;
  const uint8_t* c = ct + hs * P::CT;
  HQ_MARK(16);
  // u doubled straight from the ct's u words (bits >= n as received; the word straddling into v is
  // cut), u || v bytes staged, supports -- all of the handshake's global reads before the barrier
  constexpr int VALID = P::NB - 4 * (P::NW32 - 1);
  constexpr uint32_t BM = VALID >= 4 ? 0xFFFFFFFFu : ((1u << (8 * VALID)) - 1);
  for (int j = t; j < (P::NB + P::VB + 3) / 4; j += P::TPB) MB[j] = ld32_masked(c, j, P::NB + P::VB);
  supports_raw<L>(rw + P::RWW, P::W, SY);
  __syncthreads();
  build_doubled<L>(D1, [&](int j) { return j == P::NW32 - 1 ? (MB[j] & BM) : MB[j]; });
  HQ_MARK(17);
  if (wave == 0) dedupe_wave<P::W>(SY);
  __syncthreads();
  HQ_MARK(18);
  uint32_t acc[1][P::WPT] = {};
  const uint32_t* const Ds[1] = {D1};
  sparse_dense<L, 1, P::WPT, P::NBT>(SY, P::W, Ds, acc);
  HQ_MARK(19);
  // T = v - u y (words >= VW32 zero): fold v into class 0's partial sums, then combine
  if (t < P::NBT) {
    const int j0 = t * P::WPT;
#pragma unroll
    for (int q = 0; q < P::WPT; ++q) {
      const int j = j0 + q;
      acc[0][q] = j < P::VW32 ? acc[0][q] ^ lds_u32_unaligned(mb, P::NB + 4 * j) : 0u;
    }
  } else {
    const int j0 = (t % P::NBT) * P::WPT;
#pragma unroll
    for (int q = 0; q < P::WPT; ++q) acc[0][q] = j0 + q < P::VW32 ? acc[0][q] : 0u;
  }
  __syncthreads();  // every v read done before T overwrites it
  uint32_t* const outs[1] = {T};
  prod_combine<1, P::WPT, P::NBT>(outs, acc, [] {});
  HQ_MARK(20);
  // duplicated RM(1,7): one wave per symbol pair (two independent chains interleave), lane l
  // holds positions l and l + 64 of each symbol; the Hadamard butterflies exchange through DPP
  // and v_permlane16/32_swap (no LDS round trips), the first maximum is a DPP + readlane max
  constexpr int NWAVE = P::TPB / 64;
  for (int base = wave; base < P::N1; base += 2 * NWAVE) {
    const int sy[2] = {base, base + NWAVE < P::N1 ? base + NWAVE : base};
    int x0[2], x1[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const uint32_t* cw = T + sy[u] * 4 * P::MULT;
      x0[u] = 0;
      x1[u] = 0;
#pragma unroll
      for (int cp = 0; cp < P::MULT; ++cp) {
        x0[u] += (int)(cw[4 * cp + (lane >> 5)] >> (lane & 31) & 1);
        x1[u] += (int)(cw[4 * cp + 2 + (lane >> 5)] >> (lane & 31) & 1);
      }
      const int a0 = x0[u], b0 = x1[u];
      x0[u] = a0 + b0;
      x1[u] = a0 - b0;
    }
    butterflies<0>(x0, x1, lane);
    butterflies<1>(x0, x1, lane);
    butterflies<2>(x0, x1, lane);
    butterflies<3>(x0, x1, lane);
    butterflies<4>(x0, x1, lane);
    butterflies<5>(x0, x1, lane);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      if (lane == 0) x0[u] -= 64 * P::MULT;
      // first maximum of |value| (lowest index), sign -> bit 7
      const uint32_t k0 = ((uint32_t)abs(x0[u]) << 8) | ((uint32_t)(127 - lane) << 1) | (x0[u] > 0 ? 1u : 0u);
      const uint32_t k1 = ((uint32_t)abs(x1[u]) << 8) | ((uint32_t)(63 - lane) << 1) | (x1[u] > 0 ? 1u : 0u);
      const uint32_t k = max_wave(k0 > k1 ? k0 : k1);
      if (lane == 0) SYM[sy[u]] = (uint8_t)((127 - ((k >> 1) & 127)) | ((k & 1) << 7));
    }
  }
  __syncthreads();
  HQ_MARK(21);
  if (t < P::N1) syms[hs * sym_stride + t] = SYM[t];
  HQ_MARK(22);
}

// wave-scope LDS ordering (the wave's lanes exchange through LDS)
__device__ __forceinline__ void wsync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// XOR over the 64 lanes (all active), wave-uniform result: DPP within each 16-lane row
// (quad swaps, half-row and row mirrors), then the four row values by v_readlane.
__device__ __forceinline__ uint32_t xor_wave(uint32_t d) {
  d ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)d, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
  d ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)d, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
  d ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)d, 0x141, 0xF, 0xF, false);  // row_half_mirror
  d ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)d, 0x140, 0xF, 0xF, false);  // row_mirror
  return (uint32_t)(__builtin_amdgcn_readlane((int)d, 0) ^ __builtin_amdgcn_readlane((int)d, 16) ^
                    __builtin_amdgcn_readlane((int)d, 32) ^ __builtin_amdgcn_readlane((int)d, 48));
}

// ---------------------------------------------------------------- Decaps: Reed-Solomon decoding
// One wave per handshake, 4 per workgroup (GF(2^8) exp/log tables shared in LDS).  Bounded-distance
// decoding as the spec: syndromes S_1..S_2delta, Berlekamp-Massey, Omega = S C mod x^(2 delta),
// Chien search + Forney over the n1 positions; the corrected message symbols are m'.  Every sum
// is taken in the log domain over independent table lookups (no dependent multiply chains);
// zero is log 255.
template <int L>
__global__ __launch_bounds__(256) void k_hqc_rs(size_t n, const uint8_t* __restrict__ syms, size_t sym_stride,
                                                uint8_t* __restrict__ mp) {
  using P = HQ<L>;
  constexpr uint32_t Z = 255;
  __shared__ uint8_t GE[512], GL[256];
  __shared__ uint8_t SYMW[4][128], LSW[4][128], LSYNW[4][64], CLW[4][64], LCLW[4][64], LOMW[4][64];
  fill_gf(GE, GL);
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const size_t hs = (size_t)blockIdx.x * 4 + wave;
  if (hs >= n) return;
  uint8_t *SYM = SYMW[wave], *LS = LSW[wave], *LSYN = LSYNW[wave], *CL = CLW[wave], *LCL = LCLW[wave],
          *LOM = LOMW[wave];
  auto lg = [&](uint32_t a) { return a ? (uint32_t)GL[a] : Z; };
  auto mod255 = [](uint32_t x) { return x >= 255 ? x - 255 : x; };
  for (int j = lane; j < P::N1; j += 64) {
    const uint32_t r = syms[hs * sym_stride + j];
    SYM[j] = (uint8_t)r;
    LS[j] = (uint8_t)lg(r);
  }
  wsync();
  // syndromes S_{i+1} = sum_j r_j alpha^((i+1) j), lane i
  if (lane < P::T2) {
    uint32_t s = 0, e = 0;
    const uint32_t step = (uint32_t)(lane + 1);
#pragma unroll 16
    for (int j = 0; j < P::N1; ++j) {
      const uint32_t l = LS[j];
      s ^= l != Z ? (uint32_t)GE[l + e] : 0u;
      e = mod255(e + step);
    }
    LSYN[lane] = (uint8_t)lg(s);
  }
  wsync();
  // Berlekamp-Massey: lane j holds C_j and log B_j; the discrepancy is wave-uniform
  uint32_t Cj = lane == 0 ? 1u : 0u, LBj = lane == 0 ? 0u : Z, lb = 0;
  int Lr = 0, m = 1;
  for (int i = 0; i < P::T2; ++i) {
    const uint32_t lbsh = (uint32_t)__shfl((int)LBj, lane - m >= 0 ? lane - m : 0);
    const uint32_t lc = lg(Cj);
    const uint32_t ls = lane <= i ? (uint32_t)LSYN[i - lane] : Z;
    const uint32_t term = (lane <= Lr && lc != Z && ls != Z) ? (uint32_t)GE[lc + ls] : 0u;
    const uint32_t d = xor_wave(term);
    if (d != 0) {
      const uint32_t ld = GL[d];
      const uint32_t lcoef = mod255(ld + 255 - lb);
      const uint32_t cn = Cj ^ ((lane >= m && lbsh != Z) ? (uint32_t)GE[lcoef + lbsh] : 0u);
      if (2 * Lr <= i) {
        LBj = lc;
        lb = ld;
        Lr = i + 1 - Lr;
        m = 1;
      } else {
        ++m;
      }
      Cj = cn;
    } else {
      ++m;
    }
  }
  if (lane <= P::T2) {
    CL[lane] = (uint8_t)Cj;
    LCL[lane] = (uint8_t)lg(Cj);
  }
  wsync();
  // Omega_i = sum_{j <= i} S_{i-j+1} C_j, i < 2 delta
  if (lane < P::T2) {
    uint32_t o = 0;
#pragma unroll 8
    for (int j = 0; j < P::T2; ++j) {
      const uint32_t ls = j <= lane ? (uint32_t)LSYN[lane - j] : Z, lc = LCL[j];
      o ^= (ls != Z && lc != Z) ? (uint32_t)GE[ls + lc] : 0u;
    }
    LOM[lane] = (uint8_t)lg(o);
  }
  wsync();
  // Chien search + Forney, lane per position: x = alpha^(-pos);
  // C(x), C'(x) = sum_{i even} C_{i+1} x^i, Omega(x); error value Omega(x) / C'(x) where C(x) = 0
  for (int pos = lane; pos < P::N1; pos += 64) {
    const uint32_t lx = (uint32_t)((255 - pos) % 255);
    uint32_t cv = CL[0], dv = 0, ov = 0, e = 0;  // e = log x^i
#pragma unroll 8
    for (int i = 0; i < P::T2; ++i) {
      const uint32_t lo = LOM[i], ld = (i & 1) == 0 ? (uint32_t)LCL[i + 1] : Z, lc1 = LCL[i + 1];
      const uint32_t e1 = mod255(e + lx);  // log x^(i+1)
      ov ^= lo != Z ? (uint32_t)GE[lo + e] : 0u;
      dv ^= ld != Z ? (uint32_t)GE[ld + e] : 0u;
      cv ^= lc1 != Z ? (uint32_t)GE[lc1 + e1] : 0u;
      e = e1;
    }
    const uint32_t fix = (cv == 0 && dv != 0 && ov != 0) ? (uint32_t)GE[GL[ov] + 255 - GL[dv]] : 0u;
    SYM[pos] ^= (uint8_t)fix;
  }
  wsync();
  if (lane < P::K) mp[hs * 32 + lane] = SYM[P::T2 + lane];
}

// ---------------------------------------------------------------- fixed-weight supports alone
// (test hook behind qrk_hqc_supports: r words -> deduplicated supports, one workgroup per vector)
template <int L, int WT>
__global__ __launch_bounds__(HQ<L>::TPB) void k_hqc_supports(size_t n, const uint32_t* __restrict__ r,
                                                      uint32_t* __restrict__ sup) {
  using P = HQ<L>;
  __shared__ uint32_t SS[P::WMAX];
  const size_t v = blockIdx.x;
  if (v >= n) return;
  for (int i = threadIdx.x; i < WT; i += P::TPB) SS[i] = (uint32_t)i + __umulhi(r[v * WT + i], (uint32_t)(P::N - i));
  __syncthreads();
  if (threadIdx.x < 64) dedupe_wave<WT>(SS);  // the product kernels' duplicate removal
  __syncthreads();
  for (int i = threadIdx.x; i < WT; i += P::TPB) sup[v * WT + i] = SS[i];
}

template <int L>
hipError_t supports_t(int kind, size_t n, const uint32_t* r, uint32_t* sup, hipStream_t st) {
  using P = HQ<L>;
  if (kind == 0)
    QRK_LAUNCH("k_hqc_supports", st, (k_hqc_supports<L, P::W>), dim3((unsigned)n), dim3(P::TPB), 0, st, n, r, sup);
  else
    QRK_LAUNCH("k_hqc_supports", st, (k_hqc_supports<L, P::WR>), dim3((unsigned)n), dim3(P::TPB), 0, st, n, r, sup);
  return hipGetLastError();
}

// ---------------------------------------------------------------- launchers
inline unsigned blocks_for(size_t t) { return (unsigned)((t + 255) / 256); }
inline size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }
template <int L>
void launch_enc_expand(const uint8_t* m, size_t m_stride, const uint8_t* pk, size_t pk_stride, const uint8_t* salt,
                       size_t salt_stride, size_t n, uint64_t* row, hipStream_t st) {
  if (n <= QRK_HQC_COOP_MAX) {
    QRK_LAUNCH("k_hqc_enc_expand", st, k_hqc_enc_expand_c<L>, dim3((unsigned)(2 * n)), dim3(64), 0, st, m, m_stride, pk,
               pk_stride, salt, salt_stride, n, row);
  } else {
    const size_t C64 = (n + 63) & ~(size_t)63;
    QRK_LAUNCH("k_hqc_enc_expand", st, k_hqc_enc_expand<L>, dim3(blocks_for(2 * C64)), dim3(256), 0, st, m, m_stride,
               pk, pk_stride, salt, salt_stride, n, C64, row);
  }
}
template <int L>
void launch_hash(const uint64_t* msg, size_t n, uint8_t* ss, hipStream_t st) {
  if (n <= QRK_HQC_COOP_MAX)
    QRK_LAUNCH("k_hqc_hash", st, k_hqc_hash_c<L>, dim3((unsigned)n), dim3(64), 0, st, msg, n, ss);
  else
    QRK_LAUNCH("k_hqc_hash", st, k_hqc_hash<L>, dim3(blocks_for(n)), dim3(256), 0, st, msg, n, ss);
}

template <int L>
size_t scratch_t(size_t C) {
  using P = HQ<L>;
  return al256(C * P::ROWW * 8) + al256(C * P::MW * 8) + al256(C * 32) + al256(C * 4);
}
struct View {
  uint64_t* row;
  uint64_t* msg;
  uint8_t* mp;
  int32_t* st;
};
template <int L>
View carve(void* base, size_t C) {
  using P = HQ<L>;
  uint8_t* p = (uint8_t*)base;
  View v;
  v.row = (uint64_t*)p;
  p += al256(C * P::ROWW * 8);
  v.msg = (uint64_t*)p;
  p += al256(C * P::MW * 8);
  v.mp = p;
  p += al256(C * 32);
  v.st = (int32_t*)p;
  return v;
}

template <int L>
hipError_t keypair_t(size_t n, uint8_t* pk, uint8_t* sk, const uint8_t* coins, void* scratch, hipStream_t st) {
  View v = carve<L>(scratch, n);
  if (n <= QRK_HQC_COOP_MAX)
    QRK_LAUNCH("k_hqc_kg_expand", st, k_hqc_kg_expand_c<L>, dim3((unsigned)(2 * n)), dim3(64), 0, st, coins, n, v.row);
  else
    QRK_LAUNCH("k_hqc_kg_expand", st, k_hqc_kg_expand<L>, dim3(blocks_for(n)), dim3(256), 0, st, coins, n, v.row);
  QRK_LAUNCH("k_hqc_kg_mul", st, k_hqc_kg_mul<L>, dim3((unsigned)n), dim3(HQ<L>::TPB), 0, st, n, v.row, coins, pk, sk);
  return hipGetLastError();
}

template <int L>
hipError_t encaps_t(size_t n, uint8_t* ct, uint8_t* ss, const uint8_t* pk, const uint8_t* coins, void* scratch,
                    hipStream_t st) {
  using P = HQ<L>;
  View v = carve<L>(scratch, n);
  launch_enc_expand<L>(coins, (size_t)P::ENC, pk, (size_t)P::PK, coins + P::K, (size_t)P::ENC, n, v.row, st);
  QRK_LAUNCH("k_hqc_enc_mul", st, (k_hqc_enc_mul<L, false>), dim3((unsigned)n), dim3(P::TPB), 0, st, n, v.row, coins,
             pk, ct, (const uint8_t*)nullptr, (const uint8_t*)nullptr, (const uint8_t*)nullptr, (int32_t*)nullptr,
             v.msg);
  launch_hash<L>(v.msg, n, ss, st);
  return hipGetLastError();
}

template <int L>
hipError_t decaps_t(size_t n, uint8_t* ss, const uint8_t* ct, const uint8_t* sk, int32_t* status, void* scratch,
                    hipStream_t st) {
  using P = HQ<L>;
  View v = carve<L>(scratch, n);
  int32_t* stp = status ? status : v.st;
  if (n <= QRK_HQC_COOP_MAX)
    QRK_LAUNCH("k_hqc_dec_expand", st, k_hqc_dec_expand_c<L>, dim3((unsigned)n), dim3(64), 0, st, sk, n, v.row);
  else
    QRK_LAUNCH("k_hqc_dec_expand", st, k_hqc_dec_expand<L>, dim3(blocks_for(n)), dim3(256), 0, st, sk, n, v.row);
  // the RM stage's symbols go through the K-hash message area, which is free until the re-encryption
  uint8_t* syms = (uint8_t*)v.msg;
  QRK_LAUNCH("k_hqc_decode", st, k_hqc_decode<L>, dim3((unsigned)n), dim3(P::TPB), 0, st, n, v.row, ct, syms,
             (size_t)P::MW * 8);
  QRK_LAUNCH("k_hqc_rs", st, k_hqc_rs<L>, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, st, n, (const uint8_t*)syms,
             (size_t)P::MW * 8, v.mp);
  launch_enc_expand<L>(v.mp, (size_t)32, sk + SEED + P::K, (size_t)P::SK, ct + P::NB + P::VB, (size_t)P::CT, n, v.row,
                       st);
  QRK_LAUNCH("k_hqc_enc_mul", st, (k_hqc_enc_mul<L, true>), dim3((unsigned)n), dim3(P::TPB), 0, st, n, v.row,
             (const uint8_t*)nullptr, (const uint8_t*)nullptr, (uint8_t*)nullptr, v.mp, sk, ct, stp, v.msg);
  launch_hash<L>(v.msg, n, ss, st);
  return hipGetLastError();
}

template <int L>
hipError_t cleanse_t(size_t n, void* scratch, hipStream_t st) {
  const View v = carve<L>(scratch, n);
  return hipMemsetAsync(v.msg, 0, (size_t)((uint8_t*)v.st - (uint8_t*)v.msg), st);  // msg | m'
}

}  // namespace hqc

hipError_t hqc_cleanse(const AlgInfo& a, size_t n, void* scratch, hipStream_t st) {
  if (n == 0) return hipSuccess;
  switch (a.k) {
    case 128: return hqc::cleanse_t<128>(n, scratch, st);
    case 192: return hqc::cleanse_t<192>(n, scratch, st);
    case 256: return hqc::cleanse_t<256>(n, scratch, st);
  }
  return hipErrorInvalidValue;
}

size_t hqc_scratch_bytes(const AlgInfo& a, size_t chunk) {
  switch (a.k) {
    case 128: return hqc::scratch_t<128>(chunk);
    case 192: return hqc::scratch_t<192>(chunk);
    default: return hqc::scratch_t<256>(chunk);
  }
}

hipError_t hqc_keypair(const AlgInfo& a, size_t n, uint8_t* pk, uint8_t* sk, const uint8_t* coins, void* scratch,
                       const Streams& s) {
  if (n == 0) return hipSuccess;
  switch (a.k) {
    case 128: return hqc::keypair_t<128>(n, pk, sk, coins, scratch, s.main);
    case 192: return hqc::keypair_t<192>(n, pk, sk, coins, scratch, s.main);
    case 256: return hqc::keypair_t<256>(n, pk, sk, coins, scratch, s.main);
  }
  return hipErrorInvalidValue;
}

hipError_t hqc_encaps(const AlgInfo& a, size_t n, uint8_t* ct, uint8_t* ss, const uint8_t* pk, const uint8_t* coins,
                      void* scratch, const Streams& s) {
  if (n == 0) return hipSuccess;
  switch (a.k) {
    case 128: return hqc::encaps_t<128>(n, ct, ss, pk, coins, scratch, s.main);
    case 192: return hqc::encaps_t<192>(n, ct, ss, pk, coins, scratch, s.main);
    case 256: return hqc::encaps_t<256>(n, ct, ss, pk, coins, scratch, s.main);
  }
  return hipErrorInvalidValue;
}

hipError_t hqc_supports(const AlgInfo& a, int kind, size_t n, const uint32_t* r, uint32_t* sup, hipStream_t st) {
  if (n == 0) return hipSuccess;
  switch (a.k) {
    case 128: return hqc::supports_t<128>(kind, n, r, sup, st);
    case 192: return hqc::supports_t<192>(kind, n, r, sup, st);
    case 256: return hqc::supports_t<256>(kind, n, r, sup, st);
  }
  return hipErrorInvalidValue;
}

hipError_t hqc_decaps(const AlgInfo& a, size_t n, uint8_t* ss, const uint8_t* ct, const uint8_t* sk, int32_t* status,
                      void* scratch, const Streams& s) {
  if (n == 0) return hipSuccess;
  switch (a.k) {
    case 128: return hqc::decaps_t<128>(n, ss, ct, sk, status, scratch, s.main);
    case 192: return hqc::decaps_t<192>(n, ss, ct, sk, status, scratch, s.main);
    case 256: return hqc::decaps_t<256>(n, ss, ct, sk, status, scratch, s.main);
  }
  return hipErrorInvalidValue;
}

}  // namespace qrk

#if QRK_HQC_TRACE
extern "C" int qrk_dbg_hqc_trace(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(qrk::hqc::g_hqc_trace), sizeof(qrk::hqc::g_hqc_trace)) == hipSuccess ? 0 : -1;
}
#endif
