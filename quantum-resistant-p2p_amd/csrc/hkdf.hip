// HKDF-SHA256 (RFC 5869) over a batch of independent keys, one lane per key, for gfx950.
//
// Replaces, for N handshakes at once, the key derivation the reference runs after
// every key exchange: SecureMessaging._derive_symmetric_key
// (quantum_resistant_p2p/app/messaging.py:350-382), i.e.
//   HKDF(algorithm=SHA256, length=symmetric.key_size, salt=None,
//        info=b"quantum_resistant_p2p-v1-{idA}-{idB}-{sym}").derive(shared_secret)
// called by the responder after Encaps (:845) and the initiator after Decaps (:1068).
//
// SHA-256 (FIPS 180-4) runs in registers: 8 state words + a 16-word rolling message
// schedule per lane; every rotate is one v_alignbit_b32, Ch/Maj are single v_bitop3.
// Per key with L = 32 and a 110-byte info: extract 4 compressions (ipad/opad blocks,
// IKM block, outer block), expand 5 (ipad/opad, two info blocks, outer) -- 9 in all.
// This is a small fraction of a KEM handshake; the kernel is latency-, not VALU-bound
// (its info bytes are gathered with byte loads because every key's info has its own
// length and offset).
#include "qrkem_internal.h"

namespace qrk {
namespace sha {

struct K256T {
  uint32_t k[64];
};
constexpr K256T K256 = {{
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u, 0xab1c5ed5u,
    0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu, 0x9bdc06a7u, 0xc19bf174u,
    0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu, 0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau,
    0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u, 0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u,
    0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu, 0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u,
    0xa2bfe8a1u, 0xa81a664bu, 0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u,
    0x19a4c116u, 0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u, 0xc67178f2u}};

struct H8 {
  uint32_t h[8];
};
__device__ __forceinline__ H8 init() {
  return H8{{0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au, 0x510e527fu, 0x9b05688cu, 0x1f83d9abu,
             0x5be0cd19u}};
}

__device__ __forceinline__ uint32_t rotr(uint32_t x, int n) { return __builtin_amdgcn_alignbit(x, x, n); }

// One SHA-256 compression of the 16 big-endian words w into s.
__device__ __forceinline__ void compress(H8& s, const uint32_t win[16]) {
  uint32_t w[16];
#pragma unroll
  for (int t = 0; t < 16; ++t) w[t] = win[t];
  uint32_t a = s.h[0], b = s.h[1], c = s.h[2], d = s.h[3], e = s.h[4], f = s.h[5], g = s.h[6], h = s.h[7];
#pragma unroll
  for (int t = 0; t < 64; ++t) {
    if (t >= 16) {
      const uint32_t x = w[(t + 1) & 15], y = w[(t + 14) & 15];
      const uint32_t s0 = rotr(x, 7) ^ rotr(x, 18) ^ (x >> 3);
      const uint32_t s1 = rotr(y, 17) ^ rotr(y, 19) ^ (y >> 10);
      w[t & 15] += s0 + w[(t + 9) & 15] + s1;
    }
    const uint32_t S1 = rotr(e, 6) ^ rotr(e, 11) ^ rotr(e, 25);
    const uint32_t ch = (e & f) ^ (~e & g);
    const uint32_t t1 = h + S1 + ch + K256.k[t] + w[t & 15];
    const uint32_t S0 = rotr(a, 2) ^ rotr(a, 13) ^ rotr(a, 22);
    const uint32_t maj = (a & b) ^ (a & c) ^ (b & c);
    h = g;
    g = f;
    f = e;
    e = d + t1;
    d = c;
    c = b;
    b = a;
    a = t1 + S0 + maj;
  }
  s.h[0] += a, s.h[1] += b, s.h[2] += c, s.h[3] += d;
  s.h[4] += e, s.h[5] += f, s.h[6] += g, s.h[7] += h;
}

// Compress the padded tail of a message whose first `prefix` bytes (a multiple of 64)
// are already in s and whose remaining `len` bytes are byte_at(0 .. len-1).
// word_over(b, t, w) may replace word t of tail block b (used for register-held data).
template <class ByteAt, class WordOver>
__device__ __forceinline__ void tail(H8& s, uint32_t prefix, uint32_t len, ByteAt byte_at, WordOver word_over) {
  const uint32_t nblk = (len + 9 + 63) / 64;
  const uint64_t bits = (uint64_t)(prefix + len) * 8;
#pragma unroll 1
  for (uint32_t b = 0; b < nblk; ++b) {
    uint32_t w[16];
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      uint32_t x = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t pos = 64 * b + 4 * t + k;
        const uint32_t v = pos < len ? byte_at(pos) : (pos == len ? 0x80u : 0u);
        x = (x << 8) | v;
      }
      w[t] = word_over(b, t, x);
    }
    if (b == nblk - 1) {
      w[14] = (uint32_t)(bits >> 32);
      w[15] = (uint32_t)bits;
    }
    compress(s, w);
  }
}

__device__ __forceinline__ void pad_state(H8& s, const uint32_t k0[16], uint32_t pad) {
  uint32_t w[16];
#pragma unroll
  for (int t = 0; t < 16; ++t) w[t] = k0[t] ^ pad;
  compress(s, w);
}

// outer HMAC hash: s (after the opad block) absorbs the 32-byte inner digest
__device__ __forceinline__ void outer(H8& s, const H8& inner) {
  uint32_t w[16];
#pragma unroll
  for (int t = 0; t < 8; ++t) w[t] = inner.h[t];
  w[8] = 0x80000000u;
#pragma unroll
  for (int t = 9; t < 15; ++t) w[t] = 0;
  w[15] = (64 + 32) * 8;
  compress(s, w);
}

}  // namespace sha

// okm_i = HKDF-SHA256(salt, ikm_i, info_i, L).  RFC 5869 section 2.2 (extract: PRK = HMAC(salt, IKM),
// salt = HashLen zeros when absent) and 2.3 (expand: T(i) = HMAC(PRK, T(i-1) || info || i)).
__global__ __launch_bounds__(256) void k_hkdf_sha256(size_t n, const uint8_t* __restrict__ ikm, uint32_t ikm_len,
                                                     size_t ikm_stride, const uint8_t* __restrict__ salt,
                                                     uint32_t salt_len, const uint8_t* __restrict__ info,
                                                     const uint64_t* __restrict__ info_off, uint32_t info_len,
                                                     uint32_t L, uint8_t* __restrict__ okm, size_t okm_stride) {
  using namespace sha;
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  auto none = [](uint32_t, int, uint32_t x) { return x; };

  // ---- extract
  uint32_t k0[16];
#pragma unroll
  for (int t = 0; t < 16; ++t) k0[t] = 0;
  if (salt_len > 64) {  // RFC 2104: keys longer than the block are hashed first
    H8 hs = init();
    tail(hs, 0, salt_len, [&](uint32_t p) { return (uint32_t)salt[p]; }, none);
#pragma unroll
    for (int t = 0; t < 8; ++t) k0[t] = hs.h[t];
  } else if (salt_len > 0) {
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      uint32_t x = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t p = 4 * t + k;
        x = (x << 8) | (p < salt_len ? (uint32_t)salt[p] : 0u);
      }
      k0[t] = x;
    }
  }
  const uint8_t* key_in = ikm + i * ikm_stride;
  H8 ih = init();
  pad_state(ih, k0, 0x36363636u);
  tail(ih, 64, ikm_len, [&](uint32_t p) { return (uint32_t)key_in[p]; }, none);
  H8 prk = init();
  pad_state(prk, k0, 0x5c5c5c5cu);
  outer(prk, ih);

  // ---- expand
#pragma unroll
  for (int t = 0; t < 8; ++t) k0[t] = prk.h[t], k0[t + 8] = 0;
  H8 ipad = init(), opad = init();
  pad_state(ipad, k0, 0x36363636u);
  pad_state(opad, k0, 0x5c5c5c5cu);
  const uint8_t* inf = info_off ? info + info_off[i] : info;
  const uint32_t ilen = info_off ? (uint32_t)(info_off[i + 1] - info_off[i]) : info_len;
  uint8_t* out = okm + i * okm_stride;
  H8 tprev{};
  const uint32_t nt = (L + 31) / 32;
#pragma unroll 1
  for (uint32_t r = 1; r <= nt; ++r) {
    const uint32_t plen = r > 1 ? 32u : 0u;  // T(r-1) occupies words 0..7 of the first block
    const uint32_t len = plen + ilen + 1;
    const uint32_t ctr = r;
    H8 h = ipad;
    tail(
        h, 64, len,
        [&](uint32_t p) {
          const uint32_t q = p - plen;
          return q < ilen ? (uint32_t)inf[q] : ctr;
        },
        [&](uint32_t b, int t, uint32_t x) { return (plen && b == 0 && t < 8) ? tprev.h[t] : x; });
    H8 o = opad;
    outer(o, h);
    tprev = o;
    const uint32_t base = 32 * (r - 1);
    const uint32_t take = L - base < 32 ? L - base : 32;
#pragma unroll
    for (int t = 0; t < 8; ++t) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t p = 4 * t + k;
        if (p < take) out[base + p] = (uint8_t)(o.h[t] >> (24 - 8 * k));
      }
    }
  }
}

// agree_i = 1 iff a_i == b_i (len bytes each)
__global__ __launch_bounds__(256) void k_keys_equal(size_t n, const uint8_t* __restrict__ a,
                                                    const uint8_t* __restrict__ b, uint32_t len,
                                                    int32_t* __restrict__ agree) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  uint32_t d = 0;
  for (uint32_t p = 0; p < len; ++p) d |= (uint32_t)(a[i * len + p] ^ b[i * len + p]);
  agree[i] = d == 0 ? 1 : 0;
}

hipError_t hkdf_sha256(size_t n, const uint8_t* ikm, size_t ikm_len, size_t ikm_stride, const uint8_t* salt,
                       size_t salt_len, const uint8_t* info, const uint64_t* info_off, size_t info_len, size_t L,
                       uint8_t* okm, size_t okm_stride, hipStream_t st) {
  if (n == 0) return hipSuccess;
  if (L == 0 || L > 255 * 32) return hipErrorInvalidValue;
  QRK_LAUNCH("k_hkdf_sha256", st, k_hkdf_sha256, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, n, ikm,
             (uint32_t)ikm_len, ikm_stride, salt, (uint32_t)salt_len, info, info_off, (uint32_t)info_len,
             (uint32_t)L, okm, okm_stride);
  return hipGetLastError();
}

hipError_t keys_equal(size_t n, const uint8_t* a, const uint8_t* b, size_t len, int32_t* agree, hipStream_t st) {
  if (n == 0) return hipSuccess;
  QRK_LAUNCH("k_keys_equal", st, k_keys_equal, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, n, a, b,
             (uint32_t)len, agree);
  return hipGetLastError();
}

}  // namespace qrk
