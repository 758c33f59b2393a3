// Batched base64 codec for the key-exchange wire fields, gfx950.
//
// The reference puts every KEM payload on the wire as standard base64 (RFC 4648 section 4,
// '=' padding) inside JSON: the initiator's public key (quantum_resistant_p2p/app/
// messaging.py:607), the responder's ciphertext and public key (:852-853); the peers decode
// them with base64.b64decode (:829 public key, and the response's ciphertext).  These
// kernels do that for N records per launch.
//
// Layout: records are contiguous AoS rows, [n][L] bytes in, [n][4 ceil(L/3)] characters out
// (decode: the reverse).  One lane handles a 12-byte / 16-character chunk of one record,
// lanes walk (record, chunk) so a wave reads and writes consecutive memory (HBM-bound:
// 7/3 bytes moved per payload byte).  The 64-entry alphabet and the 256-entry inverse
// table live in LDS with one copy per bank (entry e of lane l at dword 32 e + (l & 31)), so
// the per-character lookups never conflict.  Grid-stride loops amortise the table fill.
#include "qrkem_internal.h"

namespace qrk {
namespace b64 {

struct Tables {
  uint8_t enc[64];
  uint8_t dec[256];  // 0..63, or 0xFF for a byte outside the alphabet ('=' included)
};
constexpr Tables make_tables() {
  Tables t{};
  for (int v = 0; v < 64; ++v) {
    const int c = v < 26 ? 'A' + v : v < 52 ? 'a' + v - 26 : v < 62 ? '0' + v - 52 : v == 62 ? '+' : '/';
    t.enc[v] = (uint8_t)c;
  }
  for (int c = 0; c < 256; ++c) t.dec[c] = 0xFF;
  for (int v = 0; v < 64; ++v) t.dec[t.enc[v]] = (uint8_t)v;
  return t;
}
__constant__ static const Tables TAB = make_tables();

__device__ __forceinline__ uint32_t ld_byte(const uint8_t* p, size_t i, size_t len) { return i < len ? p[i] : 0u; }

// 12 input bytes -> 16 characters; `have` = bytes present (1..12); missing groups / bytes give
// '=' padding (RFC 4648: 1 byte -> xx==, 2 bytes -> xxx=).
__device__ __forceinline__ void encode_chunk(const uint32_t (&w)[3], uint32_t have, const char* tb, uint32_t tl,
                                             uint8_t* dst) {
  uint32_t o[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    // bytes 3g .. 3g+2 of the chunk as a big-endian 24-bit value
    const int b = 3 * g;
    const uint32_t b0 = (w[b >> 2] >> (8 * (b & 3))) & 0xFF;
    const uint32_t b1 = (w[(b + 1) >> 2] >> (8 * ((b + 1) & 3))) & 0xFF;
    const uint32_t b2 = (w[(b + 2) >> 2] >> (8 * ((b + 2) & 3))) & 0xFF;
    const uint32_t x = b0 << 16 | b1 << 8 | b2;
    const uint32_t c0 = *(const uint32_t*)(tb + (((x >> 11) & 0x1F80u) | tl));
    const uint32_t c1 = *(const uint32_t*)(tb + (((x >> 5) & 0x1F80u) | tl));
    const uint32_t c2 = *(const uint32_t*)(tb + (((x << 1) & 0x1F80u) | tl));
    const uint32_t c3 = *(const uint32_t*)(tb + (((x << 7) & 0x1F80u) | tl));
    uint32_t v = c0 | c1 << 8 | c2 << 16 | c3 << 24;
    const int rem = (int)have - b;  // bytes of this group present
    if (rem <= 0) v = 0;            // beyond the record: not stored
    else if (rem == 1) v = (v & 0xFFFFu) | 0x3D3D0000u;
    else if (rem == 2) v = (v & 0xFFFFFFu) | 0x3D000000u;
    o[g] = v;
  }
  const uint32_t ngroups = (have + 2) / 3;
  if (ngroups == 4 && ((uintptr_t)dst & 3) == 0) {
#pragma unroll
    for (int g = 0; g < 4; ++g) ((uint32_t*)dst)[g] = o[g];
  } else {
    for (uint32_t g = 0; g < ngroups; ++g)
#pragma unroll
      for (int k = 0; k < 4; ++k) dst[4 * g + k] = (uint8_t)(o[g] >> (8 * k));
  }
}

// Each lane takes ENC_U chunks of the grid-stride walk per iteration and issues all their loads
// before the first use: HBM-bound, the kernel needs bytes in flight, and one 12-byte load per
// lane at a time (rounds 2-4) held 0.42 of the 8 TB/s peak.  Same box, three interleaved rounds
// (profiles/r5/wire/): the wire step 2.61e8 -> 3.19e8 exchanges/s at 4 in flight, 2 the same,
// 8 slower (66 / 93 VGPRs for encode / decode: fewer waves).
constexpr int ENC_U = 4;
__global__ __launch_bounds__(256) void k_b64_encode(size_t n, const uint8_t* __restrict__ in, uint32_t L,
                                                    uint8_t* __restrict__ out, uint32_t OL) {
  __shared__ uint32_t tab[64 * 32];
  for (int e = threadIdx.x; e < 64 * 32; e += 256) tab[e] = TAB.enc[e >> 5];
  __syncthreads();
  const uint32_t cpr = (L + 11) / 12;  // chunks per record
  const uint32_t tl = (threadIdx.x & 31) * 4;
  const char* tb = (const char*)tab;
  // (record, chunk) walk without per-iteration 64-bit division
  const size_t t0 = (size_t)blockIdx.x * 256 + threadIdx.x, S = (size_t)gridDim.x * 256;
  size_t rec = t0 / cpr;
  uint32_t c = (uint32_t)(t0 % cpr);
  const size_t srec = S / cpr;
  const uint32_t sc = (uint32_t)(S % cpr);
  const size_t nL = n * L;  // bytes in the input buffer
#pragma unroll 1
  while (rec < n) {
    size_t r[ENC_U];
    uint32_t ch[ENC_U], w[ENC_U][3];
#pragma unroll
    for (int u = 0; u < ENC_U; ++u) {
      r[u] = rec;
      ch[u] = c;
      rec += srec, c += sc;
      if (c >= cpr) c -= cpr, ++rec;
    }
#pragma unroll
    for (int u = 0; u < ENC_U; ++u) {
      const uint8_t* src = in + r[u] * L + 12 * ch[u];
      const uint32_t have = L - 12 * ch[u] < 12 ? L - 12 * ch[u] : 12;
      if (r[u] >= n) {
        w[u][0] = w[u][1] = w[u][2] = 0u;
      } else if (((uintptr_t)src & 3) == 0 && r[u] * L + 12 * ch[u] + 12 <= nL) {
        // a record's short last chunk may read into the following records (the same buffer) and
        // masks those bytes off, so the wave rarely takes the byte-wise path; the bound is the
        // buffer's real end, since a short record (L < 12 - have) spans fewer than 12 bytes
        const uint3 v = *(const uint3*)src;
        w[u][0] = v.x, w[u][1] = v.y, w[u][2] = v.z;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          const int keep = (int)have - 4 * k;  // bytes of word k inside the record
          w[u][k] &= keep >= 4 ? 0xFFFFFFFFu : keep <= 0 ? 0u : (1u << (8 * keep)) - 1u;
        }
      } else {
#pragma unroll
        for (int k = 0; k < 3; ++k)
          w[u][k] = ld_byte(src, 4 * k, have) | ld_byte(src, 4 * k + 1, have) << 8 |
                    ld_byte(src, 4 * k + 2, have) << 16 | ld_byte(src, 4 * k + 3, have) << 24;
      }
    }
#pragma unroll
    for (int u = 0; u < ENC_U; ++u) {
      if (r[u] >= n) break;  // the walk is monotonic: the later slots are past the end too
      const uint32_t have = L - 12 * ch[u] < 12 ? L - 12 * ch[u] : 12;
      encode_chunk(w[u], have, tb, tl, out + r[u] * OL + 16 * ch[u]);
    }
  }
}

// 16 characters -> 12 bytes (fewer in the record's last chunk).  Strict: a character outside
// the alphabet, '=' anywhere but the final 1-2 padding positions, or a padding count that does
// not match the output length marks the record invalid (status -1); the caller zeroes status.
// Loads of DEC_U chunks per lane in flight before the first use, as in the encoder.
constexpr int DEC_U = 4;
__global__ __launch_bounds__(256) void k_b64_decode(size_t n, const uint8_t* __restrict__ in, uint32_t IL,
                                                    uint8_t* __restrict__ out, uint32_t L,
                                                    int32_t* __restrict__ status) {
  __shared__ uint32_t tab[128 * 32];  // 7-bit ASCII; bytes >= 0x80 are rejected by their top bit
  for (int e = threadIdx.x; e < 128 * 32; e += 256) tab[e] = TAB.dec[e >> 5];
  __syncthreads();
  const uint32_t cpr = (IL + 15) / 16;
  const uint32_t tl = (threadIdx.x & 31) * 4;
  const char* tb = (const char*)tab;
  const uint32_t have_last = L - 12 * (cpr - 1);
  const uint32_t pad = (3 - L % 3) % 3;  // '=' characters at the record's end
  const size_t t0 = (size_t)blockIdx.x * 256 + threadIdx.x, S = (size_t)gridDim.x * 256;
  size_t rec = t0 / cpr;
  uint32_t c = (uint32_t)(t0 % cpr);
  const size_t srec = S / cpr;
  const uint32_t sc = (uint32_t)(S % cpr);
  const size_t nIL = n * IL;  // characters in the input buffer
#pragma unroll 1
  while (rec < n) {
    size_t r[DEC_U];
    uint32_t chs[DEC_U], w[DEC_U][4];
#pragma unroll
    for (int u = 0; u < DEC_U; ++u) {
      r[u] = rec;
      chs[u] = c;
      rec += srec, c += sc;
      if (c >= cpr) c -= cpr, ++rec;
    }
#pragma unroll
    for (int u = 0; u < DEC_U; ++u) {
      const uint8_t* src = in + r[u] * IL + 16 * chs[u];
      const uint32_t nch = IL - 16 * chs[u] < 16 ? IL - 16 * chs[u] : 16;  // a multiple of 4
      if (r[u] >= n) {
#pragma unroll
        for (int k = 0; k < 4; ++k) w[u][k] = 0u;
      } else if (((uintptr_t)src & 3) == 0 && r[u] * IL + 16 * chs[u] + 16 <= nIL) {
        // a record's short last chunk may read into the following records (never past the
        // buffer's end); words past nch are never used
#pragma unroll
        for (int k = 0; k < 4; ++k) w[u][k] = ((const uint32_t*)src)[k];
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k)
          w[u][k] = 4 * k < (int)nch ? (uint32_t)src[4 * k] | (uint32_t)src[4 * k + 1] << 8 |
                                          (uint32_t)src[4 * k + 2] << 16 | (uint32_t)src[4 * k + 3] << 24
                                    : 0u;
      }
    }
#pragma unroll
    for (int u = 0; u < DEC_U; ++u) {
      if (r[u] >= n) break;  // the walk is monotonic
      const uint32_t cc = chs[u];
      const uint32_t nch = IL - 16 * cc < 16 ? IL - 16 * cc : 16;
      const uint32_t last_chunk = cc + 1 == cpr;
      const uint32_t have = last_chunk ? have_last : 12;  // output bytes of this chunk
      uint32_t bad = 0, o[3] = {0, 0, 0};
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        if (4 * g >= (int)nch) break;
        uint32_t v = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const uint32_t ch = (w[u][g] >> (8 * k)) & 0xFF;
          uint32_t d = *(const uint32_t*)(tb + (((ch << 7) & 0x3F80u) | tl)) | (ch & 0x80u);
          // padding is legal only in the last group of the record, last `pad` positions
          const bool is_pad_pos = last_chunk && 4 * g + 4 == (int)nch && k >= 4 - (int)pad;
          if (is_pad_pos) {
            bad |= ch != '=';
            d = 0;
          } else {
            bad |= d >> 6;
          }
          v = v << 6 | (d & 63);
        }
        // v = 24-bit big-endian group -> bytes 3g .. 3g+2 of the chunk
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          const int b = 3 * g + k;
          o[b >> 2] |= ((v >> (16 - 8 * k)) & 0xFF) << (8 * (b & 3));
        }
      }
      uint8_t* dst = out + r[u] * L + 12 * cc;
      if (have == 12 && ((uintptr_t)dst & 3) == 0) {
#pragma unroll
        for (int k = 0; k < 3; ++k) ((uint32_t*)dst)[k] = o[k];
      } else {
        for (uint32_t b = 0; b < have; ++b) dst[b] = (uint8_t)(o[b >> 2] >> (8 * (b & 3)));
      }
      if (bad && status) status[r[u]] = -1;
    }
  }
}

// grid-stride launches: enough workgroups to fill 256 CUs several times over, few enough
// that the per-workgroup LDS table fill is amortised over many chunks per lane
inline unsigned grid(size_t threads) {
  const size_t want = (threads + 255) / 256;
  return (unsigned)(want < 4096 ? want : 4096);
}

}  // namespace b64

hipError_t base64_encode(size_t n, const uint8_t* in, size_t L, uint8_t* out, hipStream_t st) {
  if (n == 0 || L == 0) return hipSuccess;
  const size_t OL = 4 * ((L + 2) / 3);
  const size_t threads = n * ((L + 11) / 12);
  QRK_LAUNCH("k_b64_encode", st, b64::k_b64_encode, dim3(b64::grid(threads)), dim3(256), 0, st, n, in,
             (uint32_t)L, out, (uint32_t)OL);
  return hipGetLastError();
}

hipError_t base64_decode(size_t n, const uint8_t* in, size_t L, uint8_t* out, int32_t* status, hipStream_t st) {
  if (n == 0 || L == 0) return hipSuccess;
  const size_t IL = 4 * ((L + 2) / 3);
  const size_t threads = n * ((IL + 15) / 16);
  QRK_LAUNCH("k_b64_decode", st, b64::k_b64_decode, dim3(b64::grid(threads)), dim3(256), 0, st, n, in,
             (uint32_t)IL, out, (uint32_t)L, status);
  return hipGetLastError();
}

}  // namespace qrk
