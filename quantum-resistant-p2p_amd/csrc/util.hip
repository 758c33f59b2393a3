// Bench-input helpers that run on the device so that 2^20..2^24-handshake
// inputs never cross PCIe.
#include "keccak.cuh"
#include "qrkem_internal.h"

namespace qrk {

// coins_i = SHAKE256("qrk-bench" || LE64(seed) || LE64(first + i), len), len <= 136
__global__ __launch_bounds__(256) void k_bench_coins(size_t n, int nwords, uint64_t seed, uint64_t first,
                                                     uint64_t* __restrict__ out) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const uint64_t idx = first + i;
  // 25-byte message: "qrk-benc" | "h" seed[0..6] | seed[7] idx[0..6] | idx[7] DS
  const uint64_t w0 = 0x636e65622d6b7271ull;  // "qrk-benc" little-endian
  const uint64_t w1 = 0x68ull | (seed << 8);
  const uint64_t w2 = (seed >> 56) | (idx << 8);
  const uint64_t w3 = (idx >> 56) | ((uint64_t)DS_SHAKE << 8);
  KState s;
  kzero(s);
  kxor(s, 0, w0);
  kxor(s, 1, w1);
  kxor(s, 2, w2);
  kxor(s, 3, w3);
  s.a[RW_SHAKE256 - 1].hi ^= 0x80000000u;
  keccak_f(s);
  uint64_t* o = out + i * (size_t)nwords;
#pragma unroll
  for (int w = 0; w < RW_SHAKE256; ++w)
    if (w < nwords) o[w] = kword(s, w);
}

hipError_t bench_coins(size_t n, size_t len, uint64_t seed, uint64_t first, uint8_t* out, hipStream_t st) {
  if (len % 8 || len > 136) return hipErrorInvalidValue;
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_bench_coins, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, n, (int)(len / 8), seed,
                     first, (uint64_t*)out);
  return hipGetLastError();
}

// h_i = SHAKE256("qrk-tamper" || LE64(seed) || LE64(i)) first 8 bytes;
// tamper iff mode == 1, or mode == 2 and (h_i & 1); flipped bit = (h_i >> 1) mod (8 * ctlen)
__global__ __launch_bounds__(256) void k_tamper(size_t n, size_t ctlen, uint64_t seed, int mode,
                                                uint8_t* __restrict__ ct) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  // 26-byte message: "qrk-tamp" | "er" seed[0..5] | seed[6..7] i[0..5] | i[6..7] DS
  const uint64_t idx = i;
  KState s;
  kzero(s);
  kxor(s, 0, 0x706d61742d6b7271ull);  // "qrk-tamp"
  kxor(s, 1, 0x7265ull | (seed << 16));
  kxor(s, 2, (seed >> 48) | (idx << 16));
  kxor(s, 3, (idx >> 48) | ((uint64_t)DS_SHAKE << 16));
  s.a[RW_SHAKE256 - 1].hi ^= 0x80000000u;
  keccak_f(s);
  const uint64_t h = kword(s, 0);
  const bool flip = mode == 1 || (mode == 2 && (h & 1));
  if (flip) {
    const uint64_t bit = (h >> 1) % (8 * ctlen);
    ct[i * ctlen + bit / 8] ^= (uint8_t)(1u << (bit % 8));
  }
}

hipError_t tamper_ciphertexts(size_t n, size_t ctlen, uint64_t seed, int mode, uint8_t* ct, hipStream_t st) {
  if (n == 0 || mode == 0) return hipSuccess;
  hipLaunchKernelGGL(k_tamper, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, n, ctlen, seed, mode, ct);
  return hipGetLastError();
}

// out_i = SHA3-256(a_i || b_i) for n records (a_i = a + i*al, b_i = b + i*bl, bl may be 0):
// per-record digests of a batch's outputs, from which the sharded bench builds its shard
// digests (identical whatever the GPU count).  One lane per record;
// word loads when both lengths are multiples of 8, byte assembly otherwise.
__device__ __forceinline__ uint64_t rec_word(const uint8_t* a, size_t al, const uint8_t* b, size_t bl, size_t p,
                                             size_t total, bool words) {
  if (words && p + 8 <= total) {
    if (p + 8 <= al) return *(const uint64_t*)(a + p);
    if (p >= al) return *(const uint64_t*)(b + (p - al));
  }
  uint64_t w = 0;
  for (int j = 0; j < 8; ++j) {
    const size_t q = p + j;
    uint64_t v = 0;
    if (q < al)
      v = a[q];
    else if (q < total)
      v = b[q - al];
    else if (q == total)
      v = DS_SHA3;
    w |= v << (8 * j);
  }
  return w;
}

__global__ __launch_bounds__(256) void k_digest_rows(size_t n, const uint8_t* __restrict__ a, size_t al,
                                                     const uint8_t* __restrict__ b, size_t bl,
                                                     uint8_t* __restrict__ out) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const uint8_t* ai = a + i * al;
  const uint8_t* bi = b ? b + i * bl : nullptr;
  const size_t total = al + bl;
  const bool words = (al % 8 == 0) && (bl % 8 == 0);
  const size_t nblk = total / (8 * RW_SHA3_256) + 1;  // the pad always fits in the last block
  KState s;
  kzero(s);
#pragma unroll 1
  for (size_t blk = 0; blk < nblk; ++blk) {
#pragma unroll
    for (int w = 0; w < RW_SHA3_256; ++w) kxor(s, w, rec_word(ai, al, bi, bl, blk * 136 + 8 * w, total, words));
    if (blk + 1 == nblk) s.a[RW_SHA3_256 - 1].hi ^= 0x80000000u;
    keccak_f(s);
  }
  uint64_t* o = (uint64_t*)(out + i * 32);
#pragma unroll
  for (int w = 0; w < 4; ++w) o[w] = kword(s, w);
}

hipError_t digest_rows(size_t n, const uint8_t* a, size_t al, const uint8_t* b, size_t bl, uint8_t* out,
                       hipStream_t st) {
  if (n == 0) return hipSuccess;
  QRK_LAUNCH("k_digest_rows", st, k_digest_rows, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, n, a, al, b,
             bl, out);
  return hipGetLastError();
}

}  // namespace qrk
