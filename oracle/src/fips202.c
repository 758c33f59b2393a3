/* Keccak-f[1600] and the FIPS 202 sponge -- oracle / CPU-baseline only.
 * See fips202.h for scope.  Written from the FIPS 202 section 3.2 step
 * mappings (theta, rho, pi, chi, iota) with lanes A[x + 5y].
 */
#include "fips202.h"

#include <string.h>

static const uint64_t RC[24] = {
    0x0000000000000001ULL, 0x0000000000008082ULL, 0x800000000000808aULL,
    0x8000000080008000ULL, 0x000000000000808bULL, 0x0000000080000001ULL,
    0x8000000080008081ULL, 0x8000000000008009ULL, 0x000000000000008aULL,
    0x0000000000000088ULL, 0x0000000080008009ULL, 0x000000008000000aULL,
    0x000000008000808bULL, 0x800000000000008bULL, 0x8000000000008089ULL,
    0x8000000000008003ULL, 0x8000000000008002ULL, 0x8000000000000080ULL,
    0x000000000000800aULL, 0x800000008000000aULL, 0x8000000080008081ULL,
    0x8000000000008080ULL, 0x0000000080000001ULL, 0x8000000080008008ULL};

/* rho offsets r[x][y] indexed by x + 5y */
static const unsigned RHO[25] = {0,  1,  62, 28, 27, 36, 44, 6,  55, 20, 3,  10, 43,
                                 25, 39, 41, 45, 15, 21, 8,  18, 2,  61, 56, 14};

static inline uint64_t rol(uint64_t v, unsigned n) {
  return n ? (v << n) | (v >> (64 - n)) : v;
}

void orc_keccakf1600(uint64_t A[25]) {
  uint64_t C[5], D[5], B[25];
  for (int round = 0; round < 24; ++round) {
    for (int x = 0; x < 5; ++x)
      C[x] = A[x] ^ A[x + 5] ^ A[x + 10] ^ A[x + 15] ^ A[x + 20];
    for (int x = 0; x < 5; ++x) D[x] = C[(x + 4) % 5] ^ rol(C[(x + 1) % 5], 1);
    for (int i = 0; i < 25; ++i) A[i] ^= D[i % 5];
    /* rho + pi: B[y, 2x+3y] = rot(A[x,y], r[x,y]) */
    for (int x = 0; x < 5; ++x)
      for (int y = 0; y < 5; ++y) {
        int X = y, Y = (2 * x + 3 * y) % 5;
        B[X + 5 * Y] = rol(A[x + 5 * y], RHO[x + 5 * y]);
      }
    for (int y = 0; y < 5; ++y)
      for (int x = 0; x < 5; ++x)
        A[x + 5 * y] = B[x + 5 * y] ^ (~B[(x + 1) % 5 + 5 * y] & B[(x + 2) % 5 + 5 * y]);
    A[0] ^= RC[round];
  }
}

void orc_keccak_init(orc_keccak *c, unsigned rate) {
  memset(c->s, 0, sizeof c->s);
  c->pos = 0;
  c->rate = rate;
}

static inline void xor_byte(uint64_t *s, unsigned pos, uint8_t b) {
  s[pos >> 3] ^= (uint64_t)b << (8 * (pos & 7));
}

void orc_keccak_absorb(orc_keccak *c, const uint8_t *in, size_t len) {
  while (len) {
    if (c->pos == 0 && len >= c->rate) {
      for (unsigned i = 0; i < c->rate / 8; ++i) {
        uint64_t w;
        memcpy(&w, in + 8 * i, 8); /* little-endian host */
        c->s[i] ^= w;
      }
      orc_keccakf1600(c->s);
      in += c->rate;
      len -= c->rate;
      continue;
    }
    xor_byte(c->s, c->pos++, *in++);
    --len;
    if (c->pos == c->rate) {
      orc_keccakf1600(c->s);
      c->pos = 0;
    }
  }
}

void orc_keccak_finalize(orc_keccak *c, uint8_t ds) {
  xor_byte(c->s, c->pos, ds);
  xor_byte(c->s, c->rate - 1, 0x80);
  orc_keccakf1600(c->s);
  c->pos = 0;
}

void orc_keccak_squeeze(orc_keccak *c, uint8_t *out, size_t len) {
  while (len) {
    if (c->pos == c->rate) {
      orc_keccakf1600(c->s);
      c->pos = 0;
    }
    *out++ = (uint8_t)(c->s[c->pos >> 3] >> (8 * (c->pos & 7)));
    c->pos++;
    --len;
  }
}

static void sponge(uint8_t *out, size_t outlen, const uint8_t *in, size_t inlen,
                   unsigned rate, uint8_t ds) {
  orc_keccak c;
  orc_keccak_init(&c, rate);
  orc_keccak_absorb(&c, in, inlen);
  orc_keccak_finalize(&c, ds);
  orc_keccak_squeeze(&c, out, outlen);
}

void orc_shake128(uint8_t *out, size_t outlen, const uint8_t *in, size_t inlen) {
  sponge(out, outlen, in, inlen, ORC_SHAKE128_RATE, 0x1F);
}
void orc_shake256(uint8_t *out, size_t outlen, const uint8_t *in, size_t inlen) {
  sponge(out, outlen, in, inlen, ORC_SHAKE256_RATE, 0x1F);
}
void orc_sha3_256(uint8_t out[32], const uint8_t *in, size_t inlen) {
  sponge(out, 32, in, inlen, ORC_SHA3_256_RATE, 0x06);
}
void orc_sha3_512(uint8_t out[64], const uint8_t *in, size_t inlen) {
  sponge(out, 64, in, inlen, ORC_SHA3_512_RATE, 0x06);
}
