/* ML-KEM-512/768/1024 (FIPS 203) C restatement -- oracle / CPU-baseline only.
 *
 * TEST INFRASTRUCTURE: linked into oracle/liboracle.so only.
 *
 * Follows FIPS 203 Algorithms 13-18 (K-PKE.KeyGen/Encrypt/Decrypt,
 * ML-KEM.KeyGen/Encaps/Decaps_internal).  The reference's path reaches the
 * same algorithm through liboqs at quantum_resistant_p2p/vendor/oqs.py:318
 * (keypair), :348 (encaps), :372 (decaps); randomness granularity follows the
 * pq-crystals "standard" code liboqs 0.12 wraps: KeyGen coins = d||z (64 B),
 * Encaps coins = m (32 B).
 *
 * Independent of oracle/py/mlkem_spec.py (written separately, different
 * arithmetic style: canonical residues kept as uint16 with a 32-bit Barrett
 * reduction here, Python big ints there) -- the two are cross-checked in
 * tests/test_oracle.py and against tests/golden/.
 */
#include "mlkem.h"

#include <string.h>

#include "fips202.h"

#define Q 3329
#define NN 256

typedef struct {
  uint16_t c[NN];
} poly;

/* canonical x mod q for 0 <= x < 2^32 / something; Barrett with 2^32 */
static inline uint16_t redq(uint32_t x) {
  /* floor(2^32 / q) = 1290167 */
  uint32_t t = (uint32_t)(((uint64_t)x * 1290167u) >> 32);
  uint32_t r = x - t * Q;
  return (uint16_t)(r >= Q ? r - Q : r);
}

static uint16_t ZETA[128];  /* 17^bitrev7(i) */
static uint16_t GAMMA[128]; /* 17^(2 bitrev7(i) + 1) */
static int tables_ready = 0;

static unsigned bitrev7(unsigned i) {
  unsigned r = 0;
  for (int b = 0; b < 7; ++b) r |= ((i >> b) & 1u) << (6 - b);
  return r;
}

static uint32_t powq(uint32_t b, unsigned e) {
  uint32_t r = 1;
  while (e--) r = (r * b) % Q;
  return r;
}

static void init_tables(void) {
  if (tables_ready) return;
  for (unsigned i = 0; i < 128; ++i) {
    ZETA[i] = (uint16_t)powq(17, bitrev7(i));
    GAMMA[i] = (uint16_t)powq(17, 2 * bitrev7(i) + 1);
  }
  __atomic_store_n(&tables_ready, 1, __ATOMIC_RELEASE);
}

static int params_of(const char *alg, int *k, int *eta1, int *eta2, int *du, int *dv) {
  if (!strcmp(alg, "ML-KEM-512")) {
    *k = 2, *eta1 = 3, *eta2 = 2, *du = 10, *dv = 4;
  } else if (!strcmp(alg, "ML-KEM-768")) {
    *k = 3, *eta1 = 2, *eta2 = 2, *du = 10, *dv = 4;
  } else if (!strcmp(alg, "ML-KEM-1024")) {
    *k = 4, *eta1 = 2, *eta2 = 2, *du = 11, *dv = 5;
  } else {
    return -1;
  }
  return 0;
}

int orc_mlkem_sizes(const char *alg, size_t *pk, size_t *sk, size_t *ct, size_t *ss) {
  int k, e1, e2, du, dv;
  if (params_of(alg, &k, &e1, &e2, &du, &dv)) return -1;
  *pk = 384 * k + 32;
  *sk = 768 * k + 96;
  *ct = 32 * (du * k + dv);
  *ss = 32;
  return 0;
}

/* ---------------- NTT (Alg. 9-12) ---------------- */
static void ntt(poly *f) {
  unsigned i = 1;
  for (unsigned len = 128; len >= 2; len >>= 1)
    for (unsigned start = 0; start < NN; start += 2 * len) {
      uint32_t z = ZETA[i++];
      for (unsigned j = start; j < start + len; ++j) {
        uint16_t t = redq(z * f->c[j + len]);
        f->c[j + len] = redq(f->c[j] + Q - t);
        f->c[j] = redq(f->c[j] + t);
      }
    }
}

static void ntt_inv(poly *f) {
  unsigned i = 127;
  for (unsigned len = 2; len <= 128; len <<= 1)
    for (unsigned start = 0; start < NN; start += 2 * len) {
      uint32_t z = ZETA[i--];
      for (unsigned j = start; j < start + len; ++j) {
        uint16_t t = f->c[j];
        f->c[j] = redq(t + f->c[j + len]);
        f->c[j + len] = redq(z * (uint32_t)(f->c[j + len] + Q - t));
      }
    }
  for (unsigned j = 0; j < NN; ++j) f->c[j] = redq(3303u * f->c[j]);
}

/* h += f o g in T_q */
static void mul_acc(poly *h, const poly *f, const poly *g) {
  for (unsigned i = 0; i < 128; ++i) {
    uint32_t a0 = f->c[2 * i], a1 = f->c[2 * i + 1], b0 = g->c[2 * i], b1 = g->c[2 * i + 1];
    uint32_t c0 = redq(a0 * b0) + redq(redq(a1 * b1) * (uint32_t)GAMMA[i]);
    uint32_t c1 = redq(a0 * b1) + redq(a1 * b0);
    h->c[2 * i] = redq(h->c[2 * i] + c0);
    h->c[2 * i + 1] = redq(h->c[2 * i + 1] + c1);
  }
}

static void poly_add(poly *r, const poly *a) {
  for (unsigned j = 0; j < NN; ++j) r->c[j] = redq(r->c[j] + a->c[j]);
}

/* ---------------- encodings (Alg. 5, 6) ---------------- */
static void byte_encode(uint8_t *out, const poly *f, int d) {
  uint32_t acc = 0;
  int bits = 0;
  size_t o = 0;
  for (unsigned i = 0; i < NN; ++i) {
    acc |= (uint32_t)(f->c[i] & ((1u << d) - 1)) << bits;
    bits += d;
    while (bits >= 8) {
      out[o++] = (uint8_t)acc;
      acc >>= 8;
      bits -= 8;
    }
  }
}

static void byte_decode(poly *f, const uint8_t *in, int d) {
  uint32_t acc = 0;
  int bits = 0;
  size_t p = 0;
  for (unsigned i = 0; i < NN; ++i) {
    while (bits < d) {
      acc |= (uint32_t)in[p++] << bits;
      bits += 8;
    }
    uint32_t v = acc & ((1u << d) - 1);
    acc >>= d;
    bits -= d;
    f->c[i] = (uint16_t)(d == 12 ? (v >= Q ? v - Q : v) : v);
  }
}

static inline uint16_t compress_d(uint16_t x, int d) {
  return (uint16_t)((((uint32_t)x << d) + Q / 2) / Q & ((1u << d) - 1));
}
static inline uint16_t decompress_d(uint16_t y, int d) {
  return (uint16_t)(((uint32_t)Q * y + (1u << (d - 1))) >> d);
}

/* ---------------- sampling (Alg. 7, 8) ---------------- */
static void sample_ntt(poly *a, const uint8_t rho[32], uint8_t j, uint8_t i) {
  uint8_t seed[34];
  memcpy(seed, rho, 32);
  seed[32] = j;
  seed[33] = i;
  orc_keccak c;
  orc_keccak_init(&c, ORC_SHAKE128_RATE);
  orc_keccak_absorb(&c, seed, 34);
  orc_keccak_finalize(&c, 0x1F);
  unsigned n = 0;
  uint8_t buf[ORC_SHAKE128_RATE];
  while (n < NN) {
    orc_keccak_squeeze(&c, buf, sizeof buf);
    for (unsigned p = 0; p + 3 <= sizeof buf && n < NN; p += 3) {
      uint16_t d1 = (uint16_t)(buf[p] | ((buf[p + 1] & 0x0F) << 8));
      uint16_t d2 = (uint16_t)((buf[p + 1] >> 4) | (buf[p + 2] << 4));
      if (d1 < Q) a->c[n++] = d1;
      if (d2 < Q && n < NN) a->c[n++] = d2;
    }
  }
}

static void sample_cbd(poly *f, const uint8_t *b, int eta) {
  for (unsigned i = 0; i < NN; ++i) {
    int x = 0, y = 0;
    for (int j = 0; j < eta; ++j) {
      unsigned bx = 2 * i * eta + j, by = 2 * i * eta + eta + j;
      x += (b[bx >> 3] >> (bx & 7)) & 1;
      y += (b[by >> 3] >> (by & 7)) & 1;
    }
    f->c[i] = (uint16_t)((x - y + Q) % Q);
  }
}

static void prf_cbd(poly *f, const uint8_t s[32], uint8_t nonce, int eta) {
  uint8_t in[33], out[64 * 3];
  memcpy(in, s, 32);
  in[32] = nonce;
  orc_shake256(out, 64 * eta, in, 33);
  sample_cbd(f, out, eta);
}

/* ---------------- K-PKE (Alg. 13-15) ---------------- */
#define KMAX 4

static void kpke_keygen(uint8_t *ek, uint8_t *dk, const uint8_t d[32], int k, int eta1) {
  uint8_t gin[33], g[64];
  memcpy(gin, d, 32);
  gin[32] = (uint8_t)k;
  orc_sha3_512(g, gin, 33);
  const uint8_t *rho = g, *sigma = g + 32;
  poly s[KMAX], e[KMAX], a;
  uint8_t nonce = 0;
  for (int i = 0; i < k; ++i) prf_cbd(&s[i], sigma, nonce++, eta1);
  for (int i = 0; i < k; ++i) prf_cbd(&e[i], sigma, nonce++, eta1);
  for (int i = 0; i < k; ++i) ntt(&s[i]), ntt(&e[i]);
  for (int i = 0; i < k; ++i) {
    poly t;
    memset(&t, 0, sizeof t);
    for (int j = 0; j < k; ++j) {
      sample_ntt(&a, rho, (uint8_t)j, (uint8_t)i);
      mul_acc(&t, &a, &s[j]);
    }
    poly_add(&t, &e[i]);
    byte_encode(ek + 384 * i, &t, 12);
    byte_encode(dk + 384 * i, &s[i], 12);
  }
  memcpy(ek + 384 * k, rho, 32);
}

static void kpke_encrypt(uint8_t *c, const uint8_t *ek, const uint8_t m[32], const uint8_t r[32],
                         int k, int eta1, int eta2, int du, int dv) {
  poly t[KMAX], y[KMAX], a, u, v, e;
  const uint8_t *rho = ek + 384 * k;
  for (int i = 0; i < k; ++i) byte_decode(&t[i], ek + 384 * i, 12);
  uint8_t nonce = 0;
  for (int i = 0; i < k; ++i) prf_cbd(&y[i], r, nonce++, eta1), ntt(&y[i]);
  for (int i = 0; i < k; ++i) {
    memset(&u, 0, sizeof u);
    for (int j = 0; j < k; ++j) {
      sample_ntt(&a, rho, (uint8_t)i, (uint8_t)j); /* A_hat[j][i] = SampleNTT(rho||i||j) */
      mul_acc(&u, &a, &y[j]);
    }
    ntt_inv(&u);
    prf_cbd(&e, r, (uint8_t)(k + i), eta2);
    poly_add(&u, &e);
    for (unsigned x = 0; x < NN; ++x) u.c[x] = compress_d(u.c[x], du);
    byte_encode(c + 32 * du * i, &u, du);
  }
  memset(&v, 0, sizeof v);
  for (int j = 0; j < k; ++j) mul_acc(&v, &t[j], &y[j]);
  ntt_inv(&v);
  prf_cbd(&e, r, (uint8_t)(2 * k), eta2);
  poly_add(&v, &e);
  for (unsigned x = 0; x < NN; ++x) {
    uint16_t bit = (m[x >> 3] >> (x & 7)) & 1;
    v.c[x] = redq(v.c[x] + decompress_d(bit, 1));
    v.c[x] = compress_d(v.c[x], dv);
  }
  byte_encode(c + 32 * du * k, &v, dv);
}

static void kpke_decrypt(uint8_t m[32], const uint8_t *dk, const uint8_t *c, int k, int du, int dv) {
  poly u, s, w, v;
  memset(&w, 0, sizeof w);
  for (int i = 0; i < k; ++i) {
    byte_decode(&u, c + 32 * du * i, du);
    for (unsigned x = 0; x < NN; ++x) u.c[x] = decompress_d(u.c[x], du);
    ntt(&u);
    byte_decode(&s, dk + 384 * i, 12);
    mul_acc(&w, &s, &u);
  }
  ntt_inv(&w);
  byte_decode(&v, c + 32 * du * k, dv);
  memset(m, 0, 32);
  for (unsigned x = 0; x < NN; ++x) {
    uint16_t vv = decompress_d(v.c[x], dv);
    uint16_t d = redq(vv + Q - w.c[x]);
    m[x >> 3] |= (uint8_t)(compress_d(d, 1) << (x & 7));
  }
}

/* ---------------- ML-KEM (Alg. 16-18) ---------------- */
int orc_mlkem_keypair_derand(const char *alg, uint8_t *pk, uint8_t *sk, const uint8_t coins[64]) {
  int k, e1, e2, du, dv;
  if (params_of(alg, &k, &e1, &e2, &du, &dv)) return -1;
  init_tables();
  kpke_keygen(pk, sk, coins, k, e1);
  size_t pklen = 384 * k + 32;
  memcpy(sk + 384 * k, pk, pklen);
  orc_sha3_256(sk + 384 * k + pklen, pk, pklen);
  memcpy(sk + 384 * k + pklen + 32, coins + 32, 32);
  return 0;
}

int orc_mlkem_ek_check(const char *alg, const uint8_t *pk) {
  int k, e1, e2, du, dv;
  if (params_of(alg, &k, &e1, &e2, &du, &dv)) return -1;
  for (int i = 0; i < k; ++i)
    for (int x = 0; x < NN / 2; ++x) {
      const uint8_t *p = pk + 384 * i + 3 * x;
      uint16_t d1 = (uint16_t)(p[0] | ((p[1] & 0x0F) << 8));
      uint16_t d2 = (uint16_t)((p[1] >> 4) | (p[2] << 4));
      if (d1 >= Q || d2 >= Q) return -1;
    }
  return 0;
}

int orc_mlkem_encaps_derand(const char *alg, uint8_t *ct, uint8_t *ss, const uint8_t *pk,
                            const uint8_t coins[32]) {
  int k, e1, e2, du, dv;
  if (params_of(alg, &k, &e1, &e2, &du, &dv)) return -1;
  if (orc_mlkem_ek_check(alg, pk)) return -1;
  init_tables();
  uint8_t gin[64], g[64];
  memcpy(gin, coins, 32);
  orc_sha3_256(gin + 32, pk, 384 * k + 32);
  orc_sha3_512(g, gin, 64);
  kpke_encrypt(ct, pk, coins, g + 32, k, e1, e2, du, dv);
  memcpy(ss, g, 32);
  return 0;
}

int orc_mlkem_decaps(const char *alg, uint8_t *ss, const uint8_t *ct, const uint8_t *sk) {
  int k, e1, e2, du, dv;
  if (params_of(alg, &k, &e1, &e2, &du, &dv)) return -1;
  init_tables();
  const size_t ctlen = 32 * (du * k + dv);
  const uint8_t *ek = sk + 384 * k, *h = sk + 768 * k + 32, *z = sk + 768 * k + 64;
  uint8_t gin[64], g[64], cprime[1568], jin[32 + 1568], kbar[32];
  kpke_decrypt(gin, sk, ct, k, du, dv);
  memcpy(gin + 32, h, 32);
  orc_sha3_512(g, gin, 64);
  memcpy(jin, z, 32);
  memcpy(jin + 32, ct, ctlen);
  orc_shake256(kbar, 32, jin, 32 + ctlen);
  kpke_encrypt(cprime, ek, gin, g + 32, k, e1, e2, du, dv);
  uint8_t diff = 0;
  for (size_t i = 0; i < ctlen; ++i) diff |= (uint8_t)(ct[i] ^ cprime[i]);
  /* constant-time select: mask = 0xFF if equal */
  uint8_t mask = (uint8_t)(((uint32_t)diff - 1u) >> 8);
  for (int i = 0; i < 32; ++i) ss[i] = (uint8_t)((g[i] & mask) | (kbar[i] & ~mask));
  return 0;
}
