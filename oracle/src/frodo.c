/* FrodoKEM-640/976/1344 (-SHAKE and -AES), round-3 specification -- oracle only.
 *
 * TEST INFRASTRUCTURE (oracle/liboracle.so).  Restates the FrodoKEM round-3
 * spec (KeyGen/Encaps/Decaps, Gen(A), CDF sampler, Pack/Unpack, Encode/Decode)
 * with the byte conventions of its reference code, which liboqs 0.12 vendors and
 * the reference reaches via quantum_resistant_p2p/vendor/oqs.py:318,348,372 for
 * the variants named at quantum_resistant_p2p/crypto/key_exchange.py:332-343.
 * Independent of oracle/py/frodo_spec.py (numpy); both are cross-checked.
 */
#include <stdlib.h>
#include <string.h>

#include "fips202.h"
#include "mlkem.h"

#define NBAR 8

typedef struct {
  int n, logq, B, sec, aes;
  const uint16_t *cdf;
  int cdf_len;
} fparams;

static const uint16_t CDF640[13] = {4643,  13363, 20579, 25843, 29227, 31145, 32103,
                                    32525, 32689, 32745, 32762, 32766, 32767};
static const uint16_t CDF976[11] = {5638,  15915, 23689, 28571, 31116, 32217,
                                    32613, 32731, 32760, 32766, 32767};
static const uint16_t CDF1344[7] = {9142, 23462, 30338, 32361, 32725, 32765, 32767};

static int params_of(const char *alg, fparams *p) {
  int aes;
  if (strncmp(alg, "FrodoKEM-", 9) != 0) return -1;
  const char *t = alg + 9;
  int n = atoi(t);
  const char *dash = strchr(t, '-');
  if (!dash) return -1;
  if (!strcmp(dash + 1, "AES"))
    aes = 1;
  else if (!strcmp(dash + 1, "SHAKE"))
    aes = 0;
  else
    return -1;
  p->aes = aes;
  p->n = n;
  if (n == 640) {
    p->logq = 15, p->B = 2, p->sec = 16, p->cdf = CDF640, p->cdf_len = 13;
  } else if (n == 976) {
    p->logq = 16, p->B = 3, p->sec = 24, p->cdf = CDF976, p->cdf_len = 11;
  } else if (n == 1344) {
    p->logq = 16, p->B = 4, p->sec = 32, p->cdf = CDF1344, p->cdf_len = 7;
  } else {
    return -1;
  }
  return 0;
}

static size_t pk_len(const fparams *p) { return 16 + (size_t)p->logq * p->n * NBAR / 8; }
static size_t ct_len(const fparams *p) {
  return (size_t)p->logq * p->n * NBAR / 8 + (size_t)p->logq * NBAR * NBAR / 8;
}
static size_t sk_len(const fparams *p) { return p->sec + pk_len(p) + 2 * (size_t)p->n * NBAR + p->sec; }
static size_t mu_len(const fparams *p) { return (size_t)p->B * NBAR * NBAR / 8; }

int orc_frodo_sizes(const char *alg, size_t *pk, size_t *sk, size_t *ct, size_t *ss,
                    size_t *kp_coins, size_t *enc_coins) {
  fparams p;
  if (params_of(alg, &p)) return -1;
  *pk = pk_len(&p);
  *sk = sk_len(&p);
  *ct = ct_len(&p);
  *ss = p.sec;
  *kp_coins = 2 * p.sec + 16;
  *enc_coins = mu_len(&p);
  return 0;
}

static void hashf(const fparams *p, uint8_t *out, size_t outlen, const uint8_t *in, size_t inlen) {
  if (p->n == 640)
    orc_shake128(out, outlen, in, inlen);
  else
    orc_shake256(out, outlen, in, inlen);
}

/* row i of A (n values) */
static void gen_a_row(const fparams *p, const uint8_t seed_a[16], int i, uint16_t *row) {
  if (!p->aes) {
    uint8_t in[18];
    in[0] = (uint8_t)i;
    in[1] = (uint8_t)(i >> 8);
    memcpy(in + 2, seed_a, 16);
    uint8_t *buf = (uint8_t *)row; /* little-endian host */
    orc_shake128(buf, 2 * (size_t)p->n, in, 18);
  } else {
    for (int j = 0; j < p->n; j += 8) {
      uint8_t blk[16] = {0}, out[16];
      blk[0] = (uint8_t)i, blk[1] = (uint8_t)(i >> 8);
      blk[2] = (uint8_t)j, blk[3] = (uint8_t)(j >> 8);
      orc_aes_encrypt_block(seed_a, 128, blk, out);
      for (int t = 0; t < 8; ++t) row[j + t] = (uint16_t)(out[2 * t] | (out[2 * t + 1] << 8));
    }
  }
}

static void sample_n(const fparams *p, uint16_t *s, size_t cnt) {
  for (size_t i = 0; i < cnt; ++i) {
    uint16_t prnd = s[i] >> 1, sign = s[i] & 1, v = 0;
    for (int j = 0; j < p->cdf_len - 1; ++j) v += (uint16_t)(p->cdf[j] - prnd) >> 15;
    s[i] = (uint16_t)(((uint16_t)(-sign) ^ v) + sign);
  }
}

/* MSB-first packing of d-bit values */
static void pack(uint8_t *out, const uint16_t *in, size_t cnt, int d) {
  uint32_t acc = 0;
  int bits = 0;
  size_t o = 0;
  for (size_t i = 0; i < cnt; ++i) {
    acc = (acc << d) | (in[i] & ((1u << d) - 1));
    bits += d;
    while (bits >= 8) {
      out[o++] = (uint8_t)(acc >> (bits - 8));
      bits -= 8;
    }
  }
}

static void unpack(uint16_t *out, const uint8_t *in, size_t cnt, int d) {
  uint32_t acc = 0;
  int bits = 0;
  size_t p = 0;
  for (size_t i = 0; i < cnt; ++i) {
    while (bits < d) {
      acc = (acc << 8) | in[p++];
      bits += 8;
    }
    out[i] = (uint16_t)((acc >> (bits - d)) & ((1u << d) - 1));
    bits -= d;
  }
}

static void encode_mu(const fparams *p, uint16_t *out, const uint8_t *mu) {
  for (int i = 0; i < NBAR * NBAR; ++i) {
    unsigned bit0 = (unsigned)(p->B * i), v = 0;
    for (int b = 0; b < p->B; ++b) v |= ((mu[(bit0 + b) >> 3] >> ((bit0 + b) & 7)) & 1u) << b;
    out[i] = (uint16_t)(v << (p->logq - p->B));
  }
}

static void decode_mu(const fparams *p, uint8_t *mu, const uint16_t *in) {
  memset(mu, 0, mu_len(p));
  unsigned qmask = (1u << p->logq) - 1;
  for (int i = 0; i < NBAR * NBAR; ++i) {
    unsigned t = (((in[i] & qmask) + (1u << (p->logq - p->B - 1))) >> (p->logq - p->B)) &
                 ((1u << p->B) - 1);
    unsigned bit0 = (unsigned)(p->B * i);
    for (int b = 0; b < p->B; ++b)
      mu[(bit0 + b) >> 3] |= (uint8_t)(((t >> b) & 1u) << ((bit0 + b) & 7));
  }
}

int orc_frodo_keypair_derand(const char *alg, uint8_t *pk, uint8_t *sk, const uint8_t *coins) {
  fparams p;
  if (params_of(alg, &p)) return -1;
  const int n = p.n, sec = p.sec;
  const uint8_t *s = coins, *seed_se = coins + sec, *z = coins + 2 * sec;
  uint8_t *seed_a = pk;
  hashf(&p, seed_a, 16, z, 16);
  uint16_t *SE = (uint16_t *)malloc(2 * (size_t)n * NBAR * 2);
  uint16_t *Bm = (uint16_t *)malloc((size_t)n * NBAR * 2);
  uint16_t *row = (uint16_t *)malloc((size_t)n * 2);
  uint8_t in[1 + 32];
  in[0] = 0x5F;
  memcpy(in + 1, seed_se, sec);
  hashf(&p, (uint8_t *)SE, 2 * (size_t)n * NBAR * 2, in, 1 + sec);
  sample_n(&p, SE, 2 * (size_t)n * NBAR);
  const uint16_t *St = SE, *E = SE + (size_t)n * NBAR; /* St: nbar x n, E: n x nbar */
  for (int i = 0; i < n; ++i) {
    gen_a_row(&p, seed_a, i, row);
    for (int k = 0; k < NBAR; ++k) {
      uint16_t acc = E[(size_t)i * NBAR + k];
      for (int j = 0; j < n; ++j) acc = (uint16_t)(acc + row[j] * St[(size_t)k * n + j]);
      Bm[(size_t)i * NBAR + k] = acc;
    }
  }
  pack(pk + 16, Bm, (size_t)n * NBAR, p.logq);
  memcpy(sk, s, sec);
  memcpy(sk + sec, pk, pk_len(&p));
  memcpy(sk + sec + pk_len(&p), St, (size_t)n * NBAR * 2);
  hashf(&p, sk + sec + pk_len(&p) + (size_t)n * NBAR * 2, sec, pk, pk_len(&p));
  free(SE);
  free(Bm);
  free(row);
  return 0;
}

/* Bp = S'A + E' (nbar x n), C = S'B + E'' + encode(mu) (nbar x nbar), both mod q */
static void encrypt_core(const fparams *p, const uint8_t *pk, const uint8_t *seed_se,
                         const uint8_t *mu, uint16_t *Bp, uint16_t *C) {
  const int n = p->n, sec = p->sec;
  const uint16_t qmask = (uint16_t)((1u << p->logq) - 1);
  size_t rlen = (2 * (size_t)n + NBAR) * NBAR;
  uint16_t *r = (uint16_t *)malloc(rlen * 2);
  uint16_t *row = (uint16_t *)malloc((size_t)n * 2);
  uint16_t *Bpk = (uint16_t *)malloc((size_t)n * NBAR * 2);
  uint8_t in[1 + 32];
  in[0] = 0x96;
  memcpy(in + 1, seed_se, sec);
  hashf(p, (uint8_t *)r, rlen * 2, in, 1 + sec);
  sample_n(p, r, rlen);
  const uint16_t *Sp = r, *Ep = r + (size_t)n * NBAR, *Epp = r + 2 * (size_t)n * NBAR;
  for (size_t t = 0; t < (size_t)n * NBAR; ++t) Bp[t] = Ep[t];
  for (int j = 0; j < n; ++j) {
    gen_a_row(p, pk, j, row);
    for (int k = 0; k < NBAR; ++k) {
      uint16_t s = Sp[(size_t)k * n + j];
      uint16_t *o = Bp + (size_t)k * n;
      for (int i = 0; i < n; ++i) o[i] = (uint16_t)(o[i] + s * row[i]);
    }
  }
  for (size_t t = 0; t < (size_t)n * NBAR; ++t) Bp[t] &= qmask;
  unpack(Bpk, pk + 16, (size_t)n * NBAR, p->logq);
  uint16_t enc[NBAR * NBAR];
  encode_mu(p, enc, mu);
  for (int k = 0; k < NBAR; ++k)
    for (int i = 0; i < NBAR; ++i) {
      uint16_t acc = Epp[k * NBAR + i];
      for (int j = 0; j < n; ++j) acc = (uint16_t)(acc + Sp[(size_t)k * n + j] * Bpk[(size_t)j * NBAR + i]);
      C[k * NBAR + i] = (uint16_t)((acc + enc[k * NBAR + i]) & qmask);
    }
  free(r);
  free(row);
  free(Bpk);
}

int orc_frodo_encaps_derand(const char *alg, uint8_t *ct, uint8_t *ss, const uint8_t *pk,
                            const uint8_t *mu) {
  fparams p;
  if (params_of(alg, &p)) return -1;
  const int n = p.n, sec = p.sec;
  const size_t ml = mu_len(&p), c1 = (size_t)p.logq * n * NBAR / 8, cl = ct_len(&p);
  uint8_t gin[32 + 32], g[64];
  hashf(&p, gin, sec, pk, pk_len(&p));
  memcpy(gin + sec, mu, ml);
  hashf(&p, g, 2 * sec, gin, sec + ml);
  uint16_t *Bp = (uint16_t *)malloc((size_t)n * NBAR * 2);
  uint16_t C[NBAR * NBAR];
  encrypt_core(&p, pk, g, mu, Bp, C);
  pack(ct, Bp, (size_t)n * NBAR, p.logq);
  pack(ct + c1, C, NBAR * NBAR, p.logq);
  uint8_t *fin = (uint8_t *)malloc(cl + sec);
  memcpy(fin, ct, cl);
  memcpy(fin + cl, g + sec, sec);
  hashf(&p, ss, sec, fin, cl + sec);
  free(fin);
  free(Bp);
  return 0;
}

int orc_frodo_decaps(const char *alg, uint8_t *ss, const uint8_t *ct, const uint8_t *sk) {
  fparams p;
  if (params_of(alg, &p)) return -1;
  const int n = p.n, sec = p.sec;
  const uint16_t qmask = (uint16_t)((1u << p.logq) - 1);
  const size_t pl = pk_len(&p), ml = mu_len(&p), c1 = (size_t)p.logq * n * NBAR / 8, cl = ct_len(&p);
  const uint8_t *s = sk, *pk = sk + sec, *Sb = sk + sec + pl, *pkh = sk + sec + pl + (size_t)n * NBAR * 2;
  uint16_t *Bp = (uint16_t *)malloc((size_t)n * NBAR * 2);
  uint16_t *Bp2 = (uint16_t *)malloc((size_t)n * NBAR * 2);
  uint16_t C[NBAR * NBAR], C2[NBAR * NBAR], M[NBAR * NBAR];
  unpack(Bp, ct, (size_t)n * NBAR, p.logq);
  unpack(C, ct + c1, NBAR * NBAR, p.logq);
  for (int a = 0; a < NBAR; ++a)
    for (int b = 0; b < NBAR; ++b) {
      uint16_t acc = 0;
      for (int j = 0; j < n; ++j) {
        uint16_t sv = (uint16_t)(Sb[2 * ((size_t)b * n + j)] | (Sb[2 * ((size_t)b * n + j) + 1] << 8));
        acc = (uint16_t)(acc + Bp[(size_t)a * n + j] * sv);
      }
      M[a * NBAR + b] = (uint16_t)((C[a * NBAR + b] - acc) & qmask);
    }
  uint8_t gin[64], g[64];
  memcpy(gin, pkh, sec);
  decode_mu(&p, gin + sec, M);
  hashf(&p, g, 2 * sec, gin, sec + ml);
  encrypt_core(&p, pk, g, gin + sec, Bp2, C2);
  uint16_t diff = 0;
  for (size_t t = 0; t < (size_t)n * NBAR; ++t) diff |= (uint16_t)(Bp[t] ^ Bp2[t]);
  for (int t = 0; t < NBAR * NBAR; ++t) diff |= (uint16_t)(C[t] ^ C2[t]);
  uint8_t mask = (uint8_t)(((uint32_t)diff - 1u) >> 24); /* 0xFF iff equal */
  uint8_t *fin = (uint8_t *)malloc(cl + sec);
  memcpy(fin, ct, cl);
  for (int i = 0; i < sec; ++i) fin[cl + i] = (uint8_t)((g[sec + i] & mask) | (s[i] & ~mask));
  hashf(&p, ss, sec, fin, cl + sec);
  free(fin);
  free(Bp);
  free(Bp2);
  return 0;
}
