/* HQC (round-4 submission, version 2023-04-30) -- oracle / CPU-baseline only.
 *
 * TEST INFRASTRUCTURE: compiled into oracle/liboracle.so, which only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg load.
 *
 * The reference selects HQC at quantum_resistant_p2p/crypto/key_exchange.py:189-309
 * (names :206-223) and calls liboqs through vendor/oqs.py:318,348,372.  liboqs 0.12
 * vendors the 2023-04-30 HQC reference implementation; it is absent here and the
 * reference holds no HQC vectors: PARITY UNPINNED.  This file
 * restates the published algorithm independently of oracle/py/hqc_spec.py (pure
 * Python, same conventions, documented there); tests/test_hqc_oracle.py holds the
 * two against each other and against the code's algebraic properties.
 *
 * Layout: vectors of F2[X]/(X^n-1) as little-endian uint64 words (bit i = X^i).
 */
#include <stdlib.h>
#include <string.h>

#include "fips202.h"

#define SEED 40
#define SALT 16
#define SSB 64

typedef struct {
  int n, n1, n2, w, wr, we, k, delta, mult;
} hparams;

static int hparams_of(const char *alg, hparams *p) {
  static const struct {
    const char *name;
    hparams p;
  } T[] = {
      {"HQC-128", {17669, 46, 384, 66, 75, 75, 16, 15, 3}},
      {"HQC-192", {35851, 56, 640, 100, 114, 114, 24, 16, 5}},
      {"HQC-256", {57637, 90, 640, 131, 149, 149, 32, 29, 5}},
  };
  for (size_t i = 0; i < sizeof T / sizeof T[0]; ++i)
    if (!strcmp(T[i].name, alg)) {
      *p = T[i].p;
      return 0;
    }
  return -1;
}

static size_t nbytes(const hparams *p) { return ((size_t)p->n + 7) / 8; }
static size_t vbytes(const hparams *p) { return (size_t)p->n1 * p->n2 / 8; }
static size_t nwords(const hparams *p) { return ((size_t)p->n + 63) / 64; }

int orc_hqc_sizes(const char *alg, size_t out[6]) {
  hparams p;
  if (hparams_of(alg, &p)) return -1;
  out[0] = SEED + nbytes(&p);                    /* pk = pk_seed || s */
  out[1] = SEED + (size_t)p.k + out[0];          /* sk = sk_seed || sigma || pk */
  out[2] = nbytes(&p) + vbytes(&p) + SALT;       /* ct = u || v || salt */
  out[3] = SSB;
  out[4] = 2 * SEED + (size_t)p.k;               /* keypair coins: sk_seed || sigma || pk_seed */
  out[5] = (size_t)p.k + SALT;                   /* encaps coins: m || salt */
  return 0;
}

/* ---------------------------------------------------------------- GF(2^8) */
static uint8_t GEXP[512], GLOG[256];
static int g_init;
static void gf_init(void) {
  if (g_init) return;
  unsigned x = 1;
  for (int i = 0; i < 255; ++i) {
    GEXP[i] = (uint8_t)x;
    GLOG[x] = (uint8_t)i;
    x <<= 1;
    if (x & 0x100) x ^= 0x11D;
  }
  for (int i = 255; i < 512; ++i) GEXP[i] = GEXP[i - 255];
  g_init = 1;
}
static uint8_t gmul(uint8_t a, uint8_t b) { return (a && b) ? GEXP[GLOG[a] + GLOG[b]] : 0; }
static uint8_t ginv(uint8_t a) { return GEXP[255 - GLOG[a]]; }

/* ---------------------------------------------------------------- SHAKE helpers */
typedef struct {
  orc_keccak k;
} sexp;

static void sexp_init(sexp *s, const uint8_t *seed) {
  const uint8_t d = 2;
  orc_keccak_init(&s->k, ORC_SHAKE256_RATE);
  orc_keccak_absorb(&s->k, seed, SEED);
  orc_keccak_absorb(&s->k, &d, 1);
  orc_keccak_finalize(&s->k, 0x1F);
}
/* squeeze in 8-byte units: L bytes consume ceil(L/8)*8 */
static void sexp_read(sexp *s, uint8_t *out, size_t len) {
  const size_t full = len & ~(size_t)7;
  orc_keccak_squeeze(&s->k, out, full);
  if (len != full) {
    uint8_t t[8];
    orc_keccak_squeeze(&s->k, t, 8);
    memcpy(out + full, t, len - full);
  }
}

static void shake_ds(uint8_t out[SSB], const uint8_t *a, size_t al, const uint8_t *b, size_t bl,
                     const uint8_t *c, size_t cl, uint8_t domain) {
  orc_keccak k;
  orc_keccak_init(&k, ORC_SHAKE256_RATE);
  orc_keccak_absorb(&k, a, al);
  orc_keccak_absorb(&k, b, bl);
  orc_keccak_absorb(&k, c, cl);
  orc_keccak_absorb(&k, &domain, 1);
  orc_keccak_finalize(&k, 0x1F);
  orc_keccak_squeeze(&k, out, SSB);
}

/* ---------------------------------------------------------------- vectors */
static void fixed_weight(sexp *s, const hparams *p, int weight, uint32_t *sup) {
  uint8_t raw[4 * 160];
  sexp_read(s, raw, 4 * (size_t)weight);
  for (int i = 0; i < weight; ++i) {
    uint32_t r = (uint32_t)raw[4 * i] | (uint32_t)raw[4 * i + 1] << 8 | (uint32_t)raw[4 * i + 2] << 16 |
                 (uint32_t)raw[4 * i + 3] << 24;
    sup[i] = (uint32_t)i + (uint32_t)(((uint64_t)r * (uint64_t)(p->n - i)) >> 32);
  }
  for (int i = weight - 2; i >= 0; --i) {
    int found = 0;
    for (int j = i + 1; j < weight; ++j) found |= sup[j] == sup[i];
    if (found) sup[i] = (uint32_t)i;
  }
}

static void load_bytes(uint64_t *v, size_t words, const uint8_t *b, size_t len) {
  memset(v, 0, words * 8);
  for (size_t i = 0; i < len; ++i) v[i / 8] |= (uint64_t)b[i] << (8 * (i % 8));
}
static void store_bytes(uint8_t *b, size_t len, const uint64_t *v) {
  for (size_t i = 0; i < len; ++i) b[i] = (uint8_t)(v[i / 8] >> (8 * (i % 8)));
}
static void set_support(uint64_t *v, const uint32_t *sup, int weight) {
  for (int i = 0; i < weight; ++i) v[sup[i] / 64] |= (uint64_t)1 << (sup[i] % 64);
}

/* 64 bits of a starting at bit position pos (a has `words` words, zero beyond) */
static uint64_t bits_at(const uint64_t *a, size_t words, size_t pos) {
  const size_t w = pos / 64, s = pos % 64;
  const uint64_t lo = w < words ? a[w] : 0, hi = w + 1 < words ? a[w + 1] : 0;
  return s ? (lo >> s) | (hi << (64 - s)) : lo;
}

/* out = sup * b mod X^n - 1, folding the linear product once as the reference's
 * vect_mul reduction does (b may carry stray bits above X^(n-1) when read from a pk/ct) */
static void mul_sparse(uint64_t *out, const uint32_t *sup, int weight, const uint64_t *b, const hparams *p) {
  const size_t W = nwords(p), L = 2 * W + 2;
  uint64_t *a = (uint64_t *)calloc(L, 8);
  for (int t = 0; t < weight; ++t) {
    const size_t ws = sup[t] / 64, bs = sup[t] % 64;
    for (size_t i = 0; i < W; ++i) {
      a[i + ws] ^= b[i] << bs;
      if (bs) a[i + ws + 1] ^= b[i] >> (64 - bs);
    }
  }
  for (size_t i = 0; i < W; ++i) out[i] = a[i] ^ bits_at(a, L, (size_t)p->n + 64 * i);
  out[W - 1] &= ((uint64_t)1 << (p->n % 64)) - 1;
  free(a);
}

/* ---------------------------------------------------------------- code */
static void rs_generator(const hparams *p, uint8_t *g) {
  const int t2 = 2 * p->delta;
  memset(g, 0, (size_t)t2 + 1);
  g[0] = 1;
  for (int i = 1; i <= t2; ++i) { /* g *= (x + alpha^i) */
    const uint8_t a = GEXP[i];
    for (int j = i; j >= 1; --j) g[j] = g[j - 1] ^ gmul(g[j], a);
    g[0] = gmul(g[0], a);
  }
}

static void rs_encode(const hparams *p, const uint8_t *msg, uint8_t *cdw) {
  uint8_t g[64];
  rs_generator(p, g);
  const int par = p->n1 - p->k;
  memset(cdw, 0, (size_t)p->n1);
  for (int i = 0; i < p->k; ++i) {
    const uint8_t gate = msg[p->k - 1 - i] ^ cdw[par - 1];
    for (int j = par - 1; j > 0; --j) cdw[j] = cdw[j - 1] ^ gmul(gate, g[j]);
    cdw[0] = gmul(gate, g[0]);
  }
  memcpy(cdw + par, msg, (size_t)p->k);
}

/* RM(1,7) codeword of symbol b as four 32-bit words: bit j = b7 ^ <b0..6, j> */
static void rm_word(uint8_t b, uint32_t w[4]) {
  uint32_t base = (uint32_t)0 - (uint32_t)(b >> 7 & 1);
  static const uint32_t M[5] = {0xaaaaaaaau, 0xccccccccu, 0xf0f0f0f0u, 0xff00ff00u, 0xffff0000u};
  for (int i = 0; i < 5; ++i) base ^= ((uint32_t)0 - (uint32_t)(b >> i & 1)) & M[i];
  for (int q = 0; q < 4; ++q)
    w[q] = base ^ (((uint32_t)0 - (uint32_t)(b >> 5 & 1)) & ((uint32_t)0 - (uint32_t)(q & 1))) ^
           (((uint32_t)0 - (uint32_t)(b >> 6 & 1)) & ((uint32_t)0 - (uint32_t)(q >> 1 & 1)));
}

static void code_encode(const hparams *p, const uint8_t *msg, uint64_t *v /* >= n words, zeroed */) {
  uint8_t cdw[128];
  rs_encode(p, msg, cdw);
  for (int i = 0; i < p->n1; ++i) {
    uint32_t w[4];
    rm_word(cdw[i], w);
    for (int c = 0; c < p->mult; ++c) {
      const size_t base = ((size_t)i * p->mult + c) * 2; /* uint64 index of the 128-bit copy */
      v[base] = (uint64_t)w[0] | (uint64_t)w[1] << 32;
      v[base + 1] = (uint64_t)w[2] | (uint64_t)w[3] << 32;
    }
  }
}

static uint8_t rm_decode(const uint64_t *src, int mult) {
  int t[128], u[128];
  for (int j = 0; j < 128; ++j) {
    int c = 0;
    for (int k = 0; k < mult; ++k) c += (int)(src[2 * k + j / 64] >> (j % 64) & 1);
    t[j] = c;
  }
  for (int h = 1; h < 128; h <<= 1) { /* Walsh-Hadamard, natural order */
    for (int i0 = 0; i0 < 128; i0 += 2 * h)
      for (int i = i0; i < i0 + h; ++i) {
        const int a = t[i], b = t[i + h];
        u[i] = a + b;
        u[i + h] = a - b;
      }
    memcpy(t, u, sizeof t);
  }
  t[0] -= 64 * mult;
  int best = 0, val = 0, pos = 0;
  for (int i = 0; i < 128; ++i) {
    const int a = t[i] < 0 ? -t[i] : t[i];
    if (a > best) best = a, val = t[i], pos = i;
  }
  return (uint8_t)(pos | (val > 0 ? 128 : 0));
}

static uint8_t poly_eval(const uint8_t *c, int deg, uint8_t x) {
  uint8_t acc = 0;
  for (int i = deg; i >= 0; --i) acc = gmul(acc, x) ^ c[i];
  return acc;
}

/* bounded-distance decoding: syndromes, Berlekamp-Massey, Chien search, Forney */
static void rs_decode(const hparams *p, uint8_t *r) {
  const int t2 = 2 * p->delta;
  uint8_t S[64], C[65] = {1}, B[65] = {1}, T[65], om[64], dv[65];
  for (int i = 0; i < t2; ++i) S[i] = poly_eval(r, p->n1 - 1, GEXP[i + 1]);
  int L = 0, m = 1;
  uint8_t b = 1;
  for (int i = 0; i < t2; ++i) {
    uint8_t d = S[i];
    for (int j = 1; j <= L; ++j) d ^= gmul(C[j], S[i - j]);
    if (!d) {
      ++m;
      continue;
    }
    const uint8_t coef = gmul(d, ginv(b));
    memcpy(T, C, sizeof T);
    for (int j = 0; j + m <= t2; ++j) C[j + m] ^= gmul(coef, B[j]);
    if (2 * L <= i) {
      L = i + 1 - L;
      memcpy(B, T, sizeof B);
      b = d;
      m = 1;
    } else {
      ++m;
    }
  }
  for (int i = 0; i < t2; ++i) {
    om[i] = 0;
    for (int j = 0; j <= i; ++j) om[i] ^= gmul(S[i - j], C[j]);
  }
  for (int j = 0; j < t2; ++j) dv[j] = (j % 2 == 0) ? C[j + 1] : 0; /* C'(x) */
  for (int pos = 0; pos < p->n1; ++pos) {
    const uint8_t xinv = GEXP[(255 - pos) % 255];
    if (poly_eval(C, t2, xinv)) continue;
    const uint8_t den = poly_eval(dv, t2 - 1, xinv);
    if (den) r[pos] ^= gmul(poly_eval(om, t2 - 1, xinv), ginv(den));
  }
}

static void code_decode(const hparams *p, const uint64_t *v, uint8_t *msg) {
  uint8_t r[128];
  for (int i = 0; i < p->n1; ++i) r[i] = rm_decode(v + (size_t)i * p->mult * 2, p->mult);
  rs_decode(p, r);
  memcpy(msg, r + p->n1 - p->k, (size_t)p->k);
}

/* ---------------------------------------------------------------- PKE / KEM */
static void random_h(const hparams *p, const uint8_t *pk_seed, uint64_t *h) {
  sexp s;
  uint8_t *buf = (uint8_t *)malloc(nbytes(p));
  sexp_init(&s, pk_seed);
  sexp_read(&s, buf, nbytes(p));
  load_bytes(h, nwords(p), buf, nbytes(p));
  h[nwords(p) - 1] &= ((uint64_t)1 << (p->n % 64)) - 1;
  free(buf);
}

/* u (nbytes), v (vbytes) of Encrypt(pk, m, theta) */
static void pke_encrypt(const hparams *p, const uint8_t *m, const uint8_t *theta, const uint8_t *pk,
                        uint8_t *ub, uint8_t *vb) {
  const size_t W = nwords(p);
  uint64_t *h = calloc(W, 8), *s = calloc(W, 8), *u = calloc(W, 8), *t = calloc(W, 8), *cw = calloc(W, 8);
  uint32_t r1[160], r2[160], e[160];
  sexp se;
  sexp_init(&se, theta);
  fixed_weight(&se, p, p->wr, r1);
  fixed_weight(&se, p, p->wr, r2);
  fixed_weight(&se, p, p->we, e);
  random_h(p, pk, h);
  load_bytes(s, W, pk + SEED, nbytes(p));
  mul_sparse(u, r2, p->wr, h, p);
  set_support(t, r1, p->wr);
  for (size_t i = 0; i < W; ++i) u[i] ^= t[i];
  store_bytes(ub, nbytes(p), u);
  memset(u, 0, W * 8);
  mul_sparse(t, r2, p->wr, s, p);
  code_encode(p, m, cw);
  set_support(u, e, p->we); /* u reused (already stored): e as a vector, added by XOR */
  for (size_t i = 0; i < W; ++i) t[i] ^= cw[i] ^ u[i];
  store_bytes(vb, vbytes(p), t);
  free(h), free(s), free(u), free(t), free(cw);
}

int orc_hqc_keypair_derand(const char *alg, uint8_t *pk, uint8_t *sk, const uint8_t *coins) {
  hparams p;
  if (hparams_of(alg, &p)) return -1;
  gf_init();
  const size_t W = nwords(&p);
  const uint8_t *sk_seed = coins, *sigma = coins + SEED, *pk_seed = coins + SEED + p.k;
  uint64_t *h = calloc(W, 8), *s = calloc(W, 8), *x = calloc(W, 8);
  uint32_t xs[160], ys[160];
  sexp se;
  sexp_init(&se, sk_seed);
  fixed_weight(&se, &p, p.w, xs);
  fixed_weight(&se, &p, p.w, ys);
  random_h(&p, pk_seed, h);
  mul_sparse(s, ys, p.w, h, &p);
  set_support(x, xs, p.w);
  for (size_t i = 0; i < W; ++i) s[i] ^= x[i];
  memcpy(pk, pk_seed, SEED);
  store_bytes(pk + SEED, nbytes(&p), s);
  memcpy(sk, sk_seed, SEED);
  memcpy(sk + SEED, sigma, (size_t)p.k);
  memcpy(sk + SEED + p.k, pk, SEED + nbytes(&p));
  free(h), free(s), free(x);
  return 0;
}

int orc_hqc_encaps_derand(const char *alg, uint8_t *ct, uint8_t *ss, const uint8_t *pk, const uint8_t *coins) {
  hparams p;
  if (hparams_of(alg, &p)) return -1;
  gf_init();
  const uint8_t *m = coins, *salt = coins + p.k;
  uint8_t theta[SSB];
  shake_ds(theta, m, (size_t)p.k, pk, 2 * SEED, salt, SALT, 3);
  pke_encrypt(&p, m, theta, pk, ct, ct + nbytes(&p));
  memcpy(ct + nbytes(&p) + vbytes(&p), salt, SALT);
  shake_ds(ss, m, (size_t)p.k, ct, nbytes(&p), ct + nbytes(&p), vbytes(&p), 5);
  return 0;
}

/* returns 0, or -1 when the re-encryption differs (ss = K(sigma || u || v) is still written) */
int orc_hqc_decaps(const char *alg, uint8_t *ss, const uint8_t *ct, const uint8_t *sk) {
  hparams p;
  if (hparams_of(alg, &p)) return -1;
  gf_init();
  const size_t W = nwords(&p), NB = nbytes(&p), VB = vbytes(&p);
  const uint8_t *sigma = sk + SEED, *pk = sk + SEED + p.k, *salt = ct + NB + VB;
  uint64_t *u = calloc(W + 1, 8), *t = calloc(W, 8), *v = calloc(W, 8);
  uint32_t xs[160], ys[160];
  sexp se;
  sexp_init(&se, sk);
  fixed_weight(&se, &p, p.w, xs);
  fixed_weight(&se, &p, p.w, ys);
  load_bytes(u, W, ct, NB); /* unmasked, as the reference loads it */
  load_bytes(v, W, ct + NB, VB);
  mul_sparse(t, ys, p.w, u, &p);
  for (size_t i = 0; i < W; ++i) t[i] ^= v[i];
  uint8_t m1[32], theta[SSB], mc[32];
  code_decode(&p, t, m1);
  shake_ds(theta, m1, (size_t)p.k, pk, 2 * SEED, salt, SALT, 3);
  uint8_t *u2 = malloc(NB), *v2 = malloc(VB);
  pke_encrypt(&p, m1, theta, pk, u2, v2);
  uint8_t diff = 0;
  for (size_t i = 0; i < NB; ++i) diff |= u2[i] ^ ct[i];
  for (size_t i = 0; i < VB; ++i) diff |= v2[i] ^ ct[NB + i];
  const uint8_t ok = (uint8_t)(((unsigned)diff - 1u) >> 8); /* 0xFF when equal */
  for (int i = 0; i < p.k; ++i) mc[i] = (uint8_t)((m1[i] & ok) | (sigma[i] & ~ok));
  shake_ds(ss, mc, (size_t)p.k, ct, NB, ct + NB, VB, 5);
  free(u), free(t), free(v), free(u2), free(v2);
  return ok ? 0 : -1;
}
