/* SHA-256 (FIPS 180-4), HMAC-SHA256 (RFC 2104) and HKDF-SHA256 (RFC 5869) plus a
 * batched protocol-handshake driver -- TEST INFRASTRUCTURE ONLY (oracle/liboracle.so).
 *
 * Restates what the reference runs after every key exchange:
 * SecureMessaging._derive_symmetric_key (quantum_resistant_p2p/app/messaging.py:350-382)
 *   HKDF(algorithm=hashes.SHA256(), length=key_size, salt=None, info=info).derive(ss)
 * from the `cryptography` package (a dependency absent from this image: the algorithm is
 * RFC 5869's, pinned by its SHA-256 test cases 1-3 in tests/test_handshake_oracle.py),
 * and the per-handshake operation order of messaging.py:590 (initiator KeyGen), :809
 * (responder KeyGen), :830 (Encaps), :845 (HKDF), :1038 (Decaps), :1068 (HKDF).
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

int orc_sizes(const char *alg, size_t out[6]);
int orc_keypair(const char *alg, uint8_t *pk, uint8_t *sk, const uint8_t *coins);
int orc_encaps(const char *alg, uint8_t *ct, uint8_t *ss, const uint8_t *pk, const uint8_t *coins);
int orc_decaps(const char *alg, uint8_t *ss, const uint8_t *ct, const uint8_t *sk);

static const uint32_t K[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

typedef struct {
  uint32_t h[8];
  uint8_t buf[64];
  size_t fill;
  uint64_t total;
} sha256_ctx;

#define ROTR(x, n) (((x) >> (n)) | ((x) << (32 - (n))))

/* FIPS 180-4 section 6.2.2 */
static void compress(uint32_t h[8], const uint8_t blk[64]) {
  uint32_t w[64];
  for (int t = 0; t < 16; ++t)
    w[t] = (uint32_t)blk[4 * t] << 24 | (uint32_t)blk[4 * t + 1] << 16 | (uint32_t)blk[4 * t + 2] << 8 |
           blk[4 * t + 3];
  for (int t = 16; t < 64; ++t) {
    uint32_t s0 = ROTR(w[t - 15], 7) ^ ROTR(w[t - 15], 18) ^ (w[t - 15] >> 3);
    uint32_t s1 = ROTR(w[t - 2], 17) ^ ROTR(w[t - 2], 19) ^ (w[t - 2] >> 10);
    w[t] = w[t - 16] + s0 + w[t - 7] + s1;
  }
  uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
  for (int t = 0; t < 64; ++t) {
    uint32_t t1 = hh + (ROTR(e, 6) ^ ROTR(e, 11) ^ ROTR(e, 25)) + ((e & f) ^ (~e & g)) + K[t] + w[t];
    uint32_t t2 = (ROTR(a, 2) ^ ROTR(a, 13) ^ ROTR(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
    hh = g, g = f, f = e, e = d + t1, d = c, c = b, b = a, a = t1 + t2;
  }
  h[0] += a, h[1] += b, h[2] += c, h[3] += d, h[4] += e, h[5] += f, h[6] += g, h[7] += hh;
}

static void sha_init(sha256_ctx *c) {
  static const uint32_t H0[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                                 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  memcpy(c->h, H0, sizeof H0);
  c->fill = 0;
  c->total = 0;
}
static void sha_update(sha256_ctx *c, const uint8_t *p, size_t n) {
  c->total += n;
  while (n) {
    size_t t = 64 - c->fill < n ? 64 - c->fill : n;
    memcpy(c->buf + c->fill, p, t);
    c->fill += t, p += t, n -= t;
    if (c->fill == 64) compress(c->h, c->buf), c->fill = 0;
  }
}
static void sha_final(sha256_ctx *c, uint8_t out[32]) {
  uint64_t bits = c->total * 8;
  uint8_t pad = 0x80, z = 0;
  sha_update(c, &pad, 1);
  while (c->fill != 56) sha_update(c, &z, 1);
  uint8_t len[8];
  for (int i = 0; i < 8; ++i) len[i] = (uint8_t)(bits >> (56 - 8 * i));
  sha_update(c, len, 8);
  for (int i = 0; i < 8; ++i)
    out[4 * i] = (uint8_t)(c->h[i] >> 24), out[4 * i + 1] = (uint8_t)(c->h[i] >> 16),
            out[4 * i + 2] = (uint8_t)(c->h[i] >> 8), out[4 * i + 3] = (uint8_t)c->h[i];
}

void orc_sha256(uint8_t out[32], const uint8_t *in, size_t n) {
  sha256_ctx c;
  sha_init(&c);
  sha_update(&c, in, n);
  sha_final(&c, out);
}

/* RFC 2104 with B = 64, L = 32.  The message is the concatenation of up to three parts. */
static void hmac3(uint8_t out[32], const uint8_t *key, size_t klen, const uint8_t *m1, size_t n1,
                  const uint8_t *m2, size_t n2, const uint8_t *m3, size_t n3) {
  uint8_t k0[64] = {0}, pad[64], inner[32];
  if (klen > 64)
    orc_sha256(k0, key, klen);
  else if (klen)
    memcpy(k0, key, klen);
  sha256_ctx c;
  for (int i = 0; i < 64; ++i) pad[i] = k0[i] ^ 0x36;
  sha_init(&c);
  sha_update(&c, pad, 64);
  if (n1) sha_update(&c, m1, n1);
  if (n2) sha_update(&c, m2, n2);
  if (n3) sha_update(&c, m3, n3);
  sha_final(&c, inner);
  for (int i = 0; i < 64; ++i) pad[i] = k0[i] ^ 0x5c;
  sha_init(&c);
  sha_update(&c, pad, 64);
  sha_update(&c, inner, 32);
  sha_final(&c, out);
}

/* RFC 5869 section 2.2-2.3.  salt NULL / 0 length = HashLen zero bytes (same HMAC key). */
int orc_hkdf_sha256(uint8_t *okm, size_t L, const uint8_t *ikm, size_t ikm_len, const uint8_t *salt,
                    size_t salt_len, const uint8_t *info, size_t info_len) {
  if (L == 0 || L > 255 * 32) return -1;
  uint8_t prk[32], t[32];
  hmac3(prk, salt, salt ? salt_len : 0, ikm, ikm_len, NULL, 0, NULL, 0);
  size_t done = 0;
  for (unsigned i = 1; done < L; ++i) {
    uint8_t ctr = (uint8_t)i;
    hmac3(t, prk, 32, t, i > 1 ? 32 : 0, info, info_len, &ctr, 1);
    size_t take = L - done < 32 ? L - done : 32;
    memcpy(okm + done, t, take);
    done += take;
  }
  return 0;
}

/* ---- batched drivers (pthread) ---- */
typedef struct {
  size_t lo, hi;
  const char *alg;
  size_t sz[6];
  const uint8_t *ikm;
  size_t ikm_len;
  const uint8_t *salt;
  size_t salt_len;
  const uint8_t *info;
  const uint64_t *info_off;
  size_t info_len, L;
  uint8_t *okm;
  /* handshake */
  const uint8_t *c_kpi, *c_kpr, *c_enc;
  uint8_t *pk_i, *pk_r, *ct, *key_i, *key_r;
  int rc;
} hjob;

static void info_of(const hjob *j, size_t i, const uint8_t **p, size_t *n) {
  if (j->info_off) {
    *p = j->info + j->info_off[i];
    *n = (size_t)(j->info_off[i + 1] - j->info_off[i]);
  } else {
    *p = j->info;
    *n = j->info_len;
  }
}

static void *run_hkdf(void *arg) {
  hjob *j = (hjob *)arg;
  for (size_t i = j->lo; i < j->hi; ++i) {
    const uint8_t *inf;
    size_t il;
    info_of(j, i, &inf, &il);
    if (orc_hkdf_sha256(j->okm + i * j->L, j->L, j->ikm + i * j->ikm_len, j->ikm_len, j->salt, j->salt_len, inf,
                        il))
      j->rc = -1;
  }
  return NULL;
}

static void *run_handshake(void *arg) {
  hjob *j = (hjob *)arg;
  const size_t PK = j->sz[0], SK = j->sz[1], CT = j->sz[2], SS = j->sz[3], KC = j->sz[4], EC = j->sz[5];
  uint8_t *sk_i = malloc(SK), *sk_r = malloc(SK), ss_i[64], ss_r[64];
  for (size_t i = j->lo; i < j->hi; ++i) {
    const uint8_t *inf;
    size_t il;
    info_of(j, i, &inf, &il);
    int rc = orc_keypair(j->alg, j->pk_i + i * PK, sk_i, j->c_kpi + i * KC);
    rc |= orc_keypair(j->alg, j->pk_r + i * PK, sk_r, j->c_kpr + i * KC);
    rc |= orc_encaps(j->alg, j->ct + i * CT, ss_r, j->pk_i + i * PK, j->c_enc + i * EC);
    rc |= orc_hkdf_sha256(j->key_r + i * j->L, j->L, ss_r, SS, NULL, 0, inf, il);
    rc |= orc_decaps(j->alg, ss_i, j->ct + i * CT, sk_i);
    rc |= orc_hkdf_sha256(j->key_i + i * j->L, j->L, ss_i, SS, NULL, 0, inf, il);
    if (rc) j->rc = -1;
  }
  free(sk_i);
  free(sk_r);
  return NULL;
}

static int spawn(size_t n, int nthreads, hjob *tmpl, void *(*fn)(void *)) {
  if (nthreads < 1) nthreads = 1;
  if ((size_t)nthreads > n && n > 0) nthreads = (int)n;
  hjob *jobs = calloc((size_t)nthreads, sizeof(hjob));
  pthread_t *th = calloc((size_t)nthreads, sizeof(pthread_t));
  for (int t = 0; t < nthreads; ++t) {
    jobs[t] = *tmpl;
    jobs[t].lo = n * t / nthreads;
    jobs[t].hi = n * (t + 1) / nthreads;
    jobs[t].rc = 0;
    pthread_create(&th[t], NULL, fn, &jobs[t]);
  }
  int rc = 0;
  for (int t = 0; t < nthreads; ++t) {
    pthread_join(th[t], NULL);
    if (jobs[t].rc) rc = -1;
  }
  free(jobs);
  free(th);
  return rc;
}

int orc_hkdf_batch(size_t n, int nthreads, const uint8_t *ikm, size_t ikm_len, const uint8_t *salt, size_t salt_len,
                   const uint8_t *info, const uint64_t *info_off, size_t info_len, uint8_t *okm, size_t L) {
  hjob j;
  memset(&j, 0, sizeof j);
  j.ikm = ikm, j.ikm_len = ikm_len, j.salt = salt, j.salt_len = salt_len;
  j.info = info, j.info_off = info_off, j.info_len = info_len, j.okm = okm, j.L = L;
  return spawn(n, nthreads, &j, run_hkdf);
}

int orc_handshake_batch(const char *alg, size_t n, int nthreads, const uint8_t *c_kpi, const uint8_t *c_kpr,
                        const uint8_t *c_enc, const uint8_t *info, const uint64_t *info_off, size_t info_len,
                        size_t key_len, uint8_t *pk_i, uint8_t *pk_r, uint8_t *ct, uint8_t *key_i, uint8_t *key_r) {
  hjob j;
  memset(&j, 0, sizeof j);
  if (orc_sizes(alg, j.sz)) return -1;
  j.alg = alg;
  j.info = info, j.info_off = info_off, j.info_len = info_len, j.L = key_len;
  j.c_kpi = c_kpi, j.c_kpr = c_kpr, j.c_enc = c_enc;
  j.pk_i = pk_i, j.pk_r = pk_r, j.ct = ct, j.key_i = key_i, j.key_r = key_r;
  return spawn(n, nthreads, &j, run_handshake);
}
