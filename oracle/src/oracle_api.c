/* ctypes-facing entry points of oracle/liboracle.so -- TEST INFRASTRUCTURE ONLY.
 *
 * Loaded by tests/, __graft_entry__.smoke() (as the checker) and bench.py's
 * cpu_baseline leg.  Never linked into the product library.
 *
 *  - single-record derandomised KEM calls dispatching on the liboqs algorithm
 *    name (the names the reference selects at
 *    quantum_resistant_p2p/crypto/key_exchange.py:75-79, 332-343);
 *  - a pthread-parallel batch driver over AoS [n][len] buffers, used as the
 *    host-core baseline ("kind": "port");
 *  - the per-index bench coin derivation (SHAKE256("qrk-bench"||LE64 seed||LE64 i))
 *    the GPU library also implements, so the device inputs can be checked;
 *  - the NIST KAT DRBG.
 */
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "fips202.h"
#include "mlkem.h"

static int is_mlkem(const char *alg) { return !strncmp(alg, "ML-KEM-", 7); }
static int is_hqc(const char *alg) { return !strncmp(alg, "HQC-", 4); }

int orc_hqc_sizes(const char *alg, size_t out[6]);
int orc_hqc_keypair_derand(const char *alg, uint8_t *pk, uint8_t *sk, const uint8_t *coins);
int orc_hqc_encaps_derand(const char *alg, uint8_t *ct, uint8_t *ss, const uint8_t *pk, const uint8_t *coins);
int orc_hqc_decaps(const char *alg, uint8_t *ss, const uint8_t *ct, const uint8_t *sk);

int orc_sizes(const char *alg, size_t out[6]) {
  if (is_hqc(alg)) return orc_hqc_sizes(alg, out);
  if (is_mlkem(alg)) {
    if (orc_mlkem_sizes(alg, &out[0], &out[1], &out[2], &out[3])) return -1;
    out[4] = 64;
    out[5] = 32;
    return 0;
  }
  return orc_frodo_sizes(alg, &out[0], &out[1], &out[2], &out[3], &out[4], &out[5]);
}

int orc_keypair(const char *alg, uint8_t *pk, uint8_t *sk, const uint8_t *coins) {
  if (is_hqc(alg)) return orc_hqc_keypair_derand(alg, pk, sk, coins);
  return is_mlkem(alg) ? orc_mlkem_keypair_derand(alg, pk, sk, coins)
                       : orc_frodo_keypair_derand(alg, pk, sk, coins);
}
int orc_encaps(const char *alg, uint8_t *ct, uint8_t *ss, const uint8_t *pk, const uint8_t *coins) {
  if (is_hqc(alg)) return orc_hqc_encaps_derand(alg, ct, ss, pk, coins);
  return is_mlkem(alg) ? orc_mlkem_encaps_derand(alg, ct, ss, pk, coins)
                       : orc_frodo_encaps_derand(alg, ct, ss, pk, coins);
}
/* HQC returns -1 when the re-encryption check fails (ss is still written), as liboqs does */
int orc_decaps(const char *alg, uint8_t *ss, const uint8_t *ct, const uint8_t *sk) {
  if (is_hqc(alg)) return orc_hqc_decaps(alg, ss, ct, sk);
  return is_mlkem(alg) ? orc_mlkem_decaps(alg, ss, ct, sk) : orc_frodo_decaps(alg, ss, ct, sk);
}

/* ---- threaded batch driver ---- */
enum { OP_KEYPAIR = 0, OP_ENCAPS = 1, OP_DECAPS = 2 };

typedef struct {
  const char *alg;
  int op;
  size_t lo, hi;
  uint8_t *a, *b;
  const uint8_t *c, *d;
  size_t sz[6];
  int32_t *status; /* optional per-record return code */
  int rc;
} job;

static void *run_job(void *arg) {
  job *j = (job *)arg;
  const size_t PK = j->sz[0], SK = j->sz[1], CT = j->sz[2], SS = j->sz[3], KC = j->sz[4],
               EC = j->sz[5];
  j->rc = 0;
  for (size_t i = j->lo; i < j->hi; ++i) {
    int rc = 0;
    switch (j->op) {
      case OP_KEYPAIR: /* a=pk b=sk c=coins */
        rc = orc_keypair(j->alg, j->a + i * PK, j->b + i * SK, j->c + i * KC);
        break;
      case OP_ENCAPS: /* a=ct b=ss c=pk d=coins */
        rc = orc_encaps(j->alg, j->a + i * CT, j->b + i * SS, j->c + i * PK, j->d + i * EC);
        break;
      case OP_DECAPS: /* a=ss c=ct d=sk */
        rc = orc_decaps(j->alg, j->a + i * SS, j->c + i * CT, j->d + i * SK);
        break;
    }
    if (j->status) j->status[i] = rc;
    else if (rc) j->rc = rc;
  }
  return NULL;
}

/* op: 0 keypair(pk=a, sk=b, coins=c); 1 encaps(ct=a, ss=b, pk=c, coins=d);
 *     2 decaps(ss=a, ct=c, sk=d).  Returns 0 or -1. */
int orc_batch_status(const char *alg, int op, size_t n, int nthreads, uint8_t *a, uint8_t *b,
                     const uint8_t *c, const uint8_t *d, int32_t *status);
int orc_batch(const char *alg, int op, size_t n, int nthreads, uint8_t *a, uint8_t *b,
              const uint8_t *c, const uint8_t *d) {
  return orc_batch_status(alg, op, n, nthreads, a, b, c, d, NULL);
}

/* as orc_batch; with status != NULL each record's return code lands in status[i] instead */
int orc_batch_status(const char *alg, int op, size_t n, int nthreads, uint8_t *a, uint8_t *b,
                     const uint8_t *c, const uint8_t *d, int32_t *status) {
  size_t sz[6];
  if (orc_sizes(alg, sz)) return -1;
  if (nthreads < 1) nthreads = 1;
  if ((size_t)nthreads > n && n > 0) nthreads = (int)n;
  job *jobs = (job *)calloc((size_t)nthreads, sizeof(job));
  pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
  for (int t = 0; t < nthreads; ++t) {
    jobs[t].alg = alg;
    jobs[t].op = op;
    jobs[t].lo = n * t / nthreads;
    jobs[t].hi = n * (t + 1) / nthreads;
    jobs[t].a = a, jobs[t].b = b, jobs[t].c = c, jobs[t].d = d;
    jobs[t].status = status;
    memcpy(jobs[t].sz, sz, sizeof sz);
    pthread_create(&th[t], NULL, run_job, &jobs[t]);
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

/* ---- bench coin derivation: SHAKE256("qrk-bench" || LE64(seed) || LE64(i), len) ---- */
void orc_bench_coins(uint8_t *out, size_t n, size_t len, uint64_t seed, uint64_t first_index) {
  uint8_t in[9 + 16];
  memcpy(in, "qrk-bench", 9);
  for (int b = 0; b < 8; ++b) in[9 + b] = (uint8_t)(seed >> (8 * b));
  for (size_t i = 0; i < n; ++i) {
    uint64_t idx = first_index + i;
    for (int b = 0; b < 8; ++b) in[17 + b] = (uint8_t)(idx >> (8 * b));
    orc_shake256(out + i * len, len, in, sizeof in);
  }
}

/* ---- raw hash entry points (checked against hashlib) ---- */
void orc_hash(int which, uint8_t *out, size_t outlen, const uint8_t *in, size_t inlen) {
  switch (which) {
    case 0: orc_shake128(out, outlen, in, inlen); break;
    case 1: orc_shake256(out, outlen, in, inlen); break;
    case 2: orc_sha3_256(out, in, inlen); break;
    case 3: orc_sha3_512(out, in, inlen); break;
  }
}

/* ---- NIST KAT DRBG ---- */
size_t orc_drbg_size(void) { return sizeof(orc_drbg); }
void orc_drbg_init_ext(void *d, const uint8_t entropy[48]) { orc_drbg_init((orc_drbg *)d, entropy, NULL); }
void orc_drbg_bytes(void *d, uint8_t *out, size_t n) { orc_drbg_randombytes((orc_drbg *)d, out, n); }
void orc_aes(const uint8_t *key, int keybits, const uint8_t in[16], uint8_t out[16]) {
  orc_aes_encrypt_block(key, keybits, in, out);
}

/* KAT coins for `count` records: per record reseed with seed_i, then one
 * keypair draw (kp bytes) and one encaps draw (enc bytes). */
void orc_kat_coins(size_t count, size_t kp, size_t enc, uint8_t *kp_out, uint8_t *enc_out,
                   uint8_t *seeds_out) {
  orc_drbg master, rec;
  uint8_t entropy[48];
  for (int i = 0; i < 48; ++i) entropy[i] = (uint8_t)i;
  orc_drbg_init(&master, entropy, NULL);
  for (size_t i = 0; i < count; ++i) {
    uint8_t seed[48];
    orc_drbg_randombytes(&master, seed, 48);
    if (seeds_out) memcpy(seeds_out + 48 * i, seed, 48);
    orc_drbg_init(&rec, seed, NULL);
    orc_drbg_randombytes(&rec, kp_out + i * kp, kp);
    orc_drbg_randombytes(&rec, enc_out + i * enc, enc);
  }
}
