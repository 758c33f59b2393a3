/* qrkem -- MI355X-native batched post-quantum KEM engine: public C ABI.
 *
 * Built as quantum-resistant-p2p_amd/qrkem/libqrkem.so (hipcc, gfx950).
 *
 * Part 1 is the liboqs-compatible subset that the reference's vendored ctypes
 * wrapper binds (quantum_resistant_p2p/vendor/oqs.py).  A maintainer can drop
 * libqrkem.so in place of vendor/lib/linux/liboqs.so and the reference's own
 * oqs.py loads it unchanged.  Part 2 adds the batched,
 * stream-ordered, device-pointer entry points the reference has no equivalent
 * for (it calls liboqs once per handshake on the asyncio thread).
 *
 * Ownership: callers allocate every output buffer (as oqs.py:316-317, 342-347,
 * 369-371 do); the library owns only OQS_KEM handles, static strings and the
 * device scratch inside a qrk_ctx.  Errors: OQS_SUCCESS (0) / OQS_ERROR (-1),
 * as oqs.py:38-39; qrk_last_error() gives a message.
 */
#ifndef QRKEM_H
#define QRKEM_H

#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------------ *
 * Part 1: liboqs-compatible subset                                    *
 * ------------------------------------------------------------------ */

typedef enum { OQS_ERROR = -1, OQS_SUCCESS = 0 } OQS_STATUS;

/* Struct prefix read by oqs.py:241-253 (liboqs <= 0.12 layout): the wrapper
 * reads method_name .. length_shared_secret and treats the three callbacks as
 * opaque pointers. */
typedef struct OQS_KEM {
  const char *method_name;
  const char *alg_version;
  uint8_t claimed_nist_level;
  bool ind_cca;
  size_t length_public_key;
  size_t length_secret_key;
  size_t length_ciphertext;
  size_t length_shared_secret;
  OQS_STATUS (*keypair)(uint8_t *public_key, uint8_t *secret_key);
  OQS_STATUS (*encaps)(uint8_t *ciphertext, uint8_t *shared_secret, const uint8_t *public_key);
  OQS_STATUS (*decaps)(uint8_t *shared_secret, const uint8_t *ciphertext, const uint8_t *secret_key);
} OQS_KEM;

/* oqs.py:192 */
void OQS_init(void);
/* oqs.py:197-198 */
const char *OQS_version(void);
/* oqs.py:409 */
size_t OQS_KEM_alg_count(void);
/* oqs.py:397, 409 */
const char *OQS_KEM_alg_identifier(size_t i);
/* oqs.py:406 */
int OQS_KEM_alg_is_enabled(const char *method_name);
/* oqs.py:271, 396 -- NULL for unknown or not-enabled names */
OQS_KEM *OQS_KEM_new(const char *method_name);
/* oqs.py:318-322: host pointers, one handshake, randomness from the OS CSPRNG */
OQS_STATUS OQS_KEM_keypair(const OQS_KEM *kem, uint8_t *public_key, uint8_t *secret_key);
/* oqs.py:348-353 */
OQS_STATUS OQS_KEM_encaps(const OQS_KEM *kem, uint8_t *ciphertext, uint8_t *shared_secret,
                          const uint8_t *public_key);
/* oqs.py:372-377 */
OQS_STATUS OQS_KEM_decaps(const OQS_KEM *kem, uint8_t *shared_secret, const uint8_t *ciphertext,
                          const uint8_t *secret_key);
/* oqs.py:390 */
void OQS_KEM_free(OQS_KEM *kem);
/* oqs.py:386-389 */
void OQS_MEM_cleanse(void *ptr, size_t len);

/* Derandomised single-shot forms (names of liboqs >= 0.13's *_derand API):
 * KeyGen coins = d||z (ML-KEM, 64 B) or s||seedSE||z (FrodoKEM); Encaps coins
 * = m (32 B) or mu.  Host pointers. */
OQS_STATUS OQS_KEM_keypair_derand(const OQS_KEM *kem, uint8_t *public_key, uint8_t *secret_key,
                                  const uint8_t *seed);
OQS_STATUS OQS_KEM_encaps_derand(const OQS_KEM *kem, uint8_t *ciphertext, uint8_t *shared_secret,
                                 const uint8_t *public_key, const uint8_t *seed);

/* Signature half of the liboqs ABI: the reference's oqs.py binds these at
 * import time (oqs.py:684-697).  Signatures are outside this engine's scope,
 * so the registry is empty (count 0) and every call fails. */
typedef struct OQS_SIG OQS_SIG;
size_t OQS_SIG_alg_count(void);
const char *OQS_SIG_alg_identifier(size_t i);
int OQS_SIG_alg_is_enabled(const char *method_name);
OQS_SIG *OQS_SIG_new(const char *method_name);
OQS_STATUS OQS_SIG_keypair(const OQS_SIG *sig, uint8_t *public_key, uint8_t *secret_key);
OQS_STATUS OQS_SIG_sign(const OQS_SIG *sig, uint8_t *signature, size_t *signature_len, const uint8_t *message,
                        size_t message_len, const uint8_t *secret_key);
OQS_STATUS OQS_SIG_verify(const OQS_SIG *sig, const uint8_t *message, size_t message_len,
                          const uint8_t *signature, size_t signature_len, const uint8_t *public_key);
void OQS_SIG_free(OQS_SIG *sig);

/* ------------------------------------------------------------------ *
 * Part 2: batched device API (no reference equivalent)                *
 * ------------------------------------------------------------------ */

typedef struct qrk_ctx qrk_ctx;

/* One context per (process, device).  Holds device scratch, grown on demand. */
int qrk_ctx_create(qrk_ctx **out, int device);
void qrk_ctx_destroy(qrk_ctx *ctx);
/* Handshakes per internal chunk (scratch = chunk * per-handshake bytes). */
int qrk_ctx_set_chunk(qrk_ctx *ctx, size_t chunk);
size_t qrk_ctx_scratch_bytes(const qrk_ctx *ctx);
/* Zero every buffer of the context that can hold keys or secret intermediates (device
 * scratch, handshake scratch, device and pinned host staging); synchronous.  Every call
 * already zeroes the per-handshake key records it leaves in scratch (seeds, m', K', Kbar,
 * ...) and the staged copies of host secrets (coins included).  The other intermediates stay
 * in scratch until a later call overwrites them, and some of them are expanded secret-key
 * material: ML-KEM's PRF output for s and e (KeyGen) and for the re-encryption noise (Decaps),
 * FrodoKEM's sampled S / S', HQC's seedexpander rows x, y (KeyGen, Decaps) and r1, r2, e.
 * Call this (or qrk_ctx_destroy, which does the same before freeing) when a context that
 * handled secret keys is idle. */
int qrk_ctx_cleanse(qrk_ctx *ctx);
/* Diagnostics (tests): waits for the context's last call, then counts the nonzero bytes left
 * in its pinned host staging (out[0]) and device staging (out[1]) -- the buffers that carry
 * OS-drawn coins (coins == NULL) to the device, wiped before every call returns -- and in the
 * first 64 MiB of device scratch (out[2], zero after qrk_ctx_cleanse). */
int qrk_ctx_staging_residue(qrk_ctx *ctx, uint64_t out[3]);
/* Handshakes per chunk actually used for `alg` (FrodoKEM and HQC cap the chunk so their
 * scratch stays within QRK_SCRATCH_GIB = 48 GiB); 0 for an unknown algorithm. */
size_t qrk_ctx_effective_chunk(const qrk_ctx *ctx, const char *alg);
/* Schedule of one operation's kernels, all on the caller's stream: 0 (default): independent
 * kernels share multi-role launches (each role's workgroups a contiguous range of one grid, in
 * grid order); 1: serial, one kernel per launch (kernel timings in isolation).  Any other value
 * returns -1 with qrk_last_error() set.  (Round 3's value 2, the forked split pipeline, was
 * removed in round 4 and is rejected now.) */
int qrk_ctx_set_streams(qrk_ctx *ctx, int streams);

/* Sizes of `alg`: out[0..5] = pk, sk, ct, ss, keypair coin bytes, encaps coin bytes. */
int qrk_kem_sizes(const char *alg, size_t out[6]);

/* Batched operations.  ALL buffers are device pointers, contiguous AoS
 * [n][len].  `coins` may be NULL (the library draws n*len bytes from the OS
 * CSPRNG and uploads them); otherwise it is [n][keypair/encaps coin bytes].
 * `status` (nullable, device int32[n]) receives -1 for encapsulation keys that
 * fail the FIPS 203 section 7.2 modulus check, else 0.  `stream` is a
 * hipStream_t (NULL = default stream).  Calls are stream-ordered and
 * asynchronous: every kernel of a call runs on `stream`, and with caller-supplied
 * coins (or none needed) a call returns to the host before its kernels finish.
 * With coins == NULL the call returns once the OS coins are uploaded (their pinned
 * copy is wiped then).  Re-entrant across contexts.  Calls on one context may use
 * different streams: each call's stream first waits, on the device, until the
 * previous call on that context is done with the context's scratch. */
int qrk_kem_keypair_batch(qrk_ctx *ctx, const char *alg, size_t n, uint8_t *pk, uint8_t *sk,
                          const uint8_t *coins, void *stream);
int qrk_kem_encaps_batch(qrk_ctx *ctx, const char *alg, size_t n, uint8_t *ct, uint8_t *ss,
                         const uint8_t *pk, const uint8_t *coins, int32_t *status, void *stream);
int qrk_kem_decaps_batch(qrk_ctx *ctx, const char *alg, size_t n, uint8_t *ss, const uint8_t *ct,
                         const uint8_t *sk, void *stream);
/* Decaps with a per-record return code (device int32[n]): HQC writes -1 where the
 * re-encryption check fails -- the OQS_ERROR liboqs's HQC decaps returns, which makes the
 * reference's KeyEncapsulation.decap_secret raise (oqs.py:372-380); ss_i = K(sigma || ct_i)
 * is written either way.  ML-KEM and FrodoKEM (implicit rejection, return 0) write 0. */
int qrk_kem_decaps_batch_status(qrk_ctx *ctx, const char *alg, size_t n, uint8_t *ss, const uint8_t *ct,
                                const uint8_t *sk, int32_t *status, void *stream);

/* Same, with host buffers (synchronous; copies through pinned staging). */
int qrk_kem_keypair_batch_host(qrk_ctx *ctx, const char *alg, size_t n, uint8_t *pk, uint8_t *sk,
                               const uint8_t *coins);
int qrk_kem_encaps_batch_host(qrk_ctx *ctx, const char *alg, size_t n, uint8_t *ct, uint8_t *ss,
                              const uint8_t *pk, const uint8_t *coins, int32_t *status);
int qrk_kem_decaps_batch_host(qrk_ctx *ctx, const char *alg, size_t n, uint8_t *ss, const uint8_t *ct,
                              const uint8_t *sk);
int qrk_kem_decaps_batch_status_host(qrk_ctx *ctx, const char *alg, size_t n, uint8_t *ss, const uint8_t *ct,
                                     const uint8_t *sk, int32_t *status);

/* Bench inputs generated on device: out_i = SHAKE256("qrk-bench"||LE64(seed)||LE64(first+i), len),
 * len a multiple of 8, <= 136.  Device pointer. */
int qrk_bench_coins(qrk_ctx *ctx, size_t n, size_t len, uint64_t seed, uint64_t first, uint8_t *out,
                    void *stream);
/* Flip one ciphertext bit per selected index (mode 0 none, 1 all, 2 Bernoulli(1/2)):
 * h_i = SHAKE256("qrk-tamper"||LE64(seed)||LE64(i))[0..8), bit (h_i>>1) mod 8*ctlen. */
int qrk_tamper(qrk_ctx *ctx, size_t n, size_t ctlen, uint64_t seed, int mode, uint8_t *ct, void *stream);
/* Per-record digests: out_i = SHA3-256(a_i || b_i), 32 bytes, for n records of a_len and
 * b_len bytes (b may be NULL with b_len = 0).  Device pointers.  The sharded bench hashes
 * each rank's (ct, ss) records with it and combines them per block of global indices, so
 * the digests do not depend on the GPU count. */
int qrk_digest_rows(qrk_ctx *ctx, size_t n, const uint8_t *a, size_t a_len, const uint8_t *b, size_t b_len,
                    uint8_t *out, void *stream);
/* HQC fixed-weight supports (the sampling inside KeyGen / Encaps / Decaps, exposed so the
 * duplicate-removal step can be tested on inputs crafted to collide): for each of n vectors,
 * sup[v][i] = i + floor(r[v][i] * (n_HQC - i) / 2^32), then the spec's removal of duplicates.
 * kind 0: weight w (x, y), kind 1: weight w_r = w_e (r1, r2, e).  Device uint32 pointers,
 * [n][weight] each. */
int qrk_hqc_supports(qrk_ctx *ctx, const char *alg, int kind, size_t n, const uint32_t *r, uint32_t *sup,
                     void *stream);

/* HKDF-SHA256 (RFC 5869) over n keys, one GPU lane per key.  Replaces
 * SecureMessaging._derive_symmetric_key (messaging.py:350-382: HKDF(SHA256,
 * length=key_size, salt=None, info=...).derive(shared_secret)).
 * Device pointers: ikm [n][ikm_len]; salt [salt_len] shared by all keys (NULL/0 =
 * HashLen zero bytes, as salt=None); okm [n][okm_len], 1 <= okm_len <= 8160.
 * info: with info_off (device uint64[n+1]) key i uses info[info_off[i] .. info_off[i+1]);
 * with info_off NULL every key uses info[0 .. info_len). */
int qrk_hkdf_sha256_batch(qrk_ctx *ctx, size_t n, const uint8_t *ikm, size_t ikm_len, const uint8_t *salt,
                          size_t salt_len, const uint8_t *info, const uint64_t *info_off, size_t info_len,
                          uint8_t *okm, size_t okm_len, void *stream);

/* n complete protocol key exchanges with the reference's per-handshake operation mix
 * (messaging.py:546-1146): initiator KeyGen (:590); responder KeyGen (:809, its pk is
 * sent back at :853), Encaps of the initiator's pk (:830) and HKDF (:845); initiator
 * Decaps (:1038) and HKDF (:1068).  Device pointers.  Coins (each nullable = OS CSPRNG):
 * coins_kp_i / coins_kp_r [n][keypair coin bytes], coins_enc [n][encaps coin bytes].
 * info / info_off / info_len as qrk_hkdf_sha256_batch (salt = None).  Outputs (the wire
 * and the keys): pk_i, pk_r [n][pk], ct [n][ct], key_i, key_r [n][key_len]; agree
 * (nullable, int32[n]) = 1 where both sides derived the same key.  Ephemeral secret keys
 * and shared secrets stay in context scratch and are zeroed before the call returns
 * (stream-ordered). */
int qrk_handshake_batch(qrk_ctx *ctx, const char *alg, size_t n, const uint8_t *coins_kp_i,
                        const uint8_t *coins_kp_r, const uint8_t *coins_enc, const uint8_t *info,
                        const uint64_t *info_off, size_t info_len, size_t key_len, uint8_t *pk_i, uint8_t *pk_r,
                        uint8_t *ct, uint8_t *key_i, uint8_t *key_r, int32_t *agree, void *stream);

/* Wire format: standard base64 (RFC 4648 section 4, '=' padding), the encoding the reference
 * puts every KEM payload in before JSON framing (messaging.py:607 public key, :852-853
 * ciphertext and responder key; decoded at :829 with base64.b64decode).  Device pointers,
 * contiguous records.  Encode: in [n][in_len] -> out [n][4*ceil(in_len/3)] ASCII (no NUL).
 * Decode (strict): in [n][4*ceil(out_len/3)] -> out [n][out_len]; status (nullable, int32[n])
 * = -1 for a record with a byte outside the alphabet or misplaced / missing padding, else 0.
 * (Python's b64decode without validate=True would silently skip such bytes; a malformed KEM
 * field is rejected here instead.) */
int qrk_base64_encode_batch(qrk_ctx *ctx, size_t n, const uint8_t *in, size_t in_len, uint8_t *out, void *stream);
int qrk_base64_decode_batch(qrk_ctx *ctx, size_t n, const uint8_t *in, size_t out_len, uint8_t *out,
                            int32_t *status, void *stream);

/* Per-kernel HIP-event timing on the launch stream (for bench.py's roofline).
 * qrk_ctx_profile(ctx, 1) resets and enables; qrk_ctx_profile_collect()
 * synchronises the recorded events and returns the number of distinct kernel
 * names; qrk_ctx_profile_get() reads (name, total ms, launches) for entry i. */
int qrk_ctx_profile(qrk_ctx *ctx, int enable);
int qrk_ctx_profile_collect(qrk_ctx *ctx);
int qrk_ctx_profile_get(qrk_ctx *ctx, int i, const char **name, double *total_ms, uint64_t *launches);

const char *qrk_last_error(void);
int qrk_device_count(void);

#ifdef __cplusplus
}
#endif
#endif /* QRKEM_H */
