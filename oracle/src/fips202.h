/* Keccak-f[1600] sponge (FIPS 202) -- oracle / CPU-baseline only.
 *
 * TEST INFRASTRUCTURE: compiled into oracle/liboracle.so, which only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg load.
 *
 * Restates FIPS 202 (SHA3-256/512, SHAKE128/256), the hash layer liboqs uses
 * under OQS_KEM_keypair/encaps/decaps (reference call sites
 * quantum_resistant_p2p/vendor/oqs.py:318,348,372).  Pinned against Python
 * hashlib in tests/test_oracle.py.
 */
#ifndef ORC_FIPS202_H
#define ORC_FIPS202_H
#include <stddef.h>
#include <stdint.h>

#define ORC_SHAKE128_RATE 168
#define ORC_SHAKE256_RATE 136
#define ORC_SHA3_256_RATE 136
#define ORC_SHA3_512_RATE 72

typedef struct {
  uint64_t s[25];
  unsigned pos;   /* byte position inside the current rate block */
  unsigned rate;  /* bytes */
} orc_keccak;

void orc_keccakf1600(uint64_t s[25]);
void orc_keccak_init(orc_keccak *c, unsigned rate);
void orc_keccak_absorb(orc_keccak *c, const uint8_t *in, size_t len);
void orc_keccak_finalize(orc_keccak *c, uint8_t ds);
void orc_keccak_squeeze(orc_keccak *c, uint8_t *out, size_t len);

void orc_shake128(uint8_t *out, size_t outlen, const uint8_t *in, size_t inlen);
void orc_shake256(uint8_t *out, size_t outlen, const uint8_t *in, size_t inlen);
void orc_sha3_256(uint8_t out[32], const uint8_t *in, size_t inlen);
void orc_sha3_512(uint8_t out[64], const uint8_t *in, size_t inlen);

#endif
