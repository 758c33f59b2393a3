/* oracle-only ML-KEM / FrodoKEM / DRBG declarations (see mlkem.c, frodo.c, drbg.c) */
#ifndef ORC_KEMS_H
#define ORC_KEMS_H
#include <stddef.h>
#include <stdint.h>

int orc_mlkem_sizes(const char *alg, size_t *pk, size_t *sk, size_t *ct, size_t *ss);
int orc_mlkem_keypair_derand(const char *alg, uint8_t *pk, uint8_t *sk, const uint8_t coins[64]);
int orc_mlkem_ek_check(const char *alg, const uint8_t *pk);
int orc_mlkem_encaps_derand(const char *alg, uint8_t *ct, uint8_t *ss, const uint8_t *pk,
                            const uint8_t coins[32]);
int orc_mlkem_decaps(const char *alg, uint8_t *ss, const uint8_t *ct, const uint8_t *sk);

int orc_frodo_sizes(const char *alg, size_t *pk, size_t *sk, size_t *ct, size_t *ss,
                    size_t *kp_coins, size_t *enc_coins);
int orc_frodo_keypair_derand(const char *alg, uint8_t *pk, uint8_t *sk, const uint8_t *coins);
int orc_frodo_encaps_derand(const char *alg, uint8_t *ct, uint8_t *ss, const uint8_t *pk,
                            const uint8_t *mu);
int orc_frodo_decaps(const char *alg, uint8_t *ss, const uint8_t *ct, const uint8_t *sk);

void orc_aes_encrypt_block(const uint8_t *key, int keybits, const uint8_t in[16], uint8_t out[16]);

typedef struct {
  uint8_t key[32];
  uint8_t v[16];
  int reseed_counter;
} orc_drbg;
void orc_drbg_init(orc_drbg *d, const uint8_t entropy[48], const uint8_t *personalization);
void orc_drbg_randombytes(orc_drbg *d, uint8_t *out, size_t n);

#endif
