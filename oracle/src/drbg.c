/* AES (FIPS 197) and the NIST PQC KAT AES-256 CTR_DRBG -- oracle only.
 *
 * TEST INFRASTRUCTURE.  The DRBG restates randombytes_init()/randombytes() of
 * the NIST PQC rng.c (liboqs: OQS_randombytes_nist_kat_init_256bit); it is
 * pinned by tests/test_oracle.py against the per-record seeds every NIST KEM
 * KAT file starts with (count = 0, 1) and against FIPS 197 Appendix C.
 * AES-128 is also used for FrodoKEM-*-AES matrix generation.
 * The S-box is derived at first use (GF(2^8) inverse + affine map).
 */
#include <string.h>

#include "mlkem.h"

static uint8_t SB[256];
static int sb_ready = 0;

static uint8_t xt(uint8_t a) { return (uint8_t)((a << 1) ^ ((a & 0x80) ? 0x1B : 0)); }
static uint8_t gm(uint8_t a, uint8_t b) {
  uint8_t r = 0;
  while (b) {
    if (b & 1) r ^= a;
    a = xt(a);
    b >>= 1;
  }
  return r;
}

static void make_sbox(void) {
  if (sb_ready) return;
  for (int x = 0; x < 256; ++x) {
    uint8_t inv = 0;
    if (x)
      for (int y = 1; y < 256; ++y)
        if (gm((uint8_t)x, (uint8_t)y) == 1) {
          inv = (uint8_t)y;
          break;
        }
    uint8_t s = inv;
    for (int sh = 1; sh < 5; ++sh) s ^= (uint8_t)((inv << sh) | (inv >> (8 - sh)));
    SB[x] = s ^ 0x63;
  }
  __atomic_store_n(&sb_ready, 1, __ATOMIC_RELEASE);
}

static void expand(const uint8_t *key, int nk, uint8_t rk[15][16]) {
  uint8_t w[60][4];
  int nr = nk + 6;
  for (int i = 0; i < nk; ++i) memcpy(w[i], key + 4 * i, 4);
  uint8_t rcon = 1;
  for (int i = nk; i < 4 * (nr + 1); ++i) {
    uint8_t t[4];
    memcpy(t, w[i - 1], 4);
    if (i % nk == 0) {
      uint8_t t0 = t[0];
      t[0] = (uint8_t)(SB[t[1]] ^ rcon);
      t[1] = SB[t[2]];
      t[2] = SB[t[3]];
      t[3] = SB[t0];
      rcon = xt(rcon);
    } else if (nk > 6 && i % nk == 4) {
      for (int b = 0; b < 4; ++b) t[b] = SB[t[b]];
    }
    for (int b = 0; b < 4; ++b) w[i][b] = (uint8_t)(w[i - nk][b] ^ t[b]);
  }
  for (int r = 0; r <= nr; ++r)
    for (int c = 0; c < 4; ++c) memcpy(rk[r] + 4 * c, w[4 * r + c], 4);
}

void orc_aes_encrypt_block(const uint8_t *key, int keybits, const uint8_t in[16], uint8_t out[16]) {
  make_sbox();
  int nk = keybits / 32, nr = nk + 6;
  uint8_t rk[15][16], s[16], t[16];
  expand(key, nk, rk);
  for (int i = 0; i < 16; ++i) s[i] = in[i] ^ rk[0][i];
  for (int r = 1; r <= nr; ++r) {
    for (int i = 0; i < 16; ++i) s[i] = SB[s[i]];
    for (int c = 0; c < 4; ++c)
      for (int row = 0; row < 4; ++row) t[4 * c + row] = s[4 * ((c + row) & 3) + row];
    if (r != nr) {
      for (int c = 0; c < 4; ++c) {
        uint8_t a0 = t[4 * c], a1 = t[4 * c + 1], a2 = t[4 * c + 2], a3 = t[4 * c + 3];
        s[4 * c] = (uint8_t)(xt(a0) ^ (xt(a1) ^ a1) ^ a2 ^ a3);
        s[4 * c + 1] = (uint8_t)(a0 ^ xt(a1) ^ (xt(a2) ^ a2) ^ a3);
        s[4 * c + 2] = (uint8_t)(a0 ^ a1 ^ xt(a2) ^ (xt(a3) ^ a3));
        s[4 * c + 3] = (uint8_t)((xt(a0) ^ a0) ^ a1 ^ a2 ^ xt(a3));
      }
    } else {
      memcpy(s, t, 16);
    }
    for (int i = 0; i < 16; ++i) s[i] ^= rk[r][i];
  }
  memcpy(out, s, 16);
}

static void inc_v(uint8_t v[16]) {
  for (int j = 15; j >= 0; --j) {
    if (v[j] == 0xFF) {
      v[j] = 0;
    } else {
      v[j]++;
      break;
    }
  }
}

static void drbg_update(orc_drbg *d, const uint8_t *provided) {
  uint8_t temp[48];
  for (int i = 0; i < 3; ++i) {
    inc_v(d->v);
    orc_aes_encrypt_block(d->key, 256, d->v, temp + 16 * i);
  }
  if (provided)
    for (int i = 0; i < 48; ++i) temp[i] ^= provided[i];
  memcpy(d->key, temp, 32);
  memcpy(d->v, temp + 32, 16);
}

void orc_drbg_init(orc_drbg *d, const uint8_t entropy[48], const uint8_t *personalization) {
  uint8_t seed[48];
  memcpy(seed, entropy, 48);
  if (personalization)
    for (int i = 0; i < 48; ++i) seed[i] ^= personalization[i];
  memset(d->key, 0, 32);
  memset(d->v, 0, 16);
  drbg_update(d, seed);
  d->reseed_counter = 1;
}

void orc_drbg_randombytes(orc_drbg *d, uint8_t *out, size_t n) {
  uint8_t blk[16];
  while (n) {
    inc_v(d->v);
    orc_aes_encrypt_block(d->key, 256, d->v, blk);
    size_t take = n > 16 ? 16 : n;
    memcpy(out, blk, take);
    out += take;
    n -= take;
  }
  drbg_update(d, NULL);
  d->reseed_counter++;
}
