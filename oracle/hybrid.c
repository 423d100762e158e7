/*
 * dkg-amd CPU ORACLE — TEST INFRASTRUCTURE ONLY (see oracle.h).
 * Full (encrypted-share) mode of the reference: the hybrid ElGamal + ChaCha20 scheme of
 * /root/reference/src/cryptography/elgamal.rs and the member communication keys of
 * src/dkg/procedure_keys.rs, restated on this oracle's dalek-matched group arithmetic.
 * Third-party pieces (absent here, pinned via libsodium fixtures): chacha20 0.7.2 `ChaCha20`
 * (RFC 8439 IETF variant: 96-bit nonce, 32-bit block counter from 0) and blake2 0.9.1 `Blake2b`
 * (BLAKE2b-512).
 */
#include <string.h>

#include "oracle.h"

static uint32_t rd32(const uint8_t *p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
static uint32_t rotl(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }

/* RFC 8439 block: constants, key, counter (word 12), nonce (words 13-15). */
static void chacha_ietf_block(uint8_t out[64], const uint8_t key[32], uint32_t counter, const uint8_t nonce[12]) {
  uint32_t s[16], x[16];
  s[0] = 0x61707865u; s[1] = 0x3320646eu; s[2] = 0x79622d32u; s[3] = 0x6b206574u;
  for (int i = 0; i < 8; i++) s[4 + i] = rd32(key + 4 * i);
  s[12] = counter;
  for (int i = 0; i < 3; i++) s[13 + i] = rd32(nonce + 4 * i);
  memcpy(x, s, sizeof s);
#define QR(a, b, c, d)                       \
  a += b; d ^= a; d = rotl(d, 16);           \
  c += d; b ^= c; b = rotl(b, 12);           \
  a += b; d ^= a; d = rotl(d, 8);            \
  c += d; b ^= c; b = rotl(b, 7);
  for (int r = 0; r < 10; r++) {
    QR(x[0], x[4], x[8], x[12]);
    QR(x[1], x[5], x[9], x[13]);
    QR(x[2], x[6], x[10], x[14]);
    QR(x[3], x[7], x[11], x[15]);
    QR(x[0], x[5], x[10], x[15]);
    QR(x[1], x[6], x[11], x[12]);
    QR(x[2], x[7], x[8], x[13]);
    QR(x[3], x[4], x[9], x[14]);
  }
#undef QR
  for (int i = 0; i < 16; i++) {
    uint32_t v = x[i] + s[i];
    for (int b = 0; b < 4; b++) out[4 * i + b] = (uint8_t)(v >> (8 * b));
  }
}

void or_chacha20_ietf_xor(uint8_t *out, const uint8_t *in, size_t len, const uint8_t key[32],
                          const uint8_t nonce[12]) {
  uint8_t blk[64];
  uint32_t ctr = 0;
  while (len) {
    chacha_ietf_block(blk, key, ctr++, nonce);
    size_t n = len < 64 ? len : 64;
    for (size_t i = 0; i < n; i++) out[i] = in[i] ^ blk[i];
    out += n;
    in += n;
    len -= n;
  }
}

/* SymmetricKey::process (elgamal.rs:172-193): Blake2b-512(K.to_bytes()) -> key h[0..32],
 * nonce h[32..44]; XOR the ChaCha20 keystream. */
static void sym_process(uint8_t *out, const uint8_t *in, size_t len, const uint8_t K[32]) {
  uint8_t h[64];
  or_blake2b(h, 64, K, 32);
  or_chacha20_ietf_xor(out, in, len, h, h + 32);
}

/* PublicKey::hybrid_encrypt with the randomness given (elgamal.rs:134-145):
 * e1 = G * r, e2 = process(pk * r, msg). */
int or_hybrid_encrypt(uint8_t e1[32], uint8_t *e2, const uint8_t pk[32], const uint8_t r[32], const uint8_t *msg,
                      size_t len) {
  uint8_t K[32];
  if (or_pt_mul(K, pk, r)) return -1;
  or_pt_base_mul(e1, r);
  sym_process(e2, msg, len, K);
  return 0;
}

/* SecretKey::hybrid_decrypt (elgamal.rs:161-170): process(e1 * sk, e2). */
int or_hybrid_decrypt(uint8_t *msg, const uint8_t sk[32], const uint8_t e1[32], const uint8_t *e2, size_t len) {
  uint8_t K[32];
  if (or_pt_mul(K, e1, sk)) return -1;
  sym_process(msg, e2, len, K);
  return 0;
}

/* Seeded MemberCommunicationKey (procedure_keys.rs:72-82): sk = wide(ChaCha20Rng(seed) block 0),
 * seed = BLAKE2b-256("dkg-amd/v1/member" || master || u32le ceremony || u32le member). */
void or_member_sk(uint8_t sk[32], const uint8_t master[32], uint32_t ceremony, uint32_t member) {
  static const char tag[] = "dkg-amd/v1/member";
  uint8_t msg[sizeof tag - 1 + 40], seed[32], st[64];
  memcpy(msg, tag, sizeof tag - 1);
  memcpy(msg + sizeof tag - 1, master, 32);
  for (int k = 0; k < 4; k++) {
    msg[sizeof tag - 1 + 32 + k] = (uint8_t)(ceremony >> (8 * k));
    msg[sizeof tag - 1 + 36 + k] = (uint8_t)(member >> (8 * k));
  }
  or_blake2b(seed, 32, msg, sizeof msg);
  or_chacha20_stream(seed, 0, st, 64);
  or_sc_reduce_wide(sk, st);
}

/* Encryption randomness of dealer `seed` for n recipients (committee.rs:171-172 draw order, after
 * the 2(t+1) coefficient draws): r[q][0] for the randomness ciphertext, r[q][1] for the share. */
void or_enc_randomness(uint8_t *r, const uint8_t seed[32], size_t t, size_t n) {
  uint8_t blk[64];
  for (size_t q = 0; q < 2 * n; q++) {
    or_chacha20_stream(seed, 2 * (t + 1) + q, blk, 64);
    or_sc_reduce_wide(r + 32 * q, blk);
  }
}
