/*
 * dkg-amd CPU ORACLE (test infrastructure only; see oracle.h).
 * BLAKE2b (RFC 7693; blake2 0.9.1 `Blake2b` is unkeyed BLAKE2b-512, used by
 * CommitmentKey::generate at commitment.rs:13-17) and the ChaCha20 block function
 * (RFC 8439) producing the rand_chacha `ChaCha20Rng` stream (key = seed, 64-bit block
 * counter from 0, stream 0 — identical to the IETF variant with a zero nonce for the first
 * 2^32 blocks).  The seeded stream stands in for the reference tests' OsRng (§8d of SURVEY.md).
 */
#include "oracle_int.h"

static const uint64_t B2_IV[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL,
                                  0xa54ff53a5f1d36f1ULL, 0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL,
                                  0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};
static const uint8_t B2_SIGMA[12][16] = {
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
    {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4}, {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
    {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13}, {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
    {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11}, {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
    {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5}, {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0},
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3}};

static uint64_t rotr64(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }

static void b2_compress(uint64_t h[8], const uint8_t block[128], uint64_t t, int last) {
  uint64_t m[16], v[16];
  for (int i = 0; i < 16; i++) {
    m[i] = 0;
    for (int j = 7; j >= 0; j--) m[i] = (m[i] << 8) | block[8 * i + j];
  }
  for (int i = 0; i < 8; i++) {
    v[i] = h[i];
    v[i + 8] = B2_IV[i];
  }
  v[12] ^= t;
  if (last) v[14] = ~v[14];
#define B2G(a, b, c, d, x, y)        \
  a = a + b + x; d = rotr64(d ^ a, 32); \
  c = c + d; b = rotr64(b ^ c, 24);     \
  a = a + b + y; d = rotr64(d ^ a, 16); \
  c = c + d; b = rotr64(b ^ c, 63);
  for (int r = 0; r < 12; r++) {
    const uint8_t *s = B2_SIGMA[r];
    B2G(v[0], v[4], v[8], v[12], m[s[0]], m[s[1]]);
    B2G(v[1], v[5], v[9], v[13], m[s[2]], m[s[3]]);
    B2G(v[2], v[6], v[10], v[14], m[s[4]], m[s[5]]);
    B2G(v[3], v[7], v[11], v[15], m[s[6]], m[s[7]]);
    B2G(v[0], v[5], v[10], v[15], m[s[8]], m[s[9]]);
    B2G(v[1], v[6], v[11], v[12], m[s[10]], m[s[11]]);
    B2G(v[2], v[7], v[8], v[13], m[s[12]], m[s[13]]);
    B2G(v[3], v[4], v[9], v[14], m[s[14]], m[s[15]]);
  }
#undef B2G
  for (int i = 0; i < 8; i++) h[i] ^= v[i] ^ v[i + 8];
}

void or_blake2b(uint8_t *out, size_t outlen, const uint8_t *in, size_t inlen) {
  uint64_t h[8];
  for (int i = 0; i < 8; i++) h[i] = B2_IV[i];
  h[0] ^= 0x01010000ULL ^ (uint64_t)outlen;
  uint8_t block[128];
  uint64_t t = 0;
  while (inlen > 128) {
    t += 128;
    b2_compress(h, in, t, 0);
    in += 128;
    inlen -= 128;
  }
  memset(block, 0, 128);
  memcpy(block, in, inlen);
  t += inlen;
  b2_compress(h, block, t, 1);
  for (size_t i = 0; i < outlen; i++) out[i] = (uint8_t)(h[i / 8] >> (8 * (i % 8)));
}

static uint32_t rotl32(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }

static void chacha_block(uint8_t out[64], const uint32_t key[8], uint64_t counter) {
  uint32_t s[16], x[16];
  s[0] = 0x61707865u; s[1] = 0x3320646eu; s[2] = 0x79622d32u; s[3] = 0x6b206574u;
  for (int i = 0; i < 8; i++) s[4 + i] = key[i];
  s[12] = (uint32_t)counter;
  s[13] = (uint32_t)(counter >> 32);
  s[14] = 0;
  s[15] = 0;
  memcpy(x, s, sizeof s);
#define QR(a, b, c, d)                         \
  a += b; d ^= a; d = rotl32(d, 16);           \
  c += d; b ^= c; b = rotl32(b, 12);           \
  a += b; d ^= a; d = rotl32(d, 8);            \
  c += d; b ^= c; b = rotl32(b, 7);
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
    out[4 * i] = (uint8_t)v;
    out[4 * i + 1] = (uint8_t)(v >> 8);
    out[4 * i + 2] = (uint8_t)(v >> 16);
    out[4 * i + 3] = (uint8_t)(v >> 24);
  }
}

void or_chacha20_stream(const uint8_t key[32], uint64_t first_block, uint8_t *out, size_t len) {
  uint32_t k[8];
  for (int i = 0; i < 8; i++)
    k[i] = (uint32_t)key[4 * i] | ((uint32_t)key[4 * i + 1] << 8) | ((uint32_t)key[4 * i + 2] << 16) |
           ((uint32_t)key[4 * i + 3] << 24);
  uint8_t blk[64];
  uint64_t ctr = first_block;
  while (len) {
    chacha_block(blk, k, ctr++);
    size_t n = len < 64 ? len : 64;
    memcpy(out, blk, n);
    out += n;
    len -= n;
  }
}
