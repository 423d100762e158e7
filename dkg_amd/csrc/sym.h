// Device BLAKE2b / ChaCha20 for gfx950 (32- and 64-bit ARX in VALU ops), shared by the on-device
// RNG (seedgen.hip) and the hybrid share encryption (hybrid.hip).
//   blake2b_1block  : BLAKE2b of a message of at most 128 bytes (blake2 0.9.1 `Blake2b` = 512-bit
//                     output; 256-bit for the seed derivation), unkeyed.
//   chacha20_block  : original ChaCha20 block, 64-bit counter, zero nonce (rand_chacha ChaCha20Rng).
//   chacha20_ietf_block : RFC 8439 block, 32-bit counter + 96-bit nonce (chacha20 0.7 `ChaCha20`,
//                     used by SymmetricKey::process, elgamal.rs:172-193).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dkgk {
namespace sym {
__device__ static const uint64_t B2_IV[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL,
                                      0xa54ff53a5f1d36f1ULL, 0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL,
                                      0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};
__device__ static const uint8_t B2_SIGMA[10][16] = {
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
    {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4}, {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
    {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13}, {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
    {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11}, {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
    {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5}, {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0}};

__device__ __forceinline__ uint64_t rotr64(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }
__device__ __forceinline__ uint32_t rotl32(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }

// BLAKE2b of a message of at most 128 bytes given as 16 little-endian words (zero padded).
__device__ inline void blake2b_1block(uint64_t (&h)[8], const uint64_t (&m)[16], uint32_t len, uint32_t outlen) {
#pragma unroll
  for (int i = 0; i < 8; i++) h[i] = B2_IV[i];
  h[0] ^= 0x01010000ULL ^ outlen;
  uint64_t v[16];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    v[i] = h[i];
    v[8 + i] = B2_IV[i];
  }
  v[12] ^= len;
  v[14] = ~v[14];
  for (int r = 0; r < 12; r++) {
    const uint8_t* s = B2_SIGMA[r % 10];
#define G(a, b, c, d, x, y)          \
  v[a] += v[b] + (x);                \
  v[d] = rotr64(v[d] ^ v[a], 32);    \
  v[c] += v[d];                      \
  v[b] = rotr64(v[b] ^ v[c], 24);    \
  v[a] += v[b] + (y);                \
  v[d] = rotr64(v[d] ^ v[a], 16);    \
  v[c] += v[d];                      \
  v[b] = rotr64(v[b] ^ v[c], 63);
    G(0, 4, 8, 12, m[s[0]], m[s[1]]);
    G(1, 5, 9, 13, m[s[2]], m[s[3]]);
    G(2, 6, 10, 14, m[s[4]], m[s[5]]);
    G(3, 7, 11, 15, m[s[6]], m[s[7]]);
    G(0, 5, 10, 15, m[s[8]], m[s[9]]);
    G(1, 6, 11, 12, m[s[10]], m[s[11]]);
    G(2, 7, 8, 13, m[s[12]], m[s[13]]);
    G(3, 4, 9, 14, m[s[14]], m[s[15]]);
#undef G
  }
#pragma unroll
  for (int i = 0; i < 8; i++) h[i] ^= v[i] ^ v[8 + i];
}

// One ChaCha20 block (original layout: 64-bit block counter in words 12-13, zero nonce).
__device__ inline void chacha20_block(uint32_t (&out)[16], const uint32_t (&k)[8], uint64_t block) {
  const uint32_t s[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u, k[0], k[1], k[2], k[3],
                          k[4], k[5], k[6], k[7], (uint32_t)block, (uint32_t)(block >> 32), 0u, 0u};
  uint32_t x[16];
#pragma unroll
  for (int i = 0; i < 16; i++) x[i] = s[i];
#define QR(a, b, c, d)               \
  x[a] += x[b];                      \
  x[d] = rotl32(x[d] ^ x[a], 16);    \
  x[c] += x[d];                      \
  x[b] = rotl32(x[b] ^ x[c], 12);    \
  x[a] += x[b];                      \
  x[d] = rotl32(x[d] ^ x[a], 8);     \
  x[c] += x[d];                      \
  x[b] = rotl32(x[b] ^ x[c], 7);
  for (int r = 0; r < 10; r++) {
    QR(0, 4, 8, 12);
    QR(1, 5, 9, 13);
    QR(2, 6, 10, 14);
    QR(3, 7, 11, 15);
    QR(0, 5, 10, 15);
    QR(1, 6, 11, 12);
    QR(2, 7, 8, 13);
    QR(3, 4, 9, 14);
  }
#undef QR
#pragma unroll
  for (int i = 0; i < 16; i++) out[i] = x[i] + s[i];
}

// RFC 8439 block: key words 4-11, counter word 12, nonce words 13-15.
__device__ inline void chacha20_ietf_block(uint32_t (&out)[16], const uint32_t (&k)[8], uint32_t counter,
                                           const uint32_t (&nonce)[3]) {
  const uint32_t s[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u, k[0], k[1], k[2], k[3],
                          k[4], k[5], k[6], k[7], counter, nonce[0], nonce[1], nonce[2]};
  uint32_t x[16];
#pragma unroll
  for (int i = 0; i < 16; i++) x[i] = s[i];
#define QR(a, b, c, d)               \
  x[a] += x[b];                      \
  x[d] = rotl32(x[d] ^ x[a], 16);    \
  x[c] += x[d];                      \
  x[b] = rotl32(x[b] ^ x[c], 12);    \
  x[a] += x[b];                      \
  x[d] = rotl32(x[d] ^ x[a], 8);     \
  x[c] += x[d];                      \
  x[b] = rotl32(x[b] ^ x[c], 7);
  for (int r = 0; r < 10; r++) {
    QR(0, 4, 8, 12);
    QR(1, 5, 9, 13);
    QR(2, 6, 10, 14);
    QR(3, 7, 11, 15);
    QR(0, 5, 10, 15);
    QR(1, 6, 11, 12);
    QR(2, 7, 8, 13);
    QR(3, 4, 9, 14);
  }
#undef QR
#pragma unroll
  for (int i = 0; i < 16; i++) out[i] = x[i] + s[i];
}

}  // namespace sym
}  // namespace dkgk
