// On-device synthetic dealer coefficients: the seeded RNG convention of
// dkg_dealer_coeffs (host_crypto.cpp) computed on the GPU, so a batch of 10,000 ceremonies or an
// n = 4096 ceremony never ships its coefficient vectors over PCIe.
//   seed(c, i)   = BLAKE2b-256("dkg-amd/v1/dealer" || master[32] || u32le c || u32le i)
//   keystream    = ChaCha20(key = seed, nonce = 0, 64-bit block counter from 0)
//   b_k = wide_reduce(block k), a_k = wide_reduce(block N + k)  (hiding polynomial first,
//   committee.rs:143-146; 64 bytes per scalar as dalek Scalar::random / from_bytes_mod_order_wide)
#include "kernels.h"
#include "points.h"

namespace dkgk {

namespace {
__device__ const uint64_t B2_IV[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL,
                                      0xa54ff53a5f1d36f1ULL, 0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL,
                                      0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};
__device__ const uint8_t B2_SIGMA[10][16] = {
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
    {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4}, {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
    {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13}, {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
    {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11}, {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
    {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5}, {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0}};

__device__ __forceinline__ uint64_t rotr64(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }
__device__ __forceinline__ uint32_t rotl32(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }

// BLAKE2b of a message of at most 128 bytes given as 16 little-endian words (zero padded).
__device__ void blake2b_1block(uint64_t (&h)[8], const uint64_t (&m)[16], uint32_t len, uint32_t outlen) {
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
__device__ void chacha20_block(uint32_t (&out)[16], const uint32_t (&k)[8], uint64_t block) {
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
}  // namespace

// 512-bit little-endian value (16 words) mod l: lo + hi * 2^256 = lo + MontMul(hi, R^2).
__device__ void sc_reduce512(sc& r, const uint32_t (&w)[16]) {
  uint32_t lo[8], hi[8];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    lo[i] = w[i];
    hi[i] = w[8 + i];
  }
  sc a, b, rr;
  sc_reduce256(a, lo);
  sc_reduce256(b, hi);
#pragma unroll
  for (int i = 0; i < 8; i++) rr.v[i] = sc_const::RR[i];
  sc_mont_mul(b, b, rr);  // hi * 2^256 mod l
  sc_add(r, a, b);
}

// Row r = ceremony (c0 + r / D) dealer (d0 + r % D): seed words [rows][8].
__global__ __launch_bounds__(256) void k_dealer_seeds(size_t rows, size_t D, size_t d0, uint32_t c0,
                                                      const uint32_t* __restrict__ master, uint32_t* __restrict__ seeds) {
  const size_t r = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= rows) return;
  const uint32_t ceremony = c0 + (uint32_t)(r / D), dealer = (uint32_t)(d0 + r % D);
  // message bytes: "dkg-amd/v1/dealer" (17) || master (32) || ceremony (4) || dealer (4) = 57 bytes
  uint8_t msg[64];
  const char tag[17] = {'d', 'k', 'g', '-', 'a', 'm', 'd', '/', 'v', '1', '/', 'd', 'e', 'a', 'l', 'e', 'r'};
#pragma unroll
  for (int i = 0; i < 17; i++) msg[i] = (uint8_t)tag[i];
#pragma unroll
  for (int i = 0; i < 32; i++) msg[17 + i] = (uint8_t)(master[i / 4] >> (8 * (i % 4)));
#pragma unroll
  for (int i = 0; i < 4; i++) {
    msg[49 + i] = (uint8_t)(ceremony >> (8 * i));
    msg[53 + i] = (uint8_t)(dealer >> (8 * i));
  }
#pragma unroll
  for (int i = 57; i < 64; i++) msg[i] = 0;
  uint64_t m[16];
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint64_t v = 0;
#pragma unroll
    for (int b = 7; b >= 0; b--) v = (v << 8) | msg[8 * i + b];
    m[i] = v;
  }
#pragma unroll
  for (int i = 8; i < 16; i++) m[i] = 0;
  uint64_t h[8];
  blake2b_1block(h, m, 57, 32);
#pragma unroll
  for (int i = 0; i < 4; i++) {
    seeds[8 * r + 2 * i] = (uint32_t)h[i];
    seeds[8 * r + 2 * i + 1] = (uint32_t)(h[i] >> 32);
  }
}

// One thread per (row, k, half): half 0 = hiding b_k (block k), half 1 = sharing a_k (block N + k).
__global__ __launch_bounds__(256) void k_dealer_coeffs(size_t rows, size_t N, const uint32_t* __restrict__ seeds,
                                                       uint32_t* __restrict__ a, uint32_t* __restrict__ b) {
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= rows * 2 * N) return;
  const size_t r = e / (2 * N), q = e % (2 * N);  // q = block index of the dealer's stream
  uint32_t k[8];
#pragma unroll
  for (int i = 0; i < 8; i++) k[i] = seeds[8 * r + i];
  uint32_t blk[16];
  chacha20_block(blk, k, q);
  sc s;
  sc_reduce512(s, blk);
  uint32_t* out = q < N ? b + 8 * (r * N + q) : a + 8 * (r * N + (q - N));
  st_words8(out, s.v);
}

void dealer_coeffs(size_t rows, size_t D, size_t d0, uint32_t c0, const uint32_t* master, size_t N, uint32_t* seeds,
                   uint32_t* a, uint32_t* b, hipStream_t stream) {
  if (!rows) return;
  hipLaunchKernelGGL(k_dealer_seeds, dim3((unsigned)((rows + 255) / 256)), dim3(256), 0, stream, rows, D, d0, c0,
                     master, seeds);
  const size_t tot = rows * 2 * N;
  hipLaunchKernelGGL(k_dealer_coeffs, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, stream, rows, N, seeds, a, b);
}

}  // namespace dkgk
