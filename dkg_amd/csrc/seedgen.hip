// On-device synthetic dealer coefficients: the seeded RNG convention of
// dkg_dealer_coeffs (host_crypto.cpp) computed on the GPU, so a batch of 10,000 ceremonies or an
// n = 4096 ceremony never ships its coefficient vectors over PCIe.
//   seed(c, i)   = BLAKE2b-256("dkg-amd/v1/dealer" || master[32] || u32le c || u32le i)
//   keystream    = ChaCha20(key = seed, nonce = 0, 64-bit block counter from 0)
//   b_k = wide_reduce(block k), a_k = wide_reduce(block N + k)  (hiding polynomial first,
//   committee.rs:143-146; 64 bytes per scalar as dalek Scalar::random / from_bytes_mod_order_wide)
#include "kernels.h"
#include "points.h"
#include "sym.h"

namespace dkgk {

using namespace sym;

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

// Encryption randomness (committee.rs:171-172, elgamal.rs:137): item (row, q, w) <- block 2N + 2q + w.
__global__ __launch_bounds__(256) void k_enc_randomness(size_t rows, size_t n, size_t N,
                                                        const uint32_t* __restrict__ seeds, uint32_t* __restrict__ r) {
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= rows * 2 * n) return;
  const size_t row = e / (2 * n), qw = e % (2 * n);
  uint32_t k[8];
#pragma unroll
  for (int i = 0; i < 8; i++) k[i] = seeds[8 * row + i];
  uint32_t blk[16];
  chacha20_block(blk, k, 2 * N + qw);
  sc s;
  sc_reduce512(s, blk);
  st_words8(r + 8 * e, s.v);
}

void enc_randomness(size_t rows, size_t n, size_t N, const uint32_t* seeds, uint32_t* r, hipStream_t stream) {
  const size_t tot = rows * 2 * n;
  if (!tot) return;
  hipLaunchKernelGGL(k_enc_randomness, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, stream, rows, n, N, seeds, r);
}

void dealer_seeds(size_t rows, size_t D, size_t d0, uint32_t c0, const uint32_t* master, uint32_t* seeds,
                  hipStream_t stream) {
  if (!rows) return;
  hipLaunchKernelGGL(k_dealer_seeds, dim3((unsigned)((rows + 255) / 256)), dim3(256), 0, stream, rows, D, d0, c0,
                     master, seeds);
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
