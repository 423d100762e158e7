// Point-add / field-mul throughput on gfx950 plus a tiny correctness check (B*k encodings).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include "../../dkg_amd/csrc/ge25519.h"

__global__ __launch_bounds__(256) void k_encode_mults(uint32_t* out, int kmax) {
  int k = threadIdx.x + 1;
  if (k > kmax) return;
  // base point from its encoding
  const uint32_t bw[8] = {0x0aaef2e2u, 0x714ebc6au, 0x61a984a8u, 0x5f5100c5u,
                          0x6a0be358u, 0x8ddd82a5u, 0x4559a6b6u, 0x762d8de0u};
  ge_p3 B, acc;
  bool ok = ristretto_decode(B, bw);
  ge_cached bc;
  ge_to_cached(bc, B);
  ge_identity(acc);
  for (int i = 0; i < k; i++) ge_add(acc, acc, bc);
  uint32_t w[8];
  ristretto_encode(w, acc);
  for (int i = 0; i < 8; i++) out[(k - 1) * 9 + i] = w[i];
  out[(k - 1) * 9 + 8] = ok;
}

__global__ __launch_bounds__(256) void k_addrate(uint32_t* out, int iters) {
  const uint32_t bw[8] = {0x0aaef2e2u, 0x714ebc6au, 0x61a984a8u, 0x5f5100c5u,
                          0x6a0be358u, 0x8ddd82a5u, 0x4559a6b6u, 0x762d8de0u};
  ge_p3 B, acc;
  ristretto_decode(B, bw);
  ge_cached bc;
  ge_to_cached(bc, B);
  acc = B;
  acc.X.v[0] += threadIdx.x;  // decorrelate lanes (value no longer on-curve; rate only)
  for (int i = 0; i < iters; i++) ge_add(acc, acc, bc);
  uint32_t r = 0;
  for (int i = 0; i < 10; i++) r ^= acc.X.v[i] ^ acc.Y.v[i] ^ acc.Z.v[i] ^ acc.T.v[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
__global__ __launch_bounds__(256) void k_dblrate(uint32_t* out, int iters) {
  const uint32_t bw[8] = {0x0aaef2e2u, 0x714ebc6au, 0x61a984a8u, 0x5f5100c5u,
                          0x6a0be358u, 0x8ddd82a5u, 0x4559a6b6u, 0x762d8de0u};
  ge_p3 acc;
  ristretto_decode(acc, bw);
  acc.X.v[0] += threadIdx.x;
  for (int i = 0; i < iters; i++) ge_dbl<true>(acc, acc);
  uint32_t r = 0;
  for (int i = 0; i < 10; i++) r ^= acc.X.v[i] ^ acc.Y.v[i] ^ acc.Z.v[i] ^ acc.T.v[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
__global__ __launch_bounds__(256) void k_mulrate(uint32_t* out, int iters) {
  fe a, b;
  for (int i = 0; i < 10; i++) { a.v[i] = (threadIdx.x * 7919u + i * 104729u) & 0x1ffffff; b.v[i] = (i * 3u + 5u) & 0x1ffffff; }
  fe c = a, d = b;
  for (int i = 0; i < iters; i++) { fe_mul(a, a, b); fe_mul(c, c, d); }
  uint32_t r = 0;
  for (int i = 0; i < 10; i++) r ^= a.v[i] ^ c.v[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

int main() {
  uint32_t* d; (void)hipMalloc(&d, 1 << 26);
  k_encode_mults<<<1, 64>>>(d, 16);
  uint32_t h[16 * 9];
  (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  for (int k = 1; k <= 16; k++) {
    printf("B*%-2d ok=%u ", k, h[(k - 1) * 9 + 8]);
    const unsigned char* b = (const unsigned char*)&h[(k - 1) * 9];
    for (int i = 0; i < 32; i++) printf("%02x", b[i]);
    printf("\n");
  }
  hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  struct { void (*k)(uint32_t*, int); const char* name; double fe_per_iter; int tpb; } ks[] = {
    {k_addrate, "ge_add (8M)", 8, 256}, {k_dblrate, "ge_dbl (4S+4M)", 8, 256}, {k_mulrate, "fe_mul x2", 2, 256}};
  for (int pass = 0; pass < 2; pass++)
  for (auto& k : ks) {
    int blocks = 256 * 8, iters = 2000;
    hipLaunchKernelGGL(k.k, dim3(blocks), dim3(k.tpb), 0, 0, d, 10); (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(k.k, dim3(blocks), dim3(k.tpb), 0, 0, d, iters);
    (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
    float ms; (void)hipEventElapsedTime(&ms, e0, e1);
    double ops = (double)blocks * k.tpb * iters;
    if (pass) printf("%-16s %8.3f ms  %8.3f G-ops/s   %8.3f G fe-mul-equiv/s\n", k.name, ms, ops / ms / 1e6, ops * k.fe_per_iter / ms / 1e6);
  }
  return 0;
}
