// Integer-ALU throughput microbenchmark for gfx950 (roofline denominator).
// Each kernel runs ILP independent chains per lane; reports ops/s chip-wide.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define ILP 8
#define ITERS 4096

__global__ void k_mad64(uint32_t* out, uint32_t seed) {
  uint64_t acc[ILP]; uint32_t a = seed + threadIdx.x, b = seed ^ 0x9e3779b9u;
  for (int i = 0; i < ILP; i++) acc[i] = a + i;
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int i = 0; i < ILP; i++) acc[i] = (uint64_t)(uint32_t)acc[i] * b + (acc[i] >> 32);
  }
  uint32_t r = 0; for (int i = 0; i < ILP; i++) r ^= (uint32_t)acc[i] ^ (uint32_t)(acc[i] >> 32);
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
__global__ void k_mullo(uint32_t* out, uint32_t seed) {
  uint32_t acc[ILP]; uint32_t b = seed ^ 0x9e3779b9u;
  for (int i = 0; i < ILP; i++) acc[i] = seed + threadIdx.x + i;
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int i = 0; i < ILP; i++) acc[i] = acc[i] * b;
  }
  uint32_t r = 0; for (int i = 0; i < ILP; i++) r ^= acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
__global__ void k_mulhi(uint32_t* out, uint32_t seed) {
  uint32_t acc[ILP]; uint32_t b = seed ^ 0x9e3779b9u;
  for (int i = 0; i < ILP; i++) acc[i] = seed + threadIdx.x + i;
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int i = 0; i < ILP; i++) acc[i] = __umulhi(acc[i], b) ^ acc[i];
  }
  uint32_t r = 0; for (int i = 0; i < ILP; i++) r ^= acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
__global__ void k_mul24(uint32_t* out, uint32_t seed) {
  uint32_t acc[ILP]; uint32_t b = (seed ^ 0x9e3779b9u) & 0xffffff;
  for (int i = 0; i < ILP; i++) acc[i] = seed + threadIdx.x + i;
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int i = 0; i < ILP; i++) acc[i] = __umul24(acc[i], b) + acc[i];
  }
  uint32_t r = 0; for (int i = 0; i < ILP; i++) r ^= acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
__global__ void k_add(uint32_t* out, uint32_t seed) {
  uint32_t acc[ILP]; uint32_t b = seed ^ 0x9e3779b9u;
  for (int i = 0; i < ILP; i++) acc[i] = seed + threadIdx.x + i;
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int i = 0; i < ILP; i++) acc[i] = (acc[i] + b) ^ i;
  }
  uint32_t r = 0; for (int i = 0; i < ILP; i++) r ^= acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
__global__ void k_fma64(double* out, double seed) {
  double acc[ILP]; double b = seed * 0.999;
  for (int i = 0; i < ILP; i++) acc[i] = seed + threadIdx.x + i;
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int i = 0; i < ILP; i++) acc[i] = fma(acc[i], b, 0.5);
  }
  double r = 0; for (int i = 0; i < ILP; i++) r += acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}

template <typename F>
double timeit(F f, const char* name, double ops_per_iter_per_lane, int blocks, int threads) {
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  f(); hipDeviceSynchronize();
  hipEventRecord(a); for (int r = 0; r < 5; r++) f(); hipEventRecord(b); hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b); ms /= 5;
  double ops = (double)blocks * threads * ITERS * ILP * ops_per_iter_per_lane;
  printf("%-10s %8.3f ms  %8.3f Tops/s (instr-level)\n", name, ms, ops / (ms * 1e-3) / 1e12);
  return ops / (ms * 1e-3);
}

int main() {
  int blocks = 256 * 16, threads = 256;
  uint32_t* o; hipMalloc(&o, blocks * threads * 8);
  timeit([&] { k_mad64<<<blocks, threads>>>(o, 7); }, "mad_u64", 1, blocks, threads);
  timeit([&] { k_mullo<<<blocks, threads>>>(o, 7); }, "mul_lo32", 1, blocks, threads);
  timeit([&] { k_mulhi<<<blocks, threads>>>(o, 7); }, "mul_hi32", 2, blocks, threads);
  timeit([&] { k_mul24<<<blocks, threads>>>(o, 7); }, "mad_u24", 1, blocks, threads);
  timeit([&] { k_add<<<blocks, threads>>>(o, 7); }, "add+xor", 2, blocks, threads);
  timeit([&] { k_fma64<<<blocks, threads>>>((double*)o, 1.0); }, "fma_f64", 1, blocks, threads);
  return 0;
}
