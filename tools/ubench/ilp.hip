// Issue rate of ONE wave per SIMD (the latency-bound regime of a small dealer shard) as a function
// of the number of independent dependency chains per lane, for v_add_u32 and v_mad_u64_u32.
// One 256-thread workgroup per CU (64 KB of LDS forces it), so each SIMD runs exactly one wave.
// Output: cycles per instruction per wave at the measured clock (calibrated by s_memtime).
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#define ITERS 4096

template <int C>
__global__ __launch_bounds__(256) void k_add(uint32_t* out, uint64_t* clk, uint32_t s) {
  __shared__ uint32_t pad[16384];
  pad[threadIdx.x] = s;
  uint32_t a[C];
  for (int k = 0; k < C; k++) a[k] = s + k + pad[(threadIdx.x + 1) & 255];
  uint32_t b = s * 3 + threadIdx.x;
  uint64_t t0 = __builtin_readcyclecounter();
  for (int i = 0; i < ITERS; i++) {
#pragma unroll
    for (int r = 0; r < 32 / C; r++)
#pragma unroll
      for (int k = 0; k < C; k++) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a[k]) : "v"(b));
  }
  uint64_t t1 = __builtin_readcyclecounter();
  uint32_t x = 0;
  for (int k = 0; k < C; k++) x ^= a[k];
  out[threadIdx.x + blockIdx.x * blockDim.x] = x;
  if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;
}

template <int C>
__global__ __launch_bounds__(256) void k_mad(uint32_t* out, uint64_t* clk, uint32_t s) {
  __shared__ uint32_t pad[16384];
  pad[threadIdx.x] = s;
  uint64_t a[C];
  for (int k = 0; k < C; k++) a[k] = s + k + pad[(threadIdx.x + 1) & 255];
  uint32_t b = s * 3 + threadIdx.x, c = b ^ 5;
  uint64_t t0 = __builtin_readcyclecounter();
  for (int i = 0; i < ITERS; i++) {
#pragma unroll
    for (int r = 0; r < 32 / C; r++)
#pragma unroll
      for (int k = 0; k < C; k++)
        asm volatile("v_mad_u64_u32 %0, s[20:21], %1, %2, %0" : "+v"(a[k]) : "v"(b), "v"(c) : "s20", "s21");
  }
  uint64_t t1 = __builtin_readcyclecounter();
  uint32_t x = 0;
  for (int k = 0; k < C; k++) x ^= (uint32_t)a[k];
  out[threadIdx.x + blockIdx.x * blockDim.x] = x;
  if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;
}

template <typename K>
void run(const char* name, K kern, int waves_per_simd) {
  const int blocks = 256, threads = 64 * 4 * waves_per_simd;
  uint32_t* o;
  uint64_t* c;
  (void)hipMalloc(&o, 4 * blocks * 1024);
  (void)hipMalloc(&c, 8 * blocks);
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads > 256 ? 256 : threads), 0, 0, o, c, 7u);
  (void)hipDeviceSynchronize();
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads > 256 ? 256 : threads), 0, 0, o, c, 7u);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  uint64_t cyc[256];
  (void)hipMemcpy(cyc, c, 8 * blocks, hipMemcpyDeviceToHost);
  double avg = 0;
  for (int i = 0; i < blocks; i++) avg += (double)cyc[i] / blocks;
  const double instr = (double)ITERS * 32;
  printf("%-22s %8.3f ms  %7.2f counter-ticks/instr/wave  %7.2f ns/instr/wave\n", name, ms, avg / instr,
         ms * 1e6 / instr);
  (void)hipFree(o);
  (void)hipFree(c);
}

int main() {
  run("add chains=1", k_add<1>, 1);
  run("add chains=2", k_add<2>, 1);
  run("add chains=4", k_add<4>, 1);
  run("add chains=8", k_add<8>, 1);
  run("mad64 chains=1", k_mad<1>, 1);
  run("mad64 chains=2", k_mad<2>, 1);
  run("mad64 chains=4", k_mad<4>, 1);
  run("mad64 chains=8", k_mad<8>, 1);
  return 0;
}
