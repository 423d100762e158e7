// gfx950 integer-instruction throughput (inline asm, 8 independent chains per lane).
// Output: wave64 issue cycles per instruction per SIMD, assuming the measured clock
// equals the rate of a full-rate v_add_u32 (calibrated in the same run).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define ITERS 32768

#define BODY8(INS) INS(0) INS(1) INS(2) INS(3) INS(4) INS(5) INS(6) INS(7)

__global__ void k_add(uint32_t* out, uint32_t s) {
  uint32_t a0=s,a1=s+1,a2=s+2,a3=s+3,a4=s+4,a5=s+5,a6=s+6,a7=s+7; uint32_t b = s*3+threadIdx.x;
  for (int i = 0; i < ITERS; i++) {
#define I(k) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a##k) : "v"(b));
    BODY8(I) BODY8(I)
#undef I
  }
  out[threadIdx.x + blockIdx.x*blockDim.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ void k_addco(uint32_t* out, uint32_t s) {
  uint32_t a0=s,a1=s+1,a2=s+2,a3=s+3,a4=s+4,a5=s+5,a6=s+6,a7=s+7; uint32_t b = s*3+threadIdx.x;
  for (int i = 0; i < ITERS; i++) {
#define I(k) asm volatile("v_add_co_u32 %0, vcc, %0, %1\n v_addc_co_u32 %0, vcc, %0, %1, vcc" : "+v"(a##k) : "v"(b) : "vcc");
    BODY8(I)
#undef I
  }
  out[threadIdx.x + blockIdx.x*blockDim.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ void k_mad64(uint32_t* out, uint32_t s) {
  uint64_t a0=s,a1=s+1,a2=s+2,a3=s+3,a4=s+4,a5=s+5,a6=s+6,a7=s+7; uint32_t b = s*3+threadIdx.x, c = b ^ 5;
  for (int i = 0; i < ITERS; i++) {
#define I(k) asm volatile("v_mad_u64_u32 %0, s[20:21], %1, %2, %0" : "+v"(a##k) : "v"(b), "v"(c) : "s20", "s21");
    BODY8(I) BODY8(I)
#undef I
  }
  out[threadIdx.x + blockIdx.x*blockDim.x] = (uint32_t)(a0^a1^a2^a3^a4^a5^a6^a7);
}
__global__ void k_mullo(uint32_t* out, uint32_t s) {
  uint32_t a0=s,a1=s+1,a2=s+2,a3=s+3,a4=s+4,a5=s+5,a6=s+6,a7=s+7; uint32_t b = s*3+threadIdx.x;
  for (int i = 0; i < ITERS; i++) {
#define I(k) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a##k) : "v"(b));
    BODY8(I) BODY8(I)
#undef I
  }
  out[threadIdx.x + blockIdx.x*blockDim.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ void k_mulhi(uint32_t* out, uint32_t s) {
  uint32_t a0=s,a1=s+1,a2=s+2,a3=s+3,a4=s+4,a5=s+5,a6=s+6,a7=s+7; uint32_t b = s*3+threadIdx.x;
  for (int i = 0; i < ITERS; i++) {
#define I(k) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a##k) : "v"(b));
    BODY8(I) BODY8(I)
#undef I
  }
  out[threadIdx.x + blockIdx.x*blockDim.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ void k_mul24(uint32_t* out, uint32_t s) {
  uint32_t a0=s,a1=s+1,a2=s+2,a3=s+3,a4=s+4,a5=s+5,a6=s+6,a7=s+7; uint32_t b = s*3+threadIdx.x;
  for (int i = 0; i < ITERS; i++) {
#define I(k) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(a##k) : "v"(b));
    BODY8(I) BODY8(I)
#undef I
  }
  out[threadIdx.x + blockIdx.x*blockDim.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ void k_mulhi24(uint32_t* out, uint32_t s) {
  uint32_t a0=s,a1=s+1,a2=s+2,a3=s+3,a4=s+4,a5=s+5,a6=s+6,a7=s+7; uint32_t b = s*3+threadIdx.x;
  for (int i = 0; i < ITERS; i++) {
#define I(k) asm volatile("v_mul_hi_u32_u24 %0, %0, %1" : "+v"(a##k) : "v"(b));
    BODY8(I) BODY8(I)
#undef I
  }
  out[threadIdx.x + blockIdx.x*blockDim.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ void k_mad24(uint32_t* out, uint32_t s) {
  uint32_t a0=s,a1=s+1,a2=s+2,a3=s+3,a4=s+4,a5=s+5,a6=s+6,a7=s+7; uint32_t b = s*3+threadIdx.x;
  for (int i = 0; i < ITERS; i++) {
#define I(k) asm volatile("v_mad_u32_u24 %0, %0, %1, %0" : "+v"(a##k) : "v"(b));
    BODY8(I) BODY8(I)
#undef I
  }
  out[threadIdx.x + blockIdx.x*blockDim.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ void k_add3(uint32_t* out, uint32_t s) {
  uint32_t a0=s,a1=s+1,a2=s+2,a3=s+3,a4=s+4,a5=s+5,a6=s+6,a7=s+7; uint32_t b = s*3+threadIdx.x;
  for (int i = 0; i < ITERS; i++) {
#define I(k) asm volatile("v_add3_u32 %0, %0, %1, %1" : "+v"(a##k) : "v"(b));
    BODY8(I) BODY8(I)
#undef I
  }
  out[threadIdx.x + blockIdx.x*blockDim.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ void k_alignbit(uint32_t* out, uint32_t s) {
  uint32_t a0=s,a1=s+1,a2=s+2,a3=s+3,a4=s+4,a5=s+5,a6=s+6,a7=s+7; uint32_t b = s*3+threadIdx.x;
  for (int i = 0; i < ITERS; i++) {
#define I(k) asm volatile("v_alignbit_b32 %0, %0, %1, 13" : "+v"(a##k) : "v"(b));
    BODY8(I) BODY8(I)
#undef I
  }
  out[threadIdx.x + blockIdx.x*blockDim.x] = a0^a1^a2^a3^a4^a5^a6^a7;
}
__global__ void k_lshladd64(uint32_t* out, uint32_t s) {
  uint64_t a0=s,a1=s+1,a2=s+2,a3=s+3,a4=s+4,a5=s+5,a6=s+6,a7=s+7; uint64_t b = s*3+threadIdx.x;
  for (int i = 0; i < ITERS; i++) {
#define I(k) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(a##k) : "v"(b));
    BODY8(I) BODY8(I)
#undef I
  }
  out[threadIdx.x + blockIdx.x*blockDim.x] = (uint32_t)(a0^a1^a2^a3^a4^a5^a6^a7);
}
__global__ void k_fma64(uint32_t* out, uint32_t s) {
  double a0=s,a1=s+1,a2=s+2,a3=s+3,a4=s+4,a5=s+5,a6=s+6,a7=s+7; double b = 0.999 + threadIdx.x*1e-9;
  for (int i = 0; i < ITERS; i++) {
#define I(k) asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(a##k) : "v"(b));
    BODY8(I) BODY8(I)
#undef I
  }
  out[threadIdx.x + blockIdx.x*blockDim.x] = (uint32_t)(a0+a1+a2+a3+a4+a5+a6+a7);
}
__global__ void k_fma32(uint32_t* out, uint32_t s) {
  float a0=s,a1=s+1,a2=s+2,a3=s+3,a4=s+4,a5=s+5,a6=s+6,a7=s+7; float b = 0.999f + threadIdx.x*1e-9f;
  for (int i = 0; i < ITERS; i++) {
#define I(k) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(a##k) : "v"(b));
    BODY8(I) BODY8(I)
#undef I
  }
  out[threadIdx.x + blockIdx.x*blockDim.x] = (uint32_t)(a0+a1+a2+a3+a4+a5+a6+a7);
}

typedef void (*kfn)(uint32_t*, uint32_t);
int main() {
  int blocks = 256 * 8, threads = 256;
  uint32_t* o; (void)hipMalloc(&o, blocks * threads * 8);
  struct { kfn f; const char* name; double per_iter; } ks[] = {
    {k_add, "v_add_u32", 16}, {k_addco, "add_co+addc", 16}, {k_mad64, "v_mad_u64_u32", 16},
    {k_mullo, "v_mul_lo_u32", 16}, {k_mulhi, "v_mul_hi_u32", 16}, {k_mul24, "v_mul_u32_u24", 16},
    {k_mulhi24, "v_mul_hi_u32_u24", 16}, {k_mad24, "v_mad_u32_u24", 16}, {k_add3, "v_add3_u32", 16},
    {k_alignbit, "v_alignbit_b32", 16}, {k_lshladd64, "v_lshl_add_u64", 16},
    {k_fma64, "v_fma_f64", 16}, {k_fma32, "v_fma_f32", 16}};
  hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
  double base = 0;
  for (int pass = 0; pass < 2; pass++) for (auto& k : ks) {
    hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, o, 7u); (void)hipDeviceSynchronize();
    (void)hipEventRecord(a);
    for (int r = 0; r < 3; r++) hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, o, 7u);
    (void)hipEventRecord(b); (void)hipEventSynchronize(b);
    float ms; (void)hipEventElapsedTime(&ms, a, b); ms /= 3;
    double ins = (double)blocks * threads * ITERS * k.per_iter;
    double rate = ins / (ms * 1e-3);
    if (pass == 0 && base == 0) base = rate; if (pass == 0) continue;
    printf("%-18s %8.3f ms  %8.2f T lane-instr/s  rel-to-add %.3f\n", k.name, ms, rate / 1e12, rate / base);
  }
  return 0;
}
