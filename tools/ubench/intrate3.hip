// gfx950 issue rates of the non-multiply VALU instructions in the field arithmetic's carry and
// pre-multiply code (fe25519.h): 64-bit shift, shift-add, bitfield ops.  Same method as
// intrate2.hip (inline asm, 8 independent chains per lane, 2048 x 256 threads), rates relative to
// a full-rate v_add_u32 measured in the same run.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define ITERS 32768
#define BODY8(INS) INS(0) INS(1) INS(2) INS(3) INS(4) INS(5) INS(6) INS(7)
#define K32(NAME, ASM)                                                                          \
  __global__ void NAME(uint32_t* out, uint32_t s) {                                             \
    uint32_t a0 = s, a1 = s + 1, a2 = s + 2, a3 = s + 3, a4 = s + 4, a5 = s + 5, a6 = s + 6,     \
             a7 = s + 7;                                                                        \
    uint32_t b = s * 3 + threadIdx.x;                                                           \
    for (int i = 0; i < ITERS; i++) {                                                           \
      BODY8(ASM) BODY8(ASM)                                                                     \
    }                                                                                           \
    out[threadIdx.x + blockIdx.x * blockDim.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;         \
  }
#define I_ADD(k) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a##k) : "v"(b));
#define I_LSHLADD(k) asm volatile("v_lshl_add_u32 %0, %0, 4, %1" : "+v"(a##k) : "v"(b));
#define I_LSHL(k) asm volatile("v_lshlrev_b32 %0, 1, %0" : "+v"(a##k));
#define I_AND(k) asm volatile("v_and_b32 %0, %1, %0" : "+v"(a##k) : "v"(b));
#define I_BFE(k) asm volatile("v_bfe_u32 %0, %0, 3, 26" : "+v"(a##k));
#define I_LSHLOR(k) asm volatile("v_lshl_or_b32 %0, %0, 3, %1" : "+v"(a##k) : "v"(b));
#define I_ANDOR(k) asm volatile("v_and_or_b32 %0, %0, %1, %1" : "+v"(a##k) : "v"(b));
#define I_SUB(k) asm volatile("v_sub_u32 %0, %1, %0" : "+v"(a##k) : "v"(b));
#define I_MULLO(k) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a##k) : "v"(b));
K32(k_add, I_ADD)
K32(k_lshladd, I_LSHLADD)
K32(k_lshl, I_LSHL)
K32(k_and, I_AND)
K32(k_bfe, I_BFE)
K32(k_lshlor, I_LSHLOR)
K32(k_andor, I_ANDOR)
K32(k_sub, I_SUB)
K32(k_mullo, I_MULLO)
__global__ void k_lshr64(uint32_t* out, uint32_t s) {
  uint64_t a0 = s, a1 = s + 1, a2 = s + 2, a3 = s + 3, a4 = s + 4, a5 = s + 5, a6 = s + 6, a7 = s + 7;
  for (int i = 0; i < ITERS; i++) {
#define I(k) asm volatile("v_lshrrev_b64 %0, 1, %0" : "+v"(a##k));
    BODY8(I) BODY8(I)
#undef I
  }
  out[threadIdx.x + blockIdx.x * blockDim.x] = (uint32_t)(a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7);
}
typedef void (*kfn)(uint32_t*, uint32_t);
int main() {
  int blocks = 256 * 8, threads = 256;
  uint32_t* o;
  (void)hipMalloc(&o, blocks * threads * 8);
  struct {
    kfn f;
    const char* name;
  } ks[] = {{k_add, "v_add_u32"},         {k_lshladd, "v_lshl_add_u32"}, {k_lshl, "v_lshlrev_b32"},
            {k_and, "v_and_b32"},         {k_bfe, "v_bfe_u32"},          {k_lshlor, "v_lshl_or_b32"},
            {k_andor, "v_and_or_b32"},    {k_sub, "v_sub_u32"},          {k_mullo, "v_mul_lo_u32"},
            {k_lshr64, "v_lshrrev_b64"}};
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  double base = 0;
  for (int pass = 0; pass < 2; pass++)
    for (auto& k : ks) {
      hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, o, 7u);
      (void)hipDeviceSynchronize();
      (void)hipEventRecord(a);
      for (int r = 0; r < 3; r++) hipLaunchKernelGGL(k.f, dim3(blocks), dim3(threads), 0, 0, o, 7u);
      (void)hipEventRecord(b);
      (void)hipEventSynchronize(b);
      float ms;
      (void)hipEventElapsedTime(&ms, a, b);
      ms /= 3;
      double rate = (double)blocks * threads * ITERS * 16 / (ms * 1e-3);
      if (pass == 0 && base == 0) base = rate;
      if (pass == 0) continue;
      printf("%-18s %8.3f ms  %8.2f T lane-instr/s  rel-to-add %.3f\n", k.name, ms, rate / 1e12, rate / base);
    }
  return 0;
}
