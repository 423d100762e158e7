// Where the per-step binomial's time goes: one Horner step of the headline's
// tables (n=1024, t=511, U=4: 8192 columns of L = 128 positions) through k_binom_step<true> and
// through stripped variants of the same item, each timed with HIP events over REPS launches:
//   full     k_binom_step<true> as the library runs it
//   noload   the two points come from registers (a hash of the lane), no global loads
//   nostore  loads and chain, the result is folded into one word per lane instead of stored
//   chain    only the m-chain on a register point: no loads, no first addition, no store
//   pair2    two column groups per lane (the same m: identical chains, ILP 2), 2 waves per SIMD
//   tiled    the table tiled [N][npad/64][40][64]: a wave's point is one contiguous 10-KB block
//   tiled_nt tiled, nontemporal stores;  full_nt  the library layout, nontemporal stores
// (argv: reps, first variant)
// Build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -I dkg_amd/csrc tools/ubench/binom.hip -o tools/ubench/binom
// Output: one line per (variant, r): microseconds per launch (tools/ubench/binom.py prices it).
#include "../../dkg_amd/csrc/kernels.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

namespace dkgk {

__device__ __forceinline__ void pt_fake(ge_p3& p, uint32_t seed) {
  uint32_t x = seed * 2654435761u + 12345u;
#pragma unroll
  for (int w = 0; w < PT_WORDS; w++) {
    x = x * 1664525u + 1013904223u;
    pt_word(p, w) = x & ((w & 1) ? 0x1ffffffu : 0x3ffffffu);
  }
}

// VAR 1 noload, 2 nostore, 3 chain only
template <int VAR>
__global__ __launch_bounds__(64, 4) void k_binom_var(int r, size_t npad, size_t N, const uint32_t* __restrict__ ein,
                                                     uint32_t* __restrict__ eout, uint32_t* __restrict__ flags) {
  __shared__ uint32_t qs[PT_WORDS * 64];
  uint32_t* q = qs + threadIdx.x;
  const size_t d = (size_t)blockIdx.x * 64 + threadIdx.x;
  const size_t S = N * npad;
  const int m = r - (int)blockIdx.y;
  if (m == 0) return;
  bool bad = false;
  ge_p3 x;
  if (VAR == 3) {
    pt_fake(x, (uint32_t)d + m);
  } else {
    {
      ge_p3 cur;
      if (VAR == 1) pt_fake(cur, (uint32_t)d * 3 + m);
      else pt_load(cur, ein, S, (size_t)m * npad + d);
      ge_cached cc;
      ge_to_cached_ded(cc, cur);
      lds_put_cached(q, cc);
    }
    __builtin_amdgcn_sched_barrier(0);
    if (VAR == 1) pt_fake(x, (uint32_t)d * 5 + m);
    else pt_load(x, ein, S, (size_t)(m - 1) * npad + d);
    ge_add_ded_lds(x, x, q);
    bad |= fe_tight_zero(x.Z);
  }
  mul_small_ded_lds(x, (uint32_t)m, q, bad);
  if (__ballot(bad) != 0 && threadIdx.x == 0) flags[0] = 1u;
  if (VAR == 2 || VAR == 3) {
    uint32_t acc = 0;
#pragma unroll
    for (int w = 0; w < PT_WORDS; w++) acc ^= pt_word(x, w);
    if (acc == 0x12345678u) eout[d] = acc;  // keeps the chain live; practically never stores
  } else {
    pt_store(eout, S, (size_t)m * npad + d, x);
  }
}

// pair2: two column groups per lane (ILP 2 over identical chains: the same m), 2 waves per SIMD
__device__ __forceinline__ void mul_small_ded_lds2(ge_p3 (&y)[2], uint32_t m, uint32_t* q0, uint32_t* q1,
                                                   bool& bad) {
  uint32_t pos = 0, neg = 0;
  int len = 0;
  for (uint32_t v = m; v; v >>= 1, len++) {
    if (v & 1u) {
      if ((v & 3u) == 1u) {
        pos |= 1u << len;
        v -= 1;
      } else {
        neg |= 1u << len;
        v += 1;
      }
    }
  }
  if (len <= 1) return;
  {
    ge_cached xc;
    ge_to_cached_ded(xc, y[0]);
    lds_put_cached(q0, xc);
    ge_to_cached_ded(xc, y[1]);
    lds_put_cached(q1, xc);
  }
#pragma unroll 1
  for (int i = len - 2; i >= 0; i--) {
    const uint32_t bit = 1u << i;
    const bool nz = ((pos | neg) & bit) != 0;
    ge_dbl_lean(y[0], y[0], nz || i == 0);
    ge_dbl_lean(y[1], y[1], nz || i == 0);
    if (nz) {
      ge_add_ded_lds_s(y[0], y[0], q0, (neg & bit) != 0, 64, i == 0);
      ge_add_ded_lds_s(y[1], y[1], q1, (neg & bit) != 0, 64, i == 0);
      bad |= fe_tight_zero(y[0].Z) | fe_tight_zero(y[1].Z);
    }
  }
}

__global__ __launch_bounds__(64, 2) void k_binom_pair2(int r, size_t npad, size_t N, const uint32_t* __restrict__ ein,
                                                       uint32_t* __restrict__ eout, uint32_t* __restrict__ flags) {
  __shared__ uint32_t qs[2 * PT_WORDS * 64];
  uint32_t* q0 = qs + threadIdx.x;
  uint32_t* q1 = qs + PT_WORDS * 64 + threadIdx.x;
  const size_t d0 = (size_t)blockIdx.x * 128 + threadIdx.x, d1 = d0 + 64;
  const size_t S = N * npad;
  const int m = r - (int)blockIdx.y;
  if (m == 0) return;
  bool bad = false;
  ge_p3 x[2];
  {
    ge_p3 cur;
    ge_cached cc;
    pt_load(cur, ein, S, (size_t)m * npad + d0);
    ge_to_cached_ded(cc, cur);
    lds_put_cached(q0, cc);
    pt_load(cur, ein, S, (size_t)m * npad + d1);
    ge_to_cached_ded(cc, cur);
    lds_put_cached(q1, cc);
  }
  __builtin_amdgcn_sched_barrier(0);
  pt_load(x[0], ein, S, (size_t)(m - 1) * npad + d0);
  pt_load(x[1], ein, S, (size_t)(m - 1) * npad + d1);
  ge_add_ded_lds(x[0], x[0], q0);
  ge_add_ded_lds(x[1], x[1], q1);
  bad |= fe_tight_zero(x[0].Z) | fe_tight_zero(x[1].Z);
  mul_small_ded_lds2(x, (uint32_t)m, q0, q1, bad);
  if (__ballot(bad) != 0 && threadIdx.x == 0) flags[0] = 1u;
  pt_store(eout, S, (size_t)m * npad + d0, x[0]);
  uint32_t* eo = eout;
  asm volatile("" : "+s"(eo));
  pt_store(eo, S, (size_t)m * npad + d1, x[1]);
}

// tiled: the same item on a tiled position-major table [N][npad/64][40][64] -- a wave's point is one
// contiguous 10-KB block instead of 40 rows 4 MB apart (VAR 5; VAR 6 = tiled + nontemporal stores;
// VAR 7 = the library layout with nontemporal stores)
DKG_DEV void pt_load_tiled(ge_p3& p, const uint32_t* __restrict__ blk) {
#pragma unroll
  for (int w = 0; w < PT_WORDS; w++) pt_word(p, w) = blk[w * 64 + threadIdx.x];
}
template <bool NT>
DKG_DEV void pt_store_tiled(uint32_t* __restrict__ blk, const ge_p3& p) {
#pragma unroll
  for (int w = 0; w < PT_WORDS; w++) {
    if (NT) __builtin_nontemporal_store(pt_word(p, w), blk + w * 64 + threadIdx.x);
    else blk[w * 64 + threadIdx.x] = pt_word(p, w);
  }
}
template <int VAR>
__global__ __launch_bounds__(64, 4) void k_binom_tiled(int r, size_t npad, size_t N, const uint32_t* __restrict__ ein,
                                                       uint32_t* __restrict__ eout, uint32_t* __restrict__ flags) {
  __shared__ uint32_t qs[PT_WORDS * 64];
  uint32_t* q = qs + threadIdx.x;
  const size_t g = blockIdx.x, G = npad / 64;
  const size_t d = g * 64 + threadIdx.x;
  const size_t S = N * npad;
  const int m = r - (int)blockIdx.y;
  if (m == 0) return;
  bool bad = false;
  {
    ge_p3 cur;
    if (VAR == 7) pt_load(cur, ein, S, (size_t)m * npad + d);
    else pt_load_tiled(cur, ein + ((size_t)m * G + g) * (PT_WORDS * 64));
    ge_cached cc;
    ge_to_cached_ded(cc, cur);
    lds_put_cached(q, cc);
  }
  __builtin_amdgcn_sched_barrier(0);
  ge_p3 x;
  if (VAR == 7) pt_load(x, ein, S, (size_t)(m - 1) * npad + d);
  else pt_load_tiled(x, ein + ((size_t)(m - 1) * G + g) * (PT_WORDS * 64));
  ge_add_ded_lds(x, x, q);
  bad |= fe_tight_zero(x.Z);
  mul_small_ded_lds(x, (uint32_t)m, q, bad);
  if (__ballot(bad) != 0 && threadIdx.x == 0) flags[0] = 1u;
  uint32_t* eo = eout;
  asm volatile("" : "+s"(eo));
  if (VAR == 7) {
#pragma unroll
    for (int w = 0; w < PT_WORDS; w++)
      __builtin_nontemporal_store(pt_word(x, w), eo + (size_t)w * S + (size_t)m * npad + d);
  } else {
    pt_store_tiled<VAR == 6>(eo + ((size_t)m * G + g) * (PT_WORDS * 64), x);
  }
}

}  // namespace dkgk

int main(int argc, char** argv) {
  const size_t N = 128, npad = 8192, reps = argc > 1 ? (size_t)atoi(argv[1]) : 10;
  const size_t words = PT_WORDS * N * npad;
  uint32_t *ein, *eout, *C, *flags;
  (void)hipMalloc(&ein, words * 4);
  (void)hipMalloc(&eout, words * 4);
  (void)hipMalloc(&C, words * 4);
  (void)hipMalloc(&flags, 64);
  std::vector<uint32_t> h(words);
  uint32_t x = 7;
  for (size_t i = 0; i < words; i++) {
    x = x * 1664525u + 1013904223u;
    h[i] = x & 0x1ffffffu;
  }
  (void)hipMemcpy(ein, h.data(), words * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(C, h.data(), words * 4, hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int rs[] = {16, 32, 64, 96, 127};
  const char* names[] = {"full", "noload", "nostore", "chain", "pair2", "tiled", "tiled_nt", "full_nt"};
  const int first = argc > 2 ? atoi(argv[2]) : 0;
  for (int var = first; var < 8; var++) {
    for (int r : rs) {
      const dim3 grid((unsigned)(npad / (var == 4 ? 128 : 64)), (unsigned)(r + 1));
      auto launch = [&] {
        switch (var) {
          case 0:
            hipLaunchKernelGGL(dkgk::k_binom_step<true>, grid, dim3(64), 0, nullptr, r, (int)(N - 1 - r), npad, N,
                               C, ein, eout, (size_t)2048, 32u, 3u, 0, flags, (size_t)0, (size_t)1 << 30, 64u, 1);
            break;
          case 1: hipLaunchKernelGGL(dkgk::k_binom_var<1>, grid, dim3(64), 0, nullptr, r, npad, N, ein, eout, flags); break;
          case 2: hipLaunchKernelGGL(dkgk::k_binom_var<2>, grid, dim3(64), 0, nullptr, r, npad, N, ein, eout, flags); break;
          case 3: hipLaunchKernelGGL(dkgk::k_binom_var<3>, grid, dim3(64), 0, nullptr, r, npad, N, ein, eout, flags); break;
          case 4: hipLaunchKernelGGL(dkgk::k_binom_pair2, grid, dim3(64), 0, nullptr, r, npad, N, ein, eout, flags); break;
          case 5: hipLaunchKernelGGL(dkgk::k_binom_tiled<5>, grid, dim3(64), 0, nullptr, r, npad, N, ein, eout, flags); break;
          case 6: hipLaunchKernelGGL(dkgk::k_binom_tiled<6>, grid, dim3(64), 0, nullptr, r, npad, N, ein, eout, flags); break;
          default: hipLaunchKernelGGL(dkgk::k_binom_tiled<7>, grid, dim3(64), 0, nullptr, r, npad, N, ein, eout, flags); break;
        }
      };
      launch();
      (void)hipDeviceSynchronize();
      (void)hipEventRecord(e0, nullptr);
      for (size_t i = 0; i < reps; i++) launch();
      (void)hipEventRecord(e1, nullptr);
      (void)hipEventSynchronize(e1);
      float ms = 0;
      (void)hipEventElapsedTime(&ms, e0, e1);
      const hipError_t err = hipGetLastError();
      if (err != hipSuccess) {
        fprintf(stderr, "%s\n", hipGetErrorString(err));
        return 1;
      }
      printf("%s r=%d us=%.2f\n", names[var], r, ms * 1e3 / reps);
      fflush(stdout);
    }
  }
  return 0;
}
