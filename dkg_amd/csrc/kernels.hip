// gfx950 kernels for the DKG share-generation / share-verification hot path.
// Reference loops replaced (file:line in /root/reference):
//   K1 share_eval   <- committee.rs:164-167 -> polynomial.rs:68-74
//   K2 commit       <- committee.rs:151-159
//   K3 binomial / stepping / check  <- committee.rs:287-305 (round 2), :532-548 (round 4)
//   K5 decode / encode              <- groups.rs:72-81
// See DESIGN.md for the algorithm (exact finite-difference evaluation of the committed
// polynomial in the exponent) and the roofline of each kernel.
// Built twice (dkg_amd/Makefile): as namespace dkgk with the product-scanning field
// multiplication, and with DKG_FE_ILP as namespace dkgk_ilp with the column-sum one.
#ifdef DKG_FE_ILP
#define dkgk dkgk_ilp
#endif
#include "kernels.h"
#include "split.h"

#include <algorithm>
#include <cmath>
#include "points.h"

namespace dkgk {

constexpr int COMB_WORDS = AFF_WORDS * COMB_ENTRIES;  // 15360 words = 61440 B per base

// ------------------------------------------------------------------ K5 decode / encode
// pm_N != 0: element e = i * pm_N + k (dealer-major input) is stored at k * pm_npad + i, i.e.
// straight into the position-major layout of the binomial (the decode is compute-bound, so the
// scattered 40 stores per point cost nothing next to its exponentiation, and no transpose pass or
// second copy of the points is needed).
// With interleaved segments (nseg > 1) dealer i of segment seg goes to column
// (i / 64) * 64 * nseg + seg * 64 + i % 64, and ok[] is indexed by column * pm_N + k.
#ifndef DKG_DECODE_WAVES
#define DKG_DECODE_WAVES 2
#endif
__global__ __launch_bounds__(256, DKG_DECODE_WAVES) void k_decode(const uint32_t* __restrict__ comp, size_t count,
                                                uint32_t* __restrict__ ext, size_t stride,
                                                uint8_t* __restrict__ ok, size_t pm_N, size_t pm_npad,
                                                uint32_t nseg, uint32_t seg, size_t pm_L, size_t pm_pstride) {
  size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= count) return;
  uint32_t w[8];
  ld_words8(w, comp + 8 * e);
  ge_p3 p;
  bool v = ristretto_decode(p, w);
  if (!v) ge_identity(p);
  size_t idx = e, oidx = e;
  if (pm_N) {
    const size_t i = e / pm_N, k = e % pm_N;
    const size_t col = (i / 64) * 64 * nseg + seg * 64 + i % 64;
    // degree split: coefficient k of column col is position k % L of piece k / L, whose columns
    // start pm_pstride apart (pm_L == pm_N: one piece)
    idx = (k % pm_L) * pm_npad + (k / pm_L) * pm_pstride + col;
    oidx = col * pm_N + k;
  }
  pt_store(ext, stride, idx, p);
  ok[oidx] = v ? 1 : 0;
}

// Same placement as k_decode's position-major mode for points that are already in extended form
// (round-1 commitments generated on this device: the reference's broadcasts carry group elements,
// not encodings, so nothing is decoded).  src: [D][N] points, word stride sstride.
// [D][N] dealer-major extended points -> the position-major table, one word (blockIdx.z) of a
// 64-dealer x 64-coefficient tile per workgroup through LDS: the reads run along a dealer's
// coefficients, the writes along 64 consecutive table columns (straight per-element placement wrote
// one 4-B word per lane npad words apart: 0.33 ms per 1024 x 512 segment).
__global__ __launch_bounds__(256) void k_place_pm(const uint32_t* __restrict__ src, size_t sstride, size_t D,
                                                  size_t N, uint32_t* __restrict__ out, size_t npad, uint32_t nseg,
                                                  uint32_t seg, size_t L, size_t pstride) {
  __shared__ uint32_t tile[64][65];
  const size_t w = blockIdx.z, k0 = (size_t)blockIdx.x * 64, i0 = (size_t)blockIdx.y * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
#pragma unroll
  for (int r = 0; r < 16; r++) {
    const size_t i = i0 + ty + 4 * r, k = k0 + tx;
    if (i < D && k < N) tile[ty + 4 * r][tx] = src[w * sstride + i * N + k];
  }
  __syncthreads();
  const size_t i = i0 + tx;
  const size_t col = (i / 64) * 64 * nseg + seg * 64 + i % 64;
  uint32_t* o = out + w * L * npad + col;
#pragma unroll
  for (int r = 0; r < 16; r++) {
    const size_t k = k0 + ty + 4 * r;
    if (i < D && k < N) o[(k % L) * npad + (k / L) * pstride] = tile[tx][ty + 4 * r];
  }
}

void place_position_major(const uint32_t* src, size_t sstride, size_t D, size_t N, size_t npad, uint32_t* out,
                          hipStream_t stream, int nseg, int seg, size_t L, size_t pstride) {
  if (!D || !N) return;
  if (!L) L = N;
  hipLaunchKernelGGL(k_place_pm, dim3((unsigned)((N + 63) / 64), (unsigned)((D + 63) / 64), (unsigned)PT_WORDS),
                     dim3(256), 0, stream, src, sstride, D, N, out, npad, (uint32_t)nseg, (uint32_t)seg, L, pstride);
}

// dst[i] = src[i * step + k0] for i < count (extended points; word strides sstride / dstride)
__global__ void k_gather_pts(const uint32_t* __restrict__ src, size_t sstride, size_t step, size_t k0, size_t count,
                             uint32_t* __restrict__ dst, size_t dstride) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
#pragma unroll 8
  for (int w = 0; w < PT_WORDS; w++) dst[w * dstride + i] = src[w * sstride + i * step + k0];
}

void gather_points(const uint32_t* src, size_t sstride, size_t step, size_t k0, size_t count, uint32_t* dst,
                   size_t dstride, hipStream_t stream) {
  if (!count) return;
  hipLaunchKernelGGL(k_gather_pts, dim3((unsigned)((count + 255) / 256)), dim3(256), 0, stream, src, sstride, step, k0,
                     count, dst, dstride);
}

#ifndef DKG_ENCODE_WAVES  // minimum waves per SIMD of k_encode (3: 157 VGPRs, no scratch; 4: 128 + 88 B)
#define DKG_ENCODE_WAVES 3
#endif
// DKG_ENCODE_RECOMP: only t crosses the inverse square root (u1, u2 recomputed from the reloaded point,
// two products); DKG_ENCODE_PAIR: each lane encodes points e and e + ceil(count / 2) with the two
// inverse square roots interleaved (fe_invsqrt_x2).  A/B knobs.
#ifndef DKG_ENCODE_RECOMP
#define DKG_ENCODE_RECOMP 0
#endif
#ifndef DKG_ENCODE_PAIR
#define DKG_ENCODE_PAIR 0
#endif
#if DKG_ENCODE_PAIR
__global__ __launch_bounds__(256, DKG_ENCODE_WAVES) void k_encode(const uint32_t* __restrict__ ext, size_t stride,
                                                size_t count, uint32_t* __restrict__ comp) {
  const size_t half = (count + 1) / 2;
  const size_t e0 = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e0 >= half) return;
  const size_t e1 = e0 + half;
  const bool two = e1 < count;  // an odd count's last lane encodes one point (twice)
  fe t[2], inv[2];
#pragma unroll
  for (int k = 0; k < 2; k++) {
    ge_p3 p;
    fe u1, u2;
    pt_load(p, ext, stride, (k && two) ? e1 : e0);
    ristretto_encode_pre(u1, u2, t[k], p);
  }
  fe_invsqrt_x2(inv, t);
  const uint32_t* ext2 = ext;
  asm volatile("" : "+s"(ext2));
#pragma unroll
  for (int k = 0; k < 2; k++) {
    if (k && !two) break;
    const size_t e = k ? e1 : e0;
    ge_p3 p;
    pt_load(p, ext2, stride, e);
    fe u1, u2;
    ristretto_encode_u(u1, u2, p);
    uint32_t w[8];
    ristretto_encode_post(w, p, u1, u2, inv[k]);
    st_words8(comp + 8 * e, w);
  }
}
#else
__global__ __launch_bounds__(256, DKG_ENCODE_WAVES) void k_encode(const uint32_t* __restrict__ ext, size_t stride,
                                                size_t count, uint32_t* __restrict__ comp) {
  size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= count) return;
  fe u1, u2, t, inv, one;
  {
    ge_p3 p;
    pt_load(p, ext, stride, e);
    ristretto_encode_pre(u1, u2, t, p);
  }
  fe_one(one);
  fe_sqrt_ratio_m1(inv, one, t);
  // the point again (160 B from L2 / HBM) rather than 40 registers held across the exponentiation:
  // an opaque base makes it a real reload
  const uint32_t* ext2 = ext;
  asm volatile("" : "+s"(ext2));
  ge_p3 p;
  pt_load(p, ext2, stride, e);
  if (DKG_ENCODE_RECOMP) ristretto_encode_u(u1, u2, p);
  uint32_t w[8];
  ristretto_encode_post(w, p, u1, u2, inv);
  st_words8(comp + 8 * e, w);
}
#endif

void decode_points(const uint32_t* comp, size_t count, uint32_t* ext, size_t stride, uint8_t* ok,
                   hipStream_t stream) {
  if (!count) return;
  hipLaunchKernelGGL(k_decode, dim3((unsigned)((count + 255) / 256)), dim3(256), 0, stream, comp, count,
                     ext, stride, ok, (size_t)0, (size_t)0, 1u, 0u, (size_t)1, (size_t)0);
}

void decode_position_major(const uint32_t* comp, size_t D, size_t N, size_t npad, uint32_t* out, uint8_t* ok,
                           hipStream_t stream, int nseg, int seg, size_t L, size_t pstride) {
  const size_t count = D * N;
  if (!count) return;
  if (!L) L = N;
  hipLaunchKernelGGL(k_decode, dim3((unsigned)((count + 255) / 256)), dim3(256), 0, stream, comp, count, out,
                     L * npad, ok, N, npad, (uint32_t)nseg, (uint32_t)seg, L, pstride);
}

void encode_points(const uint32_t* ext, size_t stride, size_t count, uint32_t* comp, hipStream_t stream) {
  if (!count) return;
  const size_t lanes = DKG_ENCODE_PAIR ? (count + 1) / 2 : count;
  hipLaunchKernelGGL(k_encode, dim3((unsigned)((lanes + 255) / 256)), dim3(256), 0, stream, ext, stride,
                     count, comp);
}

// ------------------------------------------------------------------ comb tables
// Thread w (0..63) builds window w: B_w = 16^w B, entries d B_w (d = 1..8) in affine Niels form.
// Workgroup g builds the table of point e0 + g into tab + g * COMB_WORDS (one table per
// workgroup, so a batch of bases -- e.g. every member's communication key -- is one launch).
__global__ __launch_bounds__(64) void k_build_comb(const uint32_t* __restrict__ ext, size_t stride, size_t e0,
                                                   uint32_t* __restrict__ tab) {
  const int w = threadIdx.x;
  tab += (size_t)blockIdx.x * COMB_WORDS;
  ge_p3 b;
  pt_load(b, ext, stride, e0 + blockIdx.x);
  for (int i = 0; i < 4 * w; i++) ge_dbl<true>(b, b);
  ge_cached bc;
  ge_to_cached(bc, b);
  ge_p3 m = b;
  fe d2;
  fe_ld(d2, ge_const::D2);
  for (int d = 1; d <= 8; d++) {
    if (d > 1) ge_add(m, m, bc);
    fe zi, x, y, t;
    fe_invert(zi, m.Z);
    fe_mul(x, m.X, zi);
    fe_mul(y, m.Y, zi);
    const int e = w * 8 + d - 1;
    fe_add(t, y, x);
    fe_carry(t, t);
#pragma unroll
    for (int i = 0; i < 10; i++) tab[i * COMB_ENTRIES + e] = t.v[i];
    fe_sub(t, y, x);
    fe_carry(t, t);
#pragma unroll
    for (int i = 0; i < 10; i++) tab[(10 + i) * COMB_ENTRIES + e] = t.v[i];
    fe_mul(t, x, y);
    fe_mul(t, t, d2);
#pragma unroll
    for (int i = 0; i < 10; i++) tab[(20 + i) * COMB_ENTRIES + e] = t.v[i];
  }
}

void build_comb(const uint32_t* ext, size_t stride, size_t e0, uint32_t* tab, hipStream_t stream, size_t count) {
  if (!count) return;
  hipLaunchKernelGGL(k_build_comb, dim3((unsigned)count), dim3(64), 0, stream, ext, stride, e0, tab);
}

__device__ __forceinline__ void lds_fill(uint32_t* lds, const uint32_t* __restrict__ g, int words) {
  const uint4* src = reinterpret_cast<const uint4*>(g);
  uint4* dst = reinterpret_cast<uint4*>(lds);
  for (int i = threadIdx.x; i < words / 4; i += blockDim.x) dst[i] = src[i];
}


// ------------------------------------------------------------------ K2 commitments
__global__ __launch_bounds__(256, DKG_COMB_WAVES) void k_commit(size_t count, const uint32_t* __restrict__ a,
                                                const uint32_t* __restrict__ b,
                                                const uint32_t* __restrict__ tab_g,
                                                const uint32_t* __restrict__ tab_h,
                                                uint32_t* __restrict__ A_ext, uint32_t* __restrict__ E_ext,
                                                size_t stride) {
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= count) return;
  sc x;  // one scalar live at a time: b is loaded after a's comb (fewer VGPRs across the chain)
  sc_load(x, a + 8 * e);
  ge_p3 acc;
  ge_identity(acc);
  combw_mul_add(acc, x, tab_g);                // apub = G::generator() * a   (committee.rs:155)
  pt_store(A_ext, stride, e, acc);
  sc_load(x, b + 8 * e);
  combw_mul_add(acc, x, tab_h);                // coeff_comm = h * b + apub   (committee.rs:156)
  pt_store(E_ext, stride, e, acc);
}

void commit(size_t count, const uint32_t* a, const uint32_t* b, const uint32_t* tab_g, const uint32_t* tab_h,
            uint32_t* A_ext, uint32_t* E_ext, hipStream_t stream, size_t stride) {
  if (!count) return;
  hipLaunchKernelGGL(k_commit, dim3((unsigned)((count + 255) / 256)), dim3(256), 0, stream, count, a, b, tab_g, tab_h,
                     A_ext, E_ext, stride ? stride : count);
}

// The commitments of dealers [0, D) written straight into the fused verification's position-major
// table (the deferred round 1 of a batch, runtime.hip BatchRound1): one wave per (64-dealer group,
// coefficient k), lanes = dealers, so the E and A columns of a group (columns 128 g + lane and
// 128 g + 64 + lane, piece k / L at position k % L) are written coalesced; no extended-form E/A
// arrays and no placement pass.  The lanes of k = 0 also write A_i0 (A0 [40][A0stride], finalise).
// 3 waves per SIMD: the comb's mixed additions need ~140 VGPRs (at 128 it spills 52 B per lane).
__global__ __launch_bounds__(64, 3) void k_commit_pm(size_t D, size_t N, const uint32_t* __restrict__ a,
                                                   const uint32_t* __restrict__ b,
                                                   const uint32_t* __restrict__ tab_g,
                                                   const uint32_t* __restrict__ tab_h, uint32_t* __restrict__ out,
                                                   size_t W, size_t L, size_t pstride,
                                                   uint32_t* __restrict__ A0, size_t A0stride) {
  const size_t g = blockIdx.x, i = g * 64 + threadIdx.x;
  const uint32_t k = blockIdx.y, Lu = (uint32_t)L;  // 32-bit: uniform position arithmetic
  if (i >= D) return;
  sc x;  // one scalar live at a time (b loaded after a's comb)
  sc_load(x, a + 8 * (i * N + k));
  ge_p3 acc;
  ge_identity(acc);
  combw_mul_add(acc, x, tab_g);                     // apub = G::generator() * a   (committee.rs:155)
  // this (position, piece) row of the table: a wave-uniform base
  uint32_t* o = out + (size_t)(k % Lu) * W + (size_t)(k / Lu) * pstride + g * 128;
  asm volatile("" : "+s"(o));
  pt_store(o + 64, L * W, threadIdx.x, acc);        // the A column (round 4)
  if (k == 0) pt_store(A0, A0stride, i, acc);
  sc_load(x, b + 8 * (i * N + k));
  combw_mul_add(acc, x, tab_h);                     // coeff_comm = h * b + apub   (committee.rs:156)
  // an opaque copy of the base again: otherwise the 40 store addresses of the A column (the same
  // words 64 columns on) stay live across h's comb and spill (168 VGPRs + 92 B of scratch per lane;
  // with it 140 VGPRs and none)
  asm volatile("" : "+s"(o));
  pt_store(o, L * W, threadIdx.x, acc);             // the E column (round 2)
}

void commit_position_major(size_t D, size_t N, const uint32_t* a, const uint32_t* b, const uint32_t* tab_g,
                           const uint32_t* tab_h, uint32_t* out, size_t W, size_t L, size_t pstride, uint32_t* A0,
                           size_t A0stride, hipStream_t stream) {
  if (!D || !N) return;
  hipLaunchKernelGGL(k_commit_pm, dim3((unsigned)((D + 63) / 64), (unsigned)N), dim3(64), 0, stream, D, N, a, b, tab_g,
                     tab_h, out, W, L, pstride, A0, A0stride);
}

// ------------------------------------------------------------------ K1 share evaluation
// Horner at x = j+1: identical field value to the power-sum of polynomial.rs:68-74.  One thread per
// (dealer i, receiver j), flattened (the dealer count of a batch of ceremonies exceeds grid.y).
__global__ __launch_bounds__(256) void k_share_eval(size_t D, size_t n, size_t N, const uint32_t* __restrict__ a,
                                                    const uint32_t* __restrict__ b, uint32_t* __restrict__ s,
                                                    uint32_t* __restrict__ sp) {
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= D * n) return;
  size_t i = e / n;
  const size_t j = e % n;
  // n % 64 == 0: a wave's lanes share the dealer, so its coefficients are scalar (broadcast) loads
  if (n % 64 == 0) i = (size_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)i);
  const uint32_t x = (uint32_t)(j + 1);
  const uint32_t* ai = a + 8 * i * N;
  const uint32_t* bi = b + 8 * i * N;
  sc fa, fb, c;
  sc_load(fa, ai + 8 * (N - 1));
  sc_load(fb, bi + 8 * (N - 1));
  size_t k = N - 1;
  if (x < 8192) {  // lazy reduction: one fold per SC_LAZY_STEPS Horner steps (sc25519.h)
    uint32_t va[10], vb[10];
#pragma unroll
    for (int i = 0; i < 10; i++) {
      va[i] = i < 8 ? fa.v[i] : 0u;
      vb[i] = i < 8 ? fb.v[i] : 0u;
    }
    while (k > 0) {
      const int steps = k < (size_t)SC_LAZY_STEPS ? (int)k : SC_LAZY_STEPS;
#pragma unroll 1
      for (int u = 0; u < steps; u++) {
        k--;
        sc_load(c, ai + 8 * k);
        sc_lazy_step(va, x, c);
        sc_load(c, bi + 8 * k);
        sc_lazy_step(vb, x, c);
      }
      sc_lazy_fold(va);
      sc_lazy_fold(vb);
    }
    sc_lazy_final(fa, va);
    sc_lazy_final(fb, vb);
  }
  while (k-- > 0) {
    sc_load(c, ai + 8 * k);
    sc_mul_small_add(fa, fa, x, c);
    sc_load(c, bi + 8 * k);
    sc_mul_small_add(fb, fb, x, c);
  }
  st_words8(s + 8 * e, fa.v);
  st_words8(sp + 8 * e, fb.v);
}

void share_eval(size_t D, size_t n, size_t N, const uint32_t* a, const uint32_t* b, uint32_t* s, uint32_t* sp,
                hipStream_t stream) {
  if (!D || !n) return;
  hipLaunchKernelGGL(k_share_eval, dim3((unsigned)((D * n + 255) / 256)), dim3(256), 0, stream, D, n, N, a, b, s,
                     sp);
}

__global__ __launch_bounds__(256) void k_poly_eval(size_t D, size_t N, const uint32_t* __restrict__ coeffs,
                                                   size_t M, const uint32_t* __restrict__ xs,
                                                   uint32_t* __restrict__ out) {
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= D * M) return;
  const size_t i = e / M, m = e % M;
  const uint32_t* ci = coeffs + 8 * i * N;
  sc f, c;
  sc_load(f, ci + 8 * (N - 1));
  for (size_t k = N - 1; k-- > 0;) {
    sc_load(c, ci + 8 * k);
    sc_mul_small_add(f, f, xs[m], c);
  }
  st_words8(out + 8 * e, f.v);
}

void poly_eval(size_t D, size_t N, const uint32_t* coeffs, size_t M, const uint32_t* xs, uint32_t* out,
               hipStream_t stream) {
  if (!D || !M) return;
  hipLaunchKernelGGL(k_poly_eval, dim3((unsigned)((D * M + 255) / 256)), dim3(256), 0, stream, D, N, coeffs, M, xs,
                     out);
}

// Paired products (ge25519.h, IL = true) per kernel family: the per-step binomial's m-chain, the
// per-wave binomial's, the recombination's chain, the checks' combs (ge_madd: its result products
// only).  Off for the binomials: capped at 128 / 168 VGPRs, the pairs push them into scratch
// (k_binom_step 0 -> 56 B per lane, k_binom_wave 28 -> 84 B; pairing only the result products
// still spills).  Each is an A/B knob.
#ifndef DKG_BINOM_IL
#define DKG_BINOM_IL 0
#endif
#ifndef DKG_WAVE_IL
#define DKG_WAVE_IL 0
#endif
#ifndef DKG_AFF_IL
#define DKG_AFF_IL 1
#endif
#ifndef DKG_CHECK_IL
#define DKG_CHECK_IL 1
#endif

// ------------------------------------------------------------------ K3a binomial-basis Horner
// y = m * y, m wave-uniform; q = this lane's column of the wave's 40 x 64-word LDS slot (clobbered).
template <bool IL = false>
__device__ __forceinline__ void mul_small_lds(ge_p3& y, uint32_t m, uint32_t* q) {
  uint32_t pos, neg;
  const int len = small_recode(m, pos, neg);
  if (len <= 1) return;
  {
    ge_cached xc;
    ge_to_cached(xc, y);
    lds_put_cached(q, xc);
  }
#pragma unroll 1
  for (int i = len - 2; i >= 0; i--) {
    const uint32_t bit = 1u << i;
    const bool nz = ((pos | neg) & bit) != 0;
    ge_dbl_lean<IL>(y, y, nz || i == 0);
    if (nz) ge_add_lds<IL>(y, y, q, (neg & bit) != 0, 64, i == 0);  // T only for the result
  }
}

// mul_small_lds with the dedicated additions (k_binom_wave<.., DED>): the base's cached form needs no
// product by d; `bad` is set when an addition's Z vanished (then the caller redoes the column group
// with the complete formula)
template <bool IL = false>
__device__ __forceinline__ void mul_small_ded_lds(ge_p3& y, uint32_t m, uint32_t* q, bool& bad) {
  uint32_t pos, neg;
  const int len = small_recode(m, pos, neg);
  if (len <= 1) return;
  {
    ge_cached xc;
    ge_to_cached_ded(xc, y);
    lds_put_cached(q, xc);
  }
#pragma unroll 1
  for (int i = len - 2; i >= 0; i--) {
    const uint32_t bit = 1u << i;
    const bool nz = ((pos | neg) & bit) != 0;
    ge_dbl_lean<IL>(y, y, nz || i == 0);
    if (nz) {
      ge_add_ded_lds_s<IL>(y, y, q, (neg & bit) != 0, 64, i == 0);  // T only for the result
      bad |= fe_tight_zero(y.Z);
    }
  }
}

// y = m * x for a wave-uniform small m (non-adjacent form, left to right).
__device__ __forceinline__ void mul_small_uniform(ge_p3& y, const ge_p3& x, uint32_t m) {
  uint32_t pos = 0, neg = 0;
  int len = 0;
  uint32_t v = m;
  while (v) {
    if (v & 1u) {
      if ((v & 3u) == 1u) {
        pos |= 1u << len;
        v -= 1;
      } else {
        neg |= 1u << len;
        v += 1;
      }
    }
    v >>= 1;
    len++;
  }
  y = x;
  if (len <= 1) return;
  ge_cached xc;
  ge_to_cached(xc, x);
  for (int i = len - 2; i >= 0; i--) {
    const uint32_t bit = 1u << i;
    const bool nz = ((pos | neg) & bit) != 0;
    ge_dbl_rt(y, y, nz || i == 0);           // T only when an addition (or the result) needs it
    if (nz) ge_add_signed(y, y, xc, (neg & bit) != 0, i == 0);
  }
}

// Radix-2^COMBW_BITS comb of point e0 + blockIdx.y of ext: block (window w = blockIdx.x, entries
// blockIdx.z * COMBW_BUILD_BS ..), thread d-1 writes d * 2^(COMBW_BITS w) B in affine Niels form
// (points.h combw_mul_add).
template <int BITS>
constexpr int comb_build_bs() { return CombGeo<BITS>::ENTRIES < 512 ? CombGeo<BITS>::ENTRIES : 512; }
template <int BITS>
__global__ __launch_bounds__(comb_build_bs<BITS>()) void k_build_combw(const uint32_t* __restrict__ ext,
                                                                        size_t stride, size_t e0,
                                                                        uint32_t* __restrict__ tab) {
  using G = CombGeo<BITS>;
  const int w = blockIdx.x, d = blockIdx.z * comb_build_bs<BITS>() + threadIdx.x + 1;
  tab += (size_t)blockIdx.y * G::WORDS;
  ge_p3 b, m;
  pt_load(b, ext, stride, e0 + blockIdx.y);
  for (int i = 0; i < BITS * w; i++) ge_dbl<true>(b, b);
  mul_small_uniform(m, b, (uint32_t)d);
  fe zi, x, y, t, d2;
  fe_ld(d2, ge_const::D2);
  fe_invert(zi, m.Z);
  fe_mul(x, m.X, zi);
  fe_mul(y, m.Y, zi);
  uint32_t* out = tab + ((size_t)w * G::ENTRIES + (d - 1)) * COMBW_STRIDE;
  fe_add(t, y, x);
  fe_carry(t, t);
#pragma unroll
  for (int i = 0; i < 10; i++) out[i] = t.v[i];
  fe_sub(t, y, x);
  fe_carry(t, t);
#pragma unroll
  for (int i = 0; i < 10; i++) out[10 + i] = t.v[i];
  fe_mul(t, x, y);
  fe_mul(t, t, d2);
#pragma unroll
  for (int i = 0; i < 10; i++) out[20 + i] = t.v[i];
  out[30] = 0;
  out[31] = 0;
}

static_assert(COMBW_WORDS * 4 == (size_t)(256 / DKG_COMBW_BITS + 1) * (1u << (DKG_COMBW_BITS - 1)) * 32 * 4,
              "runtime.hip COMBW_BYTES must match points.h");
static_assert(CombGeo<COMBW_BITS>::WORDS == COMBW_WORDS, "one comb geometry");

int fixed_base_windows() { return COMBW_WINDOWS; }

template <int BITS>
void build_combw_r(const uint32_t* ext, size_t stride, size_t e0, uint32_t* tab, hipStream_t stream, size_t count) {
  if (!count) return;
  using G = CombGeo<BITS>;
  hipLaunchKernelGGL(k_build_combw<BITS>, dim3((unsigned)G::WINDOWS, (unsigned)count, G::ENTRIES / comb_build_bs<BITS>()),
                     dim3(comb_build_bs<BITS>()), 0, stream, ext, stride, e0, tab);
}

void build_combw(const uint32_t* ext, size_t stride, size_t e0, uint32_t* tab, hipStream_t stream, size_t count) {
  build_combw_r<COMBW_BITS>(ext, stride, e0, tab, stream, count);
}

size_t key_comb_words() { return CombGeo<DKG_KEY_COMB_BITS>::WORDS; }
int key_comb_windows() { return CombGeo<DKG_KEY_COMB_BITS>::WINDOWS; }

void build_key_combs(const uint32_t* ext, size_t stride, size_t e0, uint32_t* tab, hipStream_t stream,
                     size_t count) {
  build_combw_r<DKG_KEY_COMB_BITS>(ext, stride, e0, tab, stream, count);
}

__global__ __launch_bounds__(256) void k_copy_pos(size_t width, size_t npad, size_t N, const uint32_t* __restrict__ C,
                                                  size_t kpos, uint32_t* __restrict__ e, size_t pstride) {
  const size_t dl = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (dl >= width) return;
  const size_t d = blockIdx.y * pstride + dl;  // piece blockIdx.y of a degree-split table
  const size_t S = N * npad;
#pragma unroll 8
  for (int w = 0; w < PT_WORDS; w++) e[w * S + d] = C[w * S + kpos * npad + d];
}

// The per-step binomial's table stores (k_binom_step<.., NT>): nontemporal for the large steps.
// A launch rereads the previous step's rows (each position by two items) while writing the new
// ones; once a step's rows read + written exceed the 256-MB Infinity Cache, plain stores evict the
// rows still to be read (the steps above r ~ 105 at n=1024 took 290-330 us, bimodal), while below
// it the next launch finds the plain-stored rows cached.  runtime.hip picks NT per step by that
// footprint (binom_nt, DKG_BINOM_NT_BYTES; profiles/r06_binom_levers_ab.txt).
// A/B knobs of the same kind for the other large table writers (0: plain stores, the default): the
// stepping's evaluations R and dense Z copy, the normalisation's affine addends, the per-wave binomial,
// the recombination's output -- each measured neutral on the whole ceremony (round 6, recipe r06d,
// profiles/r06_binom_levers_ab.txt), so they stay off
#ifndef DKG_STEP_NT
#define DKG_STEP_NT 0
#endif
#ifndef DKG_AFF_NT
#define DKG_AFF_NT 0
#endif
#ifndef DKG_BINOM_WAVE_NT
#define DKG_BINOM_WAVE_NT 0
#endif
#ifndef DKG_COMB_NT  // the recombination's b_j P(j) (read by the checks)
#define DKG_COMB_NT 0
#endif
template <bool NT>
DKG_DEV void binom_st(uint32_t* p, uint32_t v) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}
template <bool NT>
DKG_DEV void binom_pt_store(uint32_t* __restrict__ base, size_t stride, size_t e, const ge_p3& p) {
  if constexpr (NT) pt_store_nt(base, stride, e, p);
  else pt_store(base, stride, e, p);
}

// One Horner step in the binomial basis: e'_0 = C_k, e'_m = m (e_{m-1} + e_m), m = 1..r.
// Lanes = dealers (so m is uniform per wave: no divergence in the m-chain); one wave per
// (position, 64 dealers); position 0 just copies the next coefficient C_k.  Grid (dealer groups x
// pieces, r+1) with m = r - blockIdx.y: workgroups are dispatched x-fastest, so the longest NAF
// chains (largest m) of EVERY piece start first and the launch tail is made of the short ones.

// DED: the dedicated additions (no product by d in the cached forms); a wave whose real columns met
// Z = 0 marks flags[0] (fany: the driver's guard word, runtime.hip with_binom_ded, which reruns the
// verification with the complete formula) or flags[its (piece, column group)] (binomial_wave_redo
// rebuilds the marked groups after the last step, DKG_BINOM_STEP_DED=2).
// IL: the m-chain's doublings and additions with paired products (ge25519.h IL) under a 2-wave launch
// bound (<= 256 VGPRs, no scratch), for the steps that leave at most ~2 waves per SIMD anyway (small
// shards): there a step lasts as long as its longest chain, and pairs shorten the chain's latency.
#ifndef DKG_BINOM_STEP_WAVES  // launch bound of k_binom_step: waves per SIMD (4: <= 128 VGPRs)
#define DKG_BINOM_STEP_WAVES 4
#endif
template <bool DED, bool NT, bool IL = false>
__global__ __launch_bounds__(64, IL ? 2 : DKG_BINOM_STEP_WAVES) void k_binom_step(int r, int k, size_t npad, size_t N,
                                                    const uint32_t* __restrict__ C,
                                                    const uint32_t* __restrict__ ein, uint32_t* __restrict__ eout,
                                                    size_t pstride, unsigned gx, unsigned last_piece,
                                                    int last_off, uint32_t* __restrict__ flags, size_t col_base,
                                                    size_t dreal, unsigned gw, int fany) {
  __shared__ uint32_t qs[PT_WORDS * 64];  // this wave's cached addend (lane-interleaved)
  uint32_t* q = qs + threadIdx.x;
  const unsigned piece = blockIdx.x / gx, grp = blockIdx.x - piece * gx;
  const size_t d = piece * pstride + (size_t)grp * blockDim.x + threadIdx.x;
  const size_t S = N * npad;
  const int m = r - (int)blockIdx.y;
  if (m == 0) {
#pragma unroll 8
    for (int w = 0; w < PT_WORDS; w++) binom_st<NT>(eout + w * S + d, C[w * S + (size_t)k * npad + d]);
    return;
  }
  // A short last piece (last_off = L - its length) holds the identity in its top last_off
  // coefficients: its polynomial has degree re = r - last_off after step r, and positions above
  // re are never read (later steps mask position re, the stepping stops at the piece's length).
  const int re = r - (piece == last_piece ? last_off : 0);
  if (m > re) return;
  {
    ge_p3 cur;
    pt_load(cur, ein, S, (size_t)m * npad + d);
    // degree re-1 input: position re is zero.  Branch-free, opaque select (a visible branch lets the
    // compiler specialise the identity path and doubles the register footprint).
    uint32_t keep = (m == re) ? 0u : 0xffffffffu;
    asm volatile("" : "+v"(keep));
    uint32_t* cw = reinterpret_cast<uint32_t*>(&cur);
#pragma unroll
    for (int w = 0; w < PT_WORDS; w++) cw[w] = (cw[w] & keep) | ((w == 10 || w == 20) ? ~keep & 1u : 0u);
    ge_cached cc;
    if constexpr (DED) ge_to_cached_ded(cc, cur);
    else ge_to_cached(cc, cur);
    lds_put_cached(q, cc);
  }
  __builtin_amdgcn_sched_barrier(0);  // keep the second point's loads after the first is retired
  ge_p3 x;
  pt_load(x, ein, S, (size_t)(m - 1) * npad + d);
  if constexpr (DED) {
    bool bad = false;
    ge_add_ded_lds(x, x, q);                   // e_{m-1} + e_m
    bad |= fe_tight_zero(x.Z);
    mul_small_ded_lds<IL || DKG_BINOM_IL != 0>(x, (uint32_t)m, q, bad);  // * m
    const size_t gcol = col_base + (size_t)grp * blockDim.x + threadIdx.x;
    const bool real = (gcol / gw) * 64 + (gcol % gw) % 64 < dreal;
    if (__ballot(bad && real) != 0 && threadIdx.x == 0)  // fany: one word for the whole table
      flags[fany ? 0 : (size_t)piece * (pstride / 64) + (col_base / 64) + grp] = 1u;
  } else {
    ge_add_lds<IL>(x, x, q, false);          // e_{m-1} + e_m
    mul_small_lds<IL>(x, (uint32_t)m, q);    // * m
  }
  binom_pt_store<NT>(eout, S, (size_t)m * npad + d, x);
}

// k_binom_step with lane pairs (split.h): one wave per (position, 32 columns), each column's point
// held by two lanes that compute half of every field product each -- half the dependent
// instructions per lane for a latency-bound step (few waves per SIMD), at twice the lanes.
__global__ __launch_bounds__(64, 4) void k_binom_pair(int r, int k, size_t npad, size_t N,
                                                    const uint32_t* __restrict__ C,
                                                    const uint32_t* __restrict__ ein, uint32_t* __restrict__ eout,
                                                    size_t pstride, unsigned gx, unsigned last_piece,
                                                    int last_off) {
  __shared__ uint32_t xb[20 * 64];
  __shared__ uint32_t qs[PT_WORDS * 32];
  const int lane = threadIdx.x;
  const unsigned piece = blockIdx.x / gx, grp = blockIdx.x - piece * gx;
  const size_t d = piece * pstride + (size_t)grp * 32 + (lane >> 1);
  const size_t S = N * npad;
  const int m = r - (int)blockIdx.y;
  if (m == 0) {
    if (lane & 1) return;
#pragma unroll 8
    for (int w = 0; w < PT_WORDS; w++) eout[w * S + d] = C[w * S + (size_t)k * npad + d];
    return;
  }
  const int re = r - (piece == last_piece ? last_off : 0);
  if (m > re) return;
  const pair_ctx c{xb, qs + (lane >> 1), lane & 1, lane};
  {
    ge_p3 cur;
    pt_load(cur, ein, S, (size_t)m * npad + d);
    uint32_t keep = (m == re) ? 0u : 0xffffffffu;
    asm volatile("" : "+v"(keep));
    uint32_t* cw = reinterpret_cast<uint32_t*>(&cur);
#pragma unroll
    for (int w = 0; w < PT_WORDS; w++) cw[w] = (cw[w] & keep) | ((w == 10 || w == 20) ? ~keep & 1u : 0u);
    pair_put_cached(c, cur);
  }
  ge_p3 x;
  pt_load(x, ein, S, (size_t)(m - 1) * npad + d);
  ge_add_pair(x, x, c, false);             // e_{m-1} + e_m
  mul_small_pair(x, (uint32_t)m, c);       // * m
  if (lane & 1) return;
  pt_store(eout, S, (size_t)m * npad + d, x);
}

void binom_step_pair(size_t r, size_t width, size_t npad, size_t N, const uint32_t* C, const uint32_t* in,
                     uint32_t* out, hipStream_t stream, size_t pieces, size_t pstride, size_t last_len) {
  const int last_off = (last_len && last_len < N) ? (int)(N - last_len) : 0;
  // width is a multiple of 64: one wave per (position 0..r, 32 columns, piece)
  hipLaunchKernelGGL(k_binom_pair, dim3((unsigned)(width / 32 * pieces), (unsigned)(r + 1)), dim3(64), 0, stream,
                     (int)r, (int)(N - 1 - r), npad, N, C, in, out, pstride, (unsigned)(width / 32),
                     (unsigned)(pieces - 1), last_off);
}

void binom_init(size_t width, size_t npad, size_t N, const uint32_t* C, uint32_t* e0, hipStream_t stream,
                size_t pieces, size_t pstride) {
  hipLaunchKernelGGL(k_copy_pos, dim3((unsigned)((width + 255) / 256), (unsigned)pieces), dim3(256), 0, stream, width,
                     npad, N, C, N - 1, e0, pstride);
}

void binom_step(size_t r, size_t width, size_t npad, size_t N, const uint32_t* C, const uint32_t* in, uint32_t* out,
                hipStream_t stream, size_t pieces, size_t pstride, size_t last_len, uint32_t* flags, size_t col_base,
                size_t dreal, unsigned gw, bool flag_any, bool nt, bool il) {
  const int last_off = (last_len && last_len < N) ? (int)(N - last_len) : 0;
  // width is a multiple of 64: one wave per (position 0..r, 64 dealers, piece)
  const dim3 grid((unsigned)(width / 64 * pieces), (unsigned)(r + 1));
  auto go = [&](auto kern, uint32_t* fl, int fany) {
    hipLaunchKernelGGL(kern, grid, dim3(64), 0, stream, (int)r, (int)(N - 1 - r), npad, N, C, in, out, pstride,
                       (unsigned)(width / 64), (unsigned)(pieces - 1), last_off, fl, col_base, dreal, gw ? gw : 64u,
                       fany);
  };
  if (il) {
    if (flags && nt) go(k_binom_step<true, true, true>, flags, flag_any ? 1 : 0);
    else if (flags) go(k_binom_step<true, false, true>, flags, flag_any ? 1 : 0);
    else if (nt) go(k_binom_step<false, true, true>, nullptr, 0);
    else go(k_binom_step<false, false, true>, nullptr, 0);
    return;
  }
  if (flags && nt) go(k_binom_step<true, true>, flags, flag_any ? 1 : 0);
  else if (flags) go(k_binom_step<true, false>, flags, flag_any ? 1 : 0);
  else if (nt) go(k_binom_step<false, true>, nullptr, 0);
  else go(k_binom_step<false, false>, nullptr, 0);
}

// Every Horner step of one column group in ONE wave (short tables of many columns: config 5's
// 10,000 ceremonies x 128 columns of t + 1 = 32 positions).  One launch per step there runs 31
// launches of up to 640,000 waves that each load two points (480 B per item with the store) for a
// NAF chain of a few additions: the small-m items are HBM-bound and the large-m ones VALU-bound,
// and the launch boundaries keep the two phases apart (2.4-6.3 TB/s per launch, 0.68 of the issue
// peak over the binomial, profiles/r04_b5_schedule_ab.txt).  Here a wave walks the steps r = 1..L-1
// and, inside a step, the positions m = r..1 downwards, updating its columns' table IN PLACE
// (e_m <- m (e_{m-1} + e_m) reads the old e_{m-1}, which the next item overwrites only after
// reading it), then writes e_0 = C_{L-1-r}.  The old e_{m-1} is the next item's e_m (CARRY below),
// and the grid's waves drift through the steps independently: chain-heavy and load-heavy items
// overlap on every CU.  Before
// each step the wave drains its stores (the next step rereads them; the CU's L1 is write-through,
// so its own stores keep it current -- a workgroup-scope acquire compiles to nothing here).
// CARRY: the old e_{m-1} an item loads stays in registers as the next item's e_m (40 more VGPRs:
// 3 waves per SIMD instead of 4): one load per item instead of two -- the reread otherwise misses
// L2, evicted during the item's chain by the CU's other waves (profiles/r04_b5_schedule_ab.txt).
#ifndef DKG_BINOM_WAVE_CARRY
#define DKG_BINOM_WAVE_CARRY 1
#endif
// PF (with CARRY): the next item's e_{m-2} is loaded before this item's chain starts, so the load
// latency hides behind the chain instead of behind the other waves of the SIMD (40 more VGPRs: 2
// waves per SIMD instead of 3).
#ifndef DKG_BINOM_WAVE_WAVES  // resident waves per SIMD of the carried schedule (168 VGPRs at 3)
#define DKG_BINOM_WAVE_WAVES 3
#endif
// DED: the dedicated additions (no product by d in the cached forms: two fewer products per item);
// a wave whose real columns met an addition with Z = 0 marks flags[its group], and the same grid
// relaunched with DED = false and the flags redoes only the marked groups with the complete formula,
// from the coefficients (every position is rebuilt from C, so the first pass's table is irrelevant).
// Identity padding columns (past `dreal` dealers, `gw` columns per dealer group) never mark, and
// they are never redone: after a dedicated pass their table entries (and everything the stepping
// and recombination derive from them) are UNDEFINED (identity + identity has Z = 0).  That is safe
// because nothing reads a padding column's values: the checks, k_affine_pieces' outputs that reach
// a decision, the round outcomes and every sum over dealers index real dealers only (the checks'
// grids run over ndealers, not npad).  A new kernel that reduces across columns must keep to that.
template <bool CARRY, bool PF, bool DED>
__global__ __launch_bounds__(64, PF ? 2 : (CARRY ? DKG_BINOM_WAVE_WAVES : 4)) void k_binom_wave(int L, size_t npad,
                                                                           const uint32_t* __restrict__ C,
                                                                           uint32_t* e, size_t pstride, unsigned gx,
                                                                           unsigned last_piece, int last_off,
                                                                           uint32_t* eT, uint32_t* __restrict__ flags,
                                                                           size_t col_base, size_t dreal, unsigned gw) {
  static_assert(!PF || CARRY, "the prefetch runs on the carried schedule");
  static_assert(!DED || (CARRY && !PF), "the dedicated pass runs on the carried schedule");
  __shared__ uint32_t qs[PT_WORDS * 64];
  uint32_t* q = qs + threadIdx.x;
  const unsigned piece = blockIdx.x / gx, grp = blockIdx.x - piece * gx;
  // this group's flag word: one per (piece, dealer-column group) over the whole table
  const size_t fidx = (size_t)piece * (pstride / 64) + (col_base / 64) + grp;
  if (!DED && flags && !flags[fidx]) return;  // a redo launch: this group's table was exact
  // wave-uniform bases (SGPRs) and a 32-bit lane index: no 64-bit per-lane address stays live
  const size_t col0 = piece * pstride + (size_t)grp * 64;
  uint32_t* eb = e + col0;
  const uint32_t* cb = C + col0;
  const uint32_t lane = threadIdx.x;
  const size_t S = (size_t)L * npad;
  const int off = piece == last_piece ? last_off : 0;
  bool bad = false;
  const size_t gcol = col_base + (size_t)grp * 64 + lane;  // the column within its piece
  const bool real = (gcol / gw) * 64 + (gcol % gw) % 64 < dreal;
  // one position: no step follows, so the top coefficient goes straight into the column-major
  // table (with L = 1 both layouts are [40][npad])
  uint32_t* e_top = (L == 1 && eT) ? eT + col0 : eb;
#pragma unroll 8
  for (int w = 0; w < PT_WORDS; w++) e_top[w * S + lane] = cb[w * S + (size_t)(L - 1) * npad + lane];
#pragma unroll 1
  for (int r = 1; r < L; r++) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's stores land before it rereads them
    const int re = r - off;  // a short last piece joins late (as k_binom_step)
    ge_p3 carry, nx;
    if constexpr (CARRY) ge_identity(carry);  // position re is still the identity
    if constexpr (PF) {
      if (re >= 1) pt_load(nx, eb, S, (size_t)(re - 1) * npad + lane);
    }
#pragma unroll 1
    for (int m = re; m >= 1; m--) {
      {
        ge_cached cc;
        if constexpr (CARRY) {
          if constexpr (DED) ge_to_cached_ded(cc, carry);
          else ge_to_cached(cc, carry);
        } else {
          ge_p3 cur;
          pt_load(cur, eb, S, (size_t)m * npad + lane);
          uint32_t keep = (m == re) ? 0u : 0xffffffffu;  // position re is still the identity
          asm volatile("" : "+v"(keep));
          uint32_t* cw = reinterpret_cast<uint32_t*>(&cur);
#pragma unroll
          for (int w = 0; w < PT_WORDS; w++) cw[w] = (cw[w] & keep) | ((w == 10 || w == 20) ? ~keep & 1u : 0u);
          ge_to_cached(cc, cur);
        }
        lds_put_cached(q, cc);
      }
      __builtin_amdgcn_sched_barrier(0);
      ge_p3 x;
      if constexpr (PF) {
        x = nx;
        // item m-1's operand: position m-2 is rewritten only by item m-2, after this load
        if (m >= 2) pt_load(nx, eb, S, (size_t)(m - 2) * npad + lane);
      } else {
        pt_load(x, eb, S, (size_t)(m - 1) * npad + lane);
      }
      if constexpr (CARRY) carry = x;    // the old e_{m-1}: the next item's e_m
      if constexpr (DED) {
        ge_add_ded_lds(x, x, q);         // e_{m-1} + e_m
        bad |= fe_tight_zero(x.Z);
        mul_small_ded_lds<DKG_WAVE_IL != 0>(x, (uint32_t)m, q, bad);  // * m
      } else {
        ge_add_lds(x, x, q, false);        // e_{m-1} + e_m
        mul_small_lds(x, (uint32_t)m, q);  // * m
      }
      // an opaque copy of the base: otherwise the compiler keeps the 40 addresses of the `cur` load
      // (the same words) live across the chain for this store, and spills them
      if (r + 1 < L || !eT) {
        uint32_t* eo = eb;
        asm volatile("" : "+s"(eo));
        if (DKG_BINOM_WAVE_NT) pt_store_nt(eo, S, (size_t)m * npad + lane, x);
        else pt_store(eo, S, (size_t)m * npad + lane, x);
      } else {  // the last step writes the stepping's column-major table (no to_column_major pass):
        // the L positions of a column's word w are one line, filled by this lane within the step
        uint32_t* eo = eT + col0 * L;
        asm volatile("" : "+s"(eo));
        pt_store(eo, S, (size_t)lane * L + m, x);
      }
    }
    if (r + 1 < L || !eT) {
#pragma unroll 8
      for (int w = 0; w < PT_WORDS; w++) eb[w * S + lane] = cb[w * S + (size_t)(L - 1 - r) * npad + lane];
    } else {
      uint32_t* eo = eT + col0 * L;
#pragma unroll 8
      for (int w = 0; w < PT_WORDS; w++) eo[w * S + (size_t)lane * L] = cb[w * S + lane];
    }
  }
  if constexpr (DED) {
    if (__ballot(bad && real) != 0 && lane == 0) flags[fidx] = 1u;
  }
}

uint32_t* binomial_wave(size_t width, size_t npad, size_t N, const uint32_t* C, uint32_t* e, hipStream_t stream,
                        size_t pieces, size_t pstride, size_t last_len, uint32_t* eT, bool prefetch,
                        uint32_t* flags, size_t col_base, size_t dreal, unsigned gw) {
  const int last_off = (last_len && last_len < N) ? (int)(N - last_len) : 0;
  const dim3 grid((unsigned)(width / 64 * pieces));
  const unsigned gx = (unsigned)(width / 64), lp = (unsigned)(pieces - 1);
  if (!gw) gw = 64;
  if (prefetch) {
    hipLaunchKernelGGL((k_binom_wave<true, true, false>), grid, dim3(64), 0, stream, (int)N, npad, C, e, pstride, gx,
                       lp, last_off, eT, nullptr, col_base, dreal, gw);
  } else if (flags && DKG_BINOM_WAVE_CARRY) {  // dedicated pass, then the complete redo of marked groups
    hipLaunchKernelGGL((k_binom_wave<true, false, true>), grid, dim3(64), 0, stream, (int)N, npad, C, e, pstride, gx,
                       lp, last_off, eT, flags, col_base, dreal, gw);
    hipLaunchKernelGGL((k_binom_wave<true, false, false>), grid, dim3(64), 0, stream, (int)N, npad, C, e, pstride,
                       gx, lp, last_off, eT, flags, col_base, dreal, gw);
  } else {
    hipLaunchKernelGGL((k_binom_wave<DKG_BINOM_WAVE_CARRY != 0, false, false>), grid, dim3(64), 0, stream, (int)N,
                       npad, C, e, pstride, gx, lp, last_off, eT, nullptr, col_base, dreal, gw);
  }
  return e;
}

void binomial_wave_redo(size_t width, size_t npad, size_t N, const uint32_t* C, uint32_t* e, hipStream_t stream,
                        size_t pieces, size_t pstride, size_t last_len, uint32_t* flags, size_t col_base,
                        size_t dreal, unsigned gw) {
  const int last_off = (last_len && last_len < N) ? (int)(N - last_len) : 0;
  hipLaunchKernelGGL((k_binom_wave<true, false, false>), dim3((unsigned)(width / 64 * pieces)), dim3(64), 0, stream,
                     (int)N, npad, C, e, pstride, (unsigned)(width / 64), (unsigned)(pieces - 1), last_off, nullptr,
                     flags, col_base, dreal, gw ? gw : 64u);
}

uint32_t* binomial(size_t width, size_t npad, size_t N, const uint32_t* C, uint32_t* e0, uint32_t* e1,
                   hipStream_t stream, size_t pieces, size_t pstride, size_t last_len) {
  binom_init(width, npad, N, C, e0, stream, pieces, pstride);
  uint32_t* in = e0;
  uint32_t* out = e1;
  for (size_t r = 1; r < N; r++) {
    binom_step(r, width, npad, N, C, in, out, stream, pieces, pstride, last_len);
    std::swap(in, out);
  }
  return in;
}

// ------------------------------------------------------------------ K3b stepping
// D_m <- D_m + D_{m+1} (m = 0..t-1) once per receiver; D_0 after step j is P_i(j+1).
// Positions are cut into blocks of BS lanes (one position per lane, registers only).  D_m depends
// only on D_{m+1}, so block b never waits on block b-1: blocks run as separate launches from the
// top block down, and each launch streams its lowest position's per-step value (cached form,
// [dealer][step][40]) to the launch below.  Inside a block the neighbour value crosses lanes
// through LDS; one workgroup per dealer.  BS = 512 (80 KB of LDS, 2 workgroups = 16 waves per CU)
// keeps t = 511 in ONE launch: each launch is a chain of n dependent additions per lane, so fewer,
// wider blocks shorten the serial part when few dealers are resident (a small multi-GPU shard).

// The binomial's position-major table [40][N][npad] (lanes = columns) -> column-major [40][npad][N]
// (lanes = positions of one column, as the stepping reads it), for the columns
// [u * pstride, u * pstride + width) of each piece u.  64 x 64 tiles through LDS: both sides move
// 256 contiguous bytes per wave and word; read straight from the position-major table, a stepping
// lane's 4-byte word would cost a whole line (npad words apart).
__global__ __launch_bounds__(256) void k_to_column_major(size_t width, size_t npad, size_t N,
                                                         const uint32_t* __restrict__ e, uint32_t* __restrict__ eT,
                                                         size_t pstride) {
  __shared__ uint32_t tile[64][65];
  // one word of one 64 x 64 tile per workgroup: grid.z = piece * PT_WORDS + word
  const size_t w = blockIdx.z % PT_WORDS, base = (blockIdx.z / PT_WORDS) * pstride;
  const size_t c0 = (size_t)blockIdx.x * 64, p0 = (size_t)blockIdx.y * 64;
  const size_t S = N * npad;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < 16; i++) {
    const size_t p = p0 + ty + 4 * i, c = c0 + tx;
    if (p < N && c < width) tile[ty + 4 * i][tx] = e[w * S + p * npad + base + c];
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 16; i++) {
    const size_t c = c0 + ty + 4 * i, p = p0 + tx;
    if (p < N && c < width) eT[w * S + (base + c) * N + p] = tile[tx][ty + 4 * i];
  }
}

void to_column_major(size_t width, size_t npad, size_t N, const uint32_t* e, uint32_t* eT, size_t pieces,
                     size_t pstride, hipStream_t stream) {
  if (!width || !N) return;
  hipLaunchKernelGGL(k_to_column_major,
                     dim3((unsigned)((width + 63) / 64), (unsigned)((N + 63) / 64), (unsigned)(pieces * PT_WORDS)),
                     dim3(256), 0, stream, width, npad, N, e, eT, pstride);
}

// One launch covers position block [pos0, pos0 + P) of every dealer.  Lanes are cut into column
// slots of Ncol = (nseg - 1) P + Plast lanes, one dealer column each, holding nseg segments: pieces
// piece0 + blockIdx.y + s of a degree-split table, P lanes each except the last (Plast).  nseg = 1:
// one piece per launch (P = N when the whole table fits one block: a t = 31 table packs 8 dealers
// into a 256-lane workgroup instead of idling half of a 64-lane one).  nseg = U: every piece of a
// column in one slot (N = 512 split 192 + 192 + 128: one 512-lane workgroup per column).
//
// DED: additions by the dedicated formula (ge_add_ded_lds: no product by d, one fewer per lane and
// step); a lane whose sum comes out with Z = 0 (an exceptional pair, never for honest tables but
// reachable by crafted commitments or identity padding) marks its workgroup in flags[wg].  !DED with
// flags: the complete formula, only in the workgroups marked (the same grid is relaunched), which
// recompute their tables from the start -- so every value is the complete formula's.
//
// Receiver parts: steps j0 .. j1-1 only.  j0 > 0 starts from `sin` (the table after step j0 - 1,
// laid out like e) instead of e; j1 < nrecv leaves the table after step j1 - 1 in `sout` (another
// buffer: a part's redo launch restarts from the unchanged `sin`, and rewrites `sout` for the
// workgroups it redoes before the next part reads it).
template <int MAXBS, bool DED, bool PARTS>
__global__ __launch_bounds__(MAXBS) __attribute__((amdgpu_waves_per_eu(4, 4))) void k_stepping(
    size_t ndealers, size_t npad, size_t N, const uint32_t* __restrict__ e, size_t nrecv, size_t pos0, int P,
    const uint32_t* __restrict__ up,  // NULL: top block
    uint32_t* __restrict__ down,      // NULL: block 0
    uint32_t* __restrict__ R, size_t pstride, size_t Nlive, unsigned piece0, int nseg, int Plast,
    uint32_t* __restrict__ flags, size_t col0, size_t dreal, unsigned gw, uint32_t* __restrict__ Rz, size_t j0,
    size_t j1, const uint32_t* __restrict__ sin, uint32_t* __restrict__ sout, size_t nin, size_t nout) {
  const size_t wg = (size_t)blockIdx.y * gridDim.x + blockIdx.x;
  if (!DED && flags && !flags[wg]) return;  // a redo launch: this workgroup's tables were exact
  // Lane l's cached value sits in LDS column l (word k at cols[k * MAXBS + l]); the lane at
  // segment position q adds column q + 1 of its segment.  Column q = 0 is never read inside a
  // segment (its value leaves through `down` / R), so the segment's top lane parks the upstream
  // value there: position q reads segment column (q + 1) mod Pseg.  160 B of LDS per lane (a
  // compile-time stride keeps the address arithmetic out of the VGPR budget); the addend never
  // occupies VGPRs.
  __shared__ uint32_t cols[PT_WORDS * MAXBS];
  const int l = threadIdx.x, bs = blockDim.x;
  const int Ncol = (nseg - 1) * P + Plast;
  const int slot = l / Ncol, p = l - slot * Ncol;
  const int sg = min(p / P, nseg - 1), q = p - sg * P;
  const int Pseg = sg == nseg - 1 ? Plast : P;
  const size_t dl = (size_t)blockIdx.x * (bs / Ncol) + slot;
  const bool live = slot < bs / Ncol && dl < ndealers;
  // a column of a real dealer (dealer groups of 64 in `gw`-column groups; the padding columns of a
  // group past the last dealer hold the identity, whose dedicated additions always have Z = 0):
  // only real columns mark their workgroup for the complete redo
  const size_t gcol = col0 + dl;
  const bool real = live && (gcol / gw) * 64 + (gcol % gw) % 64 < dreal;
  const size_t d = (blockIdx.y + piece0 + sg) * pstride + dl;  // piece of a degree-split table
  const size_t S = N * npad;
  const size_t pos = pos0 + q;
  ge_p3 D;
  // positions >= Nlive (a short last piece) are the identity whatever the table holds there
  // column-major: a segment reads contiguously (a part's starting state `sin` has its own column
  // stride nin: only the positions still live there are kept)
  if (live && pos < Nlive) {
    if (PARTS && j0) pt_load(D, sin, nin * npad, d * nin + pos);
    else pt_load(D, e, S, d * N + pos);
  } else {
    ge_identity(D);
  }
  const bool top_lane = live && (q == Pseg - 1);
  const uint4* upd = (up && live) ? reinterpret_cast<const uint4*>(up + d * nrecv * PT_WORDS) : nullptr;
  uint4* downd = (down && live) ? reinterpret_cast<uint4*>(down + d * nrecv * PT_WORDS) : nullptr;
  uint32_t* mine = cols + l;
  uint32_t* base = cols + (l - q);
  const uint32_t* nbr = base + ((q + 1) % Pseg);
  bool bad = false;
  // PARTS = false: the whole receiver range, and nothing of the part machinery in the kernel (the
  // loop body sits at the 128-VGPR budget)
  const size_t jbeg = PARTS ? j0 : 0, jend = PARTS ? j1 : nrecv;
  for (size_t j = jbeg; j < jend; j++) {
    {
      ge_cached c0;
      if (DED) ge_to_cached_ded(c0, D);
      else ge_to_cached(c0, D);
      if (q == 0) {
        if (downd) {
          const uint4* w4 = reinterpret_cast<const uint4*>(&c0);
#pragma unroll
          for (int k = 0; k < PT_WORDS / 4; k++) downd[j * (PT_WORDS / 4) + k] = w4[k];
        }
      } else {
        lds_put_cached(mine, c0, MAXBS);
      }
    }
    if (top_lane && upd) {  // the block above's lowest position, parked in column 0
      ge_cached u;
      uint4* u4 = reinterpret_cast<uint4*>(&u);
#pragma unroll
      for (int k = 0; k < PT_WORDS / 4; k++) u4[k] = upd[j * (PT_WORDS / 4) + k];
      lds_put_cached(base, u, MAXBS);
    }
    __syncthreads();
    // D_pos after step j reaches an output only through D_0 after step j + pos, so positions with
    // pos + j >= nrecv are dead for the rest of the launch: a wave whose lowest position is past
    // that line skips its additions (the last 64 steps of every piece's upper wave at L = 128)
    if (live && pos + 1 < Nlive && (q + 1 < Pseg || up) && pos + j < nrecv) {
      if (DED) {
        ge_add_ded_lds(D, D, nbr, MAXBS);
        bad |= real && fe_tight_zero(D.Z);
      } else {
        ge_add_lds(D, D, nbr, false, MAXBS);
      }
    }
    __syncthreads();  // every column read before the next step overwrites it
    if (live && q == 0 && R) {
      pt_store_aos<DKG_STEP_NT != 0>(R, d * nrecv + j, D);
      // Z once more in a dense 40-B record: the affine normalisation reads only Z in its first pass
      if (Rz) {
        uint2* z2 = reinterpret_cast<uint2*>(Rz + (d * nrecv + j) * 10);
#pragma unroll
        for (int k = 0; k < 5; k++) {
          if (DKG_STEP_NT) __builtin_nontemporal_store(D.Z.v[2 * k], reinterpret_cast<uint32_t*>(z2 + k));
          if (DKG_STEP_NT) __builtin_nontemporal_store(D.Z.v[2 * k + 1], reinterpret_cast<uint32_t*>(z2 + k) + 1);
          if (!DKG_STEP_NT) z2[k] = make_uint2(D.Z.v[2 * k], D.Z.v[2 * k + 1]);
        }
      }
    }
  }
  if constexpr (PARTS) {
    if (j1 < nrecv) {  // uniform; an opaque copy keeps the index out of the loop's live set
      size_t dd = d;
      int qq = q;
      asm volatile("" : "+v"(dd), "+v"(qq));
      if (live && pos0 + qq < Nlive && pos0 + qq < nout) pt_store(sout, nout * npad, dd * nout + pos0 + qq, D);
    }
  }
  if (DED && bad) flags[wg] = 1u;  // any lane: the same value
}

// Lanes given to an N-position table: 512-lane blocks (balanced when N > 512), or P = N lanes per
// segment with floor(MAXBS / N) segments per workgroup.  MAXBS (the LDS variant: 160 B per lane)
// is picked for the most useful lanes x resident waves: a 192-lane table in the 256 variant leaves
// 4 workgroups = 12 waves per CU (LDS-bound), in the 192 variant 5 = 15 waves.
double step_occupancy(size_t bs, size_t maxbs) {
  const double wgs = std::min(std::floor(160.0 * 1024 / (160.0 * maxbs)), std::floor(16.0 / (bs / 64.0)));
  const double wps = wgs * (bs / 64.0) / 4.0;  // waves per SIMD (VGPRs cap it at 4)
  return wps >= 4 ? 1.0 : (wps >= 3 ? 0.85 + 0.15 * (wps - 3) : 0.7);
}

StepShape stepping_shape(size_t N) {
  StepShape sh;
  if (N > 512) {
    sh.nblk = (N + 511) / 512;
    sh.P = (N + sh.nblk - 1) / sh.nblk;
    sh.per = 1;
    sh.bs = (sh.P + 63) / 64 * 64;
    sh.maxbs = 512;
    return sh;
  }
  double best = -1;
  for (size_t maxbs : {256, 192, 512}) {
    if (maxbs < N) continue;
    StepShape o;
    o.nblk = 1;
    o.P = N;
    o.per = maxbs / N;
    o.bs = (o.per * N + 63) / 64 * 64;
    o.maxbs = maxbs;
    const double score = (double)(o.per * N) / o.bs * step_occupancy(o.bs, maxbs);
    if (score > best + 0.02) {
      best = score;
      sh = o;
    }
  }
  return sh;
}

// Every piece of a column in one slot: usable when the whole split table has <= 512 positions.
bool stepping_whole_columns(size_t L, size_t pieces, size_t last_len) {
  return pieces > 1 && (pieces - 1) * L + last_len <= 512;
}

// Model of stepping()'s launches in SIMD cycles per receiver step and addition instruction: each
// launch runs ceil(workgroups / resident) rounds of its long-lived workgroups; a round costs one
// wave's chain of n additions at max(w * THR / occ(w), LAT) cycles per instruction with w the
// waves per SIMD of that round: issue-shared, at a rate that still grows from 2 to 4 resident
// waves (occ 0.7 .. 1: n=4096 at U=5 runs 448-lane tables at 3.5 waves per SIMD 16 % slower
// than U=4's 512-lane ones at 4, profiles/r02_split_ab.txt), latency-bound below.
double stepping_cycles(size_t cols, size_t N, size_t pieces, size_t last_len, bool whole) {
  const double THR = 4.5, LAT = 8, SIMDS = 1024;
  if (!last_len || last_len > N) last_len = N;
  auto launch = [&](const StepShape& s, double np) {
    const double per_cu = std::min(std::floor(1024.0 / s.maxbs), std::floor(16.0 / (s.bs / 64.0)));
    const double wgs = std::ceil((double)cols / s.per) * np * s.nblk, cap = 256 * per_cu;
    const double rounds = std::ceil(wgs / cap), in_round = wgs / rounds;
    const double w = in_round * (s.bs / 64.0) / SIMDS;
    const double occ = std::min(1.0, std::max(0.7, 0.7 + 0.15 * (w - 2)));
    return rounds * std::max(w * THR / occ, LAT);
  };
  if (whole && stepping_whole_columns(N, pieces, last_len)) return launch(stepping_shape((pieces - 1) * N + last_len), 1);
  const StepShape sh = stepping_shape(N);
  if (sh.nblk > 1 || last_len == N) return launch(sh, (double)pieces);
  return (pieces > 1 ? launch(sh, (double)(pieces - 1)) : 0.0) + launch(stepping_shape(last_len), 1);
}

double stepping_waves_per_simd(size_t cols, size_t N, size_t pieces, size_t last_len, bool whole) {
  if (!last_len || last_len > N) last_len = N;
  const bool wc = whole && stepping_whole_columns(N, pieces, last_len);
  const StepShape s = stepping_shape(wc ? (pieces - 1) * N + last_len : N);
  const double np = wc ? 1.0 : (last_len == N || s.nblk > 1 ? (double)pieces : (double)(pieces - 1));
  const double per_cu = std::min(std::floor(1024.0 / s.maxbs), std::floor(16.0 / (s.bs / 64.0)));
  const double wgs = std::ceil((double)cols / s.per) * np * s.nblk, cap = 256 * per_cu;
  return wgs / std::ceil(wgs / cap) * (s.bs / 64.0) / 1024;
}

// Flag words one stepping() call may use.  A grid has at most ndealers x pieces workgroups, plus one
// launch for a short last piece; the dead-position repack of an unsplit table (stepping_tail_phases)
// runs up to TAIL_MAX_PHASES launches of at most ndealers workgroups each (512 -> 4 lanes: 8).
constexpr size_t TAIL_MAX_PHASES = 8;
size_t stepping_flag_words(size_t ndealers, size_t pieces) {
  return ndealers * (pieces == 1 ? TAIL_MAX_PHASES : pieces + 1);
}

struct ColReal {  // which table columns belong to real dealers (k_stepping's `real`); Rz: dense Z copy
  size_t col0, dreal;
  unsigned gw;
  uint32_t* Rz;
};

template <bool DED, bool PARTS>
void step_launch_p(int maxbs, dim3 grid, dim3 block, hipStream_t stream, size_t ndealers, size_t npad, size_t N,
                   const uint32_t* e, size_t nrecv, size_t pos0, int P, const uint32_t* up, uint32_t* down,
                   uint32_t* R, size_t pstride, size_t Nlive, unsigned piece0, int nseg, int Plast, uint32_t* flags,
                   const ColReal& cr, size_t j0, size_t j1, const uint32_t* sin, uint32_t* sout, size_t nin,
                   size_t nout) {
  if (maxbs == 192)
    hipLaunchKernelGGL((k_stepping<192, DED, PARTS>), grid, block, 0, stream, ndealers, npad, N, e, nrecv, pos0, P,
                       up, down, R, pstride, Nlive, piece0, nseg, Plast, flags, cr.col0, cr.dreal, cr.gw,
                       R ? cr.Rz : nullptr, j0, j1, sin, sout, nin, nout);
  else if (maxbs == 256)
    hipLaunchKernelGGL((k_stepping<256, DED, PARTS>), grid, block, 0, stream, ndealers, npad, N, e, nrecv, pos0, P,
                       up, down, R, pstride, Nlive, piece0, nseg, Plast, flags, cr.col0, cr.dreal, cr.gw,
                       R ? cr.Rz : nullptr, j0, j1, sin, sout, nin, nout);
  else
    hipLaunchKernelGGL((k_stepping<512, DED, PARTS>), grid, block, 0, stream, ndealers, npad, N, e, nrecv, pos0, P,
                       up, down, R, pstride, Nlive, piece0, nseg, Plast, flags, cr.col0, cr.dreal, cr.gw,
                       R ? cr.Rz : nullptr, j0, j1, sin, sout, nin, nout);
}

template <bool DED>
void step_launch(int maxbs, dim3 grid, dim3 block, hipStream_t stream, size_t ndealers, size_t npad, size_t N,
                 const uint32_t* e, size_t nrecv, size_t pos0, int P, const uint32_t* up, uint32_t* down,
                 uint32_t* R, size_t pstride, size_t Nlive, unsigned piece0, int nseg, int Plast, uint32_t* flags,
                 const ColReal& cr, size_t j0, size_t j1, const uint32_t* sin, uint32_t* sout, size_t nin = 0,
                 size_t nout = 0) {
  if (j0 != 0 || j1 != nrecv)
    step_launch_p<DED, true>(maxbs, grid, block, stream, ndealers, npad, N, e, nrecv, pos0, P, up, down, R, pstride,
                             Nlive, piece0, nseg, Plast, flags, cr, j0, j1, sin, sout, nin ? nin : N,
                             nout ? nout : N);
  else
    step_launch_p<DED, false>(maxbs, grid, block, stream, ndealers, npad, N, e, nrecv, pos0, P, up, down, R, pstride,
                              Nlive, piece0, nseg, Plast, flags, cr, 0, nrecv, nullptr, nullptr, N, N);
}

// Dead-position repack: worth its state copies when the dead lane-steps are a large share of the
// launch (about N / 2n of them: config 5, n = 64, t = 31, 24 %), not for long tables of big
// ceremonies whose dead positions fill only the upper wave of the last N steps (n = 1024: 3 %).
constexpr size_t TAIL_MIN_P = 4;
int stepping_tail_phases(size_t N, size_t nrecv, size_t pieces) {
  if (pieces != 1 || N > 512 || N < 2 * TAIL_MIN_P || 10 * N < 2 * nrecv || nrecv + 1 < N) return 1;
  int k = 1;
  for (size_t P = N / 2; P >= TAIL_MIN_P; P /= 2) k++;
  static_assert(TAIL_MIN_P << (TAIL_MAX_PHASES - 1) >= 512, "flag words of the tail phases");
  return k;
}
size_t stepping_tail_words(size_t ndealers, size_t N) { return PT_WORDS * ndealers * (N / 2); }

bool stepping(size_t ndealers, size_t npad, size_t N, const uint32_t* e, size_t nrecv, uint32_t* R,
              uint32_t* stream_a, uint32_t* stream_b, hipStream_t stream, size_t pieces, size_t pstride,
              size_t last_len, bool whole, uint32_t* flags, size_t col0, size_t dreal, unsigned gw, uint32_t* Rz,
              uint32_t* tail_a, uint32_t* tail_b) {
  if (!ndealers || !nrecv) return true;
  const ColReal cr{col0, dreal, gw ? gw : 64u, Rz};
  if (!last_len || last_len > N) last_len = N;
  // with flags (stepping_flag_words zeroed words): every launch below runs dedicated, then again
  // complete in its marked workgroups (its own flag words: a grid has at most ndealers x pieces);
  // a layout that would pass stepping_flag_words fails the call before anything is launched
  size_t foff = 0;
  const size_t fcap = flags ? stepping_flag_words(ndealers, pieces) : 0;
  auto fits = [&](size_t words) { return !flags || foff + words <= fcap; };
  auto run = [&](int maxbs, dim3 grid, dim3 block, size_t pos0, int P, const uint32_t* up, uint32_t* down,
                 uint32_t* Rout, size_t Nlive, unsigned piece0, int nseg, int Plast, uint32_t* f) {
    if (f) {
      step_launch<true>(maxbs, grid, block, stream, ndealers, npad, N, e, nrecv, pos0, P, up, down, Rout, pstride,
                        Nlive, piece0, nseg, Plast, f, cr, 0, nrecv, nullptr, nullptr);
    }
    step_launch<false>(maxbs, grid, block, stream, ndealers, npad, N, e, nrecv, pos0, P, up, down, Rout, pstride,
                       Nlive, piece0, nseg, Plast, f, cr, 0, nrecv, nullptr, nullptr);
  };
  auto launch = [&](const StepShape& s, size_t Nlive, unsigned piece0, size_t np, int nseg, int Plast) {
    const dim3 grid((unsigned)((ndealers + s.per - 1) / s.per), (unsigned)np), block((unsigned)s.bs);
    if (!fits((size_t)grid.x * grid.y)) return false;
    uint32_t* f = flags ? flags + foff : nullptr;
    foff += (size_t)grid.x * grid.y;
    run((int)s.maxbs, grid, block, 0, (int)s.P, nullptr, nullptr, R, Nlive, piece0, nseg, Plast, f);
    return true;
  };
  const int phases = (tail_a && tail_b) ? stepping_tail_phases(N, nrecv, pieces) : 1;
  if (phases > 1) {
    // phase k: steps [J_k, J_{k+1}) on P_k-lane segments, J_k = nrecv - P_k + 1; it starts from the
    // state phase k-1 left (P_k positions, stride P_k) and leaves P_{k+1} positions for phase k+1.
    // Each phase's redo launch restarts from its unchanged starting state (the other buffer).
    // the compact states keep ONE layout for every phase, [40][npad][N/2] (positions past a phase's
    // segment unused): the chunks of a verification run their phases on their own streams at their
    // own pace, and a phase-dependent stride would let one chunk's state overlap another's columns
    uint32_t* st[2] = {tail_a, tail_b};
    const size_t Nh = N / 2;
    size_t P = N, j0 = 0;
    for (int k = 0; k < phases; k++) {
      const size_t Pn = P / 2, j1 = k + 1 < phases ? nrecv - Pn + 1 : nrecv;
      const StepShape s = stepping_shape(P);
      const dim3 grid((unsigned)((ndealers + s.per - 1) / s.per), 1u), block((unsigned)s.bs);
      if (!fits(grid.x)) return false;
      uint32_t* f = flags ? flags + foff : nullptr;
      foff += grid.x;
      // the states are laid out for the whole table ([40][npad][Nh], word-row stride Nh npad): this
      // call's columns start at col0
      const uint32_t* sin = k ? st[(k - 1) % 2] + col0 * Nh : nullptr;
      uint32_t* sout = k + 1 < phases ? st[k % 2] + col0 * Nh : nullptr;
      for (int pass = f ? 0 : 1; pass < 2; pass++) {
        if (pass == 0)
          step_launch_p<true, true>((int)s.maxbs, grid, block, stream, ndealers, npad, N, e, nrecv, 0, (int)P,
                                    nullptr, nullptr, R, 0, N, 0u, 1, (int)P, f, cr, j0, j1, sin, sout, Nh, Nh);
        else
          step_launch_p<false, true>((int)s.maxbs, grid, block, stream, ndealers, npad, N, e, nrecv, 0, (int)P,
                                     nullptr, nullptr, R, 0, N, 0u, 1, (int)P, f, cr, j0, j1, sin, sout, Nh, Nh);
      }
      P = Pn;
      j0 = j1;
    }
    return true;
  }
  if (whole && stepping_whole_columns(N, pieces, last_len)) {
    // one slot of (pieces - 1) N + last_len lanes per column: every workgroup does the same work
    // (a column), so a launch of ndealers columns has no tail of lone pieces
    StepShape s = stepping_shape((pieces - 1) * N + last_len);
    s.P = N;
    return launch(s, N, 0u, 1, (int)pieces, (int)last_len);
  }
  const StepShape sh = stepping_shape(N);
  if (sh.nblk > 1) {  // one dealer per workgroup, top block first, block values streamed down
    // the blocks of a column share one flag word (same grid in every block launch): the dedicated
    // pass runs all blocks top-down, then the complete pass redoes all blocks of marked columns
    auto blocks = [&](size_t Nlive, unsigned piece0, size_t np) {
      const dim3 grid((unsigned)ndealers, (unsigned)np), block((unsigned)sh.bs);
      if (!fits((size_t)grid.x * grid.y)) return false;
      uint32_t* f = flags ? flags + foff : nullptr;
      foff += (size_t)grid.x * grid.y;
      for (int pass = f ? 0 : 1; pass < 2; pass++) {
        uint32_t* up = nullptr;
        for (size_t b = sh.nblk; b-- > 0;) {
          uint32_t* down = b ? ((sh.nblk - 1 - b) % 2 ? stream_b : stream_a) : nullptr;
          if (pass == 0)
            step_launch<true>(512, grid, block, stream, ndealers, npad, N, e, nrecv, b * sh.P, (int)sh.P, up, down,
                              b ? nullptr : R, pstride, Nlive, piece0, 1, (int)sh.P, f, cr, 0, nrecv,
                              nullptr, nullptr);
          else
            step_launch<false>(512, grid, block, stream, ndealers, npad, N, e, nrecv, b * sh.P, (int)sh.P, up, down,
                               b ? nullptr : R, pstride, Nlive, piece0, 1, (int)sh.P, f, cr, 0, nrecv,
                              nullptr, nullptr);
          up = down;
        }
      }
      return true;
    };
    // a short last piece runs the same blocks with its positions >= last_len as the identity
    if (last_len == N || pieces == 1) return blocks(last_len, 0u, pieces);
    return blocks(N, 0u, pieces - 1) && blocks(last_len, (unsigned)(pieces - 1), 1);
  }
  // whole table in one segment of N lanes, sh.per tables per workgroup; a short last piece in its
  // own launch with segments of last_len lanes (the same column-major stride N)
  if (last_len == N) return launch(sh, N, 0u, pieces, 1, (int)sh.P);
  if (pieces > 1 && !launch(sh, N, 0u, pieces - 1, 1, (int)sh.P)) return false;
  const StepShape sl = stepping_shape(last_len);
  return launch(sl, last_len, (unsigned)(pieces - 1), 1, 1, (int)sl.P);
}

// Degree split: P(x) = sum_u x^(uL) Q_u(x).  With the stepped values Q_u(j) of
// the U pieces in columns u * pstride + c, P(j) = sum_u y^u Q_u(j), y = j^L mod l, replaces the
// piece-0 value.  Lanes = columns, blockIdx.y = receiver: the multipliers are wave-uniform.  The
// pieces are taken in pairs, Horner in y^2:  acc <- y^2 acc + y Q_{2v+1} + Q_{2v},  each step one
// joint (Straus-Shamir) double-and-add over the NAFs of y^2 and y (253 doublings for both
// products) with the two addends' cached forms parked in LDS; the top pair of an even U starts
// with y Q_{U-1} + Q_{U-2}.  digits[j][s][0..255] in {0, +1, -1} is the NAF of y (s = 0) and
// y^2 (s = 1), top[j][s] its highest nonzero digit (-1: zero).
template <int SLOTS>
__global__ __launch_bounds__(64, SLOTS == 1 ? 4 : 2) void k_combine(size_t width, size_t pstride, int pieces, size_t nrecv,
                                                 const int8_t* __restrict__ digits, const int16_t* __restrict__ top,
                                                 uint32_t* __restrict__ R) {
  __shared__ uint32_t qs[SLOTS * PT_WORDS * 64];
  uint32_t* slot_y = qs + threadIdx.x;                   // addend of y's digits
  uint32_t* slot_y2 = qs + (SLOTS - 1) * PT_WORDS * 64 + threadIdx.x;  // of y^2's (SLOTS == 2)
  const size_t c = (size_t)blockIdx.x * 64 + threadIdx.x;
  const size_t j = blockIdx.y;
  const bool live = c < width;
  const size_t cc = live ? c : 0;
  const int8_t* d1 = digits + j * 512;
  const int8_t* d2 = d1 + 256;
  const int t1 = top[2 * j], t2 = top[2 * j + 1];
  auto load_q = [&](ge_p3& q, int u) { pt_load_aos(q, R, ((size_t)u * pstride + cc) * nrecv + j); };
  auto put = [&](uint32_t* slot, const ge_p3& p) {
    ge_cached xc;
    ge_to_cached(xc, p);
    lds_put_cached(slot, xc);
  };
  ge_p3 acc, q;
  int v = (pieces - 1) / 2;
  if (pieces % 2 == 0) {  // top pair: y Q_{2v+1} + Q_{2v}
    load_q(acc, 2 * v + 1);
    put(slot_y, acc);
#pragma unroll 1
    for (int b = t1 - 1; b >= 0; b--) {  // leading NAF digit +1: acc already holds 1 * Q
      const int dg = __builtin_amdgcn_readfirstlane((int)d1[b]);
      ge_dbl_lean(acc, acc, dg != 0 || b == 0);
      if (dg != 0) ge_add_lds(acc, acc, slot_y, dg < 0, 64, b == 0);
    }
    load_q(q, 2 * v);
    put(slot_y, q);  // the chain is done with slot_y: the last addend goes through LDS too
    ge_add_lds(acc, acc, slot_y, false);
  } else {
    load_q(acc, 2 * v);
  }
  if (SLOTS == 2) {
#pragma unroll 1
    for (v = v - 1; v >= 0; v--) {  // acc <- y^2 acc + y Q_{2v+1} + Q_{2v}
      put(slot_y2, acc);
      load_q(q, 2 * v + 1);
      put(slot_y, q);
      ge_identity(acc);
#pragma unroll 1
      for (int b = (t1 > t2 ? t1 : t2); b >= 0; b--) {
        const int e1 = __builtin_amdgcn_readfirstlane((int)d1[b]);
        const int e2 = __builtin_amdgcn_readfirstlane((int)d2[b]);
        ge_dbl_lean(acc, acc, e1 != 0 || e2 != 0 || b == 0);
        if (e2 != 0) ge_add_lds(acc, acc, slot_y2, e2 < 0, 64, e1 != 0 || b == 0);
        if (e1 != 0) ge_add_lds(acc, acc, slot_y, e1 < 0, 64, b == 0);
      }
      load_q(q, 2 * v);
      put(slot_y, q);
      ge_add_lds(acc, acc, slot_y, false);
    }
  }
  if (live) pt_store_aos<DKG_COMB_NT != 0>(R, c * nrecv + j, acc);
}

// Recombination with short multipliers (lattice.cpp, U = K <= 4): b_j P(j) = sum_u v_ju Q_u(j) with
// v_j = (b_j, a_j1, ..) entries of ~253 (K-1)/K bits, in ONE joint double-and-add chain over the K
// NAFs (126 / 168 / 189 doublings for K = 2 / 3 / 4 instead of 253 per pair of pieces); the checks
// compare b_j P(j) with g*(b_j s) + h*(b_j s').  The first KL addends' cached forms are parked in
// LDS (10 KB each per wave), the others stay in VGPRs, so that K = 3 and 4 keep 2 waves per SIMD.
// digits[j][b] packs the K signed digits of position b, one byte each; top[j] the highest position.
// (Compile-time recursion over the pieces keeps the register-resident addends out of scratch.)
// digits of pieces above U at this chain position (wave-uniform): another addition follows
template <int U, int K>
DKG_DEV bool higher_digits(uint32_t w) {
  if constexpr (U + 1 < K) return (w >> (8 * (U + 1))) != 0;
  else return false;
}
// the same over the 64-bit digit word of up to 8 pieces (k_combine_aff: piece u in byte u)
template <int U, int K>
DKG_DEV bool higher_digits64(uint64_t w) {
  if constexpr (U + 1 < K) return (w >> (8 * (U + 1))) != 0;
  else return false;
}

template <int U, int K, int KL>
DKG_DEV void short_addends(uint32_t* qs, ge_cached* qr, const uint32_t* R, size_t pstride, size_t cc, size_t nrecv,
                           size_t j) {
  if constexpr (U < K) {
    ge_p3 q;
    pt_load_aos(q, R, ((size_t)U * pstride + cc) * nrecv + j);
    if constexpr (U < KL) {
      ge_cached xc;
      ge_to_cached(xc, q);
      lds_put_cached(qs + U * PT_WORDS * 64 + threadIdx.x, xc);
    } else {
      ge_to_cached(qr[U - KL], q);
    }
    short_addends<U + 1, K, KL>(qs, qr, R, pstride, cc, nrecv, j);
  }
}
template <int U, int K, int KL>
DKG_DEV void short_position(ge_p3& acc, uint32_t w, const uint32_t* qs, const ge_cached* qr, bool last) {
  if constexpr (U < K) {
    const int e = (int8_t)(w >> (8 * U));
    if (e != 0) {
      const bool t = last || higher_digits<U, K>(w);  // else a doubling follows: no T
      if constexpr (U < KL) ge_add_lds(acc, acc, qs + U * PT_WORDS * 64 + threadIdx.x, e < 0, 64, t);
      else ge_add_signed(acc, acc, qr[U - KL], e < 0, t);
    }
    short_position<U + 1, K, KL>(acc, w, qs, qr, last);
  }
}

template <int K, int KL>
__global__ __launch_bounds__(64, K == 2 ? 3 : 2) void k_combine_short(size_t width, size_t pstride, size_t nrecv,
                                                        const uint32_t* __restrict__ digits,
                                                        const int16_t* __restrict__ top, uint32_t* __restrict__ R) {
  __shared__ uint32_t qs[KL * PT_WORDS * 64];
  const size_t c = (size_t)blockIdx.x * 64 + threadIdx.x;
  const size_t j = blockIdx.y;
  const bool live = c < width;
  const size_t cc = live ? c : 0;
  ge_cached qr[K - KL > 0 ? K - KL : 1];
  short_addends<0, K, KL>(qs, qr, R, pstride, cc, nrecv, j);
  const uint32_t* dw = digits + j * 256;
  const int tp = top[j];
  ge_p3 acc;
  ge_identity(acc);
#pragma unroll 1
  for (int b = tp; b >= 0; b--) {
    const uint32_t w = __builtin_amdgcn_readfirstlane(dw[b]);
    if (b != tp) ge_dbl_lean(acc, acc, w != 0 || b == 0);
    short_position<0, K, KL>(acc, w, qs, qr, b == 0);
  }
  if (live) pt_store_aos<DKG_COMB_NT != 0>(R, c * nrecv + j, acc);
}

void combine_short(size_t width, size_t pstride, size_t pieces, size_t nrecv, const uint32_t* digits,
                   const int16_t* top, uint32_t* R, hipStream_t stream) {
  if (!width || !nrecv || pieces < 2 || pieces > 4) return;
  const dim3 grid((unsigned)((width + 63) / 64), (unsigned)nrecv);
  if (pieces == 2)
    hipLaunchKernelGGL((k_combine_short<2, 1>), grid, dim3(64), 0, stream, width, pstride, nrecv, digits, top, R);
  else if (pieces == 3)
    hipLaunchKernelGGL((k_combine_short<3, 2>), grid, dim3(64), 0, stream, width, pstride, nrecv, digits, top, R);
  else
    hipLaunchKernelGGL((k_combine_short<4, 2>), grid, dim3(64), 0, stream, width, pstride, nrecv, digits, top, R);
}

// Affine addends.  Every addition of the recombination chain adds one of the U stepped values
// Q_u(j); in affine Niels form (Z = 1) that addition is 7M instead of 8M (d = 2Z1 needs no product),
// ~250 additions per (column, receiver) at U = 4.  Normalising needs 1/Z of every stepped value:
// Montgomery's trick over AFF_RUN = 32 receivers per lane (one inversion, ~50 k slots, per 32
// points).  Half a wave takes one (piece, column) and 1024 consecutive receivers, lane r the
// receivers r, r + 32, .. so that every load instruction reads consecutive points.  Two levels keep
// the prefixes out of memory: blocks of 4 points; pass 1 multiplies the block products into a
// running product and parks the exclusive block prefix in the block's first output slot; after the
// inversion, pass 2 walks the blocks backwards, rebuilds the 4 in-block prefixes in registers and
// converts (x, y, 2dxy): ~7.75 M per point + 1/32 inversion.
constexpr int AFFP_WORDS = 32;  // slot of an affine addend: y+x, y-x, 2dxy, 2 pad (128 B)
constexpr int AFF_RUN = 32;     // points per lane
constexpr int AFF_BLK = 4;      // points per block

DKG_DEV void st_fe3(uint32_t* slot, const fe& a, const fe& b, const fe& c) {
  constexpr bool NT = DKG_AFF_NT != 0;
  st16<NT>(slot, a.v[0], a.v[1], a.v[2], a.v[3]);
  st16<NT>(slot + 4, a.v[4], a.v[5], a.v[6], a.v[7]);
  st16<NT>(slot + 8, a.v[8], a.v[9], b.v[0], b.v[1]);
  st16<NT>(slot + 12, b.v[2], b.v[3], b.v[4], b.v[5]);
  st16<NT>(slot + 16, b.v[6], b.v[7], b.v[8], b.v[9]);
  st16<NT>(slot + 20, c.v[0], c.v[1], c.v[2], c.v[3]);
  st16<NT>(slot + 24, c.v[4], c.v[5], c.v[6], c.v[7]);
  st16<NT>(slot + 28, c.v[8], c.v[9], 0u, 0u);
}

// f(K-1), f(K-2), .., f(0) with compile-time arguments
template <int K, typename F>
DKG_DEV void for_desc(F&& f) {
  if constexpr (K > 0) {
    f(std::integral_constant<int, K - 1>{});
    for_desc<K - 1>(f);
  }
}

DKG_DEV void ld_z(fe& z, const uint32_t* R, const uint32_t* Rz, size_t e) {  // Z of point e
  if (Rz) {  // the stepping's dense copy: 40 B per point, a half-wave reads 1280 contiguous bytes
    const uint2* z2 = reinterpret_cast<const uint2*>(Rz + e * 10);
    const uint2 a = z2[0], b = z2[1], c = z2[2], d = z2[3], f = z2[4];
    z = fe{{a.x, a.y, b.x, b.y, c.x, c.y, d.x, d.y, f.x, f.y}};
    return;
  }
  const uint4* p4 = reinterpret_cast<const uint4*>(R + e * PT_WORDS);  // words 20..29 of the point
  const uint4 z0 = p4[5], z1 = p4[6], z2 = p4[7];
  z = fe{{z0.x, z0.y, z0.z, z0.w, z1.x, z1.y, z1.z, z1.w, z2.x, z2.y}};
}

// Receivers [j0, j0 + jn) of rows nrecv long; ls (a power of two <= 32) lanes share a run of
// ls * AFF_RUN receivers, lane k taking receivers k, k + ls, .. of it.
__global__ __launch_bounds__(256) void k_affine_pieces(size_t width, size_t pstride, size_t pieces, size_t nrecv,
                                                       const uint32_t* __restrict__ R, uint32_t* __restrict__ A,
                                                       const uint32_t* __restrict__ Rz, size_t j0, size_t jn,
                                                       unsigned ls) {
  const size_t span = (size_t)ls * AFF_RUN, runs = (jn + span - 1) / span;
  const size_t gid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t item = gid / ls;
  if (item >= pieces * width * runs) return;
  const size_t c = item % width, rest = item / width, run = rest % runs, u = rest / runs;
  const size_t e0 = (u * pstride + c) * nrecv + j0;
  const size_t jb = run * span + (gid % ls);  // receivers j0 + jb + ls i, i < cnt
  const int cnt = jb < jn ? (int)min((size_t)AFF_RUN, (jn - jb + ls - 1) / ls) : 0;
  const int nblk = (cnt + AFF_BLK - 1) / AFF_BLK;
  auto pt = [&](int i) { return e0 + jb + ls * (size_t)i; };
  // points past cnt in the last block count as Z = 1
  fe acc;
  fe_one(acc);
#pragma unroll 1
  for (int b = 0; b < nblk; b++) {
    uint4* a4 = reinterpret_cast<uint4*>(A + pt(AFF_BLK * b) * AFFP_WORDS);
    a4[0] = make_uint4(acc.v[0], acc.v[1], acc.v[2], acc.v[3]);
    a4[1] = make_uint4(acc.v[4], acc.v[5], acc.v[6], acc.v[7]);
    a4[2] = make_uint4(acc.v[8], acc.v[9], 0u, 0u);
#pragma unroll 1
    for (int k = 0; k < AFF_BLK; k++) {
      const int i = AFF_BLK * b + k;
      if (i < cnt) {
        fe z;
        ld_z(z, R, Rz, pt(i));
        fe_mul(acc, acc, z);
      }
    }
  }
  fe inv;
  fe_invert(inv, acc);
  fe d2;
  fe_ld(d2, ge_const::D2);
#pragma unroll 1
  for (int b = nblk - 1; b >= 0; b--) {
    fe z[AFF_BLK], q[AFF_BLK];  // q[k] = z[0] .. z[k-1] (q[0] = 1 is never formed)
    static_assert(AFF_BLK >= 2, "q[1] = z[0] below");
#pragma unroll
    for (int k = 0; k < AFF_BLK; k++) {
      if (AFF_BLK * b + k < cnt) ld_z(z[k], R, Rz, pt(AFF_BLK * b + k));
      else fe_one(z[k]);
    }
    fe_copy(q[1], z[0]);
#pragma unroll
    for (int k = 2; k < AFF_BLK; k++) fe_mul(q[k], q[k - 1], z[k - 1]);
    fe blk, ib;
    fe_mul(blk, q[AFF_BLK - 1], z[AFF_BLK - 1]);  // the block's product
    {
      const uint4* a4 = reinterpret_cast<const uint4*>(A + pt(AFF_BLK * b) * AFFP_WORDS);
      const uint4 q0 = a4[0], q1 = a4[1], q2 = a4[2];
      const fe pre = {{q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w, q2.x, q2.y}};
      fe_mul(ib, inv, pre);   // 1 / (this block's product)
    }
    fe_mul(inv, inv, blk);    // 1 / (the earlier blocks' product)
    // the in-block points from the last down, each k a compile-time constant (q[k], z[k] in VGPRs)
    auto point = [&](auto kc) {
      constexpr int k = decltype(kc)::value;
      const int i = AFF_BLK * b + k;
      fe zi;
      if constexpr (k > 0) {
        fe_mul(zi, ib, q[k]);   // 1 / Z_i
        fe_mul(ib, ib, z[k]);
      } else {
        fe_copy(zi, ib);
      }
      if (i < cnt) {
        ge_p3 p;
        pt_load_aos(p, R, pt(i));
        fe x, y;
        fe_mul(x, p.X, zi);
        fe_mul(y, p.Y, zi);
        fe_mul(p.T, p.T, zi);   // xy
        fe_mul(p.T, p.T, d2);   // 2dxy
        fe_add(p.X, y, x);      // y + x <= 2^27
        fe_sub(p.Y, y, x);      // y - x <= 2^27.585
        st_fe3(A + pt(i) * AFFP_WORDS, p.X, p.Y, p.T);
      }
    };
    for_desc<AFF_BLK>(point);
  }
}

void affine_pieces(size_t width, size_t pstride, size_t pieces, size_t nrecv, const uint32_t* R, uint32_t* A,
                   hipStream_t stream, const uint32_t* Rz, size_t j0, size_t jn) {
  if (!jn) jn = nrecv - j0;
  if (!width || !jn || !pieces) return;
  // lanes per run: 32, or fewer for a short receiver part so that each lane still normalises up to
  // AFF_RUN points with its one inversion
  unsigned ls = 32;
  while (ls > 1 && (size_t)(ls / 2) * AFF_RUN >= jn) ls /= 2;
  const size_t runs = (jn + (size_t)ls * AFF_RUN - 1) / ((size_t)ls * AFF_RUN), lanes = pieces * width * runs * ls;
  hipLaunchKernelGGL(k_affine_pieces, dim3((unsigned)((lanes + 255) / 256)), dim3(256), 0, stream, width, pstride,
                     pieces, nrecv, R, A, Rz, j0, jn, ls);
}

template <int U, int K, int KL>
DKG_DEV void aff_addends(uint32_t* qs, ge_aff* qr, const uint32_t* A, size_t pstride, size_t cc, size_t nrecv,
                         size_t j) {
  if constexpr (U < K) {
    const uint4* a4 = reinterpret_cast<const uint4*>(A + (((size_t)U * pstride + cc) * nrecv + j) * AFFP_WORDS);
    uint32_t w[AFFP_WORDS];
#pragma unroll
    for (int k = 0; k < AFFP_WORDS / 4; k++) {
      const uint4 v = a4[k];
      w[4 * k] = v.x;
      w[4 * k + 1] = v.y;
      w[4 * k + 2] = v.z;
      w[4 * k + 3] = v.w;
    }
    if constexpr (U < KL) {
      uint32_t* s = qs + U * AFF_WORDS * 64 + threadIdx.x;
#pragma unroll
      for (int k = 0; k < AFF_WORDS; k++) s[k * 64] = w[k];
    } else {
#pragma unroll
      for (int i = 0; i < 10; i++) {
        qr[U - KL].ypx.v[i] = w[i];
        qr[U - KL].ymx.v[i] = w[10 + i];
        qr[U - KL].xy2d.v[i] = w[20 + i];
      }
    }
    aff_addends<U + 1, K, KL>(qs, qr, A, pstride, cc, nrecv, j);
  }
}
template <int U, int K, int KL>
DKG_DEV void aff_position(ge_p3& acc, uint64_t w, const uint32_t* qs, const ge_aff* qr, bool last) {
  if constexpr (U < K) {
    const int e = (int8_t)(w >> (8 * U));
    if (e != 0) {
      const bool t = last || higher_digits64<U, K>(w);  // else a doubling follows: no T
      if constexpr (U < KL) ge_madd_lds<DKG_AFF_IL != 0>(acc, acc, qs + U * AFF_WORDS * 64 + threadIdx.x, e < 0, 64, t);
      else ge_madd_signed<DKG_AFF_IL != 0>(acc, acc, qr[U - KL], e < 0, t);
    }
    aff_position<U + 1, K, KL>(acc, w, qs, qr, last);
  }
}

template <int K, int KL>
__global__ __launch_bounds__(64, K == 2 ? 3 : 2) void k_combine_aff(size_t width, size_t pstride, size_t nrecv,
                                                      const uint32_t* __restrict__ digits,
                                                      const int16_t* __restrict__ top,
                                                      const uint32_t* __restrict__ A, uint32_t* __restrict__ R,
                                                      size_t j0) {
  __shared__ uint32_t qs[KL * AFF_WORDS * 64];
  const size_t c = (size_t)blockIdx.x * 64 + threadIdx.x;
  const size_t j = j0 + blockIdx.y;
  const bool live = c < width;
  const size_t cc = live ? c : 0;
  ge_aff qr[K - KL > 0 ? K - KL : 1];
  aff_addends<0, K, KL>(qs, qr, A, pstride, cc, nrecv, j);
  // digit words: pieces 0..3 in word 0 (digits[j][b]), pieces 4.. in word 1 (digits + nrecv * 256)
  const uint32_t* dw = digits + j * 256;
  const uint32_t* dw1 = digits + (nrecv + j) * 256;
  const int tp = top[j];
  ge_p3 acc;
  ge_identity(acc);
#pragma unroll 1
  for (int b = tp; b >= 0; b--) {
    // readfirstlane returns a signed int: zero-extend, or a negative piece-3 digit would sign-fill
    // the bytes of pieces 4..7
    uint64_t w = (uint32_t)__builtin_amdgcn_readfirstlane(dw[b]);
    if constexpr (K > 4) w |= (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane(dw1[b]) << 32;
    if (b != tp) ge_dbl_lean<DKG_AFF_IL != 0>(acc, acc, w != 0 || b == 0);
    aff_position<0, K, KL>(acc, w, qs, qr, b == 0);
  }
  if (live) pt_store_aos<DKG_COMB_NT != 0>(R, c * nrecv + j, acc);
}

void combine_short_aff(size_t width, size_t pstride, size_t pieces, size_t nrecv, const uint32_t* digits,
                       const int16_t* top, const uint32_t* A, uint32_t* R, hipStream_t stream, size_t j0, size_t jn) {
  if (!jn) jn = nrecv - j0;
  if (!width || !jn || pieces < 2 || pieces > 5) return;
  const dim3 grid((unsigned)((width + 63) / 64), (unsigned)jn);
  if (pieces == 2)
    hipLaunchKernelGGL((k_combine_aff<2, 1>), grid, dim3(64), 0, stream, width, pstride, nrecv, digits, top, A, R, j0);
  else if (pieces == 3)
    hipLaunchKernelGGL((k_combine_aff<3, 2>), grid, dim3(64), 0, stream, width, pstride, nrecv, digits, top, A, R, j0);
  else if (pieces == 4)
    hipLaunchKernelGGL((k_combine_aff<4, 2>), grid, dim3(64), 0, stream, width, pstride, nrecv, digits, top, A, R, j0);
  else
    hipLaunchKernelGGL((k_combine_aff<5, 2>), grid, dim3(64), 0, stream, width, pstride, nrecv, digits, top, A, R, j0);
}

void combine(size_t width, size_t pstride, size_t pieces, size_t nrecv, const int8_t* digits, const int16_t* top,
             uint32_t* R, hipStream_t stream) {
  if (!width || !nrecv || pieces < 2) return;
  const dim3 grid((unsigned)((width + 63) / 64), (unsigned)nrecv);
  if (pieces == 2)  // one product, one LDS slot (10 KB per wave: occupancy bound by VGPRs only)
    hipLaunchKernelGGL(k_combine<1>, grid, dim3(64), 0, stream, width, pstride, (int)pieces, nrecv, digits, top, R);
  else
    hipLaunchKernelGGL(k_combine<2>, grid, dim3(64), 0, stream, width, pstride, (int)pieces, nrecv, digits, top, R);
}

// ------------------------------------------------------------------ K3c check
__global__ __launch_bounds__(256, DKG_COMB_WAVES) void k_check(size_t ndealers, size_t nrecv, size_t dealer_base, size_t recv_base,
                                               uint32_t nmod, int round,
                                               const uint32_t* __restrict__ s, const uint32_t* __restrict__ sp,
                                               const uint32_t* __restrict__ R,
                                               const uint32_t* __restrict__ tab_g,
                                               const uint32_t* __restrict__ tab_h,
                                               const uint8_t* __restrict__ dok, uint8_t* __restrict__ dec,
                                               const uint32_t* __restrict__ scale) {
  const size_t p = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= ndealers * nrecv) return;
  const size_t i = p / nrecv, j = p % nrecv;
  ge_p3 acc, r;
  ge_identity(acc);
  sc x, f;
  if (scale) sc_load(f, scale + 8 * j);            // R holds b_j P(j): compare with g*(b_j s) + h*(b_j s')
  sc_load(x, s + 8 * p);
  if (scale) sc_mont_mul(x, x, f);
  combw_mul_add(acc, x, tab_g);                    // G::generator() * s       (committee.rs:294, :537)
  if (round == 2) {
    sc_load(x, sp + 8 * p);
    if (scale) sc_mont_mul(x, x, f);
    combw_mul_add(acc, x, tab_h);                  // + h * s'                 (committee.rs:292-293)
  }
  pt_load_aos(r, R, p);
  const bool eq = ristretto_eq(acc, r);            // check_element != multi_scalar (:305, :541)
  // a dealer whose broadcast does not decode is missing data: disqualified without a complaint in
  // round 2 (committee.rs:331-335), an accusation in round 4 (:549-555)
  uint8_t v = dok[i] ? (eq ? 1 : 0) : (round == 2 ? 4 : 0);
  if ((uint32_t)((i + dealer_base) % nmod) == (uint32_t)(j + recv_base)) v = 2;  // self (batched: per ceremony)
  dec[p] = v;
}

void check(size_t ndealers, size_t nrecv, size_t dealer_base, size_t recv_base, size_t nmod, int round,
           const uint32_t* s, const uint32_t* sp, const uint32_t* R, const uint32_t* tab_g,
           const uint32_t* tab_h, const uint8_t* dok, uint8_t* dec, hipStream_t stream, const uint32_t* scale) {
  const size_t total = ndealers * nrecv;
  if (!total) return;
  hipLaunchKernelGGL(k_check, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, stream, ndealers, nrecv,
                     dealer_base, recv_base, (uint32_t)nmod, round, s, sp, R, tab_g, tab_h, dok, dec, scale);
}

// Fused round-2 + round-4 check of dealers [dealer0, dealer0 + ndealers) (local indices) whose E and A
// difference tables sit in interleaved columns: dealer i's E row is column (i / 64) * 128 + i % 64
// and its A row the column 64 after it.  g*s_ij is computed ONCE: compared with R_A (round 4,
// committee.rs:537-541), then h*s'_ij is added and the sum compared with R_E (round 2,
// committee.rs:292-305) -- the same group elements the two rounds compute separately.
// PASS 0: both in one launch (the default).  PASS 1 / 2: the same work as two launches that each
// read ONE comb: pass 1 computes g*s, decides round 4 and parks g*s in acc[p] (160 B), pass 2 adds
// h*s' to it and decides round 2 -- a split made for the radix-2^11 combs (3.1 MB per base, one
// XCD's 4-MB L2); the radix-2^19 combs are 470 MB per base (HBM / Infinity Cache) either way.
template <int PASS>
__global__ __launch_bounds__(256, DKG_COMB_WAVES) void k_check_both(size_t ndealers, size_t nrecv, size_t dealer0, size_t dealer_base,
                                                    uint32_t nmod, const uint32_t* __restrict__ s,
                                                    const uint32_t* __restrict__ sp, const uint32_t* __restrict__ R,
                                                    const uint32_t* __restrict__ tab_g,
                                                    const uint32_t* __restrict__ tab_h,
                                                    const uint8_t* __restrict__ dok, uint8_t* __restrict__ dec2,
                                                    uint8_t* __restrict__ dec4, const uint32_t* __restrict__ scale,
                                                    size_t j0, size_t jn, uint32_t* __restrict__ accb) {
  const size_t p = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= ndealers * jn) return;
  const size_t i = dealer0 + p / jn, j = j0 + p % jn;
  const size_t cE = (i / 64) * 128 + i % 64, cA = cE + 64;
  const size_t q = i * nrecv + j;  // share / decision index
  const bool self = (uint32_t)((i + dealer_base) % nmod) == (uint32_t)j;
  ge_p3 acc, r;
  sc x, f;
  if (scale) sc_load(f, scale + 8 * j);            // R holds b_j P(j): compare with g*(b_j s) + h*(b_j s')
  if constexpr (PASS != 2) {
    ge_identity(acc);
    sc_load(x, s + 8 * q);
    if (scale) sc_mont_mul(x, x, f);
    combw_mul_add<DKG_CHECK_IL != 0>(acc, x, tab_g);  // G::generator() * s   (committee.rs:294, :537)
    pt_load_aos(r, R, cA * nrecv + j);
    const bool eq = ristretto_eq(acc, r);          // round 4 (:541)
    dec4[q] = self ? 2 : ((dok[cA] && eq) ? 1 : 0);  // missing A: accusation (committee.rs:549-555)
    if constexpr (PASS == 1) {
      pt_store_aos(accb, p, acc);
      return;
    }
  } else {
    pt_load_aos(acc, accb, p);
  }
  sc_load(x, sp + 8 * q);
  if (scale) sc_mont_mul(x, x, f);
  combw_mul_add<DKG_CHECK_IL != 0>(acc, x, tab_h);  // + h * s'              (committee.rs:292-293)
  pt_load_aos(r, R, cE * nrecv + j);
  const bool eq = ristretto_eq(acc, r);            // round 2 (:305)
  dec2[q] = self ? 2 : (dok[cE] ? (eq ? 1 : 0) : 4);  // missing E: disqualified, no complaint (:331-335)
}

void check_both(size_t ndealers, size_t nrecv, size_t dealer0, size_t dealer_base, size_t nmod, const uint32_t* s,
                const uint32_t* sp, const uint32_t* R, const uint32_t* tab_g, const uint32_t* tab_h,
                const uint8_t* dok, uint8_t* dec2, uint8_t* dec4, hipStream_t stream, const uint32_t* scale, size_t j0,
                size_t jn, uint32_t* acc) {
  if (!jn) jn = nrecv - j0;
  const size_t total = ndealers * jn;
  if (!total) return;
  const dim3 grid((unsigned)((total + 255) / 256));
  if (!acc) {
    hipLaunchKernelGGL(k_check_both<0>, grid, dim3(256), 0, stream, ndealers, nrecv, dealer0, dealer_base,
                       (uint32_t)nmod, s, sp, R, tab_g, tab_h, dok, dec2, dec4, scale, j0, jn, acc);
    return;
  }
  hipLaunchKernelGGL(k_check_both<1>, grid, dim3(256), 0, stream, ndealers, nrecv, dealer0, dealer_base,
                     (uint32_t)nmod, s, sp, R, tab_g, tab_h, dok, dec2, dec4, scale, j0, jn, acc);
  hipLaunchKernelGGL(k_check_both<2>, grid, dim3(256), 0, stream, ndealers, nrecv, dealer0, dealer_base,
                     (uint32_t)nmod, s, sp, R, tab_g, tab_h, dok, dec2, dec4, scale, j0, jn, acc);
}

// Identity in every column of a position-major table [40][S] (S = N * npad words apart).
__global__ void k_fill_all_identity(size_t S, uint32_t* __restrict__ out) {
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= S) return;
  ge_p3 id;
  ge_identity(id);
  pt_store(out, S, e, id);
}

void fill_identity(size_t S, uint32_t* out, hipStream_t stream) {
  if (!S) return;
  hipLaunchKernelGGL(k_fill_all_identity, dim3((unsigned)((S + 255) / 256)), dim3(256), 0, stream, S, out);
}

__global__ void k_dealer_ok(size_t ndealers, size_t N, const uint8_t* __restrict__ pok, uint8_t* __restrict__ ok) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= ndealers) return;
  uint8_t v = 1;
  for (size_t k = 0; k < N; k++) v &= pok[i * N + k];
  ok[i] = v;
}

// dok[column of dealer i in segment seg] &= extra[i] (interleaved column layout of verify_device)
__global__ void k_and_dealer_mask(size_t D, uint32_t nseg, uint32_t seg, const uint8_t* __restrict__ extra,
                                  uint8_t* __restrict__ dok) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= D) return;
  const size_t col = (i / 64) * 64 * nseg + seg * 64 + i % 64;
  dok[col] &= extra[i];
}

void and_dealer_mask(size_t D, int nseg, int seg, const uint8_t* extra, uint8_t* dok, hipStream_t stream) {
  if (!D) return;
  hipLaunchKernelGGL(k_and_dealer_mask, dim3((unsigned)((D + 255) / 256)), dim3(256), 0, stream, D, (uint32_t)nseg,
                     (uint32_t)seg, extra, dok);
}

// out[i] = !a[i] && (b == NULL || b[i]): the qualified set from the rows that reject (b = NULL), the
// honest set from the qualified set and the round-4 rejections (a = rej4, b = qualified)
__global__ __launch_bounds__(256) void k_mask_not_and(size_t V, const uint8_t* __restrict__ a,
                                                      const uint8_t* __restrict__ b, uint8_t* __restrict__ out) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i < V) out[i] = !a[i] && (!b || b[i]);
}

void mask_not_and(size_t V, const uint8_t* a, const uint8_t* b, uint8_t* out, hipStream_t stream) {
  if (!V) return;
  hipLaunchKernelGGL(k_mask_not_and, dim3((unsigned)((V + 255) / 256)), dim3(256), 0, stream, V, a, b, out);
}

void dealer_ok(size_t ndealers, size_t N, const uint8_t* point_ok, uint8_t* ok, hipStream_t stream) {
  if (!ndealers) return;
  hipLaunchKernelGGL(k_dealer_ok, dim3((unsigned)((ndealers + 255) / 256)), dim3(256), 0, stream, ndealers, N,
                     point_ok, ok);
}

// Horner in the exponent for one receiver index x per blockIdx.y (x = x0 + blockIdx.y, uniform per
// wave): R[i][y] = sum_k x^k C_i[k] = C_0 + x (C_1 + x (...)), lanes = dealers.  This is the
// single-party view of committee.rs:287-296 (t small-scalar multiplications instead of an MSM).
__global__ __launch_bounds__(64, 3) void k_horner(size_t ndealers, size_t npad, size_t N, const uint32_t* __restrict__ C,
                                                uint32_t x0, size_t nrecv, uint32_t* __restrict__ R) {
  const size_t d = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t x = x0 + blockIdx.y;
  if (d >= npad) return;
  const size_t S = N * npad;
  ge_p3 acc, c;
  pt_load(acc, C, S, (N - 1) * npad + d);
  for (size_t k = N - 1; k-- > 0;) {
    mul_small_uniform(acc, acc, x);
    pt_load(c, C, S, k * npad + d);
    ge_cached cc;
    ge_to_cached(cc, c);
    ge_add(acc, acc, cc);
  }
  if (d < ndealers) pt_store_aos(R, d * nrecv + blockIdx.y, acc);
}

void horner(size_t ndealers, size_t npad, size_t N, const uint32_t* C, uint32_t x0, size_t nrecv, uint32_t* R,
            hipStream_t stream) {
  if (!ndealers || !nrecv) return;
  hipLaunchKernelGGL(k_horner, dim3((unsigned)(npad / 64), (unsigned)nrecv), dim3(64), 0, stream, ndealers, npad, N,
                     C, x0, nrecv, R);
}

// Sums of the masked points of an SoA vector, one workgroup (tree reduction) per group g:
// out column col + g = sum over e in [g*count, (g+1)*count) of mask[e] P_e.
__global__ __launch_bounds__(256) void k_sum_points(size_t count, const uint32_t* __restrict__ pts, size_t stride,
                                                    const uint8_t* __restrict__ mask, uint32_t* __restrict__ out,
                                                    size_t ostride, size_t col) {
  __shared__ uint32_t red[256][PT_WORDS];
  ge_p3 acc;
  ge_identity(acc);
  const size_t g = blockIdx.x;
  for (size_t e = g * count + threadIdx.x; e < (g + 1) * count; e += blockDim.x) {
    if (mask && !mask[e]) continue;
    ge_p3 p;
    pt_load(p, pts, stride, e);
    ge_cached pc;
    ge_to_cached(pc, p);
    ge_add(acc, acc, pc);
  }
  uint32_t* aw = reinterpret_cast<uint32_t*>(&acc);
  for (int w = 0; w < PT_WORDS; w++) red[threadIdx.x][w] = aw[w];
  __syncthreads();
  for (int h = 128; h > 0; h >>= 1) {
    if ((int)threadIdx.x < h) {
      ge_p3 x, y;
      uint32_t* xw = reinterpret_cast<uint32_t*>(&x);
      uint32_t* yw = reinterpret_cast<uint32_t*>(&y);
      for (int w = 0; w < PT_WORDS; w++) {
        xw[w] = red[threadIdx.x][w];
        yw[w] = red[threadIdx.x + h][w];
      }
      ge_cached yc;
      ge_to_cached(yc, y);
      ge_add(x, x, yc);
      for (int w = 0; w < PT_WORDS; w++) red[threadIdx.x][w] = xw[w];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0)
    for (int w = 0; w < PT_WORDS; w++) out[w * ostride + col + g] = red[0][w];
}

void sum_points(size_t count, const uint32_t* pts, size_t stride, const uint8_t* mask, uint32_t* out,
                size_t ostride, size_t col, hipStream_t stream, size_t groups) {
  if (!groups) return;
  hipLaunchKernelGGL(k_sum_points, dim3((unsigned)groups), dim3(256), 0, stream, count, pts, stride, mask, out,
                     ostride, col);
}

// out[e] = a[e] + b[e] (SoA points, same stride), e < count.
__global__ __launch_bounds__(256) void k_add_points(size_t count, const uint32_t* __restrict__ a,
                                                    const uint32_t* __restrict__ b, size_t stride,
                                                    uint32_t* __restrict__ out) {
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= count) return;
  ge_p3 x, y;
  pt_load(x, a, stride, e);
  pt_load(y, b, stride, e);
  ge_cached yc;
  ge_to_cached(yc, y);
  ge_add(x, x, yc);
  pt_store(out, stride, e, x);
}

void add_points(size_t count, const uint32_t* a, const uint32_t* b, size_t stride, uint32_t* out,
                hipStream_t stream) {
  if (!count) return;
  hipLaunchKernelGGL(k_add_points, dim3((unsigned)((count + 255) / 256)), dim3(256), 0, stream, count, a, b, stride,
                     out);
}

// RistrettoPoint::from_uniform_bytes of 64 hash bytes (hash_to_group, groups.rs:68-70) -> SoA point.
__global__ void k_from_uniform(const uint32_t* __restrict__ in16, uint32_t* __restrict__ out) {
  uint32_t a[8], b[8];
  for (int i = 0; i < 8; i++) {
    a[i] = in16[i];
    b[i] = in16[8 + i];
  }
  ge_p3 p, q;
  ristretto_elligator(p, a);
  ristretto_elligator(q, b);
  ge_cached qc;
  ge_to_cached(qc, q);
  ge_add(p, p, qc);
  pt_store(out, 1, 0, p);
}

void from_uniform(const uint32_t* in16, uint32_t* out, hipStream_t stream) {
  hipLaunchKernelGGL(k_from_uniform, dim3(1), dim3(1), 0, stream, in16, out);
}

// ------------------------------------------------------------------ generic MSM / fixed base
// PrimeGroupElement::vartime_multiscalar_multiplication (traits.rs:234-237) for B independent MSMs
// of N terms: Straus with 4-bit windows split over the workgroup.  k_msm_tables stores d*P_k,
// d = 1..15, of every term (cached form, 15 x 40 words); in k_msm thread q of an MSM keeps its own
// accumulator over the terms k = q, q + T, ...: per window 4 doublings and one table addition per
// term, then a tree reduction of the T partial sums.  T = min(256, N up to a power of two >= 64).
__global__ __launch_bounds__(256) void k_msm_tables(size_t count, const uint32_t* __restrict__ pts, size_t stride,
                                                  uint32_t* __restrict__ tab) {
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= count) return;
  ge_p3 p, acc;
  pt_load(p, pts, stride, e);
  ge_cached pc;
  ge_to_cached(pc, p);
  acc = p;
  uint4* out = reinterpret_cast<uint4*>(tab + e * 15 * PT_WORDS);
#pragma unroll 1
  for (int d = 1; d <= 15; d++) {
    if (d > 1) ge_add(acc, acc, pc);
    ge_cached c;
    ge_to_cached(c, acc);
    const uint4* c4 = reinterpret_cast<const uint4*>(&c);
#pragma unroll
    for (int w = 0; w < PT_WORDS / 4; w++) out[(d - 1) * (PT_WORDS / 4) + w] = c4[w];
  }
}

__global__ __launch_bounds__(256) void k_msm(size_t N, const uint32_t* __restrict__ scalars,
                                             const uint32_t* __restrict__ tab, uint32_t* __restrict__ out,
                                             size_t ostride) {
  __shared__ uint32_t red[256][PT_WORDS];
  const size_t b = blockIdx.x;
  const int T = blockDim.x, q = threadIdx.x;
  ge_p3 acc;
  ge_identity(acc);
  if ((size_t)q < N) {
#pragma unroll 1
    for (int w = 63; w >= 0; w--) {
      if (w != 63) {
#pragma unroll 1
        for (int i = 0; i < 4; i++) ge_dbl_lean(acc, acc, i == 3);
      }
#pragma unroll 1
      for (size_t k = q; k < N; k += T) {
        const uint32_t word = scalars[8 * (b * N + k) + (w >> 3)];
        const uint32_t nib = (word >> (4 * (w & 7))) & 15u;
        if (nib) {
          ge_cached c;
          const uint4* src = reinterpret_cast<const uint4*>(tab + ((b * N + k) * 15 + nib - 1) * PT_WORDS);
          uint4* c4 = reinterpret_cast<uint4*>(&c);
#pragma unroll
          for (int x = 0; x < PT_WORDS / 4; x++) c4[x] = src[x];
          ge_add(acc, acc, c);
        }
      }
    }
  }
  uint32_t* aw = reinterpret_cast<uint32_t*>(&acc);
  for (int w = 0; w < PT_WORDS; w++) red[q][w] = aw[w];
  __syncthreads();
  for (int h = T / 2; h > 0; h >>= 1) {
    if (q < h) {
      ge_p3 x, y;
      uint32_t* xw = reinterpret_cast<uint32_t*>(&x);
      uint32_t* yw = reinterpret_cast<uint32_t*>(&y);
      for (int w = 0; w < PT_WORDS; w++) {
        xw[w] = red[q][w];
        yw[w] = red[q + h][w];
      }
      ge_cached yc;
      ge_to_cached(yc, y);
      ge_add(x, x, yc);
      for (int w = 0; w < PT_WORDS; w++) red[q][w] = xw[w];
    }
    __syncthreads();
  }
  if (q == 0) {
    ge_p3 r;
    uint32_t* rw = reinterpret_cast<uint32_t*>(&r);
    for (int w = 0; w < PT_WORDS; w++) rw[w] = red[0][w];
    pt_store(out, ostride, b, r);
  }
}

// tab: scratch of B * N * 15 * 40 words
void msm_batch(size_t B, size_t N, const uint32_t* scalars, const uint32_t* pts, size_t stride, uint32_t* tab,
               uint32_t* out_ext, hipStream_t stream) {
  if (!B) return;
  const size_t count = B * N;
  if (count)
    hipLaunchKernelGGL(k_msm_tables, dim3((unsigned)((count + 255) / 256)), dim3(256), 0, stream, count, pts, stride,
                       tab);
  size_t T = 64;  // a power of two (tree reduction), 64..256
  while (T < N && T < 256) T <<= 1;
  hipLaunchKernelGGL(k_msm, dim3((unsigned)B), dim3((unsigned)T), 0, stream, N, scalars, tab, out_ext, B);
}

__global__ __launch_bounds__(256, 4) void k_fixed_base(size_t count, const uint32_t* __restrict__ scalars,
                                                    const uint32_t* __restrict__ tab, uint32_t* __restrict__ out) {
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= count) return;
  sc x;
  sc_load(x, scalars + 8 * e);
  ge_p3 acc;
  ge_identity(acc);
  combw_mul_add(acc, x, tab);
  pt_store(out, count, e, acc);
}

// tab: a radix-2^11 comb (build_combw)
void fixed_base(size_t count, const uint32_t* scalars, const uint32_t* tab, uint32_t* out_ext, hipStream_t stream) {
  if (!count) return;
  hipLaunchKernelGGL(k_fixed_base, dim3((unsigned)((count + 255) / 256)), dim3(256), 0, stream, count, scalars, tab,
                     out_ext);
}

// ------------------------------------------------------------------ layout / scalar helpers
__global__ void k_to_pos_major(size_t D, size_t N, size_t npad, const uint32_t* __restrict__ in,
                               uint32_t* __restrict__ out) {
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;  // e = k * npad + i
  if (e >= N * npad) return;
  const size_t k = e / npad, i = e % npad;
  const size_t S = N * npad, Sin = D * N;
  for (int w = 0; w < PT_WORDS; w++) {
    uint32_t v;
    if (i < D) v = in[w * Sin + i * N + k];
    else v = (w == 10 || w == 20) ? 1u : 0u;  // padded dealers hold the identity (0 : 1 : 1 : 0)
    out[w * S + e] = v;
  }
}

void to_position_major(size_t D, size_t N, size_t npad, const uint32_t* in, uint32_t* out, hipStream_t stream) {
  const size_t tot = N * npad;
  if (!tot) return;
  hipLaunchKernelGGL(k_to_pos_major, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, stream, D, N, npad, in, out);
}

__global__ void k_reduce_scalars(size_t count, const uint32_t* __restrict__ in, uint32_t* __restrict__ out) {
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= count) return;
  uint32_t w[8];
  ld_words8(w, in + 8 * e);
  sc r;
  sc_reduce256(r, w);
  st_words8(out + 8 * e, r.v);
}

void reduce_scalars(size_t count, const uint32_t* in, uint32_t* out, hipStream_t stream) {
  if (!count) return;
  hipLaunchKernelGGL(k_reduce_scalars, dim3((unsigned)((count + 255) / 256)), dim3(256), 0, stream, count, in, out);
}

// Group g (blockIdx.y) of D dealers: out[g][j] = sum over dealers i of group g with mask of s[g][i][j].
// 256-thread blocks of 64 receivers x 4 dealer slices when D is large (one ceremony: the dealer
// loop is the latency), one thread per receiver otherwise (batches: many groups already).
template <int SLICES>
__global__ __launch_bounds__(64 * SLICES) void k_sum_shares(size_t D, size_t n, const uint32_t* __restrict__ s,
                                                          const uint8_t* __restrict__ mask,
                                                          uint32_t* __restrict__ out) {
  __shared__ uint32_t part[SLICES > 1 ? SLICES * 8 * 64 : 1];
  const int lane = threadIdx.x & 63, slice = threadIdx.x >> 6;
  const size_t j = (size_t)blockIdx.x * 64 + lane;
  const size_t g = blockIdx.y;
  s += g * D * n * 8;
  mask += g * D;
  out += g * n * 8;
  sc acc, x;
  sc_zero(acc);
  if (j < n)
    for (size_t i = slice; i < D; i += SLICES) {
      if (!mask[i]) continue;
      sc_load(x, s + 8 * (i * n + j));
      sc_add(acc, acc, x);
    }
  if (SLICES > 1) {
#pragma unroll
    for (int w = 0; w < 8; w++) part[(slice * 8 + w) * 64 + lane] = acc.v[w];
    __syncthreads();
    if (slice != 0) return;
    for (int q = 1; q < SLICES; q++) {
#pragma unroll
      for (int w = 0; w < 8; w++) x.v[w] = part[(q * 8 + w) * 64 + lane];
      sc_add(acc, acc, x);
    }
  }
  if (j < n) st_words8(out + 8 * j, acc.v);
}

void sum_shares(size_t D, size_t n, const uint32_t* s, const uint8_t* mask, uint32_t* out, hipStream_t stream,
                size_t groups) {
  if (!n) return;
  for (size_t g0 = 0; g0 < groups; g0 += 65535) {  // grid.y limit
    const size_t gc = groups - g0 < 65535 ? groups - g0 : 65535;
    const dim3 grid((unsigned)((n + 63) / 64), (unsigned)gc);
    if (gc * ((n + 63) / 64) >= 1024)
      hipLaunchKernelGGL(k_sum_shares<1>, grid, dim3(64), 0, stream, D, n, s + g0 * D * n * 8, mask + g0 * D,
                         out + g0 * n * 8);
    else
      hipLaunchKernelGGL(k_sum_shares<16>, grid, dim3(1024), 0, stream, D, n, s + g0 * D * n * 8, mask + g0 * D,
                         out + g0 * n * 8);
  }
}

// Row / column summaries of a decision matrix [rows][n] (rows = groups x n dealers of batched
// ceremonies): row_reject[i] = some receiver rejected dealer i or its data is missing (it is not
// qualified); complaints[g][j] = number of dealers of group g rejected (REJECT only, MISSING is no
// complaint) by receiver j (committee.rs:311-316, 331-335, 340-347).
// One wave per row: the lanes read the row's bytes coalesced, a ballot reduces.
__global__ __launch_bounds__(256) void k_row_reject(size_t rows, size_t n, const uint8_t* __restrict__ dec,
                                                    uint8_t* __restrict__ out) {
  const size_t i = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= rows) return;  // wave-uniform
  bool r = false;
  for (size_t j = threadIdx.x & 63; j < n; j += 64) r |= dec[i * n + j] == 0 || dec[i * n + j] == 4;  // REJECT / MISSING
  const bool any = __ballot(r) != 0;
  if ((threadIdx.x & 63) == 0) out[i] = any;
}

// Column counts of a stacked decision matrix: 64 columns (lanes) x 16 row slices (waves) per
// workgroup, the slices summed through LDS -- one thread per column alone leaves a 1024-party
// ceremony with 16 waves walking 1024 rows each.
constexpr int COL_SLICES = 16;
template <typename Pred>
__device__ __forceinline__ int32_t column_count(size_t groups, size_t n, const uint8_t* __restrict__ dec, Pred pred,
                                                size_t& e_out) {
  __shared__ int32_t part[COL_SLICES][64];
  const int lane = threadIdx.x & 63, slice = threadIdx.x >> 6;
  const size_t e = (size_t)blockIdx.x * 64 + lane;  // e = g * n + j
  const bool live = e < groups * n;
  const size_t g = live ? e / n : 0, j = live ? e % n : 0;
  int32_t c = 0;
  if (live)
    for (size_t i = slice; i < n; i += COL_SLICES) c += pred(g * n + i, dec[(g * n + i) * n + j]);
  part[slice][lane] = c;
  __syncthreads();
  int32_t s = 0;
  if (slice == 0)
    for (int k = 0; k < COL_SLICES; k++) s += part[k][lane];
  e_out = live && slice == 0 ? e : SIZE_MAX;
  return s;
}

__global__ __launch_bounds__(64 * COL_SLICES) void k_col_complaints(size_t groups, size_t n,
                                                                   const uint8_t* __restrict__ dec,
                                                                   int32_t* __restrict__ out) {
  size_t e;
  const int32_t c = column_count(groups, n, dec, [](size_t, uint8_t d) { return (int32_t)(d == 0); }, e);  // REJECT
  if (e != SIZE_MAX) out[e] = c;
}

// Round-4 error of receiver j (committee.rs:515-516, 567-569): itself plus the qualified dealers
// whose check it accepted are fewer than t+1.
__global__ __launch_bounds__(64 * COL_SLICES) void k_r4_error(size_t groups, size_t n, size_t t,
                                                             const uint8_t* __restrict__ dec,
                                                             const uint8_t* __restrict__ qmask,
                                                             uint8_t* __restrict__ out) {
  size_t e;
  const int32_t c = column_count(
      groups, n, dec, [qmask](size_t row, uint8_t d) { return (int32_t)(qmask[row] && d == 1); }, e);  // ACCEPT
  if (e != SIZE_MAX) out[e] = (size_t)(1 + c) < t + 1;
}

void r4_error(size_t groups, size_t n, size_t t, const uint8_t* dec, const uint8_t* qmask, uint8_t* out,
              hipStream_t stream) {
  const size_t rows = groups * n;
  if (!rows) return;
  hipLaunchKernelGGL(k_r4_error, dim3((unsigned)((rows + 63) / 64)), dim3(64 * COL_SLICES), 0, stream, groups, n, t,
                     dec, qmask, out);
}

// Round 4 skips the dealers round 2 disqualified (committee.rs:522): row i of a group whose
// dealer is not qualified becomes SKIPPED except its SELF diagonal.  One wave per row.
__global__ __launch_bounds__(256) void k_apply_skipped(size_t rows, size_t n, uint8_t* __restrict__ dec,
                                                       const uint8_t* __restrict__ qmask) {
  const size_t i = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= rows || qmask[i]) return;  // wave-uniform
  const size_t self = i % n;
  for (size_t j = threadIdx.x & 63; j < n; j += 64)
    if (j != self) dec[i * n + j] = 3;  // DKG_SKIPPED
}

void apply_skipped(size_t groups, size_t n, uint8_t* dec, const uint8_t* qmask, hipStream_t stream) {
  const size_t rows = groups * n;
  if (!rows) return;
  hipLaunchKernelGGL(k_apply_skipped, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, stream, rows, n, dec, qmask);
}

// Compaction of all-gathered per-rank blocks: rank r's block sits at in + r * R * width and holds
// d1(r) - d0(r) valid rows of `width` bytes (dealer partition [r * n / ws, (r + 1) * n / ws));
// out is the dense [n][width] matrix.  One thread per element of T (16, 4 or 1 bytes).
template <typename T>
__global__ __launch_bounds__(256) void k_compact_ranks(size_t n, size_t ws, size_t R, size_t q,
                                                       const T* __restrict__ in, T* __restrict__ out) {
  const size_t e = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= n * q) return;
  const size_t i = e / q, w = e % q;
  size_t r = (i * ws) / n;  // the rank owning row i: the largest r with r * n / ws <= i
  while (r + 1 < ws && ((r + 1) * n) / ws <= i) r++;
  while (r > 0 && (r * n) / ws > i) r--;
  out[e] = in[(r * R + (i - (r * n) / ws)) * q + w];
}

void compact_ranks(size_t n, size_t ws, size_t R, size_t width, const void* in, void* out, hipStream_t stream) {
  if (!n || !width) return;
  const uintptr_t al = (uintptr_t)in | (uintptr_t)out | width;
  if (al % 16 == 0) {
    const size_t q = width / 16, total = n * q;
    hipLaunchKernelGGL(k_compact_ranks<uint4>, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, stream, n, ws, R,
                       q, (const uint4*)in, (uint4*)out);
  } else if (al % 4 == 0) {
    const size_t q = width / 4, total = n * q;
    hipLaunchKernelGGL(k_compact_ranks<uint32_t>, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, stream, n, ws,
                       R, q, (const uint32_t*)in, (uint32_t*)out);
  } else {
    const size_t total = n * width;
    hipLaunchKernelGGL(k_compact_ranks<uint8_t>, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, stream, n, ws,
                       R, width, (const uint8_t*)in, (uint8_t*)out);
  }
}

// Packed decision rows: what the ranks of a sharded ceremony all-gather instead of n bytes per row
// (north_star: the complaint / verification bitmaps).  A rank's raw rows hold
// REJECT / ACCEPT (round 4 as well: SKIPPED is applied after the exchange), SELF on the global
// diagonal and, in round 2, whole rows of MISSING (an undecodable broadcast), so row r becomes
// W = ceil(n / 32) words of ACCEPT bits plus one kind word (0 checked, 1 MISSING row, 2 SKIPPED
// row); the diagonal is implied by the dealer index.  Rows past nvalid (the padding of a rank block)
// are zero.  A row the encoding cannot hold sets err[0] (vector store: lanes are divergent).
__global__ __launch_bounds__(64) void k_pack_rows(size_t nvalid, size_t n, size_t d0, const uint8_t* __restrict__ dec,
                                                  uint32_t* __restrict__ out, uint32_t* __restrict__ err) {
  const size_t r = blockIdx.y, W = (n + 31) / 32, w = (size_t)blockIdx.x * 64 + threadIdx.x;
  if (w > W) return;
  uint32_t* o = out + r * (W + 1);
  if (r >= nvalid) {
    o[w] = 0;
    return;
  }
  const uint8_t* row = dec + r * n;
  const size_t self = d0 + r;
  const uint8_t ref = n > 1 ? row[self == 0 ? 1 : 0] : 1;  // any entry off the diagonal
  const uint32_t kind = ref == 4 ? 1u : ref == 3 ? 2u : 0u;
  if (w == W) {
    o[w] = kind;
    return;
  }
  uint32_t bits = 0, bad = 0;
  for (int b = 0; b < 32; b++) {
    const size_t j = w * 32 + b;
    if (j >= n) break;
    const uint32_t v = row[j];
    if (j == self) bad |= v != 2;
    else if (kind == 0) {
      bad |= v > 1;
      bits |= (v & 1u) << b;
    } else {
      bad |= v != (kind == 1 ? 4u : 3u);
    }
  }
  o[w] = bits;
  if (bad) err[0] = 1u;
}

void pack_rows(size_t rows, size_t nvalid, size_t n, size_t d0, const uint8_t* dec, uint32_t* out, uint32_t* err,
               hipStream_t stream) {
  if (!rows || !n) return;
  const size_t W1 = (n + 31) / 32 + 1;
  hipLaunchKernelGGL(k_pack_rows, dim3((unsigned)((W1 + 63) / 64), (unsigned)rows), dim3(64), 0, stream, nvalid, n,
                     d0, dec, out, err);
}

// All-gathered packed blocks [ws][R][W + 1] -> the dense decision matrix [n][n]: one thread per
// (global row i, word w), 32 entries each (eight 4-byte stores when rows are 4-byte aligned).
__global__ __launch_bounds__(256) void k_unpack_ranks(size_t n, size_t ws, size_t R, const uint32_t* __restrict__ in,
                                                      uint8_t* __restrict__ out) {
  const size_t W = (n + 31) / 32, e = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= n * W) return;
  const size_t i = e / W, w = e % W;
  size_t r = (i * ws) / n;  // the rank owning row i (as k_compact_ranks)
  while (r + 1 < ws && ((r + 1) * n) / ws <= i) r++;
  while (r > 0 && (r * n) / ws > i) r--;
  const uint32_t* src = in + (r * R + (i - (r * n) / ws)) * (W + 1);
  const uint32_t kind = src[W], bits = src[w];
  const uint32_t fill = kind == 1 ? 4u : kind == 2 ? 3u : 0u;
  uint8_t* o = out + i * n;
  const size_t j0 = w * 32;
  auto val = [&](size_t j, int b) -> uint32_t { return j == i ? 2u : kind ? fill : (bits >> b) & 1u; };
  if (n % 4 == 0 && j0 + 32 <= n) {
    uint32_t* o4 = reinterpret_cast<uint32_t*>(o + j0);
#pragma unroll
    for (int q = 0; q < 8; q++) {
      uint32_t v = 0;
#pragma unroll
      for (int b = 0; b < 4; b++) v |= val(j0 + 4 * q + b, 4 * q + b) << (8 * b);
      o4[q] = v;
    }
  } else {
    for (int b = 0; b < 32 && j0 + b < n; b++) o[j0 + b] = (uint8_t)val(j0 + b, b);
  }
}

void unpack_ranks(size_t n, size_t ws, size_t R, const uint32_t* in, uint8_t* out, hipStream_t stream) {
  const size_t total = n * ((n + 31) / 32);
  if (!total) return;
  hipLaunchKernelGGL(k_unpack_ranks, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, stream, n, ws, R, in, out);
}

void row_reject(size_t rows, size_t n, const uint8_t* dec, uint8_t* out, hipStream_t stream) {
  if (!rows) return;
  hipLaunchKernelGGL(k_row_reject, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, stream, rows, n, dec, out);
}

void decision_summary(size_t groups, size_t n, const uint8_t* dec, uint8_t* row_reject, int32_t* complaints,
                      hipStream_t stream) {
  const size_t rows = groups * n;
  if (!rows) return;
  if (row_reject)
    hipLaunchKernelGGL(k_row_reject, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, stream, rows, n, dec,
                       row_reject);
  if (complaints)
    hipLaunchKernelGGL(k_col_complaints, dim3((unsigned)((rows + 63) / 64)), dim3(64 * COL_SLICES), 0, stream, groups,
                       n, dec, complaints);
}

}  // namespace dkgk
