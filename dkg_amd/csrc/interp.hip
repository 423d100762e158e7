// Committee verification by interpolation (opt-in: dkg_ctx_set_verify_mode).
//
// When one verifier holds ALL n shares of a dealer (the all-parties ceremony drivers), the t+1
// shares at receivers 1..t+1 determine the dealer's scalar polynomials exactly: F, F' with
// F(j) = s_j, F'(j) = s'_j (j = 1..t+1) have monomial coefficients F = W s, W = V^-1 the inverse
// Vandermonde matrix of the points 1..t+1 (mod l).  Then, for the round-2 row of dealer i:
//   case A: E_k == g F_k + h F'_k for every k.  The committed polynomial IS g F + h F', so the
//           reference's check at receiver j, g s_j + h s'_j == sum_k j^k E_k, is
//           g (s_j - F(j)) + h (s'_j - F'(j)) == 0: true when the scalars agree, else decided by
//           computing that group element (one double-comb product, only for deviating shares).
//   case B: some E_k differs: then some receiver in 1..t+1 rejects (the values at t+1 distinct
//           points determine a degree-t polynomial), and the row is verified the general way
//           (difference tables, verify_device) -- exact either way.
// Round 4 (A_k == g F_k, g s_j == sum_k j^k A_k) is the same with h = 0; in case A its decision is
// the scalar comparison s_j == F(j) exactly (g has prime order l).  Every decision equals the
// reference's per-pair check; no randomness, no assumption on the inputs.
#include "kernels.h"
#include "points.h"

namespace dkgk {

DKG_DEV void sc_sub(sc& r, const sc& a, const sc& b) {  // a - b mod l, a, b < l
  uint32_t w[9];
  int64_t acc = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    acc += (int64_t)a.v[i] - b.v[i];
    w[i] = (uint32_t)acc;
    acc >>= 32;
  }
  sc t;
#pragma unroll
  for (int i = 0; i < 8; i++) t.v[i] = w[i];
  sc_add_l_if(t, acc < 0);
  r = t;
}

DKG_DEV bool sc_eq(const sc& a, const sc& b) {
  uint32_t d = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) d |= a.v[i] ^ b.v[i];
  return d == 0;
}

// F[d][k] = sum_j W[k][j] s[d][j] (and F' from s'), j, k < N, as an exact integer dot product with
// one reduction at the end: W[k][j] * 2^256 mod l is stored in 11 limbs of 24 bits (W24[j][a][k],
// coalesced over k = lanes), the dealer's shares (wave-uniform) are split the same way, and the
// 21 radix-2^24 columns accumulate in 64 bits (<= 11 * N * 2^48 < 2^64 for N <= 2^13): 121
// v_mad_u64_u32 per term, no carries.  The sum (< N l^2) is then Montgomery-reduced (REDC by 2^256
// cancels W's factor) and folded to canonical form.
constexpr int L24 = 11;

DKG_DEV void to_limbs24(uint32_t (&o)[L24], const uint32_t* w) {
  uint32_t v[8];
  ld_words8(v, w);
#pragma unroll
  for (int a = 0; a < L24; a++) {
    const int bit = 24 * a, wi = bit >> 5, sh = bit & 31;
    uint64_t x = (uint64_t)(wi < 8 ? v[wi] : 0u) | ((uint64_t)(wi + 1 < 8 ? v[wi + 1] : 0u) << 32);
    o[a] = (uint32_t)(x >> sh) & 0xffffffu;
  }
}

// acc (21 columns of radix 2^24, 64-bit) -> canonical scalar: repack into 17 words, REDC, fold
DKG_DEV void limbs24_redc(sc& r, const uint64_t (&col)[2 * L24 - 1]) {
  uint32_t t[18];
#pragma unroll
  for (int i = 0; i < 18; i++) t[i] = 0;
  uint64_t carry = 0;
#pragma unroll
  for (int c = 0; c < 2 * L24; c++) {  // value = sum_c col[c] 2^(24c); emit 24 bits per column
    const uint64_t v = (c < 2 * L24 - 1 ? col[c] : 0ull) + carry;
    const uint32_t limb = (uint32_t)v & 0xffffffu;
    carry = v >> 24;
    const int bit = 24 * c, wi = bit >> 5, sh = bit & 31;
    t[wi] |= limb << sh;
    if (sh > 8) t[wi + 1] |= limb >> (32 - sh);
  }
  // REDC: t <- (t + m l) / 2^256, 8 word steps (t < 2^515 -> result < 2^260)
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint32_t m = t[i] * sc_const::LINV;
    uint64_t c = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) {
      c += (uint64_t)m * sc_const::L[j] + t[i + j];
      t[i + j] = (uint32_t)c;
      c >>= 32;
    }
#pragma unroll
    for (int j = i + 8; j < 18; j++) {
      c += t[j];
      t[j] = (uint32_t)c;
      c >>= 32;
    }
  }
  uint32_t w9[9];
#pragma unroll
  for (int i = 0; i < 9; i++) w9[i] = t[8 + i];
  sc_reduce9(r, w9);
}

__global__ __launch_bounds__(64) void k_interp(size_t N, size_t nrecv, const uint32_t* __restrict__ W24,
                                               const uint32_t* __restrict__ s, const uint32_t* __restrict__ sp,
                                               uint32_t* __restrict__ F, uint32_t* __restrict__ Fp) {
  const size_t k = (size_t)blockIdx.x * 64 + threadIdx.x, d = blockIdx.y;
  const bool live = k < N;
  const size_t kk = live ? k : 0;
  uint64_t acc[2 * L24 - 1], accp[2 * L24 - 1];
#pragma unroll
  for (int c = 0; c < 2 * L24 - 1; c++) acc[c] = accp[c] = 0;
  const uint32_t* sd = s + 8 * d * nrecv;
  const uint32_t* spd = sp ? sp + 8 * d * nrecv : sd;
#pragma unroll 1
  for (size_t j = 0; j < N; j++) {
    uint32_t w[L24], x[L24], y[L24];
#pragma unroll
    for (int a = 0; a < L24; a++) w[a] = W24[(j * L24 + a) * N + kk];
    to_limbs24(x, sd + 8 * j);
    to_limbs24(y, spd + 8 * j);
#pragma unroll
    for (int a = 0; a < L24; a++)
#pragma unroll
      for (int b = 0; b < L24; b++) {
        acc[a + b] += (uint64_t)w[a] * x[b];
        accp[a + b] += (uint64_t)w[a] * y[b];
      }
  }
  if (!live) return;
  sc r;
  limbs24_redc(r, acc);
  st_words8(F + 8 * (d * N + k), r.v);
  if (Fp) {
    limbs24_redc(r, accp);
    st_words8(Fp + 8 * (d * N + k), r.v);
  }
}

void interp(size_t D, size_t N, size_t nrecv, const uint32_t* W24, const uint32_t* s, const uint32_t* sp, uint32_t* F,
            uint32_t* Fp, hipStream_t stream) {
  if (!D || !N) return;
  hipLaunchKernelGGL(k_interp, dim3((unsigned)((N + 63) / 64), (unsigned)D), dim3(64), 0, stream, N, nrecv, W24, s,
                     sp, F, Fp);
}

// Coefficient test of (dealer d, k): okA = (g F_k == A_k), okE = (g F_k + h F'_k == E_k).
// Commitments: extended points [D][N] (index d * N + k, word stride cstride).
__global__ __launch_bounds__(256, 4) void k_coef_check(size_t count, const uint32_t* __restrict__ F,
                                                       const uint32_t* __restrict__ Fp,
                                                       const uint32_t* __restrict__ Eext,
                                                       const uint32_t* __restrict__ Aext, size_t cstride,
                                                       const uint32_t* __restrict__ tab_g,
                                                       const uint32_t* __restrict__ tab_h, uint8_t* __restrict__ okE,
                                                       uint8_t* __restrict__ okA) {
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= count) return;
  sc x;
  ge_p3 acc, c;
  ge_identity(acc);
  sc_load(x, F + 8 * e);
  combw_mul_add(acc, x, tab_g);
  pt_load(c, Aext, cstride, e);
  okA[e] = ristretto_eq(acc, c) ? 1 : 0;
  sc_load(x, Fp + 8 * e);
  combw_mul_add(acc, x, tab_h);
  pt_load(c, Eext, cstride, e);
  okE[e] = ristretto_eq(acc, c) ? 1 : 0;
}

void coef_check(size_t D, size_t N, const uint32_t* F, const uint32_t* Fp, const uint32_t* Eext, const uint32_t* Aext,
                size_t cstride, const uint32_t* tab_g, const uint32_t* tab_h, uint8_t* okE, uint8_t* okA,
                hipStream_t stream) {
  const size_t count = D * N;
  if (!count) return;
  hipLaunchKernelGGL(k_coef_check, dim3((unsigned)((count + 255) / 256)), dim3(256), 0, stream, count, F, Fp, Eext,
                     Aext, cstride, tab_g, tab_h, okE, okA);
}

// Decisions of the rows in case A (cE / cA: the dealer's coefficient test passed; rows in case B
// are written 0 here and re-verified by the caller).  Lanes = receivers j of dealer d.
__global__ __launch_bounds__(256, 4) void k_interp_decide(size_t D, size_t nrecv, size_t N, size_t dealer_base,
                                                          uint32_t nmod, const uint32_t* __restrict__ s,
                                                          const uint32_t* __restrict__ sp,
                                                          const uint32_t* __restrict__ F,
                                                          const uint32_t* __restrict__ Fp,
                                                          const uint8_t* __restrict__ dokE,
                                                          const uint8_t* __restrict__ dokA,
                                                          const uint8_t* __restrict__ cE, const uint8_t* __restrict__ cA,
                                                          const uint32_t* __restrict__ tab_g,
                                                          const uint32_t* __restrict__ tab_h,
                                                          uint8_t* __restrict__ dec2, uint8_t* __restrict__ dec4) {
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= D * nrecv) return;
  const size_t d = e / nrecv, j = e % nrecv;
  if ((uint32_t)((d + dealer_base) % nmod) == (uint32_t)j) {
    dec2[e] = 2;
    dec4[e] = 2;
    return;
  }
  const bool rowE = dokE[d] && cE[d], rowA = dokA[d] && cA[d];
  bool eqF = true, eqFp = true;
  sc fx, fpx, sj, spj;
  if (j >= N && (rowE || rowA)) {  // receivers 1..t+1 agree with F, F' by construction
    const uint32_t x = (uint32_t)(j + 1);
    const uint32_t* Fd = F + 8 * d * N;
    const uint32_t* Fpd = Fp + 8 * d * N;
    sc c, c0;
    sc_load(fx, Fd + 8 * (N - 1));
    sc_load(fpx, Fpd + 8 * (N - 1));
    size_t k = N - 1;
    if (x < 2048) {  // Horner (Polynomial::evaluate's value, polynomial.rs:68-74), two steps per reduction
#pragma unroll 1
      for (; k >= 2; k -= 2) {
        sc_load(c, Fd + 8 * (k - 1));
        sc_load(c0, Fd + 8 * (k - 2));
        sc_horner2(fx, fx, x, c, c0);
        sc_load(c, Fpd + 8 * (k - 1));
        sc_load(c0, Fpd + 8 * (k - 2));
        sc_horner2(fpx, fpx, x, c, c0);
      }
    }
#pragma unroll 1
    while (k-- > 0) {
      sc_load(c, Fd + 8 * k);
      sc_mul_small_add(fx, fx, x, c);
      sc_load(c, Fpd + 8 * k);
      sc_mul_small_add(fpx, fpx, x, c);
    }
    sc_load(sj, s + 8 * e);
    sc_load(spj, sp + 8 * e);
    eqF = sc_eq(sj, fx);
    eqFp = sc_eq(spj, fpx);
  }
  // round 4 (committee.rs:537-541): g s_j == g F(j)  <=>  s_j == F(j)
  dec4[e] = !dokA[d] ? 0 : (rowA ? (eqF ? 1 : 0) : 0);
  uint8_t v2 = !dokE[d] ? 4 : 0;  // missing E: disqualified without a complaint (:331-335)
  if (rowE) {
    if (eqF && eqFp) {
      v2 = 1;
    } else {  // g (s_j - F(j)) + h (s'_j - F'(j)) == identity?  (:292-305)
      sc a, b;
      sc_sub(a, sj, fx);
      sc_sub(b, spj, fpx);
      ge_p3 acc, id;
      ge_identity(acc);
      combw_mul_add(acc, a, tab_g);
      combw_mul_add(acc, b, tab_h);
      ge_identity(id);
      v2 = ristretto_eq(acc, id) ? 1 : 0;
    }
  }
  dec2[e] = v2;
}

void interp_decide(size_t D, size_t nrecv, size_t N, size_t dealer_base, size_t nmod, const uint32_t* s,
                   const uint32_t* sp, const uint32_t* F, const uint32_t* Fp, const uint8_t* dokE, const uint8_t* dokA,
                   const uint8_t* cE, const uint8_t* cA, const uint32_t* tab_g, const uint32_t* tab_h, uint8_t* dec2,
                   uint8_t* dec4, hipStream_t stream) {
  const size_t count = D * nrecv;
  if (!count) return;
  hipLaunchKernelGGL(k_interp_decide, dim3((unsigned)((count + 255) / 256)), dim3(256), 0, stream, D, nrecv, N,
                     dealer_base, (uint32_t)nmod, s, sp, F, Fp, dokE, dokA, cE, cA, tab_g, tab_h, dec2, dec4);
}

// ok[i] &= extra[i]
__global__ void k_and_mask(size_t D, const uint8_t* __restrict__ extra, uint8_t* __restrict__ ok) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < D) ok[i] &= extra[i];
}

void and_mask(size_t D, const uint8_t* extra, uint8_t* ok, hipStream_t stream) {
  if (!D || !extra) return;
  hipLaunchKernelGGL(k_and_mask, dim3((unsigned)((D + 255) / 256)), dim3(256), 0, stream, D, extra, ok);
}

}  // namespace dkgk
