// Scalar field Z_l (l = 2^252 + delta, delta = 27742317777372353535851937790883648493) on gfx950:
// eight 32-bit little-endian limbs, canonical (< l) between operations.
//
// The hot scalar work on this path is Horner evaluation at small integer points
// (Polynomial::evaluate, polynomial.rs:68-74, called at committee.rs:166-167 with x = 1..n), so
// the core primitive is acc <- acc * x + c with x < 2^24: one 8x1 v_mad_u64_u32 row, then a
// pseudo-Mersenne fold x = q 2^252 + lo  ->  lo - q delta (+ l if negative) that needs no division.
// General products (powers j^k for the MSM boundary) use 8x32-bit Montgomery multiplication
// (R = 2^256) in sc_mont_mul.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#ifndef DKG_DEV
#define DKG_DEV __device__ __forceinline__
#endif

struct sc {
  uint32_t v[8];
};

namespace sc_const {
// l in 32-bit limbs
__device__ static const uint32_t L[8] = {0x5cf5d3edu, 0x5812631au, 0xa2f79cd6u, 0x14def9deu,
                                         0u, 0u, 0u, 0x10000000u};
// delta = l - 2^252 (4 limbs)
__device__ static const uint32_t DELTA[4] = {0x5cf5d3edu, 0x5812631au, 0xa2f79cd6u, 0x14def9deu};
// -l^-1 mod 2^32 and R^2 mod l (R = 2^256) for Montgomery products
constexpr uint32_t LINV = 0x12547e1bu;
__device__ static const uint32_t RR[8] = {0x449c0f01u, 0xa40611e3u, 0x68859347u, 0xd00e1ba7u,
                                          0x17f5be65u, 0xceec73d2u, 0x7c309a3du, 0x0399411bu};
}  // namespace sc_const

DKG_DEV void sc_zero(sc& r) {
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = 0;
}

// r = r + (l if neg) : helper for the final correction.
DKG_DEV void sc_add_l_if(sc& r, bool cond) {
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    c += (uint64_t)r.v[i] + (cond ? sc_const::L[i] : 0u);
    r.v[i] = (uint32_t)c;
    c >>= 32;
  }
}

// Reduce a 9-word value x (x < 2^277) mod l.
DKG_DEV void sc_reduce9(sc& r, const uint32_t (&x)[9]) {
  // q = x >> 252 (< 2^25), lo = x mod 2^252
  uint32_t q = (x[7] >> 28) | (x[8] << 4);
  uint32_t lo[8];
#pragma unroll
  for (int i = 0; i < 7; i++) lo[i] = x[i];
  lo[7] = x[7] & 0x0fffffffu;
  // t = q * delta (5 limbs)
  uint32_t t[5];
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    c += (uint64_t)q * sc_const::DELTA[i];
    t[i] = (uint32_t)c;
    c >>= 32;
  }
  t[4] = (uint32_t)c;
  // r = lo - t
  int64_t b = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    int64_t d = (int64_t)lo[i] - (int64_t)(i < 5 ? t[i] : 0u) + b;
    r.v[i] = (uint32_t)d;
    b = d >> 32;  // 0 or -1
  }
  sc_add_l_if(r, b < 0);
}

// r = a * x + c mod l for a, c < l and x < 2^24.
DKG_DEV void sc_mul_small_add(sc& r, const sc& a, uint32_t x, const sc& c) {
  uint32_t w[9];
  uint64_t acc = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    acc += (uint64_t)a.v[i] * x + c.v[i];
    w[i] = (uint32_t)acc;
    acc >>= 32;
  }
  w[8] = (uint32_t)acc;
  sc_reduce9(r, w);
}

// Horner with one reduction per two steps: r = ((a x + c1) x + c0) mod l for a, c1, c0 < l and
// x < 2^11 -- the unreduced 9-word intermediate (< 2^265) times x stays below 2^277, sc_reduce9's range.
DKG_DEV void sc_horner2(sc& r, const sc& a, uint32_t x, const sc& c1, const sc& c0) {
  uint32_t w[9];
  uint64_t acc = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    acc += (uint64_t)a.v[i] * x + c1.v[i];
    w[i] = (uint32_t)acc;
    acc >>= 32;
  }
  w[8] = (uint32_t)acc;
  acc = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) {
    acc += (uint64_t)w[i] * x + (i < 8 ? c0.v[i] : 0u);
    w[i] = (uint32_t)acc;
    acc >>= 32;
  }
  sc_reduce9(r, w);
}

// Horner at a small point with lazy reduction (share evaluation, x < 2^13): the accumulator is ten
// 32-bit limbs and takes up to SC_LAZY_STEPS steps acc * x + c (13 bits each) from below 2^254
// before one fold with 2^252 = -delta mod l:
//   V = H 2^252 + Lo  ->  Lo + l - H delta,
// H < 2^68 so H delta < 2^193 < l: never negative, below 2^254 again.  One fold per five steps
// instead of a full reduction per one or two (sc_mul_small_add / sc_horner2).
constexpr int SC_LAZY_STEPS = 5;  // 2^254 * (2^13)^5 + the coefficients < 2^320
DKG_DEV void sc_lazy_step(uint32_t (&v)[10], uint32_t x, const sc& c) {
  uint64_t t = 0;
#pragma unroll
  for (int i = 0; i < 10; i++) {
    t = (uint64_t)v[i] * x + (i < 8 ? c.v[i] : 0u) + (t >> 32);
    v[i] = (uint32_t)t;
  }
}

DKG_DEV void sc_lazy_fold(uint32_t (&v)[10]) {
  const uint32_t h[3] = {(v[7] >> 28) | (v[8] << 4), (v[8] >> 28) | (v[9] << 4), v[9] >> 28};
  // P = H delta (7 limbs, < 2^193), column by column
  uint32_t p[7];
  uint64_t acc = 0, hiacc = 0;
#pragma unroll
  for (int k = 0; k < 7; k++) {
#pragma unroll
    for (int i = 0; i < 3; i++) {
      const int j = k - i;
      if (j >= 0 && j < 4) {
        const uint64_t m = (uint64_t)h[i] * sc_const::DELTA[j];
        acc += (uint32_t)m;
        hiacc += m >> 32;
      }
    }
    p[k] = (uint32_t)acc;
    acc = (acc >> 32) + hiacc;
    hiacc = 0;
  }
  // Lo + l - P over 8 limbs (the result is positive and below 2^254)
  int64_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint32_t lo = i < 7 ? v[i] : (v[7] & 0x0fffffffu);
    c += (int64_t)lo + sc_const::L[i] - (i < 7 ? p[i] : 0u);
    v[i] = (uint32_t)c;
    c >>= 32;  // arithmetic: a borrow is -1
  }
  v[8] = 0;
  v[9] = 0;
}

// the canonical value of a folded accumulator (< 2^254)
DKG_DEV void sc_lazy_final(sc& r, const uint32_t (&v)[10]) {
  uint32_t w[9];
#pragma unroll
  for (int i = 0; i < 9; i++) w[i] = v[i];
  sc_reduce9(r, w);
}

// r = a + b mod l
DKG_DEV void sc_add(sc& r, const sc& a, const sc& b) {
  uint32_t w[9];
  uint64_t acc = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    acc += (uint64_t)a.v[i] + b.v[i];
    w[i] = (uint32_t)acc;
    acc >>= 32;
  }
  w[8] = (uint32_t)acc;
  sc_reduce9(r, w);
}

// Reduce any 256-bit value (e.g. a `from_bits` input, groups.rs:29-36) to canonical form.
DKG_DEV void sc_reduce256(sc& r, const uint32_t (&x)[8]) {
  uint32_t w[9];
#pragma unroll
  for (int i = 0; i < 8; i++) w[i] = x[i];
  w[8] = 0;
  sc_reduce9(r, w);
}

// Montgomery product a * b / 2^256 mod l (CIOS over 8 words), inputs < l.
DKG_DEV void sc_mont_mul(sc& r, const sc& a, const sc& b) {
  uint32_t t[10];
#pragma unroll
  for (int i = 0; i < 10; i++) t[i] = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint64_t c = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) {
      c += (uint64_t)a.v[j] * b.v[i] + t[j];
      t[j] = (uint32_t)c;
      c >>= 32;
    }
    c += t[8];
    t[8] = (uint32_t)c;
    t[9] = (uint32_t)(c >> 32);
    uint32_t m = t[0] * sc_const::LINV;
    c = (uint64_t)m * sc_const::L[0] + t[0];
    c >>= 32;
#pragma unroll
    for (int j = 1; j < 8; j++) {
      c += (uint64_t)m * sc_const::L[j] + t[j];
      t[j - 1] = (uint32_t)c;
      c >>= 32;
    }
    c += t[8];
    t[7] = (uint32_t)c;
    t[8] = t[9] + (uint32_t)(c >> 32);
  }
  // t < 2l: subtract l once if needed
  uint32_t d[8];
  int64_t bb = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    int64_t x = (int64_t)t[i] - (int64_t)sc_const::L[i] + bb;
    d[i] = (uint32_t)x;
    bb = x >> 32;
  }
  bool ge = (t[8] != 0) || (bb == 0);
#pragma unroll
  for (int i = 0; i < 8; i++) r.v[i] = ge ? d[i] : t[i];
}

// r = a * b mod l
DKG_DEV void sc_mul(sc& r, const sc& a, const sc& b) {
  sc ab, rr;
#pragma unroll
  for (int i = 0; i < 8; i++) rr.v[i] = sc_const::RR[i];
  sc_mont_mul(ab, a, b);    // a b / R
  sc_mont_mul(r, ab, rr);   // a b
}

// Signed radix-16 recoding (64 digits in [-8, 8)), as dalek Scalar::to_radix_16; s < 2^255.
DKG_DEV void sc_radix16(int8_t (&d)[64], const sc& s) {
#pragma unroll
  for (int i = 0; i < 8; i++)
#pragma unroll
    for (int k = 0; k < 8; k++) d[8 * i + k] = (int8_t)((s.v[i] >> (4 * k)) & 15u);
#pragma unroll
  for (int i = 0; i < 63; i++) {
    int8_t carry = (int8_t)((d[i] + 8) >> 4);
    d[i] -= (int8_t)(carry << 4);
    d[i + 1] += carry;
  }
}
