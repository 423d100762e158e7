// Edwards25519 group law (a = -1, twisted Edwards, extended coordinates) and Ristretto255
// encode / decode / equality on gfx950.  Formulas: Hisil-Wong-Carter-Dawson 2008 unified
// addition ("add-2008-hwcd-3") and doubling ("dbl-2008-hwcd"); Ristretto per RFC 9496 section 4.
// The reference reaches the same group through curve25519-dalek (groups.rs:55-90): every value
// that leaves the device is a canonical 32-byte encoding, so results are implementation-independent.
//
// Operand bounds: see fe25519.h (machine-checked by tools/fe_bounds.py).  The comments "<= 2^x"
// below track the worst limb bound of each temporary.
#pragma once
#include "fe25519.h"

struct ge_p3 {  // extended (X : Y : Z : T), x = X/Z, y = Y/Z, xy = T/Z; all tight
  fe X, Y, Z, T;
};
struct ge_cached {  // (Y+X, Y-X, 2Z, 2dT), all tight: an addend prepared for ge_add
  fe YpX, YmX, Z2, T2d;
};
struct ge_aff {  // affine Niels (y+x, y-x, 2dxy), tight: fixed-base table entries (Z = 1)
  fe ypx, ymx, xy2d;
};

namespace ge_const {
__device__ static const uint32_t D[10] = {0x35978a3u, 0xd37284u, 0x3156ebdu, 0x6a0a0eu, 0x1c029u,
                                          0x179e898u, 0x3a03cbbu, 0x1ce7198u, 0x2e2b6ffu, 0x1480db3u};
__device__ static const uint32_t D2[10] = {0x2b2f159u, 0x1a6e509u, 0x22add7au, 0xd4141du, 0x38052u,
                                           0xf3d130u, 0x3407977u, 0x19ce331u, 0x1c56dffu, 0x901b67u};
__device__ static const uint32_t SQRT_M1[10] = {0x20ea0b0u, 0x186c9d2u, 0x8f189du, 0x35697fu,
                                                0xbd0c60u, 0x1fbd7a7u, 0x2804c9eu, 0x1e16569u,
                                                0x4fc1du, 0xae0c92u};
__device__ static const uint32_t SQRT_AD_MINUS_ONE[10] = {
    0x17b2e1bu, 0x1fda812u, 0x297afd2u, 0x60dbc2u, 0x2be7638u,
    0x1f5d1fdu, 0x27e6498u, 0x11581e7u, 0x3f2b834u, 0xdda4c6u};
__device__ static const uint32_t INVSQRT_A_MINUS_D[10] = {
    0x5d40eau, 0x3f6aa0u, 0x257d339u, 0xbad20bu, 0x274bc58u,
    0x1d840u, 0x13dc8ffu, 0x19442d8u, 0x5cfaffu, 0x1e1b224u};
__device__ static const uint32_t ONE_MINUS_D_SQ[10] = {
    0x5fc176u, 0x1027065u, 0x2a1fc4fu, 0x1c66af1u, 0xb20684u,
    0x70dfe4u, 0x255eedfu, 0x1af332u, 0x28b2b3eu, 0xa41cau};
__device__ static const uint32_t D_MINUS_ONE_SQ[10] = {
    0xed4d20u, 0x156aa91u, 0x3332635u, 0x16580f0u, 0x34a7928u,
    0x9b4eebu, 0x26997a9u, 0x48299bu, 0x3af66c2u, 0x165a2cdu};
}  // namespace ge_const

DKG_DEV void fe_ld(fe& r, const uint32_t* c) {
#pragma unroll
  for (int i = 0; i < 10; i++) r.v[i] = c[i];
}

DKG_DEV void ge_identity(ge_p3& p) {
  fe_zero(p.X);
  fe_one(p.Y);
  fe_one(p.Z);
  fe_zero(p.T);
}

DKG_DEV void ge_to_cached(ge_cached& c, const ge_p3& p) {
  // Y+X <= 2^27, Y-X+2p <= 2^27.585 and 2Z <= 2^27 are left uncarried: a cached value is only
  // ever the second (x19) operand of fe_mul, which takes them (tools/fe_bounds.py)
  fe_add(c.YpX, p.Y, p.X);
  fe_sub(c.YmX, p.Y, p.X);
  fe_dbl(c.Z2, p.Z);
  fe d2;
  fe_ld(d2, ge_const::D2);
  fe_mul(c.T2d, p.T, d2);
}

DKG_DEV void ge_cached_neg(ge_cached& r, const ge_cached& c) {
  fe_copy(r.YpX, c.YmX);
  fe_copy(r.YmX, c.YpX);
  fe_copy(r.Z2, c.Z2);
  fe_neg(r.T2d, c.T2d);
  fe_carry(r.T2d, r.T2d);
}

// IL = true (the template argument of the formulas below): the same products, operand for operand,
// as pairs (fe_mul2 / fe_sq2: two interleaved chains, fewer hazard wait states) at the cost of one
// more field temporary live; for the kernels with VGPRs to spare (profiles/r06_pair_ab.txt).
// Additions are written so that (a, b) collapse into (e, h) before (c, d) are formed: at most
// four field temporaries are live next to the operands (keeps the kernels at <= 128 VGPRs).
// r = p + q  (8M).  r may alias p.
template <bool IL = false>
DKG_DEV void ge_add(ge_p3& r, const ge_p3& p, const ge_cached& q) {
  if constexpr (IL && DKG_PW) {
    // the same products, operand for operand, as four pairs (fe_mul2)
    fe a, b, e, h, t, u;
    fe_sub(t, p.Y, p.X);
    fe_add(u, p.Y, p.X);
    fe_mul2(a, t, q.YmX, b, u, q.YpX);
    fe_sub(e, b, a);
    fe_add(h, b, a);
    fe_mul2(a, p.T, q.T2d, b, p.Z, q.Z2);  // c, d
    fe_sub(t, b, a);          // f
    fe_add(b, b, a);          // g
    fe_mul2(r.X, e, t, r.Y, b, h);
    fe_mul2(r.Z, b, t, r.T, e, h);
    return;
  }
  fe a, b, e, h, t;
  fe_sub(t, p.Y, p.X);      // <= 1.5*2^27
  fe_mul(a, t, q.YmX);
  fe_add(t, p.Y, p.X);      // <= 2^27
  fe_mul(b, t, q.YpX);
  fe_sub(e, b, a);          // <= 1.5*2^27
  fe_add(h, b, a);          // <= 2^27
  fe_mul(a, p.T, q.T2d);    // c
  fe_mul(b, p.Z, q.Z2);     // d
  fe_sub(t, b, a);          // f = d - c <= 1.5*2^27
  fe_add(b, b, a);          // g = d + c <= 2^27
  fe_mul(r.X, e, t);
  fe_mul(r.Y, b, h);
  fe_mul(r.Z, b, t);        // the x19 operands are F (X, Z) and H (Y, T): computed once each
  fe_mul(r.T, e, h);
}

// r = p - q
DKG_DEV void ge_sub(ge_p3& r, const ge_p3& p, const ge_cached& q) {
  fe a, b, e, h, t;
  fe_sub(t, p.Y, p.X);
  fe_mul(a, t, q.YpX);
  fe_add(t, p.Y, p.X);
  fe_mul(b, t, q.YmX);
  fe_sub(e, b, a);
  fe_add(h, b, a);
  fe_mul(a, p.T, q.T2d);    // c
  fe_mul(b, p.Z, q.Z2);     // d
  fe_add(t, b, a);          // f = d + c (sign of c flipped for -q)
  fe_sub(b, b, a);          // g = d - c
  fe_mul(r.X, e, t);
  fe_mul(r.Y, b, h);
  fe_mul(r.Z, b, t);        // the x19 operands are F (X, Z) and H (Y, T): computed once each
  fe_mul(r.T, e, h);
}

// r = p + q with q affine Niels (Z = 1): 7M.
template <bool IL = false>
DKG_DEV void ge_madd(ge_p3& r, const ge_p3& p, const ge_aff& q) {
  if constexpr (IL && DKG_PW) {
    // the four result products as two pairs; A and B stay single (pairing them too pushes the 128-VGPR
    // comb kernels into scratch)
    fe a, b, e, h, t;
    fe_sub(t, p.Y, p.X);
    fe_mul(a, t, q.ymx);
    fe_add(t, p.Y, p.X);
    fe_mul(b, t, q.ypx);
    fe_sub(e, b, a);
    fe_add(h, b, a);
    fe_mul(a, p.T, q.xy2d);   // c
    fe_dbl(b, p.Z);           // d <= 2^27
    fe_sub(t, b, a);          // f
    fe_add(b, b, a);          // g
    fe_mul2(r.X, t, e, r.Y, h, b);
    fe_mul2(r.Z, t, b, r.T, h, e);
    return;
  }
  fe a, b, e, h, t;
  fe_sub(t, p.Y, p.X);
  fe_mul(a, t, q.ymx);
  fe_add(t, p.Y, p.X);
  fe_mul(b, t, q.ypx);
  fe_sub(e, b, a);
  fe_add(h, b, a);
  fe_mul(a, p.T, q.xy2d);   // c
  fe_dbl(b, p.Z);           // d <= 2^27
  fe_sub(t, b, a);          // f = d - c <= 2^27 + 2^27
  fe_add(b, b, a);          // g = d + c <= 1.5*2^27
  fe_mul(r.X, t, e);        // f <= 2^28 as first operand
  fe_mul(r.Y, h, b);        // x19 operands E (X, T) and G (Y, Z), computed once each
  fe_mul(r.Z, t, b);
  fe_mul(r.T, h, e);
}

DKG_DEV void ge_msub(ge_p3& r, const ge_p3& p, const ge_aff& q) {
  fe a, b, e, h, t;
  fe_sub(t, p.Y, p.X);
  fe_mul(a, t, q.ypx);
  fe_add(t, p.Y, p.X);
  fe_mul(b, t, q.ymx);
  fe_sub(e, b, a);
  fe_add(h, b, a);
  fe_mul(a, p.T, q.xy2d);   // c
  fe_dbl(b, p.Z);           // d
  fe_add(t, b, a);          // f = d + c <= 1.5*2^27
  fe_sub(b, b, a);          // g = d - c <= 2^28
  fe_mul(r.X, e, t);        // x19 operands F (X, Z) and H (Y, T), computed once each
  fe_mul(r.Y, b, h);        // g <= 2^28 first operand
  fe_mul(r.Z, b, t);
  fe_mul(r.T, e, h);
}

// r = 2p (4S + 4M); with_t = false skips T (valid when the next op is another doubling).
template <bool with_t = true, bool IL = false>
DKG_DEV void ge_dbl(ge_p3& r, const ge_p3& p) {
  if constexpr (IL && DKG_PW) {
    fe a, b, c, e, f, g, h, t;
    fe_add(t, p.X, p.Y);
    fe_sq2(a, p.X, b, p.Y);
    fe_sq2(c, p.Z, t, t);
    fe_dbl(c, c);
    fe_add(h, a, b);
    fe_sub(e, h, t);
    fe_sub(g, a, b);
    fe_add(f, c, g);
    fe_carry(f, f);
    fe_mul2(r.X, e, f, r.Y, g, h);
    if (with_t) fe_mul2(r.Z, g, f, r.T, e, h);
    else fe_mul(r.Z, g, f);
    return;
  }
  fe a, b, c, e, f, g, h, t;
  fe_sq(a, p.X);
  fe_sq(b, p.Y);
  fe_sq(c, p.Z);
  fe_dbl(c, c);             // <= 2^27
  fe_add(t, p.X, p.Y);      // <= 2^27
  fe_sq(t, t);
  fe_add(h, a, b);          // <= 2^27             (= -H_std)
  fe_sub(e, h, t);          // <= 2^28             (= -E_std)
  fe_sub(g, a, b);          // <= 1.5*2^27         (= -G_std)
  fe_add(f, c, g);          // <= 2.5*2^27
  fe_carry(f, f);           // tight               (= -F_std)
  fe_mul(r.X, e, f);
  fe_mul(r.Y, g, h);
  fe_mul(r.Z, g, f);        // x19 operands f (X, Z) and h (Y, T), computed once each
  if (with_t) fe_mul(r.T, e, h);
}

// Doubling with a run-time (wave-uniform) choice of whether T is produced.
template <bool IL = false>
DKG_DEV void ge_dbl_rt(ge_p3& r, const ge_p3& p, bool with_t) {
  if constexpr (IL && DKG_PW) {
    fe a, b, c, t, h, e, g;
    fe_add(t, p.X, p.Y);
    fe_sq2(a, p.X, b, p.Y);
    fe_sq2(c, p.Z, t, t);
    fe_dbl(c, c);
    fe_add(h, a, b);
    fe_sub(e, h, t);
    fe_sub(g, a, b);
    fe_add(c, c, g);
    fe_carry(c, c);
    fe_mul2(r.X, e, c, r.Y, g, h);
    if (with_t) fe_mul2(r.Z, g, c, r.T, e, h);
    else fe_mul(r.Z, g, c);
    return;
  }
  fe a, b, c, t, h, e, g;
  fe_sq(a, p.X);
  fe_sq(b, p.Y);
  fe_sq(c, p.Z);
  fe_dbl(c, c);             // <= 2^27
  fe_add(t, p.X, p.Y);      // <= 2^27
  fe_sq(t, t);              // (X+Y)^2
  fe_add(h, a, b);          // <= 2^27             (= -H_std)
  fe_sub(e, h, t);          // <= 2^28             (= -E_std)
  fe_sub(g, a, b);          // <= 1.5*2^27         (= -G_std)
  fe_add(c, c, g);          // f <= 2.5*2^27
  fe_carry(c, c);           // tight               (= -F_std)
  fe_mul(r.X, e, c);
  fe_mul(r.Y, g, h);
  fe_mul(r.Z, g, c);        // x19 operands f (X, Z) and h (Y, T), computed once each
  if (with_t) fe_mul(r.T, e, h);
}

// Doubling with the fewest simultaneously live temporaries (inputs consumed early; r may alias p).
template <bool IL = false>
DKG_DEV void ge_dbl_lean(ge_p3& r, const ge_p3& p, bool with_t) {
  if constexpr (IL && DKG_PW) {
    fe a, b, t, h, g;
    fe_sq2(a, p.X, b, p.Y);
    fe_add(h, a, b);
    fe_sub(g, a, b);
    fe_add(a, p.X, p.Y);
    fe_sq2(t, p.Z, a, a);     // Z^2, (X+Y)^2
    fe_dbl(t, t);
    fe_add(t, t, g);
    fe_carry(t, t);           // f
    fe_sub(b, h, a);          // e
    fe_mul2(r.X, b, t, r.Y, g, h);
    if (with_t) fe_mul2(r.Z, g, t, r.T, b, h);
    else fe_mul(r.Z, g, t);
    return;
  }
  fe a, b, t, h, g;
  fe_sq(a, p.X);
  fe_sq(b, p.Y);
  fe_add(h, a, b);          // <= 2^27             (= -H_std)
  fe_sub(g, a, b);          // <= 1.5*2^27         (= -G_std)
  fe_sq(t, p.Z);
  fe_dbl(t, t);             // 2Z^2 <= 2^27
  fe_add(t, t, g);          // <= 2.5*2^27
  fe_carry(t, t);           // f, tight            (= -F_std)
  fe_add(a, p.X, p.Y);      // <= 2^27
  fe_sq(a, a);              // (X+Y)^2
  fe_sub(b, h, a);          // e <= 2^28           (= -E_std)
  fe_mul(r.X, b, t);
  fe_mul(r.Y, g, h);
  fe_mul(r.Z, g, t);        // x19 operands f (X, Z) and h (Y, T), computed once each
  if (with_t) fe_mul(r.T, b, h);
}

// r = p + q (neg = false) or p - q (neg = true) with one code path: the sign only selects
// which of (Y+X, Y-X) multiplies which, and the sign of the 2dT product.
// with_t = false skips T (one product): valid when the next operation is a doubling, which does not
// read it.
template <bool IL = false>
DKG_DEV void ge_add_signed(ge_p3& r, const ge_p3& p, const ge_cached& q, bool neg, bool with_t = true) {
  fe a, b, e, h, t, qa, qb;
#pragma unroll
  for (int i = 0; i < 10; i++) {
    qa.v[i] = neg ? q.YpX.v[i] : q.YmX.v[i];
    qb.v[i] = neg ? q.YmX.v[i] : q.YpX.v[i];
  }
  if constexpr (IL && DKG_PW) {
    fe u;
    fe_sub(t, p.Y, p.X);
    fe_add(u, p.Y, p.X);
    fe_mul2(a, t, qa, b, u, qb);
  } else {
    fe_sub(t, p.Y, p.X);
    fe_mul(a, t, qa);
    fe_add(t, p.Y, p.X);
    fe_mul(b, t, qb);
  }
  fe_sub(e, b, a);
  fe_add(h, b, a);
  if constexpr (IL && DKG_PW) {
    fe_mul2(a, p.T, q.T2d, b, p.Z, q.Z2);  // c (the term whose sign flips with q), d
  } else {
    fe_mul(a, p.T, q.T2d);  // c  (the term whose sign flips with q)
    fe_mul(b, p.Z, q.Z2);   // d
  }
  fe na;
  fe_neg(na, a);            // -c = 2p - c <= 2p limbwise: a valid fe_sub subtrahend as is
  fe_cmov(a, na, neg);      // a = +/-c (limbs <= 2^27)
  fe_sub(t, b, a);          // f = d - (+/-c) <= 1.5*2^27
  fe_add(b, b, a);          // g <= 2^27
  if constexpr (IL && DKG_PW) {
    fe_mul2(r.X, e, t, r.Y, b, h);
    if (with_t) fe_mul2(r.Z, b, t, r.T, e, h);
    else fe_mul(r.Z, b, t);
  } else {
    fe_mul(r.X, e, t);
    fe_mul(r.Y, b, h);
    fe_mul(r.Z, b, t);      // the x19 operands are F (X, Z) and H (Y, T): computed once each
    if (with_t) fe_mul(r.T, e, h);
  }
}

// r = p + q (neg = false) or p - q (neg = true), q affine Niels (Z = 1): 7M, one code path.  The
// sign selects which of (y+x, y-x) multiplies which and the sign of c; d = 2Z is carried so that
// f and g keep ge_add_signed's bounds whatever the sign.  q's fields are second operands only, so
// they may carry the cached form's uncarried bounds (y+x <= 2^27, y-x <= 2^27.585;
// tools/fe_bounds.py).
template <bool IL = false>
DKG_DEV void ge_madd_signed(ge_p3& r, const ge_p3& p, const ge_aff& q, bool neg, bool with_t = true) {
  fe a, b, e, h, t, qa, qb;
#pragma unroll
  for (int i = 0; i < 10; i++) {
    qa.v[i] = neg ? q.ypx.v[i] : q.ymx.v[i];
    qb.v[i] = neg ? q.ymx.v[i] : q.ypx.v[i];
  }
  if constexpr (IL && DKG_PW) {
    fe u;
    fe_sub(t, p.Y, p.X);
    fe_add(u, p.Y, p.X);
    fe_mul2(a, t, qa, b, u, qb);
  } else {
    fe_sub(t, p.Y, p.X);
    fe_mul(a, t, qa);
    fe_add(t, p.Y, p.X);
    fe_mul(b, t, qb);
  }
  fe_sub(e, b, a);
  fe_add(h, b, a);
  fe_mul(a, p.T, q.xy2d);   // c
  fe na;
  fe_neg(na, a);            // -c = 2p - c <= 2p limbwise
  fe_cmov(a, na, neg);      // a = +/-c
  fe_dbl(b, p.Z);
  fe_carry(b, b);           // d = 2Z, tight
  fe_sub(t, b, a);          // f = d - (+/-c)
  fe_add(b, b, a);          // g = d + (+/-c)
  if constexpr (IL && DKG_PW) {
    fe_mul2(r.X, e, t, r.Y, b, h);
    if (with_t) fe_mul2(r.Z, b, t, r.T, e, h);
    else fe_mul(r.Z, b, t);
  } else {
    fe_mul(r.X, e, t);
    fe_mul(r.Y, b, h);
    fe_mul(r.Z, b, t);      // the x19 operands are F (X, Z) and H (Y, T): computed once each
    if (with_t) fe_mul(r.T, e, h);
  }
}

// ---- Ristretto255 (RFC 9496 section 4.3) ----

// (was_square, r) = SQRT_RATIO_M1(u, v); u, v tight.
DKG_DEV bool fe_sqrt_ratio_m1(fe& r, const fe& u, const fe& v) {
  fe v3, v7, t, chk, neg_u, neg_u_i, sqrtm1;
  fe_ld(sqrtm1, ge_const::SQRT_M1);
  fe_sq(v3, v);
  fe_mul(v3, v3, v);        // v^3
  fe_sq(v7, v3);
  fe_mul(v7, v7, v);        // v^7
  fe_mul(t, u, v7);
  fe_pow22523(t, t);        // (u v^7)^((p-5)/8)
  fe_mul(t, t, v3);
  fe_mul(r, t, u);          // r = u v^3 (u v^7)^((p-5)/8)
  fe_sq(chk, r);
  fe_mul(chk, chk, v);      // v r^2
  fe_neg(neg_u, u);
  fe_carry(neg_u, neg_u);
  fe_mul(neg_u_i, neg_u, sqrtm1);
  fe d;
  fe_sub(d, chk, u);
  bool correct = fe_iszero(d);
  fe_sub(d, chk, neg_u);
  bool flipped = fe_iszero(d);
  fe_sub(d, chk, neg_u_i);
  bool flipped_i = fe_iszero(d);
  fe r_prime;
  fe_mul(r_prime, r, sqrtm1);
  fe_cmov(r, r_prime, flipped || flipped_i);
  fe_abs(r, r);
  return correct || flipped;
}

// Two independent SQRT_RATIO_M1 chains at once (k_encode with DKG_ENCODE_PAIR: the inverse square
// roots of a lane's two points), every product and square as a pair (fe_mul2 / fe_sq2): the same
// operations, operand for operand, as fe_sqrt_ratio_m1 on each.
DKG_DEV void fe_sq_x2(fe (&r)[2], const fe (&a)[2]) { fe_sq2(r[0], a[0], r[1], a[1]); }
DKG_DEV void fe_mul_x2(fe (&r)[2], const fe (&a)[2], const fe (&b)[2]) {
  fe_mul2(r[0], a[0], b[0], r[1], a[1], b[1]);
}
DKG_DEV void fe_sqn_x2(fe (&r)[2], const fe (&a)[2], int n) {
  fe_sq_x2(r, a);
  for (int i = 1; i < n; i++) fe_sq_x2(r, r);
}
DKG_DEV void fe_pow22523_x2(fe (&out)[2], const fe (&z)[2]) {
  fe t0[2], t1[2], t2[2];
  fe_sq_x2(t0, z);            // 2
  fe_sqn_x2(t1, t0, 2);       // 8
  fe_mul_x2(t1, z, t1);       // 9
  fe_mul_x2(t0, t0, t1);      // 11
  fe_sq_x2(t0, t0);           // 22
  fe_mul_x2(t0, t1, t0);      // 2^5 - 1
  fe_sqn_x2(t1, t0, 5);
  fe_mul_x2(t0, t1, t0);      // 2^10 - 1
  fe_sqn_x2(t1, t0, 10);
  fe_mul_x2(t1, t1, t0);      // 2^20 - 1
  fe_sqn_x2(t2, t1, 20);
  fe_mul_x2(t1, t2, t1);      // 2^40 - 1
  fe_sqn_x2(t1, t1, 10);
  fe_mul_x2(t0, t1, t0);      // 2^50 - 1
  fe_sqn_x2(t1, t0, 50);
  fe_mul_x2(t1, t1, t0);      // 2^100 - 1
  fe_sqn_x2(t2, t1, 100);
  fe_mul_x2(t1, t2, t1);      // 2^200 - 1
  fe_sqn_x2(t1, t1, 50);
  fe_mul_x2(t0, t1, t0);      // 2^250 - 1
  fe_sqn_x2(t0, t0, 2);       // 2^252 - 4
  fe_mul_x2(out, t0, z);      // 2^252 - 3
}
// r[k] = SQRT_RATIO_M1(1, v[k]).r (the encoding's inverse square root; was_square is not needed there)
DKG_DEV void fe_invsqrt_x2(fe (&r)[2], const fe (&v)[2]) {
  fe v3[2], t[2];
  fe_sq_x2(v3, v);
  fe_mul_x2(v3, v3, v);       // v^3
  fe_sq_x2(t, v3);
  fe_mul_x2(t, t, v);         // v^7 (= u v^7 with u = 1)
  fe_pow22523_x2(t, t);       // (v^7)^((p-5)/8)
  fe_mul_x2(r, t, v3);        // r = v^3 (v^7)^((p-5)/8)
  fe chk[2];
  fe_sq_x2(chk, r);
  fe_mul_x2(chk, chk, v);     // v r^2
  fe sqrtm1, one, neg_one, neg_i;
  fe_ld(sqrtm1, ge_const::SQRT_M1);
  fe_one(one);
  fe_neg(neg_one, one);
  fe_carry(neg_one, neg_one);
  fe_mul(neg_i, neg_one, sqrtm1);
#pragma unroll
  for (int k = 0; k < 2; k++) {
    fe d, r_prime;
    fe_sub(d, chk[k], neg_one);
    const bool flipped = fe_iszero(d);
    fe_sub(d, chk[k], neg_i);
    const bool flipped_i = fe_iszero(d);
    fe_mul(r_prime, r[k], sqrtm1);
    fe_cmov(r[k], r_prime, flipped || flipped_i);
    fe_abs(r[k], r[k]);
  }
}

// Decode 32 bytes (as 8 LE words).  Returns false for a non-canonical / invalid encoding
// (dalek CompressedRistretto::decompress -> None, groups.rs:78-81).
DKG_DEV bool ristretto_decode(ge_p3& p, const uint32_t (&w)[8]) {
  // canonical: s < p and s even
  fe s;
  fe_frombytes32(s, w);
  uint32_t chk[8];
  fe_tobytes32(chk, s);
  uint32_t diff = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) diff |= chk[i] ^ w[i];
  bool ok = (diff == 0) && ((w[0] & 1u) == 0);
  fe ss, u1, u2, u2sq, v, one, t, inv, den_x, den_y, dd;
  fe_one(one);
  fe_sq(ss, s);
  fe_sub(u1, one, ss);
  fe_carry(u1, u1);
  fe_add(u2, one, ss);
  fe_carry(u2, u2);
  fe_sq(u2sq, u2);
  fe_ld(dd, ge_const::D);
  fe_sq(t, u1);
  fe_mul(t, t, dd);          // D u1^2
  fe_add(t, t, u2sq);
  fe_carry(t, t);
  fe_neg(v, t);              // v = -(D u1^2) - u2^2
  fe_carry(v, v);
  fe_mul(t, v, u2sq);
  bool was_sq = fe_sqrt_ratio_m1(inv, one, t);
  fe_mul(den_x, inv, u2);
  fe_mul(den_y, inv, den_x);
  fe_mul(den_y, den_y, v);
  fe_add(t, s, s);
  fe_carry(t, t);
  fe_mul(t, t, den_x);
  fe_abs(p.X, t);
  fe_mul(p.Y, u1, den_y);
  fe_one(p.Z);
  fe_mul(p.T, p.X, p.Y);
  ok = ok && was_sq && !fe_isneg(p.T) && !fe_iszero(p.Y);
  return ok;
}

// Encode to 8 LE words (RFC 9496 ENCODE).
// The encoding in two halves around its inverse square root, so that a caller can drop the point
// across the exponentiation and reload it (k_encode: the point's 40 registers are not live during the
// 265-operation chain).
DKG_DEV void ristretto_encode_pre(fe& u1, fe& u2, fe& t, const ge_p3& p) {
  fe_add(t, p.Z, p.Y);
  fe_sub(u1, p.Z, p.Y);
  fe_mul(u1, t, u1);                 // (Z+Y)(Z-Y)
  fe_mul(u2, p.X, p.Y);
  fe_sq(t, u2);
  fe_mul(t, t, u1);
}
DKG_DEV void ristretto_encode_post(uint32_t (&w)[8], const ge_p3& p, const fe& u1, const fe& u2, const fe& inv);
// u1 = (Z+Y)(Z-Y), u2 = X Y again from the reloaded point (k_encode keeps only t across the chain)
DKG_DEV void ristretto_encode_u(fe& u1, fe& u2, const ge_p3& p) {
  fe t;
  fe_add(t, p.Z, p.Y);
  fe_sub(u1, p.Z, p.Y);
  fe_mul(u1, t, u1);
  fe_mul(u2, p.X, p.Y);
}
DKG_DEV void ristretto_encode(uint32_t (&w)[8], const ge_p3& p) {
  fe u1, u2, t, inv, one;
  fe_one(one);
  ristretto_encode_pre(u1, u2, t, p);
  fe_sqrt_ratio_m1(inv, one, t);
  ristretto_encode_post(w, p, u1, u2, inv);
}
DKG_DEV void ristretto_encode_post(uint32_t (&w)[8], const ge_p3& p, const fe& u1, const fe& u2, const fe& inv) {
  fe t, den1, den2, z_inv, ix0, iy0, ench, x, y, den_inv, sqrtm1;
  fe_ld(sqrtm1, ge_const::SQRT_M1);
  fe_mul(den1, inv, u1);
  fe_mul(den2, inv, u2);
  fe_mul(z_inv, den1, den2);
  fe_mul(z_inv, z_inv, p.T);
  fe_mul(ix0, p.X, sqrtm1);
  fe_mul(iy0, p.Y, sqrtm1);
  fe_ld(t, ge_const::INVSQRT_A_MINUS_D);
  fe_mul(ench, den1, t);
  fe_mul(t, p.T, z_inv);
  bool rotate = fe_isneg(t);
  fe_copy(x, p.X);
  fe_copy(y, p.Y);
  fe_cmov(x, iy0, rotate);
  fe_cmov(y, ix0, rotate);
  fe_copy(den_inv, den2);
  fe_cmov(den_inv, ench, rotate);
  fe_mul(t, x, z_inv);
  if (fe_isneg(t)) {
    fe_neg(y, y);
    fe_carry(y, y);
  }
  fe_sub(t, p.Z, y);
  fe_mul(t, den_inv, t);
  fe_abs(t, t);
  fe_tobytes32(w, t);
}

// Ristretto equality (RFC 9496 EQUALS): X1 Y2 == Y1 X2 or Y1 Y2 == X1 X2.
DKG_DEV bool ristretto_eq(const ge_p3& p, const ge_p3& q) {
  fe a, b, d;
  fe_mul(a, p.X, q.Y);
  fe_mul(b, p.Y, q.X);
  fe_sub(d, a, b);
  bool e1 = fe_iszero(d);
  fe_mul(a, p.Y, q.Y);
  fe_mul(b, p.X, q.X);
  fe_sub(d, a, b);
  return e1 || fe_iszero(d);
}

// Elligator one-way map (RFC 9496 MAP) of 255 bits given as 8 words (bit 255 masked).
DKG_DEV void ristretto_elligator(ge_p3& p, const uint32_t (&w)[8]) {
  uint32_t m[8];
#pragma unroll
  for (int i = 0; i < 8; i++) m[i] = w[i];
  m[7] &= 0x7fffffffu;
  fe t0, r, u, v, s, s_prime, c, n, w0, w1, w2, w3, one, dd, tmp, tmp2, sqrtm1;
  fe_frombytes32(t0, m);
  fe_carry(t0, t0);
  fe_one(one);
  fe_ld(dd, ge_const::D);
  fe_ld(sqrtm1, ge_const::SQRT_M1);
  fe_sq(r, t0);
  fe_mul(r, r, sqrtm1);                       // r = i t^2
  fe_add(tmp, r, one);
  fe_ld(tmp2, ge_const::ONE_MINUS_D_SQ);
  fe_mul(u, tmp, tmp2);                       // u = (r+1)(1-d^2)
  fe_mul(tmp, r, dd);
  fe_add(tmp, tmp, one);
  fe_neg(tmp, tmp);
  fe_carry(tmp, tmp);                         // -1 - r d
  fe_add(tmp2, r, dd);
  fe_mul(v, tmp, tmp2);                       // v = (-1 - r d)(r + d)
  bool was_sq = fe_sqrt_ratio_m1(s, u, v);
  fe_mul(s_prime, s, t0);
  fe_abs(s_prime, s_prime);
  fe_neg(s_prime, s_prime);
  fe_carry(s_prime, s_prime);
  if (!was_sq) fe_copy(s, s_prime);
  fe_neg(c, one);
  fe_carry(c, c);
  if (!was_sq) fe_copy(c, r);
  fe_sub(tmp, r, one);
  fe_mul(n, c, tmp);
  fe_ld(tmp2, ge_const::D_MINUS_ONE_SQ);
  fe_mul(n, n, tmp2);
  fe_sub(n, n, v);
  fe_carry(n, n);                             // N = c (r-1) (d-1)^2 - v
  fe_add(tmp, s, s);
  fe_carry(tmp, tmp);
  fe_mul(w0, tmp, v);                         // 2 s v
  fe_ld(tmp2, ge_const::SQRT_AD_MINUS_ONE);
  fe_mul(w1, n, tmp2);
  fe_sq(tmp, s);
  fe_sub(w2, one, tmp);
  fe_carry(w2, w2);
  fe_add(w3, one, tmp);
  fe_mul(p.X, w0, w3);
  fe_mul(p.Y, w2, w1);
  fe_mul(p.Z, w1, w3);
  fe_mul(p.T, w0, w2);
}
