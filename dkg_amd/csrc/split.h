// Lane-pair group operations: the two lanes 2p and 2p+1 of a wave hold the same point and each
// computes half of every formula's field products; the halves cross through LDS (no VALU work:
// each lane writes its two products and reads both lanes' from a per-wave exchange buffer).
// A latency-bound chain (a binomial step of a small multi-GPU shard: one NAF chain per wave, a
// wave or two per SIMD) then runs half as many dependent instructions per lane, at twice the lanes.
//
// The formulas are ge_dbl_lean / ge_add_lds term for term with the same operand order, so every
// limb equals the single-lane result (and tools/fe_bounds.py's bounds hold as they are):
//   doubling: role 0 squares X and Z, role 1 Y and X+Y; after the exchange both form h, g, f, e;
//             then o1 = e N, o2 = g N with N = f (role 0: X3, Z3) or N = h (role 1: T3, Y3).
//   addition: role 0 forms A = (Y1-X1) q_a and C = T1 2dT2, role 1 B = (Y1+X1) q_b and D = Z1 2Z2
//             (q_a, q_b = Y2-X2, Y2+X2, swapped when subtracting), then the outputs as above.
// The cached addend of a pair sits once in LDS ([40 words][32 pairs]); the exchange buffer holds
// [20 words][64 lanes] per wave.  Both are per wave, so no cross-wave synchronisation is involved;
// the kernels run one wave per workgroup and __syncthreads() orders the LDS traffic.
#pragma once
#include "points.h"

struct pair_ctx {
  uint32_t* xb;  // exchange buffer of this wave: word k of lane l at xb[k * 64 + l]
  uint32_t* qs;  // cached addend of this lane's pair: word k at qs[k * 32] (qs = base + pair)
  int role;      // lane & 1
  int lane;
};

DKG_DEV void fe_sel(fe& r, const fe& a, const fe& b, bool c) {  // r = c ? b : a
#pragma unroll
  for (int i = 0; i < 10; i++) r.v[i] = c ? b.v[i] : a.v[i];
}

// Each lane contributes (u, v); returns role 0's pair in (u0, v0) and role 1's in (u1, v1).
DKG_DEV void pair_xchg(const pair_ctx& c, const fe& u, const fe& v, fe& u0, fe& v0, fe& u1, fe& v1) {
  uint32_t* w = c.xb + c.lane;
#pragma unroll
  for (int k = 0; k < 10; k++) {
    w[k * 64] = u.v[k];
    w[(10 + k) * 64] = v.v[k];
  }
  __syncthreads();  // one-wave workgroup: orders the LDS writes before the partner's reads
  const uint32_t* r0 = c.xb + (c.lane & ~1);
  const uint32_t* r1 = r0 + 1;
#pragma unroll
  for (int k = 0; k < 10; k++) {
    u0.v[k] = r0[k * 64];
    v0.v[k] = r0[(10 + k) * 64];
    u1.v[k] = r1[k * 64];
    v1.v[k] = r1[(10 + k) * 64];
  }
  __syncthreads();  // the buffer is reused by the next exchange
}

// r = 2p (ge_dbl_lean); T is computed whatever with_t says (role 1's second product).
DKG_DEV void ge_dbl_pair(ge_p3& r, const ge_p3& p, const pair_ctx& c) {
  fe s1, s2;
  {
    fe xy, in1, in2;
    fe_add(xy, p.X, p.Y);            // <= 2^27
    fe_sel(in1, p.X, p.Y, c.role);   // role 0: X^2, role 1: Y^2
    fe_sel(in2, p.Z, xy, c.role);    // role 0: Z^2, role 1: (X+Y)^2
    fe_sq(s1, in1);
    fe_sq(s2, in2);
  }
  fe a, zz, b, t;
  pair_xchg(c, s1, s2, a, zz, b, t);
  fe h, g, f, e;
  fe_add(h, a, b);                   // <= 2^27             (= -H_std)
  fe_sub(g, a, b);                   // <= 1.5*2^27         (= -G_std)
  fe_dbl(f, zz);                     // 2Z^2 <= 2^27
  fe_add(f, f, g);                   // <= 2.5*2^27
  fe_carry(f, f);                    // f, tight            (= -F_std)
  fe_sub(e, h, t);                   // e <= 2^28           (= -E_std)
  fe n, o1, o2;
  fe_sel(n, f, h, c.role);
  fe_mul(o1, e, n);                  // role 0: X3 = e f, role 1: T3 = e h
  fe_mul(o2, g, n);                  // role 0: Z3 = g f, role 1: Y3 = g h
  pair_xchg(c, o1, o2, r.X, r.Z, r.T, r.Y);
}

// The cached form (ge_to_cached) of p into the pair's LDS slot: role 0 writes Y+X and Y-X, role 1
// 2Z and 2dT.
DKG_DEV void pair_put_cached(const pair_ctx& c, const ge_p3& p) {
  ge_cached q;
  ge_to_cached(q, p);
  fe w1, w2;
  fe_sel(w1, q.YpX, q.Z2, c.role);
  fe_sel(w2, q.YmX, q.T2d, c.role);
  uint32_t* s = c.qs + c.role * 20 * 32;
#pragma unroll
  for (int k = 0; k < 10; k++) {
    s[k * 32] = w1.v[k];
    s[(10 + k) * 32] = w2.v[k];
  }
  __syncthreads();
}

// r = p +/- Q, Q the pair's cached addend (ge_add_lds); `neg` wave-uniform.
DKG_DEV void ge_add_pair(ge_p3& r, const ge_p3& p, const pair_ctx& c, bool neg) {
  fe o1, o2;
  {
    // role 0: A = (Y1 - X1) * (neg ? Y2+X2 : Y2-X2), C = T1 * 2dT2
    // role 1: B = (Y1 + X1) * (neg ? Y2-X2 : Y2+X2), D = Z1 * 2Z2
    fe ym, yp, in1, in2, q1, q2;
    fe_sub(ym, p.Y, p.X);
    fe_add(yp, p.Y, p.X);
    fe_sel(in1, ym, yp, c.role);
    fe_sel(in2, p.T, p.Z, c.role);
    const int f1 = c.role ? (neg ? 1 : 0) : (neg ? 0 : 1);  // field: 0 Y+X, 1 Y-X, 2 2Z, 3 2dT
    const int f2 = c.role ? 2 : 3;
    const uint32_t* s1 = c.qs + f1 * 10 * 32;
    const uint32_t* s2 = c.qs + f2 * 10 * 32;
#pragma unroll
    for (int k = 0; k < 10; k++) {
      q1.v[k] = s1[k * 32];
      q2.v[k] = s2[k * 32];
    }
    fe_mul(o1, in1, q1);
    fe_mul(o2, in2, q2);
  }
  fe a, cc, b, d;
  pair_xchg(c, o1, o2, a, cc, b, d);
  fe e, h, f, g;
  fe_sub(e, b, a);                   // <= 1.5*2^27
  fe_add(h, b, a);                   // <= 2^27
  if (neg) fe_neg(cc, cc);           // 2p - c <= 2p limbwise: a valid fe_sub subtrahend
  fe_sub(f, d, cc);                  // f
  fe_add(g, d, cc);                  // g
  fe n;
  fe_sel(n, f, h, c.role);
  fe_mul(o1, e, n);                  // role 0: X3 = e f, role 1: T3 = e h
  fe_mul(o2, g, n);                  // role 0: Z3 = g f, role 1: Y3 = g h
  pair_xchg(c, o1, o2, r.X, r.Z, r.T, r.Y);
}

// y = m y for a wave-uniform small m (mul_small_lds's NAF chain, with the pair operations)
DKG_DEV void mul_small_pair(ge_p3& y, uint32_t m, const pair_ctx& c) {
  uint32_t pos, neg;
  const int len = small_recode(m, pos, neg);
  if (len <= 1) return;
  pair_put_cached(c, y);
#pragma unroll 1
  for (int i = len - 2; i >= 0; i--) {
    const uint32_t bit = 1u << i;
    ge_dbl_pair(y, y, c);
    if ((pos | neg) & bit) ge_add_pair(y, y, c, (neg & bit) != 0);
  }
}
