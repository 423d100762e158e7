// GF(2^255-19) arithmetic for gfx950 in 32-bit VALU ops.
//
// Representation: ten unsigned 32-bit limbs in radix 2^25.5 (limb i holds 26 bits for even i,
// 25 bits for odd i; bit offsets 0,26,51,77,102,128,153,179,204,230).  A product limb pair is
// one v_mad_u64_u32 (32x32 -> 64 plus a 64-bit addend), so a field multiply is 100 MADs + 9 x19
// pre-multiplies + the carries (a square is 55 MADs).  The pseudo-Mersenne fold 2^255 = 19 is
// applied inside the product (no Montgomery form).  Two flavours of the multiply, fixed per
// translation unit: product scanning (default; fewest issue slots) and column sums (DKG_FE_ILP;
// ten independent chains, for latency-bound launches) -- see fe_mul below and DESIGN.md section 5.
//
// Bounds (machine-checked: tools/fe_bounds.py propagates worst-case limb bounds through both
// flavours of every primitive and every formula of ge25519.h / points.h as written, and
// tests/test_bounds.py runs it).  TIGHT = every fe_mul / fe_sq / fe_carry output and every stored
// point coordinate: limbs below 2^26 + 2^6 (even) / 2^25 + 2^12 (odd).  fe_mul(f, g) is
// overflow-free for uniform limb bounds up to (f, g) = (2^28, 2^27.75), (2^28.32, 2^27.585) or
// (2^29, 2^26) -- g carries the x19 fold (19 g < 2^32), f the x2 weight, and every 64-bit column
// sum stays below 2^64.  The formulas hand it at most f = (h - t) + 2p <= 2^28 (doubling) and
// g = (d - c) + 2p <= 1.5 * 2^27 = 2^27.585 (additions) or 2p - xy2d <= 2^27 (comb entries).
// fe_sub(a, b) = a + 2p - b needs b <= 2p limbwise (a TIGHT b always is); anything looser goes
// through fe_carry first.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define DKG_DEV __device__ __forceinline__

struct fe {
  uint32_t v[10];
};

namespace fe_const {
// 2*p in radix 2^25.5 (limbwise), the bias added by fe_sub.
constexpr uint32_t P2_0 = 0x7ffffdau;  // 2*(2^26 - 19)
constexpr uint32_t P2_E = 0x7fffffeu;  // 2*(2^26 - 1)
constexpr uint32_t P2_O = 0x3fffffeu;  // 2*(2^25 - 1)
}  // namespace fe_const

DKG_DEV void fe_set(fe& r, const uint32_t (&c)[10]) {
#pragma unroll
  for (int i = 0; i < 10; i++) r.v[i] = c[i];
}
DKG_DEV void fe_zero(fe& r) {
#pragma unroll
  for (int i = 0; i < 10; i++) r.v[i] = 0;
}
DKG_DEV void fe_one(fe& r) {
  fe_zero(r);
  r.v[0] = 1;
}
DKG_DEV void fe_copy(fe& r, const fe& a) {
#pragma unroll
  for (int i = 0; i < 10; i++) r.v[i] = a.v[i];
}
DKG_DEV void fe_add(fe& r, const fe& a, const fe& b) {
#pragma unroll
  for (int i = 0; i < 10; i++) r.v[i] = a.v[i] + b.v[i];
}
// r = a - b + 2p  (b must be tight)
DKG_DEV void fe_sub(fe& r, const fe& a, const fe& b) {
  r.v[0] = a.v[0] + fe_const::P2_0 - b.v[0];
#pragma unroll
  for (int i = 1; i < 10; i++) r.v[i] = a.v[i] + ((i & 1) ? fe_const::P2_O : fe_const::P2_E) - b.v[i];
}
// r = 2p - a  (a tight)
DKG_DEV void fe_neg(fe& r, const fe& a) {
  r.v[0] = fe_const::P2_0 - a.v[0];
#pragma unroll
  for (int i = 1; i < 10; i++) r.v[i] = ((i & 1) ? fe_const::P2_O : fe_const::P2_E) - a.v[i];
}

// One parallel carry pass on 32-bit limbs: output limbs <= 2^26/2^25 + 2^7 (tight).
DKG_DEV void fe_carry(fe& r, const fe& a) {
  uint32_t c[10];
#pragma unroll
  for (int i = 0; i < 10; i++) c[i] = a.v[i] >> ((i & 1) ? 25 : 26);
  r.v[0] = (a.v[0] & 0x3ffffffu) + 19u * c[9];
#pragma unroll
  for (int i = 1; i < 10; i++) r.v[i] = (a.v[i] & ((i & 1) ? 0x1ffffffu : 0x3ffffffu)) + c[i - 1];
}

DKG_DEV uint64_t mul32(uint32_t a, uint32_t b) { return (uint64_t)a * (uint64_t)b; }

// 2x as a full-rate v_add_u32: the compiler turns x + x into v_lshlrev_b32, which issues at half
// rate on gfx950 like every shift (profiles/r02_ubench_intrate3.txt); non-volatile, so it CSEs.
DKG_DEV uint32_t dbl32(uint32_t x) {
  uint32_t r;
  asm("v_add_u32 %0, %1, %1" : "=v"(r) : "v"(x));
  return r;
}
// r = 2a limb by limb with dbl32 (fe_add(r, a, a) compiles to half-rate shifts)
DKG_DEV void fe_dbl(fe& r, const fe& a) {
#pragma unroll
  for (int i = 0; i < 10; i++) r.v[i] = dbl32(a.v[i]);
}

// One v_mad_u64_u32 (h = a * b + h) the compiler cannot reassociate.  The products are summed
// column by column ("product scanning") and each column's chain STARTS from the carry out of the
// previous column, so the carry costs no separate 64-bit add: per column one v_and (full rate) and
// one v_lshrrev_b64 (half rate) besides the ten half-rate mads (profiles/r02_ubench_intrate3.txt:
// shifts and 64-bit adds issue at half rate on gfx950, only add/sub/and/or at full rate).  The
// serial chain costs few issue slots: a wave issues a mad only every ~9.5 cycles anyway
// (tools/ubench/ilp.hip) and the SIMD interleaves the resident waves; the s_nop the compiler puts
// before every mad that reads its own accumulator is mostly hidden by the other waves (the pair
// products below recover part of it).  The carry-out SGPR pair is unused.
DKG_DEV void mad_acc(uint64_t& h, uint32_t a, uint32_t b) {
  uint64_t cc;
  asm("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(h), "=s"(cc) : "v"(a), "v"(b));
}
DKG_DEV uint64_t mad_first(uint32_t a, uint32_t b) {
  uint64_t h, cc;
  asm("v_mad_u64_u32 %0, %1, %2, %3, 0" : "=v"(h), "=s"(cc) : "v"(a), "v"(b));
  return h;
}
// The same for the pair products: volatile, so the two chains stay interleaved as written (the
// compiler would otherwise regroup each chain's mads back to back), and each chain with its own
// carry-out SGPR pair `cc` (read-write, so the two stay distinct registers).  The hazard recogniser
// puts one s_nop before each mad that reads its own chain's accumulator, at any distance, and one
// between back-to-back writes of one SGPR pair: K interleaved chains with K pairs need one s_nop per
// K mads (two chains: the stepping loop's 731 -> 356; profiles/r06_pair_ab.txt).
DKG_DEV void mad_acc_v(uint64_t& h, uint32_t a, uint32_t b, uint64_t& cc) {
  asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(h), "+s"(cc) : "v"(a), "v"(b));
}
DKG_DEV uint64_t mad_first_v(uint32_t a, uint32_t b, uint64_t& cc) {
  uint64_t h;
  asm volatile("v_mad_u64_u32 %0, %1, %2, %3, 0" : "=v"(h), "+s"(cc) : "v"(a), "v"(b));
  return h;
}
// limb k of the result from the column in h, carry left in h
#define FE_LIMB(r, k, h)                                             \
  r.v[k] = (uint32_t)h & ((k) & 1 ? 0x1ffffffu : 0x3ffffffu);        \
  h >>= ((k) & 1 ? 25 : 26);
// fold of the carry out of limb 9 (< 2^38): 19 h into limb 0, its carry into limb 1
#define FE_FOLD(r, h)                                                \
  {                                                                  \
    uint64_t t_ = (uint64_t)r.v[0];                                  \
    mad_acc(t_, (uint32_t)h, 19u);                                   \
    t_ += (uint64_t)(19u * (uint32_t)(h >> 32)) << 32;               \
    r.v[0] = (uint32_t)t_ & 0x3ffffffu;                              \
    r.v[1] += (uint32_t)(t_ >> 26);                                  \
  }

DKG_DEV void fe_mul_ps(fe& r, const fe& f, const fe& g) {
  const uint32_t f0 = f.v[0], f1 = f.v[1], f2 = f.v[2], f3 = f.v[3], f4 = f.v[4];
  const uint32_t f5 = f.v[5], f6 = f.v[6], f7 = f.v[7], f8 = f.v[8], f9 = f.v[9];
  const uint32_t g0 = g.v[0], g1 = g.v[1], g2 = g.v[2], g3 = g.v[3], g4 = g.v[4];
  const uint32_t g5 = g.v[5], g6 = g.v[6], g7 = g.v[7], g8 = g.v[8], g9 = g.v[9];
  const uint32_t g1_19 = 19u * g1, g2_19 = 19u * g2, g3_19 = 19u * g3, g4_19 = 19u * g4;
  const uint32_t g5_19 = 19u * g5, g6_19 = 19u * g6, g7_19 = 19u * g7, g8_19 = 19u * g8;
  const uint32_t g9_19 = 19u * g9;
  const uint32_t f1_2 = dbl32(f1), f3_2 = dbl32(f3), f5_2 = dbl32(f5), f7_2 = dbl32(f7), f9_2 = dbl32(f9);
  // column k: sum of f_i g_j over i + j = k, and 19 f_i g_j over i + j = k + 10; odd x odd doubled
  uint64_t h = mad_first(f0, g0);
  mad_acc(h, f1_2, g9_19); mad_acc(h, f2, g8_19); mad_acc(h, f3_2, g7_19); mad_acc(h, f4, g6_19);
  mad_acc(h, f5_2, g5_19); mad_acc(h, f6, g4_19); mad_acc(h, f7_2, g3_19); mad_acc(h, f8, g2_19);
  mad_acc(h, f9_2, g1_19);
  FE_LIMB(r, 0, h)
  mad_acc(h, f0, g1); mad_acc(h, f1, g0); mad_acc(h, f2, g9_19); mad_acc(h, f3, g8_19); mad_acc(h, f4, g7_19);
  mad_acc(h, f5, g6_19); mad_acc(h, f6, g5_19); mad_acc(h, f7, g4_19); mad_acc(h, f8, g3_19); mad_acc(h, f9, g2_19);
  FE_LIMB(r, 1, h)
  mad_acc(h, f0, g2); mad_acc(h, f1_2, g1); mad_acc(h, f2, g0); mad_acc(h, f3_2, g9_19); mad_acc(h, f4, g8_19);
  mad_acc(h, f5_2, g7_19); mad_acc(h, f6, g6_19); mad_acc(h, f7_2, g5_19); mad_acc(h, f8, g4_19);
  mad_acc(h, f9_2, g3_19);
  FE_LIMB(r, 2, h)
  mad_acc(h, f0, g3); mad_acc(h, f1, g2); mad_acc(h, f2, g1); mad_acc(h, f3, g0); mad_acc(h, f4, g9_19);
  mad_acc(h, f5, g8_19); mad_acc(h, f6, g7_19); mad_acc(h, f7, g6_19); mad_acc(h, f8, g5_19); mad_acc(h, f9, g4_19);
  FE_LIMB(r, 3, h)
  mad_acc(h, f0, g4); mad_acc(h, f1_2, g3); mad_acc(h, f2, g2); mad_acc(h, f3_2, g1); mad_acc(h, f4, g0);
  mad_acc(h, f5_2, g9_19); mad_acc(h, f6, g8_19); mad_acc(h, f7_2, g7_19); mad_acc(h, f8, g6_19);
  mad_acc(h, f9_2, g5_19);
  FE_LIMB(r, 4, h)
  mad_acc(h, f0, g5); mad_acc(h, f1, g4); mad_acc(h, f2, g3); mad_acc(h, f3, g2); mad_acc(h, f4, g1);
  mad_acc(h, f5, g0); mad_acc(h, f6, g9_19); mad_acc(h, f7, g8_19); mad_acc(h, f8, g7_19); mad_acc(h, f9, g6_19);
  FE_LIMB(r, 5, h)
  mad_acc(h, f0, g6); mad_acc(h, f1_2, g5); mad_acc(h, f2, g4); mad_acc(h, f3_2, g3); mad_acc(h, f4, g2);
  mad_acc(h, f5_2, g1); mad_acc(h, f6, g0); mad_acc(h, f7_2, g9_19); mad_acc(h, f8, g8_19);
  mad_acc(h, f9_2, g7_19);
  FE_LIMB(r, 6, h)
  mad_acc(h, f0, g7); mad_acc(h, f1, g6); mad_acc(h, f2, g5); mad_acc(h, f3, g4); mad_acc(h, f4, g3);
  mad_acc(h, f5, g2); mad_acc(h, f6, g1); mad_acc(h, f7, g0); mad_acc(h, f8, g9_19); mad_acc(h, f9, g8_19);
  FE_LIMB(r, 7, h)
  mad_acc(h, f0, g8); mad_acc(h, f1_2, g7); mad_acc(h, f2, g6); mad_acc(h, f3_2, g5); mad_acc(h, f4, g4);
  mad_acc(h, f5_2, g3); mad_acc(h, f6, g2); mad_acc(h, f7_2, g1); mad_acc(h, f8, g0); mad_acc(h, f9_2, g9_19);
  FE_LIMB(r, 8, h)
  mad_acc(h, f0, g9); mad_acc(h, f1, g8); mad_acc(h, f2, g7); mad_acc(h, f3, g6); mad_acc(h, f4, g5);
  mad_acc(h, f5, g4); mad_acc(h, f6, g3); mad_acc(h, f7, g2); mad_acc(h, f8, g1); mad_acc(h, f9, g0);
  FE_LIMB(r, 9, h)
  FE_FOLD(r, h)
}

DKG_DEV void fe_sq_ps(fe& r, const fe& f) {
  // Symmetric products counted once; x19 factors kept on limbs 5..9 (19 * 2^27.585 < 2^32) and
  // the extra 2 / 4 weights moved onto the partner limb so every operand fits in 32 bits.
  const uint32_t f0 = f.v[0], f1 = f.v[1], f2 = f.v[2], f3 = f.v[3], f4 = f.v[4];
  const uint32_t f5 = f.v[5], f6 = f.v[6], f7 = f.v[7], f8 = f.v[8], f9 = f.v[9];
  const uint32_t f0_2 = dbl32(f0), f1_2 = dbl32(f1), f2_2 = dbl32(f2), f3_2 = dbl32(f3), f4_2 = dbl32(f4);
  const uint32_t f5_2 = dbl32(f5), f6_2 = dbl32(f6), f7_2 = dbl32(f7), f8_2 = dbl32(f8), f9_2 = dbl32(f9);
  const uint32_t f1_4 = dbl32(f1_2), f3_4 = dbl32(f3_2), f5_4 = dbl32(f5_2), f7_4 = dbl32(f7_2);
  const uint32_t f5_19 = 19u * f5, f6_19 = 19u * f6, f7_19 = 19u * f7, f8_19 = 19u * f8;
  const uint32_t f9_19 = 19u * f9;
  uint64_t h = mad_first(f0, f0);
  mad_acc(h, f1_4, f9_19); mad_acc(h, f2_2, f8_19); mad_acc(h, f3_4, f7_19); mad_acc(h, f4_2, f6_19);
  mad_acc(h, f5_2, f5_19);
  FE_LIMB(r, 0, h)
  mad_acc(h, f0_2, f1); mad_acc(h, f2_2, f9_19); mad_acc(h, f3_2, f8_19); mad_acc(h, f4_2, f7_19);
  mad_acc(h, f5_2, f6_19);
  FE_LIMB(r, 1, h)
  mad_acc(h, f0_2, f2); mad_acc(h, f1_2, f1); mad_acc(h, f3_4, f9_19); mad_acc(h, f4_2, f8_19);
  mad_acc(h, f5_4, f7_19); mad_acc(h, f6, f6_19);
  FE_LIMB(r, 2, h)
  mad_acc(h, f0_2, f3); mad_acc(h, f1_2, f2); mad_acc(h, f4_2, f9_19); mad_acc(h, f5_2, f8_19);
  mad_acc(h, f6_2, f7_19);
  FE_LIMB(r, 3, h)
  mad_acc(h, f0_2, f4); mad_acc(h, f1_2, f3_2); mad_acc(h, f2, f2); mad_acc(h, f5_4, f9_19);
  mad_acc(h, f6_2, f8_19); mad_acc(h, f7_2, f7_19);
  FE_LIMB(r, 4, h)
  mad_acc(h, f0_2, f5); mad_acc(h, f1_2, f4); mad_acc(h, f2_2, f3); mad_acc(h, f6_2, f9_19);
  mad_acc(h, f7_2, f8_19);
  FE_LIMB(r, 5, h)
  mad_acc(h, f0_2, f6); mad_acc(h, f1_2, f5_2); mad_acc(h, f2_2, f4); mad_acc(h, f3_2, f3);
  mad_acc(h, f7_4, f9_19); mad_acc(h, f8, f8_19);
  FE_LIMB(r, 6, h)
  mad_acc(h, f0_2, f7); mad_acc(h, f1_2, f6); mad_acc(h, f2_2, f5); mad_acc(h, f3_2, f4);
  mad_acc(h, f8_2, f9_19);
  FE_LIMB(r, 7, h)
  mad_acc(h, f0_2, f8); mad_acc(h, f1_2, f7_2); mad_acc(h, f2_2, f6); mad_acc(h, f3_2, f5_2);
  mad_acc(h, f4, f4); mad_acc(h, f9_2, f9_19);
  FE_LIMB(r, 8, h)
  mad_acc(h, f0_2, f9); mad_acc(h, f1_2, f8); mad_acc(h, f2_2, f7); mad_acc(h, f3_2, f6);
  mad_acc(h, f4_2, f5);
  FE_LIMB(r, 9, h)
  FE_FOLD(r, h)
}

// ---- BEGIN generated pair products (tools/gen_fe_pair.py)
// Two independent products in one instruction stream (pair versions of fe_mul_ps / fe_sq_ps):
// statement by statement interleaved, so consecutive v_mad_u64_u32 belong to different chains and
// need no hazard wait state between them (the single chain puts an s_nop 0 between its back-to-back
// mads).  All inputs are read before the first output limb is written: outputs may alias inputs.
// Generated from the single versions (tools/gen_fe_pair.py); the same terms in the same order.
DKG_DEV void fe_mul_ps2(fe& ra, const fe& fa, const fe& ga, fe& rb, const fe& fb, const fe& gb) {
  uint64_t cc_a = 0, cc_b = 0;  // carry-out pairs, one per chain
  const uint32_t f0_a = fa.v[0], f1_a = fa.v[1], f2_a = fa.v[2], f3_a = fa.v[3], f4_a = fa.v[4];
  const uint32_t f0_b = fb.v[0], f1_b = fb.v[1], f2_b = fb.v[2], f3_b = fb.v[3], f4_b = fb.v[4];
  const uint32_t f5_a = fa.v[5], f6_a = fa.v[6], f7_a = fa.v[7], f8_a = fa.v[8], f9_a = fa.v[9];
  const uint32_t f5_b = fb.v[5], f6_b = fb.v[6], f7_b = fb.v[7], f8_b = fb.v[8], f9_b = fb.v[9];
  const uint32_t g0_a = ga.v[0], g1_a = ga.v[1], g2_a = ga.v[2], g3_a = ga.v[3], g4_a = ga.v[4];
  const uint32_t g0_b = gb.v[0], g1_b = gb.v[1], g2_b = gb.v[2], g3_b = gb.v[3], g4_b = gb.v[4];
  const uint32_t g5_a = ga.v[5], g6_a = ga.v[6], g7_a = ga.v[7], g8_a = ga.v[8], g9_a = ga.v[9];
  const uint32_t g5_b = gb.v[5], g6_b = gb.v[6], g7_b = gb.v[7], g8_b = gb.v[8], g9_b = gb.v[9];
  const uint32_t g1_19_a = 19u * g1_a, g2_19_a = 19u * g2_a, g3_19_a = 19u * g3_a, g4_19_a = 19u * g4_a;
  const uint32_t g1_19_b = 19u * g1_b, g2_19_b = 19u * g2_b, g3_19_b = 19u * g3_b, g4_19_b = 19u * g4_b;
  const uint32_t g5_19_a = 19u * g5_a, g6_19_a = 19u * g6_a, g7_19_a = 19u * g7_a, g8_19_a = 19u * g8_a;
  const uint32_t g5_19_b = 19u * g5_b, g6_19_b = 19u * g6_b, g7_19_b = 19u * g7_b, g8_19_b = 19u * g8_b;
  const uint32_t g9_19_a = 19u * g9_a;
  const uint32_t g9_19_b = 19u * g9_b;
  const uint32_t f1_2_a = dbl32(f1_a), f3_2_a = dbl32(f3_a), f5_2_a = dbl32(f5_a), f7_2_a = dbl32(f7_a), f9_2_a = dbl32(f9_a);
  const uint32_t f1_2_b = dbl32(f1_b), f3_2_b = dbl32(f3_b), f5_2_b = dbl32(f5_b), f7_2_b = dbl32(f7_b), f9_2_b = dbl32(f9_b);
  uint64_t h_a = mad_first_v(f0_a, g0_a, cc_a);
  uint64_t h_b = mad_first_v(f0_b, g0_b, cc_b);
  mad_acc_v(h_a, f1_2_a, g9_19_a, cc_a);
  mad_acc_v(h_b, f1_2_b, g9_19_b, cc_b);
  mad_acc_v(h_a, f2_a, g8_19_a, cc_a);
  mad_acc_v(h_b, f2_b, g8_19_b, cc_b);
  mad_acc_v(h_a, f3_2_a, g7_19_a, cc_a);
  mad_acc_v(h_b, f3_2_b, g7_19_b, cc_b);
  mad_acc_v(h_a, f4_a, g6_19_a, cc_a);
  mad_acc_v(h_b, f4_b, g6_19_b, cc_b);
  mad_acc_v(h_a, f5_2_a, g5_19_a, cc_a);
  mad_acc_v(h_b, f5_2_b, g5_19_b, cc_b);
  mad_acc_v(h_a, f6_a, g4_19_a, cc_a);
  mad_acc_v(h_b, f6_b, g4_19_b, cc_b);
  mad_acc_v(h_a, f7_2_a, g3_19_a, cc_a);
  mad_acc_v(h_b, f7_2_b, g3_19_b, cc_b);
  mad_acc_v(h_a, f8_a, g2_19_a, cc_a);
  mad_acc_v(h_b, f8_b, g2_19_b, cc_b);
  mad_acc_v(h_a, f9_2_a, g1_19_a, cc_a);
  mad_acc_v(h_b, f9_2_b, g1_19_b, cc_b);
  FE_LIMB(ra, 0, h_a)
  FE_LIMB(rb, 0, h_b)
  mad_acc_v(h_a, f0_a, g1_a, cc_a);
  mad_acc_v(h_b, f0_b, g1_b, cc_b);
  mad_acc_v(h_a, f1_a, g0_a, cc_a);
  mad_acc_v(h_b, f1_b, g0_b, cc_b);
  mad_acc_v(h_a, f2_a, g9_19_a, cc_a);
  mad_acc_v(h_b, f2_b, g9_19_b, cc_b);
  mad_acc_v(h_a, f3_a, g8_19_a, cc_a);
  mad_acc_v(h_b, f3_b, g8_19_b, cc_b);
  mad_acc_v(h_a, f4_a, g7_19_a, cc_a);
  mad_acc_v(h_b, f4_b, g7_19_b, cc_b);
  mad_acc_v(h_a, f5_a, g6_19_a, cc_a);
  mad_acc_v(h_b, f5_b, g6_19_b, cc_b);
  mad_acc_v(h_a, f6_a, g5_19_a, cc_a);
  mad_acc_v(h_b, f6_b, g5_19_b, cc_b);
  mad_acc_v(h_a, f7_a, g4_19_a, cc_a);
  mad_acc_v(h_b, f7_b, g4_19_b, cc_b);
  mad_acc_v(h_a, f8_a, g3_19_a, cc_a);
  mad_acc_v(h_b, f8_b, g3_19_b, cc_b);
  mad_acc_v(h_a, f9_a, g2_19_a, cc_a);
  mad_acc_v(h_b, f9_b, g2_19_b, cc_b);
  FE_LIMB(ra, 1, h_a)
  FE_LIMB(rb, 1, h_b)
  mad_acc_v(h_a, f0_a, g2_a, cc_a);
  mad_acc_v(h_b, f0_b, g2_b, cc_b);
  mad_acc_v(h_a, f1_2_a, g1_a, cc_a);
  mad_acc_v(h_b, f1_2_b, g1_b, cc_b);
  mad_acc_v(h_a, f2_a, g0_a, cc_a);
  mad_acc_v(h_b, f2_b, g0_b, cc_b);
  mad_acc_v(h_a, f3_2_a, g9_19_a, cc_a);
  mad_acc_v(h_b, f3_2_b, g9_19_b, cc_b);
  mad_acc_v(h_a, f4_a, g8_19_a, cc_a);
  mad_acc_v(h_b, f4_b, g8_19_b, cc_b);
  mad_acc_v(h_a, f5_2_a, g7_19_a, cc_a);
  mad_acc_v(h_b, f5_2_b, g7_19_b, cc_b);
  mad_acc_v(h_a, f6_a, g6_19_a, cc_a);
  mad_acc_v(h_b, f6_b, g6_19_b, cc_b);
  mad_acc_v(h_a, f7_2_a, g5_19_a, cc_a);
  mad_acc_v(h_b, f7_2_b, g5_19_b, cc_b);
  mad_acc_v(h_a, f8_a, g4_19_a, cc_a);
  mad_acc_v(h_b, f8_b, g4_19_b, cc_b);
  mad_acc_v(h_a, f9_2_a, g3_19_a, cc_a);
  mad_acc_v(h_b, f9_2_b, g3_19_b, cc_b);
  FE_LIMB(ra, 2, h_a)
  FE_LIMB(rb, 2, h_b)
  mad_acc_v(h_a, f0_a, g3_a, cc_a);
  mad_acc_v(h_b, f0_b, g3_b, cc_b);
  mad_acc_v(h_a, f1_a, g2_a, cc_a);
  mad_acc_v(h_b, f1_b, g2_b, cc_b);
  mad_acc_v(h_a, f2_a, g1_a, cc_a);
  mad_acc_v(h_b, f2_b, g1_b, cc_b);
  mad_acc_v(h_a, f3_a, g0_a, cc_a);
  mad_acc_v(h_b, f3_b, g0_b, cc_b);
  mad_acc_v(h_a, f4_a, g9_19_a, cc_a);
  mad_acc_v(h_b, f4_b, g9_19_b, cc_b);
  mad_acc_v(h_a, f5_a, g8_19_a, cc_a);
  mad_acc_v(h_b, f5_b, g8_19_b, cc_b);
  mad_acc_v(h_a, f6_a, g7_19_a, cc_a);
  mad_acc_v(h_b, f6_b, g7_19_b, cc_b);
  mad_acc_v(h_a, f7_a, g6_19_a, cc_a);
  mad_acc_v(h_b, f7_b, g6_19_b, cc_b);
  mad_acc_v(h_a, f8_a, g5_19_a, cc_a);
  mad_acc_v(h_b, f8_b, g5_19_b, cc_b);
  mad_acc_v(h_a, f9_a, g4_19_a, cc_a);
  mad_acc_v(h_b, f9_b, g4_19_b, cc_b);
  FE_LIMB(ra, 3, h_a)
  FE_LIMB(rb, 3, h_b)
  mad_acc_v(h_a, f0_a, g4_a, cc_a);
  mad_acc_v(h_b, f0_b, g4_b, cc_b);
  mad_acc_v(h_a, f1_2_a, g3_a, cc_a);
  mad_acc_v(h_b, f1_2_b, g3_b, cc_b);
  mad_acc_v(h_a, f2_a, g2_a, cc_a);
  mad_acc_v(h_b, f2_b, g2_b, cc_b);
  mad_acc_v(h_a, f3_2_a, g1_a, cc_a);
  mad_acc_v(h_b, f3_2_b, g1_b, cc_b);
  mad_acc_v(h_a, f4_a, g0_a, cc_a);
  mad_acc_v(h_b, f4_b, g0_b, cc_b);
  mad_acc_v(h_a, f5_2_a, g9_19_a, cc_a);
  mad_acc_v(h_b, f5_2_b, g9_19_b, cc_b);
  mad_acc_v(h_a, f6_a, g8_19_a, cc_a);
  mad_acc_v(h_b, f6_b, g8_19_b, cc_b);
  mad_acc_v(h_a, f7_2_a, g7_19_a, cc_a);
  mad_acc_v(h_b, f7_2_b, g7_19_b, cc_b);
  mad_acc_v(h_a, f8_a, g6_19_a, cc_a);
  mad_acc_v(h_b, f8_b, g6_19_b, cc_b);
  mad_acc_v(h_a, f9_2_a, g5_19_a, cc_a);
  mad_acc_v(h_b, f9_2_b, g5_19_b, cc_b);
  FE_LIMB(ra, 4, h_a)
  FE_LIMB(rb, 4, h_b)
  mad_acc_v(h_a, f0_a, g5_a, cc_a);
  mad_acc_v(h_b, f0_b, g5_b, cc_b);
  mad_acc_v(h_a, f1_a, g4_a, cc_a);
  mad_acc_v(h_b, f1_b, g4_b, cc_b);
  mad_acc_v(h_a, f2_a, g3_a, cc_a);
  mad_acc_v(h_b, f2_b, g3_b, cc_b);
  mad_acc_v(h_a, f3_a, g2_a, cc_a);
  mad_acc_v(h_b, f3_b, g2_b, cc_b);
  mad_acc_v(h_a, f4_a, g1_a, cc_a);
  mad_acc_v(h_b, f4_b, g1_b, cc_b);
  mad_acc_v(h_a, f5_a, g0_a, cc_a);
  mad_acc_v(h_b, f5_b, g0_b, cc_b);
  mad_acc_v(h_a, f6_a, g9_19_a, cc_a);
  mad_acc_v(h_b, f6_b, g9_19_b, cc_b);
  mad_acc_v(h_a, f7_a, g8_19_a, cc_a);
  mad_acc_v(h_b, f7_b, g8_19_b, cc_b);
  mad_acc_v(h_a, f8_a, g7_19_a, cc_a);
  mad_acc_v(h_b, f8_b, g7_19_b, cc_b);
  mad_acc_v(h_a, f9_a, g6_19_a, cc_a);
  mad_acc_v(h_b, f9_b, g6_19_b, cc_b);
  FE_LIMB(ra, 5, h_a)
  FE_LIMB(rb, 5, h_b)
  mad_acc_v(h_a, f0_a, g6_a, cc_a);
  mad_acc_v(h_b, f0_b, g6_b, cc_b);
  mad_acc_v(h_a, f1_2_a, g5_a, cc_a);
  mad_acc_v(h_b, f1_2_b, g5_b, cc_b);
  mad_acc_v(h_a, f2_a, g4_a, cc_a);
  mad_acc_v(h_b, f2_b, g4_b, cc_b);
  mad_acc_v(h_a, f3_2_a, g3_a, cc_a);
  mad_acc_v(h_b, f3_2_b, g3_b, cc_b);
  mad_acc_v(h_a, f4_a, g2_a, cc_a);
  mad_acc_v(h_b, f4_b, g2_b, cc_b);
  mad_acc_v(h_a, f5_2_a, g1_a, cc_a);
  mad_acc_v(h_b, f5_2_b, g1_b, cc_b);
  mad_acc_v(h_a, f6_a, g0_a, cc_a);
  mad_acc_v(h_b, f6_b, g0_b, cc_b);
  mad_acc_v(h_a, f7_2_a, g9_19_a, cc_a);
  mad_acc_v(h_b, f7_2_b, g9_19_b, cc_b);
  mad_acc_v(h_a, f8_a, g8_19_a, cc_a);
  mad_acc_v(h_b, f8_b, g8_19_b, cc_b);
  mad_acc_v(h_a, f9_2_a, g7_19_a, cc_a);
  mad_acc_v(h_b, f9_2_b, g7_19_b, cc_b);
  FE_LIMB(ra, 6, h_a)
  FE_LIMB(rb, 6, h_b)
  mad_acc_v(h_a, f0_a, g7_a, cc_a);
  mad_acc_v(h_b, f0_b, g7_b, cc_b);
  mad_acc_v(h_a, f1_a, g6_a, cc_a);
  mad_acc_v(h_b, f1_b, g6_b, cc_b);
  mad_acc_v(h_a, f2_a, g5_a, cc_a);
  mad_acc_v(h_b, f2_b, g5_b, cc_b);
  mad_acc_v(h_a, f3_a, g4_a, cc_a);
  mad_acc_v(h_b, f3_b, g4_b, cc_b);
  mad_acc_v(h_a, f4_a, g3_a, cc_a);
  mad_acc_v(h_b, f4_b, g3_b, cc_b);
  mad_acc_v(h_a, f5_a, g2_a, cc_a);
  mad_acc_v(h_b, f5_b, g2_b, cc_b);
  mad_acc_v(h_a, f6_a, g1_a, cc_a);
  mad_acc_v(h_b, f6_b, g1_b, cc_b);
  mad_acc_v(h_a, f7_a, g0_a, cc_a);
  mad_acc_v(h_b, f7_b, g0_b, cc_b);
  mad_acc_v(h_a, f8_a, g9_19_a, cc_a);
  mad_acc_v(h_b, f8_b, g9_19_b, cc_b);
  mad_acc_v(h_a, f9_a, g8_19_a, cc_a);
  mad_acc_v(h_b, f9_b, g8_19_b, cc_b);
  FE_LIMB(ra, 7, h_a)
  FE_LIMB(rb, 7, h_b)
  mad_acc_v(h_a, f0_a, g8_a, cc_a);
  mad_acc_v(h_b, f0_b, g8_b, cc_b);
  mad_acc_v(h_a, f1_2_a, g7_a, cc_a);
  mad_acc_v(h_b, f1_2_b, g7_b, cc_b);
  mad_acc_v(h_a, f2_a, g6_a, cc_a);
  mad_acc_v(h_b, f2_b, g6_b, cc_b);
  mad_acc_v(h_a, f3_2_a, g5_a, cc_a);
  mad_acc_v(h_b, f3_2_b, g5_b, cc_b);
  mad_acc_v(h_a, f4_a, g4_a, cc_a);
  mad_acc_v(h_b, f4_b, g4_b, cc_b);
  mad_acc_v(h_a, f5_2_a, g3_a, cc_a);
  mad_acc_v(h_b, f5_2_b, g3_b, cc_b);
  mad_acc_v(h_a, f6_a, g2_a, cc_a);
  mad_acc_v(h_b, f6_b, g2_b, cc_b);
  mad_acc_v(h_a, f7_2_a, g1_a, cc_a);
  mad_acc_v(h_b, f7_2_b, g1_b, cc_b);
  mad_acc_v(h_a, f8_a, g0_a, cc_a);
  mad_acc_v(h_b, f8_b, g0_b, cc_b);
  mad_acc_v(h_a, f9_2_a, g9_19_a, cc_a);
  mad_acc_v(h_b, f9_2_b, g9_19_b, cc_b);
  FE_LIMB(ra, 8, h_a)
  FE_LIMB(rb, 8, h_b)
  mad_acc_v(h_a, f0_a, g9_a, cc_a);
  mad_acc_v(h_b, f0_b, g9_b, cc_b);
  mad_acc_v(h_a, f1_a, g8_a, cc_a);
  mad_acc_v(h_b, f1_b, g8_b, cc_b);
  mad_acc_v(h_a, f2_a, g7_a, cc_a);
  mad_acc_v(h_b, f2_b, g7_b, cc_b);
  mad_acc_v(h_a, f3_a, g6_a, cc_a);
  mad_acc_v(h_b, f3_b, g6_b, cc_b);
  mad_acc_v(h_a, f4_a, g5_a, cc_a);
  mad_acc_v(h_b, f4_b, g5_b, cc_b);
  mad_acc_v(h_a, f5_a, g4_a, cc_a);
  mad_acc_v(h_b, f5_b, g4_b, cc_b);
  mad_acc_v(h_a, f6_a, g3_a, cc_a);
  mad_acc_v(h_b, f6_b, g3_b, cc_b);
  mad_acc_v(h_a, f7_a, g2_a, cc_a);
  mad_acc_v(h_b, f7_b, g2_b, cc_b);
  mad_acc_v(h_a, f8_a, g1_a, cc_a);
  mad_acc_v(h_b, f8_b, g1_b, cc_b);
  mad_acc_v(h_a, f9_a, g0_a, cc_a);
  mad_acc_v(h_b, f9_b, g0_b, cc_b);
  FE_LIMB(ra, 9, h_a)
  FE_LIMB(rb, 9, h_b)
  FE_FOLD(ra, h_a)
  FE_FOLD(rb, h_b)
  asm volatile("" : : "s"(cc_a), "s"(cc_b));  // both pairs live to the end: distinct registers
}

DKG_DEV void fe_sq_ps2(fe& ra, const fe& fa, fe& rb, const fe& fb) {
  uint64_t cc_a = 0, cc_b = 0;  // carry-out pairs, one per chain
  const uint32_t f0_a = fa.v[0], f1_a = fa.v[1], f2_a = fa.v[2], f3_a = fa.v[3], f4_a = fa.v[4];
  const uint32_t f0_b = fb.v[0], f1_b = fb.v[1], f2_b = fb.v[2], f3_b = fb.v[3], f4_b = fb.v[4];
  const uint32_t f5_a = fa.v[5], f6_a = fa.v[6], f7_a = fa.v[7], f8_a = fa.v[8], f9_a = fa.v[9];
  const uint32_t f5_b = fb.v[5], f6_b = fb.v[6], f7_b = fb.v[7], f8_b = fb.v[8], f9_b = fb.v[9];
  const uint32_t f0_2_a = dbl32(f0_a), f1_2_a = dbl32(f1_a), f2_2_a = dbl32(f2_a), f3_2_a = dbl32(f3_a), f4_2_a = dbl32(f4_a);
  const uint32_t f0_2_b = dbl32(f0_b), f1_2_b = dbl32(f1_b), f2_2_b = dbl32(f2_b), f3_2_b = dbl32(f3_b), f4_2_b = dbl32(f4_b);
  const uint32_t f5_2_a = dbl32(f5_a), f6_2_a = dbl32(f6_a), f7_2_a = dbl32(f7_a), f8_2_a = dbl32(f8_a), f9_2_a = dbl32(f9_a);
  const uint32_t f5_2_b = dbl32(f5_b), f6_2_b = dbl32(f6_b), f7_2_b = dbl32(f7_b), f8_2_b = dbl32(f8_b), f9_2_b = dbl32(f9_b);
  const uint32_t f1_4_a = dbl32(f1_2_a), f3_4_a = dbl32(f3_2_a), f5_4_a = dbl32(f5_2_a), f7_4_a = dbl32(f7_2_a);
  const uint32_t f1_4_b = dbl32(f1_2_b), f3_4_b = dbl32(f3_2_b), f5_4_b = dbl32(f5_2_b), f7_4_b = dbl32(f7_2_b);
  const uint32_t f5_19_a = 19u * f5_a, f6_19_a = 19u * f6_a, f7_19_a = 19u * f7_a, f8_19_a = 19u * f8_a;
  const uint32_t f5_19_b = 19u * f5_b, f6_19_b = 19u * f6_b, f7_19_b = 19u * f7_b, f8_19_b = 19u * f8_b;
  const uint32_t f9_19_a = 19u * f9_a;
  const uint32_t f9_19_b = 19u * f9_b;
  uint64_t h_a = mad_first_v(f0_a, f0_a, cc_a);
  uint64_t h_b = mad_first_v(f0_b, f0_b, cc_b);
  mad_acc_v(h_a, f1_4_a, f9_19_a, cc_a);
  mad_acc_v(h_b, f1_4_b, f9_19_b, cc_b);
  mad_acc_v(h_a, f2_2_a, f8_19_a, cc_a);
  mad_acc_v(h_b, f2_2_b, f8_19_b, cc_b);
  mad_acc_v(h_a, f3_4_a, f7_19_a, cc_a);
  mad_acc_v(h_b, f3_4_b, f7_19_b, cc_b);
  mad_acc_v(h_a, f4_2_a, f6_19_a, cc_a);
  mad_acc_v(h_b, f4_2_b, f6_19_b, cc_b);
  mad_acc_v(h_a, f5_2_a, f5_19_a, cc_a);
  mad_acc_v(h_b, f5_2_b, f5_19_b, cc_b);
  FE_LIMB(ra, 0, h_a)
  FE_LIMB(rb, 0, h_b)
  mad_acc_v(h_a, f0_2_a, f1_a, cc_a);
  mad_acc_v(h_b, f0_2_b, f1_b, cc_b);
  mad_acc_v(h_a, f2_2_a, f9_19_a, cc_a);
  mad_acc_v(h_b, f2_2_b, f9_19_b, cc_b);
  mad_acc_v(h_a, f3_2_a, f8_19_a, cc_a);
  mad_acc_v(h_b, f3_2_b, f8_19_b, cc_b);
  mad_acc_v(h_a, f4_2_a, f7_19_a, cc_a);
  mad_acc_v(h_b, f4_2_b, f7_19_b, cc_b);
  mad_acc_v(h_a, f5_2_a, f6_19_a, cc_a);
  mad_acc_v(h_b, f5_2_b, f6_19_b, cc_b);
  FE_LIMB(ra, 1, h_a)
  FE_LIMB(rb, 1, h_b)
  mad_acc_v(h_a, f0_2_a, f2_a, cc_a);
  mad_acc_v(h_b, f0_2_b, f2_b, cc_b);
  mad_acc_v(h_a, f1_2_a, f1_a, cc_a);
  mad_acc_v(h_b, f1_2_b, f1_b, cc_b);
  mad_acc_v(h_a, f3_4_a, f9_19_a, cc_a);
  mad_acc_v(h_b, f3_4_b, f9_19_b, cc_b);
  mad_acc_v(h_a, f4_2_a, f8_19_a, cc_a);
  mad_acc_v(h_b, f4_2_b, f8_19_b, cc_b);
  mad_acc_v(h_a, f5_4_a, f7_19_a, cc_a);
  mad_acc_v(h_b, f5_4_b, f7_19_b, cc_b);
  mad_acc_v(h_a, f6_a, f6_19_a, cc_a);
  mad_acc_v(h_b, f6_b, f6_19_b, cc_b);
  FE_LIMB(ra, 2, h_a)
  FE_LIMB(rb, 2, h_b)
  mad_acc_v(h_a, f0_2_a, f3_a, cc_a);
  mad_acc_v(h_b, f0_2_b, f3_b, cc_b);
  mad_acc_v(h_a, f1_2_a, f2_a, cc_a);
  mad_acc_v(h_b, f1_2_b, f2_b, cc_b);
  mad_acc_v(h_a, f4_2_a, f9_19_a, cc_a);
  mad_acc_v(h_b, f4_2_b, f9_19_b, cc_b);
  mad_acc_v(h_a, f5_2_a, f8_19_a, cc_a);
  mad_acc_v(h_b, f5_2_b, f8_19_b, cc_b);
  mad_acc_v(h_a, f6_2_a, f7_19_a, cc_a);
  mad_acc_v(h_b, f6_2_b, f7_19_b, cc_b);
  FE_LIMB(ra, 3, h_a)
  FE_LIMB(rb, 3, h_b)
  mad_acc_v(h_a, f0_2_a, f4_a, cc_a);
  mad_acc_v(h_b, f0_2_b, f4_b, cc_b);
  mad_acc_v(h_a, f1_2_a, f3_2_a, cc_a);
  mad_acc_v(h_b, f1_2_b, f3_2_b, cc_b);
  mad_acc_v(h_a, f2_a, f2_a, cc_a);
  mad_acc_v(h_b, f2_b, f2_b, cc_b);
  mad_acc_v(h_a, f5_4_a, f9_19_a, cc_a);
  mad_acc_v(h_b, f5_4_b, f9_19_b, cc_b);
  mad_acc_v(h_a, f6_2_a, f8_19_a, cc_a);
  mad_acc_v(h_b, f6_2_b, f8_19_b, cc_b);
  mad_acc_v(h_a, f7_2_a, f7_19_a, cc_a);
  mad_acc_v(h_b, f7_2_b, f7_19_b, cc_b);
  FE_LIMB(ra, 4, h_a)
  FE_LIMB(rb, 4, h_b)
  mad_acc_v(h_a, f0_2_a, f5_a, cc_a);
  mad_acc_v(h_b, f0_2_b, f5_b, cc_b);
  mad_acc_v(h_a, f1_2_a, f4_a, cc_a);
  mad_acc_v(h_b, f1_2_b, f4_b, cc_b);
  mad_acc_v(h_a, f2_2_a, f3_a, cc_a);
  mad_acc_v(h_b, f2_2_b, f3_b, cc_b);
  mad_acc_v(h_a, f6_2_a, f9_19_a, cc_a);
  mad_acc_v(h_b, f6_2_b, f9_19_b, cc_b);
  mad_acc_v(h_a, f7_2_a, f8_19_a, cc_a);
  mad_acc_v(h_b, f7_2_b, f8_19_b, cc_b);
  FE_LIMB(ra, 5, h_a)
  FE_LIMB(rb, 5, h_b)
  mad_acc_v(h_a, f0_2_a, f6_a, cc_a);
  mad_acc_v(h_b, f0_2_b, f6_b, cc_b);
  mad_acc_v(h_a, f1_2_a, f5_2_a, cc_a);
  mad_acc_v(h_b, f1_2_b, f5_2_b, cc_b);
  mad_acc_v(h_a, f2_2_a, f4_a, cc_a);
  mad_acc_v(h_b, f2_2_b, f4_b, cc_b);
  mad_acc_v(h_a, f3_2_a, f3_a, cc_a);
  mad_acc_v(h_b, f3_2_b, f3_b, cc_b);
  mad_acc_v(h_a, f7_4_a, f9_19_a, cc_a);
  mad_acc_v(h_b, f7_4_b, f9_19_b, cc_b);
  mad_acc_v(h_a, f8_a, f8_19_a, cc_a);
  mad_acc_v(h_b, f8_b, f8_19_b, cc_b);
  FE_LIMB(ra, 6, h_a)
  FE_LIMB(rb, 6, h_b)
  mad_acc_v(h_a, f0_2_a, f7_a, cc_a);
  mad_acc_v(h_b, f0_2_b, f7_b, cc_b);
  mad_acc_v(h_a, f1_2_a, f6_a, cc_a);
  mad_acc_v(h_b, f1_2_b, f6_b, cc_b);
  mad_acc_v(h_a, f2_2_a, f5_a, cc_a);
  mad_acc_v(h_b, f2_2_b, f5_b, cc_b);
  mad_acc_v(h_a, f3_2_a, f4_a, cc_a);
  mad_acc_v(h_b, f3_2_b, f4_b, cc_b);
  mad_acc_v(h_a, f8_2_a, f9_19_a, cc_a);
  mad_acc_v(h_b, f8_2_b, f9_19_b, cc_b);
  FE_LIMB(ra, 7, h_a)
  FE_LIMB(rb, 7, h_b)
  mad_acc_v(h_a, f0_2_a, f8_a, cc_a);
  mad_acc_v(h_b, f0_2_b, f8_b, cc_b);
  mad_acc_v(h_a, f1_2_a, f7_2_a, cc_a);
  mad_acc_v(h_b, f1_2_b, f7_2_b, cc_b);
  mad_acc_v(h_a, f2_2_a, f6_a, cc_a);
  mad_acc_v(h_b, f2_2_b, f6_b, cc_b);
  mad_acc_v(h_a, f3_2_a, f5_2_a, cc_a);
  mad_acc_v(h_b, f3_2_b, f5_2_b, cc_b);
  mad_acc_v(h_a, f4_a, f4_a, cc_a);
  mad_acc_v(h_b, f4_b, f4_b, cc_b);
  mad_acc_v(h_a, f9_2_a, f9_19_a, cc_a);
  mad_acc_v(h_b, f9_2_b, f9_19_b, cc_b);
  FE_LIMB(ra, 8, h_a)
  FE_LIMB(rb, 8, h_b)
  mad_acc_v(h_a, f0_2_a, f9_a, cc_a);
  mad_acc_v(h_b, f0_2_b, f9_b, cc_b);
  mad_acc_v(h_a, f1_2_a, f8_a, cc_a);
  mad_acc_v(h_b, f1_2_b, f8_b, cc_b);
  mad_acc_v(h_a, f2_2_a, f7_a, cc_a);
  mad_acc_v(h_b, f2_2_b, f7_b, cc_b);
  mad_acc_v(h_a, f3_2_a, f6_a, cc_a);
  mad_acc_v(h_b, f3_2_b, f6_b, cc_b);
  mad_acc_v(h_a, f4_2_a, f5_a, cc_a);
  mad_acc_v(h_b, f4_2_b, f5_b, cc_b);
  FE_LIMB(ra, 9, h_a)
  FE_LIMB(rb, 9, h_b)
  FE_FOLD(ra, h_a)
  FE_FOLD(rb, h_b)
  asm volatile("" : : "s"(cc_a), "s"(cc_b));  // both pairs live to the end: distinct registers
}

// ---- END generated pair products

DKG_DEV void fe_mul_small_ps(fe& r, const fe& a, uint32_t k) {
  uint64_t h = mad_first(a.v[0], k);
  FE_LIMB(r, 0, h)
  mad_acc(h, a.v[1], k); FE_LIMB(r, 1, h)
  mad_acc(h, a.v[2], k); FE_LIMB(r, 2, h)
  mad_acc(h, a.v[3], k); FE_LIMB(r, 3, h)
  mad_acc(h, a.v[4], k); FE_LIMB(r, 4, h)
  mad_acc(h, a.v[5], k); FE_LIMB(r, 5, h)
  mad_acc(h, a.v[6], k); FE_LIMB(r, 6, h)
  mad_acc(h, a.v[7], k); FE_LIMB(r, 7, h)
  mad_acc(h, a.v[8], k); FE_LIMB(r, 8, h)
  mad_acc(h, a.v[9], k); FE_LIMB(r, 9, h)
  FE_FOLD(r, h)
}

// ---- the same three functions as ten independent column sums ("operand scanning") and one
// parallel 64-bit carry pass afterwards: 12 % more issue slots than product scanning, but ten
// independent mad chains per multiplication instead of one, which pays where a SIMD holds too few
// waves to hide the chain (small multi-GPU shards, the first binomial steps).  Compiled into the
// dkgk_ilp copy of the kernels (kernels.hip with DKG_FE_ILP); the runtime picks the copy per
// launch by occupancy.
// Carry the ten 64-bit column sums into a tight element.
DKG_DEV void fe_carry64(fe& r, uint64_t h0, uint64_t h1, uint64_t h2, uint64_t h3, uint64_t h4,
                        uint64_t h5, uint64_t h6, uint64_t h7, uint64_t h8, uint64_t h9) {
  uint64_t c;
  c = h0 >> 26; h1 += c; h0 &= 0x3ffffff;
  c = h4 >> 26; h5 += c; h4 &= 0x3ffffff;
  c = h1 >> 25; h2 += c; h1 &= 0x1ffffff;
  c = h5 >> 25; h6 += c; h5 &= 0x1ffffff;
  c = h2 >> 26; h3 += c; h2 &= 0x3ffffff;
  c = h6 >> 26; h7 += c; h6 &= 0x3ffffff;
  c = h3 >> 25; h4 += c; h3 &= 0x1ffffff;
  c = h7 >> 25; h8 += c; h7 &= 0x1ffffff;
  c = h4 >> 26; h5 += c; h4 &= 0x3ffffff;
  c = h8 >> 26; h9 += c; h8 &= 0x3ffffff;
  c = h9 >> 25; h0 += c * 19; h9 &= 0x1ffffff;
  c = h0 >> 26; h1 += c; h0 &= 0x3ffffff;
  r.v[0] = (uint32_t)h0; r.v[1] = (uint32_t)h1; r.v[2] = (uint32_t)h2; r.v[3] = (uint32_t)h3;
  r.v[4] = (uint32_t)h4; r.v[5] = (uint32_t)h5; r.v[6] = (uint32_t)h6; r.v[7] = (uint32_t)h7;
  r.v[8] = (uint32_t)h8; r.v[9] = (uint32_t)h9;
}

DKG_DEV void fe_mul_cs(fe& r, const fe& f, const fe& g) {
  const uint32_t f0 = f.v[0], f1 = f.v[1], f2 = f.v[2], f3 = f.v[3], f4 = f.v[4];
  const uint32_t f5 = f.v[5], f6 = f.v[6], f7 = f.v[7], f8 = f.v[8], f9 = f.v[9];
  const uint32_t g0 = g.v[0], g1 = g.v[1], g2 = g.v[2], g3 = g.v[3], g4 = g.v[4];
  const uint32_t g5 = g.v[5], g6 = g.v[6], g7 = g.v[7], g8 = g.v[8], g9 = g.v[9];
  const uint32_t g1_19 = 19u * g1, g2_19 = 19u * g2, g3_19 = 19u * g3, g4_19 = 19u * g4;
  const uint32_t g5_19 = 19u * g5, g6_19 = 19u * g6, g7_19 = 19u * g7, g8_19 = 19u * g8;
  const uint32_t g9_19 = 19u * g9;
  const uint32_t f1_2 = dbl32(f1), f3_2 = dbl32(f3), f5_2 = dbl32(f5), f7_2 = dbl32(f7), f9_2 = dbl32(f9);
  uint64_t h0 = mul32(f0, g0) + mul32(f1_2, g9_19) + mul32(f2, g8_19) + mul32(f3_2, g7_19) +
                mul32(f4, g6_19) + mul32(f5_2, g5_19) + mul32(f6, g4_19) + mul32(f7_2, g3_19) +
                mul32(f8, g2_19) + mul32(f9_2, g1_19);
  uint64_t h1 = mul32(f0, g1) + mul32(f1, g0) + mul32(f2, g9_19) + mul32(f3, g8_19) +
                mul32(f4, g7_19) + mul32(f5, g6_19) + mul32(f6, g5_19) + mul32(f7, g4_19) +
                mul32(f8, g3_19) + mul32(f9, g2_19);
  uint64_t h2 = mul32(f0, g2) + mul32(f1_2, g1) + mul32(f2, g0) + mul32(f3_2, g9_19) +
                mul32(f4, g8_19) + mul32(f5_2, g7_19) + mul32(f6, g6_19) + mul32(f7_2, g5_19) +
                mul32(f8, g4_19) + mul32(f9_2, g3_19);
  uint64_t h3 = mul32(f0, g3) + mul32(f1, g2) + mul32(f2, g1) + mul32(f3, g0) + mul32(f4, g9_19) +
                mul32(f5, g8_19) + mul32(f6, g7_19) + mul32(f7, g6_19) + mul32(f8, g5_19) +
                mul32(f9, g4_19);
  uint64_t h4 = mul32(f0, g4) + mul32(f1_2, g3) + mul32(f2, g2) + mul32(f3_2, g1) + mul32(f4, g0) +
                mul32(f5_2, g9_19) + mul32(f6, g8_19) + mul32(f7_2, g7_19) + mul32(f8, g6_19) +
                mul32(f9_2, g5_19);
  uint64_t h5 = mul32(f0, g5) + mul32(f1, g4) + mul32(f2, g3) + mul32(f3, g2) + mul32(f4, g1) +
                mul32(f5, g0) + mul32(f6, g9_19) + mul32(f7, g8_19) + mul32(f8, g7_19) +
                mul32(f9, g6_19);
  uint64_t h6 = mul32(f0, g6) + mul32(f1_2, g5) + mul32(f2, g4) + mul32(f3_2, g3) + mul32(f4, g2) +
                mul32(f5_2, g1) + mul32(f6, g0) + mul32(f7_2, g9_19) + mul32(f8, g8_19) +
                mul32(f9_2, g7_19);
  uint64_t h7 = mul32(f0, g7) + mul32(f1, g6) + mul32(f2, g5) + mul32(f3, g4) + mul32(f4, g3) +
                mul32(f5, g2) + mul32(f6, g1) + mul32(f7, g0) + mul32(f8, g9_19) + mul32(f9, g8_19);
  uint64_t h8 = mul32(f0, g8) + mul32(f1_2, g7) + mul32(f2, g6) + mul32(f3_2, g5) + mul32(f4, g4) +
                mul32(f5_2, g3) + mul32(f6, g2) + mul32(f7_2, g1) + mul32(f8, g0) +
                mul32(f9_2, g9_19);
  uint64_t h9 = mul32(f0, g9) + mul32(f1, g8) + mul32(f2, g7) + mul32(f3, g6) + mul32(f4, g5) +
                mul32(f5, g4) + mul32(f6, g3) + mul32(f7, g2) + mul32(f8, g1) + mul32(f9, g0);
  fe_carry64(r, h0, h1, h2, h3, h4, h5, h6, h7, h8, h9);
}

DKG_DEV void fe_sq_cs(fe& r, const fe& f) {
  // Symmetric products counted once; x19 factors kept on limbs 5..9 (19 * 2^27.585 < 2^32) and
  // the extra 2 / 4 weights moved onto the partner limb so every operand fits in 32 bits.
  const uint32_t f0 = f.v[0], f1 = f.v[1], f2 = f.v[2], f3 = f.v[3], f4 = f.v[4];
  const uint32_t f5 = f.v[5], f6 = f.v[6], f7 = f.v[7], f8 = f.v[8], f9 = f.v[9];
  const uint32_t f0_2 = dbl32(f0), f1_2 = dbl32(f1), f2_2 = dbl32(f2), f3_2 = dbl32(f3), f4_2 = dbl32(f4);
  const uint32_t f5_2 = dbl32(f5), f6_2 = dbl32(f6), f7_2 = dbl32(f7), f8_2 = dbl32(f8), f9_2 = dbl32(f9);
  const uint32_t f1_4 = dbl32(f1_2), f3_4 = dbl32(f3_2), f5_4 = dbl32(f5_2), f7_4 = dbl32(f7_2);
  const uint32_t f5_19 = 19u * f5, f6_19 = 19u * f6, f7_19 = 19u * f7, f8_19 = 19u * f8;
  const uint32_t f9_19 = 19u * f9;
  uint64_t h0 = mul32(f0, f0) + mul32(f1_4, f9_19) + mul32(f2_2, f8_19) + mul32(f3_4, f7_19) +
                mul32(f4_2, f6_19) + mul32(f5_2, f5_19);
  uint64_t h1 = mul32(f0_2, f1) + mul32(f2_2, f9_19) + mul32(f3_2, f8_19) + mul32(f4_2, f7_19) +
                mul32(f5_2, f6_19);
  uint64_t h2 = mul32(f0_2, f2) + mul32(f1_2, f1) + mul32(f3_4, f9_19) + mul32(f4_2, f8_19) +
                mul32(f5_4, f7_19) + mul32(f6, f6_19);
  uint64_t h3 = mul32(f0_2, f3) + mul32(f1_2, f2) + mul32(f4_2, f9_19) + mul32(f5_2, f8_19) +
                mul32(f6_2, f7_19);
  uint64_t h4 = mul32(f0_2, f4) + mul32(f1_2, f3_2) + mul32(f2, f2) + mul32(f5_4, f9_19) +
                mul32(f6_2, f8_19) + mul32(f7_2, f7_19);
  uint64_t h5 = mul32(f0_2, f5) + mul32(f1_2, f4) + mul32(f2_2, f3) + mul32(f6_2, f9_19) +
                mul32(f7_2, f8_19);
  uint64_t h6 = mul32(f0_2, f6) + mul32(f1_2, f5_2) + mul32(f2_2, f4) + mul32(f3_2, f3) +
                mul32(f7_4, f9_19) + mul32(f8, f8_19);
  uint64_t h7 = mul32(f0_2, f7) + mul32(f1_2, f6) + mul32(f2_2, f5) + mul32(f3_2, f4) +
                mul32(f8_2, f9_19);
  uint64_t h8 = mul32(f0_2, f8) + mul32(f1_2, f7_2) + mul32(f2_2, f6) + mul32(f3_2, f5_2) +
                mul32(f4, f4) + mul32(f9_2, f9_19);
  uint64_t h9 = mul32(f0_2, f9) + mul32(f1_2, f8) + mul32(f2_2, f7) + mul32(f3_2, f6) +
                mul32(f4_2, f5);
  fe_carry64(r, h0, h1, h2, h3, h4, h5, h6, h7, h8, h9);
}

// r = a * k for a small constant k < 2^12 (a tight).
DKG_DEV void fe_mul_small_cs(fe& r, const fe& a, uint32_t k) {
  uint64_t h[10];
#pragma unroll
  for (int i = 0; i < 10; i++) h[i] = mul32(a.v[i], k);
  fe_carry64(r, h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7], h[8], h[9]);
}

// r = f * g, r = f^2, r = a * k (k < 2^12): all inputs tight or as bounded in tools/fe_bounds.py,
// outputs tight.  The flavour is fixed per translation unit.
DKG_DEV void fe_mul(fe& r, const fe& f, const fe& g) {
#ifdef DKG_FE_ILP
  fe_mul_cs(r, f, g);
#else
  fe_mul_ps(r, f, g);
#endif
}
DKG_DEV void fe_sq(fe& r, const fe& f) {
#ifdef DKG_FE_ILP
  fe_sq_cs(r, f);
#else
  fe_sq_ps(r, f);
#endif
}
DKG_DEV void fe_mul_small(fe& r, const fe& a, uint32_t k) {
#ifdef DKG_FE_ILP
  fe_mul_small_cs(r, a, k);
#else
  fe_mul_small_ps(r, a, k);
#endif
}

// Two independent products at once (the pair versions above; the column-sum flavour already has ten
// independent chains per product and just runs both).  DKG_FE_PAIR=0 keeps single products, 1 the
// two-chain interleave, 2 the four-chain split (A/B only: its functions are generated with
// tools/gen_fe_pair.py --four; measured 4-5 % slower, profiles/r06_pair_ab.txt).
#ifndef DKG_FE_PAIR
#define DKG_FE_PAIR 1
#endif
// DKG_PAIR_WIDE=1: the group formulas beyond the dedicated addition (doublings, the complete and mixed
// additions) pair their products too; 0 keeps them single (A/B).
#ifndef DKG_PAIR_WIDE
#define DKG_PAIR_WIDE 1
#endif
#if DKG_PAIR_WIDE && DKG_FE_PAIR && !defined(DKG_FE_ILP)
#define DKG_PW 1
#else
#define DKG_PW 0
#endif
DKG_DEV void fe_mul2(fe& ra, const fe& fa, const fe& ga, fe& rb, const fe& fb, const fe& gb) {
#if defined(DKG_FE_ILP) || !DKG_FE_PAIR
  fe a, b;
  fe_mul(a, fa, ga);
  fe_mul(b, fb, gb);
  fe_copy(ra, a);
  fe_copy(rb, b);
#elif DKG_FE_PAIR == 2
  fe_mul_ps4(ra, fa, ga, rb, fb, gb);
#else
  fe_mul_ps2(ra, fa, ga, rb, fb, gb);
#endif
}
DKG_DEV void fe_sq2(fe& ra, const fe& fa, fe& rb, const fe& fb) {
#if defined(DKG_FE_ILP) || !DKG_FE_PAIR
  fe a, b;
  fe_sq(a, fa);
  fe_sq(b, fb);
  fe_copy(ra, a);
  fe_copy(rb, b);
#elif DKG_FE_PAIR == 2
  fe_sq_ps4(ra, fa, rb, fb);
#else
  fe_sq_ps2(ra, fa, rb, fb);
#endif
}

DKG_DEV void fe_sqn(fe& r, const fe& a, int n) {
  fe_sq(r, a);
  for (int i = 1; i < n; i++) fe_sq(r, r);
}

// z^(2^252 - 3), the exponent of sqrt_ratio (RFC 9496 section 4.2 / ref10 pow22523).
DKG_DEV void fe_pow22523(fe& out, const fe& z) {
  fe t0, t1, t2;
  fe_sq(t0, z);             // 2
  fe_sqn(t1, t0, 2);        // 8
  fe_mul(t1, z, t1);        // 9
  fe_mul(t0, t0, t1);       // 11
  fe_sq(t0, t0);            // 22
  fe_mul(t0, t1, t0);       // 2^5 - 1
  fe_sqn(t1, t0, 5);
  fe_mul(t0, t1, t0);       // 2^10 - 1
  fe_sqn(t1, t0, 10);
  fe_mul(t1, t1, t0);       // 2^20 - 1
  fe_sqn(t2, t1, 20);
  fe_mul(t1, t2, t1);       // 2^40 - 1
  fe_sqn(t1, t1, 10);
  fe_mul(t0, t1, t0);       // 2^50 - 1
  fe_sqn(t1, t0, 50);
  fe_mul(t1, t1, t0);       // 2^100 - 1
  fe_sqn(t2, t1, 100);
  fe_mul(t1, t2, t1);       // 2^200 - 1
  fe_sqn(t1, t1, 50);
  fe_mul(t0, t1, t0);       // 2^250 - 1
  fe_sqn(t0, t0, 2);        // 2^252 - 4
  fe_mul(out, t0, z);       // 2^252 - 3
}

// z^(p-2) = 1/z
DKG_DEV void fe_invert(fe& out, const fe& z) {
  fe t0, t1, t2, t3;
  fe_sq(t0, z);             // 2
  fe_sqn(t1, t0, 2);        // 8
  fe_mul(t1, z, t1);        // 9
  fe_mul(t0, t0, t1);       // 11
  fe_sq(t2, t0);            // 22
  fe_mul(t1, t1, t2);       // 2^5 - 1
  fe_sqn(t2, t1, 5);
  fe_mul(t1, t2, t1);       // 2^10 - 1
  fe_sqn(t2, t1, 10);
  fe_mul(t2, t2, t1);       // 2^20 - 1
  fe_sqn(t3, t2, 20);
  fe_mul(t2, t3, t2);       // 2^40 - 1
  fe_sqn(t2, t2, 10);
  fe_mul(t1, t2, t1);       // 2^50 - 1
  fe_sqn(t2, t1, 50);
  fe_mul(t2, t2, t1);       // 2^100 - 1
  fe_sqn(t3, t2, 100);
  fe_mul(t2, t3, t2);       // 2^200 - 1
  fe_sqn(t2, t2, 50);
  fe_mul(t1, t2, t1);       // 2^250 - 1
  fe_sqn(t1, t1, 5);        // 2^255 - 32
  fe_mul(out, t1, t0);      // 2^255 - 21
}

// Fully reduce to the canonical representative and pack little-endian into 8 words.
DKG_DEV void fe_tobytes32(uint32_t (&s)[8], const fe& a) {
  fe t;
  fe_carry(t, a);
  fe_carry(t, t);
  // t < 2^255 + small; compute q = floor((t + 19) / 2^255) in {0,1}
  uint32_t q = (t.v[0] + 19u) >> 26;
  q = (t.v[1] + q) >> 25;
  q = (t.v[2] + q) >> 26;
  q = (t.v[3] + q) >> 25;
  q = (t.v[4] + q) >> 26;
  q = (t.v[5] + q) >> 25;
  q = (t.v[6] + q) >> 26;
  q = (t.v[7] + q) >> 25;
  q = (t.v[8] + q) >> 26;
  q = (t.v[9] + q) >> 25;
  t.v[0] += 19u * q;
  uint32_t c;
  c = t.v[0] >> 26; t.v[1] += c; t.v[0] &= 0x3ffffffu;
  c = t.v[1] >> 25; t.v[2] += c; t.v[1] &= 0x1ffffffu;
  c = t.v[2] >> 26; t.v[3] += c; t.v[2] &= 0x3ffffffu;
  c = t.v[3] >> 25; t.v[4] += c; t.v[3] &= 0x1ffffffu;
  c = t.v[4] >> 26; t.v[5] += c; t.v[4] &= 0x3ffffffu;
  c = t.v[5] >> 25; t.v[6] += c; t.v[5] &= 0x1ffffffu;
  c = t.v[6] >> 26; t.v[7] += c; t.v[6] &= 0x3ffffffu;
  c = t.v[7] >> 25; t.v[8] += c; t.v[7] &= 0x1ffffffu;
  c = t.v[8] >> 26; t.v[9] += c; t.v[8] &= 0x3ffffffu;
  t.v[9] &= 0x1ffffffu;
  // pack: bit offsets 0,26,51,77,102,128,153,179,204,230
  s[0] = t.v[0] | (t.v[1] << 26);
  s[1] = (t.v[1] >> 6) | (t.v[2] << 19);
  s[2] = (t.v[2] >> 13) | (t.v[3] << 13);
  s[3] = (t.v[3] >> 19) | (t.v[4] << 6);
  s[4] = t.v[5] | (t.v[6] << 25);
  s[5] = (t.v[6] >> 7) | (t.v[7] << 19);
  s[6] = (t.v[7] >> 13) | (t.v[8] << 12);
  s[7] = (t.v[8] >> 20) | (t.v[9] << 6);
}

// Unpack 255 bits (bit 255 ignored, as dalek FieldElement::from_bytes); result may be >= p.
DKG_DEV void fe_frombytes32(fe& r, const uint32_t (&s)[8]) {
  r.v[0] = s[0] & 0x3ffffffu;
  r.v[1] = ((s[0] >> 26) | (s[1] << 6)) & 0x1ffffffu;
  r.v[2] = ((s[1] >> 19) | (s[2] << 13)) & 0x3ffffffu;
  r.v[3] = ((s[2] >> 13) | (s[3] << 19)) & 0x1ffffffu;
  r.v[4] = (s[3] >> 6) & 0x3ffffffu;
  r.v[5] = s[4] & 0x1ffffffu;
  r.v[6] = ((s[4] >> 25) | (s[5] << 7)) & 0x3ffffffu;
  r.v[7] = ((s[5] >> 19) | (s[6] << 13)) & 0x1ffffffu;
  r.v[8] = ((s[6] >> 12) | (s[7] << 20)) & 0x3ffffffu;
  r.v[9] = (s[7] >> 6) & 0x1ffffffu;
}

// Canonical low bit (RFC 9496 IS_NEGATIVE) and zero test.
DKG_DEV uint32_t fe_isneg(const fe& a) {
  uint32_t s[8];
  fe_tobytes32(s, a);
  return s[0] & 1u;
}
DKG_DEV bool fe_iszero(const fe& a) {
  uint32_t s[8];
  fe_tobytes32(s, a);
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) o |= s[i];
  return o == 0;
}
// a == 0 (mod p) for `a` an fe_mul / fe_sq output (either flavour): such a value is below 2p and
// its limbs sit in their nominal widths except limbs 1 and 5, which can exceed 2^25 - 1 by a small
// carry (< 2^11, far below another 2^25), so 0 and p each have exactly one representation: all limbs zero, or p's
// canonical limbs (tools/fe_bounds.py asserts the output bounds this relies on).  ~30 full-rate ops.
DKG_DEV bool fe_tight_zero(const fe& a) {
  uint32_t z = a.v[0], q = a.v[0] ^ 0x3ffffedu;
#pragma unroll
  for (int i = 1; i < 10; i++) {
    z |= a.v[i];
    q |= a.v[i] ^ ((i & 1) ? 0x1ffffffu : 0x3ffffffu);
  }
  return (z == 0u) | (q == 0u);
}
DKG_DEV void fe_cmov(fe& r, const fe& a, bool c) {
#pragma unroll
  for (int i = 0; i < 10; i++) r.v[i] = c ? a.v[i] : r.v[i];
}
// r = |a| (non-negative representative), a tight
DKG_DEV void fe_abs(fe& r, const fe& a) {
  fe n;
  fe_neg(n, a);
  fe_carry(n, n);
  bool neg = fe_isneg(a);
  fe_copy(r, a);
  fe_cmov(r, n, neg);
}
