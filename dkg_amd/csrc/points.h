// Device-memory layouts for group elements and the LDS fixed-base (comb) tables.
//
// Extended points live in HBM as structure-of-arrays: word w (0..39: X0..X9, Y0..Y9, Z0..Z9,
// T0..T9) of element e at base[w * stride + e], so a wave reading 64 consecutive elements issues
// 40 fully coalesced 256-byte loads.  Comb tables (affine Niels, 30 words per entry) use the same
// SoA shape with 512 entries per base: entry (window w, digit d) = d * 16^w * B, d = 1..8.
#pragma once
#include "ge25519.h"
#include "sc25519.h"

constexpr int PT_WORDS = 40;
constexpr int AFF_WORDS = 30;
constexpr int COMB_ENTRIES = 512;  // 64 windows x 8 digits

DKG_DEV void pt_load(ge_p3& p, const uint32_t* __restrict__ base, size_t stride, size_t e) {
#pragma unroll
  for (int i = 0; i < 10; i++) {
    p.X.v[i] = base[(size_t)(i)*stride + e];
    p.Y.v[i] = base[(size_t)(10 + i) * stride + e];
    p.Z.v[i] = base[(size_t)(20 + i) * stride + e];
    p.T.v[i] = base[(size_t)(30 + i) * stride + e];
  }
}

DKG_DEV void pt_store(uint32_t* __restrict__ base, size_t stride, size_t e, const ge_p3& p) {
#pragma unroll
  for (int i = 0; i < 10; i++) {
    base[(size_t)(i)*stride + e] = p.X.v[i];
    base[(size_t)(10 + i) * stride + e] = p.Y.v[i];
    base[(size_t)(20 + i) * stride + e] = p.Z.v[i];
    base[(size_t)(30 + i) * stride + e] = p.T.v[i];
  }
}

// pt_store with nontemporal (streaming) stores: the data goes out without displacing L2 lines the
// kernel still reads.  The per-step binomial stores one table row per item and rereads its input
// rows (each position is read by two items of a launch); with plain stores one Horner step of the
// headline's tables took 324 us, with these 268 us (tools/ubench/binom, profiles/r06_binom_levers_ab.txt).
DKG_DEV void pt_store_nt(uint32_t* __restrict__ base, size_t stride, size_t e, const ge_p3& p) {
#pragma unroll
  for (int i = 0; i < 10; i++) {
    __builtin_nontemporal_store(p.X.v[i], base + (size_t)(i)*stride + e);
    __builtin_nontemporal_store(p.Y.v[i], base + (size_t)(10 + i) * stride + e);
    __builtin_nontemporal_store(p.Z.v[i], base + (size_t)(20 + i) * stride + e);
    __builtin_nontemporal_store(p.T.v[i], base + (size_t)(30 + i) * stride + e);
  }
}

// Point-major (AoS) element e: 40 consecutive words, moved as ten 16-B accesses.  Used for the
// per-(column, receiver) evaluations R, which one lane writes per step (stepping, recombination):
// a point fills whole cache lines instead of 40 scattered 4-B words.  base must be 16-B aligned.
// word w of a point (X, Y, Z, T limbs in order); constant w after unrolling, so no address is taken
DKG_DEV uint32_t& pt_word(ge_p3& p, int w) {
  fe& f = w < 10 ? p.X : (w < 20 ? p.Y : (w < 30 ? p.Z : p.T));
  return f.v[w % 10];
}
DKG_DEV uint32_t pt_word(const ge_p3& p, int w) {
  const fe& f = w < 10 ? p.X : (w < 20 ? p.Y : (w < 30 ? p.Z : p.T));
  return f.v[w % 10];
}

// Signed-digit recoding of a small positive multiplier m for the binomial's chains (mul_small_*):
// the NAF, except that a leading 1 0 -1 (2^k - 2^(k-2)) becomes 1 1 (2^(k-1) + 2^(k-2)): one
// doubling fewer for the same additions.  That is the cheapest signed-binary chain of every m < 256
// under this build's slot costs (checked exhaustively by tests/test_bench.py against all signed-digit
// representations; bench.py binom_digits): m = 3, 6, 11-13, 22-26, 44-52, ...  pos / neg hold the
// +1 / -1 digits; returns the length (the top digit is +1 at len - 1).
DKG_DEV int small_recode(uint32_t m, uint32_t& pos, uint32_t& neg) {
  pos = 0;
  neg = 0;
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
  if (len >= 3 && !((pos | neg) >> (len - 2) & 1u) && (neg >> (len - 3) & 1u)) {
    pos = (pos & ~(1u << (len - 1))) | (3u << (len - 3));
    neg &= ~(1u << (len - 3));
    len--;
  }
  return len;
}

// one 16-B store, nontemporal (streaming) when NT
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
template <bool NT>
DKG_DEV void st16(void* p, uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  const u32x4_t v = {a, b, c, d};
  if constexpr (NT) __builtin_nontemporal_store(v, reinterpret_cast<u32x4_t*>(p));
  else *reinterpret_cast<u32x4_t*>(p) = v;
}

DKG_DEV void pt_load_aos(ge_p3& p, const uint32_t* __restrict__ base, size_t e) {
  const uint4* b = reinterpret_cast<const uint4*>(base + e * PT_WORDS);
#pragma unroll
  for (int k = 0; k < PT_WORDS / 4; k++) {
    const uint4 v = b[k];
    pt_word(p, 4 * k) = v.x;
    pt_word(p, 4 * k + 1) = v.y;
    pt_word(p, 4 * k + 2) = v.z;
    pt_word(p, 4 * k + 3) = v.w;
  }
}

template <bool NT = false>
DKG_DEV void pt_store_aos(uint32_t* __restrict__ base, size_t e, const ge_p3& p) {
  uint32_t* b = base + e * PT_WORDS;
#pragma unroll
  for (int k = 0; k < PT_WORDS / 4; k++)
    st16<NT>(b + 4 * k, pt_word(p, 4 * k), pt_word(p, 4 * k + 1), pt_word(p, 4 * k + 2), pt_word(p, 4 * k + 3));
}

DKG_DEV void ld_words8(uint32_t (&w)[8], const uint32_t* __restrict__ p) {
  const uint4* q = reinterpret_cast<const uint4*>(p);
  uint4 a = q[0], b = q[1];
  w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w;
  w[4] = b.x; w[5] = b.y; w[6] = b.z; w[7] = b.w;
}

DKG_DEV void st_words8(uint32_t* __restrict__ p, const uint32_t (&w)[8]) {
  uint4* q = reinterpret_cast<uint4*>(p);
  q[0] = make_uint4(w[0], w[1], w[2], w[3]);
  q[1] = make_uint4(w[4], w[5], w[6], w[7]);
}

DKG_DEV void sc_load(sc& s, const uint32_t* __restrict__ p) {
  uint32_t w[8];
  ld_words8(w, p);
#pragma unroll
  for (int i = 0; i < 8; i++) s.v[i] = w[i];
}

// Read comb entry e (SoA, 512 entries) from LDS / global.
DKG_DEV void aff_load(ge_aff& q, const uint32_t* tab, int e) {
#pragma unroll
  for (int i = 0; i < 10; i++) {
    q.ypx.v[i] = tab[i * COMB_ENTRIES + e];
    q.ymx.v[i] = tab[(10 + i) * COMB_ENTRIES + e];
    q.xy2d.v[i] = tab[(20 + i) * COMB_ENTRIES + e];
  }
}

// acc += s * B using the 64-window signed radix-16 comb of B (no doublings: one mixed
// addition per window).  Digits are recentred on the fly exactly as dalek's to_radix_16.
DKG_DEV void comb_mul_add(ge_p3& acc, const sc& s, const uint32_t* tab) {
  int carry = 0;
  for (int w = 0; w < 64; w++) {
    const int wi = w >> 3;
    uint32_t word = s.v[0];
#pragma unroll
    for (int k = 1; k < 8; k++) word = (wi == k) ? s.v[k] : word;
    int d = (int)((word >> (4 * (w & 7))) & 15u) + carry;
    carry = (d + 8) >> 4;
    d -= carry << 4;
    const int ad = d < 0 ? -d : d;
    // Branch-free select (lanes carry independent scalars): identity for d = 0, and -Q =
    // (y-x, y+x, -2dxy) for d < 0, so every lane runs the same single mixed addition.
    ge_aff q, r;
    aff_load(q, tab, w * 8 + (ad == 0 ? 0 : ad - 1));
    fe nxy;
    fe_neg(nxy, q.xy2d);
    const bool neg = d < 0, zero = ad == 0;
#pragma unroll
    for (int i = 0; i < 10; i++) {
      r.ypx.v[i] = zero ? (i == 0 ? 1u : 0u) : (neg ? q.ymx.v[i] : q.ypx.v[i]);
      r.ymx.v[i] = zero ? (i == 0 ? 1u : 0u) : (neg ? q.ypx.v[i] : q.ymx.v[i]);
      r.xy2d.v[i] = zero ? 0u : (neg ? nxy.v[i] : q.xy2d.v[i]);
    }
    ge_madd(acc, acc, r);
  }
}

// Radix-2^19 comb in global memory (470 MB per base: HBM, read through L2 and the 256-MB Infinity
// Cache): 14 windows B_w = 2^(19 w) B of 262,144 affine Niels entries d B_w (d = 1..2^18),
// entry-major, 32 words per entry (ypx | ymx | xy2d | 2 pad).  Signed digits in [-2^18, 2^18 - 1]:
// one mixed addition per 19 scalar bits (14 per scalar; radix 2^17 took 16, 2^11 24, 2^8 32, the
// LDS radix-16 comb 64), for the bases every kernel shares (g, h).  The checks and commitments are
// VALU-bound: each window fewer pays more than the misses on the larger tables cost (radix 2^9 ..
// 2^11: profiles/r04_comb_radix_ab.txt; 2^11 .. 2^17: profiles/r05_comb_radix_ab.txt -- config 5
// device time 2^11 -> 2^15 -> 2^17: 303.6 -> 282.2 -> 273.3 ms per batch; 2^17 / 2^18 / 2^19:
// profiles/r06_comb_radix_ab.txt -- config 5 -2.3 ms, the headline -0.4 ms at 2^19, 2^18 flat).
#ifndef DKG_COMBW_BITS
#define DKG_COMBW_BITS 19  // -DDKG_COMBW_BITS=11 .. 19: the A/B builds
#endif
constexpr int COMBW_BITS = DKG_COMBW_BITS;
constexpr int COMBW_WINDOWS = 256 / COMBW_BITS + 1;  // the top window absorbs the signed recoding's carry
constexpr int COMBW_ENTRIES = 1 << (COMBW_BITS - 1);
constexpr int COMBW_STRIDE = 32;
constexpr size_t COMBW_WORDS = (size_t)COMBW_WINDOWS * COMBW_ENTRIES * COMBW_STRIDE;
static_assert(COMBW_WINDOWS * COMBW_BITS > 256 && (1 << (256 - (COMBW_WINDOWS - 1) * COMBW_BITS)) < COMBW_ENTRIES,
              "the top window must absorb the signed recoding's carry for any 256-bit scalar");

// Radix of the member keys' combs (full mode's encryption, K = pk_q r: one table per recipient key,
// shared by the wave's dealers, read through L2).
#ifndef DKG_KEY_COMB_BITS
#define DKG_KEY_COMB_BITS 10
#endif

// The comb geometry of radix 2^BITS: 256/BITS + 1 windows of 2^(BITS-1) entries of 32 words.
template <int BITS>
struct CombGeo {
  static constexpr int WINDOWS = 256 / BITS + 1;  // the top window absorbs the signed recoding's carry
  static constexpr int ENTRIES = 1 << (BITS - 1);
  static constexpr size_t WORDS = (size_t)WINDOWS * ENTRIES * 32;
  static_assert(WINDOWS * BITS > 256 && (1 << (256 - (WINDOWS - 1) * BITS)) < ENTRIES,
                "the top window must absorb the signed recoding's carry for any 256-bit scalar");
};

// Window w's signed digit (carry in / out) and its entry in the radix-2^BITS comb of base `tab`.
template <int BITS>
DKG_DEV const uint32_t* combw_entry_r(const sc& s, int w, int& carry, bool& neg, bool& zero,
                                      const uint32_t* __restrict__ tab) {
  constexpr int ENTRIES = CombGeo<BITS>::ENTRIES;
  // bits [B w, B w + B) of the scalar: words wi and wi + 1 (wave-uniform selects)
  const int bit = BITS * w, wi = bit >> 5, sh = bit & 31;
  uint32_t lo = 0, hi = 0;
#pragma unroll
  for (int k = 0; k < 8; k++) {
    lo = (wi == k) ? s.v[k] : lo;
    hi = (wi + 1 == k) ? s.v[k] : hi;
  }
  const uint32_t raw = (uint32_t)(((uint64_t)hi << 32 | lo) >> sh) & ((1u << BITS) - 1);
  int d = (int)raw + carry;
  carry = (d + ENTRIES) >> BITS;
  d -= carry << BITS;
  const int ad = d < 0 ? -d : d;
  neg = d < 0;
  zero = ad == 0;
  return tab + ((size_t)w * ENTRIES + (ad == 0 ? 0 : ad - 1)) * COMBW_STRIDE;
}

// The entry's 30 words as an affine Niels addend: -Q = (y-x, y+x, -2dxy), 0 = (1, 1, 0).
DKG_DEV void combw_select(ge_aff& r, const uint4 (&e)[8], bool neg, bool zero) {
  const uint32_t* q = reinterpret_cast<const uint32_t*>(e);  // ypx 0..9 | ymx 10..19 | xy2d 20..29
#pragma unroll
  for (int i = 0; i < 10; i++) {
    const uint32_t ypx = q[i], ymx = q[10 + i];
    r.ypx.v[i] = zero ? (i == 0 ? 1u : 0u) : (neg ? ymx : ypx);
    r.ymx.v[i] = zero ? (i == 0 ? 1u : 0u) : (neg ? ypx : ymx);
  }
#pragma unroll
  for (int i = 0; i < 10; i++) {
    const uint32_t p2 = i == 0 ? fe_const::P2_0 : ((i & 1) ? fe_const::P2_O : fe_const::P2_E);
    r.xy2d.v[i] = zero ? 0u : (neg ? p2 - q[20 + i] : q[20 + i]);
  }
}

// minimum resident waves per SIMD of the fixed-base kernels (check, commitments): 4 caps them at 128
// VGPRs, 3 at 168, 2 at 256
#ifndef DKG_COMB_WAVES
#define DKG_COMB_WAVES 4
#endif

// acc += s * B with the radix-2^BITS comb of B.  (Loading each window's entry one window ahead
// measured no gain -- check 48.0 vs 47.7 ms on config 5 -- and pushed the kernels into scratch at 128
// VGPRs: profiles/r05_comb_radix_ab.txt.)
template <int BITS, bool IL = false>
DKG_DEV void combw_mul_add_r(ge_p3& acc, const sc& s, const uint32_t* __restrict__ tab) {
  int carry = 0;
  bool neg, zero;
#pragma unroll 1
  for (int w = 0; w < CombGeo<BITS>::WINDOWS; w++) {
    const uint4* p = reinterpret_cast<const uint4*>(combw_entry_r<BITS>(s, w, carry, neg, zero, tab));
    uint4 e[8];
#pragma unroll
    for (int k = 0; k < 8; k++) e[k] = p[k];
    ge_aff r;
    combw_select(r, e, neg, zero);
    ge_madd<IL>(acc, acc, r);
  }
}
// the shared bases' combs (g, h: radix 2^DKG_COMBW_BITS)
template <bool IL = false>
DKG_DEV void combw_mul_add(ge_p3& acc, const sc& s, const uint32_t* __restrict__ tab) {
  combw_mul_add_r<COMBW_BITS, IL>(acc, s, tab);
}


// Register-lean variants for the m-chains: the cached addend lives in LDS (lane-interleaved,
// word w of lane l at q[w * 64 + l], conflict-free) and is read field by field when the addition
// needs it, so a chain keeps one point + the doubling temporaries in VGPRs (<= 128: 4 waves/SIMD).
// q points at this lane's column (base + lane); consecutive words are `stride` apart.
DKG_DEV void lds_put_cached(uint32_t* q, const ge_cached& c, int stride = 64) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(&c);
#pragma unroll
  for (int k = 0; k < PT_WORDS; k++) q[k * stride] = w[k];
}
// which: 0 = Y+X, 1 = Y-X, 2 = 2Z, 3 = 2dT
DKG_DEV void lds_get_fe(fe& r, const uint32_t* q, int which, int stride = 64) {
#pragma unroll
  for (int i = 0; i < 10; i++) r.v[i] = q[(which * 10 + i) * stride];
  // Opaque use of all ten limbs at once (one lgkmcnt wait for the group): stops LICM from
  // hoisting the loads and their x19 products out of the chain loop (~140 extra VGPRs).
  asm volatile("" : "+v"(r.v[0]), "+v"(r.v[1]), "+v"(r.v[2]), "+v"(r.v[3]), "+v"(r.v[4]), "+v"(r.v[5]),
               "+v"(r.v[6]), "+v"(r.v[7]), "+v"(r.v[8]), "+v"(r.v[9]));
}

// r = p +/- Q with Q the cached point in LDS; `neg` must be wave-uniform.
template <bool IL = false>
DKG_DEV void ge_add_lds(ge_p3& r, const ge_p3& p, const uint32_t* q, bool neg, int stride = 64,
                        bool with_t = true) {
  if constexpr (IL && DKG_PW) {
    fe a, b, e, h, t, u, qv, qw;
    fe_sub(t, p.Y, p.X);
    lds_get_fe(qv, q, neg ? 0 : 1, stride);
    fe_add(u, p.Y, p.X);
    lds_get_fe(qw, q, neg ? 1 : 0, stride);
    fe_mul2(a, t, qv, b, u, qw);
    fe_sub(e, b, a);
    fe_add(h, b, a);
    lds_get_fe(qv, q, 3, stride);
    lds_get_fe(qw, q, 2, stride);
    fe_mul2(a, p.T, qv, b, p.Z, qw);  // c, d
    if (neg) fe_neg(a, a);
    fe_sub(t, b, a);          // f
    fe_add(b, b, a);          // g
    fe_mul2(r.X, e, t, r.Y, b, h);
    if (with_t) fe_mul2(r.Z, b, t, r.T, e, h);
    else fe_mul(r.Z, b, t);
    return;
  }
  fe a, b, e, h, t, qv;
  fe_sub(t, p.Y, p.X);
  lds_get_fe(qv, q, neg ? 0 : 1, stride);
  fe_mul(a, t, qv);
  fe_add(t, p.Y, p.X);
  lds_get_fe(qv, q, neg ? 1 : 0, stride);
  fe_mul(b, t, qv);
  fe_sub(e, b, a);          // <= 1.5*2^27
  fe_add(h, b, a);          // <= 2^27
  lds_get_fe(qv, q, 3, stride);
  fe_mul(a, p.T, qv);       // c
  if (neg) fe_neg(a, a);    // 2p - c <= 2p limbwise: a valid fe_sub subtrahend, no carry needed
  lds_get_fe(qv, q, 2, stride);
  fe_mul(b, p.Z, qv);       // d
  fe_sub(t, b, a);          // f
  fe_add(b, b, a);          // g
  fe_mul(r.X, e, t);
  fe_mul(r.Y, b, h);
  fe_mul(r.Z, b, t);        // the x19 operands are F (X, Z) and H (Y, T): computed once each
  if (with_t) fe_mul(r.T, e, h);
}

// Dedicated addition (Hisil-Wong-Carter-Dawson 2008, "add-2008-hwcd-4", a = -1): r = p + Q with Q
// prepared by ge_to_cached_ded as (Y+X, Y-X, 2Z, 2T) in LDS.  8M and no multiplication by d (the
// cached form needs none either: the stepping saves one product per lane and step), but the formula
// is not complete: F = 2(X1 Y2 - Y1 X2) vanishes when p - Q is 0 or the 2-torsion point, G = 2(Y1 Y2
// - X1 X2) when p + Q meets the 4-torsion, and then the result has Z = F G = 0.  Whenever Z != 0 the
// result is p + Q exactly (tools/ded_check.py checks both claims over every 8-torsion offset).
// Callers test Z with fe_tight_zero and redo the work with the complete ge_add_lds.
DKG_DEV void ge_to_cached_ded(ge_cached& c, const ge_p3& p) {
  fe_add(c.YpX, p.Y, p.X);
  fe_sub(c.YmX, p.Y, p.X);
  fe_dbl(c.Z2, p.Z);
  fe_dbl(c.T2d, p.T);       // 2T in the 2dT slot
}
DKG_DEV void ge_add_ded_lds(ge_p3& r, const ge_p3& p, const uint32_t* q, int stride = 64) {
#if DKG_FE_PAIR && !defined(DKG_FE_ILP)
  // the eight products as four independent pairs (fe_mul2: no hazard wait states between the mads)
  fe a, b, e, h, t, u, qv, qw;
  fe_sub(t, p.Y, p.X);
  lds_get_fe(qv, q, 0, stride);  // Y2 + X2
  fe_add(u, p.Y, p.X);
  lds_get_fe(qw, q, 1, stride);  // Y2 - X2
  fe_mul2(a, t, qv, b, u, qw);   // A = (Y1 - X1)(Y2 + X2), B = (Y1 + X1)(Y2 - X2)
  fe_sub(e, b, a);               // F = B - A <= 1.5*2^27
  fe_add(h, b, a);               // G = B + A <= 2^27
  lds_get_fe(qv, q, 3, stride);  // 2 T2
  lds_get_fe(qw, q, 2, stride);  // 2 Z2
  fe_mul2(a, p.Z, qv, b, p.T, qw);  // C = 2 Z1 T2, D = 2 T1 Z2
  fe_add(t, b, a);               // E = D + C <= 2^27
  fe_sub(b, b, a);               // H = D - C <= 1.5*2^27
  fe_mul2(r.X, t, e, r.T, t, b);  // X3 = E F, T3 = E H
  fe_mul2(r.Y, h, b, r.Z, h, e);  // Y3 = G H, Z3 = F G
#else
  fe a, b, e, h, t, qv;
  fe_sub(t, p.Y, p.X);
  lds_get_fe(qv, q, 0, stride);  // Y2 + X2
  fe_mul(a, t, qv);              // A = (Y1 - X1)(Y2 + X2)
  fe_add(t, p.Y, p.X);
  lds_get_fe(qv, q, 1, stride);  // Y2 - X2
  fe_mul(b, t, qv);              // B = (Y1 + X1)(Y2 - X2)
  fe_sub(e, b, a);               // F = B - A <= 1.5*2^27
  fe_add(h, b, a);               // G = B + A <= 2^27
  lds_get_fe(qv, q, 3, stride);  // 2 T2
  fe_mul(a, p.Z, qv);            // C = 2 Z1 T2
  lds_get_fe(qv, q, 2, stride);  // 2 Z2
  fe_mul(b, p.T, qv);            // D = 2 T1 Z2
  fe_add(t, b, a);               // E = D + C <= 2^27
  fe_sub(b, b, a);               // H = D - C <= 1.5*2^27
  fe_mul(r.X, t, e);             // X3 = E F
  fe_mul(r.Y, h, b);             // Y3 = G H
  fe_mul(r.T, t, b);             // T3 = E H
  fe_mul(r.Z, h, e);             // Z3 = F G  (x19 operands F and H, computed once each)
#endif
}

// The dedicated addition with a signed addend and an optional T (the m-chains of the per-wave
// binomial): r = p +/- Q, Q as ge_to_cached_ded in LDS, -Q = (Y-X, Y+X, 2Z, -2T) -- the fields
// swapped and C negated exactly as ge_add_lds does (the same bounds).  `neg` wave-uniform.  Not
// complete (above): the caller tests r.Z.
template <bool IL = false>
DKG_DEV void ge_add_ded_lds_s(ge_p3& r, const ge_p3& p, const uint32_t* q, bool neg, int stride = 64,
                              bool with_t = true) {
  if constexpr (IL && DKG_PW) {
    fe a, b, e, h, t, u, qv, qw;
    fe_sub(t, p.Y, p.X);
    lds_get_fe(qv, q, neg ? 1 : 0, stride);
    fe_add(u, p.Y, p.X);
    lds_get_fe(qw, q, neg ? 0 : 1, stride);
    fe_mul2(a, t, qv, b, u, qw);   // A, B
    fe_sub(e, b, a);               // F
    fe_add(h, b, a);               // G
    lds_get_fe(qv, q, 3, stride);
    lds_get_fe(qw, q, 2, stride);
    fe_mul2(a, p.Z, qv, b, p.T, qw);  // C, D
    if (neg) fe_neg(a, a);
    fe_add(t, b, a);               // E
    fe_sub(b, b, a);               // H
    fe_mul2(r.X, t, e, r.Y, h, b);
    if (with_t) fe_mul2(r.Z, h, e, r.T, t, b);
    else fe_mul(r.Z, h, e);
    return;
  }
  fe a, b, e, h, t, qv;
  fe_sub(t, p.Y, p.X);
  lds_get_fe(qv, q, neg ? 1 : 0, stride);
  fe_mul(a, t, qv);              // A
  fe_add(t, p.Y, p.X);
  lds_get_fe(qv, q, neg ? 0 : 1, stride);
  fe_mul(b, t, qv);              // B
  fe_sub(e, b, a);               // F
  fe_add(h, b, a);               // G
  lds_get_fe(qv, q, 3, stride);
  fe_mul(a, p.Z, qv);            // C = 2 Z1 T2
  if (neg) fe_neg(a, a);         // 2p - C <= 2p limbwise: a valid fe_sub subtrahend
  lds_get_fe(qv, q, 2, stride);
  fe_mul(b, p.T, qv);            // D = 2 T1 Z2
  fe_add(t, b, a);               // E = D + C
  fe_sub(b, b, a);               // H = D - C
  fe_mul(r.X, t, e);             // X3 = E F
  fe_mul(r.Y, h, b);             // Y3 = G H
  fe_mul(r.Z, h, e);             // Z3 = F G
  if (with_t) fe_mul(r.T, t, b); // T3 = E H
}

// r = p +/- Q with Q affine Niels (y+x, y-x, 2dxy) in LDS, read like the cached form above (fields
// 0, 1, 2): 7M, d = 2Z carried as in ge_madd_signed.  `neg` must be wave-uniform.
template <bool IL = false>
DKG_DEV void ge_madd_lds(ge_p3& r, const ge_p3& p, const uint32_t* q, bool neg, int stride = 64,
                         bool with_t = true) {
  if constexpr (IL && DKG_PW) {
    fe a, b, e, h, t, u, qv, qw;
    fe_sub(t, p.Y, p.X);
    lds_get_fe(qv, q, neg ? 0 : 1, stride);
    fe_add(u, p.Y, p.X);
    lds_get_fe(qw, q, neg ? 1 : 0, stride);
    fe_mul2(a, t, qv, b, u, qw);
    fe_sub(e, b, a);
    fe_add(h, b, a);
    lds_get_fe(qv, q, 2, stride);
    fe_mul(a, p.T, qv);       // c
    if (neg) fe_neg(a, a);
    fe_dbl(b, p.Z);
    fe_carry(b, b);           // d = 2Z, tight
    fe_sub(t, b, a);          // f
    fe_add(b, b, a);          // g
    fe_mul2(r.X, e, t, r.Y, b, h);
    if (with_t) fe_mul2(r.Z, b, t, r.T, e, h);
    else fe_mul(r.Z, b, t);
    return;
  }
  fe a, b, e, h, t, qv;
  fe_sub(t, p.Y, p.X);
  lds_get_fe(qv, q, neg ? 0 : 1, stride);
  fe_mul(a, t, qv);
  fe_add(t, p.Y, p.X);
  lds_get_fe(qv, q, neg ? 1 : 0, stride);
  fe_mul(b, t, qv);
  fe_sub(e, b, a);
  fe_add(h, b, a);
  lds_get_fe(qv, q, 2, stride);
  fe_mul(a, p.T, qv);       // c
  if (neg) fe_neg(a, a);    // 2p - c <= 2p limbwise
  fe_dbl(b, p.Z);
  fe_carry(b, b);           // d = 2Z, tight
  fe_sub(t, b, a);          // f
  fe_add(b, b, a);          // g
  fe_mul(r.X, e, t);
  fe_mul(r.Y, b, h);
  fe_mul(r.Z, b, t);        // the x19 operands are F (X, Z) and H (Y, T): computed once each
  if (with_t) fe_mul(r.T, e, h);
}

