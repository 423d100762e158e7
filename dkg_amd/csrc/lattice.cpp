// Short recombination multipliers for the degree split.
//
// P(j) = sum_{u<K} y^u Q_u(j) with y = j^L mod l costs K-1 products by full 253-bit scalars.  Any
// vector v = (b, a_1, .., a_{K-1}) of the lattice  Lambda_y = { v in Z^K : a_u = b y^u (mod l) }
// with b != 0 (mod l) gives the same decision with shorter scalars:
//     b P(j) = b Q_0(j) + a_1 Q_1(j) + .. + a_{K-1} Q_{K-1}(j),
// and  P(j) == g*s + h*s'  <=>  b P(j) == g*(b s) + h*(b s')  in the prime-order group (b is
// invertible mod l; a Ristretto element is a coset of the 4-torsion, and D in 2E lies in E[4] iff
// b D does).  det Lambda_y = l^(K-1), so a reduced basis holds a vector with entries near
// l^((K-1)/K): 126 bits for K = 2, 168 for K = 3, 189 for K = 4 -- one joint double-and-add chain
// of that many doublings instead of 253.
//
// The reduction is textbook LLL (delta = 0.99) on exact 512-bit two's-complement integer vectors
// with the Gram-Schmidt coefficients in long double, size reduction repeated until every |mu| is
// <= 1/2 (Schnorr-Euchner).  Integer row operations keep every row in the lattice whatever the
// floating-point accuracy, and the chosen row is re-checked in Z_l before it is used, so precision
// only affects how short the result is; a row that fails the check or is not shorter than the
// powers themselves falls back to (1, y, .., y^(K-1)).
//
// The row used is not simply the shortest: every combination sum_i c_i B_i, c_i in {-4..4}, of the
// reduced basis is priced as the recombination chain runs -- (NAF length - 1) doublings plus one
// addition per nonzero NAF digit of each entry -- and the cheapest is kept (5.5 % less chain work
// than the shortest row on average at U = 4, n = 1024).
#include <math.h>
#include <string.h>

#include "host_crypto.h"

namespace dkgh {
namespace {

struct I512 {  // two's complement, little-endian 64-bit limbs; arithmetic is mod 2^512
  uint64_t w[8];
};
typedef unsigned __int128 u128;

I512 i_zero() {
  I512 r;
  memset(r.w, 0, sizeof r.w);
  return r;
}
bool i_neg_p(const I512& a) { return (a.w[7] >> 63) != 0; }
I512 i_neg(const I512& a) {
  I512 r;
  u128 c = 1;
  for (int i = 0; i < 8; i++) {
    c += (u128)(~a.w[i]);
    r.w[i] = (uint64_t)c;
    c >>= 64;
  }
  return r;
}
I512 i_sub(const I512& a, const I512& b) {
  I512 r;
  u128 bb = 0;
  for (int i = 0; i < 8; i++) {
    const u128 d = (u128)a.w[i] - b.w[i] - bb;
    r.w[i] = (uint64_t)d;
    bb = (d >> 64) & 1;
  }
  return r;
}
// a * m * 2^e (m signed 64-bit, e >= 0), mod 2^512
I512 i_mul_shift(const I512& a, int64_t m, int e) {
  const bool neg = m < 0;
  const uint64_t um = neg ? (uint64_t)0 - (uint64_t)m : (uint64_t)m;
  I512 r;
  u128 c = 0;
  for (int i = 0; i < 8; i++) {
    c += (u128)a.w[i] * um;
    r.w[i] = (uint64_t)c;
    c >>= 64;
  }
  if (e > 0) {
    const int wl = e / 64, bl = e % 64;
    I512 s = i_zero();
    for (int i = 7; i >= wl; i--) {
      uint64_t v = r.w[i - wl] << bl;
      if (bl && i - wl - 1 >= 0) v |= r.w[i - wl - 1] >> (64 - bl);
      s.w[i] = v;
    }
    r = s;
  }
  return neg ? i_neg(r) : r;
}
int i_bits(const I512& a) {  // bit length of |a|
  const I512 m = i_neg_p(a) ? i_neg(a) : a;
  for (int i = 7; i >= 0; i--)
    if (m.w[i]) return 64 * i + 64 - __builtin_clzll(m.w[i]);
  return 0;
}
long double i_ld(const I512& a) {  // to 64 significant bits: the top two nonzero limbs
  const bool neg = i_neg_p(a);
  const I512 m = neg ? i_neg(a) : a;
  static const long double P64[8] = {1.0L, 0x1p64L, 0x1p128L, 0x1p192L, 0x1p256L, 0x1p320L, 0x1p384L, 0x1p448L};
  int t = 7;
  while (t > 0 && !m.w[t]) t--;
  const long double v = t > 0 ? ((long double)m.w[t] * P64[1] + (long double)m.w[t - 1]) * P64[t - 1]
                              : (long double)m.w[0];
  return neg ? -v : v;
}
I512 i_add(const I512& a, const I512& b) {
  I512 r;
  u128 c = 0;
  for (int i = 0; i < 8; i++) {
    c += (u128)a.w[i] + b.w[i];
    r.w[i] = (uint64_t)c;
    c >>= 64;
  }
  return r;
}
// NAF of |a|: length (highest digit position + 1) = bit length of 3|a| / 2, weight =
// popcount((3|a| ^ |a|) / 2)
void i_naf_shape(const I512& a, int& len, int& weight) {
  const I512 m = i_neg_p(a) ? i_neg(a) : a;
  const I512 m3 = i_add(m, i_add(m, m));
  len = 0;
  weight = 0;
  for (int i = 0; i < 8; i++) {
    const uint64_t h = (m3.w[i] >> 1) | (i < 7 ? m3.w[i + 1] << 63 : 0);
    const uint64_t x = (m3.w[i] ^ m.w[i]) >> 1 | (i < 7 ? (m3.w[i + 1] ^ m.w[i + 1]) << 63 : 0);
    weight += __builtin_popcountll(x);
    if (h) len = 64 * i + 64 - __builtin_clzll(h);
  }
}
// issue-slot estimate of the recombination chain for the row v (doubling ~1815, mixed addition ~2002)
double chain_cost(const I512* v, int K) {
  int top = 0, adds = 0;
  for (int u = 0; u < K; u++) {
    int len, w;
    i_naf_shape(v[u], len, w);
    top = top > len ? top : len;
    adds += w;
  }
  return (top > 0 ? top - 1 : 0) * 1815.0 + adds * 2002.0;
}

I512 i_from_zl(const Zl& z) {
  I512 r = i_zero();
  for (int i = 0; i < 4; i++) r.w[i] = z.w[i];
  return r;
}
Zl zl_of(const I512& a) {  // a mod l for |a| < 2^512
  const bool neg = i_neg_p(a);
  const I512 m = neg ? i_neg(a) : a;
  uint8_t b[64];
  for (int i = 0; i < 64; i++) b[i] = (uint8_t)(m.w[i / 8] >> (8 * (i % 8)));
  const Zl z = zl_from_bytes_wide(b, 64);
  return neg ? zl_sub(zl_from_u64(0), z) : z;
}

const int KMAX = 5;

// v -= q v_j for the long double integer q
void sub_multiple(I512* v, const I512* vj, int K, long double q) {
  if (q == 0) return;
  int e;
  const long double fr = frexpl(q, &e);  // q = fr 2^e, 0.5 <= |fr| < 1
  int64_t m;
  int sh;
  if (e <= 62) {
    m = (int64_t)q;  // exact: q is an integer below 2^62
    sh = 0;
  } else {
    m = (int64_t)ldexpl(fr, 62);  // the top 62 bits of q (the rest of q's mantissa is zeros
    sh = e - 62;                  // below 2^-64 relative: q's integer part is m 2^sh + junk < 2^sh)
  }
  for (int u = 0; u < K; u++) v[u] = i_sub(v[u], i_mul_shift(vj[u], m, sh));
}

void gram_schmidt(const I512 (*B)[KMAX], int K, long double (*mu)[KMAX], long double* nrm) {
  long double bs[KMAX][KMAX];
  for (int i = 0; i < K; i++) {
    long double bi[KMAX];
    for (int u = 0; u < K; u++) bs[i][u] = bi[u] = i_ld(B[i][u]);
    for (int j = 0; j < i; j++) {
      long double d = 0;
      for (int u = 0; u < K; u++) d += bi[u] * bs[j][u];
      mu[i][j] = nrm[j] > 0 ? d / nrm[j] : 0;
      for (int u = 0; u < K; u++) bs[i][u] -= mu[i][j] * bs[j][u];
    }
    long double s = 0;
    for (int u = 0; u < K; u++) s += bs[i][u] * bs[i][u];
    nrm[i] = s;
  }
}

}  // namespace

bool short_multipliers(const Zl& y, int K, uint8_t (*mag)[32], int8_t* sign) {
  if (K < 2 || K > KMAX) return false;
  I512 B[KMAX][KMAX];
  Zl p = zl_from_u64(1), pw[KMAX];
  for (int u = 0; u < K; u++) {
    pw[u] = p;
    p = zl_mul(p, y);
  }
  I512 lv;
  {
    const uint64_t Lw[4] = {0x5812631a5cf5d3edull, 0x14def9dea2f79cd6ull, 0ull, 0x1000000000000000ull};
    lv = i_zero();
    for (int i = 0; i < 4; i++) lv.w[i] = Lw[i];
  }
  for (int u = 0; u < K; u++) B[0][u] = i_from_zl(pw[u]);
  for (int i = 1; i < K; i++)
    for (int u = 0; u < K; u++) B[i][u] = u == i ? lv : i_zero();
  long double mu[KMAX][KMAX], nrm[KMAX];
  int k = 1, guard = 0;
  while (k < K && guard++ < 4096) {
    for (int pass = 0; pass < 16; pass++) {  // size-reduce row k against rows k-1..0
      gram_schmidt(B, K, mu, nrm);
      bool done = true;
      for (int j = k - 1; j >= 0; j--) {
        const long double q = roundl(mu[k][j]);
        if (q == 0) continue;
        done = false;
        sub_multiple(B[k], B[j], K, q);
        for (int i = 0; i < j; i++) mu[k][i] -= q * mu[j][i];
      }
      if (done) break;
    }
    gram_schmidt(B, K, mu, nrm);
    if (nrm[k] >= (0.99L - mu[k][k - 1] * mu[k][k - 1]) * nrm[k - 1]) {
      k++;
    } else {
      for (int u = 0; u < K; u++) {
        const I512 t = B[k][u];
        B[k][u] = B[k - 1][u];
        B[k - 1][u] = t;
      }
      k = k > 1 ? k - 1 : 1;
    }
  }
  // the cheapest chain among the small combinations of the reduced rows with every entry below
  // 2^253 (the NAF digit arrays hold 256 positions); v and -v cost the same, so only combinations
  // whose first nonzero coefficient is positive are priced.  Integer combinations of lattice rows
  // are lattice rows: the Z_l check of the winner below is a safety net.
  // coefficients in {-4..4} (6561 combinations at K = 4, ~0.5 s once per (n, L, U) on 16 threads):
  // 1.0 % less recombination work than {-2..2} (625), which was 0.9 % below {-1..1}; K = 5 keeps
  // {-2..2} (3125 combinations; {-4..4} would be 59049)
  const int CRMAX = 4, CR = K <= 4 ? 4 : 2;
  I512 mult[KMAX][2 * CRMAX + 1][KMAX];  // mult[i][c + CR] = c B_i, |c| <= CR
  for (int i = 0; i < K; i++)
    for (int c = -CR; c <= CR; c++)
      for (int u = 0; u < K; u++) mult[i][c + CR][u] = i_mul_shift(B[i][u], c, 0);
  I512 v[KMAX];
  for (int u = 0; u < K; u++) v[u] = i_from_zl(pw[u]);  // fallback: the powers themselves
  double best = chain_cost(v, K);
  I512 win[KMAX];
  bool have = false;
  int ncomb = 1;
  for (int i = 0; i < K; i++) ncomb *= 2 * CR + 1;
  for (int code = 0; code < ncomb; code++) {
    int cf[KMAX], first = 0;
    for (int i = 0, cd = code; i < K; i++, cd /= 2 * CR + 1) {
      cf[i] = cd % (2 * CR + 1) - CR;
      if (!first && cf[i]) first = cf[i];
    }
    if (first <= 0) continue;  // zero, or the negation of a combination priced already
    I512 c[KMAX];
    bool small = true;
    for (int u = 0; u < K && small; u++) {
      c[u] = i_zero();
      for (int i = 0; i < K; i++)
        if (cf[i]) c[u] = i_add(c[u], mult[i][cf[i] + CR][u]);
      small = i_bits(c[u]) < 253;
    }
    if (!small) continue;
    const double cost = chain_cost(c, K);
    if (!(cost < best)) continue;
    if (zl_is_zero(zl_of(c[0]))) continue;  // b must be invertible mod l ((l, 0, .., 0) is not)
    best = cost;
    have = true;
    for (int u = 0; u < K; u++) win[u] = c[u];
  }
  if (have) {
    const Zl b = zl_of(win[0]);
    bool ok = true;  // a_u == b y^u (mod l), exactly
    for (int u = 1; u < K && ok; u++) ok = zl_is_zero(zl_sub(zl_of(win[u]), zl_mul(b, pw[u])));
    const bool flip = i_neg_p(win[0]);  // b > 0
    if (ok)
      for (int u = 0; u < K; u++) v[u] = flip ? i_neg(win[u]) : win[u];
  }
  for (int u = 0; u < K; u++) {
    sign[u] = i_neg_p(v[u]) ? -1 : 1;
    const I512 m = sign[u] < 0 ? i_neg(v[u]) : v[u];
    for (int i = 0; i < 32; i++) mag[u][i] = (uint8_t)(m.w[i / 8] >> (8 * (i % 8)));
  }
  return true;
}

}  // namespace dkgh
