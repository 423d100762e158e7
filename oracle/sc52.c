/*
 * dkg-amd CPU ORACLE (test infrastructure only; see oracle.h).
 * Scalar field Z_l, l = 2^252 + 27742317777372353535851937790883648493, as five 52-bit limbs with
 * Montgomery multiplication (R = 2^260) — the algorithm of curve25519-dalek 3.x
 * `backend::serial::u64::scalar::Scalar52` [dalek-3.x, external] behind the reference's
 * `impl Scalar for RScalar` (groups.rs:11-53).  Products by R^2 leave Montgomery form.
 */
#include "oracle_int.h"

#define M52 ((1ULL << 52) - 1)
typedef unsigned __int128 u128;

static const sc52 SC_L = {{0x2631a5cf5d3edULL, 0xdea2f79cd6581ULL, 0x14def9ULL, 0x0ULL, 0x100000000000ULL}};
static const uint64_t SC_LFACTOR = 0x51da312547e1bULL; /* -l^-1 mod 2^52 */
static const sc52 SC_R = {{0xf48bd6721e6edULL, 0x3bab5ac67e45aULL, 0xfffffeb35e51bULL, 0xfffffffffffffULL,
                           0xfffffffffffULL}}; /* 2^260 mod l */
static const sc52 SC_RR = {{0x9d265e952d13bULL, 0xd63c715bea69fULL, 0x5be65cb687604ULL, 0x3dceec73d217fULL,
                            0x9411b7c309aULL}}; /* 2^520 mod l */

static void bytes_to_words(uint64_t *w, const uint8_t *s, int nwords) {
  for (int i = 0; i < nwords; i++) {
    w[i] = 0;
    for (int j = 7; j >= 0; j--) w[i] = (w[i] << 8) | s[8 * i + j];
  }
}

void sc52_unpack(sc52 *r, const uint8_t s[32]) {
  uint64_t w[4];
  bytes_to_words(w, s, 4);
  r->v[0] = w[0] & M52;
  r->v[1] = ((w[0] >> 52) | (w[1] << 12)) & M52;
  r->v[2] = ((w[1] >> 40) | (w[2] << 24)) & M52;
  r->v[3] = ((w[2] >> 28) | (w[3] << 36)) & M52;
  r->v[4] = (w[3] >> 16) & ((1ULL << 48) - 1);
}

void sc52_pack(uint8_t s[32], const sc52 *a) {
  uint64_t w[4];
  w[0] = a->v[0] | (a->v[1] << 52);
  w[1] = (a->v[1] >> 12) | (a->v[2] << 40);
  w[2] = (a->v[2] >> 24) | (a->v[3] << 28);
  w[3] = (a->v[3] >> 36) | (a->v[4] << 16);
  for (int i = 0; i < 4; i++)
    for (int j = 0; j < 8; j++) s[8 * i + j] = (uint8_t)(w[i] >> (8 * j));
}

/* r = a - b mod l for a, b < l (also used as the final conditional subtraction) */
void sc52_sub(sc52 *r, const sc52 *a, const sc52 *b) {
  uint64_t d[5], borrow = 0;
  for (int i = 0; i < 5; i++) {
    borrow = a->v[i] - (b->v[i] + (borrow >> 63));
    d[i] = borrow & M52;
  }
  /* borrow >> 63 == 1 iff a < b: add l back */
  uint64_t mask = 0 - (borrow >> 63), carry = 0;
  for (int i = 0; i < 5; i++) {
    carry = (carry >> 52) + d[i] + (SC_L.v[i] & mask);
    r->v[i] = carry & M52;
  }
}

void sc52_add(sc52 *r, const sc52 *a, const sc52 *b) {
  sc52 s;
  uint64_t carry = 0;
  for (int i = 0; i < 5; i++) {
    carry = a->v[i] + b->v[i] + (carry >> 52);
    s.v[i] = carry & M52;
  }
  sc52_sub(r, &s, &SC_L);
}

/* Montgomery reduction of a 9-limb product t (each < 2^108 + carries): returns t / R mod l. */
static void sc52_mont_reduce(sc52 *r, const u128 t[9]) {
  u128 acc[10];
  for (int i = 0; i < 9; i++) acc[i] = t[i];
  acc[9] = 0;
  uint64_t n[5];
  for (int i = 0; i < 5; i++) {
    /* n_i makes limb i vanish: n_i = acc_i * (-l^-1) mod 2^52 */
    n[i] = ((uint64_t)acc[i] * SC_LFACTOR) & M52;
    for (int j = 0; j < 5; j++) acc[i + j] += (u128)n[i] * SC_L.v[j];
    acc[i + 1] += acc[i] >> 52;
  }
  sc52 s;
  u128 c = 0;
  for (int i = 0; i < 5; i++) {
    c += acc[5 + i];
    s.v[i] = (uint64_t)c & M52;
    c >>= 52;
  }
  sc52_sub(r, &s, &SC_L);
}

static void sc52_mul_internal(u128 t[9], const sc52 *a, const sc52 *b) {
  for (int i = 0; i < 9; i++) t[i] = 0;
  for (int i = 0; i < 5; i++)
    for (int j = 0; j < 5; j++) t[i + j] += (u128)a->v[i] * b->v[j];
}

static void sc52_mont_mul(sc52 *r, const sc52 *a, const sc52 *b) {
  u128 t[9];
  sc52_mul_internal(t, a, b);
  sc52_mont_reduce(r, t);
}

/* r = a * b mod l (dalek: montgomery_mul(montgomery_mul(a, b), RR)) */
void sc52_mul(sc52 *r, const sc52 *a, const sc52 *b) {
  sc52 ab;
  sc52_mont_mul(&ab, a, b);
  sc52_mont_mul(r, &ab, &SC_RR);
}

/* from_bytes_mod_order_wide: 64 bytes as lo (260 bits) + hi * 2^260 */
void or_sc_reduce_wide(uint8_t out[32], const uint8_t in[64]) {
  uint64_t w[8];
  bytes_to_words(w, in, 8);
  sc52 lo, hi;
  lo.v[0] = w[0] & M52;
  lo.v[1] = ((w[0] >> 52) | (w[1] << 12)) & M52;
  lo.v[2] = ((w[1] >> 40) | (w[2] << 24)) & M52;
  lo.v[3] = ((w[2] >> 28) | (w[3] << 36)) & M52;
  lo.v[4] = ((w[3] >> 16) | (w[4] << 48)) & M52;
  hi.v[0] = (w[4] >> 4) & M52;
  hi.v[1] = ((w[4] >> 56) | (w[5] << 8)) & M52;
  hi.v[2] = ((w[5] >> 44) | (w[6] << 20)) & M52;
  hi.v[3] = ((w[6] >> 32) | (w[7] << 32)) & M52;
  hi.v[4] = w[7] >> 20;
  sc52 a, b, r;
  sc52_mont_mul(&a, &lo, &SC_R);  /* lo * R / R = lo mod l */
  sc52_mont_mul(&b, &hi, &SC_RR); /* hi * R^2 / R = hi * R mod l */
  sc52_add(&r, &a, &b);
  sc52_pack(out, &r);
}

void or_sc_reduce(uint8_t out[32], const uint8_t in[32]) {
  uint8_t w[64];
  memcpy(w, in, 32);
  memset(w + 32, 0, 32);
  or_sc_reduce_wide(out, w);
}

void or_sc_from_u64(uint8_t out[32], uint64_t x) {
  memset(out, 0, 32);
  for (int i = 0; i < 8; i++) out[i] = (uint8_t)(x >> (8 * i));
}

void or_sc_add(uint8_t out[32], const uint8_t a[32], const uint8_t b[32]) {
  sc52 x, y, r;
  sc52_unpack(&x, a);
  sc52_unpack(&y, b);
  sc52_add(&r, &x, &y);
  sc52_pack(out, &r);
}

void or_sc_sub(uint8_t out[32], const uint8_t a[32], const uint8_t b[32]) {
  sc52 x, y, r;
  sc52_unpack(&x, a);
  sc52_unpack(&y, b);
  sc52_sub(&r, &x, &y);
  sc52_pack(out, &r);
}

void or_sc_neg(uint8_t out[32], const uint8_t a[32]) {
  sc52 z = {{0, 0, 0, 0, 0}}, x, r;
  sc52_unpack(&x, a);
  sc52_sub(&r, &z, &x);
  sc52_pack(out, &r);
}

void or_sc_mul(uint8_t out[32], const uint8_t a[32], const uint8_t b[32]) {
  sc52 x, y, r;
  sc52_unpack(&x, a);
  sc52_unpack(&y, b);
  sc52_mul(&r, &x, &y);
  sc52_pack(out, &r);
}

/* a^(l-2) by square-and-multiply over the bits of l-2 (Fermat inversion) */
void or_sc_invert(uint8_t out[32], const uint8_t a[32]) {
  static const uint8_t LM2[32] = {0xeb, 0xd3, 0xf5, 0x5c, 0x1a, 0x63, 0x12, 0x58, 0xd6, 0x9c, 0xf7,
                                  0xa2, 0xde, 0xf9, 0xde, 0x14, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                                  0, 0, 0, 0x10};
  sc52 x, acc;
  sc52_unpack(&x, a);
  memset(&acc, 0, sizeof acc);
  acc.v[0] = 1;
  for (int i = 255; i >= 0; i--) {
    sc52_mul(&acc, &acc, &acc);
    if ((LM2[i >> 3] >> (i & 7)) & 1) sc52_mul(&acc, &acc, &x);
  }
  sc52_pack(out, &acc);
}
