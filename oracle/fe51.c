/*
 * dkg-amd CPU ORACLE (test infrastructure only; see oracle.h).
 * GF(2^255-19) with five 51-bit limbs and unsigned __int128 products — the representation
 * of curve25519-dalek 3.x `u64_backend::field::FieldElement51` [dalek-3.x, external], which the
 * reference's group operations run on (groups.rs:55-90).
 */
#include "oracle_int.h"

#define M51 ((1ULL << 51) - 1)

void fe51_frombytes(fe51 *r, const uint8_t s[32]) {
  uint64_t w[4];
  for (int i = 0; i < 4; i++) {
    w[i] = 0;
    for (int j = 7; j >= 0; j--) w[i] = (w[i] << 8) | s[8 * i + j];
  }
  r->v[0] = w[0] & M51;
  r->v[1] = ((w[0] >> 51) | (w[1] << 13)) & M51;
  r->v[2] = ((w[1] >> 38) | (w[2] << 26)) & M51;
  r->v[3] = ((w[2] >> 25) | (w[3] << 39)) & M51;
  r->v[4] = (w[3] >> 12) & M51; /* bit 255 ignored */
}

static void fe51_weak(fe51 *r) {
  uint64_t c;
  c = r->v[0] >> 51; r->v[0] &= M51; r->v[1] += c;
  c = r->v[1] >> 51; r->v[1] &= M51; r->v[2] += c;
  c = r->v[2] >> 51; r->v[2] &= M51; r->v[3] += c;
  c = r->v[3] >> 51; r->v[3] &= M51; r->v[4] += c;
  c = r->v[4] >> 51; r->v[4] &= M51; r->v[0] += 19 * c;
}

void fe51_tobytes(uint8_t s[32], const fe51 *a) {
  fe51 t = *a;
  fe51_weak(&t);
  fe51_weak(&t);
  /* t < 2^255 + 2^13ish; subtract p if t >= p */
  uint64_t q = (t.v[0] + 19) >> 51;
  q = (t.v[1] + q) >> 51;
  q = (t.v[2] + q) >> 51;
  q = (t.v[3] + q) >> 51;
  q = (t.v[4] + q) >> 51;
  t.v[0] += 19 * q;
  uint64_t c;
  c = t.v[0] >> 51; t.v[0] &= M51; t.v[1] += c;
  c = t.v[1] >> 51; t.v[1] &= M51; t.v[2] += c;
  c = t.v[2] >> 51; t.v[2] &= M51; t.v[3] += c;
  c = t.v[3] >> 51; t.v[3] &= M51; t.v[4] += c;
  t.v[4] &= M51;
  uint64_t w[4];
  w[0] = t.v[0] | (t.v[1] << 51);
  w[1] = (t.v[1] >> 13) | (t.v[2] << 38);
  w[2] = (t.v[2] >> 26) | (t.v[3] << 25);
  w[3] = (t.v[3] >> 39) | (t.v[4] << 12);
  for (int i = 0; i < 4; i++)
    for (int j = 0; j < 8; j++) s[8 * i + j] = (uint8_t)(w[i] >> (8 * j));
}

void fe51_add(fe51 *r, const fe51 *a, const fe51 *b) {
  for (int i = 0; i < 5; i++) r->v[i] = a->v[i] + b->v[i];
}

/* r = a - b; b limbs must be < 2^54 (16p bias) */
void fe51_sub(fe51 *r, const fe51 *a, const fe51 *b) {
  r->v[0] = (a->v[0] + 36028797018963664ULL) - b->v[0]; /* 16*(2^51-19) */
  for (int i = 1; i < 5; i++) r->v[i] = (a->v[i] + 36028797018963952ULL) - b->v[i]; /* 16*(2^51-1) */
  fe51_weak(r);
}

void fe51_neg(fe51 *r, const fe51 *a) {
  fe51 z = {{0, 0, 0, 0, 0}};
  fe51_sub(r, &z, a);
}

void fe51_mul(fe51 *r, const fe51 *a, const fe51 *b) {
  typedef unsigned __int128 u128;
  const uint64_t a0 = a->v[0], a1 = a->v[1], a2 = a->v[2], a3 = a->v[3], a4 = a->v[4];
  const uint64_t b0 = b->v[0], b1 = b->v[1], b2 = b->v[2], b3 = b->v[3], b4 = b->v[4];
  const uint64_t b1_19 = 19 * b1, b2_19 = 19 * b2, b3_19 = 19 * b3, b4_19 = 19 * b4;
  u128 c0 = (u128)a0 * b0 + (u128)a1 * b4_19 + (u128)a2 * b3_19 + (u128)a3 * b2_19 + (u128)a4 * b1_19;
  u128 c1 = (u128)a0 * b1 + (u128)a1 * b0 + (u128)a2 * b4_19 + (u128)a3 * b3_19 + (u128)a4 * b2_19;
  u128 c2 = (u128)a0 * b2 + (u128)a1 * b1 + (u128)a2 * b0 + (u128)a3 * b4_19 + (u128)a4 * b3_19;
  u128 c3 = (u128)a0 * b3 + (u128)a1 * b2 + (u128)a2 * b1 + (u128)a3 * b0 + (u128)a4 * b4_19;
  u128 c4 = (u128)a0 * b4 + (u128)a1 * b3 + (u128)a2 * b2 + (u128)a3 * b1 + (u128)a4 * b0;
  c1 += (uint64_t)(c0 >> 51);
  c2 += (uint64_t)(c1 >> 51);
  c3 += (uint64_t)(c2 >> 51);
  c4 += (uint64_t)(c3 >> 51);
  uint64_t carry = (uint64_t)(c4 >> 51);
  u128 t0 = (u128)((uint64_t)c0 & M51) + (u128)carry * 19;
  r->v[0] = (uint64_t)t0 & M51;
  r->v[1] = ((uint64_t)c1 & M51) + (uint64_t)(t0 >> 51);
  r->v[2] = (uint64_t)c2 & M51;
  r->v[3] = (uint64_t)c3 & M51;
  r->v[4] = (uint64_t)c4 & M51;
}

void fe51_sq(fe51 *r, const fe51 *a) { fe51_mul(r, a, a); }

static void fe51_sqn(fe51 *r, const fe51 *a, int n) {
  fe51_sq(r, a);
  for (int i = 1; i < n; i++) fe51_sq(r, r);
}

/* returns (t^(2^250-1), t^11) — shared prefix of invert and pow_p58 */
static void fe51_pow22501(fe51 *t19, fe51 *t3, const fe51 *z) {
  fe51 t0, t1, t2, t4, t5, t6, t7, t8, t9, t10, t11, t12, t13, t14, t15, t16, t17, t18;
  fe51_sq(&t0, z);            /* 2 */
  fe51_sqn(&t1, &t0, 2);      /* 8 */
  fe51_mul(&t2, z, &t1);      /* 9 */
  fe51_mul(t3, &t0, &t2);     /* 11 */
  fe51_sq(&t4, t3);           /* 22 */
  fe51_mul(&t5, &t2, &t4);    /* 31 = 2^5-1 */
  fe51_sqn(&t6, &t5, 5);
  fe51_mul(&t7, &t6, &t5);    /* 2^10-1 */
  fe51_sqn(&t8, &t7, 10);
  fe51_mul(&t9, &t8, &t7);    /* 2^20-1 */
  fe51_sqn(&t10, &t9, 20);
  fe51_mul(&t11, &t10, &t9);  /* 2^40-1 */
  fe51_sqn(&t12, &t11, 10);
  fe51_mul(&t13, &t12, &t7);  /* 2^50-1 */
  fe51_sqn(&t14, &t13, 50);
  fe51_mul(&t15, &t14, &t13); /* 2^100-1 */
  fe51_sqn(&t16, &t15, 100);
  fe51_mul(&t17, &t16, &t15); /* 2^200-1 */
  fe51_sqn(&t18, &t17, 50);
  fe51_mul(t19, &t18, &t13);  /* 2^250-1 */
}

void fe51_invert(fe51 *r, const fe51 *z) {
  fe51 t19, t3, t20;
  fe51_pow22501(&t19, &t3, z);
  fe51_sqn(&t20, &t19, 5);
  fe51_mul(r, &t20, &t3); /* 2^255 - 21 */
}

static void fe51_pow_p58(fe51 *r, const fe51 *z) {
  fe51 t19, t3, t20;
  fe51_pow22501(&t19, &t3, z);
  fe51_sqn(&t20, &t19, 2);
  fe51_mul(r, z, &t20); /* 2^252 - 3 */
}

int fe51_isneg(const fe51 *a) {
  uint8_t s[32];
  fe51_tobytes(s, a);
  return s[0] & 1;
}

int fe51_iszero(const fe51 *a) {
  uint8_t s[32];
  fe51_tobytes(s, a);
  uint8_t o = 0;
  for (int i = 0; i < 32; i++) o |= s[i];
  return o == 0;
}

int fe51_eq(const fe51 *a, const fe51 *b) {
  uint8_t s[32], t[32];
  fe51_tobytes(s, a);
  fe51_tobytes(t, b);
  return memcmp(s, t, 32) == 0;
}

void fe51_abs(fe51 *r, const fe51 *a) {
  if (fe51_isneg(a)) fe51_neg(r, a);
  else *r = *a;
}

/* RFC 9496 SQRT_RATIO_M1 */
int fe51_sqrt_ratio_m1(fe51 *r, const fe51 *u, const fe51 *v) {
  fe51 v3, v7, t, chk, nu, nui;
  fe51_sq(&v3, v);
  fe51_mul(&v3, &v3, v);
  fe51_sq(&v7, &v3);
  fe51_mul(&v7, &v7, v);
  fe51_mul(&t, u, &v7);
  fe51_pow_p58(&t, &t);
  fe51_mul(&t, &t, &v3);
  fe51_mul(r, &t, u);
  fe51_sq(&chk, r);
  fe51_mul(&chk, &chk, v);
  fe51_neg(&nu, u);
  fe51_mul(&nui, &nu, &FE51_SQRT_M1);
  int correct = fe51_eq(&chk, u);
  int flipped = fe51_eq(&chk, &nu);
  int flipped_i = fe51_eq(&chk, &nui);
  if (flipped || flipped_i) fe51_mul(r, r, &FE51_SQRT_M1);
  fe51_abs(r, r);
  return correct || flipped;
}

const fe51 FE51_ZERO = {{0, 0, 0, 0, 0}};
const fe51 FE51_ONE = {{1, 0, 0, 0, 0}};
const fe51 FE51_D = {{0x34dca135978a3ULL, 0x1a8283b156ebdULL, 0x5e7a26001c029ULL, 0x739c663a03cbbULL,
                      0x52036cee2b6ffULL}};
const fe51 FE51_D2 = {{0x69b9426b2f159ULL, 0x35050762add7aULL, 0x3cf44c0038052ULL,
                       0x6738cc7407977ULL, 0x2406d9dc56dffULL}};
const fe51 FE51_SQRT_M1 = {{0x61b274a0ea0b0ULL, 0xd5a5fc8f189dULL, 0x7ef5e9cbd0c60ULL,
                            0x78595a6804c9eULL, 0x2b8324804fc1dULL}};
const fe51 FE51_SQRT_AD_MINUS_ONE = {{0x7f6a0497b2e1bULL, 0x1836f0a97afd2ULL, 0x7d747f6be7638ULL,
                                      0x456079e7e6498ULL, 0x376931bf2b834ULL}};
const fe51 FE51_INVSQRT_A_MINUS_D = {{0xfdaa805d40eaULL, 0x2eb482e57d339ULL, 0x7610274bc58ULL,
                                      0x6510b613dc8ffULL, 0x786c8905cfaffULL}};
const fe51 FE51_ONE_MINUS_D_SQ = {{0x409c1945fc176ULL, 0x719abc6a1fc4fULL, 0x1c37f90b20684ULL,
                                   0x6bccca55eedfULL, 0x29072a8b2b3eULL}};
const fe51 FE51_D_MINUS_ONE_SQ = {{0x55aaa44ed4d20ULL, 0x59603c3332635ULL, 0x26d3baf4a7928ULL,
                                   0x120a66e6997a9ULL, 0x5968b37af66c2ULL}};
