/* dkg-amd CPU ORACLE internals (test infrastructure only; see oracle.h). */
#ifndef DKG_ORACLE_INT_H
#define DKG_ORACLE_INT_H
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include "oracle.h"

typedef struct { uint64_t v[5]; } fe51;          /* 5 x 51-bit limbs */
typedef struct { uint64_t v[5]; } sc52;          /* 5 x 52-bit limbs, Z_l */
typedef struct { fe51 X, Y, Z, T; } ge_ext;      /* extended */
typedef struct { fe51 X, Y, Z; } ge_proj;        /* projective */
typedef struct { fe51 X, Y, Z, T; } ge_comp;     /* completed ((X:Z),(Y:T)) */
typedef struct { fe51 YpX, YmX, Z, T2d; } ge_pniels;

extern const fe51 FE51_ZERO, FE51_ONE, FE51_D, FE51_D2, FE51_SQRT_M1, FE51_SQRT_AD_MINUS_ONE,
    FE51_INVSQRT_A_MINUS_D, FE51_ONE_MINUS_D_SQ, FE51_D_MINUS_ONE_SQ;

void fe51_frombytes(fe51 *r, const uint8_t s[32]);
void fe51_tobytes(uint8_t s[32], const fe51 *a);
void fe51_add(fe51 *r, const fe51 *a, const fe51 *b);
void fe51_sub(fe51 *r, const fe51 *a, const fe51 *b);
void fe51_neg(fe51 *r, const fe51 *a);
void fe51_mul(fe51 *r, const fe51 *a, const fe51 *b);
void fe51_sq(fe51 *r, const fe51 *a);
void fe51_invert(fe51 *r, const fe51 *z);
int fe51_isneg(const fe51 *a);
int fe51_iszero(const fe51 *a);
int fe51_eq(const fe51 *a, const fe51 *b);
void fe51_abs(fe51 *r, const fe51 *a);
int fe51_sqrt_ratio_m1(fe51 *r, const fe51 *u, const fe51 *v);

void sc52_unpack(sc52 *r, const uint8_t s[32]);
void sc52_pack(uint8_t s[32], const sc52 *a);
void sc52_mul(sc52 *r, const sc52 *a, const sc52 *b);
void sc52_add(sc52 *r, const sc52 *a, const sc52 *b);
void sc52_sub(sc52 *r, const sc52 *a, const sc52 *b);

void ge_identity(ge_ext *p);
int ge_decode(ge_ext *p, const uint8_t s[32]);
void ge_encode(uint8_t s[32], const ge_ext *p);
int ge_eq(const ge_ext *p, const ge_ext *q);
void ge_add_ext(ge_ext *r, const ge_ext *p, const ge_ext *q);
void ge_sub_ext(ge_ext *r, const ge_ext *p, const ge_ext *q);
void ge_mul_vartime_base(ge_ext *r, const ge_ext *p, const uint8_t s[32]);
void ge_msm(ge_ext *r, size_t n, const uint8_t *scalars, const ge_ext *points);
void ge_base_point(ge_ext *p);
void ge_from_uniform(ge_ext *p, const uint8_t in[64]);
#endif
