/*
 * dkg-amd CPU ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C restatement of the reference's hot path (danielSanchezQ/dkg @ 2025-01-17):
 * Pedersen-VSS share generation and the receiver share checks over Ristretto255, with
 * the group arithmetic algorithm-matched to curve25519-dalek 3.x `u64_backend`
 * (5x51-bit field limbs, 5x52-bit Montgomery scalars, radix-16 variable-base mul,
 * Straus NAF-5 / Pippenger w=6,7,8 vartime MSM), which the reference reaches through
 * /root/reference/src/groups.rs:11-90.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this
 * library, and only as the checker (or the timed CPU baseline) — never as the product.
 * Parity of this oracle is pinned by tests/golden/ fixtures generated from libsodium
 * 1.0.18 (an independent RFC 9496 implementation) and a pure-Python big-int restatement.
 */
#ifndef DKG_ORACLE_H
#define DKG_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- hashing / RNG (blake2 0.9.1 `Blake2b` = BLAKE2b-512; rand ChaCha20Rng stream) ---- */
void or_blake2b(uint8_t *out, size_t outlen, const uint8_t *in, size_t inlen);
void or_chacha20_stream(const uint8_t key[32], uint64_t first_block, uint8_t *out, size_t len);

/* ---- scalar field Z_l (dalek Scalar; groups.rs:11-53) ---- */
void or_sc_reduce_wide(uint8_t out[32], const uint8_t in[64]);  /* from_bytes_mod_order_wide */
void or_sc_reduce(uint8_t out[32], const uint8_t in[32]);       /* x mod l for any 256-bit x */
void or_sc_from_u64(uint8_t out[32], uint64_t x);               /* groups.rs:19-21 */
void or_sc_add(uint8_t out[32], const uint8_t a[32], const uint8_t b[32]);
void or_sc_sub(uint8_t out[32], const uint8_t a[32], const uint8_t b[32]);
void or_sc_mul(uint8_t out[32], const uint8_t a[32], const uint8_t b[32]);
void or_sc_neg(uint8_t out[32], const uint8_t a[32]);
void or_sc_invert(uint8_t out[32], const uint8_t a[32]);        /* groups.rs:46-48 */

/* ---- group (RistrettoPoint; groups.rs:55-90). Points are 32-byte compressed encodings.
 * Functions returning int give 0 on success, -1 when an input point fails to decode
 * (dalek `CompressedRistretto::decompress` -> None, groups.rs:78-81). ---- */
int  or_pt_valid(const uint8_t p[32]);
void or_pt_base(uint8_t out[32]);
void or_pt_identity(uint8_t out[32]);
void or_pt_hash_to_group(uint8_t out[32], const uint8_t *in, size_t inlen); /* groups.rs:68-70 */
void or_pt_from_uniform_bytes(uint8_t out[32], const uint8_t in[64]);
int  or_pt_add(uint8_t out[32], const uint8_t a[32], const uint8_t b[32]);
int  or_pt_sub(uint8_t out[32], const uint8_t a[32], const uint8_t b[32]);
int  or_pt_neg(uint8_t out[32], const uint8_t a[32]);
int  or_pt_mul(uint8_t out[32], const uint8_t p[32], const uint8_t s[32]); /* variable-base, radix 16 */
void or_pt_base_mul(uint8_t out[32], const uint8_t s[32]);                 /* generator() * s */
int  or_pt_eq(const uint8_t a[32], const uint8_t b[32]);                   /* 1 equal, 0 not, -1 decode */
/* vartime_multiscalar_multiplication (traits.rs:234-237 -> dalek Straus N<190 / Pippenger). */
int  or_msm(uint8_t out[32], size_t N, const uint8_t *scalars, const uint8_t *points);

/* ---- polynomial (polynomial.rs:59-74) ---- */
/* power-sum evaluation sum_k c_k x^k exactly as Polynomial::evaluate */
void or_poly_eval(uint8_t out[32], const uint8_t *coeffs, size_t ncoeffs, const uint8_t x[32]);

/* ---- ceremony pieces (committee.rs) ---- */
/* Per-dealer seed: BLAKE2b-256("dkg-amd/v1/dealer" || master[32] || u32le ceremony || u32le dealer) */
void or_dealer_seed(uint8_t out[32], const uint8_t master[32], uint32_t ceremony, uint32_t dealer);
/* Polynomial::random x2 from a ChaCha20Rng(seed): hiding b_0..b_t FIRST, then sharing a_0..a_t
 * (committee.rs:143-146); each Scalar::random draws 64 bytes and wide-reduces. */
void or_dealer_coeffs(const uint8_t seed[32], size_t t, uint8_t *a, uint8_t *b);
/* Round 1 for dealers [0,D): a,b: [D][t+1][32]; E,A: [D][t+1][32]; s,sp: [D][n][32]
 * E_k = h*b_k + g*a_k, A_k = g*a_k (committee.rs:151-159); s = f(j), s' = f'(j), j=1..n (:164-167). */
void or_share_gen(size_t D, size_t n, size_t t, const uint8_t *a, const uint8_t *b,
                  const uint8_t h[32], uint8_t *E, uint8_t *A, uint8_t *s, uint8_t *sp, int nthreads);
/* Round-2 (round=2, committee.rs:287-305) / round-4 (round=4, h unused, :532-541) checks for
 * dealers [d0,d1) x receivers [r0,r1), computed as the reference does: lhs = h*s' + g*s (or g*s),
 * rhs = vartime MSM(j^0..j^t, C_i). C: [n][t+1][32]; s, sp: [n dealer][n receiver][32].
 * accept: byte matrix [d1-d0][r1-r0]; 1 = equal, 0 = reject, 2 = self (i == j, not checked).
 * Returns -1 if a commitment fails to decode: its dealer is missing data, so its row reads 4
 * (DKG_MISSING: disqualified without a complaint, committee.rs:331-335) in round 2 and 0 in round 4. */
int or_verify_pairs(size_t n, size_t t, int round, const uint8_t *C, const uint8_t h[32],
                    const uint8_t *s, const uint8_t *sp, size_t d0, size_t d1, size_t r0, size_t r1,
                    uint8_t *accept, int nthreads);
/* The same on row-local arrays (one rank's block of a sharded run): C [d1-d0][t+1][32],
 * s, sp [d1-d0][n][32]; dealer indices (the SELF diagonal i == j) stay global. */
int or_verify_pairs_rows(size_t n, size_t t, int round, const uint8_t *C, const uint8_t h[32],
                         const uint8_t *s, const uint8_t *sp, size_t d0, size_t d1, size_t r0, size_t r1,
                         uint8_t *accept, int nthreads);
/* ---- full (encrypted-share) mode: hybrid.c (elgamal.rs, procedure_keys.rs) ---- */
/* bench.py's full-mode CPU baseline: seconds per encrypt + decrypt of one 32-byte share */
double or_bench_hybrid(size_t items, int nthreads);
void or_chacha20_ietf_xor(uint8_t *out, const uint8_t *in, size_t len, const uint8_t key[32],
                          const uint8_t nonce[12]);
/* e1 = G r, e2 = msg XOR ChaCha20(Blake2b-512(pk r)) (elgamal.rs:134-145, 172-193); -1 if pk is invalid */
int or_hybrid_encrypt(uint8_t e1[32], uint8_t *e2, const uint8_t pk[32], const uint8_t r[32], const uint8_t *msg,
                      size_t len);
/* msg = e2 XOR ChaCha20(Blake2b-512(e1 sk)) (elgamal.rs:161-170); -1 if e1 does not decode */
int or_hybrid_decrypt(uint8_t *msg, const uint8_t sk[32], const uint8_t e1[32], const uint8_t *e2, size_t len);
void or_member_sk(uint8_t sk[32], const uint8_t master[32], uint32_t ceremony, uint32_t member);
void or_enc_randomness(uint8_t *r, const uint8_t seed[32], size_t t, size_t n);
/* ---- complaint proofs (hybrid.c; dl_equality/zkp.rs, broadcast.rs) ---- */
void or_hash_to_scalar(uint8_t out[32], const uint8_t *in, size_t len); /* groups.rs:50-52 */
int or_dleq_prove(uint8_t c[32], uint8_t r[32], const uint8_t b1[32], const uint8_t b2[32], const uint8_t p1[32],
                  const uint8_t p2[32], const uint8_t dlog[32], const uint8_t w[32]);
int or_dleq_verify(const uint8_t b1[32], const uint8_t b2[32], const uint8_t p1[32], const uint8_t p2[32],
                   const uint8_t c[32], const uint8_t r[32]);
/* enc = e1_rand || ct_rand || e1_share || ct_share; proof = share_key || randomness_key || c1 || r1 || c2 || r2 */
int or_misbehaviour_prove(uint8_t proof[192], const uint8_t sk[32], const uint8_t enc[128], const uint8_t w[64]);
int or_complaint1_verify(const uint8_t h[32], size_t t, uint32_t accuser, const uint8_t pk[32], const uint8_t enc[128],
                         const uint8_t *E, const uint8_t proof[192]);
int or_complaint3_verify(const uint8_t h[32], size_t t, uint32_t accuser, const uint8_t share[32],
                         const uint8_t randomness[32], const uint8_t *E, const uint8_t *A);
/* Lagrange interpolation at x (polynomial.rs:162-184). */
void or_lagrange(uint8_t out[32], const uint8_t x[32], const uint8_t *ys, const uint8_t *xs, size_t m);
/* single-thread cost calibration (bench.py cpu_baseline): ns per field multiplication, ms per MSM */
double or_bench_fe_mul(uint64_t iters);
double or_bench_msm(size_t N, int reps);

#ifdef __cplusplus
}
#endif
#endif
