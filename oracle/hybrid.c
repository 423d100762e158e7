/*
 * dkg-amd CPU ORACLE — TEST INFRASTRUCTURE ONLY (see oracle.h).
 * Full (encrypted-share) mode of the reference: the hybrid ElGamal + ChaCha20 scheme of
 * /root/reference/src/cryptography/elgamal.rs and the member communication keys of
 * src/dkg/procedure_keys.rs, restated on this oracle's dalek-matched group arithmetic.
 * Third-party pieces (absent here, pinned via libsodium fixtures): chacha20 0.7.2 `ChaCha20`
 * (RFC 8439 IETF variant: 96-bit nonce, 32-bit block counter from 0) and blake2 0.9.1 `Blake2b`
 * (BLAKE2b-512).
 */
#include <stdlib.h>
#include <string.h>
#include <time.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "oracle.h"

static uint32_t rd32(const uint8_t *p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
static uint32_t rotl(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }

/* RFC 8439 block: constants, key, counter (word 12), nonce (words 13-15). */
static void chacha_ietf_block(uint8_t out[64], const uint8_t key[32], uint32_t counter, const uint8_t nonce[12]) {
  uint32_t s[16], x[16];
  s[0] = 0x61707865u; s[1] = 0x3320646eu; s[2] = 0x79622d32u; s[3] = 0x6b206574u;
  for (int i = 0; i < 8; i++) s[4 + i] = rd32(key + 4 * i);
  s[12] = counter;
  for (int i = 0; i < 3; i++) s[13 + i] = rd32(nonce + 4 * i);
  memcpy(x, s, sizeof s);
#define QR(a, b, c, d)                       \
  a += b; d ^= a; d = rotl(d, 16);           \
  c += d; b ^= c; b = rotl(b, 12);           \
  a += b; d ^= a; d = rotl(d, 8);            \
  c += d; b ^= c; b = rotl(b, 7);
  for (int r = 0; r < 10; r++) {
    QR(x[0], x[4], x[8], x[12]);
    QR(x[1], x[5], x[9], x[13]);
    QR(x[2], x[6], x[10], x[14]);
    QR(x[3], x[7], x[11], x[15]);
    QR(x[0], x[5], x[10], x[15]);
    QR(x[1], x[6], x[11], x[12]);
    QR(x[2], x[7], x[8], x[13]);
    QR(x[3], x[4], x[9], x[14]);
  }
#undef QR
  for (int i = 0; i < 16; i++) {
    uint32_t v = x[i] + s[i];
    for (int b = 0; b < 4; b++) out[4 * i + b] = (uint8_t)(v >> (8 * b));
  }
}

void or_chacha20_ietf_xor(uint8_t *out, const uint8_t *in, size_t len, const uint8_t key[32],
                          const uint8_t nonce[12]) {
  uint8_t blk[64];
  uint32_t ctr = 0;
  while (len) {
    chacha_ietf_block(blk, key, ctr++, nonce);
    size_t n = len < 64 ? len : 64;
    for (size_t i = 0; i < n; i++) out[i] = in[i] ^ blk[i];
    out += n;
    in += n;
    len -= n;
  }
}

/* SymmetricKey::process (elgamal.rs:172-193): Blake2b-512(K.to_bytes()) -> key h[0..32],
 * nonce h[32..44]; XOR the ChaCha20 keystream. */
static void sym_process(uint8_t *out, const uint8_t *in, size_t len, const uint8_t K[32]) {
  uint8_t h[64];
  or_blake2b(h, 64, K, 32);
  or_chacha20_ietf_xor(out, in, len, h, h + 32);
}

/* PublicKey::hybrid_encrypt with the randomness given (elgamal.rs:134-145):
 * e1 = G * r, e2 = process(pk * r, msg). */
int or_hybrid_encrypt(uint8_t e1[32], uint8_t *e2, const uint8_t pk[32], const uint8_t r[32], const uint8_t *msg,
                      size_t len) {
  uint8_t K[32];
  if (or_pt_mul(K, pk, r)) return -1;
  or_pt_base_mul(e1, r);
  sym_process(e2, msg, len, K);
  return 0;
}

/* SecretKey::hybrid_decrypt (elgamal.rs:161-170): process(e1 * sk, e2). */
int or_hybrid_decrypt(uint8_t *msg, const uint8_t sk[32], const uint8_t e1[32], const uint8_t *e2, size_t len) {
  uint8_t K[32];
  if (or_pt_mul(K, e1, sk)) return -1;
  sym_process(msg, e2, len, K);
  return 0;
}

/* Seeded MemberCommunicationKey (procedure_keys.rs:72-82): sk = wide(ChaCha20Rng(seed) block 0),
 * seed = BLAKE2b-256("dkg-amd/v1/member" || master || u32le ceremony || u32le member). */
void or_member_sk(uint8_t sk[32], const uint8_t master[32], uint32_t ceremony, uint32_t member) {
  static const char tag[] = "dkg-amd/v1/member";
  uint8_t msg[sizeof tag - 1 + 40], seed[32], st[64];
  memcpy(msg, tag, sizeof tag - 1);
  memcpy(msg + sizeof tag - 1, master, 32);
  for (int k = 0; k < 4; k++) {
    msg[sizeof tag - 1 + 32 + k] = (uint8_t)(ceremony >> (8 * k));
    msg[sizeof tag - 1 + 36 + k] = (uint8_t)(member >> (8 * k));
  }
  or_blake2b(seed, 32, msg, sizeof msg);
  or_chacha20_stream(seed, 0, st, 64);
  or_sc_reduce_wide(sk, st);
}

/* Encryption randomness of dealer `seed` for n recipients (committee.rs:171-172 draw order, after
 * the 2(t+1) coefficient draws): r[q][0] for the randomness ciphertext, r[q][1] for the share. */
void or_enc_randomness(uint8_t *r, const uint8_t seed[32], size_t t, size_t n) {
  uint8_t blk[64];
  for (size_t q = 0; q < 2 * n; q++) {
    or_chacha20_stream(seed, 2 * (t + 1) + q, blk, 64);
    or_sc_reduce_wide(r + 32 * q, blk);
  }
}

/* ---------------- complaint proofs ---------------- */

/* Scalar::hash_from_bytes::<Blake2b> (groups.rs:50-52): wide reduction of Blake2b-512. */
void or_hash_to_scalar(uint8_t out[32], const uint8_t *in, size_t len) {
  uint8_t h[64];
  or_blake2b(h, 64, in, len);
  or_sc_reduce_wide(out, h);
}

/* challenge of ChallengeContext (challenge_context.rs:14-41): H(b1 || b2 || p1 || p2 || a1 || a2) */
static void dleq_challenge(uint8_t c[32], const uint8_t *b1, const uint8_t *b2, const uint8_t *p1, const uint8_t *p2,
                           const uint8_t *a1, const uint8_t *a2) {
  uint8_t buf[192];
  memcpy(buf, b1, 32);
  memcpy(buf + 32, b2, 32);
  memcpy(buf + 64, p1, 32);
  memcpy(buf + 96, p2, 32);
  memcpy(buf + 128, a1, 32);
  memcpy(buf + 160, a2, 32);
  or_hash_to_scalar(c, buf, 192);
}

/* DleqZkp::generate (dl_equality/zkp.rs:29-49) with the nonce w given. */
int or_dleq_prove(uint8_t c[32], uint8_t r[32], const uint8_t b1[32], const uint8_t b2[32], const uint8_t p1[32],
                  const uint8_t p2[32], const uint8_t dlog[32], const uint8_t w[32]) {
  uint8_t a1[32], a2[32], cd[32];
  if (or_pt_mul(a1, b1, w) || or_pt_mul(a2, b2, w)) return -1;
  dleq_challenge(c, b1, b2, p1, p2, a1, a2);
  or_sc_mul(cd, c, dlog);
  or_sc_add(r, cd, w); /* response = challenge * dlog + w */
  return 0;
}

/* DleqZkp::verify (dl_equality/zkp.rs:52-74): 1 valid, 0 invalid, -1 decode failure. */
int or_dleq_verify(const uint8_t b1[32], const uint8_t b2[32], const uint8_t p1[32], const uint8_t p2[32],
                   const uint8_t c[32], const uint8_t r[32]) {
  uint8_t t1[32], t2[32], a1[32], a2[32], c2[32];
  if (or_pt_mul(t1, b1, r) || or_pt_mul(t2, p1, c) || or_pt_sub(a1, t1, t2)) return -1;
  if (or_pt_mul(t1, b2, r) || or_pt_mul(t2, p2, c) || or_pt_sub(a2, t1, t2)) return -1;
  dleq_challenge(c2, b1, b2, p1, p2, a1, a2);
  return memcmp(c2, c, 32) == 0;
}

/* ProofOfMisbehaviour::generate (broadcast.rs:189-226).  enc = e1_rand, ct_rand, e1_share, ct_share
 * (4 x 32 B); w[0] is the nonce of the share's decryption proof (drawn first), w[1] the
 * randomness's.  proof = share_key || randomness_key || c1 || r1 || c2 || r2 (192 B). */
int or_misbehaviour_prove(uint8_t proof[192], const uint8_t sk[32], const uint8_t enc[128], const uint8_t w[64]) {
  uint8_t pk[32], g[32];
  or_pt_base(g);
  or_pt_base_mul(pk, sk);
  const uint8_t *e1r = enc, *e1s = enc + 64;
  if (or_pt_mul(proof, e1s, sk) || or_pt_mul(proof + 32, e1r, sk)) return -1;  /* recover_symmetric_key */
  /* CorrectHybridDecrKeyZkp::generate (correct_hybrid_decryption_key/zkp.rs:27-47):
   * DLEQ(g, e1, pk, K) with witness sk */
  if (or_dleq_prove(proof + 64, proof + 96, g, e1s, pk, proof, sk, w)) return -1;
  if (or_dleq_prove(proof + 128, proof + 160, g, e1r, pk, proof + 32, sk, w + 32)) return -1;
  return 0;
}

static void sym_scalar(uint8_t out[32], const uint8_t K[32], const uint8_t ct[32]) {
  uint8_t m[32];
  sym_process(m, ct, 32, K);
  m[31] &= 0x7f; /* from_bits (groups.rs:29-36), reduced */
  or_sc_reduce(out, m);
}

/* sum_k j^k C_k (the reference's vartime MSM with from_u64(j).exp_iter().take(t+1)) */
static int index_msm(uint8_t out[32], uint32_t j, size_t t, const uint8_t *C) {
  uint8_t *pw = (uint8_t *)malloc(32 * (t + 1)), x[32];
  or_sc_from_u64(x, j);
  or_sc_from_u64(pw, 1);
  for (size_t k = 1; k <= t; k++) or_sc_mul(pw + 32 * k, pw + 32 * (k - 1), x);
  int rc = or_msm(out, t + 1, pw, C);
  free(pw);
  return rc;
}

/* h*a + g*b */
static int hg(uint8_t out[32], const uint8_t h[32], const uint8_t a[32], const uint8_t b[32]) {
  uint8_t t1[32], t2[32];
  if (or_pt_mul(t1, h, a)) return -1;
  or_pt_base_mul(t2, b);
  return or_pt_add(out, t1, t2);
}

/* MisbehavingPartiesRound1::verify (broadcast.rs:50-99) with ProofOfMisbehaviour::verify
 * (:228-283).  0 Ok (valid complaint), 1 InvalidProofOfMisbehaviour, 2 FalseClaimedInequality,
 * -1 a point does not decode. */
int or_complaint1_verify(const uint8_t h[32], size_t t, uint32_t accuser, const uint8_t pk[32], const uint8_t enc[128],
                         const uint8_t *E, const uint8_t proof[192]) {
  uint8_t g[32], p1[32], p2[32], q[32], rhs[32];
  or_pt_base(g);
  const uint8_t *e1r = enc, *ctr = enc + 32, *e1s = enc + 64, *cts = enc + 96;
  int v1 = or_dleq_verify(g, e1s, pk, proof, proof + 64, proof + 96);
  int v2 = or_dleq_verify(g, e1r, pk, proof + 32, proof + 128, proof + 160);
  if (v1 < 0 || v2 < 0) return -1;
  if (!v1 || !v2) return 1;
  sym_scalar(p1, proof, cts);        /* plaintext_1: the share */
  sym_scalar(p2, proof + 32, ctr);   /* plaintext_2: the randomness */
  if (index_msm(rhs, accuser, t, E)) return -1;
  if (hg(q, h, p1, p2)) return -1;   /* quirk: h * share + g * randomness (broadcast.rs:271-274) */
  if (memcmp(q, rhs, 32) == 0) return 1;
  if (hg(q, h, p2, p1)) return -1;   /* the accusation: h * randomness + g * share (:87-96) */
  if (memcmp(q, rhs, 32) == 0) return 2;
  return 0;
}

/* MisbehavingPartiesRound3::verify (broadcast.rs:105-135): 0 Ok, 3 FalseClaimedEquality,
 * 2 FalseClaimedInequality, -1 decode failure. */
int or_complaint3_verify(const uint8_t h[32], size_t t, uint32_t accuser, const uint8_t share[32],
                         const uint8_t randomness[32], const uint8_t *E, const uint8_t *A) {
  uint8_t pass[32], fail[32], rE[32], rA[32];
  if (hg(pass, h, randomness, share) || index_msm(rE, accuser, t, E) || index_msm(rA, accuser, t, A)) return -1;
  or_pt_base_mul(fail, share);
  if (memcmp(pass, rE, 32) != 0) return 3;
  if (memcmp(fail, rA, 32) == 0) return 2;
  return 0;
}

/* ---- CPU baseline of full mode (bench.py --mode full): seconds per (encrypt + decrypt) of one
 * 32-byte share, as committee.rs:169-172 and :282-286 do them for every (dealer, recipient, w),
 * over `items` items on `nthreads` threads (recipients' keys cycle over 16 seeded members). */
double or_bench_hybrid(size_t items, int nthreads) {
  enum { K = 16 };
  uint8_t sk[K][32], pk[K][32], master[32] = {9};
  for (int j = 0; j < K; j++) {
    or_member_sk(sk[j], master, 0, (uint32_t)j);
    or_pt_base_mul(pk[j], sk[j]);
  }
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
  struct timespec a, b;
  int bad = 0;
  clock_gettime(CLOCK_MONOTONIC, &a);
#pragma omp parallel for schedule(static) reduction(| : bad)
  for (long long i = 0; i < (long long)items; i++) {
    uint8_t r[32], msg[32], e1[32], e2[32], back[32], seed[32] = {0};
    memcpy(seed, &i, sizeof i);
    or_chacha20_stream(seed, 0, r, 32);
    r[31] &= 0x0f;
    memcpy(msg, r, 32);
    msg[0] ^= 0x5a;
    const int q = (int)(i % K);
    bad |= or_hybrid_encrypt(e1, e2, pk[q], r, msg, 32);
    bad |= or_hybrid_decrypt(back, sk[q], e1, e2, 32);
    bad |= memcmp(back, msg, 32) != 0;
  }
  clock_gettime(CLOCK_MONOTONIC, &b);
  if (bad) return -1.0;
  return ((b.tv_sec - a.tv_sec) + 1e-9 * (b.tv_nsec - a.tv_nsec)) / (double)items;
}
