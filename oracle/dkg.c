/*
 * dkg-amd CPU ORACLE (test infrastructure only; see oracle.h).
 * The reference's round-1 share generation and round-2 / round-4 share checks, restated
 * loop-for-loop from /root/reference/src/dkg/committee.rs and src/polynomial.rs, on top of the
 * dalek-matched group arithmetic in ge.c / sc52.c.  OpenMP parallelism over dealers/receivers is
 * the only addition (the reference is single-threaded); results do not depend on it.
 */
#include "oracle_int.h"
#ifdef _OPENMP
#include <omp.h>
#endif

/* Polynomial::evaluate (polynomial.rs:68-74): sum_k c_k * x^k with x^k from exp_iter
 * (traits.rs:172-197), folded left to right from zero. */
void or_poly_eval(uint8_t out[32], const uint8_t *coeffs, size_t ncoeffs, const uint8_t x[32]) {
  sc52 acc = {{0, 0, 0, 0, 0}}, xp = {{1, 0, 0, 0, 0}}, xs, c, term;
  sc52_unpack(&xs, x);
  for (size_t k = 0; k < ncoeffs; k++) {
    sc52_unpack(&c, coeffs + 32 * k);
    sc52_mul(&term, &c, &xp);
    sc52_add(&acc, &acc, &term);
    sc52_mul(&xp, &xp, &xs); /* ScalarExp::next: next = next * x */
  }
  sc52_pack(out, &acc);
}

void or_dealer_seed(uint8_t out[32], const uint8_t master[32], uint32_t ceremony, uint32_t dealer) {
  static const char tag[] = "dkg-amd/v1/dealer";
  uint8_t buf[sizeof tag - 1 + 32 + 8];
  memcpy(buf, tag, sizeof tag - 1);
  memcpy(buf + sizeof tag - 1, master, 32);
  for (int i = 0; i < 4; i++) {
    buf[sizeof tag - 1 + 32 + i] = (uint8_t)(ceremony >> (8 * i));
    buf[sizeof tag - 1 + 36 + i] = (uint8_t)(dealer >> (8 * i));
  }
  or_blake2b(out, 32, buf, sizeof buf);
}

/* committee.rs:143-146: hiding_polynomial drawn first, then sharing_polynomial; each
 * Polynomial::random (polynomial.rs:59-65) draws t+1 Scalar::random = 64 rng bytes, wide-reduced. */
void or_dealer_coeffs(const uint8_t seed[32], size_t t, uint8_t *a, uint8_t *b) {
  size_t nbytes = 2 * (t + 1) * 64;
  uint8_t *stream = malloc(nbytes);
  or_chacha20_stream(seed, 0, stream, nbytes);
  for (size_t k = 0; k <= t; k++) or_sc_reduce_wide(b + 32 * k, stream + 64 * k);
  for (size_t k = 0; k <= t; k++) or_sc_reduce_wide(a + 32 * k, stream + 64 * (t + 1 + k));
  free(stream);
}

static void set_threads(int nthreads) {
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#else
  (void)nthreads;
#endif
}

void or_share_gen(size_t D, size_t n, size_t t, const uint8_t *a, const uint8_t *b,
                  const uint8_t h[32], uint8_t *E, uint8_t *A, uint8_t *s, uint8_t *sp, int nthreads) {
  ge_ext hp, g;
  ge_decode(&hp, h);
  ge_base_point(&g);
  set_threads(nthreads);
  const size_t N = t + 1;
#pragma omp parallel for schedule(dynamic)
  for (long long q = 0; q < (long long)(D * N); q++) {
    size_t i = (size_t)q / N, k = (size_t)q % N;
    ge_ext apub, hb, e;
    /* committee.rs:155-156: apub = G::generator() * a; coeff_comm = h * b + apub */
    ge_mul_vartime_base(&apub, &g, a + 32 * (i * N + k));
    ge_mul_vartime_base(&hb, &hp, b + 32 * (i * N + k));
    ge_add_ext(&e, &hb, &apub);
    ge_encode(A + 32 * (i * N + k), &apub);
    ge_encode(E + 32 * (i * N + k), &e);
  }
#pragma omp parallel for schedule(dynamic)
  for (long long q = 0; q < (long long)(D * n); q++) {
    size_t i = (size_t)q / n, j = (size_t)q % n;
    uint8_t idx[32];
    or_sc_from_u64(idx, (uint64_t)(j + 1)); /* committee.rs:165 */
    or_poly_eval(sp + 32 * (i * n + j), b + 32 * i * N, N, idx); /* randomness = f'(j) */
    or_poly_eval(s + 32 * (i * n + j), a + 32 * i * N, N, idx);  /* share = f(j) */
  }
}

/* or_verify_pairs on row-local arrays: C [d1-d0][N], s / sp [d1-d0][n] hold dealers d0..d1-1 only
 * (one rank's block of a sharded run); dealer indices (the SELF diagonal) stay global. */
int or_verify_pairs_rows(size_t n, size_t t, int round, const uint8_t *C, const uint8_t h[32],
                         const uint8_t *s, const uint8_t *sp, size_t d0, size_t d1, size_t r0, size_t r1,
                         uint8_t *accept, int nthreads) {
  const size_t N = t + 1, nd = d1 - d0, nr = r1 - r0;
  ge_ext hp, g;
  ge_base_point(&g);
  if (round == 2) ge_decode(&hp, h);
  ge_ext *pts = malloc(nd * N * sizeof *pts);
  int *bad = calloc(nd, sizeof *bad);
  int rc = 0;
  for (size_t i = 0; i < nd; i++)
    for (size_t k = 0; k < N; k++)
      if (ge_decode(&pts[i * N + k], C + 32 * (i * N + k))) bad[i] = 1;
  for (size_t i = 0; i < nd; i++) rc |= bad[i] ? -1 : 0;
  set_threads(nthreads);
#pragma omp parallel for schedule(dynamic)
  for (long long q = 0; q < (long long)(nr * nd); q++) {
    size_t jj = (size_t)q / nd, ii = (size_t)q % nd;
    size_t i = d0 + ii, j = r0 + jj; /* dealer i, receiver j (0-based; index j+1) */
    uint8_t *out = accept + ii * nr + jj;
    if (i == j) {
      *out = 2;
      continue;
    }
    if (bad[ii]) { /* no decodable broadcast: round 2 MISSING (committee.rs:331-335), round 4 REJECT (:549-555) */
      *out = round == 2 ? 4 : 0;
      continue;
    }
    /* committee.rs:287-290 / 532-535: index_pow = from_u64(me).exp_iter().take(t+1) */
    uint8_t *pw = malloc(32 * N);
    uint8_t x[32];
    or_sc_from_u64(x, (uint64_t)(j + 1));
    sc52 xs, acc = {{1, 0, 0, 0, 0}};
    sc52_unpack(&xs, x);
    for (size_t k = 0; k < N; k++) {
      sc52_pack(pw + 32 * k, &acc);
      sc52_mul(&acc, &acc, &xs);
    }
    ge_ext lhs, rhs, tmp;
    uint8_t sv[32];
    or_sc_reduce(sv, s + 32 * (ii * n + j));
    ge_mul_vartime_base(&lhs, &g, sv);
    if (round == 2) {
      /* committee.rs:292-294: h * decrypted_randomness + G::generator() * decrypted_share */
      uint8_t spv[32];
      or_sc_reduce(spv, sp + 32 * (ii * n + j));
      ge_mul_vartime_base(&tmp, &hp, spv);
      ge_add_ext(&lhs, &tmp, &lhs);
    }
    ge_msm(&rhs, N, pw, pts + ii * N); /* committee.rs:295-296 / 538-539 */
    *out = (uint8_t)ge_eq(&lhs, &rhs);  /* committee.rs:305 / 541 */
    free(pw);
  }
  free(pts);
  free(bad);
  return rc;
}

/* dealers d0..d1-1 of whole arrays C [n][N], s / sp [n][n] (committee.rs:287-305, 532-548) */
int or_verify_pairs(size_t n, size_t t, int round, const uint8_t *C, const uint8_t h[32],
                    const uint8_t *s, const uint8_t *sp, size_t d0, size_t d1, size_t r0, size_t r1,
                    uint8_t *accept, int nthreads) {
  return or_verify_pairs_rows(n, t, round, C + 32 * d0 * (t + 1), h, s + 32 * d0 * n,
                              round == 2 ? sp + 32 * d0 * n : sp, d0, d1, r0, r1, accept, nthreads);
}

/* polynomial.rs:162-184 */
void or_lagrange(uint8_t out[32], const uint8_t x[32], const uint8_t *ys, const uint8_t *xs, size_t m) {
  uint8_t result[32] = {0};
  for (size_t a = 0; a < m; a++) {
    uint8_t coef[32];
    or_sc_from_u64(coef, 1);
    for (size_t b = 0; b < m; b++) {
      if (memcmp(xs + 32 * a, xs + 32 * b, 32) == 0) continue; /* i != coefficient_index */
      uint8_t num[32], den[32], inv[32];
      or_sc_sub(num, x, xs + 32 * b);
      or_sc_sub(den, xs + 32 * a, xs + 32 * b);
      or_sc_invert(inv, den);
      or_sc_mul(coef, coef, num);
      or_sc_mul(coef, coef, inv);
    }
    uint8_t term[32];
    or_sc_mul(term, coef, ys + 32 * a);
    or_sc_add(result, result, term);
  }
  memcpy(out, result, 32);
}

/* ---- single-thread cost calibration of this port (bench.py cpu_baseline): dalek-3's published
 * u64-backend figures are per field multiplication and per MSM, so the port's own are reported
 * next to its verified-shares rate. */
#include <time.h>
static double now_s(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

/* ns per fe51_mul in a dependent chain of `iters` multiplications */
double or_bench_fe_mul(uint64_t iters) {
  fe51 a = {{1234567, 7654321, 1111111, 2222222, 3333333}}, b = {{99, 98, 97, 96, 95}};
  const double t0 = now_s();
  for (uint64_t i = 0; i < iters; i++) fe51_mul(&a, &a, &b);
  const double dt = now_s() - t0;
  volatile uint64_t sink = a.v[0];
  (void)sink;
  return dt / (double)iters * 1e9;
}

/* ms per vartime MSM of N random-looking terms (dalek's Straus / Pippenger choice), `reps` runs */
double or_bench_msm(size_t N, int reps) {
  ge_ext g, *pts = malloc(N * sizeof *pts), r;
  uint8_t *sc = malloc(32 * N), seed[32] = {7};
  ge_base_point(&g);
  or_chacha20_stream(seed, 0, sc, 32 * N);
  for (size_t k = 0; k < N; k++) {
    sc[32 * k + 31] &= 0x0f;
    uint8_t e[32] = {0};
    e[0] = (uint8_t)(k + 3);
    e[1] = (uint8_t)((k + 3) >> 8);
    ge_mul_vartime_base(&pts[k], &g, e);
  }
  const double t0 = now_s();
  for (int i = 0; i < reps; i++) ge_msm(&r, N, sc, pts);
  const double dt = now_s() - t0;
  free(pts);
  free(sc);
  return dt / reps * 1e3;
}
