/*
 * dkg_amd.h — C ABI of the MI355X (gfx950) backend for the share-generation and
 * share-verification hot path of danielSanchezQ/dkg (Pedersen-VSS DKG over Ristretto255).
 *
 * Encodings (identical to the reference's wire values):
 *   scalar = 32 bytes little-endian, canonical mod l      (groups.rs:23-27)
 *   point  = 32 bytes compressed Ristretto255             (groups.rs:72-76)
 * Every buffer is caller-owned host memory unless a function name ends in `_device`
 * (then the pointers are HIP device pointers).  No pointer is retained after return.
 * One dkg_ctx drives one GPU (one process per GPU); a ctx is not re-entrant.
 *
 * Status codes: protocol outcomes (a rejected share, MisbehaviourHigherThreshold) are DATA,
 * returned in decision matrices and flags; negative codes are call failures only.
 */
#ifndef DKG_AMD_H
#define DKG_AMD_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DKG_OK 0
#define DKG_E_ARG (-1)    /* where the reference panics: length mismatch, t >= (n+1)/2, index range */
#define DKG_E_DECODE (-2) /* an input point does not decode (CompressedRistretto::decompress -> None) */
#define DKG_E_DEVICE (-3) /* HIP runtime failure (message in dkg_ctx_last_error) */
#define DKG_E_NOMEM (-4)

/* decision matrix values ([dealer][receiver], one byte per pair) */
#define DKG_REJECT 0
#define DKG_ACCEPT 1
#define DKG_SELF 2       /* i == j: a party never checks itself (qualified_set starts at 1) */
#define DKG_SKIPPED 3    /* round 4 only: dealer not qualified, check skipped (committee.rs:522) */
#define DKG_MISSING 4    /* round 2 only: the dealer's broadcast does not decode (no data): it is
                          * disqualified WITHOUT a complaint (committee.rs:331-335); in round 4 the
                          * same case is an accusation (:549-555) and reads DKG_REJECT */

typedef struct dkg_ctx dkg_ctx;

/* ---- context ---- */
int dkg_ctx_create(int device, dkg_ctx **out);
void dkg_ctx_destroy(dkg_ctx *ctx);
const char *dkg_ctx_last_error(const dkg_ctx *ctx);
/* Device time (ms) of one phase of the last ceremony's round-2 / round-4 checks, by name
 * "r2.binomial", "r2.stepping", "r2.combine" (degree split only, else 0), "r2.check", "r4.*", or
 * "r24.*" for the fused rounds (HIP events
 * on the ctx stream, recorded only with dkg_ctx_set_streams(ctx, 1)); -1 if unknown. */
double dkg_ctx_phase_ms(const dkg_ctx *ctx, const char *name);
/* Scheduling of the round-2/4 checks: the dealers are cut into nsub chunks (1..8, default 2)
 * whose pipelines run on their own HIP streams and overlap on the GPU.  nsub = 1 serialises
 * them and is the only mode that records dkg_ctx_phase_ms.  Results do not depend on nsub. */
int dkg_ctx_set_streams(dkg_ctx *ctx, int nsub);
/* on != 0 (default): the ceremony drivers verify round 2 (committee.rs:273-338) and round 4
 * (committee.rs:520-559) as ONE fused pipeline over both commitment vectors.  The round-4 inputs
 * (A_i, s_ij) are fixed in round 1 and only the SKIPPED mask of disqualified dealers depends on
 * round 2 (it is applied afterwards), so every output is identical to protocol order; ms_round2
 * then covers both rounds' checks and ms_round4 only the copy-back.  on == 0: protocol order.
 * Phase times (dkg_ctx_phase_ms, nsub == 1) are recorded under "r24.*" when fused. */
int dkg_ctx_set_overlap(dkg_ctx *ctx, int on);
/* Degree split of the difference tables: pieces = U > 1 evaluates the
 * committed polynomial as U pieces of degree < ceil((t+1)/U) recombined per receiver with U-1
 * multiplications by j^L; 0 (default) picks U with the cost model dkg_split_model_ms; 1 disables.
 * Decisions and outputs do not depend on it. */
int dkg_ctx_set_split(dkg_ctx *ctx, int pieces);
/* How the stepping covers its tables: 0 (default) by the cost model; 1 one workgroup slot per
 * column holding all its pieces (split tables whose pieces fit one 512-lane workgroup); 2 one slot
 * per piece; 3 as 0 without the dead-position repack of short unsplit tables (DESIGN.md section 4:
 * the last steps on halved segments once the top positions stop adding).  Outputs do not depend
 * on it. */
int dkg_ctx_set_stepping(dkg_ctx *ctx, int mode);
/* Field multiplication of the verification kernels: 0 (default) per launch by occupancy, 1 always
 * product scanning (fewest issue slots), 2 always column sums (most independent chains; for
 * latency-bound launches).  Outputs do not depend on it. */
int dkg_ctx_set_field_mode(dkg_ctx *ctx, int mode);
/* Schedule of the binomial-basis Horner: 0 (default) -- tables of many column
 * groups (config 5) as ONE launch in which every wave runs all steps of its 64 columns in place,
 * others one grid launch per step with the steps under one wave per SIMD on lane pairs (each point
 * on two lanes sharing its field products); 1 -- per step, no lane pairs; 2 -- per step, lane pairs
 * for every step; 3 -- per step as 0's; 4 -- per wave always; 5 -- per wave always, each item's
 * operand loaded during the previous item's chain.  Outputs do not depend on it. */
int dkg_ctx_set_binomial(dkg_ctx *ctx, int mode);
/* The fused round-2/4 checks (g*s compared in round 4, + h*s' in round 2): 0 (default) one launch
 * reading both fixed-base combs; 1 two launches that each read one comb, g*s parked in device memory
 * between them.  Mode 1 dates from the radix-2^11 combs (3.1 MB per base, one XCD's 4-MB L2 held
 * one); the radix-2^19 combs (470 MB per base, HBM / Infinity Cache) leave it no cache to win, and
 * it stays as an A/B option.  Outputs do not depend on it. */
int dkg_ctx_set_check(dkg_ctx *ctx, int mode);
/* Verification algorithm of the ceremony drivers (all-receivers views: dkg_ceremony_*, batch, shard):
 *  0 (default) -- difference tables: every P_i(j) = sum_k j^k C_k is computed as a group element and
 *                 compared with g s_ij + h s'_ij, as each receiver of the reference does;
 *  1           -- committee verification by interpolation: the shares at receivers 1..t+1 fix the
 *                 dealer's scalar polynomials F, F' (inverse Vandermonde); its commitments are
 *                 tested once against g F_k + h F'_k, and each remaining pair reduces to comparing
 *                 s_ij with F(j) (a deviating share is decided by its own group equation); rows
 *                 whose commitments are not of that form are re-verified with mode 0.  Every
 *                 decision equals mode 0's.  Needs all n shares of a dealer,
 *                 so dkg_verify_receiver (one party's column) always uses its own path. */
int dkg_ctx_set_verify_mode(dkg_ctx *ctx, int mode);
/* Mode 1: rows of the last verification that were re-verified with difference tables. */
size_t dkg_ctx_fallback_rows(const dkg_ctx *ctx);
/* U used by the last ceremony's checks on this ctx. */
int dkg_ctx_last_split(const dkg_ctx *ctx);
/* Piece length L of that split: pieces 0..U-2 hold L coefficients, the last one t+1-(U-1)L. */
size_t dkg_ctx_last_split_len(const dkg_ctx *ctx);
/* The cost model's estimate (ms) of binomial + recombination for `columns` difference tables. */
double dkg_split_model_ms(size_t columns, size_t n, size_t t, int pieces);
/* The piece length L the runtime uses for a `pieces`-way split of such tables (0 on bad input). */
size_t dkg_split_len(size_t columns, size_t n, size_t t, int pieces);
/* Recombination of a degree split: 0 (default) short multipliers for 2..5 pieces (2..4 with
 * projective addends) -- receiver j's pieces are combined as b_j P(j) = b_j Q_0(j) + a_j1 Q_1(j) + ..
 * with a short lattice vector (b_j, a_j1, ..), a_ju = b_j j^(uL) mod l (126 / 168 / 189 / 202-bit
 * scalars for 2 / 3 / 4 / 5 pieces instead of 253), and the checks compare with g*(b_j s) +
 * h*(b_j s'); 1 powers of y = j^L (253-bit
 * NAFs, pairwise Horner in y^2, any number of pieces); 2 = 0.  Decisions do not depend on it
 * (DESIGN.md section 2). */
int dkg_ctx_set_combine(dkg_ctx *ctx, int mode);
/* What the last verification recombined with: 0 no split, 1 powers of y, 2 short multipliers. */
int dkg_ctx_last_combine(const dkg_ctx *ctx);
/* How the last verification ran its binomial: 0 one launch per Horner step, 1 per-wave loops
 * (k_binom_wave, one launch per chunk stream). */
int dkg_ctx_last_binomial(const dkg_ctx *ctx);
/* Addends of the short-multiplier recombination: 0 (default) affine Niels (the stepped values
 * normalised with one inversion per run of receivers; mixed additions, 7M instead of 8M), 1 cached
 * projective.  Outputs do not depend on it. */
int dkg_ctx_set_addends(dkg_ctx *ctx, int mode);
/* Additions of the finite-difference stepping: 0 (default) the dedicated formula (HWCD 2008, no
 * product by d; not complete), with every workgroup that met an exceptional pair (a sum with Z = 0:
 * equal or 2-/4-torsion-related points, which crafted commitments can reach) recomputed by the
 * complete formula; 1 the complete formula only.  Outputs do not depend on it. */
int dkg_ctx_set_stepping_formula(dkg_ctx *ctx, int mode);
/* Workgroups of the last verification's stepping that were recomputed by the complete formula
 * (synchronises the context's stream; 0 in mode 1; -1 on error). */
long long dkg_ctx_stepping_redos(dkg_ctx *ctx);
/* 1 when the last single-ceremony or dealer-shard call reran its verification with the complete
 * formula because a dedicated addition of the per-step binomial met Z = 0 (an exceptional pair, e.g.
 * a crafted all-identity commitment row), else 0 (-1 on a NULL ctx). */
int dkg_ctx_binomial_reruns(dkg_ctx *ctx);
/* The short multipliers (b_j, a_j1, .., a_j(U-1)) of receivers j = 1..n for a `pieces`-way split of
 * piece length L (2 <= pieces <= 5): magnitudes mag[n][pieces][32] (little-endian), signs
 * sign[n][pieces] (+1 / -1); a_ju = b_j j^(uL) mod l and b_j > 0.  DKG_E_ARG on bad input. */
int dkg_split_multipliers(size_t n, size_t L, int pieces, uint8_t *mag, int8_t *sign);
/* Number of GPUs visible to this process (counts only; does not create a context). */
int dkg_device_count(void);
/* Measurement aids (bench.py; no reference counterpart).
 * dkg_ctx_clock_probe: 4 waves per SIMD on every CU of the ctx's device each run `iters` dependent
 * VALU iterations, reading the shader clock (s_memtime) and the constant-rate clock (s_memrealtime,
 * hipDeviceAttributeWallClockRate) around them; *sclk_mhz = the median over waves of shader cycles
 * per real-time microsecond (the clock the VALU ran at under full occupancy), *busy_ms = the
 * probe's real-time span (median).  dkg_device_pci_bus_id: the device's PCI bus id
 * ("dddd:bb:dd.f", hipDeviceGetPCIBusId) into buf[len]. */
int dkg_ctx_clock_probe(dkg_ctx *ctx, unsigned iters, double *sclk_mhz, double *busy_ms);
int dkg_device_pci_bus_id(int device, char *buf, int len);

/* ---- Environment::init (committee.rs:72-83) ----
 * Checks threshold < (nr_members + 1) / 2 (DKG_E_ARG otherwise, where the reference asserts) and
 * derives the Pedersen commitment key h = hash_to_group::<Blake2b>(ck_bytes) (commitment.rs:13-17),
 * caching its fixed-base table on the device.  h_out may be NULL. */
int dkg_env_init(dkg_ctx *ctx, size_t threshold, size_t nr_members, const uint8_t *ck_bytes, size_t ck_len,
                 uint8_t h_out[32]);
/* Same check without a context (pure function). */
int dkg_env_check(size_t threshold, size_t nr_members);

/* ---- trait-level batches (traits.rs:142-238, groups.rs:11-90) ---- */
/* PrimeGroupElement::vartime_multiscalar_multiplication (traits.rs:234-237), B independent MSMs of
 * N terms: out[b] = sum_k scalars[b][k] * points[b][k].  scalars [B][N][32], points [B][N][32]. */
int dkg_msm_batch(dkg_ctx *ctx, size_t B, size_t N, const uint8_t *scalars, const uint8_t *points, uint8_t *out);
/* Mul<Scalar> by a fixed base (traits.rs:212): out[c] = scalars[c] * base.  base == NULL means
 * PrimeGroupElement::generator() (groups.rs:60-62). */
int dkg_fixed_base_batch(dkg_ctx *ctx, const uint8_t base[32], size_t count, const uint8_t *scalars, uint8_t *out);
/* Polynomial::evaluate (polynomial.rs:68-74) of D polynomials with N coefficients each
 * (coeffs [D][N][32]) at M small integer points xs[m] < 2^24: out [D][M][32]. */
int dkg_poly_eval_batch(dkg_ctx *ctx, size_t D, size_t N, const uint8_t *coeffs, size_t M, const uint32_t *xs,
                        uint8_t *out);
/* PrimeGroupElement::from_bytes validity (groups.rs:78-81): ok[c] = 1 iff points[c] decodes. */
int dkg_points_valid_batch(dkg_ctx *ctx, size_t count, const uint8_t *points, uint8_t *ok);

/* ---- round 1: share generation (Phases<Initialise>::init, committee.rs:124-216) ----
 * For dealers i in [0, D): coefficients a (sharing) and b (hiding), [D][t+1][32];
 * E[i][k] = h*b[i][k] + g*a[i][k], A[i][k] = g*a[i][k] ([D][t+1][32], committee.rs:151-159);
 * s[i][j] = f_i(j+1), s_prime[i][j] = f'_i(j+1) for receivers j in [0, n) ([D][n][32], :164-167).
 * Requires dkg_env_init (for h).  Any output may be NULL to skip it. */
int dkg_share_gen(dkg_ctx *ctx, size_t D, size_t n, size_t t, const uint8_t *a, const uint8_t *b, uint8_t *E,
                  uint8_t *A, uint8_t *s, uint8_t *s_prime);
/* The same on device buffers (canonical scalars d_a, d_b [D][t+1][32] in; d_E, d_A [D][t+1][32]
 * compressed -- either may be NULL -- and d_s, d_s_prime [D][n][32] out), e.g. to build the
 * broadcasts of a large committee in HBM for dkg_ceremony_shard_verify_device. */
int dkg_share_gen_device(dkg_ctx *ctx, size_t D, size_t n, size_t t, const void *d_a, const void *d_b, void *d_E,
                         void *d_A, void *d_s, void *d_s_prime);

/* ---- rounds 2 and 4: share checks ----
 * round 2 (Phases<Phase1>::proceed, committee.rs:273-338): h*s' + g*s == sum_k (j+1)^k E_i[k]
 * round 4 (Phases<Phase3>::proceed, committee.rs:520-559):          g*s == sum_k (j+1)^k A_i[k]
 * for dealers i in [d0, d1) and ALL receivers j in [0, n).  C = E (round 2) or A (round 4) of those
 * dealers, [d1-d0][t+1][32]; s, s_prime = the dealers' share rows [d1-d0][n][32] (s_prime unused in
 * round 4).  decision [d1-d0][n] (DKG_ACCEPT / DKG_REJECT / DKG_SELF).  A dealer whose commitment
 * vector does not decode reads DKG_MISSING for every receiver in round 2 (disqualified without a
 * complaint, committee.rs:331-335) and DKG_REJECT in round 4 (:549-555); the call returns DKG_OK. */
int dkg_verify_pairs(dkg_ctx *ctx, size_t n, size_t t, int round, size_t d0, size_t d1, const uint8_t *C,
                     const uint8_t *s, const uint8_t *s_prime, uint8_t *decision);
/* The same check seen from ONE receiver j (what one party runs in the reference): decisions of
 * receiver j (0-based; index j+1) over all n dealers.  C [n][t+1][32], s / s_prime [n][32] = the
 * column of shares addressed to j.  decision [n]. */
int dkg_verify_receiver(dkg_ctx *ctx, size_t n, size_t t, int round, size_t j, const uint8_t *C, const uint8_t *s,
                        const uint8_t *s_prime, uint8_t *decision);

/* ---- whole ceremony (rounds 1-5, every party played in one process as the reference tests do,
 * committee.rs:1518-1656) in plaintext-share mode. ---- */
typedef struct {
  /* host outputs; any pointer may be NULL */
  uint8_t *E, *A;               /* [n][t+1][32] (round-1 broadcast; A = round-3 broadcast) */
  uint8_t *s, *s_prime;         /* [n][n][32] */
  uint8_t *dec2, *dec4;         /* [n dealer][n receiver] */
  uint8_t *qualified;           /* [n] common qualified set after round 3 */
  uint8_t *r2_error;            /* [n] receiver j: more than t complaints (MisbehaviourHigherThreshold) */
  uint8_t *r4_error;            /* [n] receiver j: fewer than t+1 honest dealers (itself included) in
                                   round 4, MisbehaviourHigherThreshold (committee.rs:567-569) */
  int32_t *complaints2;         /* [n] complaints raised by receiver j in round 2 */
  uint8_t *reconstruct;         /* [n] dealers whose secret is reconstructed in finalise */
  uint8_t *final_share;         /* [n][32] s_j = sum_{i in Q} s_ij (committee.rs:454-462) */
  uint8_t *public_share;        /* [n][32] g * s_j (committee.rs:464-466) */
  uint8_t mpk[32];              /* MasterPublicKey (committee.rs:726-805) that every finalising
                                   final party (qualified, not reconstructable, no r2 / r4 error)
                                   computes when all phase-5 disclosures arrive: a reconstructed
                                   dealer's secret is interpolated at zero over exactly the shares of
                                   the final parties that disclose (:754-788) -- a party with an r2 /
                                   r4 error never broadcasts its phase-5 shares (:340-347, 567-569,
                                   684); with exactly t of them a wrong secret, as the reference.
                                   ALL ZERO and meaningless when phase4_error == 1, and when a
                                   dealer is reconstructed and fewer than t final parties disclose
                                   (InsufficientSharesForRecovery for everyone, :779-781).
                                   Other parties' views, and missing disclosures:
                                   dkg_finalise_parties. */
  int32_t n_qualified;
  int32_t phase4_error;         /* 1: qualified minus reconstructable <= t, every party's
                                   Phases<Phase4>::proceed fails with MisbehaviourHigherThreshold
                                   (committee.rs:673-677): nobody finalises, there is no mpk */
  /* device times of each phase, milliseconds (HIP events) */
  double ms_round1, ms_round2, ms_round3, ms_round4, ms_finalise, ms_total;
} dkg_ceremony_out;

/* Honest run from coefficients a, b ([n][t+1][32], host). */
int dkg_ceremony_run(dkg_ctx *ctx, size_t n, size_t t, const uint8_t *a, const uint8_t *b, dkg_ceremony_out *out);
/* Receiver side (rounds 2-5) from broadcast values that may have been tampered with:
 * E, A [n][t+1][32]; s, s_prime [n][n][32]. */
int dkg_ceremony_verify(dkg_ctx *ctx, size_t n, size_t t, const uint8_t *E, const uint8_t *A, const uint8_t *s,
                        const uint8_t *s_prime, dkg_ceremony_out *out);
/* dkg_ceremony_verify after the broadcast intake of MembersFetchedState1/3::from_broadcast
 * (committee.rs:825-870, 921-966): fetched1[i] = 0 when dealer i's phase-1 broadcast is absent or
 * malformed (committed_coefficients.len() != t+1 or encrypted_shares.len() != n): no fetched data,
 * DKG_MISSING for every receiver in round 2 (disqualified, no complaint, :331-335).
 * fetched3[i] = 0 when its phase-3 broadcast is absent or has the wrong length: a qualified dealer
 * is accused by every receiver in round 4 (:549-555) and reconstructed.  The E / A rows of such
 * dealers are not read for decisions (any bytes). */
int dkg_ceremony_verify_fetched(dkg_ctx *ctx, size_t n, size_t t, const uint8_t *E, const uint8_t *A,
                                const uint8_t *s, const uint8_t *s_prime, const uint8_t *fetched1,
                                const uint8_t *fetched3, dkg_ceremony_out *out);
/* Device-resident variant for benchmarks: d_a, d_b are device pointers to [n][t+1][32] canonical
 * scalars; intermediates stay in HBM; only the small outputs (mpk, flags, counts, timings) are
 * copied back into *out (its array pointers are ignored except qualified / r2_error / r4_error / complaints2). */
int dkg_ceremony_run_device(dkg_ctx *ctx, size_t n, size_t t, const void *d_a, const void *d_b,
                            dkg_ceremony_out *out);
/* Sharded variant (one rank of a multi-GPU run): this ctx owns dealers [d0, d1) of the same
 * ceremony.  Produces this rank's commitments E/A and decision rows; the caller all-gathers
 * (RCCL over xGMI) the rows, A_0 values and share partial sums.  Device pointers throughout:
 * d_a, d_b [d1-d0][t+1][32]; d_dec2, d_dec4 [d1-d0][n]; d_A0 [d1-d0][32] = each dealer's
 * compressed master-key term A_i0 (a dealer that round-4 accusations put in the reconstructable set
 * gets g * a_i0 after the exchange, dkg_ceremony_shard_recon_device, because the interpolation
 * points -- the final parties -- depend on every rank's rows; then mpk = sum of the qualified
 * dealers' terms); d_partial [n][32] = sum over this rank's QUALIFIED dealers of s_ij (qualification
 * of a dealer is decided by its own round-2 row, so it needs no exchange). */
int dkg_ceremony_shard_device(dkg_ctx *ctx, size_t n, size_t t, size_t d0, size_t d1, const void *d_a,
                              const void *d_b, void *d_dec2, void *d_dec4, void *d_A0, void *d_partial,
                              double *ms_total);
/* Sharded verification of received broadcasts (the rank's dealers' rows of MembersFetchedState1 /
 * Phase1 / Phase3, committee.rs:260-366, 508-580, 726-805): d_E, d_A [d1-d0][t+1][32] compressed
 * commitments as broadcast, d_s, d_s_prime [d1-d0][n][32] the shares (Scalar::from_bytes
 * semantics).  Outputs as dkg_ceremony_shard_device; an undecodable E row is DKG_MISSING in round 2
 * (disqualified, no complaint), an undecodable A row an accusation in round 4. */
int dkg_ceremony_shard_verify_device(dkg_ctx *ctx, size_t n, size_t t, size_t d0, size_t d1, const void *d_E,
                                     const void *d_A, const void *d_s, const void *d_s_prime, void *d_dec2,
                                     void *d_dec4, void *d_A0, void *d_partial, double *ms_total);
/* Finalise step of a sharded run, after the exchange (committee.rs:747-789): for this rank's dealers
 * [d0, d1) with reconstruct[i] (host [n], the combined round-4 outcome), d_terms[i - d0] (device
 * [d1-d0][32], the rank's exchanged master-key terms, in/out) is replaced by g * a_i0 recovered by
 * Lagrange interpolation at zero over the shares of the DISCLOSING final parties: qualified[j] &&
 * !reconstruct[j] && !r2_error[j] && !r4_error[j] (host [n]; r2_error / r4_error may be NULL) -- a
 * party whose Phase1 or Phase3 failed never broadcasts its phase-5 disclosures (:340-347, 567-569,
 * 684) -- the value every finalising party computes.  When some dealer is reconstructed and fewer
 * than t parties disclose, every finalising party fails with InsufficientSharesForRecovery
 * (:779-781): *recovery_error (may be NULL) = 1, d_terms is untouched and the caller has no mpk
 * (pass it as phase4_error to dkg_shard_finalise_device); else 0.  It depends on the common outcome
 * only, so every rank gets the same.  d_s: the dealers' share rows [d1-d0][n][32] (from_bits
 * semantics), or NULL for the rows of the last dkg_ceremony_shard_device / _shard_verify_device call
 * on this ctx (same n, d0, d1).  Dealers without reconstruct are untouched. */
int dkg_ceremony_shard_recon_device(dkg_ctx *ctx, size_t n, size_t t, size_t d0, size_t d1, const uint8_t *qualified,
                                    const uint8_t *reconstruct, const uint8_t *r2_error, const uint8_t *r4_error,
                                    const void *d_s, void *d_terms, int32_t *recovery_error);
/* Combine step of the sharded run (device pointers):
 * round-3 sum (committee.rs:454-462): out[j] = sum over rows r with mask[r] (NULL = all) of in[r][j]
 * mod l; in [rows][n][32] canonical scalars (e.g. the all-gathered per-rank partials), out [n][32]. */
int dkg_scalar_sum_device(dkg_ctx *ctx, size_t rows, size_t n, const void *d_in, const void *d_mask, void *d_out);
/* finalise (committee.rs:790-795): out = sum of points[c] with mask[c] (NULL = all), points
 * [count][32] compressed, out [32] compressed.  DKG_E_DECODE if a selected point does not decode. */
int dkg_point_sum_device(dkg_ctx *ctx, size_t count, const void *d_points, const void *d_mask, void *d_out);

/* ---- the sharded run's protocol layer (multi-GPU, one process per GPU) ----
 * The reference has no transport (its broadcast channel is abstract, src/lib.rs:91-115); a
 * multi-rank driver supplies the all-gathers (RCCL over xGMI) and calls, on every rank:
 *   dkg_ceremony_shard_device / _shard_verify_device   this rank's dealers' rows
 *   all-gather dec2, dec4 (each rank's [R][n] block), A0 ([R][32]), partials ([n][32])
 *   dkg_shard_combine_device                           the common outcome (identical on every rank)
 *   if reconstruct has any member and !phase4_error:
 *     dkg_ceremony_shard_recon_device, all-gather the terms again (unless recovery_error)
 *   dkg_shard_finalise_device                          final shares, public shares, mpk
 * Rank r of world_size owns dealers [r*n/ws, (r+1)*n/ws); R = dkg_shard_rows(n, ws) is the padded
 * block height every rank gathers. */
void dkg_shard_range(size_t n, size_t world_size, size_t rank, size_t *d0, size_t *d1);
size_t dkg_shard_rows(size_t n, size_t world_size);

typedef struct {
  /* host arrays [n] (any may be NULL) */
  uint8_t *qualified;     /* round 2: no REJECT and no MISSING in the dealer's row (committee.rs:311-335, 370-398) */
  int32_t *complaints2;   /* REJECTs raised by receiver j */
  uint8_t *r2_error;      /* complaints2[j] > t (:340-347) */
  uint8_t *reconstruct;   /* qualified dealers some receiver rejected in round 4 (:660-670) */
  uint8_t *r4_error;      /* receiver j: itself plus the qualified dealers it accepted < t+1 (:515-516, 567-569) */
  int32_t n_qualified;
  int32_t phase4_error;   /* qualified minus reconstructable <= t (:673-677) */
} dkg_shard_outcome;

/* Combine step after the decision all-gathers: d_dec2_g, d_dec4_g device [ws][R][n] (rank blocks as
 * gathered, rows past a rank's dealer count ignored).  Derives the common outcome with the same code
 * as the single-GPU drivers (runtime.hip round2_device / round4_device and their host halves).  d_dec2, d_dec4 (device
 * [n][n], may be NULL): the compacted decision matrices, dec4 with the SKIPPED rows of disqualified
 * dealers applied (:522). */
int dkg_shard_combine_device(dkg_ctx *ctx, size_t n, size_t t, size_t world_size, const void *d_dec2_g,
                             const void *d_dec4_g, void *d_dec2, void *d_dec4, dkg_shard_outcome *out);
/* Packed decision rows: the complaint / verification bitmaps a multi-rank driver all-gathers instead
 * of n bytes per row (committee.rs:311-347: every party learns every complaint).  A rank's raw rows
 * hold REJECT / ACCEPT (round 4 too: SKIPPED is applied by the combine), SELF on the global diagonal
 * and, in round 2, whole rows of MISSING; row r becomes dkg_packed_row_words(n) = ceil(n/32) + 1
 * little-endian u32 words: bit j % 32 of word j / 32 set iff entry j is ACCEPT, then a kind word (0
 * checked, 1 MISSING row, 2 SKIPPED row).  n = 4096: 516 bytes per row instead of 4096. */
size_t dkg_packed_row_words(size_t n);
/* Windows (one mixed addition each) per scalar of the fixed-base combs of g and h the checks and
 * commitments use (radix 2^DKG_COMBW_BITS, a build-time choice): the closed-form work of bench.py. */
int dkg_fixed_base_windows(void);
/* The same for the member keys' combs (full mode's K = pk_q r, radix 2^DKG_KEY_COMB_BITS). */
int dkg_key_comb_windows(void);
/* d_dec device [nvalid][n] raw rows of dealers d0 .. d0+nvalid-1 (dkg_ceremony_shard_device's
 * output) -> d_packed device [rows][dkg_packed_row_words(n)] u32, rows past nvalid zero (the padded
 * rank block, rows = dkg_shard_rows).  DKG_E_ARG if a row holds values the encoding cannot carry
 * (nothing is lost silently). */
int dkg_decisions_pack_device(dkg_ctx *ctx, size_t rows, size_t nvalid, size_t n, size_t d0, const void *d_dec,
                              void *d_packed);
/* dkg_shard_combine_device on the gathered packed blocks: d_pack2_g, d_pack4_g device
 * [ws][R][dkg_packed_row_words(n)] u32; outputs as dkg_shard_combine_device (d_dec2 / d_dec4 are the
 * unpacked matrices, bit-identical to the byte exchange's). */
int dkg_shard_combine_packed_device(dkg_ctx *ctx, size_t n, size_t t, size_t world_size, const void *d_pack2_g,
                                    const void *d_pack4_g, void *d_dec2, void *d_dec4, dkg_shard_outcome *out);
/* Finalise of the sharded run: d_terms_g device [ws][R][32] the gathered master-key terms (A_i0, or
 * g * a_i0 for reconstructed dealers after dkg_ceremony_shard_recon_device), d_partials_g device
 * [ws][n][32] the gathered partial final shares, qualified host [n] (the combine's).  Outputs:
 * d_final_share device [n][32] s_j = sum of the partials (committee.rs:454-462), d_public_share device
 * [n][32] g * s_j (:463-467; may be NULL), mpk host [32] = sum of the qualified dealers' terms
 * (:790-795), zero when phase4_error (nobody finalises, :673-677). */
int dkg_shard_finalise_device(dkg_ctx *ctx, size_t n, size_t t, size_t world_size, const void *d_terms_g,
                              const void *d_partials_g, const uint8_t *qualified, int phase4_error,
                              void *d_final_share, void *d_public_share, uint8_t *mpk);

/* ---- in-library multi-device context: ONE process, several GPUs (SURVEY.md section 8(b),
 * threading row; dkg_amd/csrc/multi.cpp) ----
 * The same dealer sharding as the one-process-per-GPU protocol above, driven inside the library:
 * shard i (on devices[i]) owns dealers dkg_shard_range(n, ndev, i) and runs them on its own host
 * thread; the exchange is a gather of every shard's rows, master-key terms and partial shares into
 * devices[0] by peer copies over xGMI; the combine, the round-4 reconstruction (on the owning
 * shards) and the finalise are the dkg_shard_* steps.  Outputs equal dkg_ceremony_run /
 * dkg_ceremony_verify's.  A device may be listed more than once (its shards share the GPU).
 * The reference is single-threaded and has no transport (src/lib.rs:91-115); this replaces the
 * caller's loop over parties (committee.rs:1518-1656) spread over a node's GPUs.  Not re-entrant
 * on the same context. */
typedef struct dkg_multi dkg_multi;
int dkg_multi_create(const int *devices, int ndev, dkg_multi **out);
void dkg_multi_destroy(dkg_multi *m);
int dkg_multi_size(const dkg_multi *m);
/* shard i's dkg_ctx (its tuning knobs: dkg_ctx_set_split, _set_streams, ...); owned by m */
dkg_ctx *dkg_multi_ctx(dkg_multi *m, int shard);
const char *dkg_multi_last_error(const dkg_multi *m);
/* host wall milliseconds of the last ceremony's steps: "shard_max" / "shard_min" (the shards' device
 * times), "exchange", "combine", "recon", "finalise"; -1 if unknown */
double dkg_multi_phase_ms(const dkg_multi *m, const char *name);
/* Environment::init (committee.rs:72-83) on every shard's context */
int dkg_multi_env_init(dkg_multi *m, size_t threshold, size_t nr_members, const uint8_t *ck_bytes, size_t ck_len,
                       uint8_t h_out[32]);
/* dkg_ceremony_run over the shards: a, b host [n][t+1][32].  out->E, A, s, s_prime must be NULL
 * (they stay on the shards' devices); every other output as dkg_ceremony_run.  Times: ms_round2 =
 * the slowest shard, ms_round3 = exchange, ms_round4 = combine + reconstruction, ms_finalise,
 * ms_total = host wall from the shards' start (after the uploads) to the outputs. */
int dkg_multi_ceremony_run(dkg_multi *m, size_t n, size_t t, const uint8_t *a, const uint8_t *b,
                           dkg_ceremony_out *out);
/* d_a[i], d_b[i]: device pointers on devices[i] to shard i's dealers' coefficients [D_i][t+1][32] */
int dkg_multi_ceremony_run_device(dkg_multi *m, size_t n, size_t t, const void *const *d_a, const void *const *d_b,
                                  dkg_ceremony_out *out);
/* dkg_ceremony_verify over the shards (received broadcasts, host arrays as there) */
int dkg_multi_ceremony_verify(dkg_multi *m, size_t n, size_t t, const uint8_t *E, const uint8_t *A, const uint8_t *s,
                              const uint8_t *s_prime, dkg_ceremony_out *out);

/* ---- per-party finalise: Phases<Phase5>::finalise (committee.rs:726-805) as EVERY party p runs it ----
 * Inputs are the ceremony's common outcome (host arrays [n]): qualified, reconstruct (round 4,
 * committee.rs:660-670), r2_error / r4_error (may be NULL: a party whose Phase1 / Phase3 proceed failed
 * never finalises), disclosed (may be NULL = all): 0 for a party whose phase-5 broadcast (its
 * disclosed shares, BroadcastPhase5) party p does not fetch; A0 [n][32] the dealers' A_i0 (phase-3
 * broadcasts); s [n dealer][n receiver][32] the shares.  For each reconstructed dealer i party p
 * interpolates at zero over its own share s_ip and the disclosed shares of the OTHER final parties
 * (:754-775); it fails with InsufficientSharesForRecovery(i) -- i the first reconstructed dealer --
 * when it has fewer than `threshold` = t points (:779-781; exactly t points interpolate a wrong
 * secret, as the reference does).  Outputs [n]: mpk[p] (32 bytes, zero unless status[p] == OK),
 * status[p], recovery_index[p] (the dealer i of InsufficientSharesForRecovery / the panic, else
 * -1; may be NULL).  Dealers are visited in index order and the first failure wins, as in the loop
 * of committee.rs:745-797. */
#define DKG_FIN_OK 0
#define DKG_FIN_R2_ERROR 1      /* Phases<Phase1>::proceed: MisbehaviourHigherThreshold (committee.rs:340-347) */
#define DKG_FIN_R4_ERROR 2      /* Phases<Phase3>::proceed: MisbehaviourHigherThreshold (committee.rs:567-569) */
#define DKG_FIN_PHASE4_ERROR 3  /* Phases<Phase4>::proceed: MisbehaviourHigherThreshold (committee.rs:673-677) */
#define DKG_FIN_INSUFFICIENT 4  /* finalise: InsufficientSharesForRecovery(i) (committee.rs:779-781) */
#define DKG_FIN_PANIC 5         /* finalise panics at dealer i: i is disqualified and i != p, so its
                                   committed coefficients were never recorded (committee.rs:791-794
                                   expect()s them; they are stored only at :190 and :527-530).  A
                                   disqualified party p itself adds its own A_p0 (:190). */
int dkg_finalise_parties(dkg_ctx *ctx, size_t n, size_t t, const uint8_t *qualified, const uint8_t *reconstruct,
                         const uint8_t *r2_error, const uint8_t *r4_error, const uint8_t *disclosed, const uint8_t *A0,
                         const uint8_t *s, uint8_t *mpk, int32_t *status, int32_t *recovery_index);

/* ---- batches of independent ceremonies (BASELINE config 5: e.g. 10,000 ceremonies of n = 64) ----
 * B ceremonies with the same (n, t) and commitment key, each played as dkg_ceremony_run plays one
 * (full_valid_run, committee.rs:1518-1656): rounds 1-5 for every party of every ceremony.
 * Ceremony c's dealers are rows c*n .. c*n + n-1 of every [B*n]-row array; every output equals
 * what B separate single-ceremony calls return (the work of all B shares each kernel launch). */
typedef struct {
  /* host outputs; any pointer may be NULL */
  uint8_t *mpk;                 /* [B][32] MasterPublicKey per ceremony (committee.rs:726-805), as in
                                   dkg_ceremony_out; all zero for a ceremony with phase4_error */
  int32_t *n_qualified;         /* [B] */
  uint8_t *phase4_error;        /* [B] qualified minus reconstructable <= t (committee.rs:673-677) */
  uint8_t *qualified;           /* [B][n] */
  uint8_t *r2_error;            /* [B][n] receiver saw more than t complaints */
  uint8_t *r4_error;            /* [B][n] receiver saw fewer than t+1 honest dealers in round 4 */
  int32_t *complaints2;         /* [B][n] complaints raised by each receiver in round 2 */
  uint8_t *reconstruct;         /* [B][n] */
  uint8_t *final_share;         /* [B][n][32] */
  uint8_t *public_share;        /* [B][n][32] */
  uint8_t *dec2, *dec4;         /* [B][n dealer][n receiver] decision matrices (dec4 with SKIPPED) */
  /* device times, milliseconds (HIP events): round 1, the fused round-2/4 checks, round 3,
   * finalise (mpk incl. the round-4 combine), total */
  double ms_round1, ms_checks, ms_round3, ms_finalise, ms_total;
} dkg_batch_out;

/* Honest batch from device-resident coefficients d_a, d_b [B*n][t+1][32] (canonical scalars). */
int dkg_ceremony_batch_device(dkg_ctx *ctx, size_t B, size_t n, size_t t, const void *d_a, const void *d_b,
                              dkg_batch_out *out);
/* Receiver side of a batch from host broadcast values that may have been tampered with:
 * E, A [B*n][t+1][32]; s, s_prime [B*n][n][32] (row c*n + i = dealer i of ceremony c). */
int dkg_ceremony_batch_verify(dkg_ctx *ctx, size_t B, size_t n, size_t t, const uint8_t *E, const uint8_t *A,
                              const uint8_t *s, const uint8_t *s_prime, dkg_batch_out *out);

/* ---- full (encrypted-share) mode: the round-1 shares travel hybrid-encrypted
 * (committee.rs:164-172) under the members' communication keys and each receiver decrypts its own
 * (committee.rs:282-286).  Hybrid scheme (elgamal.rs:134-193): e1 = g*r, K = pk*r,
 * e2 = m XOR ChaCha20(key = Blake2b-512(K)[0..32], nonce = [32..44]); decryption K = sk*e1;
 * decrypted scalars are from_bits (groups.rs:29-36), reduced mod l on the device.
 * Ciphertext arrays are [D dealer][n recipient][2][32] with [..][0] = the randomness s' and
 * [..][1] = the share s (the reference encrypts the randomness first, committee.rs:171-172). ---- */
/* Seeded MemberCommunicationKey for n members (procedure_keys.rs:72-82):
 * sk_j = wide(ChaCha20Rng(BLAKE2b-256("dkg-amd/v1/member" || master || u32le ceremony || u32le j))),
 * pk_j = g*sk_j; returned SORTED by public-key bytes (committee.rs:134-135, procedure_keys.rs:26-40):
 * the party of index q+1 owns sk[q].  sk, pk [n][32]. */
int dkg_member_keys(dkg_ctx *ctx, const uint8_t master[32], uint32_t ceremony, size_t n, uint8_t *sk, uint8_t *pk);
/* Encryption randomness of dealers [d0, d0+D) for n recipients, continuing each dealer's seeded
 * stream after its 2(t+1) coefficient draws: r [D][n][2][32] (host), and the device variant for B
 * ceremonies (rows as dkg_dealer_coeffs_device). */
int dkg_enc_randomness(const uint8_t master[32], uint32_t ceremony, size_t d0, size_t D, size_t n, size_t t,
                       uint8_t *r);
int dkg_enc_randomness_device(dkg_ctx *ctx, const uint8_t master[32], uint32_t ceremony0, size_t B, size_t d0,
                              size_t D, size_t n, size_t t, void *d_r);
/* Hybrid-encrypt the share rows of D dealers (s, s_prime [D][n][32]) to the n recipients' keys
 * pk [n][32] with randomness r [D][n][2][32]: e1, ct [D][n][2][32].  DKG_E_DECODE if a key does
 * not decode. */
int dkg_encrypt_shares(dkg_ctx *ctx, size_t D, size_t n, const uint8_t *pk, const uint8_t *s, const uint8_t *s_prime,
                       const uint8_t *r, uint8_t *e1, uint8_t *ct);
/* Receivers' decryption with their secret keys sk [n][32]: s, s_prime [D][n][32];
 * ok [D][n][2] (may be NULL) = e1 decoded (a ciphertext that does not decode is missing data). */
int dkg_decrypt_shares(dkg_ctx *ctx, size_t D, size_t n, const uint8_t *sk, const uint8_t *e1, const uint8_t *ct,
                       uint8_t *s, uint8_t *s_prime, uint8_t *ok);
/* Whole ceremony in full mode from device coefficients d_a, d_b [n][t+1][32] and encryption
 * randomness d_r [n][n][2][32]; sk, pk = dkg_member_keys output (host).  With chunk streams
 * (dkg_ctx_set_streams > 1) the share evaluation, encryption and decryption run on a low-priority
 * stream beside the checks' difference tables (the checks wait for the decrypted shares), and the
 * members' key combs are kept on the ctx until the keys change; ms_round1 then times the
 * commitments and ms_round2 the rest up to the round-2/4 decisions.  With one stream: encryption in
 * ms_round1, decryption in ms_round2. */
int dkg_ceremony_run_full_device(dkg_ctx *ctx, size_t n, size_t t, const void *d_a, const void *d_b, const void *d_r,
                                 const uint8_t *sk, const uint8_t *pk, dkg_ceremony_out *out);
/* Receiver side of a full-mode ceremony from (possibly tampered) broadcast values: E, A
 * [n][t+1][32], e1, ct [n][n][2][32], the members' sorted secret keys sk [n][32].  A dealer with a
 * ciphertext that does not decode is missing data (DKG_MISSING in round 2).  out->s / s_prime
 * receive the decrypted shares. */
int dkg_ceremony_verify_full(dkg_ctx *ctx, size_t n, size_t t, const uint8_t *E, const uint8_t *A, const uint8_t *e1,
                             const uint8_t *ct, const uint8_t *sk, dkg_ceremony_out *out);

/* ---- complaint proofs: dl_equality/zkp.rs, broadcast.rs ----
 * enc [B][128] = one dealer->accuser ciphertext pair: e1_rand || ct_rand || e1_share || ct_share.
 * proof [192] = ProofOfMisbehaviour (broadcast.rs:181-186): share_key || randomness_key || c1 || r1
 * || c2 || r2, the two CorrectHybridDecrKeyZkp = DLEQ(g, e1, pk, K) proofs (challenge, response).
 * Verdicts (int32): 0 Ok (a valid complaint), 1 InvalidProofOfMisbehaviour, 2 FalseClaimedInequality,
 * 3 FalseClaimedEquality, -1 an input point does not decode. */
/* ProofOfMisbehaviour::generate (broadcast.rs:189-226) for B complaints by accusers with secret keys
 * sk [B][32]; nonces w [B][2][32]: w[0] for the share's proof (drawn first), w[1] the randomness's. */
int dkg_misbehaviour_prove(dkg_ctx *ctx, size_t B, const uint8_t *sk, const uint8_t *enc, const uint8_t *w,
                           uint8_t *proofs);
/* MisbehavingPartiesRound1::verify (broadcast.rs:50-99), including ProofOfMisbehaviour::verify
 * (:228-283) with its swapped-role check h*share + g*randomness (:271-274), reproduced as is:
 * accuser[b] = 1-based index, pk [B][32] the accuser's communication key, E [B][t+1][32] the
 * accused dealer's committed coefficients.  Requires dkg_env_init (h). */
int dkg_complaint1_verify(dkg_ctx *ctx, size_t B, size_t t, const uint32_t *accuser, const uint8_t *pk,
                          const uint8_t *enc, const uint8_t *E, const uint8_t *proofs, int32_t *result);
/* MisbehavingPartiesRound3::verify (broadcast.rs:105-135): the disclosed decrypted share and
 * randomness [B][32] must pass against E (else FalseClaimedEquality) and fail against A (else
 * FalseClaimedInequality). */
int dkg_complaint3_verify(dkg_ctx *ctx, size_t B, size_t t, const uint32_t *accuser, const uint8_t *share,
                          const uint8_t *randomness, const uint8_t *E, const uint8_t *A, int32_t *result);

/* ---- synthetic inputs: the seeded RNG convention ----
 * dealer seed = BLAKE2b-256("dkg-amd/v1/dealer" || master[32] || u32le ceremony || u32le dealer);
 * coefficients = ChaCha20Rng(seed): hiding b_0..b_t first, then sharing a_0..a_t (committee.rs:143-146),
 * each 64 bytes wide-reduced mod l (Scalar::random).  Host computation; a, b [D][t+1][32] for
 * dealers [d0, d0+D). */
int dkg_dealer_coeffs(const uint8_t master[32], uint32_t ceremony, size_t d0, size_t D, size_t t, uint8_t *a,
                      uint8_t *b);
/* The same convention on the GPU, for B ceremonies at once: row r in [0, B*D)
 * holds dealer d0 + r % D of ceremony ceremony0 + r / D; d_a, d_b are device buffers
 * [B*D][t+1][32].  Bit-identical to dkg_dealer_coeffs; keeps n = 4096 or 10,000-ceremony inputs
 * off the PCIe bus. */
int dkg_dealer_coeffs_device(dkg_ctx *ctx, const uint8_t master[32], uint32_t ceremony0, size_t B, size_t d0,
                             size_t D, size_t t, void *d_a, void *d_b);

#ifdef __cplusplus
}
#endif
#endif
