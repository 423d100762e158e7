// Host-side launchers for the gfx950 kernels (kernels.hip).  All pointers are device pointers;
// all launches go to `stream`.  Layouts are documented in points.h and DESIGN.md.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace dkgk {

// K5: 32-byte encodings [count][8 words] -> extended SoA [40][stride]; ok[e] = 1 if valid.
void decode_points(const uint32_t* comp, size_t count, uint32_t* ext, size_t stride, uint8_t* ok,
                   hipStream_t stream);
// K5 straight into the binomial's position-major layout: D dealers x N commitments ([D][N][8],
// dealer-major) -> [40][N][npad].  nseg segments are interleaved in 64-column groups: dealer i of
// segment seg lands in column (i / 64) * 64 * nseg + seg * 64 + i % 64; ok[column * N + k].
// k_decode's placement for points already in extended form (src [D][N], word stride sstride)
void place_position_major(const uint32_t* src, size_t sstride, size_t D, size_t N, size_t npad, uint32_t* out,
                          hipStream_t stream, int nseg = 1, int seg = 0, size_t L = 0, size_t pstride = 0);
// dst[i] = src[i * step + k0], i < count (extended points)
void gather_points(const uint32_t* src, size_t sstride, size_t step, size_t k0, size_t count, uint32_t* dst,
                   size_t dstride, hipStream_t stream);
// npad = the table's row width (columns); with a degree split (L < N) coefficient k of column c goes
// to position k % L, column (k / L) * pstride + c, in a table of L rows.
void decode_position_major(const uint32_t* comp, size_t D, size_t N, size_t npad, uint32_t* out, uint8_t* ok,
                           hipStream_t stream, int nseg = 1, int seg = 0, size_t L = 0, size_t pstride = 0);
// every column of a position-major table [40][S] set to the identity
void fill_identity(size_t S, uint32_t* out, hipStream_t stream);
// fused round-2/4 check over interleaved E/A columns (see k_check_both): dealers
// [dealer0, dealer0 + ndealers) of this call, s / sp / dec2 / dec4 indexed dealer * nrecv + j from
// their bases, self = (dealer + dealer_base) mod nmod == j.
void check_both(size_t ndealers, size_t nrecv, size_t dealer0, size_t dealer_base, size_t nmod, const uint32_t* s,
                const uint32_t* sp, const uint32_t* R, const uint32_t* tab_g, const uint32_t* tab_h,
                const uint8_t* dok, uint8_t* dec2, uint8_t* dec4, hipStream_t stream);
// extended SoA -> encodings [count][8]
void encode_points(const uint32_t* ext, size_t stride, size_t count, uint32_t* comp, hipStream_t stream);
// comb tables of the decoded points ext[.., e0 + c], c < count, into tab + c * 15360 (30 x 512 words each)
void build_comb(const uint32_t* ext, size_t stride, size_t e0, uint32_t* tab, hipStream_t stream, size_t count = 1);
// radix-256 combs (COMB8_WORDS words each) of `count` points: the tables of commit / check /
// fixed_base (global memory, L2-resident)
void build_comb8(const uint32_t* ext, size_t stride, size_t e0, uint32_t* tab, hipStream_t stream, size_t count = 1);

// K2: A_k = g a_k, E_k = A_k + h b_k for D*N coefficients (scalars [D*N][8]); outputs SoA [40][DN].
void commit(size_t count, const uint32_t* a, const uint32_t* b, const uint32_t* tab_g,
            const uint32_t* tab_h, uint32_t* A_ext, uint32_t* E_ext, hipStream_t stream);
// K1: s[i][j] = f_i(j+1), s'[i][j] = f'_i(j+1) (scalars [D][n][8]); coefficients [D][N][8].
void share_eval(size_t D, size_t n, size_t N, const uint32_t* a, const uint32_t* b, uint32_t* s,
                uint32_t* sp, hipStream_t stream);
// Polynomial::evaluate for D polynomials at M small integer points x[m] (< 2^24).
void poly_eval(size_t D, size_t N, const uint32_t* coeffs, size_t M, const uint32_t* xs, uint32_t* out,
               hipStream_t stream);

// K3a: binomial-basis Horner.  C: decoded commitments SoA [40][N][npad] (position-major,
// dealer-minor); e0/e1 ping-pong buffers of the same shape.  Processes `width` (multiple of 64)
// dealer columns starting at the given pointers (a dealer chunk: pass C + c0, e0 + c0, e1 + c0).
// Returns the buffer holding e_m = Delta^m P_i(0), m = 0..t.
// pieces > 1: the same for the columns [u * pstride, u * pstride + width) of every piece u
// last_len (0: N): the last piece's length when it is shorter (its coefficients >= last_len are the
// identity); its positions >= last_len are then left unwritten (never read by the stepping).
uint32_t* binomial(size_t width, size_t npad, size_t N, const uint32_t* C, uint32_t* e0, uint32_t* e1,
                   hipStream_t stream, size_t pieces = 1, size_t pstride = 0, size_t last_len = 0);
// Position-major [40][N][npad] -> column-major [40][npad][N] (element c * N + m) for the columns
// [u * pstride, u * pstride + width) of each of `pieces` pieces (the stepping's input layout).
void to_column_major(size_t width, size_t npad, size_t N, const uint32_t* e, uint32_t* eT, size_t pieces,
                     size_t pstride, hipStream_t stream);
// K3b: finite-difference stepping: R[i][j] = P_i(j+1) for j in [0, nrecv), point-major (AoS)
// [i*nrecv + j][40] (pt_store_aos), from the column-major difference table e (to_column_major;
// word stride N * npad).  stream_a / stream_b: scratch for the inter-block boundary streams, each
// >= ndealers*nrecv*160 B (unused when N <= 512).
// How k_stepping covers an N-position table: nblk blocks of P positions on bs lanes (nblk > 1), or
// `per` tables of P = N lanes each per bs-lane workgroup; maxbs = the LDS variant (192, 256 or 512).
struct StepShape {
  size_t nblk, P, per, bs, maxbs;
};
StepShape stepping_shape(size_t N);
// relative issue rate of a bs-lane workgroup in the maxbs LDS variant (resident waves per SIMD)
double step_occupancy(size_t bs, size_t maxbs);
// true when every piece of a split column fits one workgroup slot ((pieces-1) L + last_len <= 512):
// the stepping then runs one slot per column over all pieces
bool stepping_whole_columns(size_t L, size_t pieces, size_t last_len);
// cost model of stepping()'s launches over `cols` columns: SIMD cycles per (receiver step x
// instruction of one addition); compare modes / splits with it
double stepping_cycles(size_t cols, size_t N, size_t pieces, size_t last_len, bool whole);
// last_len (0: N): length of a shorter last piece (its table positions >= last_len are not read)
// whole: run the pieces of a column in one slot when they fit (stepping_whole_columns)
void stepping(size_t ndealers, size_t npad, size_t N, const uint32_t* e, size_t nrecv, uint32_t* R,
              uint32_t* stream_a, uint32_t* stream_b, hipStream_t stream, size_t pieces = 1, size_t pstride = 0,
              size_t last_len = 0, bool whole = true);
// Degree-split recombination: R[c][j] = sum_u y_j^u R[u * pstride + c][j] (pairwise Horner in y^2
// with joint NAF chains; digits [n][2][256] = NAF of y_j and y_j^2, top [n][2])
void combine(size_t width, size_t pstride, size_t pieces, size_t nrecv, const int8_t* digits, const int16_t* top,
             uint32_t* R, hipStream_t stream);
// K3c: decision[i][j] = (g s_ij + h s'_ij == R[i][j]) (round 2) or (g s_ij == R[i][j]) (round 4);
// dealer_ok[i] == 0 forces 0; self ((i + dealer_base) mod nmod == j + recv_base, nmod = parties per
// ceremony, so batched ceremonies stacked dealer-wise work too) gives 2.
// R: point-major (AoS) [i*nrecv + j][40].
void check(size_t ndealers, size_t nrecv, size_t dealer_base, size_t recv_base, size_t nmod, int round,
           const uint32_t* s, const uint32_t* sp, const uint32_t* R, const uint32_t* tab_g,
           const uint32_t* tab_h, const uint8_t* dealer_ok, uint8_t* decision, hipStream_t stream);
// dok[column of dealer i of segment seg] &= extra[i] (verify_device's interleaved column layout)
void and_dealer_mask(size_t D, int nseg, int seg, const uint8_t* extra, uint8_t* dok, hipStream_t stream);
// per-dealer validity: dealer_ok[i] = AND of point_ok over its N commitments (dealer-major [D][N])
void dealer_ok(size_t ndealers, size_t N, const uint8_t* point_ok, uint8_t* ok, hipStream_t stream);
// Horner in the exponent for receivers x0 .. x0+nrecv-1 (1-based indices): R point-major [ndealers*nrecv][40]
void horner(size_t ndealers, size_t npad, size_t N, const uint32_t* C, uint32_t x0, size_t nrecv, uint32_t* R,
            hipStream_t stream);
// out column col + g (SoA, stride ostride) = sum over e in [g*count, (g+1)*count) of mask[e] * P_e
// (mask may be NULL), for each group g < groups.
void sum_points(size_t count, const uint32_t* pts, size_t stride, const uint8_t* mask, uint32_t* out, size_t ostride,
                size_t col, hipStream_t stream, size_t groups = 1);
// out[e] = a[e] + b[e] for SoA point vectors of the same stride (out may alias a)
void add_points(size_t count, const uint32_t* a, const uint32_t* b, size_t stride, uint32_t* out, hipStream_t stream);
// Decision-matrix summaries for `groups` stacked ceremonies of n parties (dec [groups*n][n]):
// row_reject[i] = any REJECT in row i; complaints[g][j] = REJECTs by receiver j in group g.
// out[g*n+j] = 1 + #{qualified i : dec[g][i][j] == ACCEPT} < t + 1 (round-4 MisbehaviourHigherThreshold)
void r4_error(size_t groups, size_t n, size_t t, const uint8_t* dec, const uint8_t* qmask, uint8_t* out,
              hipStream_t stream);
void decision_summary(size_t groups, size_t n, const uint8_t* dec, uint8_t* row_reject, int32_t* complaints,
                      hipStream_t stream);
// hash_to_group tail: from_uniform_bytes(64 bytes as 16 LE words) -> SoA point (stride 1)
void from_uniform(const uint32_t* in16, uint32_t* out, hipStream_t stream);

// Generic batched MSM (trait boundary): out[b] = sum_k scalars[b][k] * points[b][k];
// points given decoded SoA [40][B*N] (element b*N + k), scalars [B*N][8].
void msm_batch(size_t B, size_t N, const uint32_t* scalars, const uint32_t* pts, size_t stride, uint32_t* tab,
               uint32_t* out_ext, hipStream_t stream);
// Fixed-base batch: out = s * base via comb table; out SoA [40][count]
void fixed_base(size_t count, const uint32_t* scalars, const uint32_t* tab, uint32_t* out_ext,
                hipStream_t stream);
// Transpose dealer-major point SoA [40][D*N] (element i*N+k) to position-major [40][N][npad].
void to_position_major(size_t D, size_t N, size_t npad, const uint32_t* in, uint32_t* out,
                       hipStream_t stream);
// Scalar reduction of 256-bit inputs to canonical (from_bits semantics, groups.rs:29-36).
void reduce_scalars(size_t count, const uint32_t* in, uint32_t* out, hipStream_t stream);
// Modular sum over dealers with mask: out[j] = sum_i mask[i] * s[i][j]  (round-3 final share)
void sum_shares(size_t D, size_t n, const uint32_t* s, const uint8_t* mask, uint32_t* out, hipStream_t stream,
                size_t groups = 1);
// On-device synthetic coefficients (seedgen.hip): rows r in [0, rows) are dealer d0 + r % D of
// ceremony c0 + r / D; a, b [rows][N][8] canonical, identical to the host dkg_dealer_coeffs.
// master: 8 words on the device; seeds: scratch [rows][8].
void dealer_coeffs(size_t rows, size_t D, size_t d0, uint32_t c0, const uint32_t* master, size_t N, uint32_t* seeds,
                   uint32_t* a, uint32_t* b, hipStream_t stream);

// ---- full (encrypted-share) mode, hybrid.hip (elgamal.rs:134-193) ----
// Items are (dealer i, recipient q, w) at index (i * n + q) * 2 + w; w = 0 is the randomness (s')
// ciphertext, w = 1 the share (s) ciphertext (committee.rs:171-172 order).
// R = g r, K = pk_q r for every item (r [items][8]); tab_g8: the generator's radix-256 comb;
// tabs_pk: one (radix-16) comb table per recipient.
void enc_mul(size_t D, size_t n, const uint32_t* r, const uint32_t* tab_g8, const uint32_t* tabs_pk, uint32_t* R_ext,
             uint32_t* K_ext, hipStream_t stream);
// K = sk_q * R for every item, R decoded SoA [40][items] (sk [n][8], wave-uniform per recipient)
void dec_mul(size_t D, size_t n, const uint32_t* sk, const uint32_t* R_ext, uint32_t* K_ext, hipStream_t stream);
// SymmetricKey::process: keystream from Blake2b-512(Kc) (Kc [items][8] encodings).
// encrypt: ct[item] = (w ? s : sp)[i*n+q] ^ ks.  decrypt: (w ? s : sp)[i*n+q] = reduce(from_bits(ct[item] ^ ks)).
void sym_xor(size_t D, size_t n, const uint32_t* Kc, bool decrypt, uint32_t* ct, uint32_t* s, uint32_t* sp,
             hipStream_t stream);
// per-row dealer seeds [rows][8] (row r = dealer d0 + r % D of ceremony c0 + r / D; seedgen.hip)
void dealer_seeds(size_t rows, size_t D, size_t d0, uint32_t c0, const uint32_t* master, uint32_t* seeds,
                  hipStream_t stream);
// encryption randomness rows (seedgen.hip): r [rows][n][2][8] = wide(block 2N + 2q + w) of each dealer stream
void enc_randomness(size_t rows, size_t n, size_t N, const uint32_t* seeds, uint32_t* r, hipStream_t stream);

// ---- committee verification by interpolation (interp.hip)
// F[d][k] = sum_j W[k][j] s[d][j] (and F' from s'; sp may be null), WT[j][k] = W[k][j] in Montgomery form
void interp(size_t D, size_t N, size_t nrecv, const uint32_t* WT, const uint32_t* s, const uint32_t* sp, uint32_t* F,
            uint32_t* Fp, hipStream_t stream);
// per (d, k): okA = (g F_k == A_k), okE = (g F_k + h F'_k == E_k); commitments [D][N] extended
void coef_check(size_t D, size_t N, const uint32_t* F, const uint32_t* Fp, const uint32_t* Eext, const uint32_t* Aext,
                size_t cstride, const uint32_t* tab_g, const uint32_t* tab_h, uint8_t* okE, uint8_t* okA,
                hipStream_t stream);
// round-2 / round-4 decisions of the rows whose coefficient test passed (others: 0, re-verified)
void interp_decide(size_t D, size_t nrecv, size_t N, size_t dealer_base, size_t nmod, const uint32_t* s,
                   const uint32_t* sp, const uint32_t* F, const uint32_t* Fp, const uint8_t* dokE, const uint8_t* dokA,
                   const uint8_t* cE, const uint8_t* cA, const uint32_t* tab_g, const uint32_t* tab_h, uint8_t* dec2,
                   uint8_t* dec4, hipStream_t stream);
// ok[i] &= extra[i], i < D
void and_mask(size_t D, const uint8_t* extra, uint8_t* ok, hipStream_t stream);

}  // namespace dkgk
