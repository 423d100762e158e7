// Host runtime of the MI355X DKG backend: device context, buffer arena, the C ABI of
// include/dkg_amd.h, and the ceremony driver that plays the reference's rounds 1-5
// (committee.rs:124-805) for all parties in one process on one GPU.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <map>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "../../include/dkg_amd.h"
#include "host_crypto.h"
#include "kernels.h"
#include "kernels_ilp.h"

struct dkg_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  std::string err;
  std::map<std::string, std::pair<void*, size_t>> bufs;
  std::map<std::string, std::pair<void*, size_t>> hbufs;  // pinned host staging (hbuf), grow-only
  uint32_t* tab_g = nullptr;  // comb table of the generator (15360 words)
  uint32_t* tab_h = nullptr;  // comb table of the commitment key h
  uint32_t* tab_gw = nullptr;  // radix-2^11 combs (global, L2 / MALL-resident) of g and h: commit, check,
  uint32_t* tab_hw = nullptr;  // fixed-base products
  uint8_t h[32] = {0};
  bool have_h = false;
  size_t threshold = 0, nr_members = 0;
  hipEvent_t ev[8] = {};
  hipEvent_t pev[5] = {};               // phase profiling inside verify_device (nsub == 1)
  hipEvent_t hev[9] = {};               // full mode: encrypt / decrypt kernels (nsub == 1)
  int hy_timed = 0;                     // hev[] hold the phases of the last serialised encrypt (1)
                                        // and / or decrypt (2) since the last collect_hybrid_phases
  static constexpr int MAX_SUB = 8;
  int nsub = 2;                         // dealer-chunk streams of verify_device
  hipStream_t sub[MAX_SUB] = {};
  hipEvent_t fork = nullptr, join[MAX_SUB] = {};
  // round-1 share evaluation on a low-priority side stream beside the first binomial steps
  // (round1_device with overlap_shares): the checks and round 3 wait for shares_done
  hipStream_t side = nullptr;
  hipEvent_t side_fork = nullptr, shares_done = nullptr, pub_done = nullptr;
  hipEvent_t terms_done = nullptr;      // a shard's master-key terms, encoded on the side stream
  bool shares_pending = false;
  bool overlap = true;                  // rounds 2 and 4 as one fused pipeline (verify_rounds)
  int split = 0;                        // degree split U of the difference tables (0: cost model)
  std::vector<uint8_t> key_tabs_pk;     // member keys whose decoded points and combs sit in hy.* (encrypt)
  uint8_t fb_base[32] = {0};            // dkg_fixed_base_batch: the caller base whose comb sits in fb_tabw
  bool fb_valid = false;
  int binom_mode = 0;                   // binomial: 0 per-wave Horner loops (k_binom_wave) for
                                        // tables of many column groups, else one launch per step
                                        // with lane pairs (k_binom_pair) for the steps under one
                                        // wave per SIMD; 1 per step, no lane pairs; 2 per step, lane
                                        // pairs for every step; 3 per step as 0; 4 per wave always;
                                        // 5 per wave always, operands prefetched one item ahead
  int step_mode = 0;                    // stepping slots: 0 cost model, 1 whole columns, 2 per piece,
                                        // 3 as 0 without the dead-position repack
  int check_mode = 0;                   // fused round-2/4 checks: 0 one launch, 1 the g and h combs
                                        // in two launches (g*s parked between them)
  int fe_mode = 0;                      // field multiplication per launch: 0 by occupancy, 1 product
                                        // scanning (dkgk), 2 column sums (dkgk_ilp)
  int verify_mode = 0;                  // 0: difference tables (every P_i(j) in the group); 1: interpolation
  size_t vinv_N = 0;                    // key of the cached inverse Vandermonde (v.vinv)
  size_t fallback_rows = 0;             // interpolation mode: rows re-verified the general way
  int last_split = 1;                   // U used by the last verify_device
  size_t last_split_len = 0;            // and its piece length L
  size_t ydig_n = 0, ydig_L = 0;        // key of the cached combine multipliers (v.ydig)
  int combine_mode = 0;                 // recombination: 0 short vectors for U <= 5 (4 with
                                        // projective addends), 1 powers of y, 2 = 0
  int last_combine = 0;                 // 1: the last verify_device recombined with powers, 2: short vectors
  int last_binomial = 0;                // 1: the last verify_device ran the per-wave binomial
  int step_formula = 0;                 // stepping additions: 0 dedicated + complete redo of marked
                                        // workgroups, 1 complete formula only
  uint32_t* last_step_flags = nullptr;  // the last verify_device's stepping flags (dedicated mode)
  size_t last_step_flag_words = 0;
  // the per-step binomial's dedicated additions: only inside the drivers that check its group flags
  // after their sync and rerun the verification with the complete formula when one is set
  // (receivers_rounds, shard_rows: binom_step_ded = true around the call)
  bool binom_step_ded = false;
  uint32_t* binom_any = nullptr;        // device word: a dedicated per-step binomial marked a group
                                        // since the last verify_rounds began (null: none ran)
  const uint32_t* binom_any_host = nullptr;  // its pinned copy, queued before the caller's sync
  int last_binom_rerun = 0;             // the last guarded driver reran its verification (1) or not
  int addend_mode = 0;                  // short vectors' addends: 0 affine Niels (affine_pieces, mixed
                                        // additions), 1 cached projective (read from R)
  size_t sdig_n = 0, sdig_L = 0, sdig_K = 0;  // key of the cached short multipliers (v.sdig)
  // round-1 commitments of the ceremony being verified, in extended form on this device (set by
  // the drivers that generate them, ExtScope): verify_device places them instead of decoding the
  // encodings, finalise reads A_i0 from them.  E/A [D][t+1] points, word stride ext_stride.
  const uint32_t* ext_E = nullptr;
  const uint32_t* ext_A = nullptr;
  // round-1 commitments deferred into the verification's chunks (batches, BatchRound1): coefficients
  // [r1_D][N][8]; each chunk's stream computes its dealers' E/A into ext_E / ext_A before its
  // binomial, so one chunk's commitments run beside the other chunk's pipeline
  const uint32_t* r1_a = nullptr;
  const uint32_t* r1_b = nullptr;
  size_t r1_D = 0;
  uint32_t* r1_A0 = nullptr;            // [40][r1_D]: A_i0 of the deferred commitments (finalise)
  size_t ext_stride = 0;
  // share rows [shard_D][shard_n][8] of the last sharded call's dealers [shard_d0, +shard_D)
  // (arena-owned; dkg_ceremony_shard_recon_device reads them after the exchange)
  const uint32_t* shard_s = nullptr;
  size_t shard_n = 0, shard_d0 = 0, shard_D = 0;
  std::string timed_tag;                // set while pev[] hold a serialised verify_device's phases
  std::map<std::string, double> phase_ms;  // last value per "r<round>.<phase>"
};

namespace {

constexpr size_t PTB = 160;  // bytes of one extended point (40 words)
constexpr size_t PT_WORDS_H = 40;
constexpr size_t AFFP_WORDS_H = 32;  // affine addend slot of kernels.hip affine_pieces
constexpr size_t COMB_BYTES = 30 * 512 * 4;
#ifndef DKG_COMBW_BITS
#define DKG_COMBW_BITS 19
#endif
// points.h COMBW_WORDS x 4 (radix 2^19: 14 windows x 262,144 entries x 128 B = 470 MB)
constexpr size_t COMBW_BYTES =
    (size_t)(256 / DKG_COMBW_BITS + 1) * (1u << (DKG_COMBW_BITS - 1)) * 32 * 4;
const uint8_t BASEPOINT[32] = {0xe2, 0xf2, 0xae, 0x0a, 0x6a, 0xbc, 0x4e, 0x71, 0xa8, 0x84, 0xa9,
                               0x61, 0xc5, 0x00, 0x51, 0x5f, 0x58, 0xe3, 0x0b, 0x6a, 0xa5, 0x82,
                               0xdd, 0x8d, 0xb6, 0xa6, 0x59, 0x45, 0xe0, 0x8d, 0x2d, 0x76};

struct Fail {
  int code;
};

#define HCK(call)                                                                      \
  do {                                                                                 \
    hipError_t e_ = (call);                                                            \
    if (e_ != hipSuccess) {                                                            \
      ctx->err = std::string(#call) + ": " + hipGetErrorString(e_);                    \
      throw Fail{DKG_E_DEVICE};                                                        \
    }                                                                                  \
  } while (0)

template <typename T = void>
T* buf(dkg_ctx* ctx, const char* name, size_t bytes) {
  if (bytes == 0) bytes = 16;
  auto it = ctx->bufs.find(name);
  if (it != ctx->bufs.end() && it->second.second >= bytes) return reinterpret_cast<T*>(it->second.first);
  if (it != ctx->bufs.end()) {
    HCK(hipDeviceSynchronize());  // the old buffer may still be read on any of the ctx's streams
    HCK(hipFree(it->second.first));
    ctx->bufs.erase(it);
  }
  void* p = nullptr;
  hipError_t e = hipMalloc(&p, bytes);
  if (e != hipSuccess) {
    ctx->err = std::string("hipMalloc(") + name + ", " + std::to_string(bytes) + "): " + hipGetErrorString(e);
    throw Fail{DKG_E_NOMEM};
  }
  ctx->bufs[name] = {p, bytes};
  return reinterpret_cast<T*>(p);
}

// Pinned host staging, name-keyed and grow-only like buf(): device-to-host copies into it are plain
// DMA transfers that complete with the stream, where a copy into pageable memory makes the runtime
// stage it through its own buffers on the calling thread.
template <typename T = void>
T* hbuf(dkg_ctx* ctx, const char* name, size_t bytes) {
  if (bytes == 0) bytes = 16;
  auto it = ctx->hbufs.find(name);
  if (it != ctx->hbufs.end() && it->second.second >= bytes) return reinterpret_cast<T*>(it->second.first);
  if (it != ctx->hbufs.end()) {
    HCK(hipDeviceSynchronize());  // a copy into the old buffer may still be queued
    HCK(hipHostFree(it->second.first));
    ctx->hbufs.erase(it);
  }
  void* p = nullptr;
  hipError_t e = hipHostMalloc(&p, bytes, hipHostMallocDefault);
  if (e != hipSuccess) {
    ctx->err = std::string("hipHostMalloc(") + name + ", " + std::to_string(bytes) + "): " + hipGetErrorString(e);
    throw Fail{DKG_E_NOMEM};
  }
  ctx->hbufs[name] = {p, bytes};
  return reinterpret_cast<T*>(p);
}

void h2d(dkg_ctx* ctx, void* d, const void* h, size_t n) {
  if (n) HCK(hipMemcpyAsync(d, h, n, hipMemcpyHostToDevice, ctx->stream));
}
void d2h(dkg_ctx* ctx, void* h, const void* d, size_t n) {
  if (n) HCK(hipMemcpyAsync(h, d, n, hipMemcpyDeviceToHost, ctx->stream));
}
void sync(dkg_ctx* ctx) {
  HCK(hipStreamSynchronize(ctx->stream));
}
void check_launch(dkg_ctx* ctx) { HCK(hipGetLastError()); }

size_t pad64(size_t x) { return (x + 63) / 64 * 64; }

template <typename F>
int guarded(dkg_ctx* ctx, F&& f) {
  if (!ctx) return DKG_E_ARG;
  try {
    HCK(hipSetDevice(ctx->device));
    int rc = f();
    return rc;
  } catch (const Fail& x) {
    return x.code;
  } catch (const std::exception& x) {
    ctx->err = x.what();
    return DKG_E_NOMEM;
  }
}

// Decode one 32-byte point and build its comb table into `tab`.
// Comb tables of one point: radix-16 (LDS kernels; may be null) and radix-2^11 (may be null).
void comb_for_point(dkg_ctx* ctx, const uint8_t p[32], uint32_t* tab, bool* ok, uint32_t* tab8 = nullptr) {
  uint32_t* comp = buf<uint32_t>(ctx, "comb_in", 32);
  uint32_t* ext = buf<uint32_t>(ctx, "comb_ext", PTB);
  uint8_t* okd = buf<uint8_t>(ctx, "comb_ok", 1);
  h2d(ctx, comp, p, 32);
  dkgk::decode_points(comp, 1, ext, 1, okd, ctx->stream);
  if (tab) dkgk::build_comb(ext, 1, 0, tab, ctx->stream);
  if (tab8) dkgk::build_combw(ext, 1, 0, tab8, ctx->stream);
  check_launch(ctx);
  uint8_t v = 0;
  d2h(ctx, &v, okd, 1);
  sync(ctx);
  *ok = v != 0;
}

// Upload scalars (32-byte encodings) and reduce them mod l (from_bits semantics, groups.rs:29-36).
uint32_t* upload_scalars(dkg_ctx* ctx, const char* name, const uint8_t* host, size_t count) {
  uint32_t* raw = buf<uint32_t>(ctx, "scalar_raw", 32 * count);
  uint32_t* red = buf<uint32_t>(ctx, name, 32 * count);
  h2d(ctx, raw, host, 32 * count);
  dkgk::reduce_scalars(count, raw, red, ctx->stream);
  return red;
}

// Nontemporal stores for binomial step r over `columns` table columns (all chunks run their steps
// together): when the step's rows read + written, 2 (r + 1) columns 160 B, exceed DKG_BINOM_NT_BYTES
// (kernels.hip binom_pt_store).  The environment variable overrides the default for A/B runs.
// Default 0 = every step: the serialised n=1024 binomial 21.5-21.8 -> 20.4-20.6 ms, thresholds of
// 180 / 256 / 320 MB in between; config 4 and the whole ceremony within noise
// (profiles/r06_binom_levers_ab.txt, recipe r06e).
#ifndef DKG_BINOM_NT_BYTES_DEFAULT
#define DKG_BINOM_NT_BYTES_DEFAULT 0.0
#endif
bool binom_nt(size_t r, size_t columns) {
  static const double lim = [] {
    const char* e = getenv("DKG_BINOM_NT_BYTES");
    return e ? atof(e) : DKG_BINOM_NT_BYTES_DEFAULT;
  }();
  return 2.0 * (double)(r + 1) * (double)columns * 160.0 > lim;
}

// After a sync: record the device time of binomial / stepping / check of the last verify_device
// when it ran serialised and timed (names "<tag>.binomial" etc.; tag r2, r4 or r24 = fused).
void collect_phases(dkg_ctx* ctx) {
  if (ctx->timed_tag.empty()) return;
  const char* names[4] = {"binomial", "stepping", "combine", "check"};
  for (int i = 0; i < 4; i++) {
    float ms = 0;
    HCK(hipEventElapsedTime(&ms, ctx->pev[i], ctx->pev[i + 1]));
    ctx->phase_ms[ctx->timed_tag + "." + names[i]] = ms;
  }
  ctx->timed_tag.clear();
}

// One block of rows to verify: `D` dealers [dealer_base, dealer_base + D) against receivers
// 0..n-1 in `round` (2: h*s' + g*s == sum_k j^k E_i[k]; 4: g*s == sum_k j^k A_i[k]).
// Ccomp [D][N][8] compressed commitments; s, sp [D][n][8] canonical; dec [D][n].
struct VerifySeg {
  int round;
  size_t D, dealer_base;
  const uint32_t* Ccomp;
  const uint32_t* s;
  const uint32_t* sp;
  uint8_t* dec;
  const uint8_t* extra_ok = nullptr;  // [D] device: 0 = the dealer's other broadcast data is missing
  size_t self_mod = 0;                // self = (dealer + dealer_base) mod self_mod == j; 0: n
};

// Which copy of a kernel runs a launch: product scanning (dkgk, fewer issue slots) or column sums
// (dkgk_ilp, ten independent chains per multiplication) when the launch leaves too few waves per
// SIMD to hide the serial chain (`latency_bound`), unless dkg_ctx_set_field_mode forces one.
// Binomial steps with fewer waves per SIMD than this run the column-sum copy (kernels_ilp.h).
#ifndef DKG_BINOM_PAIR_WAVES
#define DKG_BINOM_PAIR_WAVES 1.0
#endif
#ifndef DKG_BINOM_ILP_WAVES
#define DKG_BINOM_ILP_WAVES 1.5
#endif
// Product-scanning steps with fewer waves per SIMD than this run k_binom_step<.., IL> (paired
// products at a 2-wave launch bound); the environment variable DKG_BINOM_IL_WAVES overrides it (A/B).
#ifndef DKG_BINOM_IL_WAVES_DEFAULT
#define DKG_BINOM_IL_WAVES_DEFAULT 0.0
#endif
double binom_il_waves() {
  static const double v = [] {
    const char* e = getenv("DKG_BINOM_IL_WAVES");
    return e ? atof(e) : DKG_BINOM_IL_WAVES_DEFAULT;
  }();
  return v;
}
double binom_ilp_waves() {  // DKG_BINOM_ILP_WAVES, overridable the same way (A/B)
  static const double v = [] {
    const char* e = getenv("DKG_BINOM_ILP_WAVES");
    return e ? atof(e) : DKG_BINOM_ILP_WAVES;
  }();
  return v;
}
// Tables of at least this many 64-column groups (all pieces, all chunks) run the binomial as one
// launch of per-wave Horner loops (kernels.hip k_binom_wave): each wave then has a long private
// chain, and 4 rounds of a chip's resident waves keep the last round's tail small.  Fewer groups
// (n=1024: 128; n=4096: 512) keep one launch per step.
#ifndef DKG_BINOM_WAVE_PF  // the per-wave binomial's default: operands prefetched one item ahead
#define DKG_BINOM_WAVE_PF 0   // (2 waves per SIMD: config 5 +5.5 ms, profiles/r05_b5_ab.txt)
#endif
#ifndef DKG_BINOM_WAVE_DED  // the per-wave binomial with dedicated additions (+ complete redo)
#define DKG_BINOM_WAVE_DED 1
#endif
// the per-step binomial's steps without lane pairs likewise (0.5 ms on the headline, 22 ms on config
// 4, profiles/r05_binom_ded_ab.txt): in the drivers that rerun the verification with the complete
// formula when a step marked the guard word (with_binom_ded: at most twice the honest time); 2 = redo
// per wave after the last step instead (a slow worst case: a per-wave loop over a whole triangle)
#ifndef DKG_BINOM_STEP_DED
#define DKG_BINOM_STEP_DED 1
#endif
#ifndef DKG_BINOM_WAVE_COLMAJOR  // its last step writing the stepping's column-major table itself:
#define DKG_BINOM_WAVE_COLMAJOR 0  // 4-B stores 128 B apart, +10 ms against k_to_column_major's 3.3
#endif                             // (config 5, profiles/r05_b5_ab.txt)
#ifndef DKG_BINOM_WAVE_GROUPS
#define DKG_BINOM_WAVE_GROUPS 16384
#endif

bool use_ilp(const dkg_ctx* ctx, bool latency_bound) {
  return ctx->fe_mode == 2 || (ctx->fe_mode == 0 && latency_bound);
}

// Work on `st` that reads the shares waits for an overlapped share evaluation (round1_device).
void wait_shares(dkg_ctx* ctx, hipStream_t st) {
  if (ctx->shares_pending) HCK(hipStreamWaitEvent(st, ctx->shares_done, 0));
}

// Coefficients held by the last of U pieces of length L (N = t + 1).  A forced split can leave the
// last pieces without any (N = 6, U = 5: L = 2, pieces 2 + 2 + 2 + 0 + 0); such a piece is a
// full-length table of identities, as are the positions past t of a ragged one.
size_t last_piece_len(size_t N, size_t U, size_t L) {
  return (U - 1) * L < N ? N - (U - 1) * L : L;
}

// Whole-column stepping slots (all U pieces of a column in one workgroup slot) when they fit and
// the launch model says so (ties to per-piece slots: more, smaller workgroups; measured on the
// 8-way n=1024 shard at U=4, 19.8 vs 20.9 ms, profiles/r02_shard_stepping_ab.txt).
bool stepping_whole_pays(size_t cols, size_t U, size_t L, size_t Lr) {
  return dkgk::stepping_whole_columns(L, U, Lr) &&
         dkgk::stepping_cycles(cols, L, U, Lr, true) < 0.98 * dkgk::stepping_cycles(cols, L, U, Lr, false);
}

// ---- degree split ----
// P(x) = sum_{u<U} x^(uL) Q_u(x), deg Q_u < L = ceil(N / U): the binomial-basis Horner runs on the
// U pieces (quadratic in the degree: ~1/U of the work, and ~1/U of the dependent chain), the
// stepping does the same number of additions, and one recombination per (column, receiver) adds
// U-1 multiplications by y_j = j^L mod l (k_combine).  Split when that is cheaper.
// Instruction-count model of binomial + stepping + recombination (static VALU counts of the
// kernels; the check does not depend on U) in SIMD
// cycles: a SIMD retires one wave instruction per ~4.5 cycles of this mix when it has >= 2 waves,
// one per ~8 when a lone wave runs a dependent chain (tools/ubench/ilp.hip); 1024 SIMDs.
// Short multipliers are implemented up to this many pieces (k_combine_aff's digit words; the
// projective-addend k_combine_short stops at 4)
constexpr size_t SHORT_MAX = 5;
#ifndef DKG_AUTO_SHORT5
#define DKG_AUTO_SHORT5 0
#endif

double split_model_ms(size_t cols, size_t n, size_t N, size_t U, size_t L, bool short_mult) {
  const double DBL = 1000, ADD = 1400, SIMDS = 1024, THR = 4.5, LAT = 8, LAT_ILP = 6, LAUNCH = 3e-3 * 2.4e6;
  const size_t Lr = last_piece_len(N, U, L), off = L - Lr;  // the last piece: Lr positions, starts at step off
  auto cost = [&](size_t m) {  // one binomial position-step: add + multiplication by m
    // length and weight of m's recoding as the kernels do it (points.h small_recode: the NAF, a
    // leading 1 0 -1 turned into 1 1 -- one doubling fewer)
    uint64_t pos = 0, neg = 0;
    int len = 0;
    for (uint64_t v = m; v; v >>= 1, len++) {
      if (v & 1) {
        if ((v & 3) == 1) {
          pos |= 1ull << len;
          v -= 1;
        } else {
          neg |= 1ull << len;
          v += 1;
        }
      }
    }
    if (len >= 3 && !(((pos | neg) >> (len - 2)) & 1) && ((neg >> (len - 3)) & 1)) {
      pos = (pos & ~(1ull << (len - 1))) | (3ull << (len - 3));
      neg &= ~(1ull << (len - 3));
      len--;
    }
    const int nz = __builtin_popcountll(pos | neg);
    return ADD + (len > 1 ? (len - 1) * DBL + (nz - 1) * ADD : 0.0);
  };

  std::vector<double> pre(L + 1, 0.0);
  for (size_t m = 1; m <= L; m++) pre[m] = pre[m - 1] + cost(m);
  const double waves_col = (double)cols / 64;
  double cyc = 0;
  for (size_t r = 1; r < L; r++) {
    // wave-instructions of step r: U-1 full pieces, the last one from step off on
    const double work = waves_col * ((U - 1) * pre[r] + (r > off ? pre[r - off] : 0.0)) * THR / SIMDS;
    // a step pays its issue work AND its longest chain: the last waves of a launch run their chains
    // on partly idle SIMDs (the sum fits the measured shards within 5 %: 1-, 2-, 4-, 8-way n=1024,
    // one-GPU n=4096; the max alone picked U=2 for a 4-way n=1024 shard, 3 % slower than U=4).
    // Steps with under 1.5 waves per SIMD run the column-sum copy (verify_device), whose ten
    // independent chains per multiplication shorten the latency-bound chain (8-way n=1024 shard:
    // binomial 6.78 -> 6.26 ms at U=3, profiles/r02_shard_stepping_ab.txt).
    const double lat = waves_col * U * (r + 1) / SIMDS < 1.5 ? LAT_ILP : LAT;
    cyc += work + cost(r) * lat + LAUNCH;
  }
  if (U > 1) {
    // short multipliers (U <= 4): one joint chain of 253 (U-1)/U doublings over U NAFs of that
    // length (~1/3 nonzero); powers of y: pairwise joint chains, an even U starting with one
    // product (253 doublings + ~85 NAF additions), then (ceil(U/2) - 1) joint y^2 / y steps (253
    // doublings + ~170 additions)
    const double bits = 253.0 * (U - 1) / U;
    const double per = short_mult && U <= SHORT_MAX ? bits * 950 + U * bits / 3 * ADD
                                            : (U % 2 == 0 ? 253 * 950 + 85 * ADD : 0.0) +
                                                  ((U + 1) / 2 - 1) * (253 * 950 + 170 * ADD);
    const double waves = (double)cols / 64 * n;
    cyc += std::max(waves * per * THR / SIMDS, per * LAT);  // the 2-slot variant runs at 2 waves/SIMD as fast
  }
  // stepping: n dependent additions per lane, in the launches k_stepping gets (dkgk::stepping_cycles)
  cyc += n * ADD * dkgk::stepping_cycles(cols, L, U, Lr, stepping_whole_pays(cols, U, L, Lr));
  return cyc / 2.4e6;
}

// Piece length of a U-way split: ceil(N / U), or that rounded up to a multiple of 64 when the
// model prefers it -- whole 64-lane waves for the stepping's per-piece tables and a shorter last
// piece (N = 550, U = 2: 320 + 230 instead of 275 + 275, two tables of 5 and 4 waves instead of
// 5 + 5 with 45 idle lanes each).  When all pieces of a column fit one stepping workgroup
// (N <= 512) ceil(N / U) always wins: N = 512, U = 3 runs 171 + 171 + 170 on 512 lanes.
size_t split_len(size_t cols, size_t n, size_t N, size_t U, bool short_mult = true) {
  const size_t L1 = (N + U - 1) / U;
  if (U == 1) return L1;
  const size_t L64 = (L1 + 63) / 64 * 64;
  if (L64 == L1 || (U - 1) * L64 >= N) return L1;
  return split_model_ms(cols, n, N, U, L64, short_mult) < split_model_ms(cols, n, N, U, L1, short_mult) ? L64 : L1;
}

double split_model_ms(size_t cols, size_t n, size_t N, size_t U, bool short_mult = true) {
  return split_model_ms(cols, n, N, U, split_len(cols, n, N, U, short_mult), short_mult);
}

size_t choose_split(dkg_ctx* ctx, size_t cols, size_t n, size_t N) {
  if (ctx->split > 0) return std::min<size_t>((size_t)ctx->split, N);
  const bool sm = ctx->combine_mode != 1;
  const double base = split_model_ms(cols, n, N, 1, sm);
  std::vector<double> ms(17, 0.0);
  double best_ms = base;
  size_t umax = 1;
  for (size_t U = 2; U <= 16; U++) {
    if (N < 64 * U) break;  // pieces of degree < 63: the binomial is cheap already
    // five-piece short multipliers are priced for the automatic choice only with DKG_AUTO_SHORT5:
    // they are parity-tested (forced splits) but their shard timings are unmeasured, so by default
    // the model ranks U = 5 with powers as before (it then never wins) -- dkg_ctx_set_split(5)
    // runs them
    ms[U] = split_model_ms(cols, n, N, U, sm && (U <= 4 || (ctx->addend_mode == 0 && DKG_AUTO_SHORT5)));
    best_ms = std::min(best_ms, ms[U]);
    umax = U;
  }
  if (!(best_ms < 0.9 * base)) return 1;  // only for a clear win
  // the model's best (with short multipliers it ranks the measured n=1024 shards right: U=4 ahead
  // of U=3 by 0.3-0.5 ms per rank at 1-8 ranks, U=5 -- powers of y again -- far behind;
  // profiles/r02_lattice_ab.txt)
  for (size_t U = 2; U <= umax; U++)
    if (ms[U] <= best_ms) return U;
  return 1;
}

// NAF of y = (j+1)^L mod l and of y^2 for receivers j = 0..n-1 (k_combine's wave-uniform
// multipliers), cached per (n, L) on the device: digits [n][2][256] int8, top [n][2] int16.
void naf_digits(const uint8_t b[32], int8_t* d, int16_t* tp) {
  uint32_t k[9] = {0};
  for (int w = 0; w < 8; w++)
    k[w] = (uint32_t)b[4 * w] | (uint32_t)b[4 * w + 1] << 8 | (uint32_t)b[4 * w + 2] << 16 | (uint32_t)b[4 * w + 3] << 24;
  *tp = -1;
  for (int i = 0; i < 256; i++) {  // k < 2^253: the NAF fits in 254 digits
    d[i] = 0;
    if (!((k[i >> 5] >> (i & 31)) & 1u)) continue;
    int8_t dg = 1;
    if ((k[(i + 1) >> 5] >> ((i + 1) & 31)) & 1u) {  // ...11: digit -1, k += 2^i
      dg = -1;
      uint64_t carry = 1ull << (i & 31);
      for (int w = i >> 5; carry && w < 9; w++) {
        const uint64_t sum = (uint64_t)k[w] + carry;
        k[w] = (uint32_t)sum;
        carry = sum >> 32;
      }
    } else {
      k[i >> 5] &= ~(1u << (i & 31));
    }
    d[i] = dg;
    *tp = (int16_t)i;
  }
}

void split_digits(dkg_ctx* ctx, size_t n, size_t L, const int8_t** digits, const int16_t** top) {
  int8_t* dd = buf<int8_t>(ctx, "v.ydig", 512 * n);
  int16_t* dt = buf<int16_t>(ctx, "v.ytop", 4 * n);
  *digits = dd;
  *top = dt;
  if (ctx->ydig_n == n && ctx->ydig_L == L) return;
  std::vector<int8_t> hd(512 * n, 0);
  std::vector<int16_t> ht(2 * n, -1);
  for (size_t j = 0; j < n; j++) {
    dkgh::Zl x = dkgh::zl_from_u64(j + 1), y = dkgh::zl_from_u64(1);
    for (size_t e = L; e; e >>= 1) {  // y = x^L
      if (e & 1) y = dkgh::zl_mul(y, x);
      x = dkgh::zl_mul(x, x);
    }
    uint8_t b[32];
    dkgh::zl_to_bytes(b, y);
    naf_digits(b, &hd[512 * j], &ht[2 * j]);
    dkgh::zl_to_bytes(b, dkgh::zl_mul(y, y));
    naf_digits(b, &hd[512 * j + 256], &ht[2 * j + 1]);
  }
  h2d(ctx, dd, hd.data(), hd.size());
  h2d(ctx, dt, ht.data(), 4 * n);
  ctx->ydig_n = n;
  ctx->ydig_L = L;
}

// Short recombination multipliers (lattice.cpp) of receivers j = 1..n for a K-way split, K <= 4
// (k_combine_short): digits [n][256] u32, byte u of word b = the signed NAF digit at position b of
// the scalar of piece u; top [n] int16 = the highest position with a nonzero digit; scale [n][8]
// words = b_j 2^256 mod l, the checks' Montgomery factor taking s to b_j s.  Cached per (n, L, K).
// (one LLL per receiver, ~1 ms at K = 4: spread over up to 16 host threads)
void short_vectors(size_t n, size_t L, size_t K, std::vector<uint8_t>& mag, std::vector<int8_t>& sign) {
  mag.assign(n * K * 32, 0);
  sign.assign(n * K, 1);
  auto rows = [&](size_t j0, size_t j1) {
    for (size_t j = j0; j < j1; j++) {
      dkgh::Zl x = dkgh::zl_from_u64(j + 1), y = dkgh::zl_from_u64(1);
      for (size_t e = L; e; e >>= 1) {  // y = x^L
        if (e & 1) y = dkgh::zl_mul(y, x);
        x = dkgh::zl_mul(x, x);
      }
      dkgh::short_multipliers(y, (int)K, reinterpret_cast<uint8_t(*)[32]>(&mag[j * K * 32]), &sign[j * K]);
    }
  };
  const size_t nt = std::min<size_t>({(size_t)std::max(1u, std::thread::hardware_concurrency()), 16, (n + 63) / 64});
  std::vector<std::thread> th;
  for (size_t i = 1; i < nt; i++) th.emplace_back(rows, n * i / nt, n * (i + 1) / nt);
  rows(0, n / nt);
  for (auto& t : th) t.join();
}

void split_short(dkg_ctx* ctx, size_t n, size_t L, size_t K, const uint32_t** digits, const int16_t** top,
                 const uint32_t** scale) {
  uint32_t* dd = buf<uint32_t>(ctx, "v.sdig", 2 * 4 * 256 * n);  // word 0: pieces 0..3, word 1: 4..
  int16_t* dt = buf<int16_t>(ctx, "v.stop", 2 * n);
  uint32_t* ds = buf<uint32_t>(ctx, "v.sscale", 32 * n);
  *digits = dd;
  *top = dt;
  *scale = ds;
  if (ctx->sdig_n == n && ctx->sdig_L == L && ctx->sdig_K == K) return;
  std::vector<uint8_t> mag;
  std::vector<int8_t> sign;
  short_vectors(n, L, K, mag, sign);
  std::vector<uint32_t> hd(2 * 256 * n, 0), hs(8 * n, 0);
  std::vector<int16_t> ht(n, -1);
  uint8_t r256[33] = {0};
  r256[32] = 1;
  const dkgh::Zl R = dkgh::zl_from_bytes_wide(r256, 33);  // 2^256 mod l
  for (size_t j = 0; j < n; j++) {
    for (size_t u = 0; u < K; u++) {
      int8_t d[256];
      int16_t tp;
      naf_digits(&mag[(j * K + u) * 32], d, &tp);
      ht[j] = std::max(ht[j], tp);
      for (int b = 0; b < 256; b++)
        hd[(u / 4) * 256 * n + 256 * j + b] |= (uint32_t)(uint8_t)(int8_t)(d[b] * sign[j * K + u]) << (8 * (u % 4));
    }
    const dkgh::Zl b = dkgh::zl_from_bytes_wide(&mag[j * K * 32], 32);  // b > 0
    uint8_t w[32];
    dkgh::zl_to_bytes(w, dkgh::zl_mul(b, R));
    memcpy(&hs[8 * j], w, 32);
  }
  h2d(ctx, dd, hd.data(), 4 * hd.size());
  h2d(ctx, dt, ht.data(), 2 * n);
  h2d(ctx, ds, hs.data(), 4 * hs.size());
  ctx->sdig_n = n;
  ctx->sdig_L = L;
  ctx->sdig_K = K;
}

// One or two segments on device, as ONE pipeline over "virtual dealers" (table columns).  With two
// segments (round 2 on E and round 4 on A of the SAME dealers) a dealer's E row and A row are two
// independent polynomials in the exponent: the binomial-basis Horner and the stepping never look
// at which one a column is, so both run in the same launches (twice the independent work inside
// each of the t dependent binomial launches, half the launches).  Columns are interleaved in
// 64-dealer groups (E of dealers 64q.., then A of the same dealers) so that a chunk holds both rows
// of its dealers and one fused check computes g*s_ij once for both rounds.  Work is ordered after
// what is queued on ctx->stream and completes on it.  With ctx->nsub > 1 the dealer groups are cut
// into nsub chunks whose binomial -> stepping -> check pipelines run on their own streams, so one
// chunk's partly-filled binomial launches share the CUs with another chunk's work.  nsub == 1
// with `timed` records per-phase device times (dkg_ctx_phase_ms, under `tag`).
void verify_device(dkg_ctx* ctx, size_t n, size_t t, const VerifySeg* segs, int nseg, bool timed,
                   const char* tag) {
  const size_t N = t + 1, D = segs[0].D;
  if (!D) return;
  if (nseg == 2 && (segs[1].D != D || segs[1].dealer_base != segs[0].dealer_base || segs[1].s != segs[0].s ||
                    segs[0].round != 2 || segs[1].round != 4)) {
    ctx->err = "verify_device: fused segments must be round 2 then round 4 of the same dealers";
    throw Fail{DKG_E_ARG};
  }
  const size_t groups = (D + 63) / 64, gw = 64 * nseg;  // columns per dealer group
  const size_t npad = groups * gw;
  // degree split: U pieces of L positions; piece u of column c is table column u * npad + c
  const size_t U = choose_split(ctx, npad, n, N), L = split_len(npad, n, N, U, ctx->combine_mode != 1), W = U * npad;
  const size_t Lr = last_piece_len(N, U, L);  // the last piece's length (L or shorter)
  const bool whole = ctx->step_mode == 1 || ((ctx->step_mode == 0 || ctx->step_mode == 3) && stepping_whole_pays(npad, U, L, Lr));
  // the stepping keeps product scanning even at 2 waves per SIMD (8-way n=1024 shard, one stream:
  // 6.07 vs 6.12 ms with column sums, profiles/r02_shard_stepping_ab.txt); only a forced mode 2
  // switches it
  const bool step_ilp = use_ilp(ctx, false);
  ctx->last_split = (int)U;
  ctx->last_split_len = L;
  hipStream_t home = ctx->stream;
  uint8_t* pok = buf<uint8_t>(ctx, "v.pok", npad * N);
  uint8_t* dok = buf<uint8_t>(ctx, "v.dok", npad);
  uint32_t* Cpm = buf<uint32_t>(ctx, "v.Cpm", PTB * L * W);
  uint32_t* e0 = buf<uint32_t>(ctx, "v.binom0", PTB * L * W);
  uint32_t* e1 = buf<uint32_t>(ctx, "v.binom1", PTB * L * W);
  uint32_t* eT = buf<uint32_t>(ctx, "v.binomT", PTB * L * W);  // column-major copy for the stepping
  uint32_t* R = buf<uint32_t>(ctx, "v.R", PTB * W * n);
  uint32_t *sa = nullptr, *sb = nullptr;
  if (L > 512) {
    sa = buf<uint32_t>(ctx, "v.step_a", PTB * W * n);
    sb = buf<uint32_t>(ctx, "v.step_b", PTB * W * n);
  }
  const int8_t* ydig = nullptr;
  const int16_t* ytop = nullptr;
  const uint32_t *sdig = nullptr, *sscale = nullptr;  // short multipliers: R holds b_j P(j)
  const int16_t* stop = nullptr;
  // short multipliers up to SHORT_MAX pieces with affine addends, 4 with projective ones
  const bool short_mult = U > 1 && U <= (ctx->addend_mode == 0 ? SHORT_MAX : 4) && ctx->combine_mode != 1;
  // stepping flags of the dedicated additions: chunk c0's words start at stepping_flag_words(c0, U)
  uint32_t* sflags = ctx->step_formula == 0
                         ? buf<uint32_t>(ctx, "v.sflags", 4 * dkgk::stepping_flag_words(npad, U)) : nullptr;
  ctx->last_step_flags = sflags;
  ctx->last_step_flag_words = sflags ? dkgk::stepping_flag_words(npad, U) : 0;
  // affine addends: one 128-B slot per (piece column, receiver), like R
  uint32_t* Aff = short_mult && ctx->addend_mode == 0 ? buf<uint32_t>(ctx, "v.Aff", 4 * AFFP_WORDS_H * W * n) : nullptr;
  // the stepping's dense copy of each stored point's Z (40 B), read by the affine normalisation
  uint32_t* Rz = Aff ? buf<uint32_t>(ctx, "v.Rz", 40 * W * n) : nullptr;
  if (short_mult) split_short(ctx, n, L, U, &sdig, &stop, &sscale);
  else if (U > 1) split_digits(ctx, n, L, &ydig, &ytop);
  ctx->last_combine = U > 1 ? (short_mult ? 2 : 1) : 0;
  // padding columns, and the positions past t of the last piece, are the identity
  if (npad != D * nseg || U * L != N) dkgk::fill_identity(L * W, Cpm, home);
  HCK(hipMemsetAsync(pok, 1, npad * N, home));
  // deferred round 1 (BatchRound1): the fused pass over the very dealers whose coefficients wait
  const bool defer_r1 = ctx->r1_a && nseg == 2 && D == ctx->r1_D;
  for (int k = 0; k < nseg && !defer_r1; k++) {
    const uint32_t* ext = segs[k].round == 2 ? ctx->ext_E : ctx->ext_A;
    if (ext)  // generated on this device: group elements, as the reference's broadcasts carry them
      dkgk::place_position_major(ext, ctx->ext_stride, D, N, W, Cpm, home, nseg, k, L, npad);
    else  // K5 (groups.rs:78-81) into the position-major table
      dkgk::decode_position_major(segs[k].Ccomp, D, N, W, Cpm, pok, home, nseg, k, L, npad);
  }
  dkgk::dealer_ok(npad, N, pok, dok, home);
  // an extra mask produced by the overlapped decryption (full mode) is applied by each chunk's
  // checks once the shares are there; otherwise here
  const bool defer_masks = ctx->shares_pending;
  for (int k = 0; k < nseg; k++)
    if (segs[k].extra_ok && !defer_masks) dkgk::and_dealer_mask(D, nseg, k, segs[k].extra_ok, dok, home);
  // checks of dealers [d0, d1) on stream st
  auto checks = [&](size_t d0, size_t d1, hipStream_t st, size_t j0 = 0, size_t jn = 0) {
    if (d1 <= d0) return;
    wait_shares(ctx, st);
    if (defer_masks)  // dealers [d0, d1) start a column group (d0 = 64 g0): relative indexing
      for (int k = 0; k < nseg; k++)
        if (segs[k].extra_ok) dkgk::and_dealer_mask(d1 - d0, nseg, k, segs[k].extra_ok + d0, dok + d0 * nseg, st);
    const VerifySeg& g = segs[0];
    if (nseg == 2) {
      // split combs: every chunk parks its pairs' g*s at its own dealers' offset
      uint32_t* acc = ctx->check_mode == 1 ? buf<uint32_t>(ctx, "v.acc", PTB * D * n) + d0 * n * PT_WORDS_H : nullptr;
      dkgk::check_both(d1 - d0, n, d0, g.dealer_base, g.self_mod ? g.self_mod : n, g.s, g.sp, R,
                       ctx->tab_gw, ctx->tab_hw, dok, g.dec, segs[1].dec, st, sscale, j0, jn, acc);
    } else {
      dkgk::check(d1 - d0, n, g.dealer_base + d0, 0, g.self_mod ? g.self_mod : n, g.round, g.s + d0 * n * 8,
                  g.round == 2 ? g.sp + d0 * n * 8 : nullptr, R + d0 * n * PT_WORDS_H, ctx->tab_gw, ctx->tab_hw,
                  dok + d0, g.dec + d0 * n, st, sscale);
    }
  };
  // dealer groups [g0, g1) = columns [g0 * gw, g1 * gw)
  // Chunk streams pay when the binomial saturates the GPU (chunk c+1's triangle fills the CUs that
  // chunk c's launch tails leave idle), or when the stepping is long enough (W * L * n lane-steps)
  // that the chunks' phases drift apart and one chunk's recombination and checks run beside the
  // other's stepping.  A small ceremony or shard is latency-bound -- every binomial step is one
  // dependent NAF chain long whatever its width -- and two half-width pipelines only double its
  // launches.  Measured (tools/shard_time.py): chunks gain 1.2-2.4 ms on n=512 1- and 2-way (>= 6.7e7
  // lane-steps) and 0.3-0.8 ms on n=1024 1- to 4-way, and lose 0.9-2.5 ms on n=512 4-way and n=256
  // (<= 3.4e7) -- and 2 ms on the 8-way n=1024 shard (256 columns: two half-width stepping launches
  // of 128 workgroups each, 18.1 vs 20.2 ms, profiles/r02_shard_stepping_ab.txt), so a long stepping
  // needs at least 512 columns too.
  const bool saturating = (W / 64) * (L / 2) >= 4 * 1024;
  const bool long_stepping = (double)W * (double)L * (double)n >= 5e7 && npad >= 512;
  const size_t nsub = (saturating || long_stepping) ? std::min<size_t>(ctx->nsub, groups) : 1;
  // the binomial as per-wave Horner loops (k_binom_wave) for tables of many column groups
  const bool per_wave = ctx->binom_mode == 4 || ctx->binom_mode == 5 ||
                        (ctx->binom_mode == 0 && L > 1 && (double)npad / 64 * U >= DKG_BINOM_WAVE_GROUPS);
  ctx->last_binomial = per_wave ? 1 : 0;
  // the per-wave binomial's dedicated additions (with the stepping's formula setting): one redo flag
  // per (piece, 64-column group), zeroed before the chunks fork
  // (and of the per-step binomial's steps without lane pairs under DKG_BINOM_STEP_DED=2, redone per
  // wave; =1 marks the one guard word of with_binom_ded instead)
  uint32_t* bflags = nullptr;
  const bool wave_ded = per_wave && DKG_BINOM_WAVE_DED && ctx->binom_mode != 5 &&
                        !(ctx->binom_mode == 0 && DKG_BINOM_WAVE_PF);
  const bool step_ded = !per_wave && ((DKG_BINOM_STEP_DED == 1 && ctx->binom_step_ded && ctx->binom_any) ||
                                      DKG_BINOM_STEP_DED == 2);
  if (ctx->step_formula == 0 && (wave_ded || (step_ded && DKG_BINOM_STEP_DED == 2))) {
    bflags = buf<uint32_t>(ctx, "v.bflags", 4 * (W / 64));
    HCK(hipMemsetAsync(bflags, 0, 4 * (W / 64), home));
  }
  // the rerun guard's word (with_binom_ded): zeroed when the verification began (verify_rounds)
  uint32_t* bany = step_ded && DKG_BINOM_STEP_DED == 1 && ctx->step_formula == 0 ? ctx->binom_any : nullptr;
  // dead-position repack of an unsplit table (kernels.hip stepping_tail_phases): two scratch states
  const bool tails = ctx->step_mode != 3 && dkgk::stepping_tail_phases(L, n, U) > 1;
  uint32_t* tail_a = tails ? buf<uint32_t>(ctx, "v.tail_a", 4 * dkgk::stepping_tail_words(npad, L)) : nullptr;
  uint32_t* tail_b = tails ? buf<uint32_t>(ctx, "v.tail_b", 4 * dkgk::stepping_tail_words(npad, L)) : nullptr;
  auto chunk = [&](size_t g0, size_t g1, hipStream_t st, bool tm) {
    const size_t c0 = g0 * gw, w = (g1 - g0) * gw;
    if (defer_r1) {  // this chunk's dealers' commitments (committee.rs:151-159), into their columns
      const size_t d0 = g0 * 64, d1 = std::min(D, g1 * 64);
      dkgk::commit_position_major(d1 - d0, N, ctx->r1_a + d0 * N * 8, ctx->r1_b + d0 * N * 8, ctx->tab_gw,
                                  ctx->tab_hw, Cpm + c0, W, L, npad, ctx->r1_A0 + d0, D, st);
    }
    if (tm) HCK(hipEventRecord(ctx->pev[0], st));
    const uint32_t* e;
    if (per_wave) {
      e = dkgk::binomial_wave(w, W, L, Cpm + c0, e0 + c0, st, U, npad, Lr,
                              DKG_BINOM_WAVE_COLMAJOR ? eT + c0 * L : nullptr,
                              ctx->binom_mode == 5 || (ctx->binom_mode == 0 && DKG_BINOM_WAVE_PF), bflags, c0, D,
                              (unsigned)gw);
    } else {
      dkgk::binom_init(w, W, L, Cpm + c0, e0 + c0, st, U, npad);
      uint32_t *bin = e0 + c0, *bout = e1 + c0;
      for (size_t r = 1; r < L; r++) {
        // step r has (r + 1) waves per 64 columns and piece, over all chunks at once
        const double wps = (double)npad / 64 * U * (r + 1) / 1024;  // waves per SIMD, all chunks
        const bool ilp = use_ilp(ctx, wps < binom_ilp_waves());
        // lane pairs (k_binom_pair): by default the steps with under one wave per SIMD, mode 2
        // every step (1-, 2-, 4-, 8-way n=1024 shards 0.2-0.4 ms faster;
        // profiles/r03_binomial_pairs_ab.txt)
        const bool pair = ctx->binom_mode == 2 || ((ctx->binom_mode == 0 || ctx->binom_mode == 3) &&
                                                   wps < DKG_BINOM_PAIR_WAVES);
        if (pair)
          (ilp ? dkgk_ilp::binom_step_pair : dkgk::binom_step_pair)(r, w, W, L, Cpm + c0, bin, bout, st, U, npad,
                                                                    Lr);
        else
          (ilp ? dkgk_ilp::binom_step : dkgk::binom_step)(r, w, W, L, Cpm + c0, bin, bout, st, U, npad, Lr,
                                                          bany ? bany : bflags, c0, D, (unsigned)gw, bany != nullptr,
                                                          binom_nt(r, npad * U), !ilp && wps < binom_il_waves());
        std::swap(bin, bout);
      }
      e = bin;
      if (bflags && DKG_BINOM_STEP_DED == 2)
        dkgk::binomial_wave_redo(w, W, L, Cpm + c0, bin, st, U, npad, Lr, bflags, c0, D, (unsigned)gw);
    }
    if (tm) HCK(hipEventRecord(ctx->pev[1], st));
    if (!per_wave || !DKG_BINOM_WAVE_COLMAJOR)  // timed with the stepping
      dkgk::to_column_major(w, W, L, e, eT + c0 * L, U, npad, st);
    uint32_t* fl = sflags ? sflags + dkgk::stepping_flag_words(c0, U) : nullptr;
    if (fl) HCK(hipMemsetAsync(fl, 0, 4 * dkgk::stepping_flag_words(w, U), st));
    auto step = step_ilp ? dkgk_ilp::stepping : dkgk::stepping;
    if (!step(w, W, L, eT + c0 * L, n, R + c0 * n * PT_WORDS_H, sa ? sa + c0 * n * 40 : nullptr,
              sb ? sb + c0 * n * 40 : nullptr, st, U, npad, Lr, whole, fl, c0, D, (unsigned)gw,
              Rz ? Rz + c0 * n * 10 : nullptr, tail_a, tail_b))
      throw Fail{DKG_E_ARG};  // stepping flag words: an internal layout error, never silently dropped
    if (tm) HCK(hipEventRecord(ctx->pev[2], st));
    if (short_mult && Aff) {
      dkgk::affine_pieces(w, npad, U, n, R + c0 * n * PT_WORDS_H, Aff + c0 * n * AFFP_WORDS_H, st, Rz + c0 * n * 10);
      dkgk::combine_short_aff(w, npad, U, n, sdig, stop, Aff + c0 * n * AFFP_WORDS_H, R + c0 * n * PT_WORDS_H, st);
    } else if (short_mult) dkgk::combine_short(w, npad, U, n, sdig, stop, R + c0 * n * PT_WORDS_H, st);
    else dkgk::combine(w, npad, U, n, ydig, ytop, R + c0 * n * PT_WORDS_H, st);
    if (tm) HCK(hipEventRecord(ctx->pev[3], st));
    checks(g0 * 64, std::min(D, g1 * 64), st);
    if (tm) HCK(hipEventRecord(ctx->pev[4], st));
  };
  ctx->timed_tag.clear();
  if (nsub <= 1) {
    chunk(0, groups, home, timed);
    if (timed) ctx->timed_tag = tag;
  } else {
    HCK(hipEventRecord(ctx->fork, home));
    size_t g0 = 0;
    for (size_t c = 0; c < nsub; c++) {
      const size_t g1 = groups * (c + 1) / nsub;
      HCK(hipStreamWaitEvent(ctx->sub[c], ctx->fork, 0));
      chunk(g0, g1, ctx->sub[c], false);
      HCK(hipEventRecord(ctx->join[c], ctx->sub[c]));
      HCK(hipStreamWaitEvent(home, ctx->join[c], 0));
      g0 = g1;
    }
  }
  check_launch(ctx);
}

void verify_one(dkg_ctx* ctx, size_t n, size_t t, int round, size_t D, size_t dealer_base, const uint32_t* Ccomp,
                const uint32_t* s, const uint32_t* sp, uint8_t* dec, bool timed, const uint8_t* extra_ok = nullptr) {
  VerifySeg g{round, D, dealer_base, Ccomp, s, sp, dec, extra_ok};
  verify_device(ctx, n, t, &g, 1, timed, round == 2 ? "r2" : "r4");
}

// Rounds 2 and 4 of one set of dealers.  ctx->overlap (default): one fused pipeline over both
// commitment vectors -- the round-4 inputs (A_i, s_ij) are fixed in round 1 and only the SKIPPED
// mask applied afterwards depends on round 2, so every output is identical to protocol order.
// Otherwise round 2, then (after `between`, e.g. round 3) round 4, each timed when nsub == 1.
// `after2` (may be null) is recorded on ctx->stream once the round-2 decisions are complete.
// e_ok (may be null): per-dealer device mask, 0 = the dealer's round-1 data is missing (round 2:
// DKG_MISSING); a_ok (may be null): 0 = its phase-3 commitments are missing (round 4: accusation)
// (full mode), folded into the round-2 decisions like an undecodable commitment.
// host_between = false (fused rounds only): `between` only queues device work, so it follows the
// checks on the stream without a host round trip; the caller syncs and calls collect_phases.
template <typename F>
void verify_rounds_group(dkg_ctx* ctx, size_t n, size_t t, size_t D, size_t dealer_base, const uint32_t* Ecomp,
                         const uint32_t* Acomp, const uint32_t* s, const uint32_t* sp, uint8_t* dec2, uint8_t* dec4,
                         hipEvent_t after2, F&& between, const uint8_t* e_ok, const uint8_t* a_ok,
                         bool host_between) {
  if (ctx->overlap) {
    VerifySeg g[2] = {{2, D, dealer_base, Ecomp, s, sp, dec2, e_ok}, {4, D, dealer_base, Acomp, s, nullptr, dec4, a_ok}};
    verify_device(ctx, n, t, g, 2, true, "r24");
    if (after2) HCK(hipEventRecord(after2, ctx->stream));
    if (host_between) {
      sync(ctx);
      collect_phases(ctx);
    }
    between();
  } else {
    VerifySeg g2{2, D, dealer_base, Ecomp, s, sp, dec2, e_ok};
    verify_device(ctx, n, t, &g2, 1, true, "r2");
    if (after2) HCK(hipEventRecord(after2, ctx->stream));
    sync(ctx);
    collect_phases(ctx);
    between();
    verify_one(ctx, n, t, 4, D, dealer_base, Acomp, s, nullptr, dec4, true, a_ok);
    sync(ctx);
    collect_phases(ctx);
  }
}

// ---- committee verification by interpolation (ctx->verify_mode == 1; interp.hip) ----
// Inverse Vandermonde of the points 1..N mod l in Montgomery form, [x^k] L_j(x) * 2^256 (L_j the
// Lagrange basis polynomial of point j+1), as 11 limbs of 24 bits: W24[j][a][k] (k_interp).
// Cached per N.
const uint32_t* vinv_table(dkg_ctx* ctx, size_t N) {
  uint32_t* dev = buf<uint32_t>(ctx, "v.vinv", 4 * 11 * N * N);
  if (ctx->vinv_N == N) return dev;
  using dkgh::Zl;
  const Zl zero = dkgh::zl_from_u64(0);
  std::vector<Zl> M(N + 1, zero);  // M(x) = prod_m (x - (m+1)), ascending coefficients
  M[0] = dkgh::zl_from_u64(1);
  for (size_t m = 0; m < N; m++) {
    const Zl xm = dkgh::zl_from_u64(m + 1);
    for (size_t k = m + 1; k > 0; k--) M[k] = dkgh::zl_sub(M[k - 1], dkgh::zl_mul(xm, M[k]));
    M[0] = dkgh::zl_sub(zero, dkgh::zl_mul(xm, M[0]));
  }
  uint8_t r256[33] = {0};
  r256[32] = 1;
  const Zl R = dkgh::zl_from_bytes_wide(r256, 33);  // 2^256 mod l
  std::vector<uint32_t> host(11 * N * N);
  std::vector<Zl> q(N);
  for (size_t j = 0; j < N; j++) {
    const Zl xj = dkgh::zl_from_u64(j + 1);
    q[N - 1] = M[N];  // Q_j = M / (x - x_j), synthetic division
    for (size_t k = N - 1; k > 0; k--) q[k - 1] = dkgh::zl_add(M[k], dkgh::zl_mul(xj, q[k]));
    Zl den = zero;  // Q_j(x_j) = prod_{m != j} (x_j - x_m)
    for (size_t k = N; k-- > 0;) den = dkgh::zl_add(dkgh::zl_mul(den, xj), q[k]);
    const Zl scale = dkgh::zl_mul(dkgh::zl_inv(den), R);
    for (size_t k = 0; k < N; k++) {
      uint8_t b[33] = {0};
      dkgh::zl_to_bytes(b, dkgh::zl_mul(q[k], scale));
      for (size_t a = 0; a < 11; a++) {  // bits 24a .. 24a+23
        const size_t by = 3 * a;
        host[(j * 11 + a) * N + k] = (uint32_t)b[by] | (uint32_t)b[by + 1] << 8 | (uint32_t)b[by + 2] << 16;
      }
    }
  }
  h2d(ctx, dev, host.data(), 4 * host.size());
  ctx->vinv_N = N;
  return dev;
}

template <typename F>
void verify_rounds_interp(dkg_ctx* ctx, size_t n, size_t t, size_t D, size_t dealer_base, const uint32_t* Ecomp,
                          const uint32_t* Acomp, const uint32_t* s, const uint32_t* sp, uint8_t* dec2, uint8_t* dec4,
                          hipEvent_t after2, F&& between, const uint8_t* e_ok, const uint8_t* a_ok) {
  const size_t N = t + 1;
  hipStream_t st = ctx->stream;
  if (D) {
    HCK(hipEventRecord(ctx->pev[0], st));
    // the commitments as group elements [D][N]
    const uint32_t *Ee, *Ae;
    size_t cs;
    uint8_t* dokE = buf<uint8_t>(ctx, "i.dokE", D);
    uint8_t* dokA = buf<uint8_t>(ctx, "i.dokA", D);
    if (ctx->ext_E) {
      Ee = ctx->ext_E;
      Ae = ctx->ext_A;
      cs = ctx->ext_stride;
      HCK(hipMemsetAsync(dokE, 1, D, st));
      HCK(hipMemsetAsync(dokA, 1, D, st));
    } else {  // K5 (groups.rs:78-81): a row that does not decode is missing data
      uint32_t* ee = buf<uint32_t>(ctx, "i.Eext", PTB * D * N);
      uint32_t* ae = buf<uint32_t>(ctx, "i.Aext", PTB * D * N);
      uint8_t* pok = buf<uint8_t>(ctx, "i.pok", D * N);
      dkgk::decode_points(Ecomp, D * N, ee, D * N, pok, st);
      dkgk::dealer_ok(D, N, pok, dokE, st);
      dkgk::decode_points(Acomp, D * N, ae, D * N, pok, st);
      dkgk::dealer_ok(D, N, pok, dokA, st);
      Ee = ee;
      Ae = ae;
      cs = D * N;
    }
    dkgk::and_mask(D, e_ok, dokE, st);
    dkgk::and_mask(D, a_ok, dokA, st);
    const uint32_t* WT = vinv_table(ctx, N);
    uint32_t* Fa = buf<uint32_t>(ctx, "i.F", 32 * D * N);
    uint32_t* Fb = buf<uint32_t>(ctx, "i.Fp", 32 * D * N);
    dkgk::interp(D, N, n, WT, s, sp, Fa, Fb, st);  // F, F' through receivers 1..t+1
    HCK(hipEventRecord(ctx->pev[1], st));
    uint8_t* okE = buf<uint8_t>(ctx, "i.okE", D * N);
    uint8_t* okA = buf<uint8_t>(ctx, "i.okA", D * N);
    dkgk::coef_check(D, N, Fa, Fb, Ee, Ae, cs, ctx->tab_gw, ctx->tab_hw, okE, okA, st);
    uint8_t* cE = buf<uint8_t>(ctx, "i.cE", D);
    uint8_t* cA = buf<uint8_t>(ctx, "i.cA", D);
    dkgk::dealer_ok(D, N, okE, cE, st);
    dkgk::dealer_ok(D, N, okA, cA, st);
    HCK(hipEventRecord(ctx->pev[2], st));
    dkgk::interp_decide(D, n, N, dealer_base, n, s, sp, Fa, Fb, dokE, dokA, cE, cA, ctx->tab_gw, ctx->tab_hw, dec2,
                        dec4, st);
    HCK(hipEventRecord(ctx->pev[3], st));
    check_launch(ctx);
    // rows whose commitments are not g F + h F' (case B): difference tables, every P_i(j) in the group
    std::vector<uint8_t> h_dE(D), h_dA(D), h_cE(D), h_cA(D);
    d2h(ctx, h_dE.data(), dokE, D);
    d2h(ctx, h_dA.data(), dokA, D);
    d2h(ctx, h_cE.data(), cE, D);
    d2h(ctx, h_cA.data(), cA, D);
    sync(ctx);
    std::vector<size_t> rows;
    for (size_t d = 0; d < D; d++)
      if ((h_dE[d] && !h_cE[d]) || (h_dA[d] && !h_cA[d])) rows.push_back(d);
    if (!rows.empty()) {
      const size_t R = rows.size();
      uint32_t* rs = buf<uint32_t>(ctx, "i.rs", 32 * R * n);
      uint32_t* rsp = buf<uint32_t>(ctx, "i.rsp", 32 * R * n);
      uint8_t* r2 = buf<uint8_t>(ctx, "i.r2", R * n);
      uint8_t* r4 = buf<uint8_t>(ctx, "i.r4", R * n);
      uint32_t *rE = nullptr, *rA = nullptr, *rEx = nullptr, *rAx = nullptr;
      if (ctx->ext_E) {
        rEx = buf<uint32_t>(ctx, "i.rEx", PTB * R * N);
        rAx = buf<uint32_t>(ctx, "i.rAx", PTB * R * N);
      } else {
        rE = buf<uint32_t>(ctx, "i.rE", 32 * R * N);
        rA = buf<uint32_t>(ctx, "i.rA", 32 * R * N);
      }
      for (size_t r = 0; r < R; r++) {
        const size_t d = rows[r];
        HCK(hipMemcpyAsync(rs + 8 * r * n, s + 8 * d * n, 32 * n, hipMemcpyDeviceToDevice, st));
        HCK(hipMemcpyAsync(rsp + 8 * r * n, sp + 8 * d * n, 32 * n, hipMemcpyDeviceToDevice, st));
        if (rEx) {  // SoA planes: 40 words x N points per row
          HCK(hipMemcpy2DAsync(rEx + r * N, 4 * R * N, ctx->ext_E + d * N, 4 * ctx->ext_stride, 4 * N, PT_WORDS_H,
                               hipMemcpyDeviceToDevice, st));
          HCK(hipMemcpy2DAsync(rAx + r * N, 4 * R * N, ctx->ext_A + d * N, 4 * ctx->ext_stride, 4 * N, PT_WORDS_H,
                               hipMemcpyDeviceToDevice, st));
        } else {
          HCK(hipMemcpyAsync(rE + 8 * r * N, Ecomp + 8 * d * N, 32 * N, hipMemcpyDeviceToDevice, st));
          HCK(hipMemcpyAsync(rA + 8 * r * N, Acomp + 8 * d * N, 32 * N, hipMemcpyDeviceToDevice, st));
        }
      }
      // fused round-2/4 pipeline on the compact rows; dealer_base = n with modulus 2n + R marks no
      // pair as self (the diagonal is restored below)
      const uint32_t *sE = ctx->ext_E, *sA = ctx->ext_A;
      const size_t sstr = ctx->ext_stride;
      if (rEx) {
        ctx->ext_E = rEx;
        ctx->ext_A = rAx;
        ctx->ext_stride = R * N;
      }
      VerifySeg g[2] = {{2, R, n, rE, rs, rsp, r2, nullptr, 2 * n + R}, {4, R, n, rA, rs, nullptr, r4, nullptr, 2 * n + R}};
      const bool ov = ctx->overlap;
      ctx->overlap = true;
      verify_device(ctx, n, t, g, 2, false, "");
      ctx->overlap = ov;
      ctx->ext_E = sE;
      ctx->ext_A = sA;
      ctx->ext_stride = sstr;
      for (size_t r = 0; r < R; r++) {
        const size_t d = rows[r], jself = (d + dealer_base) % n;
        if (h_dE[d] && !h_cE[d]) {
          HCK(hipMemcpyAsync(dec2 + d * n, r2 + r * n, n, hipMemcpyDeviceToDevice, st));
          HCK(hipMemsetAsync(dec2 + d * n + jself, DKG_SELF, 1, st));
        }
        if (h_dA[d] && !h_cA[d]) {
          HCK(hipMemcpyAsync(dec4 + d * n, r4 + r * n, n, hipMemcpyDeviceToDevice, st));
          HCK(hipMemsetAsync(dec4 + d * n + jself, DKG_SELF, 1, st));
        }
      }
      check_launch(ctx);
    }
    HCK(hipEventRecord(ctx->pev[4], st));
    ctx->fallback_rows = rows.size();
  }
  if (after2) HCK(hipEventRecord(after2, st));
  sync(ctx);
  if (D) {
    const char* names[4] = {"interpolate", "coef_check", "decide", "fallback"};
    for (int i = 0; i < 4; i++) {
      float ms = 0;
      HCK(hipEventElapsedTime(&ms, ctx->pev[i], ctx->pev[i + 1]));
      ctx->phase_ms[std::string("interp.") + names[i]] = ms;
    }
  }
  between();
}

template <typename F>
void verify_rounds(dkg_ctx* ctx, size_t n, size_t t, size_t D, size_t dealer_base, const uint32_t* Ecomp,
                   const uint32_t* Acomp, const uint32_t* s, const uint32_t* sp, uint8_t* dec2, uint8_t* dec4,
                   hipEvent_t after2, F&& between, const uint8_t* e_ok = nullptr, const uint8_t* a_ok = nullptr,
                   bool host_between = true) {
  // dkg_ctx_stepping_redos reports THIS verification's stepping (none if it builds no tables)
  ctx->last_step_flags = nullptr;
  ctx->last_step_flag_words = 0;
  ctx->binom_any = nullptr;
  ctx->binom_any_host = nullptr;
  if (ctx->binom_step_ded && DKG_BINOM_STEP_DED == 1) {  // both rounds' binomials mark one word
    ctx->binom_any = buf<uint32_t>(ctx, "v.bany", 4);
    HCK(hipMemsetAsync(ctx->binom_any, 0, 4, ctx->stream));
  }
  if (ctx->verify_mode == 1)
    verify_rounds_interp(ctx, n, t, D, dealer_base, Ecomp, Acomp, s, sp, dec2, dec4, after2, between, e_ok, a_ok);
  else
    verify_rounds_group(ctx, n, t, D, dealer_base, Ecomp, Acomp, s, sp, dec2, dec4, after2, between, e_ok, a_ok,
                        host_between);
}

// Queues the copy of the rerun guard's word into pinned memory ahead of the caller's own sync, so
// that reading it costs no round trip of its own.
void binom_mark_copy(dkg_ctx* ctx) {
  if (!ctx->binom_any) return;
  uint32_t* h = hbuf<uint32_t>(ctx, "bany.h", 4);
  d2h(ctx, h, ctx->binom_any, 4);
  ctx->binom_any_host = h;
}

// After a sync: did the last verification's per-step binomial mark a group (a dedicated addition met
// Z = 0)?  Then its tables are not the complete formula's and the caller reruns the verification.
// (A caller that queued no copy pays a blocking read.)
bool binom_marked(dkg_ctx* ctx) {
  if (!ctx->binom_any) return false;
  uint32_t v = 0;
  if (ctx->binom_any_host)
    v = *ctx->binom_any_host;
  else
    HCK(hipMemcpy(&v, ctx->binom_any, 4, hipMemcpyDeviceToHost));
  return v != 0;
}

// Runs f() -- a verification and its outcomes, ending in a sync -- with the per-step binomial's
// dedicated additions allowed; when a group was marked, f() runs again with the complete formula.
template <typename F>
void with_binom_ded(dkg_ctx* ctx, F&& f) {
  struct Off {
    dkg_ctx* c;
    ~Off() { c->binom_step_ded = false; }
  } off{ctx};
  ctx->binom_step_ded = true;
  ctx->last_binom_rerun = 0;
  f();
  ctx->binom_step_ded = false;
  if (binom_marked(ctx)) {
    ctx->last_binom_rerun = 1;
    f();
  }
}

double ev_ms(dkg_ctx* ctx, int a, int b) {
  float ms = 0;
  HCK(hipEventElapsedTime(&ms, ctx->ev[a], ctx->ev[b]));
  return ms;
}

// Lagrange coefficients at zero (polynomial.rs:162-170 with x = 0) over the abscissae x = j + 1 of
// the parties j < n with in_set[j]: lambda_a = prod_{b != a} x_b / (x_b - x_a).  Over the full
// range 1..n the denominator is (-1)^(x_a - 1) (x_a - 1)! (n - x_a)!, so with U = {1..n}
//   lambda_a = P * prod_{e in U \ set} (x_e - x_a) * (-1)^j / ((j+1)! (n-1-j)!),  P = prod_set x_b,
// which costs O(n + |set| * |U \ set|) multiplications and one inversion (inverse factorials),
// instead of |set|^2 products and |set| inversions.  Zero for j outside the set.
std::vector<dkgh::Zl> lagrange_zero_coeffs(size_t n, const uint8_t* in_set) {
  using namespace dkgh;
  const Zl zero = zl_from_u64(0), one = zl_from_u64(1);
  std::vector<Zl> fact(n + 1), ifact(n + 1), lam(n, zero);
  fact[0] = one;
  for (size_t k = 1; k <= n; k++) fact[k] = zl_mul(fact[k - 1], zl_from_u64(k));
  ifact[n] = zl_inv(fact[n]);
  for (size_t k = n; k > 0; k--) ifact[k - 1] = zl_mul(ifact[k], zl_from_u64(k));
  Zl P = one;
  std::vector<size_t> outside;
  for (size_t j = 0; j < n; j++) {
    if (in_set[j]) P = zl_mul(P, zl_from_u64(j + 1));
    else outside.push_back(j);
  }
  for (size_t j = 0; j < n; j++) {
    if (!in_set[j]) continue;
    Zl v = zl_mul(P, zl_mul(ifact[j + 1], ifact[n - 1 - j]));
    for (size_t e : outside) v = zl_mul(v, zl_sub(zl_from_u64(e + 1), zl_from_u64(j + 1)));
    lam[j] = (j & 1) ? zl_sub(zero, v) : v;
  }
  return lam;
}

// sum_j lambda[j] * y[j] with y[j] the 32-byte scalar at ys + 32 * j (j < n, lambda[j] != 0)
dkgh::Zl lagrange_dot(const std::vector<dkgh::Zl>& lam, const uint8_t* ys, size_t n) {
  dkgh::Zl acc = dkgh::zl_from_u64(0);
  for (size_t j = 0; j < n; j++)
    if (!dkgh::zl_is_zero(lam[j])) acc = dkgh::zl_add(acc, dkgh::zl_mul(lam[j], dkgh::zl_from_bytes_wide(ys + 32 * j, 32)));
  return acc;
}

// The final parties of finalise: qualified and not reconstructable (committee.rs:733-739).
std::vector<uint8_t> final_parties(size_t n, const uint8_t* qualified, const uint8_t* recon) {
  std::vector<uint8_t> f(n);
  for (size_t j = 0; j < n; j++) f[j] = qualified[j] && !recon[j];
  return f;
}

// The final parties whose phase-5 disclosures reach the others: a party whose Phase1 or Phase3
// proceed failed (r2 / r4 error, committee.rs:340-347, 567-569) never reaches Phases<Phase4>::proceed
// and never broadcasts a BroadcastPhase5 (:684); it does not finalise either.  r2err / r4err may be
// null (no errors).
std::vector<uint8_t> disclosing_parties(size_t n, const uint8_t* qualified, const uint8_t* recon, const uint8_t* r2err,
                                        const uint8_t* r4err) {
  std::vector<uint8_t> f = final_parties(n, qualified, recon);
  for (size_t j = 0; j < n; j++) f[j] = f[j] && !(r2err && r2err[j]) && !(r4err && r4err[j]);
  return f;
}

// With reconstructed dealers, every finalising party holds its own share plus the other disclosing
// final parties' -- exactly the disclosing set S -- and fails with InsufficientSharesForRecovery when
// that is fewer than `threshold` = t points (:779-781): then no party has an mpk.
bool recovery_fails(const std::vector<uint8_t>& S, size_t t) {
  size_t c = 0;
  for (auto v : S) c += v != 0;
  return c < t;
}

// Secrets of the reconstructed dealers (rows `rows` of hs, share row r at hs + 32 * n * r) as the
// finalising parties recover them: a final party p interpolates dealer i's shares at its own index
// and at every other disclosing final party's (committee.rs:754-788), i.e. at exactly the disclosing
// set `fin` (disclosing_parties), so every finalising party computes this same value (with exactly t
// points a wrong one, as the reference does; the per-party view with missing disclosures is
// dkg_finalise_parties).  The dealer's share to itself is never used (it is not a final party), and
// its other shares all passed round 2.
std::vector<uint8_t> recon_secrets(size_t n, const std::vector<uint8_t>& fin, const uint8_t* hs,
                                   const std::vector<size_t>& rows) {
  const std::vector<dkgh::Zl> lam = lagrange_zero_coeffs(n, fin.data());
  std::vector<uint8_t> secrets(32 * rows.size());
  for (size_t r = 0; r < rows.size(); r++) dkgh::zl_to_bytes(&secrets[32 * r], lagrange_dot(lam, hs + 32 * n * rows[r], n));
  return secrets;
}

// Round-2 outcome of `groups` stacked ceremonies of n parties from the decision matrix
// dec2 [groups*n][n] on the device, as every party derives it (committee.rs:311-347, 370-398): a
// REJECT by receiver j is a complaint of j against dealer i, and a valid complaint disqualifies i for
// everyone; MISSING (no decodable broadcast) disqualifies without a complaint (:331-335); more than t
// complaints raise MisbehaviourHigherThreshold for j (:340-347); qmask (device [groups*n]) receives
// the qualified set.  Each round's outcome has a device half (kernels queued on ctx->stream, the
// per-dealer / per-receiver results left in `rej`, `cnt`, `r4d`) and a host half (applied to their
// copies after a sync), so that a caller queues both rounds' device halves and copies everything back
// in one round trip.  The single-GPU drivers, the batches and the sharded combine all decide through
// these four functions.
void round2_device(dkg_ctx* ctx, size_t groups, size_t n, const uint8_t* dec2, uint8_t* qmask, uint8_t* rej,
                   int32_t* cnt) {
  dkgk::decision_summary(groups, n, dec2, rej, cnt, ctx->stream);
  dkgk::mask_not_and(groups * n, rej, nullptr, qmask, ctx->stream);  // qualified = no rejecting row
}
// host half: `qualified` holds the copied rej flags on entry
void round2_host(size_t V, size_t t, uint8_t* qualified, const int32_t* complaints, uint8_t* r2err) {
  for (size_t i = 0; i < V; i++) {
    qualified[i] = !qualified[i];
    r2err[i] = complaints[i] > (int32_t)t;  // committee.rs:340-347
  }
}
// Round-4 outcome (committee.rs:515-522, 567-569, 660-670) from dec4 [groups*n][n] on the device and
// the round-2 qualified set (host `qualified`, device `qmask`): the rows of disqualified dealers
// become SKIPPED in place (:522); a qualified dealer some receiver rejects is reconstructed; receiver
// j's round-4 error (r4d / r4err, may be NULL) counts itself and the qualified dealers it accepted.
void round4_device(dkg_ctx* ctx, size_t groups, size_t n, size_t t, uint8_t* dec4, const uint8_t* qmask,
                   uint8_t* rej, uint8_t* r4d) {
  dkgk::decision_summary(groups, n, dec4, rej, nullptr, ctx->stream);
  if (r4d) dkgk::r4_error(groups, n, t, dec4, qmask, r4d, ctx->stream);
  dkgk::apply_skipped(groups, n, dec4, qmask, ctx->stream);
}
// host half: `recon` holds the copied rej flags on entry
void round4_host(size_t V, const uint8_t* qualified, uint8_t* recon) {
  for (size_t i = 0; i < V; i++) recon[i] = qualified[i] && recon[i];
}

// Rounds 2-5 on device-resident broadcast values (E, A compressed [n][N][8]; s, sp [n][n][8]).
// The outcomes stay on the device until the end -- one host round trip per ceremony, as the batches
// (batch_receivers): the round-2 outcome's device half gives the qualified mask for round 3, the
// round-4 half the reconstruction flags, and the master key is summed over the honest set (qualified,
// not reconstructed: committee.rs:726-805) speculatively; the host then only zeroes it (Phase4 failure,
// failed recovery) or, when a dealer is reconstructed, adds g * its recovered secret (a second trip).
void receivers_rounds_once(dkg_ctx* ctx, size_t n, size_t t, const uint32_t* Ecomp, const uint32_t* Acomp,
                           const uint32_t* s, const uint32_t* sp, dkg_ceremony_out* out, bool copy_big,
                           const uint8_t* e_ok, const uint8_t* a_ok) {
  const size_t N = t + 1;
  uint8_t* dec2 = buf<uint8_t>(ctx, "dec2", n * n);
  uint8_t* dec4 = buf<uint8_t>(ctx, "dec4", n * n);
  uint32_t* fs = buf<uint32_t>(ctx, "final_share", 32 * n);
  uint32_t* pubc = buf<uint32_t>(ctx, "pub_comp", 32 * n);
  uint8_t* qmask = buf<uint8_t>(ctx, "qmask", n);
  uint8_t* rej2 = buf<uint8_t>(ctx, "o.rej2", n);
  int32_t* cnt = buf<int32_t>(ctx, "o.cnt", 4 * n);
  // ---- rounds 2 and 4 (committee.rs:260-366, :508-580), fused or in protocol order (verify_rounds)
  auto round3 = [&] {
    wait_shares(ctx, ctx->stream);
    round2_device(ctx, 1, n, dec2, qmask, rej2, cnt);
    // ---- round 3 (committee.rs:433-476): final share s_j = sum_{i in Q} s_ij, public g s_j
    dkgk::sum_shares(n, n, s, qmask, fs, ctx->stream);
    // the public shares g s_j are an output only: computed on the side stream, off the path to
    // round 4 and finalise (joined before the outputs are read)
    uint32_t* pub = buf<uint32_t>(ctx, "pub_ext", PTB * n);
    HCK(hipEventRecord(ctx->side_fork, ctx->stream));
    HCK(hipStreamWaitEvent(ctx->side, ctx->side_fork, 0));
    dkgk::fixed_base(n, fs, ctx->tab_gw, pub, ctx->side);
    dkgk::encode_points(pub, n, n, pubc, ctx->side);
    HCK(hipEventRecord(ctx->pub_done, ctx->side));
    HCK(hipEventRecord(ctx->ev[3], ctx->stream));
  };
  verify_rounds(ctx, n, t, n, 0, Ecomp, Acomp, s, sp, dec2, dec4, ctx->ev[2], round3, e_ok, a_ok, false);
  wait_shares(ctx, ctx->stream);
  ctx->shares_pending = false;
  // round-4 outcome on the device: a qualified dealer some receiver rejects is reconstructed
  // (committee.rs:660-670); receiver j's round-4 error (:515-516, 567-569) counts itself and the
  // qualified dealers it accepted
  uint8_t* rej4 = buf<uint8_t>(ctx, "o.rej4", n);
  uint8_t* r4d = buf<uint8_t>(ctx, "o.r4err", n);
  round4_device(ctx, 1, n, t, dec4, qmask, rej4, r4d);
  HCK(hipEventRecord(ctx->ev[4], ctx->stream));
  // ---- finalise (committee.rs:726-805): mpk = sum_{i in Q \ recon} A_i0 (+ sum_{recon} g * L_i(0))
  uint32_t* A0 = buf<uint32_t>(ctx, "A0ext", PTB * n);
  if (ctx->ext_A) {
    dkgk::gather_points(ctx->ext_A, ctx->ext_stride, N, 0, n, A0, n, ctx->stream);
  } else {
    uint32_t* A0c = buf<uint32_t>(ctx, "A0c", 32 * n);
    HCK(hipMemcpy2DAsync(A0c, 32, Acomp, 32 * N, 32, n, hipMemcpyDeviceToDevice, ctx->stream));
    uint8_t* a0ok = buf<uint8_t>(ctx, "A0ok", n);
    dkgk::decode_points(A0c, n, A0, n, a0ok, ctx->stream);
  }
  uint8_t* hmask = buf<uint8_t>(ctx, "hmask", n);
  dkgk::mask_not_and(n, rej4, qmask, hmask, ctx->stream);  // the final parties: qualified, not accused
  uint32_t* mpk_ext = buf<uint32_t>(ctx, "mpk_ext", PTB);
  dkgk::sum_points(n, A0, n, hmask, mpk_ext, 1, 0, ctx->stream);
  uint32_t* mpk_c = buf<uint32_t>(ctx, "mpk_comp", 32);
  dkgk::encode_points(mpk_ext, 1, 1, mpk_c, ctx->stream);
  check_launch(ctx);
  uint8_t* h = hbuf<uint8_t>(ctx, "rr.out", 8 * n + 32);  // rej2 | rej4 | r4err | cnt | mpk
  d2h(ctx, h, rej2, n);
  d2h(ctx, h + n, rej4, n);
  d2h(ctx, h + 2 * n, r4d, n);
  d2h(ctx, h + 3 * n, cnt, 4 * n);
  d2h(ctx, h + 7 * n, mpk_c, 32);
  HCK(hipEventRecord(ctx->ev[5], ctx->stream));
  HCK(hipStreamWaitEvent(ctx->stream, ctx->pub_done, 0));  // public shares (round 3, side stream)
  if (copy_big) {
    if (out->dec2) d2h(ctx, out->dec2, dec2, n * n);
    if (out->dec4) d2h(ctx, out->dec4, dec4, n * n);  // SKIPPED rows applied (round4_device)
    if (out->final_share) d2h(ctx, out->final_share, fs, 32 * n);
    if (out->public_share) d2h(ctx, out->public_share, pubc, 32 * n);
  }
  binom_mark_copy(ctx);
  sync(ctx);
  collect_phases(ctx);
  std::vector<uint8_t> qualified(h, h + n), r2err(n), recon(h + n, h + 2 * n), r4e(h + 2 * n, h + 3 * n);
  std::vector<int32_t> complaints(n);
  memcpy(complaints.data(), h + 3 * n, 4 * n);
  round2_host(n, t, qualified.data(), complaints.data(), r2err.data());
  round4_host(n, qualified.data(), recon.data());
  const std::vector<uint8_t> disc = disclosing_parties(n, qualified.data(), recon.data(), r2err.data(), r4e.data());
  size_t nrecon = 0;
  int32_t nq = 0;
  for (size_t i = 0; i < n; i++) {
    nrecon += recon[i];
    nq += qualified[i];
  }
  // Phases<Phase4>::proceed fails for every party when qualified minus reconstructable <= t
  // (committee.rs:673-677): nobody finalises, so there is no master public key (mpk zeroed); with
  // reconstructions and fewer than t disclosing parties nobody recovers (:779-781): none either
  const bool phase4_error = nq - (int32_t)nrecon <= (int32_t)t;
  memset(out->mpk, 0, 32);
  if (!phase4_error && !(nrecon && recovery_fails(disc, t))) {
    if (nrecon) {  // + g * the reconstructed secrets, interpolated over the disclosing final parties
      std::vector<size_t> rows;
      std::vector<uint8_t> hs(32 * n * nrecon);
      for (size_t i = 0; i < n; i++)
        if (recon[i]) {
          d2h(ctx, &hs[32 * n * rows.size()], s + 8 * n * i, 32 * n);
          rows.push_back(rows.size());
        }
      sync(ctx);
      std::vector<uint8_t> secrets = recon_secrets(n, disc, hs.data(), rows);
      uint32_t* sec = buf<uint32_t>(ctx, "recon_sec", 32 * nrecon);
      h2d(ctx, sec, secrets.data(), secrets.size());
      uint32_t* gsec = buf<uint32_t>(ctx, "recon_ext", PTB * nrecon);
      uint32_t* extra = buf<uint32_t>(ctx, "recon_sum", PTB);
      dkgk::fixed_base(nrecon, sec, ctx->tab_gw, gsec, ctx->stream);
      dkgk::sum_points(nrecon, gsec, nrecon, nullptr, extra, 1, 0, ctx->stream);
      dkgk::add_points(1, mpk_ext, extra, 1, mpk_ext, ctx->stream);
      dkgk::encode_points(mpk_ext, 1, 1, mpk_c, ctx->stream);
      check_launch(ctx);
      d2h(ctx, h + 7 * n, mpk_c, 32);
      sync(ctx);
    }
    memcpy(out->mpk, h + 7 * n, 32);
  }
  // ---- outputs
  if (out->qualified) memcpy(out->qualified, qualified.data(), n);
  if (out->r2_error) memcpy(out->r2_error, r2err.data(), n);
  if (out->r4_error) memcpy(out->r4_error, r4e.data(), n);
  if (out->complaints2) memcpy(out->complaints2, complaints.data(), 4 * n);
  if (out->reconstruct) memcpy(out->reconstruct, recon.data(), n);
  out->n_qualified = nq;
  out->phase4_error = phase4_error;  // committee.rs:673-677
}

// receivers_rounds_once with the per-step binomial's dedicated additions, rerun with the complete
// formula when they marked a group (with_binom_ded)
void receivers_rounds(dkg_ctx* ctx, size_t n, size_t t, const uint32_t* Ecomp, const uint32_t* Acomp,
                      const uint32_t* s, const uint32_t* sp, dkg_ceremony_out* out, bool copy_big,
                      const uint8_t* e_ok = nullptr, const uint8_t* a_ok = nullptr) {
  with_binom_ded(ctx, [&] { receivers_rounds_once(ctx, n, t, Ecomp, Acomp, s, sp, out, copy_big, e_ok, a_ok); });
}

// Round 1 for D dealers on device: a, b canonical [D][N][8] -> Ecomp, Acomp [D][N][8], s, sp [D][n][8].
// Round 1 on device.  encode = false: the commitments stay group elements (Ecomp / Acomp are not
// written; the caller verifies through an ExtScope, as the reference's in-memory broadcasts).
// overlap_shares: the share evaluation runs on ctx->side (lowest priority) beside what follows on
// ctx->stream -- the verification's first binomial steps, which occupy few CUs -- and the
// verification's checks and round 3 wait for it (ctx->shares_pending, wait_shares).
void round1_device(dkg_ctx* ctx, size_t D, size_t n, size_t t, const uint32_t* a, const uint32_t* b,
                   uint32_t* Ecomp, uint32_t* Acomp, uint32_t* s, uint32_t* sp, bool encode = true,
                   bool overlap_shares = false) {
  const size_t N = t + 1;
  uint32_t* Aext = buf<uint32_t>(ctx, "Aext", PTB * D * N);
  uint32_t* Eext = buf<uint32_t>(ctx, "Eext", PTB * D * N);
  if (overlap_shares) {  // the side stream starts where ctx->stream is (a, b written)
    HCK(hipEventRecord(ctx->side_fork, ctx->stream));
    HCK(hipStreamWaitEvent(ctx->side, ctx->side_fork, 0));
  }
  dkgk::commit(D * N, a, b, ctx->tab_gw, ctx->tab_hw, Aext, Eext, ctx->stream);  // K2 (committee.rs:151-159)
  if (encode) {
    dkgk::encode_points(Eext, D * N, D * N, Ecomp, ctx->stream);                  // broadcast encodings
    dkgk::encode_points(Aext, D * N, D * N, Acomp, ctx->stream);
  }
  if (overlap_shares) {
    dkgk::share_eval(D, n, N, a, b, s, sp, ctx->side);                             // K1 (:164-167)
    HCK(hipEventRecord(ctx->shares_done, ctx->side));
    ctx->shares_pending = true;
  } else {
    dkgk::share_eval(D, n, N, a, b, s, sp, ctx->stream);
  }
  check_launch(ctx);
}


// Shares evaluated on the side stream (round1_device with overlap_shares) that a call leaves pending
// when it throws: the home stream -- every later call's -- waits for them, then the flag is dropped.
struct SharesScope {
  dkg_ctx* ctx;
  explicit SharesScope(dkg_ctx* c) : ctx(c) {}
  ~SharesScope() {
    if (ctx->shares_pending) (void)hipStreamWaitEvent(ctx->stream, ctx->shares_done, 0);
    ctx->shares_pending = false;
  }
};

// Verify what round1_device just generated from its extended-form commitments (no encode/decode
// round trip); restores the ctx on exit.
struct ExtScope {
  dkg_ctx* ctx;
  ExtScope(dkg_ctx* c, size_t D, size_t N) : ctx(c) {
    ctx->ext_E = buf<uint32_t>(ctx, "Eext", PTB * D * N);
    ctx->ext_A = buf<uint32_t>(ctx, "Aext", PTB * D * N);
    ctx->ext_stride = D * N;
  }
  ~ExtScope() {
    ctx->ext_E = ctx->ext_A = nullptr;
    ctx->ext_stride = 0;
  }
};

// Round 1 of a batch with the commitments deferred into the verification's chunks (r1_a above):
// the fused group pass (verify_mode 0, rounds 2 and 4 fused) computes each chunk's dealers'
// commitments on the chunk's own stream, so the second chunk's commitments (half of config 5's
// round 1) run beside the first chunk's binomial and stepping; the shares are evaluated on the
// side stream beside both.  Other schedules get the whole round 1 first (round1_device).
struct BatchRound1 {
  dkg_ctx* ctx;
  BatchRound1(dkg_ctx* c, size_t D, size_t n, size_t t, const uint32_t* a, const uint32_t* b, uint32_t* s,
              uint32_t* sp)
      : ctx(c) {
    const size_t N = t + 1;
    if (deferred()) {
      HCK(hipEventRecord(ctx->side_fork, ctx->stream));
      HCK(hipStreamWaitEvent(ctx->side, ctx->side_fork, 0));
      dkgk::share_eval(D, n, N, a, b, s, sp, ctx->side);  // K1 (committee.rs:164-167)
      HCK(hipEventRecord(ctx->shares_done, ctx->side));
      ctx->shares_pending = true;
      ctx->r1_a = a;
      ctx->r1_b = b;
      ctx->r1_D = D;
      ctx->r1_A0 = buf<uint32_t>(ctx, "r1_A0", PTB * D);
    } else {
      round1_device(ctx, D, n, t, a, b, nullptr, nullptr, s, sp, false);
    }
    check_launch(ctx);
  }
  bool deferred() const { return ctx->overlap && ctx->verify_mode == 0; }
  ~BatchRound1() {
    // after an exception the shares kernel may still be writing s / sp on the side stream: make the
    // home stream (every later call's) wait for it before the state that tracks it is dropped
    if (ctx->shares_pending) (void)hipStreamWaitEvent(ctx->stream, ctx->shares_done, 0);
    ctx->r1_a = ctx->r1_b = nullptr;
    ctx->r1_D = 0;
    ctx->r1_A0 = nullptr;
    ctx->shares_pending = false;
  }
};

// ---- batches of independent ceremonies (BASELINE config 5: many small key ceremonies)
// B ceremonies of n parties are stacked dealer-wise: dealer c*n + i is party i of ceremony c, and
// its share row addresses that ceremony's n receivers.  The verification pipeline is the same as
// for one ceremony (2*B*n virtual dealers in the fused pipeline); the per-ceremony combine steps
// (qualification, complaints, round-3 sums, mpk) are grouped kernels.  Every output equals what B
// separate ceremonies produce.
void batch_receivers(dkg_ctx* ctx, size_t B, size_t n, size_t t, const uint32_t* Ecomp, const uint32_t* Acomp,
                     const uint32_t* s, const uint32_t* sp, dkg_batch_out* out) {
  const size_t N = t + 1, V = B * n;
  uint8_t* dec2 = buf<uint8_t>(ctx, "b.dec2", V * n);
  uint8_t* dec4 = buf<uint8_t>(ctx, "b.dec4", V * n);
  uint8_t* qmask = buf<uint8_t>(ctx, "b.qmask", V);
  uint8_t* rej2 = buf<uint8_t>(ctx, "b.rej2", V);
  uint8_t* rej4 = buf<uint8_t>(ctx, "b.rej4", V);
  uint8_t* r4d = buf<uint8_t>(ctx, "b.r4err", V);
  uint8_t* hmask = buf<uint8_t>(ctx, "b.hmask", V);
  int32_t* cnt = buf<int32_t>(ctx, "b.cnt", 4 * V);
  uint32_t* fs = buf<uint32_t>(ctx, "b.final", 32 * V);
  uint32_t* pub = buf<uint32_t>(ctx, "b.pub_ext", PTB * V);
  uint32_t* pubc = buf<uint32_t>(ctx, "b.pub_comp", 32 * V);
  std::vector<uint8_t> qualified(V), r2err(V), recon(V, 0), honest(V), r4e(V), h_rej4(V);
  std::vector<int32_t> complaints(V);
  // The outcomes stay on the device until the end (one host round trip per batch): the rows that
  // reject or miss disqualify (committee.rs:311-316, 331-335, 370-398), round 3 sums the qualified
  // dealers' shares (:433-476), round 4's rejections reconstruct qualified dealers (:660-670) and the
  // honest set -- qualified, not reconstructed -- sums the master key (:726-805).
  auto round3 = [&] {
    round2_device(ctx, B, n, dec2, qmask, rej2, cnt);
    wait_shares(ctx, ctx->stream);  // shares evaluated on the side stream (BatchRound1)
    dkgk::sum_shares(n, n, s, qmask, fs, ctx->stream, B);
    dkgk::fixed_base(V, fs, ctx->tab_gw, pub, ctx->stream);
    dkgk::encode_points(pub, V, V, pubc, ctx->stream);
    HCK(hipEventRecord(ctx->ev[3], ctx->stream));
  };
  verify_rounds(ctx, n, t, V, 0, Ecomp, Acomp, s, sp, dec2, dec4, ctx->ev[2], round3, nullptr, nullptr, false);
  // round 4 (committee.rs:515-522, 567-569, 660-670): rows of disqualified dealers SKIPPED
  round4_device(ctx, B, n, t, dec4, qmask, rej4, r4d);
  dkgk::mask_not_and(V, rej4, qmask, hmask, ctx->stream);
  HCK(hipEventRecord(ctx->ev[4], ctx->stream));
  // finalise (committee.rs:726-805): mpk_c = sum of the honest A_i0 (+ g * reconstructed secrets)
  uint32_t* A0 = buf<uint32_t>(ctx, "b.A0ext", PTB * V);
  if (ctx->r1_A0) {  // written by the deferred commitments (k_commit_pm), [40][V]
    HCK(hipMemcpyAsync(A0, ctx->r1_A0, PTB * V, hipMemcpyDeviceToDevice, ctx->stream));
  } else if (ctx->ext_A) {
    dkgk::gather_points(ctx->ext_A, ctx->ext_stride, N, 0, V, A0, V, ctx->stream);
  } else {
    uint32_t* A0c = buf<uint32_t>(ctx, "b.A0c", 32 * V);
    HCK(hipMemcpy2DAsync(A0c, 32, Acomp, 32 * N, 32, V, hipMemcpyDeviceToDevice, ctx->stream));
    uint8_t* a0ok = buf<uint8_t>(ctx, "b.A0ok", V);
    dkgk::decode_points(A0c, V, A0, V, a0ok, ctx->stream);
  }
  uint32_t* mpk_ext = buf<uint32_t>(ctx, "b.mpk_ext", PTB * B);
  dkgk::sum_points(n, A0, V, hmask, mpk_ext, B, 0, ctx->stream, B);
  uint32_t* mpk_c = buf<uint32_t>(ctx, "b.mpk_comp", 32 * B);
  dkgk::encode_points(mpk_ext, B, B, mpk_c, ctx->stream);
  check_launch(ctx);
  // every outcome through pinned staging, one sync: copies into the caller's pageable buffers were
  // staged by the runtime on this thread, 1-27 ms of host time per 10,000-ceremony batch beyond the
  // device span (tools/batch_gap.py)
  struct Out {
    void* host;
    const void* dev;
    size_t bytes;
    const char* name;
  };
  const Out outs[] = {{qualified.data(), rej2, V, "hb.rej2"},  // inverted below
                      {complaints.data(), cnt, 4 * V, "hb.cnt"},
                      {h_rej4.data(), rej4, V, "hb.rej4"},
                      {r4e.data(), r4d, V, "hb.r4err"},
                      {out->mpk, mpk_c, 32 * B, "hb.mpk"},
                      {out->final_share, fs, 32 * V, "hb.final"},
                      {out->public_share, pubc, 32 * V, "hb.pub"},
                      {out->dec2, dec2, V * n, "hb.dec2"},
                      {out->dec4, dec4, V * n, "hb.dec4"}};  // SKIPPED rows applied
  void* staged[sizeof(outs) / sizeof(outs[0])] = {};
  for (size_t k = 0; k < sizeof(outs) / sizeof(outs[0]); k++)
    if (outs[k].host) {
      staged[k] = hbuf(ctx, outs[k].name, outs[k].bytes);
      d2h(ctx, staged[k], outs[k].dev, outs[k].bytes);
    }
  HCK(hipEventRecord(ctx->ev[5], ctx->stream));
  sync(ctx);
  for (size_t k = 0; k < sizeof(outs) / sizeof(outs[0]); k++)
    if (staged[k]) memcpy(outs[k].host, staged[k], outs[k].bytes);
  collect_phases(ctx);
  round2_host(V, t, qualified.data(), complaints.data(), r2err.data());
  recon = h_rej4;
  round4_host(V, qualified.data(), recon.data());
  for (size_t i = 0; i < V; i++) honest[i] = qualified[i] && !recon[i];
  std::vector<size_t> recon_cer, nompk;
  std::vector<uint8_t> p4err(B, 0);
  for (size_t c = 0; c < B; c++) {
    bool any = false;
    int32_t h = 0;
    for (size_t i = c * n; i < (c + 1) * n; i++) {
      any |= recon[i] != 0;
      h += honest[i];
    }
    p4err[c] = h <= (int32_t)t;  // committee.rs:673-677: nobody finalises, no mpk
    if (any && !p4err[c]) {
      // InsufficientSharesForRecovery for every finalising party: no mpk either (recovery_fails)
      if (recovery_fails(disclosing_parties(n, &qualified[c * n], &recon[c * n], &r2err[c * n], &r4e[c * n]), t))
        nompk.push_back(c);
      else
        recon_cer.push_back(c);
    }
  }
  if (!recon_cer.empty()) {  // ceremonies with round-4 accusations: + g * the reconstructed secrets
    uint32_t* extra = buf<uint32_t>(ctx, "b.mpk_extra", PTB * B);
    std::vector<uint8_t> hs(32 * n * n);
    for (size_t c : recon_cer) {
      d2h(ctx, hs.data(), s + c * n * n * 8, 32 * n * n);
      sync(ctx);
      std::vector<size_t> rows;
      for (size_t i = 0; i < n; i++)
        if (recon[c * n + i]) rows.push_back(i);
      std::vector<uint8_t> secrets = recon_secrets(
          n, disclosing_parties(n, &qualified[c * n], &recon[c * n], &r2err[c * n], &r4e[c * n]), hs.data(), rows);
      const size_t nr = secrets.size() / 32;
      uint32_t* sec = buf<uint32_t>(ctx, "b.recon_sec", 32 * nr);
      h2d(ctx, sec, secrets.data(), secrets.size());
      uint32_t* gsec = buf<uint32_t>(ctx, "b.recon_ext", PTB * nr);
      dkgk::fixed_base(nr, sec, ctx->tab_gw, gsec, ctx->stream);
      dkgk::sum_points(nr, gsec, nr, nullptr, extra, B, c, ctx->stream);
      dkgk::add_points(1, mpk_ext + c, extra + c, B, mpk_ext + c, ctx->stream);
      sync(ctx);  // sec / gsec are reused by the next ceremony
    }
    dkgk::encode_points(mpk_ext, B, B, mpk_c, ctx->stream);
    check_launch(ctx);
    if (out->mpk) d2h(ctx, out->mpk, mpk_c, 32 * B);
    sync(ctx);
  }
  if (out->r4_error) memcpy(out->r4_error, r4e.data(), V);
  if (out->qualified) memcpy(out->qualified, qualified.data(), V);
  if (out->r2_error) memcpy(out->r2_error, r2err.data(), V);
  if (out->complaints2) memcpy(out->complaints2, complaints.data(), 4 * V);
  if (out->reconstruct) memcpy(out->reconstruct, recon.data(), V);
  if (out->phase4_error) memcpy(out->phase4_error, p4err.data(), B);  // committee.rs:673-677
  if (out->mpk) {
    for (size_t c = 0; c < B; c++)
      if (p4err[c]) memset(out->mpk + 32 * c, 0, 32);  // no party finalises: no master key
    for (size_t c : nompk) memset(out->mpk + 32 * c, 0, 32);  // no party recovers the secrets
  }
  if (out->n_qualified)
    for (size_t c = 0; c < B; c++) {
      int32_t q = 0;
      for (size_t i = c * n; i < (c + 1) * n; i++) q += qualified[i];
      out->n_qualified[c] = q;
    }
}

void batch_times(dkg_ctx* ctx, dkg_batch_out* out, bool round1) {
  out->ms_round1 = round1 ? ev_ms(ctx, 0, 1) : 0.0;
  out->ms_checks = ev_ms(ctx, 1, 2);
  out->ms_round3 = ev_ms(ctx, 2, 3);
  out->ms_finalise = ev_ms(ctx, 3, 5);
  out->ms_total = ev_ms(ctx, 0, 5);
}

// ---- full (encrypted-share) mode: hybrid.hip (elgamal.rs:134-193, committee.rs:164-172, 282-286)
// Items (dealer i, recipient q, w) at (i * n + q) * 2 + w: w = 0 the randomness s', w = 1 the share s.
// pk_host (optional): the same keys on the host.  Member keys outlive a ceremony (procedure_keys.rs),
// so their decoded points and comb tables are kept in the arena and rebuilt only when the keys
// differ from the last build's (compared byte for byte).
void encrypt_device(dkg_ctx* ctx, size_t D, size_t n, const uint32_t* pkc, const uint32_t* s, const uint32_t* sp,
                    const uint32_t* r, uint32_t* e1, uint32_t* ct, hipStream_t st = nullptr,
                    const uint8_t* pk_host = nullptr) {
  const size_t items = 2 * D * n;
  if (!st) st = ctx->stream;
  uint32_t* pk_ext = buf<uint32_t>(ctx, "hy.pk_ext", PTB * n);
  uint8_t* pk_ok = buf<uint8_t>(ctx, "hy.pk_ok", n);
  uint32_t* tabs = buf<uint32_t>(ctx, "hy.tabs", 4 * dkgk::key_comb_words() * n);
  const bool cached = pk_host && ctx->key_tabs_pk.size() == 32 * n &&
                      memcmp(ctx->key_tabs_pk.data(), pk_host, 32 * n) == 0;
  if (!cached) {
    ctx->key_tabs_pk.clear();  // invalid until this build is queued
    dkgk::decode_points(pkc, n, pk_ext, n, pk_ok, st);
    dkgk::build_key_combs(pk_ext, n, 0, tabs, st, n);  // one comb per recipient key: r * pk_q is fixed-base
    if (pk_host) ctx->key_tabs_pk.assign(pk_host, pk_host + 32 * n);
  }
  uint32_t* R = buf<uint32_t>(ctx, "hy.R", PTB * items);
  uint32_t* K = buf<uint32_t>(ctx, "hy.K", PTB * items);
  uint32_t* Kc = buf<uint32_t>(ctx, "hy.Kc", 32 * items);
  // phase events (serialised runs, nsub == 1): the bench's per-kernel roofline of full mode
  const bool tm = ctx->nsub == 1;
  if (tm) HCK(hipEventRecord(ctx->hev[0], st));
  dkgk::enc_mul(D, n, r, ctx->tab_gw, tabs, R, K, st);
  if (tm) HCK(hipEventRecord(ctx->hev[1], st));
  dkgk::encode_points(R, items, items, e1, st);
  dkgk::encode_points(K, items, items, Kc, st);
  if (tm) HCK(hipEventRecord(ctx->hev[2], st));
  dkgk::sym_xor(D, n, Kc, false, ct, const_cast<uint32_t*>(s), const_cast<uint32_t*>(sp), st);
  if (tm) HCK(hipEventRecord(ctx->hev[3], st));
  if (tm) ctx->hy_timed |= 1;
  check_launch(ctx);
}

// Receivers' side: item_ok[item] = e1 decodes; dealer_ok_out[i] = all of dealer i's items decode (a
// broadcast that does not deserialize is missing data, committee.rs:331-335).
void decrypt_device(dkg_ctx* ctx, size_t D, size_t n, const uint32_t* sk, const uint32_t* e1, const uint32_t* ct,
                    uint32_t* s, uint32_t* sp, uint8_t* item_ok, uint8_t* dealer_ok_out, hipStream_t st = nullptr) {
  const size_t items = 2 * D * n;
  if (!st) st = ctx->stream;
  uint32_t* R = buf<uint32_t>(ctx, "hy.R", PTB * items);
  uint32_t* K = buf<uint32_t>(ctx, "hy.K", PTB * items);
  uint32_t* Kc = buf<uint32_t>(ctx, "hy.Kc", 32 * items);
  const bool tm = ctx->nsub == 1;
  if (tm) HCK(hipEventRecord(ctx->hev[4], st));
  dkgk::decode_points(e1, items, R, items, item_ok, st);
  if (tm) HCK(hipEventRecord(ctx->hev[5], st));
  const size_t tw = dkgk::dec_mul_table_words(D, n);
  dkgk::dec_mul(D, n, sk, R, K, st, tw ? buf<uint32_t>(ctx, "hy.dec_tab", 4 * tw) : nullptr);
  if (tm) HCK(hipEventRecord(ctx->hev[6], st));
  dkgk::encode_points(K, items, items, Kc, st);
  if (tm) HCK(hipEventRecord(ctx->hev[7], st));
  dkgk::sym_xor(D, n, Kc, true, const_cast<uint32_t*>(ct), s, sp, st);
  if (tm) HCK(hipEventRecord(ctx->hev[8], st));
  if (tm) ctx->hy_timed |= 2;
  if (dealer_ok_out) dkgk::dealer_ok(D, 2 * n, item_ok, dealer_ok_out, st);
  check_launch(ctx);
}

// After a sync: the full-mode kernels' device times of the last serialised encrypt + decrypt
// (dkg_ctx_phase_ms "full.enc_mul", "full.enc_encode", "full.enc_sym", "full.dec_decode",
// "full.dec_mul", "full.dec_encode", "full.dec_sym").
// Every full.* entry of an earlier ceremony is dropped first: a phase this ceremony did not time
// (chunk streams, or a verify-only ceremony without encryption) reads -1.
void collect_hybrid_phases(dkg_ctx* ctx) {
  const char* names[8] = {"enc_mul", "enc_encode", "enc_sym", "", "dec_decode", "dec_mul", "dec_encode", "dec_sym"};
  for (const char* nm : names)
    if (nm[0]) ctx->phase_ms.erase(std::string("full.") + nm);
  const int timed = ctx->hy_timed;
  ctx->hy_timed = 0;
  for (int i = 0; i < 8; i++) {
    if (!names[i][0] || !(timed & (i < 4 ? 1 : 2))) continue;
    float ms = 0;
    HCK(hipEventElapsedTime(&ms, ctx->hev[i], ctx->hev[i + 1]));
    ctx->phase_ms[std::string("full.") + names[i]] = ms;
  }
}

// ---- complaint proofs (dl_equality/zkp.rs, broadcast.rs:50-135, 181-283)
// Cold path (one proof per complaint): the group work goes to the GPU as batched MSMs (k_msm), the
// Fiat-Shamir hashes, ChaCha20 and scalar arithmetic run on the host.
// B MSMs of N terms: scalars / points host [B][N][32] -> out [B][32]; ok[b] = every point decodes.
void msm_host(dkg_ctx* ctx, size_t B, size_t N, const uint8_t* scalars, const uint8_t* points, uint8_t* out,
              std::vector<uint8_t>& ok) {
  ok.assign(B, 1);
  if (!B) return;
  uint32_t* sc = upload_scalars(ctx, "cp_sc", scalars, B * N);
  uint32_t* pc = buf<uint32_t>(ctx, "cp_pc", 32 * B * N);
  uint32_t* pe = buf<uint32_t>(ctx, "cp_pe", PTB * B * N);
  uint8_t* pok = buf<uint8_t>(ctx, "cp_ok", B * N);
  h2d(ctx, pc, points, 32 * B * N);
  dkgk::decode_points(pc, B * N, pe, B * N, pok, ctx->stream);
  uint32_t* oe = buf<uint32_t>(ctx, "cp_oe", PTB * B);
  uint32_t* oc = buf<uint32_t>(ctx, "cp_oc", 32 * B);
  uint32_t* mt = buf<uint32_t>(ctx, "msm_tab", 4 * 15 * PT_WORDS_H * B * N);
  dkgk::msm_batch(B, N, sc, pe, B * N, mt, oe, ctx->stream);
  dkgk::encode_points(oe, B, B, oc, ctx->stream);
  check_launch(ctx);
  std::vector<uint8_t> okh(B * N);
  d2h(ctx, okh.data(), pok, B * N);
  d2h(ctx, out, oc, 32 * B);
  sync(ctx);
  for (size_t b = 0; b < B; b++)
    for (size_t k = 0; k < N; k++) ok[b] &= okh[b * N + k];
}

dkgh::Zl zl32(const uint8_t* p) { return dkgh::zl_from_bytes_wide(p, 32); }
void put32(std::vector<uint8_t>& v, const uint8_t* p) { v.insert(v.end(), p, p + 32); }
void putzl(std::vector<uint8_t>& v, const dkgh::Zl& z) {
  uint8_t b[32];
  dkgh::zl_to_bytes(b, z);
  put32(v, b);
}

// Scalar::hash_from_bytes::<Blake2b> (groups.rs:50-52) of ChallengeContext b1||b2||p1||p2||a1||a2
// (challenge_context.rs:14-41)
dkgh::Zl dleq_challenge(const uint8_t* b1, const uint8_t* b2, const uint8_t* p1, const uint8_t* p2, const uint8_t* a1,
                        const uint8_t* a2) {
  uint8_t buf_[192], h[64];
  const uint8_t* parts[6] = {b1, b2, p1, p2, a1, a2};
  for (int i = 0; i < 6; i++) memcpy(buf_ + 32 * i, parts[i], 32);
  dkgh::blake2b(h, 64, buf_, 192);
  return dkgh::zl_from_bytes_wide(h, 64);
}

// SymmetricKey::process + Scalar::from_bytes (from_bits, reduced) of a 32-byte ciphertext
dkgh::Zl sym_scalar(const uint8_t K[32], const uint8_t ct[32]) {
  uint8_t h[64], m[32];
  dkgh::blake2b(h, 64, K, 32);
  dkgh::chacha20_ietf_xor(m, ct, 32, h, h + 32);
  m[31] &= 0x7f;
  return zl32(m);
}

std::vector<uint8_t> index_powers(uint32_t j, size_t N) {  // from_u64(j).exp_iter().take(N)
  std::vector<uint8_t> out;
  dkgh::Zl x = dkgh::zl_from_u64(j), p = dkgh::zl_from_u64(1);
  for (size_t k = 0; k < N; k++) {
    putzl(out, p);
    p = dkgh::zl_mul(p, x);
  }
  return out;
}

int need_env(dkg_ctx* ctx) {
  if (!ctx->have_h) {
    ctx->err = "dkg_env_init has not been called (commitment key unknown)";
    return DKG_E_ARG;
  }
  return DKG_OK;
}

}  // namespace

// dkg_ctx_clock_probe: a dependent integer chain per lane between two reads of each clock; lane 0
// of every wave writes (shader cycles, constant-clock ticks) with vector stores.
__global__ __launch_bounds__(256) void k_clock_probe(unsigned iters, unsigned long long* out) {
  uint32_t x = threadIdx.x * 2654435761u + blockIdx.x;
  const unsigned long long c0 = clock64(), r0 = wall_clock64();
  for (unsigned i = 0; i < iters; i++) x = x * 1664525u + 1013904223u;
  asm volatile("" : "+v"(x));
  const unsigned long long c1 = clock64(), r1 = wall_clock64();
  const size_t w = (size_t)blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
  if ((threadIdx.x & 63) == 0) {
    out[2 * w] = (c1 - c0) + (x == 0xffffffffu ? 1 : 0);  // x kept live: the chain is not dead code
    out[2 * w + 1] = r1 - r0;
  }
}

extern "C" {

int dkg_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int dkg_device_pci_bus_id(int device, char* buf, int len) {
  if (!buf || len < 13) return DKG_E_ARG;
  return hipDeviceGetPCIBusId(buf, len, device) == hipSuccess ? DKG_OK : DKG_E_DEVICE;
}

int dkg_ctx_clock_probe(dkg_ctx* ctx, unsigned iters, double* sclk_mhz, double* busy_ms) {
  return guarded(ctx, [&] {
    if (!sclk_mhz || !busy_ms || !iters) return DKG_E_ARG;
    int cus = 0, wall_khz = 0;
    HCK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device));
    HCK(hipDeviceGetAttribute(&wall_khz, hipDeviceAttributeWallClockRate, ctx->device));
    if (cus <= 0 || wall_khz <= 0) return DKG_E_DEVICE;
    const size_t waves = (size_t)cus * 16;  // 4 workgroups of 4 waves per CU: 4 waves per SIMD
    unsigned long long* d = buf<unsigned long long>(ctx, "clock_probe", 2 * 8 * waves);
    hipLaunchKernelGGL(k_clock_probe, dim3((unsigned)(waves / 4)), dim3(256), 0, ctx->stream, iters, d);
    check_launch(ctx);
    std::vector<unsigned long long> h(2 * waves);
    d2h(ctx, h.data(), d, 2 * 8 * waves);
    sync(ctx);
    std::vector<double> mhz(waves), ms(waves);
    for (size_t w = 0; w < waves; w++) {
      const double real_us = (double)h[2 * w + 1] / wall_khz * 1e3;
      mhz[w] = real_us > 0 ? (double)h[2 * w] / real_us : 0.0;
      ms[w] = real_us / 1e3;
    }
    std::nth_element(mhz.begin(), mhz.begin() + waves / 2, mhz.end());
    std::nth_element(ms.begin(), ms.begin() + waves / 2, ms.end());
    *sclk_mhz = mhz[waves / 2];
    *busy_ms = ms[waves / 2];
    return DKG_OK;
  });
}

int dkg_ctx_create(int device, dkg_ctx** out) {
  if (!out) return DKG_E_ARG;
  *out = nullptr;
  dkg_ctx* ctx = new dkg_ctx();
  ctx->device = device;
  int rc = guarded(ctx, [&] {
    // the ceremony's own streams at the highest priority, the side stream at the lowest: a
    // latency-bound binomial step must not queue behind the side stream's share evaluation
    int least = 0, greatest = 0;
    HCK(hipDeviceGetStreamPriorityRange(&least, &greatest));
    HCK(hipStreamCreateWithPriority(&ctx->stream, hipStreamNonBlocking, greatest));
    for (auto& e : ctx->ev) HCK(hipEventCreate(&e));
    for (auto& e : ctx->pev) HCK(hipEventCreate(&e));
    for (auto& e : ctx->hev) HCK(hipEventCreate(&e));
    for (auto& st : ctx->sub) HCK(hipStreamCreateWithPriority(&st, hipStreamNonBlocking, greatest));
    HCK(hipStreamCreateWithPriority(&ctx->side, hipStreamNonBlocking, least));
    HCK(hipEventCreateWithFlags(&ctx->side_fork, hipEventDisableTiming));
    HCK(hipEventCreateWithFlags(&ctx->shares_done, hipEventDisableTiming));
    HCK(hipEventCreateWithFlags(&ctx->pub_done, hipEventDisableTiming));
    HCK(hipEventCreateWithFlags(&ctx->terms_done, hipEventDisableTiming));
    HCK(hipEventCreateWithFlags(&ctx->fork, hipEventDisableTiming));
    for (auto& e : ctx->join) HCK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    HCK(hipMalloc(&ctx->tab_g, COMB_BYTES));
    HCK(hipMalloc(&ctx->tab_h, COMB_BYTES));
    HCK(hipMalloc(&ctx->tab_gw, COMBW_BYTES));
    HCK(hipMalloc(&ctx->tab_hw, COMBW_BYTES));
    bool ok = false;
    comb_for_point(ctx, BASEPOINT, ctx->tab_g, &ok, ctx->tab_gw);
    if (!ok) {
      ctx->err = "basepoint failed to decode on device";
      return DKG_E_DEVICE;
    }
    return DKG_OK;
  });
  if (rc != DKG_OK) {
    fprintf(stderr, "dkg_ctx_create: %s\n", ctx->err.c_str());
    dkg_ctx_destroy(ctx);
    return rc;
  }
  *out = ctx;
  return DKG_OK;
}

void dkg_ctx_destroy(dkg_ctx* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  if (ctx->stream) (void)hipDeviceSynchronize();
  for (auto& kv : ctx->bufs) (void)hipFree(kv.second.first);
  for (auto& kv : ctx->hbufs) (void)hipHostFree(kv.second.first);
  if (ctx->tab_g) (void)hipFree(ctx->tab_g);
  if (ctx->tab_h) (void)hipFree(ctx->tab_h);
  if (ctx->tab_gw) (void)hipFree(ctx->tab_gw);
  if (ctx->tab_hw) (void)hipFree(ctx->tab_hw);
  for (auto& e : ctx->ev)
    if (e) (void)hipEventDestroy(e);
  for (auto& e : ctx->pev)
    if (e) (void)hipEventDestroy(e);
  for (auto& e : ctx->hev)
    if (e) (void)hipEventDestroy(e);
  for (auto& e : ctx->join)
    if (e) (void)hipEventDestroy(e);
  if (ctx->fork) (void)hipEventDestroy(ctx->fork);
  for (auto& st : ctx->sub)
    if (st) (void)hipStreamDestroy(st);
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  if (ctx->side) (void)hipStreamDestroy(ctx->side);
  if (ctx->side_fork) (void)hipEventDestroy(ctx->side_fork);
  if (ctx->shares_done) (void)hipEventDestroy(ctx->shares_done);
  if (ctx->pub_done) (void)hipEventDestroy(ctx->pub_done);
  delete ctx;
}

const char* dkg_ctx_last_error(const dkg_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

double dkg_ctx_phase_ms(const dkg_ctx* ctx, const char* name) {
  if (!ctx || !name) return -1.0;
  auto it = ctx->phase_ms.find(name);
  return it == ctx->phase_ms.end() ? -1.0 : it->second;
}

int dkg_ctx_set_streams(dkg_ctx* ctx, int nsub) {
  if (!ctx || nsub < 1 || nsub > dkg_ctx::MAX_SUB) return DKG_E_ARG;
  ctx->nsub = nsub;
  return DKG_OK;
}

int dkg_ctx_set_verify_mode(dkg_ctx* ctx, int mode) {
  if (!ctx || mode < 0 || mode > 1) return DKG_E_ARG;
  ctx->verify_mode = mode;
  return DKG_OK;
}

size_t dkg_ctx_fallback_rows(const dkg_ctx* ctx) { return ctx ? ctx->fallback_rows : 0; }

int dkg_ctx_set_split(dkg_ctx* ctx, int pieces) {
  if (!ctx || pieces < 0 || pieces > 16) return DKG_E_ARG;
  ctx->split = pieces;
  return DKG_OK;
}

int dkg_ctx_set_binomial(dkg_ctx* ctx, int mode) {
  if (!ctx || mode < 0 || mode > 5) return DKG_E_ARG;
  ctx->binom_mode = mode;
  return DKG_OK;
}

int dkg_ctx_set_check(dkg_ctx* ctx, int mode) {
  if (!ctx || mode < 0 || mode > 1) return DKG_E_ARG;
  ctx->check_mode = mode;
  return DKG_OK;
}

int dkg_ctx_set_field_mode(dkg_ctx* ctx, int mode) {
  if (!ctx || mode < 0 || mode > 2) return DKG_E_ARG;
  ctx->fe_mode = mode;
  return DKG_OK;
}

int dkg_ctx_set_stepping(dkg_ctx* ctx, int mode) {
  if (!ctx || mode < 0 || mode > 3) return DKG_E_ARG;
  ctx->step_mode = mode;
  return DKG_OK;
}

int dkg_ctx_last_split(const dkg_ctx* ctx) { return ctx ? ctx->last_split : 0; }
size_t dkg_ctx_last_split_len(const dkg_ctx* ctx) { return ctx ? ctx->last_split_len : 0; }
int dkg_ctx_set_combine(dkg_ctx* ctx, int mode) {
  if (!ctx || mode < 0 || mode > 2) return DKG_E_ARG;
  ctx->combine_mode = mode;
  return DKG_OK;
}
int dkg_ctx_last_combine(const dkg_ctx* ctx) { return ctx ? ctx->last_combine : 0; }
int dkg_ctx_last_binomial(const dkg_ctx* ctx) { return ctx ? ctx->last_binomial : 0; }
int dkg_ctx_set_stepping_formula(dkg_ctx* ctx, int mode) {
  if (!ctx || mode < 0 || mode > 1) return DKG_E_ARG;
  ctx->step_formula = mode;
  return DKG_OK;
}
long long dkg_ctx_stepping_redos(dkg_ctx* ctx) {
  if (!ctx) return -1;
  if (!ctx->last_step_flags) return 0;
  try {
    std::vector<uint32_t> h(ctx->last_step_flag_words);
    sync(ctx);
    HCK(hipMemcpy(h.data(), ctx->last_step_flags, 4 * h.size(), hipMemcpyDeviceToHost));
    long long c = 0;
    for (uint32_t x : h) c += x != 0;
    return c;
  } catch (const Fail& f) {
    return -1;
  }
}
int dkg_ctx_binomial_reruns(dkg_ctx* ctx) { return ctx ? ctx->last_binom_rerun : -1; }
int dkg_ctx_set_addends(dkg_ctx* ctx, int mode) {
  if (!ctx || mode < 0 || mode > 1) return DKG_E_ARG;
  ctx->addend_mode = mode;
  return DKG_OK;
}
int dkg_split_multipliers(size_t n, size_t L, int pieces, uint8_t* mag, int8_t* sign) {
  if (!n || !L || pieces < 2 || pieces > (int)SHORT_MAX || !mag || !sign) return DKG_E_ARG;
  try {
    std::vector<uint8_t> m;
    std::vector<int8_t> sg;
    short_vectors(n, L, (size_t)pieces, m, sg);
    memcpy(mag, m.data(), m.size());
    memcpy(sign, sg.data(), sg.size());
  } catch (const std::exception&) {
    return DKG_E_NOMEM;
  }
  return DKG_OK;
}

double dkg_split_model_ms(size_t columns, size_t n, size_t t, int pieces) {
  if (pieces < 1 || t + 1 < (size_t)pieces) return -1;
  return split_model_ms(columns, n, t + 1, (size_t)pieces);
}

size_t dkg_split_len(size_t columns, size_t n, size_t t, int pieces) {
  if (pieces < 1 || t + 1 < (size_t)pieces) return 0;
  return split_len(columns, n, t + 1, (size_t)pieces);
}

int dkg_ctx_set_overlap(dkg_ctx* ctx, int on) {
  if (!ctx) return DKG_E_ARG;
  ctx->overlap = on != 0;
  return DKG_OK;
}

int dkg_env_check(size_t threshold, size_t nr_members) {
  // committee.rs:73: assert!(threshold < (nr_members + 1) / 2)
  if (nr_members == 0 || !(threshold < (nr_members + 1) / 2)) return DKG_E_ARG;
  return DKG_OK;
}

int dkg_env_init(dkg_ctx* ctx, size_t threshold, size_t nr_members, const uint8_t* ck, size_t ck_len,
                 uint8_t h_out[32]) {
  int rc = dkg_env_check(threshold, nr_members);
  if (rc != DKG_OK) {
    if (ctx) ctx->err = "threshold must be < (nr_members + 1) / 2 (committee.rs:73)";
    return rc;
  }
  return guarded(ctx, [&] {
    // CommitmentKey::generate: h = RistrettoPoint::hash_from_bytes::<Blake2b>(ck) (commitment.rs:13-17)
    uint8_t hash[64];
    dkgh::blake2b(hash, 64, ck, ck_len);
    uint32_t* in = buf<uint32_t>(ctx, "h_in", 64);
    uint32_t* ext = buf<uint32_t>(ctx, "h_ext", PTB);
    uint32_t* comp = buf<uint32_t>(ctx, "h_comp", 32);
    h2d(ctx, in, hash, 64);
    dkgk::from_uniform(in, ext, ctx->stream);
    dkgk::encode_points(ext, 1, 1, comp, ctx->stream);
    check_launch(ctx);
    d2h(ctx, ctx->h, comp, 32);
    sync(ctx);
    bool ok = false;
    comb_for_point(ctx, ctx->h, ctx->tab_h, &ok, ctx->tab_hw);
    if (!ok) return DKG_E_DEVICE;
    ctx->have_h = true;
    ctx->threshold = threshold;
    ctx->nr_members = nr_members;
    if (h_out) memcpy(h_out, ctx->h, 32);
    return DKG_OK;
  });
}

int dkg_msm_batch(dkg_ctx* ctx, size_t B, size_t N, const uint8_t* scalars, const uint8_t* points, uint8_t* out) {
  return guarded(ctx, [&] {
    if (B == 0) return DKG_OK;
    uint32_t* sc = upload_scalars(ctx, "msm_sc", scalars, B * N);
    uint32_t* pc = buf<uint32_t>(ctx, "msm_pc", 32 * B * N);
    uint32_t* pe = buf<uint32_t>(ctx, "msm_pe", PTB * B * N);
    uint8_t* ok = buf<uint8_t>(ctx, "msm_ok", B * N);
    h2d(ctx, pc, points, 32 * B * N);
    dkgk::decode_points(pc, B * N, pe, B * N, ok, ctx->stream);
    uint32_t* oe = buf<uint32_t>(ctx, "msm_oe", PTB * B);
    uint32_t* oc = buf<uint32_t>(ctx, "msm_oc", 32 * B);
    uint32_t* mt = buf<uint32_t>(ctx, "msm_tab", 4 * 15 * PT_WORDS_H * B * N);
  dkgk::msm_batch(B, N, sc, pe, B * N, mt, oe, ctx->stream);
    dkgk::encode_points(oe, B, B, oc, ctx->stream);
    check_launch(ctx);
    std::vector<uint8_t> okh(B * N);
    d2h(ctx, okh.data(), ok, B * N);
    d2h(ctx, out, oc, 32 * B);
    sync(ctx);
    for (auto v : okh)
      if (!v) {
        ctx->err = "msm: a point failed to decode";
        return DKG_E_DECODE;
      }
    return DKG_OK;
  });
}

int dkg_fixed_base_batch(dkg_ctx* ctx, const uint8_t base[32], size_t count, const uint8_t* scalars, uint8_t* out) {
  return guarded(ctx, [&] {
    if (count == 0) return DKG_OK;
    const uint32_t* tab = ctx->tab_gw;
    // the generator and the commitment key have their combs already; another base's comb (470 MB,
    // ~1M entry threads) is built once and kept while the caller passes the same base bytes
    if (base && memcmp(base, BASEPOINT, 32) == 0) {
      base = nullptr;
    } else if (base && ctx->have_h && ctx->tab_hw && memcmp(base, ctx->h, 32) == 0) {
      tab = ctx->tab_hw;
      base = nullptr;
    }
    if (base) {
      uint32_t* t = buf<uint32_t>(ctx, "fb_tabw", COMBW_BYTES);
      if (!ctx->fb_valid || memcmp(ctx->fb_base, base, 32) != 0) {
        ctx->fb_valid = false;
        bool ok = false;
        comb_for_point(ctx, base, nullptr, &ok, t);
        if (!ok) {
          ctx->err = "fixed_base: base point failed to decode";
          return DKG_E_DECODE;
        }
        memcpy(ctx->fb_base, base, 32);
        ctx->fb_valid = true;
      }
      tab = t;
    }
    uint32_t* sc = upload_scalars(ctx, "fb_sc", scalars, count);
    uint32_t* oe = buf<uint32_t>(ctx, "fb_oe", PTB * count);
    uint32_t* oc = buf<uint32_t>(ctx, "fb_oc", 32 * count);
    dkgk::fixed_base(count, sc, tab, oe, ctx->stream);
    dkgk::encode_points(oe, count, count, oc, ctx->stream);
    check_launch(ctx);
    d2h(ctx, out, oc, 32 * count);
    sync(ctx);
    return DKG_OK;
  });
}

int dkg_poly_eval_batch(dkg_ctx* ctx, size_t D, size_t N, const uint8_t* coeffs, size_t M, const uint32_t* xs,
                        uint8_t* out) {
  return guarded(ctx, [&] {
    if (D == 0 || M == 0) return DKG_OK;
    if (N == 0) return DKG_E_ARG;
    for (size_t m = 0; m < M; m++)
      if (xs[m] >= (1u << 24)) {
        ctx->err = "poly_eval: evaluation points must be < 2^24";
        return DKG_E_ARG;
      }
    uint32_t* c = upload_scalars(ctx, "pe_c", coeffs, D * N);
    uint32_t* x = buf<uint32_t>(ctx, "pe_x", 4 * M);
    uint32_t* o = buf<uint32_t>(ctx, "pe_o", 32 * D * M);
    h2d(ctx, x, xs, 4 * M);
    dkgk::poly_eval(D, N, c, M, x, o, ctx->stream);
    check_launch(ctx);
    d2h(ctx, out, o, 32 * D * M);
    sync(ctx);
    return DKG_OK;
  });
}

int dkg_points_valid_batch(dkg_ctx* ctx, size_t count, const uint8_t* points, uint8_t* ok) {
  return guarded(ctx, [&] {
    if (count == 0) return DKG_OK;
    uint32_t* pc = buf<uint32_t>(ctx, "pv_c", 32 * count);
    uint32_t* pe = buf<uint32_t>(ctx, "pv_e", PTB * count);
    uint8_t* od = buf<uint8_t>(ctx, "pv_ok", count);
    h2d(ctx, pc, points, 32 * count);
    dkgk::decode_points(pc, count, pe, count, od, ctx->stream);
    check_launch(ctx);
    d2h(ctx, ok, od, count);
    sync(ctx);
    return DKG_OK;
  });
}

int dkg_share_gen(dkg_ctx* ctx, size_t D, size_t n, size_t t, const uint8_t* a, const uint8_t* b, uint8_t* E,
                  uint8_t* A, uint8_t* s, uint8_t* s_prime) {
  return guarded(ctx, [&] {
    int rc = need_env(ctx);
    if (rc) return rc;
    if (D == 0) return DKG_OK;
    const size_t N = t + 1;
    uint32_t* da = upload_scalars(ctx, "sg_a", a, D * N);
    uint32_t* db = upload_scalars(ctx, "sg_b", b, D * N);
    uint32_t* Ec = buf<uint32_t>(ctx, "sg_E", 32 * D * N);
    uint32_t* Ac = buf<uint32_t>(ctx, "sg_A", 32 * D * N);
    uint32_t* ds = buf<uint32_t>(ctx, "sg_s", 32 * D * n);
    uint32_t* dsp = buf<uint32_t>(ctx, "sg_sp", 32 * D * n);
    round1_device(ctx, D, n, t, da, db, Ec, Ac, ds, dsp);
    if (E) d2h(ctx, E, Ec, 32 * D * N);
    if (A) d2h(ctx, A, Ac, 32 * D * N);
    if (s) d2h(ctx, s, ds, 32 * D * n);
    if (s_prime) d2h(ctx, s_prime, dsp, 32 * D * n);
    sync(ctx);
    return DKG_OK;
  });
}

int dkg_share_gen_device(dkg_ctx* ctx, size_t D, size_t n, size_t t, const void* d_a, const void* d_b, void* d_E,
                         void* d_A, void* d_s, void* d_s_prime) {
  return guarded(ctx, [&] {
    int rc = need_env(ctx);
    if (rc) return rc;
    if (!d_a || !d_b || !d_s || !d_s_prime) return DKG_E_ARG;
    if (D == 0) return DKG_OK;
    const size_t N = t + 1;
    uint32_t* Ec = d_E ? (uint32_t*)d_E : buf<uint32_t>(ctx, "sgd_E", 32 * D * N);
    uint32_t* Ac = d_A ? (uint32_t*)d_A : buf<uint32_t>(ctx, "sgd_A", 32 * D * N);
    round1_device(ctx, D, n, t, (const uint32_t*)d_a, (const uint32_t*)d_b, Ec, Ac, (uint32_t*)d_s,
                  (uint32_t*)d_s_prime, d_E || d_A);
    sync(ctx);
    return DKG_OK;
  });
}

int dkg_verify_pairs(dkg_ctx* ctx, size_t n, size_t t, int round, size_t d0, size_t d1, const uint8_t* C,
                     const uint8_t* s, const uint8_t* s_prime, uint8_t* decision) {
  return guarded(ctx, [&] {
    if ((round != 2 && round != 4) || d1 < d0 || d1 > n) return DKG_E_ARG;
    if (round == 2) {
      int rc = need_env(ctx);
      if (rc) return rc;
      if (!s_prime) return DKG_E_ARG;
    }
    const size_t D = d1 - d0, N = t + 1;
    if (D == 0) return DKG_OK;
    uint32_t* Cc = buf<uint32_t>(ctx, "vp_C", 32 * D * N);
    h2d(ctx, Cc, C, 32 * D * N);
    uint32_t* ds = upload_scalars(ctx, "vp_s", s, D * n);
    uint32_t* dsp = round == 2 ? upload_scalars(ctx, "vp_sp", s_prime, D * n) : nullptr;
    uint8_t* dec = buf<uint8_t>(ctx, "vp_dec", D * n);
    verify_one(ctx, n, t, round, D, d0, Cc, ds, dsp, dec, false);
    d2h(ctx, decision, dec, D * n);
    sync(ctx);
    return DKG_OK;
  });
}

int dkg_verify_receiver(dkg_ctx* ctx, size_t n, size_t t, int round, size_t j, const uint8_t* C, const uint8_t* s,
                        const uint8_t* s_prime, uint8_t* decision) {
  return guarded(ctx, [&] {
    if ((round != 2 && round != 4) || j >= n) return DKG_E_ARG;
    ctx->last_step_flags = nullptr;  // Horner per receiver: no stepping tables
    ctx->last_step_flag_words = 0;
    if (round == 2) {
      int rc = need_env(ctx);
      if (rc) return rc;
      if (!s_prime) return DKG_E_ARG;
    }
    const size_t N = t + 1, npad = pad64(n);
    uint32_t* Cc = buf<uint32_t>(ctx, "vr_C", 32 * n * N);
    h2d(ctx, Cc, C, 32 * n * N);
    uint32_t* Cext = buf<uint32_t>(ctx, "Cext", PTB * n * N);
    uint8_t* pok = buf<uint8_t>(ctx, "pok", n * N);
    uint8_t* dok = buf<uint8_t>(ctx, "dok", n);
    uint32_t* Cpm = buf<uint32_t>(ctx, "Cpm", PTB * N * npad);
    dkgk::decode_points(Cc, n * N, Cext, n * N, pok, ctx->stream);
    dkgk::dealer_ok(n, N, pok, dok, ctx->stream);
    dkgk::to_position_major(n, N, npad, Cext, Cpm, ctx->stream);
    uint32_t* R = buf<uint32_t>(ctx, "vr_R", PTB * n);
    dkgk::horner(n, npad, N, Cpm, (uint32_t)(j + 1), 1, R, ctx->stream);  // committee.rs:287-296, one party
    uint32_t* ds = upload_scalars(ctx, "vr_s", s, n);
    uint32_t* dsp = round == 2 ? upload_scalars(ctx, "vr_sp", s_prime, n) : nullptr;
    uint8_t* dec = buf<uint8_t>(ctx, "vr_dec", n);
    dkgk::check(n, 1, 0, j, n, round, ds, dsp, R, ctx->tab_gw, ctx->tab_hw, dok, dec, ctx->stream);
    check_launch(ctx);
    d2h(ctx, decision, dec, n);
    sync(ctx);
    return DKG_OK;
  });
}

int dkg_ceremony_run_device(dkg_ctx* ctx, size_t n, size_t t, const void* d_a, const void* d_b,
                            dkg_ceremony_out* out) {
  return guarded(ctx, [&] {
    int rc = need_env(ctx);
    if (rc) return rc;
    if (dkg_env_check(t, n) != DKG_OK || !out) return DKG_E_ARG;
    const size_t N = t + 1;
    HCK(hipEventRecord(ctx->ev[0], ctx->stream));
    uint32_t* Ec = buf<uint32_t>(ctx, "cer_E", 32 * n * N);
    uint32_t* Ac = buf<uint32_t>(ctx, "cer_A", 32 * n * N);
    uint32_t* ds = buf<uint32_t>(ctx, "cer_s", 32 * n * n);
    uint32_t* dsp = buf<uint32_t>(ctx, "cer_sp", 32 * n * n);
#ifdef DKG_NO_R1_OVERLAP
    round1_device(ctx, n, n, t, (const uint32_t*)d_a, (const uint32_t*)d_b, Ec, Ac, ds, dsp, false);
#else
    // with one stream (the bench's serialised roofline pass) the phases stay back to back
    round1_device(ctx, n, n, t, (const uint32_t*)d_a, (const uint32_t*)d_b, Ec, Ac, ds, dsp, false, ctx->nsub > 1);
#endif
    HCK(hipEventRecord(ctx->ev[1], ctx->stream));
    ExtScope ext(ctx, n, N);
    receivers_rounds(ctx, n, t, Ec, Ac, ds, dsp, out, false);  // small outputs only
    out->ms_round1 = ev_ms(ctx, 0, 1);
    out->ms_round2 = ev_ms(ctx, 1, 2);
    out->ms_round3 = ev_ms(ctx, 2, 3);
    out->ms_round4 = ev_ms(ctx, 3, 4);
    out->ms_finalise = ev_ms(ctx, 4, 5);
    out->ms_total = ev_ms(ctx, 0, 5);
    return DKG_OK;
  });
}

int dkg_ceremony_run(dkg_ctx* ctx, size_t n, size_t t, const uint8_t* a, const uint8_t* b, dkg_ceremony_out* out) {
  return guarded(ctx, [&] {
    int rc = need_env(ctx);
    if (rc) return rc;
    if (dkg_env_check(t, n) != DKG_OK || !out) return DKG_E_ARG;
    const size_t N = t + 1;
    uint32_t* da = upload_scalars(ctx, "cer_a", a, n * N);
    uint32_t* db = upload_scalars(ctx, "cer_b", b, n * N);
    HCK(hipEventRecord(ctx->ev[0], ctx->stream));
    uint32_t* Ec = buf<uint32_t>(ctx, "cer_E", 32 * n * N);
    uint32_t* Ac = buf<uint32_t>(ctx, "cer_A", 32 * n * N);
    uint32_t* ds = buf<uint32_t>(ctx, "cer_s", 32 * n * n);
    uint32_t* dsp = buf<uint32_t>(ctx, "cer_sp", 32 * n * n);
    round1_device(ctx, n, n, t, da, db, Ec, Ac, ds, dsp);
    HCK(hipEventRecord(ctx->ev[1], ctx->stream));
    if (out->E) d2h(ctx, out->E, Ec, 32 * n * N);
    if (out->A) d2h(ctx, out->A, Ac, 32 * n * N);
    if (out->s) d2h(ctx, out->s, ds, 32 * n * n);
    if (out->s_prime) d2h(ctx, out->s_prime, dsp, 32 * n * n);
    ExtScope ext(ctx, n, N);
    receivers_rounds(ctx, n, t, Ec, Ac, ds, dsp, out, true);
    out->ms_round1 = ev_ms(ctx, 0, 1);
    out->ms_round2 = ev_ms(ctx, 1, 2);
    out->ms_round3 = ev_ms(ctx, 2, 3);
    out->ms_round4 = ev_ms(ctx, 3, 4);
    out->ms_finalise = ev_ms(ctx, 4, 5);
    out->ms_total = ev_ms(ctx, 0, 5);
    return DKG_OK;
  });
}

int dkg_ceremony_verify(dkg_ctx* ctx, size_t n, size_t t, const uint8_t* E, const uint8_t* A, const uint8_t* s,
                        const uint8_t* s_prime, dkg_ceremony_out* out) {
  return guarded(ctx, [&] {
    int rc = need_env(ctx);
    if (rc) return rc;
    if (dkg_env_check(t, n) != DKG_OK || !out) return DKG_E_ARG;
    const size_t N = t + 1;
    uint32_t* Ec = buf<uint32_t>(ctx, "cer_E", 32 * n * N);
    uint32_t* Ac = buf<uint32_t>(ctx, "cer_A", 32 * n * N);
    h2d(ctx, Ec, E, 32 * n * N);
    h2d(ctx, Ac, A, 32 * n * N);
    uint32_t* ds = upload_scalars(ctx, "cer_s", s, n * n);
    uint32_t* dsp = upload_scalars(ctx, "cer_sp", s_prime, n * n);
    HCK(hipEventRecord(ctx->ev[0], ctx->stream));
    HCK(hipEventRecord(ctx->ev[1], ctx->stream));
    receivers_rounds(ctx, n, t, Ec, Ac, ds, dsp, out, true);
    out->ms_round1 = 0;
    out->ms_round2 = ev_ms(ctx, 1, 2);
    out->ms_round3 = ev_ms(ctx, 2, 3);
    out->ms_round4 = ev_ms(ctx, 3, 4);
    out->ms_finalise = ev_ms(ctx, 4, 5);
    out->ms_total = ev_ms(ctx, 0, 5);
    return DKG_OK;
  });
}

int dkg_ceremony_verify_fetched(dkg_ctx* ctx, size_t n, size_t t, const uint8_t* E, const uint8_t* A,
                                const uint8_t* s, const uint8_t* s_prime, const uint8_t* fetched1,
                                const uint8_t* fetched3, dkg_ceremony_out* out) {
  return guarded(ctx, [&] {
    int rc = need_env(ctx);
    if (rc) return rc;
    if (dkg_env_check(t, n) != DKG_OK || !out || !fetched1 || !fetched3) return DKG_E_ARG;
    const size_t N = t + 1;
    uint32_t* Ec = buf<uint32_t>(ctx, "cer_E", 32 * n * N);
    uint32_t* Ac = buf<uint32_t>(ctx, "cer_A", 32 * n * N);
    h2d(ctx, Ec, E, 32 * n * N);
    h2d(ctx, Ac, A, 32 * n * N);
    uint32_t* ds = upload_scalars(ctx, "cer_s", s, n * n);
    uint32_t* dsp = upload_scalars(ctx, "cer_sp", s_prime, n * n);
    uint8_t* f1 = buf<uint8_t>(ctx, "cer_f1", n);
    uint8_t* f3 = buf<uint8_t>(ctx, "cer_f3", n);
    h2d(ctx, f1, fetched1, n);
    h2d(ctx, f3, fetched3, n);
    HCK(hipEventRecord(ctx->ev[0], ctx->stream));
    HCK(hipEventRecord(ctx->ev[1], ctx->stream));
    receivers_rounds(ctx, n, t, Ec, Ac, ds, dsp, out, true, f1, f3);
    out->ms_round1 = 0;
    out->ms_round2 = ev_ms(ctx, 1, 2);
    out->ms_round3 = ev_ms(ctx, 2, 3);
    out->ms_round4 = ev_ms(ctx, 3, 4);
    out->ms_finalise = ev_ms(ctx, 4, 5);
    out->ms_total = ev_ms(ctx, 0, 5);
    return DKG_OK;
  });
}

}  // extern "C"

// Rounds 2-5 of one rank of a dealer-sharded ceremony on its dealers [d0, d0+D): E/A compressed
// [D][N][32], s/sp canonical [D][n][32] on the device -> decision rows, master-key terms, partial
// final shares (layouts of dkg_ceremony_shard_device).
void shard_rows(dkg_ctx* ctx, size_t n, size_t t, size_t d0, size_t D, const uint32_t* Ec, const uint32_t* Ac,
                const uint32_t* ds, const uint32_t* dsp, void* d_dec2, void* d_dec4, void* d_A0, void* d_partial) {
  const size_t N = t + 1;
  if (!D) {
    HCK(hipMemsetAsync(d_partial, 0, 32 * n, ctx->stream));
    return;
  }
  // the exchanged A_i0 encodings depend only on round 1: encoded on the side stream beside the checks
  // (a latency-bound chain of D lanes that otherwise ends the call), joined before it returns
  const bool side_terms = ctx->ext_A != nullptr;
  if (side_terms) {
    uint32_t* a0 = buf<uint32_t>(ctx, "sh_a0ext", PTB * D);
    HCK(hipEventRecord(ctx->side_fork, ctx->stream));
    HCK(hipStreamWaitEvent(ctx->side, ctx->side_fork, 0));
    dkgk::gather_points(ctx->ext_A, ctx->ext_stride, N, 0, D, a0, D, ctx->side);
    dkgk::encode_points(a0, D, D, (uint32_t*)d_A0, ctx->side);
    HCK(hipEventRecord(ctx->terms_done, ctx->side));
  } else {
    HCK(hipMemcpy2DAsync(d_A0, 32, Ac, 32 * N, 32, D, hipMemcpyDeviceToDevice, ctx->stream));
  }
  // Qualification of a dealer depends only on its own decision row (any REJECT disqualifies,
  // committee.rs:370-398; missing data disqualifies, :331-335), so each rank decides it for its
  // dealers with no exchange -- on the device, queued after the checks (no host round trip)
  uint8_t* rej = buf<uint8_t>(ctx, "sh_rej", D);
  uint8_t* qm = buf<uint8_t>(ctx, "sh_q", D);
  verify_rounds(
      ctx, n, t, D, d0, Ec, Ac, ds, dsp, (uint8_t*)d_dec2, (uint8_t*)d_dec4, nullptr,
      [&] {
        dkgk::row_reject(D, n, (const uint8_t*)d_dec2, rej, ctx->stream);
        dkgk::mask_not_and(D, rej, nullptr, qm, ctx->stream);
      },
      nullptr, nullptr, false);
  if (side_terms) HCK(hipStreamWaitEvent(ctx->stream, ctx->terms_done, 0));
  wait_shares(ctx, ctx->stream);  // shares evaluated on the side stream (round1_device)
  ctx->shares_pending = false;
  // A dealer accused in round 4 (committee.rs:660-670) has its term replaced after the exchange,
  // once the final parties are known (dkg_ceremony_shard_recon_device): its shares stay here.
  ctx->shard_s = ds;
  ctx->shard_n = n;
  ctx->shard_d0 = d0;
  ctx->shard_D = D;
  dkgk::sum_shares(D, n, ds, qm, (uint32_t*)d_partial, ctx->stream);  // partial of :454-462
}

extern "C" {

int dkg_ceremony_shard_device(dkg_ctx* ctx, size_t n, size_t t, size_t d0, size_t d1, const void* d_a,
                              const void* d_b, void* d_dec2, void* d_dec4, void* d_A0, void* d_partial,
                              double* ms_total) {
  return guarded(ctx, [&] {
    int rc = need_env(ctx);
    if (rc) return rc;
    if (dkg_env_check(t, n) != DKG_OK || d1 < d0 || d1 > n) return DKG_E_ARG;
    const size_t D = d1 - d0, N = t + 1;
    HCK(hipEventRecord(ctx->ev[0], ctx->stream));
    uint32_t* Ec = buf<uint32_t>(ctx, "sh_E", 32 * D * N);
    uint32_t* Ac = buf<uint32_t>(ctx, "sh_A", 32 * D * N);
    uint32_t* ds = buf<uint32_t>(ctx, "sh_s", 32 * D * n);
    uint32_t* dsp = buf<uint32_t>(ctx, "sh_sp", 32 * D * n);
    // the shares on the side stream beside the checks, which wait for them (one-stream runs: back to back);
    // on an exception the home stream still waits for them before the state is dropped
    SharesScope pending(ctx);
    if (D) round1_device(ctx, D, n, t, (const uint32_t*)d_a, (const uint32_t*)d_b, Ec, Ac, ds, dsp, false, ctx->nsub > 1);
    ExtScope ext(ctx, D, N);
    with_binom_ded(ctx, [&] {
      shard_rows(ctx, n, t, d0, D, Ec, Ac, ds, dsp, d_dec2, d_dec4, d_A0, d_partial);
      check_launch(ctx);
      HCK(hipEventRecord(ctx->ev[1], ctx->stream));
      binom_mark_copy(ctx);
      sync(ctx);
    });
    collect_phases(ctx);  // the checks' serialised phases (shard_rows queues no host round trip)
    if (ms_total) *ms_total = ev_ms(ctx, 0, 1);
    return DKG_OK;
  });
}

int dkg_ceremony_shard_verify_device(dkg_ctx* ctx, size_t n, size_t t, size_t d0, size_t d1, const void* d_E,
                                     const void* d_A, const void* d_s, const void* d_s_prime, void* d_dec2,
                                     void* d_dec4, void* d_A0, void* d_partial, double* ms_total) {
  return guarded(ctx, [&] {
    int rc = need_env(ctx);
    if (rc) return rc;
    if (dkg_env_check(t, n) != DKG_OK || d1 < d0 || d1 > n) return DKG_E_ARG;
    const size_t D = d1 - d0;
    HCK(hipEventRecord(ctx->ev[0], ctx->stream));
    // received shares: Scalar::from_bytes semantics (bit 255 cleared, reduced), as upload_scalars
    uint32_t* ds = buf<uint32_t>(ctx, "shv_s", 32 * D * n);
    uint32_t* dsp = buf<uint32_t>(ctx, "shv_sp", 32 * D * n);
    if (D) {
      dkgk::reduce_scalars(D * n, (const uint32_t*)d_s, ds, ctx->stream);
      dkgk::reduce_scalars(D * n, (const uint32_t*)d_s_prime, dsp, ctx->stream);
    }
    with_binom_ded(ctx, [&] {
      shard_rows(ctx, n, t, d0, D, (const uint32_t*)d_E, (const uint32_t*)d_A, ds, dsp, d_dec2, d_dec4, d_A0,
                 d_partial);
      check_launch(ctx);
      HCK(hipEventRecord(ctx->ev[1], ctx->stream));
      binom_mark_copy(ctx);
      sync(ctx);
    });
    collect_phases(ctx);  // the checks' serialised phases (shard_rows queues no host round trip)
    if (ms_total) *ms_total = ev_ms(ctx, 0, 1);
    return DKG_OK;
  });
}

int dkg_ceremony_shard_recon_device(dkg_ctx* ctx, size_t n, size_t t, size_t d0, size_t d1, const uint8_t* qualified,
                                    const uint8_t* reconstruct, const uint8_t* r2_error, const uint8_t* r4_error,
                                    const void* d_s, void* d_terms, int32_t* recovery_error) {
  return guarded(ctx, [&] {
    if (!qualified || !reconstruct || !d_terms || d1 < d0 || d1 > n || dkg_env_check(t, n) != DKG_OK) return DKG_E_ARG;
    const size_t D = d1 - d0;
    // decided from the common outcome alone: the same on every rank, whichever dealers it holds
    const std::vector<uint8_t> disc = disclosing_parties(n, qualified, reconstruct, r2_error, r4_error);
    bool any = false;
    for (size_t i = 0; i < n; i++) any |= reconstruct[i] != 0;
    const bool fails = any && recovery_fails(disc, t);
    if (recovery_error) *recovery_error = fails ? 1 : 0;
    if (fails) return DKG_OK;  // nobody recovers: the caller zeroes the mpk
    std::vector<size_t> rows;
    for (size_t i = 0; i < D; i++) {
      if (reconstruct[d0 + i] && !qualified[d0 + i]) {
        ctx->err = "shard_recon: only qualified members are reconstructed (committee.rs:746-747)";
        return DKG_E_ARG;
      }
      if (reconstruct[d0 + i]) rows.push_back(i);
    }
    if (rows.empty()) return DKG_OK;
    const uint32_t* ds = nullptr;
    if (d_s) {  // received shares: Scalar::from_bytes semantics
      uint32_t* red = buf<uint32_t>(ctx, "shr_s", 32 * D * n);
      dkgk::reduce_scalars(D * n, (const uint32_t*)d_s, red, ctx->stream);
      ds = red;
    } else {
      if (!ctx->shard_s || ctx->shard_n != n || ctx->shard_d0 != d0 || ctx->shard_D != D) {
        ctx->err = "shard_recon: d_s is NULL and the last sharded call on this ctx had other dealers";
        return DKG_E_ARG;
      }
      ds = ctx->shard_s;
    }
    const size_t R = rows.size();
    std::vector<uint8_t> hs(32 * n * R);
    for (size_t r = 0; r < R; r++) d2h(ctx, &hs[32 * n * r], ds + 8 * n * rows[r], 32 * n);
    sync(ctx);
    std::vector<size_t> idx(R);
    for (size_t r = 0; r < R; r++) idx[r] = r;
    std::vector<uint8_t> secrets = recon_secrets(n, disc, hs.data(), idx);
    uint32_t* sec = buf<uint32_t>(ctx, "sh_rsec", 32 * R);
    uint32_t* gsec = buf<uint32_t>(ctx, "sh_rext", PTB * R);
    uint32_t* gc = buf<uint32_t>(ctx, "sh_rcomp", 32 * R);
    h2d(ctx, sec, secrets.data(), secrets.size());
    dkgk::fixed_base(R, sec, ctx->tab_gw, gsec, ctx->stream);  // G::generator() * recovered (:789)
    dkgk::encode_points(gsec, R, R, gc, ctx->stream);
    for (size_t r = 0; r < R; r++)
      HCK(hipMemcpyAsync((uint8_t*)d_terms + 32 * rows[r], gc + 8 * r, 32, hipMemcpyDeviceToDevice, ctx->stream));
    check_launch(ctx);
    sync(ctx);
    return DKG_OK;
  });
}

int dkg_finalise_parties(dkg_ctx* ctx, size_t n, size_t t, const uint8_t* qualified, const uint8_t* reconstruct,
                         const uint8_t* r2_error, const uint8_t* r4_error, const uint8_t* disclosed, const uint8_t* A0,
                         const uint8_t* s, uint8_t* mpk, int32_t* status, int32_t* recovery_index) {
  return guarded(ctx, [&] {
    using namespace dkgh;
    if (!qualified || !reconstruct || !A0 || !s || !mpk || !status) return DKG_E_ARG;
    if (!n) return DKG_OK;
    std::vector<size_t> recon;
    int32_t nq = 0;
    for (size_t i = 0; i < n; i++) {
      if (reconstruct[i] && !qualified[i]) {
        ctx->err = "finalise: only qualified members should be reconstructed (committee.rs:746-747 panics)";
        return DKG_E_ARG;
      }
      nq += qualified[i] != 0;
      if (reconstruct[i]) recon.push_back(i);
    }
    const std::vector<uint8_t> fin = final_parties(n, qualified, reconstruct);
    const bool phase4 = nq - (int32_t)recon.size() <= (int32_t)t;  // committee.rs:673-677
    // S: final parties whose phase-5 disclosures the finalising party fetched (committee.rs:763-775).
    // A party whose Phase1 or Phase3 proceed failed never reaches Phase4::proceed and so never
    // broadcasts a BroadcastPhase5 (:340-347, :567-569, :684), whatever `disclosed` says.
    std::vector<uint8_t> S(n);
    size_t nS = 0;
    for (size_t j = 0; j < n; j++)
      nS += S[j] = fin[j] && (!disclosed || disclosed[j]) && !(r2_error && r2_error[j]) &&
                   !(r4_error && r4_error[j]);
    const Zl zero = zl_from_u64(0), one = zl_from_u64(1);
    std::vector<Zl> lamS, yrows;  // Lagrange coefficients over S; the reconstructed rows' shares
    if (!recon.empty() && !phase4) {
      lamS = lagrange_zero_coeffs(n, S.data());
      yrows.resize(recon.size() * n);
      for (size_t r = 0; r < recon.size(); r++)
        for (size_t j = 0; j < n; j++) yrows[r * n + j] = zl_from_bytes_wide(s + 32 * (recon[r] * n + j), 32);
    }
    Zl PS = one;
    for (size_t j = 0; j < n; j++)
      if (S[j]) PS = zl_mul(PS, zl_from_u64(j + 1));
    std::vector<uint8_t> sig(32 * n, 0), ok(n, 0);
    std::vector<Zl> mu(n), inv(n), pre(n);
    for (size_t p = 0; p < n; p++) {
      if (recovery_index) recovery_index[p] = -1;
      if (r2_error && r2_error[p]) { status[p] = DKG_FIN_R2_ERROR; continue; }   // committee.rs:340-347
      if (r4_error && r4_error[p]) { status[p] = DKG_FIN_R4_ERROR; continue; }   // :567-569
      if (phase4) { status[p] = DKG_FIN_PHASE4_ERROR; continue; }                // :673-677
      // the party's own share plus the fetched disclosures of the other final parties (:754-775)
      const size_t cnt = nS + (S[p] ? 0 : 1);
      // finalise walks the dealers in index order (:745-797) and stops at the first of: a
      // reconstructed dealer with fewer than `threshold` (t, not t + 1) points ->
      // InsufficientSharesForRecovery(i) (:779-781); a disqualified dealer other than itself ->
      // the reference PANICS: its committed coefficients were never recorded (committed_shares[i]
      // is set only for itself, :190, and for qualified dealers in Phase3::proceed, :527-530) and
      // :791-794 expect() them.  A disqualified party p adds its own A_p0 (its init state).
      status[p] = DKG_FIN_OK;
      for (size_t i = 0; i < n && status[p] == DKG_FIN_OK; i++) {
        if (reconstruct[i] && cnt < t) status[p] = DKG_FIN_INSUFFICIENT;
        else if (!reconstruct[i] && !qualified[i] && i != p) status[p] = DKG_FIN_PANIC;
        if (status[p] != DKG_FIN_OK && recovery_index) recovery_index[p] = (int32_t)i;
      }
      if (status[p] != DKG_FIN_OK) continue;
      ok[p] = 1;
      if (recon.empty()) continue;
      const std::vector<Zl>* lam = &lamS;
      if (!S[p]) {
        // T = S u {p}: mu_a = lambda^S_a x_p / (x_p - x_a) (a in S), mu_p = prod_{b in S} x_b / (x_b - x_p)
        const Zl xp = zl_from_u64(p + 1);
        std::vector<size_t> as;
        for (size_t a = 0; a < n; a++)
          if (S[a]) as.push_back(a);
        Zl acc = one;  // batch inversion of (x_p - x_a)
        for (size_t k = 0; k < as.size(); k++) {
          pre[k] = acc;
          inv[k] = zl_sub(xp, zl_from_u64(as[k] + 1));
          acc = zl_mul(acc, inv[k]);
        }
        Zl ia = zl_inv(acc);
        for (size_t k = as.size(); k-- > 0;) {
          const Zl d = inv[k];
          inv[k] = zl_mul(ia, pre[k]);
          ia = zl_mul(ia, d);
        }
        Zl prod = one;
        for (size_t a = 0; a < n; a++) mu[a] = zero;
        for (size_t k = 0; k < as.size(); k++) {
          mu[as[k]] = zl_mul(zl_mul(lamS[as[k]], xp), inv[k]);
          prod = zl_mul(prod, zl_sub(zero, inv[k]));  // 1 / (x_b - x_p)
        }
        mu[p] = zl_mul(PS, prod);
        lam = &mu;
      }
      Zl sigma = zero;  // sum over the reconstructed dealers of the recovered secrets (:784-789)
      for (size_t r = 0; r < recon.size(); r++)
        for (size_t a = 0; a < n; a++)
          if (!zl_is_zero((*lam)[a])) sigma = zl_add(sigma, zl_mul((*lam)[a], yrows[r * n + a]));
      zl_to_bytes(&sig[32 * p], sigma);
    }
    memset(mpk, 0, 32 * n);
    size_t nok = 0;
    for (auto v : ok) nok += v;
    if (!nok) return DKG_OK;
    // mpk_p = sum_{final i} A_i0 + G::generator() * sigma_p (:789-795), on the device
    uint32_t* a0c = buf<uint32_t>(ctx, "fp_a0c", 32 * n);
    uint32_t* a0e = buf<uint32_t>(ctx, "fp_a0e", PTB * n);
    uint8_t* a0ok = buf<uint8_t>(ctx, "fp_a0ok", n);
    uint8_t* fm = buf<uint8_t>(ctx, "fp_fin", n);
    uint32_t* hsum = buf<uint32_t>(ctx, "fp_h", PTB);
    uint32_t* hrep = buf<uint32_t>(ctx, "fp_hrep", PTB * n);
    uint32_t* sd = buf<uint32_t>(ctx, "fp_sig", 32 * n);
    uint32_t* ge = buf<uint32_t>(ctx, "fp_ge", PTB * n);
    uint32_t* oc = buf<uint32_t>(ctx, "fp_out", 32 * n);
    h2d(ctx, a0c, A0, 32 * n);
    h2d(ctx, fm, fin.data(), n);
    h2d(ctx, sd, sig.data(), 32 * n);
    dkgk::decode_points(a0c, n, a0e, n, a0ok, ctx->stream);
    dkgk::sum_points(n, a0e, n, fm, hsum, 1, 0, ctx->stream);
    dkgk::gather_points(hsum, 1, 0, 0, n, hrep, n, ctx->stream);
    // a finalising disqualified party (the only disqualified dealer) also adds its own A_p0
    for (size_t p = 0; p < n; p++)
      if (ok[p] && !qualified[p]) dkgk::add_points(1, hrep + p, a0e + p, n, hrep + p, ctx->stream);
    dkgk::fixed_base(n, sd, ctx->tab_gw, ge, ctx->stream);
    dkgk::add_points(n, ge, hrep, n, ge, ctx->stream);
    dkgk::encode_points(ge, n, n, oc, ctx->stream);
    check_launch(ctx);
    std::vector<uint8_t> okh(n), outh(32 * n);
    d2h(ctx, okh.data(), a0ok, n);
    d2h(ctx, outh.data(), oc, 32 * n);
    sync(ctx);
    for (size_t i = 0; i < n; i++)
      if ((fin[i] || (ok[i] && !qualified[i])) && !okh[i]) {
        ctx->err = "finalise: a summed A_0 commitment does not decode";
        return DKG_E_DECODE;
      }
    for (size_t p = 0; p < n; p++)
      if (ok[p]) memcpy(mpk + 32 * p, &outh[32 * p], 32);
    return DKG_OK;
  });
}

int dkg_scalar_sum_device(dkg_ctx* ctx, size_t rows, size_t n, const void* d_in, const void* d_mask, void* d_out) {
  return guarded(ctx, [&] {
    const uint8_t* mask = (const uint8_t*)d_mask;
    if (!mask) {
      uint8_t* ones = buf<uint8_t>(ctx, "ss_ones", rows);
      HCK(hipMemsetAsync(ones, 1, rows, ctx->stream));
      mask = ones;
    }
    dkgk::sum_shares(rows, n, (const uint32_t*)d_in, mask, (uint32_t*)d_out, ctx->stream);
    check_launch(ctx);
    sync(ctx);
    return DKG_OK;
  });
}

int dkg_point_sum_device(dkg_ctx* ctx, size_t count, const void* d_points, const void* d_mask, void* d_out) {
  return guarded(ctx, [&] {
    uint32_t* ext = buf<uint32_t>(ctx, "ps_ext", PTB * count);
    uint8_t* ok = buf<uint8_t>(ctx, "ps_ok", count);
    uint32_t* sum = buf<uint32_t>(ctx, "ps_sum", PTB);
    dkgk::decode_points((const uint32_t*)d_points, count, ext, count, ok, ctx->stream);
    dkgk::sum_points(count, ext, count, (const uint8_t*)d_mask, sum, 1, 0, ctx->stream);
    dkgk::encode_points(sum, 1, 1, (uint32_t*)d_out, ctx->stream);
    check_launch(ctx);
    std::vector<uint8_t> okh(count), mh(count, 1);
    d2h(ctx, okh.data(), ok, count);
    if (d_mask) d2h(ctx, mh.data(), d_mask, count);
    sync(ctx);
    for (size_t c = 0; c < count; c++)
      if (mh[c] && !okh[c]) {
        ctx->err = "point_sum: a selected point does not decode";
        return DKG_E_DECODE;
      }
    return DKG_OK;
  });
}

void dkg_shard_range(size_t n, size_t world_size, size_t rank, size_t* d0, size_t* d1) {
  const size_t ws = world_size ? world_size : 1;
  if (d0) *d0 = rank < ws ? (rank * n) / ws : n;
  if (d1) *d1 = rank < ws ? ((rank + 1) * n) / ws : n;
}

size_t dkg_shard_rows(size_t n, size_t world_size) {
  size_t R = 0;
  for (size_t r = 0; r < world_size; r++) R = std::max(R, ((r + 1) * n) / world_size - (r * n) / world_size);
  return R;
}

}  // extern "C"

// The combine of the sharded run from the gathered rank blocks: `dense` materialises them as the
// [n][n] matrices (compacted bytes or unpacked bitmaps), then the single-GPU drivers' outcome code.
template <typename F>
int shard_combine(dkg_ctx* ctx, size_t n, size_t t, void* d_dec2, void* d_dec4, dkg_shard_outcome* out, F&& dense) {
  uint8_t* dec2 = d_dec2 ? (uint8_t*)d_dec2 : buf<uint8_t>(ctx, "sc.dec2", n * n);
  uint8_t* dec4 = d_dec4 ? (uint8_t*)d_dec4 : buf<uint8_t>(ctx, "sc.dec4", n * n);
  uint8_t* qmask = buf<uint8_t>(ctx, "sc.qmask", n);
  dense(dec2, dec4);
  // both rounds' device halves, then one copy-back (pinned) and one sync
  uint8_t* rej2 = buf<uint8_t>(ctx, "sc.rej2", n);
  int32_t* cnt = buf<int32_t>(ctx, "sc.cnt", 4 * n);
  uint8_t* rej4 = buf<uint8_t>(ctx, "sc.rej4", n);
  uint8_t* r4d = buf<uint8_t>(ctx, "sc.r4err", n);
  round2_device(ctx, 1, n, dec2, qmask, rej2, cnt);
  round4_device(ctx, 1, n, t, dec4, qmask, rej4, r4d);
  check_launch(ctx);
  uint8_t* h = hbuf<uint8_t>(ctx, "sc.out", 7 * n);  // rej2 | rej4 | r4err | cnt
  d2h(ctx, h, rej2, n);
  d2h(ctx, h + n, rej4, n);
  d2h(ctx, h + 2 * n, r4d, n);
  d2h(ctx, h + 3 * n, cnt, 4 * n);
  sync(ctx);
  std::vector<uint8_t> q(h, h + n), r2e(n), recon(h + n, h + 2 * n), r4e(h + 2 * n, h + 3 * n);
  std::vector<int32_t> c(n);
  memcpy(c.data(), h + 3 * n, 4 * n);
  round2_host(n, t, q.data(), c.data(), r2e.data());
  round4_host(n, q.data(), recon.data());
  int32_t nq = 0, nr = 0;
  for (size_t i = 0; i < n; i++) {
    nq += q[i];
    nr += recon[i];
  }
  if (out->qualified) memcpy(out->qualified, q.data(), n);
  if (out->complaints2) memcpy(out->complaints2, c.data(), 4 * n);
  if (out->r2_error) memcpy(out->r2_error, r2e.data(), n);
  if (out->reconstruct) memcpy(out->reconstruct, recon.data(), n);
  if (out->r4_error) memcpy(out->r4_error, r4e.data(), n);
  out->n_qualified = nq;
  out->phase4_error = nq - nr <= (int32_t)t;  // committee.rs:673-677
  return DKG_OK;
}

extern "C" {

int dkg_shard_combine_device(dkg_ctx* ctx, size_t n, size_t t, size_t world_size, const void* d_dec2_g,
                             const void* d_dec4_g, void* d_dec2, void* d_dec4, dkg_shard_outcome* out) {
  return guarded(ctx, [&] {
    if (!out || !d_dec2_g || !d_dec4_g || !world_size || world_size > n || dkg_env_check(t, n) != DKG_OK)
      return DKG_E_ARG;
    const size_t R = dkg_shard_rows(n, world_size);
    return shard_combine(ctx, n, t, d_dec2, d_dec4, out, [&](uint8_t* dec2, uint8_t* dec4) {
      dkgk::compact_ranks(n, world_size, R, n, d_dec2_g, dec2, ctx->stream);
      dkgk::compact_ranks(n, world_size, R, n, d_dec4_g, dec4, ctx->stream);
    });
  });
}

size_t dkg_packed_row_words(size_t n) { return (n + 31) / 32 + 1; }

int dkg_fixed_base_windows(void) { return dkgk::fixed_base_windows(); }
int dkg_key_comb_windows(void) { return dkgk::key_comb_windows(); }

int dkg_decisions_pack_device(dkg_ctx* ctx, size_t rows, size_t nvalid, size_t n, size_t d0, const void* d_dec,
                              void* d_packed) {
  return guarded(ctx, [&] {
    if (!n || nvalid > rows || (nvalid && !d_dec) || (rows && !d_packed) || d0 + nvalid > n) return DKG_E_ARG;
    if (!rows) return DKG_OK;
    uint32_t* err = buf<uint32_t>(ctx, "pk.err", 4);
    HCK(hipMemsetAsync(err, 0, 4, ctx->stream));
    dkgk::pack_rows(rows, nvalid, n, d0, (const uint8_t*)d_dec, (uint32_t*)d_packed, err, ctx->stream);
    check_launch(ctx);
    uint32_t e = 0;
    d2h(ctx, &e, err, 4);
    sync(ctx);
    if (e) {
      ctx->err = "decisions_pack: a row holds values the packed encoding cannot carry";
      return DKG_E_ARG;
    }
    return DKG_OK;
  });
}

int dkg_shard_combine_packed_device(dkg_ctx* ctx, size_t n, size_t t, size_t world_size, const void* d_pack2_g,
                                    const void* d_pack4_g, void* d_dec2, void* d_dec4, dkg_shard_outcome* out) {
  return guarded(ctx, [&] {
    if (!out || !d_pack2_g || !d_pack4_g || !world_size || world_size > n || dkg_env_check(t, n) != DKG_OK)
      return DKG_E_ARG;
    const size_t R = dkg_shard_rows(n, world_size);
    return shard_combine(ctx, n, t, d_dec2, d_dec4, out, [&](uint8_t* dec2, uint8_t* dec4) {
      dkgk::unpack_ranks(n, world_size, R, (const uint32_t*)d_pack2_g, dec2, ctx->stream);
      dkgk::unpack_ranks(n, world_size, R, (const uint32_t*)d_pack4_g, dec4, ctx->stream);
    });
  });
}

int dkg_shard_finalise_device(dkg_ctx* ctx, size_t n, size_t t, size_t world_size, const void* d_terms_g,
                              const void* d_partials_g, const uint8_t* qualified, int phase4_error,
                              void* d_final_share, void* d_public_share, uint8_t* mpk) {
  return guarded(ctx, [&] {
    if (!d_terms_g || !d_partials_g || !qualified || !d_final_share || !mpk || !world_size || world_size > n ||
        dkg_env_check(t, n) != DKG_OK)
      return DKG_E_ARG;
    int rc = need_env(ctx);
    if (rc) return rc;
    const size_t R = dkg_shard_rows(n, world_size);
    // round 3 (committee.rs:454-467): s_j = sum over the ranks' partials, g * s_j
    uint8_t* ones = buf<uint8_t>(ctx, "sf.ones", world_size);
    HCK(hipMemsetAsync(ones, 1, world_size, ctx->stream));
    dkgk::sum_shares(world_size, n, (const uint32_t*)d_partials_g, ones, (uint32_t*)d_final_share, ctx->stream);
    if (d_public_share) {
      // the public shares run on the side stream beside the mpk's decode/sum/encode (both chains
      // are a few latency-bound launches of n threads); joined below before anything is read
      uint32_t* pub = buf<uint32_t>(ctx, "sf.pub", PTB * n);
      HCK(hipEventRecord(ctx->side_fork, ctx->stream));
      HCK(hipStreamWaitEvent(ctx->side, ctx->side_fork, 0));
      dkgk::fixed_base(n, (const uint32_t*)d_final_share, ctx->tab_gw, pub, ctx->side);
      dkgk::encode_points(pub, n, n, (uint32_t*)d_public_share, ctx->side);
      HCK(hipEventRecord(ctx->pub_done, ctx->side));
    }
    auto join_public = [&] {
      if (d_public_share) HCK(hipStreamWaitEvent(ctx->stream, ctx->pub_done, 0));
    };
    memset(mpk, 0, 32);
    if (!phase4_error) {
      // finalise (committee.rs:790-795): the qualified dealers' terms -- A_i0 for the final parties,
      // g * a_i0 recovered over the final parties for the reconstructed ones
      uint32_t* terms = buf<uint32_t>(ctx, "sf.terms", 32 * n);
      uint32_t* ext = buf<uint32_t>(ctx, "sf.ext", PTB * n);
      uint8_t* ok = buf<uint8_t>(ctx, "sf.ok", n);
      uint8_t* qm = buf<uint8_t>(ctx, "sf.q", n);
      uint32_t* sum = buf<uint32_t>(ctx, "sf.sum", PTB);
      uint32_t* mc = buf<uint32_t>(ctx, "sf.mpk", 32);
      // small host transfers through pinned staging ([qualified | ok | mpk]): no pageable bounce
      uint8_t* h = hbuf<uint8_t>(ctx, "sf.host", 2 * n + 32);
      memcpy(h, qualified, n);
      dkgk::compact_ranks(n, world_size, R, 32, d_terms_g, terms, ctx->stream);
      h2d(ctx, qm, h, n);
      dkgk::decode_points(terms, n, ext, n, ok, ctx->stream);
      dkgk::sum_points(n, ext, n, qm, sum, 1, 0, ctx->stream);
      dkgk::encode_points(sum, 1, 1, mc, ctx->stream);
      join_public();
      check_launch(ctx);
      d2h(ctx, h + n, ok, n);
      d2h(ctx, h + 2 * n, mc, 32);
      sync(ctx);
      for (size_t i = 0; i < n; i++)
        if (qualified[i] && !h[n + i]) {
          ctx->err = "shard_finalise: a qualified dealer's master-key term does not decode";
          return DKG_E_DECODE;
        }
      memcpy(mpk, h + 2 * n, 32);
      return DKG_OK;  // synced above, the public shares joined
    }
    join_public();
    check_launch(ctx);
    sync(ctx);
    return DKG_OK;
  });
}

int dkg_ceremony_batch_device(dkg_ctx* ctx, size_t B, size_t n, size_t t, const void* d_a, const void* d_b,
                              dkg_batch_out* out) {
  return guarded(ctx, [&] {
    int rc = need_env(ctx);
    if (rc) return rc;
    if (dkg_env_check(t, n) != DKG_OK || !out) return DKG_E_ARG;
    if (B == 0) return DKG_OK;
    const size_t N = t + 1, V = B * n;
    HCK(hipEventRecord(ctx->ev[0], ctx->stream));
    uint32_t* Ec = buf<uint32_t>(ctx, "bat_E", 32 * V * N);
    uint32_t* Ac = buf<uint32_t>(ctx, "bat_A", 32 * V * N);
    uint32_t* ds = buf<uint32_t>(ctx, "bat_s", 32 * V * n);
    uint32_t* dsp = buf<uint32_t>(ctx, "bat_sp", 32 * V * n);
    BatchRound1 r1(ctx, V, n, t, (const uint32_t*)d_a, (const uint32_t*)d_b, ds, dsp);
    HCK(hipEventRecord(ctx->ev[1], ctx->stream));
    // round 1 in extended form for the verification: from the deferred commitments' position-major
    // table (BatchRound1), else from round1_device's E/A arrays
    std::unique_ptr<ExtScope> ext(r1.deferred() ? nullptr : new ExtScope(ctx, V, N));
    batch_receivers(ctx, B, n, t, Ec, Ac, ds, dsp, out);
    batch_times(ctx, out, true);
    return DKG_OK;
  });
}

int dkg_ceremony_batch_verify(dkg_ctx* ctx, size_t B, size_t n, size_t t, const uint8_t* E, const uint8_t* A,
                              const uint8_t* s, const uint8_t* s_prime, dkg_batch_out* out) {
  return guarded(ctx, [&] {
    int rc = need_env(ctx);
    if (rc) return rc;
    if (dkg_env_check(t, n) != DKG_OK || !out || !E || !A || !s || !s_prime) return DKG_E_ARG;
    if (B == 0) return DKG_OK;
    const size_t N = t + 1, V = B * n;
    uint32_t* Ec = buf<uint32_t>(ctx, "bat_E", 32 * V * N);
    uint32_t* Ac = buf<uint32_t>(ctx, "bat_A", 32 * V * N);
    h2d(ctx, Ec, E, 32 * V * N);
    h2d(ctx, Ac, A, 32 * V * N);
    uint32_t* ds = upload_scalars(ctx, "bat_s", s, V * n);
    uint32_t* dsp = upload_scalars(ctx, "bat_sp", s_prime, V * n);
    HCK(hipEventRecord(ctx->ev[0], ctx->stream));
    HCK(hipEventRecord(ctx->ev[1], ctx->stream));
    batch_receivers(ctx, B, n, t, Ec, Ac, ds, dsp, out);
    batch_times(ctx, out, false);
    return DKG_OK;
  });
}

int dkg_dealer_coeffs_device(dkg_ctx* ctx, const uint8_t master[32], uint32_t ceremony0, size_t B, size_t d0,
                             size_t D, size_t t, void* d_a, void* d_b) {
  return guarded(ctx, [&] {
    if (!master || !d_a || !d_b) return DKG_E_ARG;
    const size_t rows = B * D;
    if (!rows) return DKG_OK;
    uint32_t* m = buf<uint32_t>(ctx, "sg_master", 32);
    uint32_t* seeds = buf<uint32_t>(ctx, "sg_seeds", 32 * rows);
    h2d(ctx, m, master, 32);
    dkgk::dealer_coeffs(rows, D, d0, ceremony0, m, t + 1, seeds, (uint32_t*)d_a, (uint32_t*)d_b, ctx->stream);
    check_launch(ctx);
    sync(ctx);
    return DKG_OK;
  });
}

int dkg_member_keys(dkg_ctx* ctx, const uint8_t master[32], uint32_t ceremony, size_t n, uint8_t* sk_out,
                    uint8_t* pk_out) {
  return guarded(ctx, [&] {
    if (!master || !sk_out || !pk_out) return DKG_E_ARG;
    if (!n) return DKG_OK;
    static const char tag[] = "dkg-amd/v1/member";
    std::vector<uint8_t> sk(32 * n), pk(32 * n);
    for (size_t j = 0; j < n; j++) {  // MemberCommunicationKey::new (procedure_keys.rs:72-76), seeded
      uint8_t msg[sizeof tag - 1 + 40], seed[32], st[64];
      memcpy(msg, tag, sizeof tag - 1);
      memcpy(msg + sizeof tag - 1, master, 32);
      for (int k = 0; k < 4; k++) {
        msg[sizeof tag - 1 + 32 + k] = (uint8_t)(ceremony >> (8 * k));
        msg[sizeof tag - 1 + 36 + k] = (uint8_t)((uint32_t)j >> (8 * k));
      }
      dkgh::blake2b(seed, 32, msg, sizeof msg);
      dkgh::chacha20(seed, 0, st, 64);
      dkgh::zl_to_bytes(&sk[32 * j], dkgh::zl_from_bytes_wide(st, 64));
    }
    uint32_t* dsk = buf<uint32_t>(ctx, "mk_sk", 32 * n);
    uint32_t* dpe = buf<uint32_t>(ctx, "mk_pk_ext", PTB * n);
    uint32_t* dpc = buf<uint32_t>(ctx, "mk_pk", 32 * n);
    h2d(ctx, dsk, sk.data(), 32 * n);
    dkgk::fixed_base(n, dsk, ctx->tab_gw, dpe, ctx->stream);  // to_public (procedure_keys.rs:78-82)
    dkgk::encode_points(dpe, n, n, dpc, ctx->stream);
    check_launch(ctx);
    d2h(ctx, pk.data(), dpc, 32 * n);
    sync(ctx);
    // committee.rs:134-135: ordered_pks.sort() by the byte order of procedure_keys.rs:26-40
    std::vector<size_t> order(n);
    for (size_t j = 0; j < n; j++) order[j] = j;
    std::sort(order.begin(), order.end(),
              [&](size_t a, size_t b) { return memcmp(&pk[32 * a], &pk[32 * b], 32) < 0; });
    for (size_t q = 0; q < n; q++) {
      memcpy(sk_out + 32 * q, &sk[32 * order[q]], 32);
      memcpy(pk_out + 32 * q, &pk[32 * order[q]], 32);
    }
    return DKG_OK;
  });
}

int dkg_enc_randomness(const uint8_t master[32], uint32_t ceremony, size_t d0, size_t D, size_t n, size_t t,
                       uint8_t* r) {
  if (!master || !r) return DKG_E_ARG;
  static const char tag[] = "dkg-amd/v1/dealer";
  std::vector<uint8_t> stream(2 * n * 64);
  for (size_t i = 0; i < D; i++) {
    uint8_t msg[sizeof tag - 1 + 40], seed[32];
    memcpy(msg, tag, sizeof tag - 1);
    memcpy(msg + sizeof tag - 1, master, 32);
    const uint32_t dealer = (uint32_t)(d0 + i);
    for (int k = 0; k < 4; k++) {
      msg[sizeof tag - 1 + 32 + k] = (uint8_t)(ceremony >> (8 * k));
      msg[sizeof tag - 1 + 36 + k] = (uint8_t)(dealer >> (8 * k));
    }
    dkgh::blake2b(seed, 32, msg, sizeof msg);
    dkgh::chacha20(seed, 2 * (t + 1), stream.data(), stream.size());  // after the 2(t+1) coefficients
    for (size_t q = 0; q < 2 * n; q++)
      dkgh::zl_to_bytes(r + 32 * (i * 2 * n + q), dkgh::zl_from_bytes_wide(&stream[64 * q], 64));
  }
  return DKG_OK;
}

int dkg_enc_randomness_device(dkg_ctx* ctx, const uint8_t master[32], uint32_t ceremony0, size_t B, size_t d0,
                              size_t D, size_t n, size_t t, void* d_r) {
  return guarded(ctx, [&] {
    if (!master || !d_r) return DKG_E_ARG;
    const size_t rows = B * D;
    if (!rows || !n) return DKG_OK;
    uint32_t* m = buf<uint32_t>(ctx, "sg_master", 32);
    uint32_t* seeds = buf<uint32_t>(ctx, "sg_seeds", 32 * rows);
    h2d(ctx, m, master, 32);
    dkgk::dealer_seeds(rows, D, d0, ceremony0, m, seeds, ctx->stream);
    dkgk::enc_randomness(rows, n, t + 1, seeds, (uint32_t*)d_r, ctx->stream);
    check_launch(ctx);
    sync(ctx);
    return DKG_OK;
  });
}

int dkg_encrypt_shares(dkg_ctx* ctx, size_t D, size_t n, const uint8_t* pk, const uint8_t* s, const uint8_t* s_prime,
                       const uint8_t* r, uint8_t* e1, uint8_t* ct) {
  return guarded(ctx, [&] {
    if (!pk || !s || !s_prime || !r || !e1 || !ct) return DKG_E_ARG;
    if (!D || !n) return DKG_OK;
    const size_t items = 2 * D * n;
    uint32_t* dpk = buf<uint32_t>(ctx, "hx_pk", 32 * n);
    h2d(ctx, dpk, pk, 32 * n);
    std::vector<uint8_t> ok(n);
    uint32_t* ds = upload_scalars(ctx, "hx_s", s, D * n);
    uint32_t* dsp = upload_scalars(ctx, "hx_sp", s_prime, D * n);
    uint32_t* dr = upload_scalars(ctx, "hx_r", r, items);
    uint32_t* de1 = buf<uint32_t>(ctx, "hx_e1", 32 * items);
    uint32_t* dct = buf<uint32_t>(ctx, "hx_ct", 32 * items);
    // the host keys: a repeated key set reuses its decoded points and combs (1.7 MB per key)
    encrypt_device(ctx, D, n, dpk, ds, dsp, dr, de1, dct, nullptr, pk);
    d2h(ctx, ok.data(), buf<uint8_t>(ctx, "hy.pk_ok", n), n);
    d2h(ctx, e1, de1, 32 * items);
    d2h(ctx, ct, dct, 32 * items);
    sync(ctx);
    for (auto v : ok)
      if (!v) {
        ctx->err = "encrypt_shares: a recipient public key does not decode";
        return DKG_E_DECODE;
      }
    return DKG_OK;
  });
}

int dkg_decrypt_shares(dkg_ctx* ctx, size_t D, size_t n, const uint8_t* sk, const uint8_t* e1, const uint8_t* ct,
                       uint8_t* s, uint8_t* s_prime, uint8_t* ok) {
  return guarded(ctx, [&] {
    if (!sk || !e1 || !ct || !s || !s_prime) return DKG_E_ARG;
    if (!D || !n) return DKG_OK;
    const size_t items = 2 * D * n;
    uint32_t* dsk = upload_scalars(ctx, "hx_sk", sk, n);
    uint32_t* de1 = buf<uint32_t>(ctx, "hx_e1", 32 * items);
    uint32_t* dct = buf<uint32_t>(ctx, "hx_ct", 32 * items);
    h2d(ctx, de1, e1, 32 * items);
    h2d(ctx, dct, ct, 32 * items);
    uint32_t* ds = buf<uint32_t>(ctx, "hx_s", 32 * D * n);
    uint32_t* dsp = buf<uint32_t>(ctx, "hx_sp", 32 * D * n);
    uint8_t* iok = buf<uint8_t>(ctx, "hx_ok", items);
    decrypt_device(ctx, D, n, dsk, de1, dct, ds, dsp, iok, nullptr);
    d2h(ctx, s, ds, 32 * D * n);
    d2h(ctx, s_prime, dsp, 32 * D * n);
    if (ok) d2h(ctx, ok, iok, items);
    sync(ctx);
    return DKG_OK;
  });
}

// Full-mode ceremony: round 1 with the shares hybrid-encrypted to the sorted member keys, the
// receivers decrypting them in round 2 (timed inside ms_round1 / ms_round2), then rounds 2-5 on
// the decrypted shares exactly as in plaintext mode.
int dkg_ceremony_run_full_device(dkg_ctx* ctx, size_t n, size_t t, const void* d_a, const void* d_b, const void* d_r,
                                 const uint8_t* sk, const uint8_t* pk, dkg_ceremony_out* out) {
  return guarded(ctx, [&] {
    int rc = need_env(ctx);
    if (rc) return rc;
    if (dkg_env_check(t, n) != DKG_OK || !out || !sk || !pk || !d_r) return DKG_E_ARG;
    const size_t N = t + 1, items = 2 * n * n;
    uint32_t* dsk = upload_scalars(ctx, "fm_sk", sk, n);
    uint32_t* dpk = buf<uint32_t>(ctx, "fm_pk", 32 * n);
    h2d(ctx, dpk, pk, 32 * n);
    HCK(hipEventRecord(ctx->ev[0], ctx->stream));
    uint32_t* Ec = buf<uint32_t>(ctx, "cer_E", 32 * n * N);
    uint32_t* Ac = buf<uint32_t>(ctx, "cer_A", 32 * n * N);
    uint32_t* ds = buf<uint32_t>(ctx, "cer_s", 32 * n * n);
    uint32_t* dsp = buf<uint32_t>(ctx, "cer_sp", 32 * n * n);
    // With chunk streams (not the serialised roofline pass) the share evaluation, the encryption and
    // the receivers' decryption run on the low-priority side stream beside the check pipeline:
    // nothing before the checks reads a share, so the pipeline's binomial, stepping and
    // recombination start on the commitments alone, and the checks (and round 3) wait for the
    // decrypted shares (wait_shares); the decode mask of the ciphertexts joins the dealer mask there.
    const bool side = ctx->nsub > 1 && ctx->verify_mode == 0;
    hipStream_t hy = side ? ctx->side : ctx->stream;
    round1_device(ctx, n, n, t, (const uint32_t*)d_a, (const uint32_t*)d_b, Ec, Ac, ds, dsp, false, side);
    uint32_t* e1 = buf<uint32_t>(ctx, "fm_e1", 32 * items);
    uint32_t* ct = buf<uint32_t>(ctx, "fm_ct", 32 * items);
    encrypt_device(ctx, n, n, dpk, ds, dsp, (const uint32_t*)d_r, e1, ct, hy, pk);  // committee.rs:169-172
    HCK(hipEventRecord(ctx->ev[1], ctx->stream));
    uint32_t* rs = buf<uint32_t>(ctx, "fm_s", 32 * n * n);
    uint32_t* rsp = buf<uint32_t>(ctx, "fm_sp", 32 * n * n);
    uint8_t* iok = buf<uint8_t>(ctx, "fm_iok", items);
    uint8_t* eok = buf<uint8_t>(ctx, "fm_eok", n);
    decrypt_device(ctx, n, n, dsk, e1, ct, rs, rsp, iok, eok, hy);  // committee.rs:282-286
    if (side) {
      HCK(hipEventRecord(ctx->shares_done, ctx->side));
      ctx->shares_pending = true;
    }
    ExtScope ext(ctx, n, N);
    receivers_rounds(ctx, n, t, Ec, Ac, rs, rsp, out, false, eok);
    collect_hybrid_phases(ctx);
    out->ms_round1 = ev_ms(ctx, 0, 1);
    out->ms_round2 = ev_ms(ctx, 1, 2);
    out->ms_round3 = ev_ms(ctx, 2, 3);
    out->ms_round4 = ev_ms(ctx, 3, 4);
    out->ms_finalise = ev_ms(ctx, 4, 5);
    out->ms_total = ev_ms(ctx, 0, 5);
    return DKG_OK;
  });
}

int dkg_ceremony_verify_full(dkg_ctx* ctx, size_t n, size_t t, const uint8_t* E, const uint8_t* A, const uint8_t* e1,
                             const uint8_t* ct, const uint8_t* sk, dkg_ceremony_out* out) {
  return guarded(ctx, [&] {
    int rc = need_env(ctx);
    if (rc) return rc;
    if (dkg_env_check(t, n) != DKG_OK || !out || !E || !A || !e1 || !ct || !sk) return DKG_E_ARG;
    const size_t N = t + 1, items = 2 * n * n;
    uint32_t* Ec = buf<uint32_t>(ctx, "cer_E", 32 * n * N);
    uint32_t* Ac = buf<uint32_t>(ctx, "cer_A", 32 * n * N);
    h2d(ctx, Ec, E, 32 * n * N);
    h2d(ctx, Ac, A, 32 * n * N);
    uint32_t* dsk = upload_scalars(ctx, "fm_sk", sk, n);
    uint32_t* de1 = buf<uint32_t>(ctx, "fm_e1", 32 * items);
    uint32_t* dct = buf<uint32_t>(ctx, "fm_ct", 32 * items);
    h2d(ctx, de1, e1, 32 * items);
    h2d(ctx, dct, ct, 32 * items);
    HCK(hipEventRecord(ctx->ev[0], ctx->stream));
    HCK(hipEventRecord(ctx->ev[1], ctx->stream));
    uint32_t* rs = buf<uint32_t>(ctx, "fm_s", 32 * n * n);
    uint32_t* rsp = buf<uint32_t>(ctx, "fm_sp", 32 * n * n);
    uint8_t* iok = buf<uint8_t>(ctx, "fm_iok", items);
    uint8_t* eok = buf<uint8_t>(ctx, "fm_eok", n);
    // the decryption on the side stream beside the check pipeline, as in dkg_ceremony_run_full_device
    const bool side = ctx->nsub > 1 && ctx->verify_mode == 0;
    if (side) {
      HCK(hipEventRecord(ctx->side_fork, ctx->stream));
      HCK(hipStreamWaitEvent(ctx->side, ctx->side_fork, 0));
    }
    decrypt_device(ctx, n, n, dsk, de1, dct, rs, rsp, iok, eok, side ? ctx->side : ctx->stream);
    if (side) {
      HCK(hipEventRecord(ctx->shares_done, ctx->side));
      ctx->shares_pending = true;
    }
    receivers_rounds(ctx, n, t, Ec, Ac, rs, rsp, out, true, eok);  // waits for the shares before it returns
    collect_hybrid_phases(ctx);  // decryption phases only (no encryption here: full.enc_* read -1)
    if (out->s) d2h(ctx, out->s, rs, 32 * n * n);
    if (out->s_prime) d2h(ctx, out->s_prime, rsp, 32 * n * n);
    sync(ctx);
    out->ms_round1 = 0;
    out->ms_round2 = ev_ms(ctx, 1, 2);
    out->ms_round3 = ev_ms(ctx, 2, 3);
    out->ms_round4 = ev_ms(ctx, 3, 4);
    out->ms_finalise = ev_ms(ctx, 4, 5);
    out->ms_total = ev_ms(ctx, 0, 5);
    return DKG_OK;
  });
}

int dkg_misbehaviour_prove(dkg_ctx* ctx, size_t B, const uint8_t* sk, const uint8_t* enc, const uint8_t* w,
                           uint8_t* proofs) {
  return guarded(ctx, [&] {
    if (!sk || !enc || !w || !proofs) return DKG_E_ARG;
    if (!B) return DKG_OK;
    // per complaint 7 single-term products: K_share, K_rand, pk, and the two DLEQ announcements
    std::vector<uint8_t> sc, pt, out(32 * 7 * B);
    for (size_t b = 0; b < B; b++) {
      const uint8_t *e1r = enc + 128 * b, *e1s = e1r + 64, *x = sk + 32 * b, *w1 = w + 64 * b, *w2 = w1 + 32;
      const uint8_t* P[7] = {e1s, e1r, BASEPOINT, BASEPOINT, e1s, BASEPOINT, e1r};
      const uint8_t* S[7] = {x, x, x, w1, w1, w2, w2};
      for (int k = 0; k < 7; k++) {
        put32(pt, P[k]);
        put32(sc, S[k]);
      }
    }
    std::vector<uint8_t> ok;
    msm_host(ctx, 7 * B, 1, sc.data(), pt.data(), out.data(), ok);
    for (size_t b = 0; b < B; b++) {
      for (int k = 0; k < 7; k++)
        if (!ok[7 * b + k]) {
          ctx->err = "misbehaviour_prove: a ciphertext point does not decode";
          return DKG_E_DECODE;
        }
      const uint8_t *o = &out[32 * 7 * b], *e1r = enc + 128 * b, *e1s = e1r + 64;
      const uint8_t *Ks = o, *Kr = o + 32, *pk = o + 64;
      uint8_t* p = proofs + 192 * b;
      memcpy(p, Ks, 32);       // share_key      (broadcast.rs:197-199, recover_symmetric_key)
      memcpy(p + 32, Kr, 32);  // randomness_key (:200-202)
      const dkgh::Zl x = zl32(sk + 32 * b);
      // CorrectHybridDecrKeyZkp = DLEQ(g, e1, pk, K; sk) (correct_hybrid_decryption_key/zkp.rs:27-47)
      dkgh::Zl c1 = dleq_challenge(BASEPOINT, e1s, pk, Ks, o + 96, o + 128);
      dkgh::Zl r1 = dkgh::zl_add(dkgh::zl_mul(c1, x), zl32(w + 64 * b));
      dkgh::Zl c2 = dleq_challenge(BASEPOINT, e1r, pk, Kr, o + 160, o + 192);
      dkgh::Zl r2 = dkgh::zl_add(dkgh::zl_mul(c2, x), zl32(w + 64 * b + 32));
      dkgh::zl_to_bytes(p + 64, c1);
      dkgh::zl_to_bytes(p + 96, r1);
      dkgh::zl_to_bytes(p + 128, c2);
      dkgh::zl_to_bytes(p + 160, r2);
    }
    return DKG_OK;
  });
}

int dkg_complaint1_verify(dkg_ctx* ctx, size_t B, size_t t, const uint32_t* accuser, const uint8_t* pk,
                          const uint8_t* enc, const uint8_t* E, const uint8_t* proofs, int32_t* result) {
  return guarded(ctx, [&] {
    int rc = need_env(ctx);
    if (rc) return rc;
    if (!accuser || !pk || !enc || !E || !proofs || !result) return DKG_E_ARG;
    if (!B) return DKG_OK;
    const size_t N = t + 1;
    // phase A, 6 two-term MSMs per complaint: both DLEQ announcements of both proofs
    // (dl_equality/zkp.rs:60-63) and the two h/g combinations of the decrypted scalars
    std::vector<uint8_t> sc, pt, outA(32 * 6 * B), sb, pb, outB(32 * B);
    for (size_t b = 0; b < B; b++) {
      const uint8_t *e1r = enc + 128 * b, *ctr = e1r + 32, *e1s = e1r + 64, *cts = e1r + 96;
      const uint8_t *P = proofs + 192 * b, *Ks = P, *Kr = P + 32, *pkb = pk + 32 * b;
      const dkgh::Zl zero = dkgh::zl_from_u64(0);
      const dkgh::Zl nc1 = dkgh::zl_sub(zero, zl32(P + 64)), nc2 = dkgh::zl_sub(zero, zl32(P + 128));
      const dkgh::Zl p1 = sym_scalar(Ks, cts), p2 = sym_scalar(Kr, ctr);  // share, randomness
      put32(sc, P + 96); putzl(sc, nc1); put32(pt, BASEPOINT); put32(pt, pkb);   // a1 = g r1 - pk c1
      put32(sc, P + 96); putzl(sc, nc1); put32(pt, e1s); put32(pt, Ks);          // a2 = e1 r1 - K c1
      put32(sc, P + 160); putzl(sc, nc2); put32(pt, BASEPOINT); put32(pt, pkb);
      put32(sc, P + 160); putzl(sc, nc2); put32(pt, e1r); put32(pt, Kr);
      putzl(sc, p1); putzl(sc, p2); put32(pt, ctx->h); put32(pt, BASEPOINT);  // quirk: h*share + g*rand
      putzl(sc, p2); putzl(sc, p1); put32(pt, ctx->h); put32(pt, BASEPOINT);  // accusation: h*rand + g*share
      std::vector<uint8_t> pw = index_powers(accuser[b], N);
      sb.insert(sb.end(), pw.begin(), pw.end());
      pb.insert(pb.end(), E + 32 * N * b, E + 32 * N * (b + 1));
    }
    std::vector<uint8_t> okA, okB;
    msm_host(ctx, 6 * B, 2, sc.data(), pt.data(), outA.data(), okA);
    msm_host(ctx, B, N, sb.data(), pb.data(), outB.data(), okB);  // sum_k j^k E_k
    for (size_t b = 0; b < B; b++) {
      bool ok = okB[b];
      for (int k = 0; k < 6; k++) ok = ok && okA[6 * b + k];
      if (!ok) {
        result[b] = -1;
        continue;
      }
      const uint8_t *e1r = enc + 128 * b, *e1s = e1r + 64, *P = proofs + 192 * b, *o = &outA[32 * 6 * b];
      uint8_t c[32];
      dkgh::zl_to_bytes(c, dleq_challenge(BASEPOINT, e1s, pk + 32 * b, P, o, o + 32));
      const bool v1 = memcmp(c, P + 64, 32) == 0;
      dkgh::zl_to_bytes(c, dleq_challenge(BASEPOINT, e1r, pk + 32 * b, P + 32, o + 64, o + 96));
      const bool v2 = memcmp(c, P + 128, 32) == 0;
      const uint8_t* rhs = &outB[32 * b];
      if (!v1 || !v2) result[b] = 1;                            // InvalidProofOfMisbehaviour
      else if (memcmp(o + 128, rhs, 32) == 0) result[b] = 1;   // ProofOfMisbehaviour::verify quirk (:271-283)
      else if (memcmp(o + 160, rhs, 32) == 0) result[b] = 2;   // FalseClaimedInequality (broadcast.rs:94-96)
      else result[b] = 0;
    }
    return DKG_OK;
  });
}

int dkg_complaint3_verify(dkg_ctx* ctx, size_t B, size_t t, const uint32_t* accuser, const uint8_t* share,
                          const uint8_t* randomness, const uint8_t* E, const uint8_t* A, int32_t* result) {
  return guarded(ctx, [&] {
    int rc = need_env(ctx);
    if (rc) return rc;
    if (!accuser || !share || !randomness || !E || !A || !result) return DKG_E_ARG;
    if (!B) return DKG_OK;
    const size_t N = t + 1;
    std::vector<uint8_t> sc, pt, outA(32 * 2 * B), sb, pb, outB(32 * 2 * B);
    const uint8_t zero[32] = {0};
    for (size_t b = 0; b < B; b++) {
      put32(sc, share + 32 * b); put32(sc, randomness + 32 * b); put32(pt, BASEPOINT); put32(pt, ctx->h);
      put32(sc, share + 32 * b); put32(sc, zero); put32(pt, BASEPOINT); put32(pt, BASEPOINT);
      std::vector<uint8_t> pw = index_powers(accuser[b], N);
      for (int r = 0; r < 2; r++) {
        sb.insert(sb.end(), pw.begin(), pw.end());
        const uint8_t* C = r == 0 ? E : A;
        pb.insert(pb.end(), C + 32 * N * b, C + 32 * N * (b + 1));
      }
    }
    std::vector<uint8_t> okA, okB;
    msm_host(ctx, 2 * B, 2, sc.data(), pt.data(), outA.data(), okA);
    msm_host(ctx, 2 * B, N, sb.data(), pb.data(), outB.data(), okB);
    for (size_t b = 0; b < B; b++) {
      if (!(okA[2 * b] && okA[2 * b + 1] && okB[2 * b] && okB[2 * b + 1])) {
        result[b] = -1;
        continue;
      }
      const uint8_t *pass = &outA[64 * b], *fail = pass + 32, *rE = &outB[64 * b], *rA = rE + 32;
      if (memcmp(pass, rE, 32) != 0) result[b] = 3;       // FalseClaimedEquality (broadcast.rs:129-130)
      else if (memcmp(fail, rA, 32) == 0) result[b] = 2;  // FalseClaimedInequality (:131-132)
      else result[b] = 0;
    }
    return DKG_OK;
  });
}

int dkg_dealer_coeffs(const uint8_t master[32], uint32_t ceremony, size_t d0, size_t D, size_t t, uint8_t* a,
                      uint8_t* b) {
  if (!master || (!a && !b)) return DKG_E_ARG;
  const size_t N = t + 1;
  static const char tag[] = "dkg-amd/v1/dealer";
  std::vector<uint8_t> stream(2 * N * 64);
  for (size_t i = 0; i < D; i++) {
    uint8_t msg[sizeof tag - 1 + 40];
    memcpy(msg, tag, sizeof tag - 1);
    memcpy(msg + sizeof tag - 1, master, 32);
    const uint32_t dealer = (uint32_t)(d0 + i);
    for (int k = 0; k < 4; k++) {
      msg[sizeof tag - 1 + 32 + k] = (uint8_t)(ceremony >> (8 * k));
      msg[sizeof tag - 1 + 36 + k] = (uint8_t)(dealer >> (8 * k));
    }
    uint8_t seed[32];
    dkgh::blake2b(seed, 32, msg, sizeof msg);
    dkgh::chacha20(seed, 0, stream.data(), stream.size());
    for (size_t k = 0; k < N; k++) {  // hiding polynomial first (committee.rs:143-146)
      if (b) dkgh::zl_to_bytes(b + 32 * (i * N + k), dkgh::zl_from_bytes_wide(&stream[64 * k], 64));
      if (a) dkgh::zl_to_bytes(a + 32 * (i * N + k), dkgh::zl_from_bytes_wide(&stream[64 * (N + k)], 64));
    }
  }
  return DKG_OK;
}

}  // extern "C"
