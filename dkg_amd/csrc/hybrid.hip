// Full (encrypted-share) mode on gfx950: the reference's hybrid ElGamal + ChaCha20 transport of the
// round-1 shares (committee.rs:164-172 encrypt, :282-286 decrypt; elgamal.rs:134-193,
// procedure_keys.rs:88-105).  Per (dealer i, recipient q) two ciphertexts: w = 0 carries the
// randomness s'_iq, w = 1 the share s_iq.
//   encrypt: e1 = g r, K = pk_q r, e2 = m XOR ChaCha20_IETF(key = B(K)[0..32], nonce = B(K)[32..44])
//   decrypt: K = sk_q e1, m = e2 XOR the same keystream, Scalar::from_bytes = from_bits
// with B = Blake2b-512 of K's 32-byte encoding.  The work is split into stages so that no kernel
// carries the register footprint of two different group algorithms:
//   enc_mul  : two fixed-base combs per item -- g (shared) and pk_q: the recipient's key is the same
//              for all n dealers, so it gets its own LDS-resident comb table (64 mixed additions,
//              no doublings) instead of a 253-doubling variable-base multiplication;
//   dec_mul  : sk_q * e1 with sk_q uniform across the wave (lanes = dealers of one recipient), a
//              branch-uniform width-4 window chain (k_dec_mul_w4; the plain NAF chain k_dec_mul
//              with -DDKG_DEC_NAF) with the addend staged in LDS;
//   encode / decode : the K5 kernels;  sym_xor : Blake2b + one ChaCha20 block + XOR (+ reduce).
#include "kernels.h"
#include "points.h"
#include "sym.h"

namespace dkgk {

// grid (ceil(2D / DKG_ENC_BS), n): recipient q = blockIdx.y.  The generator's comb (radix 2^DKG_COMBW_BITS)
// and the recipient's own comb (radix 2^DKG_KEY_COMB_BITS, 26 windows at 2^10: 1.7 MB per key, every
// dealer of the block reads the same table through L2; the radix-16 LDS comb it replaces took 64).
// 256-thread workgroups at 3 waves per SIMD: the two combs' mixed additions need ~138 VGPRs (the
// 1024-thread blocks capped it at 128 and spilled 32 B per lane)
#ifndef DKG_ENC_BS
#define DKG_ENC_BS 256
#endif
#ifndef DKG_ENC_IL  // paired result products in the combs' mixed additions (ge_madd IL; A/B knob)
#define DKG_ENC_IL 0
#endif
__global__ __launch_bounds__(DKG_ENC_BS, DKG_ENC_BS == 256 ? 3 : 1) void k_enc_mul(size_t D, size_t n, const uint32_t* __restrict__ r,
                                                  const uint32_t* __restrict__ tab_gw,
                                                  const uint32_t* __restrict__ tabs_pk, uint32_t* __restrict__ R_ext,
                                                  uint32_t* __restrict__ K_ext) {
  const size_t q = blockIdx.y;
  const uint32_t* tab_pk = tabs_pk + q * CombGeo<DKG_KEY_COMB_BITS>::WORDS;
  const size_t item = (size_t)blockIdx.x * blockDim.x + threadIdx.x;  // i * 2 + w
  if (item >= 2 * D) return;
  const size_t i = item >> 1, w = item & 1;
  const size_t idx = (i * n + q) * 2 + w;
  const size_t count = 2 * D * n;
  sc x;
  sc_load(x, r + 8 * idx);
  ge_p3 acc;
  ge_identity(acc);
  combw_mul_add<DKG_ENC_IL != 0>(acc, x, tab_gw);  // e1 = G::generator() * r  (elgamal.rs:141)
  pt_store(R_ext, count, idx, acc);
  ge_identity(acc);
  combw_mul_add_r<DKG_KEY_COMB_BITS, DKG_ENC_IL != 0>(acc, x, tab_pk);  // key = pk * r  (elgamal.rs:138-140)
  pt_store(K_ext, count, idx, acc);
}

void enc_mul(size_t D, size_t n, const uint32_t* r, const uint32_t* tab_gw, const uint32_t* tabs_pk, uint32_t* R_ext,
             uint32_t* K_ext, hipStream_t stream) {
  if (!D || !n) return;
  hipLaunchKernelGGL(k_enc_mul, dim3((unsigned)((2 * D + DKG_ENC_BS - 1) / DKG_ENC_BS), (unsigned)n), dim3(DKG_ENC_BS),
                     0, stream, D, n,
                     r, tab_gw, tabs_pk, R_ext, K_ext);
}

// grid (ceil(D / 64), n, 2): recipient q = blockIdx.y, w = blockIdx.z; lanes = dealers.
// K = sk_q * R: left-to-right NAF of the (wave-uniform) 253-bit scalar; R's cached form in LDS.
__global__ __launch_bounds__(64, 4) void k_dec_mul(size_t D, size_t n, const uint32_t* __restrict__ sk,
                                                   const uint32_t* __restrict__ R_ext, uint32_t* __restrict__ K_ext) {
  __shared__ uint32_t qs[PT_WORDS * 64];
  uint32_t* qcol = qs + threadIdx.x;
  const size_t q = blockIdx.y, w = blockIdx.z;
  const size_t i = (size_t)blockIdx.x * 64 + threadIdx.x;
  const bool live = i < D;
  const size_t count = 2 * D * n;
  const size_t idx = ((live ? i : 0) * n + q) * 2 + w;
  // NAF of sk_q (canonical, < 2^253), computed once per wave into LDS: digits[b] in {0, 1, -1};
  // reading a wave-uniform LDS byte per bit keeps the recoding out of the VGPR budget of the chain
  __shared__ int8_t digits[288];
  __shared__ int top_s;
  if (threadIdx.x == 0) {
    uint32_t k[9];
    for (int j = 0; j < 8; j++) k[j] = sk[8 * q + j];
    k[8] = 0;
    int top = -1;
    for (int b = 0; b < 287; b++) {
      int8_t d = 0;
      if ((k[b >> 5] >> (b & 31)) & 1u) {
        if ((k[(b + 1) >> 5] >> ((b + 1) & 31)) & 1u) {  // ...11: digit -1, k += 2^b (carry upwards)
          d = -1;
          uint32_t add = 1u << (b & 31);
          for (int wi = b >> 5; wi < 9; wi++) {
            const uint32_t old = k[wi];
            k[wi] = old + add;
            if (k[wi] >= old) break;
            add = 1u;
          }
        } else {  // ...01: digit +1, k -= 2^b
          d = 1;
          k[b >> 5] &= ~(1u << (b & 31));
        }
        top = b;
      }
      digits[b] = d;
    }
    top_s = top;
  }
  __syncthreads();
  const int top = __builtin_amdgcn_readfirstlane(top_s);
  ge_p3 x;
  if (live) pt_load(x, R_ext, count, idx);
  else ge_identity(x);
  if (top < 0) {  // sk = 0: K = identity
    ge_identity(x);
  } else {
    {
      ge_cached xc;
      ge_to_cached(xc, x);
      lds_put_cached(qcol, xc);
    }
    // leading digit is +1 (NAF top digit of a positive number); x already holds 1 * R
#pragma unroll 1
    for (int b = top - 1; b >= 0; b--) {
      const int d = __builtin_amdgcn_readfirstlane((int)digits[b]);
      ge_dbl_lean(x, x, d != 0 || b == 0);
      if (d != 0) ge_add_lds(x, x, qcol, d < 0, 64, b == 0);
    }
  }
  if (live) pt_store(K_ext, count, idx, x);
}

#ifndef DKG_DEC_NAF
// K = sk_q * R with a width-4 signed window (wNAF: digits 0, +-1, +-3, +-5, +-7, at least three zeros
// after each nonzero one: ~51 additions instead of NAF's ~85 for a 253-bit scalar).  Each lane's odd
// multiples R, 3R, 5R, 7R (cached form) live in a global table T laid out [wave][4][40 words][64
// lanes]; the addend of the next nonzero digit is copied into the wave's LDS slot by LDS-DMA
// (global_load_lds, no VGPRs) right after the previous addition, and lands during the >= 3 doublings
// in between.  LDS stays one point per wave.
// DKG_DEC_W4_WAVES: the launch bound's waves per SIMD; DKG_DEC_IL: paired products in the chain's
// doublings and additions (ge25519.h IL).  3 waves at <= 168 VGPRs with pairs (no scratch in the
// chain) against 4 at 128 without (24 VGPRs spilled in the table setup): full mode 111.6-111.7 against
// 112.8-113.0 ms per ceremony, k_dec_mul_w4 18.7-19.1 against 19.5-19.9 ms (profiles/r06_pair_ab.txt).
#ifndef DKG_DEC_W4_WAVES
#define DKG_DEC_W4_WAVES 3
#endif
#ifndef DKG_DEC_IL
#define DKG_DEC_IL 1
#endif
typedef __attribute__((address_space(3))) uint32_t dec_lds_u32;
typedef __attribute__((address_space(1))) uint32_t dec_g_u32;

// words 0..N-1 (64 lanes each) from sg into the LDS rows at q.  The instruction's immediate offset
// (K * 256 B) moves BOTH addresses -- the global one and the LDS one (M0 + offset + lane * 4) -- so
// the LDS base stays q for every word of the group.
template <int N, int K = 0>
DKG_DEV void glds_words(const dec_g_u32* sg, uint32_t* q) {
  if constexpr (K < N) {
    __builtin_amdgcn_global_load_lds(sg, (dec_lds_u32*)q, 4, K * 256, 0);
    glds_words<N, K + 1>(sg, q);
  }
}

__global__ __launch_bounds__(64, DKG_DEC_W4_WAVES) void k_dec_mul_w4(size_t D, size_t n, const uint32_t* __restrict__ sk,
                                                      const uint32_t* __restrict__ R_ext, uint32_t* __restrict__ K_ext,
                                                      uint32_t* __restrict__ T, size_t q0) {
  __shared__ uint32_t qs[PT_WORDS * 64];
  __shared__ int16_t nzb[96];  // bits of the nonzero digits, top first
  __shared__ int8_t nzd[96];   // their digits
  __shared__ int8_t dig[288];  // the recoding (LDS: a private array would live in scratch)
  __shared__ int nnz_s;
  uint32_t* qcol = qs + threadIdx.x;
  const size_t q = q0 + blockIdx.y, w = blockIdx.z;
  const size_t i = (size_t)blockIdx.x * 64 + threadIdx.x;
  const bool live = i < D;
  const size_t count = 2 * D * n;
  const size_t idx = ((live ? i : 0) * n + q) * 2 + w;
  const size_t wb = ((size_t)blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
  uint32_t* tb = T + wb * (4 * PT_WORDS * 64);
  if (threadIdx.x == 0) {
    uint32_t k[9];
    for (int j = 0; j < 8; j++) k[j] = sk[8 * q + j];
    k[8] = 0;
    for (int b = 0; b < 288; b++) {
      int8_t d = 0;
      if (k[0] & 1u) {
        int v = (int)(k[0] & 15u);
        if (v >= 8) v -= 16;
        d = (int8_t)v;
        if (v > 0) {  // k -= v
          uint32_t sub = (uint32_t)v;
          for (int wi = 0; wi < 9; wi++) {
            const uint32_t old = k[wi];
            k[wi] = old - sub;
            if (old >= sub) break;
            sub = 1u;
          }
        } else {      // k += -v
          uint32_t add = (uint32_t)(-v);
          for (int wi = 0; wi < 9; wi++) {
            const uint32_t old = k[wi];
            k[wi] = old + add;
            if (k[wi] >= old) break;
            add = 1u;
          }
        }
      }
      dig[b] = d;
      for (int wi = 0; wi < 8; wi++) k[wi] = (k[wi] >> 1) | (k[wi + 1] << 31);
      k[8] >>= 1;
    }
    int c = 0;
    for (int b = 287; b >= 0; b--)
      if (dig[b]) {
        nzb[c] = (int16_t)b;
        nzd[c] = dig[b];
        c++;
      }
    nnz_s = c;
  }
  // the lane's table of odd multiples
  ge_p3 x;
  if (live) pt_load(x, R_ext, count, idx);
  else ge_identity(x);
  {
    ge_cached c;
    ge_to_cached(c, x);
    lds_put_cached(tb + threadIdx.x, c);  // T[0] = R (global, lane-interleaved like the LDS slot)
    ge_p3 x2;
    ge_dbl<true>(x2, x);
    ge_to_cached(c, x2);
    lds_put_cached(qcol, c);              // 2R in the LDS slot
#pragma unroll 1
    for (int m = 1; m < 4; m++) {
      ge_add_lds(x, x, qcol, false);      // (2m+1) R
      ge_to_cached(c, x);
      lds_put_cached(tb + m * PT_WORDS * 64 + threadIdx.x, c);
    }
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");  // table stored, slot reads done
  __syncthreads();
  const int nnz = __builtin_amdgcn_readfirstlane(nnz_s);
  auto fetch = [&](int e) {  // addend of nonzero digit e into the LDS slot (LDS-DMA, one word per instr)
    const int a = (nzd[e] < 0 ? -nzd[e] : nzd[e]) >> 1;
    // one lane address per 16 words, the rest as the instruction's immediate offset (k * 256 B)
    const uint32_t* src = tb + a * PT_WORDS * 64 + threadIdx.x;
    glds_words<16>((const dec_g_u32*)src, qs);
    glds_words<16>((const dec_g_u32*)(src + 16 * 64), qs + 16 * 64);
    glds_words<8>((const dec_g_u32*)(src + 32 * 64), qs + 32 * 64);
  };
  ge_identity(x);
  if (nnz > 0) {
    fetch(0);
    int b = __builtin_amdgcn_readfirstlane((int)nzb[0]);
#pragma unroll 1
    for (int e = 0; e < nnz; e++) {
      const int be = __builtin_amdgcn_readfirstlane((int)nzb[e]);
      const int de = __builtin_amdgcn_readfirstlane((int)nzd[e]);
#pragma unroll 1
      for (; b > be; b--) ge_dbl_lean<DKG_DEC_IL != 0>(x, x, b - 1 == be);  // T only before the addition
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");     // the DMA'd addend has landed
      __builtin_amdgcn_s_barrier();
      ge_add_lds<DKG_DEC_IL != 0>(x, x, qcol, de < 0, 64, be == 0);  // a doubling follows unless be = 0
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the slot's reads are done
      if (e + 1 < nnz) fetch(e + 1);
    }
#pragma unroll 1
    for (; b > 0; b--) ge_dbl_lean<DKG_DEC_IL != 0>(x, x, b == 1);  // trailing zero digits
  }
  if (live) pt_store(K_ext, count, idx, x);
}
#endif

// The width-4 window's odd multiples live in a global table of one 40-KB slot per wave of a launch
// (T, indexed by the wave's place in its grid).  Launches are capped at DEC_TAB_WAVES waves -- eight
// rounds of a full chip's resident waves -- and cover the recipients in slices, back to back on the
// stream, so the table never exceeds DEC_TAB_WAVES slots (1.3 GB) whatever n is (n = 1024: one
// launch; n = 4096: 16 launches instead of one grid of 524,288 waves and a 21-GB table).  A cap of
// 16,384 (two launches at n = 1024) cost 0.8-1.0 ms there (profiles/r04_dec_slices_ab.txt).
#ifndef DKG_DEC_TAB_WAVES
#define DKG_DEC_TAB_WAVES 32768
#endif
constexpr size_t DEC_TAB_WAVES = DKG_DEC_TAB_WAVES;

size_t dec_mul_recipients_per_launch(size_t D, size_t n) {
  const size_t per_q = ((D + 63) / 64) * 2;
  return std::max<size_t>(1, std::min(n, DEC_TAB_WAVES / per_q));
}

void dec_mul(size_t D, size_t n, const uint32_t* sk, const uint32_t* R_ext, uint32_t* K_ext, hipStream_t stream,
             uint32_t* table) {
  if (!D || !n) return;
#ifndef DKG_DEC_NAF
  if (table) {
    const size_t qc = dec_mul_recipients_per_launch(D, n);
    for (size_t q0 = 0; q0 < n; q0 += qc)
      hipLaunchKernelGGL(k_dec_mul_w4, dim3((unsigned)((D + 63) / 64), (unsigned)std::min(qc, n - q0), 2u), dim3(64),
                         0, stream, D, n, sk, R_ext, K_ext, table, q0);
    return;
  }
#endif
  (void)table;
  hipLaunchKernelGGL(k_dec_mul, dim3((unsigned)((D + 63) / 64), (unsigned)n, 2u), dim3(64), 0, stream, D, n, sk,
                     R_ext, K_ext);
}

size_t dec_mul_table_words(size_t D, size_t n) {
#ifndef DKG_DEC_NAF
  return ((D + 63) / 64) * dec_mul_recipients_per_launch(D, n) * 2 * 4 * PT_WORDS * 64;
#else
  (void)D;
  (void)n;
  return 0;
#endif
}

// SymmetricKey::process (elgamal.rs:172-193) on 32-byte messages: one Blake2b-512 of the key's
// encoding, one ChaCha20 block (counter 0), XOR.
__global__ __launch_bounds__(256) void k_sym_xor(size_t D, size_t n, const uint32_t* __restrict__ Kc, int decrypt,
                                                 uint32_t* __restrict__ ct, uint32_t* __restrict__ s,
                                                 uint32_t* __restrict__ sp) {
  const size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= 2 * D * n) return;
  const size_t pair = idx >> 1, w = idx & 1;
  uint64_t m[16];
#pragma unroll
  for (int j = 0; j < 4; j++) m[j] = (uint64_t)Kc[8 * idx + 2 * j] | ((uint64_t)Kc[8 * idx + 2 * j + 1] << 32);
#pragma unroll
  for (int j = 4; j < 16; j++) m[j] = 0;
  uint64_t h[8];
  sym::blake2b_1block(h, m, 32, 64);
  uint32_t key[8], nonce[3];
#pragma unroll
  for (int j = 0; j < 4; j++) {
    key[2 * j] = (uint32_t)h[j];
    key[2 * j + 1] = (uint32_t)(h[j] >> 32);
  }
  nonce[0] = (uint32_t)h[4];
  nonce[1] = (uint32_t)(h[4] >> 32);
  nonce[2] = (uint32_t)h[5];
  uint32_t ks[16];
  sym::chacha20_ietf_block(ks, key, 0u, nonce);
  uint32_t* msg = w ? s + 8 * pair : sp + 8 * pair;
  if (!decrypt) {
#pragma unroll
    for (int j = 0; j < 8; j++) ct[8 * idx + j] = msg[j] ^ ks[j];
  } else {
    uint32_t v[8];
#pragma unroll
    for (int j = 0; j < 8; j++) v[j] = ct[8 * idx + j] ^ ks[j];
    v[7] &= 0x7fffffffu;  // Scalar::from_bytes = from_bits (groups.rs:29-36); reduced mod l on device
    sc r;
    sc_reduce256(r, v);
    st_words8(msg, r.v);
  }
}

void sym_xor(size_t D, size_t n, const uint32_t* Kc, bool decrypt, uint32_t* ct, uint32_t* s, uint32_t* sp,
             hipStream_t stream) {
  const size_t tot = 2 * D * n;
  if (!tot) return;
  hipLaunchKernelGGL(k_sym_xor, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, stream, D, n, Kc, decrypt ? 1 : 0,
                     ct, s, sp);
}

}  // namespace dkgk
