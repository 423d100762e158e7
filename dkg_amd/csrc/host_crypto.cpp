// Host-side helpers of the product library; see host_crypto.h.
#include "host_crypto.h"

#include <string.h>

namespace dkgh {

namespace {
constexpr uint64_t IV[8] = {0x6a09e667f3bcc908ULL, 0xbb67ae8584caa73bULL, 0x3c6ef372fe94f82bULL,
                            0xa54ff53a5f1d36f1ULL, 0x510e527fade682d1ULL, 0x9b05688c2b3e6c1fULL,
                            0x1f83d9abfb41bd6bULL, 0x5be0cd19137e2179ULL};
constexpr uint8_t SIGMA[10][16] = {
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
    {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4}, {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
    {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13}, {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
    {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11}, {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
    {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5}, {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0}};

inline uint64_t rotr(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }
inline uint64_t ld64(const uint8_t* p) {
  uint64_t v = 0;
  for (int i = 7; i >= 0; i--) v = (v << 8) | p[i];
  return v;
}

struct B2 {
  uint64_t h[8];
  uint64_t t = 0;
  void compress(const uint8_t* blk, bool last) {
    uint64_t m[16], v[16];
    for (int i = 0; i < 16; i++) m[i] = ld64(blk + 8 * i);
    for (int i = 0; i < 8; i++) v[i] = h[i], v[8 + i] = IV[i];
    v[12] ^= t;
    if (last) v[14] = ~v[14];
    auto G = [&](int a, int b, int c, int d, uint64_t x, uint64_t y) {
      v[a] += v[b] + x; v[d] = rotr(v[d] ^ v[a], 32);
      v[c] += v[d];     v[b] = rotr(v[b] ^ v[c], 24);
      v[a] += v[b] + y; v[d] = rotr(v[d] ^ v[a], 16);
      v[c] += v[d];     v[b] = rotr(v[b] ^ v[c], 63);
    };
    for (int r = 0; r < 12; r++) {
      const uint8_t* s = SIGMA[r % 10];
      G(0, 4, 8, 12, m[s[0]], m[s[1]]);
      G(1, 5, 9, 13, m[s[2]], m[s[3]]);
      G(2, 6, 10, 14, m[s[4]], m[s[5]]);
      G(3, 7, 11, 15, m[s[6]], m[s[7]]);
      G(0, 5, 10, 15, m[s[8]], m[s[9]]);
      G(1, 6, 11, 12, m[s[10]], m[s[11]]);
      G(2, 7, 8, 13, m[s[12]], m[s[13]]);
      G(3, 4, 9, 14, m[s[14]], m[s[15]]);
    }
    for (int i = 0; i < 8; i++) h[i] ^= v[i] ^ v[8 + i];
  }
};
}  // namespace

void blake2b(uint8_t* out, size_t outlen, const uint8_t* in, size_t inlen) {
  B2 st;
  for (int i = 0; i < 8; i++) st.h[i] = IV[i];
  st.h[0] ^= 0x01010000ULL ^ outlen;
  while (inlen > 128) {
    st.t += 128;
    st.compress(in, false);
    in += 128;
    inlen -= 128;
  }
  uint8_t blk[128] = {0};
  memcpy(blk, in, inlen);
  st.t += inlen;
  st.compress(blk, true);
  for (size_t i = 0; i < outlen; i++) out[i] = (uint8_t)(st.h[i / 8] >> (8 * (i % 8)));
}

void chacha20(const uint8_t key[32], uint64_t block, uint8_t* out, size_t len) {
  uint32_t k[8];
  for (int i = 0; i < 8; i++) k[i] = (uint32_t)key[4 * i] | (uint32_t)key[4 * i + 1] << 8 |
                                     (uint32_t)key[4 * i + 2] << 16 | (uint32_t)key[4 * i + 3] << 24;
  auto rotl = [](uint32_t x, int n) { return (x << n) | (x >> (32 - n)); };
  while (len) {
    uint32_t s[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u, k[0], k[1], k[2], k[3],
                      k[4], k[5], k[6], k[7], (uint32_t)block, (uint32_t)(block >> 32), 0, 0};
    uint32_t x[16];
    memcpy(x, s, sizeof s);
    auto QR = [&](int a, int b, int c, int d) {
      x[a] += x[b]; x[d] = rotl(x[d] ^ x[a], 16);
      x[c] += x[d]; x[b] = rotl(x[b] ^ x[c], 12);
      x[a] += x[b]; x[d] = rotl(x[d] ^ x[a], 8);
      x[c] += x[d]; x[b] = rotl(x[b] ^ x[c], 7);
    };
    for (int r = 0; r < 10; r++) {
      QR(0, 4, 8, 12); QR(1, 5, 9, 13); QR(2, 6, 10, 14); QR(3, 7, 11, 15);
      QR(0, 5, 10, 15); QR(1, 6, 11, 12); QR(2, 7, 8, 13); QR(3, 4, 9, 14);
    }
    uint8_t blk[64];
    for (int i = 0; i < 16; i++) {
      uint32_t v = x[i] + s[i];
      for (int b = 0; b < 4; b++) blk[4 * i + b] = (uint8_t)(v >> (8 * b));
    }
    size_t n = len < 64 ? len : 64;
    memcpy(out, blk, n);
    out += n;
    len -= n;
    block++;
  }
}

void chacha20_ietf_xor(uint8_t* out, const uint8_t* in, size_t len, const uint8_t key[32], const uint8_t nonce[12]) {
  auto rd = [](const uint8_t* p) {
    return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24;
  };
  auto rotl = [](uint32_t x, int n) { return (x << n) | (x >> (32 - n)); };
  uint32_t counter = 0;
  while (len) {
    uint32_t s[16] = {0x61707865u, 0x3320646eu, 0x79622d32u, 0x6b206574u};
    for (int i = 0; i < 8; i++) s[4 + i] = rd(key + 4 * i);
    s[12] = counter++;
    for (int i = 0; i < 3; i++) s[13 + i] = rd(nonce + 4 * i);
    uint32_t x[16];
    memcpy(x, s, sizeof s);
    auto QR = [&](int a, int b, int c, int d) {
      x[a] += x[b]; x[d] = rotl(x[d] ^ x[a], 16);
      x[c] += x[d]; x[b] = rotl(x[b] ^ x[c], 12);
      x[a] += x[b]; x[d] = rotl(x[d] ^ x[a], 8);
      x[c] += x[d]; x[b] = rotl(x[b] ^ x[c], 7);
    };
    for (int r = 0; r < 10; r++) {
      QR(0, 4, 8, 12); QR(1, 5, 9, 13); QR(2, 6, 10, 14); QR(3, 7, 11, 15);
      QR(0, 5, 10, 15); QR(1, 6, 11, 12); QR(2, 7, 8, 13); QR(3, 4, 9, 14);
    }
    size_t n = len < 64 ? len : 64;
    for (size_t i = 0; i < n; i++) out[i] = in[i] ^ (uint8_t)((x[i / 4] + s[i / 4]) >> (8 * (i % 4)));
    out += n;
    in += n;
    len -= n;
  }
}

// ---- Z_l: fold 32 bits at a time from the top with 2^252 = -delta (mod l) ----
namespace {
typedef unsigned __int128 u128;
constexpr uint64_t Lw[4] = {0x5812631a5cf5d3edULL, 0x14def9dea2f79cd6ULL, 0ULL, 0x1000000000000000ULL};
constexpr uint64_t DELTA[2] = {0x5812631a5cf5d3edULL, 0x14def9dea2f79cd6ULL};

bool ge_l(const uint64_t a[4]) {
  for (int i = 3; i >= 0; i--) {
    if (a[i] > Lw[i]) return true;
    if (a[i] < Lw[i]) return false;
  }
  return true;
}
void sub_l(uint64_t a[4]) {
  u128 b = 0;
  for (int i = 0; i < 4; i++) {
    u128 d = (u128)a[i] - Lw[i] - b;
    a[i] = (uint64_t)d;
    b = (d >> 64) & 1;
  }
}
// acc (< l) <- (acc * 2^32 + chunk) mod l
void fold32(uint64_t acc[4], uint32_t chunk) {
  uint64_t x[5];
  x[4] = acc[3] >> 32;
  for (int i = 3; i > 0; i--) x[i] = (acc[i] << 32) | (acc[i - 1] >> 32);
  x[0] = (acc[0] << 32) | chunk;
  // x < 2^285: q = x >> 252, lo = x mod 2^252
  uint64_t q = (x[3] >> 60) | (x[4] << 4);
  uint64_t lo[4] = {x[0], x[1], x[2], x[3] & 0x0fffffffffffffffULL};
  // t = q * delta (< 2^158)
  u128 c = (u128)q * DELTA[0];
  uint64_t t0 = (uint64_t)c;
  c = (c >> 64) + (u128)q * DELTA[1];
  uint64_t t1 = (uint64_t)c, t2 = (uint64_t)(c >> 64);
  uint64_t tt[4] = {t0, t1, t2, 0};
  u128 b = 0;
  for (int i = 0; i < 4; i++) {
    u128 d = (u128)lo[i] - tt[i] - b;
    acc[i] = (uint64_t)d;
    b = (d >> 64) & 1;
  }
  if (b) {  // negative: add l once
    u128 cc = 0;
    for (int i = 0; i < 4; i++) {
      cc += (u128)acc[i] + Lw[i];
      acc[i] = (uint64_t)cc;
      cc >>= 64;
    }
  }
}
}  // namespace

Zl zl_from_bytes_wide(const uint8_t* in, size_t len) {
  Zl r{{0, 0, 0, 0}};
  size_t nchunks = (len + 3) / 4;
  for (size_t c = nchunks; c-- > 0;) {
    uint32_t v = 0;
    for (int b = 3; b >= 0; b--) {
      size_t idx = 4 * c + b;
      v = (v << 8) | (idx < len ? in[idx] : 0);
    }
    fold32(r.w, v);
  }
  return r;
}

Zl zl_from_u64(uint64_t x) {
  uint8_t b[8];
  for (int i = 0; i < 8; i++) b[i] = (uint8_t)(x >> (8 * i));
  return zl_from_bytes_wide(b, 8);
}

void zl_to_bytes(uint8_t out[32], const Zl& a) {
  for (int i = 0; i < 32; i++) out[i] = (uint8_t)(a.w[i / 8] >> (8 * (i % 8)));
}

Zl zl_add(const Zl& a, const Zl& b) {
  Zl r;
  u128 c = 0;
  for (int i = 0; i < 4; i++) {
    c += (u128)a.w[i] + b.w[i];
    r.w[i] = (uint64_t)c;
    c >>= 64;
  }
  if (ge_l(r.w)) sub_l(r.w);
  return r;
}

Zl zl_sub(const Zl& a, const Zl& b) {
  Zl r;
  u128 bb = 0;
  for (int i = 0; i < 4; i++) {
    u128 d = (u128)a.w[i] - b.w[i] - bb;
    r.w[i] = (uint64_t)d;
    bb = (d >> 64) & 1;
  }
  if (bb) {
    u128 c = 0;
    for (int i = 0; i < 4; i++) {
      c += (u128)r.w[i] + Lw[i];
      r.w[i] = (uint64_t)c;
      c >>= 64;
    }
  }
  return r;
}

Zl zl_mul(const Zl& a, const Zl& b) {
  uint64_t p[8] = {0};
  for (int i = 0; i < 4; i++) {
    u128 c = 0;
    for (int j = 0; j < 4; j++) {
      c += (u128)a.w[i] * b.w[j] + p[i + j];
      p[i + j] = (uint64_t)c;
      c >>= 64;
    }
    p[i + 4] = (uint64_t)c;
  }
  uint8_t bytes[64];
  for (int i = 0; i < 64; i++) bytes[i] = (uint8_t)(p[i / 8] >> (8 * (i % 8)));
  return zl_from_bytes_wide(bytes, 64);
}

Zl zl_inv(const Zl& a) {
  // a^(l-2)
  const uint64_t e[4] = {Lw[0] - 2, Lw[1], Lw[2], Lw[3]};
  Zl r = zl_from_u64(1);
  for (int i = 255; i >= 0; i--) {
    r = zl_mul(r, r);
    if ((e[i / 64] >> (i % 64)) & 1) r = zl_mul(r, a);
  }
  return r;
}

bool zl_is_zero(const Zl& a) { return (a.w[0] | a.w[1] | a.w[2] | a.w[3]) == 0; }

}  // namespace dkgh
