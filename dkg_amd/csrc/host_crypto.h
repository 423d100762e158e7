// Host-side helpers of the product library (not the oracle): BLAKE2b-512 for the commitment key
// (commitment.rs:13-17), the ChaCha20Rng stream for seeded synthetic coefficients, and small
// Z_l arithmetic for the (cold) reconstruction path of finalise (polynomial.rs:162-184).
#pragma once
#include <stddef.h>
#include <stdint.h>

namespace dkgh {

void blake2b(uint8_t* out, size_t outlen, const uint8_t* in, size_t inlen);
// ChaCha20 keystream (key = seed, 64-bit block counter from `block`, zero stream id)
void chacha20(const uint8_t key[32], uint64_t block, uint8_t* out, size_t len);
// RFC 8439 ChaCha20 (96-bit nonce, 32-bit counter from 0) XOR -- chacha20 0.7 `ChaCha20`, used by
// SymmetricKey::process (elgamal.rs:172-193) on the (cold) complaint-proof path
void chacha20_ietf_xor(uint8_t* out, const uint8_t* in, size_t len, const uint8_t key[32], const uint8_t nonce[12]);

struct Zl {  // canonical element of Z_l, little-endian 64-bit limbs
  uint64_t w[4];
};
Zl zl_from_bytes_wide(const uint8_t* in, size_t len);  // any length, big-endian fold of LE bytes
Zl zl_from_u64(uint64_t x);
void zl_to_bytes(uint8_t out[32], const Zl& a);
Zl zl_add(const Zl& a, const Zl& b);
Zl zl_sub(const Zl& a, const Zl& b);
Zl zl_mul(const Zl& a, const Zl& b);
Zl zl_inv(const Zl& a);
bool zl_is_zero(const Zl& a);

// lattice.cpp: a short (b, a_1, .., a_{K-1}) with a_u = b y^u (mod l), b > 0, 2 <= K <= 5, as
// magnitudes (32 bytes LE) and signs; (1, y, .., y^(K-1)) when no shorter row checks out.
bool short_multipliers(const Zl& y, int K, uint8_t (*mag)[32], int8_t* sign);

}  // namespace dkgh
