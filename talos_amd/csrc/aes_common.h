// aes_common.h — AES S-box / T-table constants generated at compile time and
// small device helpers shared by the HIP kernels.
//
// The tables are derived (GF(2^8) inverse via exp/log of generator 3 plus the
// FIPS-197 affine map) rather than transcribed, and stored in the
// little-endian column layout the kernels use: a state column is one uint32
// with row 0 in bits 0-7, so Te0_le[x] = {2S, S, S, 3S} (bytes 0..3) is the
// MixColumns image of row 0 (crypto/aes/aes_core.c:55-622 keeps the
// big-endian equivalents Te0..Te3).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace tg {

struct ByteTable { uint8_t v[256]; };
struct WordTable { uint32_t v[256]; };

constexpr uint8_t xtime8(uint8_t x) {
  return (uint8_t)((x << 1) ^ ((x & 0x80) ? 0x1b : 0));
}

constexpr ByteTable make_sbox() {
  uint8_t exp[256] = {}, log[256] = {};
  uint8_t p = 1;
  for (int i = 0; i < 255; i++) {
    exp[i] = p;
    log[p] = (uint8_t)i;
    p = (uint8_t)(p ^ xtime8(p));  // multiply by generator 3
  }
  ByteTable s{};
  for (int x = 0; x < 256; x++) {
    uint8_t inv = x ? exp[(255 - log[x]) % 255] : 0;
    uint8_t r = inv;
    for (int k = 1; k <= 4; k++) r ^= (uint8_t)((inv << k) | (inv >> (8 - k)));
    s.v[x] = (uint8_t)(r ^ 0x63);
  }
  return s;
}

constexpr ByteTable kSbox = make_sbox();

constexpr WordTable make_te0_le() {
  WordTable t{};
  for (int x = 0; x < 256; x++) {
    uint32_t s = kSbox.v[x], s2 = xtime8((uint8_t)s), s3 = s2 ^ s;
    t.v[x] = s2 | (s << 8) | (s << 16) | (s3 << 24);
  }
  return t;
}

constexpr WordTable kTe0 = make_te0_le();
static_assert(kSbox.v[0] == 0x63 && kSbox.v[0x53] == 0xed, "AES S-box");

__device__ __forceinline__ uint32_t rotl32(uint32_t x, int n) {
  return (x << n) | (x >> (32 - n));
}
__device__ __forceinline__ uint32_t bswap32(uint32_t x) {
  return __builtin_amdgcn_perm(x, x, 0x00010203u);
}

// XOR of v over the 64 lanes of the wave (every lane active), returned
// uniform.  DPP row shifts and row broadcasts instead of a 6-level
// __shfl_xor butterfly: the butterfly is 6 dependent ds_bpermute round trips
// through the LDS pipe per word, this is 7 VALU ops (gfx9 DPP: row_shr 1-3
// into a 4-lane window, row_shr 4 / 8 on the upper banks -> lane 15 of each
// row holds the row's XOR, row_bcast 15 / 31 -> lane 63 holds the total).
__device__ __forceinline__ uint32_t wave_xor_total(uint32_t v) {
  uint32_t a = v ^ (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, true);
  a ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, true);
  a ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x113, 0xf, 0xf, true);
  a ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)a, 0x114, 0xf, 0xe, false);
  a ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)a, 0x118, 0xf, 0xc, false);
  a ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)a, 0x142, 0xa, 0xf, false);
  a ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)a, 0x143, 0xc, 0xf, false);
  return (uint32_t)__builtin_amdgcn_readlane((int)a, 63);
}

// Inclusive scans over the 64 lanes (all active) with DPP instead of 6
// dependent __shfl_up (ds_bpermute) levels: row_shr 1 / 2 / 4 / 8 inside each
// 16-lane row, then row_bcast 15 (rows 1, 3 take lane 15 of the row before)
// and row_bcast 31 (rows 2, 3 take lane 31): 6 VALU ops (the scan LLVM's
// atomic optimizer builds for wave64 on gfx9).  Lanes without a source read 0
// (the identity of ^ and +).
__device__ __forceinline__ uint32_t wave_scan_xor(uint32_t v) {
  v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);
  v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);
  v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);
  v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);
  v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);
  v ^= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);
  return v;
}
__device__ __forceinline__ uint32_t wave_scan_add(uint32_t v) {
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, false);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, false);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, false);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, false);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);
  return v;
}

}  // namespace tg
