// bs_aes.h — bitsliced AES-CTR keystream on the VALU (gfx950).
//
// A lane holds 32 counter blocks as 128 bit planes: st[8*b + k] bit j = bit k
// (k = 0 is the LSB) of byte b of block j.  Every VALU op then works on 32
// blocks: SubBytes is the generated 85-node v_bitop3 circuit (bs_sbox.h, from
// the Boyar-Peralta circuit, verified on all 256 inputs), ShiftRows is register
// renaming, MixColumns is ~76 ops per column, AddRoundKey XORs wave-uniform
// masks (0 / ~0 per key bit, kept in SGPRs).  No LDS is touched, so this path
// runs beside the LDS-bound T-table/GHASH work.
//
// Equivalent to AES_encrypt (crypto/aes/aes_core.c:789-972) on each of the 32
// blocks; checked bit-exact against the T-table kernel and the oracle.
#pragma once
#include <stdint.h>

namespace tg {

// v_bitop3_b32: D bit = imm[(a<<2)|(b<<1)|c] (0xF0 = a, 0xCC = b, 0xAA = c).
#define bop3(a, b, c, imm)                                                            \
  ({                                                                                 \
    uint32_t _d;                                                                     \
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:" #imm : "=v"(_d) : "v"(a), "v"(b), "v"(c)); \
    _d;                                                                              \
  })

}  // namespace tg

#include "bs_sbox.h"

namespace tg {

typedef __attribute__((address_space(4))) const uint32_t bs_cu32;

// 16 S-boxes in place.
__device__ __forceinline__ void bs_subbytes(uint32_t (&st)[128]) {
#pragma unroll
  for (int b = 0; b < 16; b++) {
    uint32_t* p = st + 8 * b;
    uint32_t o7, o6, o5, o4, o3, o2, o1, o0;
    TG_BS_SBOX(p[7], p[6], p[5], p[4], p[3], p[2], p[1], p[0], o7, o6, o5, o4, o3, o2, o1, o0);
    p[7] = o7; p[6] = o6; p[5] = o5; p[4] = o4; p[3] = o3; p[2] = o2; p[1] = o1; p[0] = o0;
  }
}

// ShiftRows as a permutation of the byte slots: output byte (col c, row r) =
// input byte (col c + r, row r).  Applied by copying through a renamed array;
// with full unrolling the compiler only renames registers.
__device__ __forceinline__ void bs_shiftrows(uint32_t (&st)[128]) {
  uint32_t t[128];
#pragma unroll
  for (int c = 0; c < 4; c++)
#pragma unroll
    for (int r = 0; r < 4; r++)
#pragma unroll
      for (int k = 0; k < 8; k++) t[8 * (4 * c + r) + k] = st[8 * (4 * ((c + r) & 3) + r) + k];
#pragma unroll
  for (int i = 0; i < 128; i++) st[i] = t[i];
}

// MixColumns on one column (bytes a[0..3], 8 planes each) + AddRoundKey:
//   out_i = xtime(a_i ^ a_{i+1}) ^ a_{i+1} ^ (a_{i+2} ^ a_{i+3})
// xtime on planes: x[0]=t[7], x[1]=t[0]^t[7], x[2]=t[1], x[3]=t[2]^t[7],
// x[4]=t[3]^t[7], x[5]=t[4], x[6]=t[5], x[7]=t[6].
__device__ __forceinline__ void bs_mixcolumn(uint32_t* a0, uint32_t* a1, uint32_t* a2,
                                             uint32_t* a3, bs_cu32* km) {
  uint32_t* a[4] = {a0, a1, a2, a3};
  uint32_t t[4][8];
#pragma unroll
  for (int i = 0; i < 4; i++)
#pragma unroll
    for (int k = 0; k < 8; k++) t[i][k] = a[i][k] ^ a[(i + 1) & 3][k];
  uint32_t o[4][8];
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const uint32_t* ti = t[i];
    const uint32_t* t2 = t[(i + 2) & 3];
    const uint32_t* n = a[(i + 1) & 3];
#pragma unroll
    for (int k = 0; k < 8; k++) {
      uint32_t v;
      if (k == 1 || k == 3 || k == 4)
        v = bop3(bop3(ti[k - 1], ti[7], n[k], 0x96), t2[k], km[8 * i + k], 0x96);
      else
        v = bop3(k == 0 ? ti[7] : ti[k - 1], n[k], t2[k], 0x96) ^ km[8 * i + k];
      o[i][k] = v;
    }
  }
#pragma unroll
  for (int i = 0; i < 4; i++)
#pragma unroll
    for (int k = 0; k < 8; k++) a[i][k] = o[i][k];
}

__device__ __forceinline__ void bs_ark(uint32_t (&st)[128], bs_cu32* km) {
#pragma unroll
  for (int i = 0; i < 128; i++) st[i] ^= km[i];
}

// Full encryption of the 32 blocks in `st` with bitsliced round-key masks
// rkm[r*128 + 8*b + k] (0 or 0xFFFFFFFF).  The final AddRoundKey is left to
// the caller (it folds into the ciphertext XOR on normal-layout words) when
// skip_last_ark is set.
template <int ROUNDS, bool SKIP_LAST_ARK>
__device__ __forceinline__ void bs_encrypt(uint32_t (&st)[128], bs_cu32* rkm) {
  bs_ark(st, rkm);
#pragma unroll 1
  for (int r = 1; r < ROUNDS; r++) {
    bs_subbytes(st);
    bs_shiftrows(st);
#pragma unroll
    for (int c = 0; c < 4; c++)
      bs_mixcolumn(st + 32 * c, st + 32 * c + 8, st + 32 * c + 16, st + 32 * c + 24,
                   rkm + 128 * r + 32 * c);
  }
  bs_subbytes(st);
  bs_shiftrows(st);
  if (!SKIP_LAST_ARK) bs_ark(st, rkm + 128 * ROUNDS);
}

// 32x32 bit transpose of x[0..31] in place (x[i] bit j <-> x[j] bit i).
// Stages 16 and 8 are byte moves (v_perm_b32), stages 4/2/1 swap-moves.
__device__ __forceinline__ void transpose32(uint32_t* x) {
  // stage 16: swap the high half of x[i] with the low half of x[i+16]
#pragma unroll
  for (int i = 0; i < 16; i++) {
    uint32_t a = x[i], b = x[i + 16];
    x[i] = __builtin_amdgcn_perm(b, a, 0x05040100u);       // [a.lo16, b.lo16]
    x[i + 16] = __builtin_amdgcn_perm(b, a, 0x07060302u);  // [a.hi16, b.hi16]
  }
  // stage 8
#pragma unroll
  for (int g = 0; g < 32; g += 16)
#pragma unroll
    for (int i = 0; i < 8; i++) {
      uint32_t a = x[g + i], b = x[g + i + 8];
      x[g + i] = __builtin_amdgcn_perm(b, a, 0x06020400u);      // [a0, b0, a2, b2]
      x[g + i + 8] = __builtin_amdgcn_perm(b, a, 0x07030501u);  // [a1, b1, a3, b3]
    }
  // stages 4, 2, 1
#pragma unroll
  for (int s = 4; s >= 1; s >>= 1) {
    const uint32_t m = s == 4 ? 0x0F0F0F0Fu : s == 2 ? 0x33333333u : 0x55555555u;
#pragma unroll
    for (int g = 0; g < 32; g += 2 * s)
#pragma unroll
      for (int i = 0; i < s; i++) {
        uint32_t a = x[g + i], b = x[g + i + s];
        uint32_t t = ((a >> s) ^ b) & m;
        x[g + i + s] = b ^ t;
        x[g + i] = a ^ (t << s);
      }
  }
}

}  // namespace tg
