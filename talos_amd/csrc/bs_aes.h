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
#define bop3(a, b, c, imm) __builtin_amdgcn_bitop3_b32((a), (b), (c), (imm))
// same with a wave-uniform third operand (round-key words: may stay in an SGPR)
#define bop3s(a, b, c, imm) __builtin_amdgcn_bitop3_b32((a), (b), (c), (imm))

}  // namespace tg

#include "bs_sbox.h"

namespace tg {

// N / 8 S-boxes in place (N = 128: 32 blocks per lane; N = 64: the packed
// 16-block layout of gcm_bs16.h, two bytes per plane).
template <int N>
__device__ __forceinline__ void bs_subbytes(uint32_t (&st)[N]) {
#pragma unroll
  for (int b = 0; b < N / 8; b++) {
    uint32_t* p = st + 8 * b;
    uint32_t o7, o6, o5, o4, o3, o2, o1, o0;
    TG_BS_SBOX(p[7], p[6], p[5], p[4], p[3], p[2], p[1], p[0], o7, o6, o5, o4, o3, o2, o1, o0);
    p[7] = o7; p[6] = o6; p[5] = o5; p[4] = o4; p[3] = o3; p[2] = o2; p[1] = o1; p[0] = o0;
    // one S-box at a time: its ~40 temporaries die before the next starts
    // (two waves per SIMD supply the issue parallelism, not interleaving)
    __builtin_amdgcn_sched_barrier(0);
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

// Round-key masks come from a KM policy: km.mask(r, i) = 0 or ~0, bit i
// (= 8 * byte + bit) of round key r.  The kernels derive them with one SALU
// s_bfe_i32 each from the round-key words, which sit in SGPRs.
template <class KM>
__device__ __forceinline__ void bs_masks8(const KM& km, int r, int i, uint32_t (&m)[8]) {
#pragma unroll
  for (int k = 0; k < 8; k++) m[k] = km.mask(r, i + k);
}

// One output plane of MixColumns + AddRoundKey:
//   out_i = xtime(a_i ^ a_{i+1}) ^ a_{i+1} ^ (a_{i+2} ^ a_{i+3})
// xtime on planes: x[0]=t[7], x[1]=t[0]^t[7], x[2]=t[1], x[3]=t[2]^t[7],
// x[4]=t[3]^t[7], x[5]=t[4], x[6]=t[5], x[7]=t[6] (t_i = a_i ^ a_{i+1}).
// Bits 1, 3, 4 take two bitop3 with the key mask folded in, the others one
// bitop3 + one XOR.
__device__ __forceinline__ uint32_t bs_mc_bit(const uint32_t (&t)[4][8], uint32_t n, int i, int k,
                                              uint32_t km) {
  const uint32_t t2 = t[(i + 2) & 3][k];
  if (k == 1 || k == 3 || k == 4) return bop3s(bop3(t[i][k - 1], t[i][7], n, 0x96), t2, km, 0x96);
  return bop3(k == 0 ? t[i][7] : t[i][k - 1], n, t2, 0x96) ^ km;
}

// MixColumns on column C (bytes a_i = st[32C + 8i + k]) + AddRoundKey of
// round r.  Outputs are produced in the order 3, 0, 1, 2 so that each input
// byte dies as soon as its last reader (out_{i-1} reads a_i) is done.
template <int C, class KM, int N>
__device__ __forceinline__ void bs_mixcolumn(uint32_t (&st)[N], const KM& km, int r) {
  uint32_t t[4][8];
#pragma unroll
  for (int i = 0; i < 4; i++)
#pragma unroll
    for (int k = 0; k < 8; k++) t[i][k] = st[32 * C + 8 * i + k] ^ st[32 * C + 8 * ((i + 1) & 3) + k];
  uint32_t m[8], o3[8];
  bs_masks8(km, r, 32 * C + 24, m);
#pragma unroll
  for (int k = 0; k < 8; k++) o3[k] = bs_mc_bit(t, st[32 * C + k], 3, k, m[k]);
#pragma unroll
  for (int i = 0; i < 3; i++) {
    bs_masks8(km, r, 32 * C + 8 * i, m);
#pragma unroll
    for (int k = 0; k < 8; k++)
      st[32 * C + 8 * i + k] = bs_mc_bit(t, st[32 * C + 8 * (i + 1) + k], i, k, m[k]);
  }
#pragma unroll
  for (int k = 0; k < 8; k++) st[32 * C + 24 + k] = o3[k];
}

// Same result, bit-serial from bit 7 down: only the column's t planes of
// bits k and k - 1 (plus bit 7) are live, 16 temporaries instead of 40 — the
// register peak of the packed 64-plane path (gcm_bs16.h).
template <int C, class KM, int N>
__device__ __forceinline__ void bs_mixcolumn_lean(uint32_t (&st)[N], const KM& km, int r) {
  uint32_t t7[4], tk[4];
#pragma unroll
  for (int i = 0; i < 4; i++) {
    t7[i] = st[32 * C + 8 * i + 7] ^ st[32 * C + 8 * ((i + 1) & 3) + 7];
    tk[i] = t7[i];
  }
#pragma unroll
  for (int k = 7; k >= 0; k--) {
    uint32_t tm[4] = {0, 0, 0, 0}, o[4];
    if (k >= 1) {
#pragma unroll
      for (int i = 0; i < 4; i++)
        tm[i] = st[32 * C + 8 * i + k - 1] ^ st[32 * C + 8 * ((i + 1) & 3) + k - 1];
    }
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const uint32_t n = st[32 * C + 8 * ((i + 1) & 3) + k], t2 = tk[(i + 2) & 3];
      const uint32_t m = km.mask(r, 32 * C + 8 * i + k);
      if (k == 1 || k == 3 || k == 4)
        o[i] = bop3s(bop3(tm[i], t7[i], n, 0x96), t2, m, 0x96);
      else
        o[i] = bop3(k == 0 ? t7[i] : tm[i], n, t2, 0x96) ^ m;
    }
#pragma unroll
    for (int i = 0; i < 4; i++) {
      st[32 * C + 8 * i + k] = o[i];
      tk[i] = tm[i];
    }
  }
}

template <class KM>
__device__ __forceinline__ void bs_ark(uint32_t (&st)[128], const KM& km, int r) {
#pragma unroll
  for (int i = 0; i < 128; i += 8) {
    uint32_t m[8];
    bs_masks8(km, r, i, m);
#pragma unroll
    for (int k = 0; k < 8; k++) st[i + k] ^= m[k];
  }
}

// Full encryption of the 32 blocks in `st`.  The final AddRoundKey is left to
// the caller when SKIP_LAST_ARK (it folds into the ciphertext XOR on
// normal-layout words).
template <int ROUNDS, bool SKIP_LAST_ARK, class KM>
__device__ __forceinline__ void bs_encrypt(uint32_t (&st)[128], const KM& km) {
  bs_ark(st, km, 0);
#pragma unroll 1
  for (int r = 1; r < ROUNDS; r++) {
    bs_subbytes(st);
    bs_shiftrows(st);
    bs_mixcolumn<0>(st, km, r);
    bs_mixcolumn<1>(st, km, r);
    bs_mixcolumn<2>(st, km, r);
    bs_mixcolumn<3>(st, km, r);
  }
  bs_subbytes(st);
  bs_shiftrows(st);
  if (!SKIP_LAST_ARK) bs_ark(st, km, ROUNDS);
}

// 32x32 bit transpose of st[O..O+31] in place (x[i] bit j <-> x[j] bit i).
// Stages 16 and 8 are byte moves (v_perm_b32), stages 4/2/1 swap-moves.
template <int S, int O, int N>
__device__ __forceinline__ void transpose_stage(uint32_t (&x)[N]) {
#pragma unroll
  for (int g = 0; g < 32; g += 2 * S)
#pragma unroll
    for (int i = 0; i < S; i++) {
      const uint32_t a = x[O + g + i], b = x[O + g + i + S];
      if (S == 16) {
        x[O + g + i] = __builtin_amdgcn_perm(b, a, 0x05040100u);      // [a.lo16, b.lo16]
        x[O + g + i + S] = __builtin_amdgcn_perm(b, a, 0x07060302u);  // [a.hi16, b.hi16]
      } else if (S == 8) {
        x[O + g + i] = __builtin_amdgcn_perm(b, a, 0x06020400u);      // [a0, b0, a2, b2]
        x[O + g + i + S] = __builtin_amdgcn_perm(b, a, 0x07030501u);  // [a1, b1, a3, b3]
      } else {
        const uint32_t m = S == 4 ? 0x0F0F0F0Fu : S == 2 ? 0x33333333u : 0x55555555u;
        const uint32_t t = ((a >> S) ^ b) & m;
        x[O + g + i + S] = b ^ t;
        x[O + g + i] = a ^ (t << S);
      }
    }
}

template <int O, int N>
__device__ __forceinline__ void transpose32(uint32_t (&x)[N]) {
  transpose_stage<16, O>(x);
  transpose_stage<8, O>(x);
  transpose_stage<4, O>(x);
  transpose_stage<2, O>(x);
  transpose_stage<1, O>(x);
}

__device__ __forceinline__ void transpose_all(uint32_t (&x)[128]) {
  transpose32<0>(x);
  transpose32<32>(x);
  transpose32<64>(x);
  transpose32<96>(x);
}

}  // namespace tg
