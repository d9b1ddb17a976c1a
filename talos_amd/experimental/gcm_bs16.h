// gcm_bs16.h — one TLS record per wave with a packed bitsliced AES-CTR
// keystream.  Included by gcm_hybrid.h (uses its helpers).
//
// Layout: lane L owns the record's blocks 64 j + L, j = 0..15 (the same
// lane chains as the T-table path, so GHASH and the finish are shared).  The
// 16 counter blocks of a lane are held as 64 packed planes:
//   st[8 g + k], g = 0..7: bits 0..15  = bit k of byte g     of blocks j = 0..15,
//                          bits 16..31 = bit k of byte g + 8 of blocks j = 0..15,
// i.e. column c = 0, 1 in the low half-words and column c + 2 in the high ones
// (byte b = 4 c + r).  SubBytes (the 85-node v_bitop3 circuit) and MixColumns
// act on both halves alike, so one record's 1024 blocks cost 8 S-box
// evaluations per round on 64 registers — half the register footprint of the
// 32-block layout of bs_aes.h, which lets four waves share a SIMD (<= 128
// VGPRs) instead of two.  ShiftRows becomes register renaming plus half-word
// swaps of four byte groups.  Round keys are wave-uniform (one record per
// wave): their packed masks are built in SGPRs (s_bfe).
//
// Rounds 1 and 2 use the TLS counter shortcut of bs_encrypt_r2 (RecPre k1a,
// k1b, sb2: counters < 2^16 differ only in bytes 14, 15).  Equivalent to
// CRYPTO_gcm128_decrypt/encrypt's CTR keystream (modes/gcm128.c:1020-1116) on
// each block; GHASH and the tag are gcm_record's (gcm_device.h).
#pragma once

namespace tg {

// Packed round-key masks: low half 0 / ~0 from bit k of byte g of round key r,
// high half from byte g + 8 (idx = 8 g + k).
struct Pk16Masks {
  cu32* rk;
  __device__ __forceinline__ uint32_t mask(int r, int idx) const {
    const int g = idx >> 3, k = idx & 7;
    const uint32_t lo =
        (uint32_t)__builtin_amdgcn_sbfe((int32_t)rk[4 * r + (g >> 2)], (uint32_t)(8 * (g & 3) + k), 1u);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_sbfe((int32_t)rk[4 * r + 2 + (g >> 2)],
                                                        (uint32_t)(8 * (g & 3) + k), 1u);
    return (lo & 0xFFFFu) | (hi << 16);
  }
};

// ShiftRows on the packed layout: new byte (r, c) = old byte (r, c + r).
// Group g = 4 cp + r holds columns cp (low) and cp + 2 (high):
//   r = 1: g1 <- g5, g5 <- swap(g1);  r = 2: g2, g6 swapped in place;
//   r = 3: g3 <- swap(g7), g7 <- g3.
__device__ __forceinline__ void bs16_shiftrows(uint32_t (&st)[64]) {
#pragma unroll
  for (int k = 0; k < 8; k++) {
    const uint32_t g1 = st[8 + k], g2 = st[16 + k], g3 = st[24 + k];
    const uint32_t g5 = st[40 + k], g6 = st[48 + k], g7 = st[56 + k];
    st[8 + k] = g5;
    st[40 + k] = rotl16(g1);
    st[16 + k] = rotl16(g2);
    st[48 + k] = rotl16(g6);
    st[24 + k] = rotl16(g7);
    st[56 + k] = g3;
  }
}

// Rounds 1 and 2 (through round 2's AddRoundKey) for the counters of lane
// base u = 2 + lane (slot j: u + 64 j), from the record constants.
template <int ROUNDS>
__device__ __forceinline__ void bs16_encrypt_r2(uint32_t (&st)[64], const RecPre* pre, uint32_t u,
                                                cu32* rk) {
  const SgprMasks km0{rk};
  uint32_t c14[8], c15[8];
  bs_ctr_c14c15(u, c14, c15);
  // both counter bytes through one S-box evaluation: c15 low, c14 high
  uint32_t pk[8], sp[8], xp[8];
#pragma unroll
  for (int k = 0; k < 8; k++) {
    const uint32_t m = (km0.mask(0, 8 * 15 + k) & 0xFFFFu) | (km0.mask(0, 8 * 14 + k) & 0xFFFF0000u);
    pk[k] = ((c15[k] & 0xFFFFu) | (c14[k] & 0xFFFF0000u)) ^ m;
  }
  TG_SBOX8(pk, sp);
  bs_xtime(sp, xp);
  cu32* P = as_const(pre);
  const uint32_t k1a = P[4], k1b = P[5], sb2a = P[10], sb2b = P[11];
  auto bit = [](uint32_t w, int i) { return (uint32_t)__builtin_amdgcn_sbfe((int32_t)w, (uint32_t)i, 1u); };
  // Round-1 output columns 0 (groups 0-3, from s15) and 1 (groups 4-7, from
  // s14) in the low halves, each group through round 2's S-box as soon as it
  // is built; the high halves (columns 2, 3) are then replaced by their S-box
  // images sb2.  Built in this order the peak stays below 128 VGPRs.
  auto sbox_group = [&](int g) {
    uint32_t* p = st + 8 * g;
    uint32_t o7, o6, o5, o4, o3, o2, o1, o0;
    TG_BS_SBOX(p[7], p[6], p[5], p[4], p[3], p[2], p[1], p[0], o7, o6, o5, o4, o3, o2, o1, o0);
    const uint32_t o[8] = {o0, o1, o2, o3, o4, o5, o6, o7};
#pragma unroll
    for (int k = 0; k < 8; k++)
      p[k] = (o[k] & 0xFFFFu) | (bit(g < 4 ? sb2a : sb2b, 8 * (g & 3) + k) & 0xFFFF0000u);
    __builtin_amdgcn_sched_barrier(0);
  };
#pragma unroll
  for (int g = 0; g < 4; g++) {
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const uint32_t kb = bit(k1a, 8 * g + k);
      st[8 * g + k] = g == 0 ? kb ^ sp[k] : g == 1 ? kb ^ sp[k] : g == 2 ? xor3(kb, xp[k], sp[k]) : kb ^ xp[k];
    }
    sbox_group(g);
  }
#pragma unroll
  for (int k = 0; k < 8; k++) { sp[k] = rotl16(sp[k]); xp[k] = rotl16(xp[k]); }  // s14, x14
#pragma unroll
  for (int g = 4; g < 8; g++) {
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const uint32_t kb = bit(k1b, 8 * (g - 4) + k);
      st[8 * g + k] = g == 4 ? kb ^ sp[k] : g == 5 ? xor3(kb, xp[k], sp[k]) : g == 6 ? kb ^ xp[k] : kb ^ sp[k];
    }
    sbox_group(g);
  }
  bs16_shiftrows(st);
  const Pk16Masks km{rk};
  bs_mixcolumn_lean<0>(st, km, 2);
  bs_mixcolumn_lean<1>(st, km, 2);
}

// Keystream of the lane's 16 blocks without the final AddRoundKey, back in
// normal layout: block j = {st[j], st[32 + j], st[16 + j], st[48 + j]} (LE words).
template <int ROUNDS>
__device__ __forceinline__ void bs16_keystream(uint32_t (&st)[64], const RecPre* pre, uint32_t u,
                                               cu32* rk) {
  bs16_encrypt_r2<ROUNDS>(st, pre, u, rk);
  __builtin_amdgcn_sched_barrier(0);
  const Pk16Masks km{rk};
#pragma unroll 1
  for (int r = 3; r < ROUNDS; r++) {
    bs_subbytes(st);
    bs16_shiftrows(st);
    bs_mixcolumn_lean<0>(st, km, r);
    bs_mixcolumn_lean<1>(st, km, r);
  }
  bs_subbytes(st);
  bs16_shiftrows(st);
  transpose32<0>(st);
  transpose32<32>(st);
  __builtin_amdgcn_sched_barrier(0);
}

// One 16-B-aligned record of at most 1024 blocks (TLS counters < 2^16): the
// keystream of all its blocks bitsliced, then 16 lane steps of CTR XOR + the
// H^64 lane chains, then gcm_finish.
template <bool SEAL, int ROUNDS>
__device__ __forceinline__ void gcm_record_bs16(const RecCtx& rc, const RecPre* pre, const DevSession* __restrict__ S,
                                int32_t* status_slot, uint32_t lane, const GhLane& gl,
                                unsigned long long* dbg) {
  PhaseClock pc(dbg);
  cu32* rk = as_const(S->rk);
  const uint32_t n = rc.n, nb = (n + 15) >> 4;
  // the record's bytes to L2 ahead of the ~10K-instruction AES phase
  const Prefetch<2> pf = l2_prefetch<2>(rc.src, n, lane);
  uint32_t st[64];
  bs16_keystream<ROUNDS>(st, pre, 2u + lane, rk);
  pc.lap(13, lane);
  const uint32_t rkl[4] = {rk[4 * ROUNDS], rk[4 * ROUNDS + 1], rk[4 * ROUNDS + 2], rk[4 * ROUNDS + 3]};
  uint32_t x[4] = {0, 0, 0, 0};
  if (rc.aad_len != 0 && lane == 63) {
    x[0] = bswap32(rc.aad_be[0]); x[1] = bswap32(rc.aad_be[1]);
    x[2] = bswap32(rc.aad_be[2]); x[3] = bswap32(rc.aad_be[3]);
  }
  auto load = [&](uint32_t j, uint32_t (&v)[4]) {
    const uint32_t i = 64u * j + lane;
    const uint32_t nbytes = i < nb ? min(16u, n - 16u * i) : 0u;
    load_block(rc.src + 16u * i, nbytes, true, v);
  };
  uint32_t cur[4], nxt[4] = {0, 0, 0, 0};
  load(0, cur);
  prefetch_done(pf);
#pragma unroll
  for (int j = 0; j < 16; j++) {
    if (64u * j < nb) {  // uniform: steps of short records past their end are skipped
      if (j + 1 < 16 && 64u * (j + 1) < nb) load(j + 1, nxt);
      const uint32_t i = 64u * j + lane;
      const bool active = i < nb;
      const uint32_t nbytes = active ? min(16u, n - 16u * i) : 0u;
      uint32_t ks[4] = {st[j] ^ rkl[0], st[32 + j] ^ rkl[1], st[16 + j] ^ rkl[2], st[48 + j] ^ rkl[3]};
#pragma unroll
      for (int w = 0; w < 4; w++) {  // zero-padded GHASH block for the partial tail
        const int32_t b = (int32_t)nbytes - 4 * w;
        ks[w] &= b >= 4 ? 0xFFFFFFFFu : (b <= 0 ? 0u : ((1u << (8 * b)) - 1u));
      }
      const uint32_t o[4] = {cur[0] ^ ks[0], cur[1] ^ ks[1], cur[2] ^ ks[2], cur[3] ^ ks[3]};
      if (active) store_block(rc.dst + 16u * i, nbytes, true, o);
      uint32_t xk[4];
      mul_k(x, xk, gl);
      if (active) {
        const uint32_t* g = SEAL ? o : cur;
        x[0] = xk[0] ^ g[0]; x[1] = xk[1] ^ g[1]; x[2] = xk[2] ^ g[2]; x[3] = xk[3] ^ g[3];
      }
#pragma unroll
      for (int w = 0; w < 4; w++) cur[w] = nxt[w];
    }
  }
  pc.lap(14, lane);
  const uint32_t ek0[4] = {as_const(pre)[0], as_const(pre)[1], as_const(pre)[2], as_const(pre)[3]};
  gcm_finish<SEAL>(rc, x, ek0, S, status_slot, lane, gl);
  pc.lap(15, lane);
}

// The queue kernel's bitsliced wave role (hy_b16_record): a
// 16-B-aligned record of at most 1024 blocks.  Its full 64-block steps take
// the bitsliced keystream with a lean consume loop (whole-wave 16-B loads and
// stores, no partial-block masking: the general loop of gcm_record_bs16 spills
// in the queue kernel), the rest (< 64 blocks) the T-table gcm_blocks path.
template <bool SEAL, int ROUNDS>
__device__ __forceinline__ void gcm_record_bs16f(const RecCtx& rc, const RecPre* pre,
                                                 const DevSession* __restrict__ S,
                                                 int32_t* status_slot, uint32_t lane,
                                                 uint32_t laneoff, const GhLane& gl) {
  cu32* rk = as_const(S->rk);
  const uint32_t steps = rc.n >> 10;  // full 64-block steps, <= 16
  const Prefetch<2> pf = l2_prefetch<2>(rc.src, steps << 10, lane);
  uint32_t st[64];
  bs16_keystream<ROUNDS>(st, pre, 2u + lane, rk);
  const uint32_t rkl[4] = {rk[4 * ROUNDS], rk[4 * ROUNDS + 1], rk[4 * ROUNDS + 2], rk[4 * ROUNDS + 3]};
  uint32_t x[4] = {0, 0, 0, 0};
  if (lane == 63) {  // AAD' at j = -1 (TLS: the 13-byte AAD)
    x[0] = bswap32(rc.aad_be[0]); x[1] = bswap32(rc.aad_be[1]);
    x[2] = bswap32(rc.aad_be[2]); x[3] = bswap32(rc.aad_be[3]);
  }
  const uint4* src = reinterpret_cast<const uint4*>(rc.src) + lane;
  uint4* dst = reinterpret_cast<uint4*>(rc.dst) + lane;
  uint4 cur = src[0];
  prefetch_done(pf);
#pragma unroll
  for (int j = 0; j < 16; j++) {
    if ((uint32_t)j < steps) {
      uint4 nxt = cur;
      if (j + 1 < 16 && (uint32_t)(j + 1) < steps) nxt = src[64 * (j + 1)];
      const uint32_t c[4] = {cur.x, cur.y, cur.z, cur.w};
      const uint32_t o[4] = {xor3(c[0], st[j], rkl[0]), xor3(c[1], st[32 + j], rkl[1]),
                             xor3(c[2], st[16 + j], rkl[2]), xor3(c[3], st[48 + j], rkl[3])};
      dst[64 * j] = make_uint4(o[0], o[1], o[2], o[3]);
      uint32_t xk[4];
      mul_k(x, xk, gl);
      const uint32_t* g = SEAL ? o : c;
      x[0] = xk[0] ^ g[0]; x[1] = xk[1] ^ g[1]; x[2] = xk[2] ^ g[2]; x[3] = xk[3] ^ g[3];
      cur = nxt;
    }
  }
  const RecConsts rcc = rec_consts_of(pre);
  uint32_t start = steps << 6;
  const CtrConst none = {};
  gcm_blocks<SEAL, ROUNDS, true>(rc, S, rcc, none, x, start, lane, laneoff, gl);
  gcm_finish<SEAL>(rc, x, rcc.ek0, S, status_slot, lane, gl);
}

}  // namespace tg
