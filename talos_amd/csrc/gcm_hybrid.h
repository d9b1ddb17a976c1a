// gcm_hybrid.h — AES-GCM TLS record kernels driven by a per-run record queue
// and per-record constants from a prep pass:
//   * gcm_prep_kernel: E_K(J0) and the round-1/2 constants of every record;
//   * gcm_hy_kernel<NT, BSW, NB>: NT threads, the first BSW waves bitsliced
//     (record pairs, AES-CTR keystream on the VALU, bs_aes.h), the others
//     T-table waves (single records, NB blocks per lane in flight).
// Instantiated per variant in gcm_queue.hip / gcm_hy128.hip / gcm_hy256.hip so
// that the (slow to compile) bitsliced instantiations build in parallel.
#pragma once
#include <utility>

#include "gcm_device.h"

namespace tg {


__device__ __forceinline__ uint32_t xor3s(uint32_t a, uint32_t b, uint32_t k) {
  return bop3s(a, b, k, 0x96);
}

// Counter-block planes for pass p (blocks 1024p .. 1024p + 1023 of both
// records).  Bytes 0..11 = the records' nonces (uniform per half), bytes 12-13
// zero, bytes 14-15 = the big-endian counter u + 64 (j & 15), u = 2 + lane +
// 1024 p < 2^16 (TLSGPU_MAX_RECORD): low 6 bits constant per lane, bits 6..9
// a rotated slot pattern, bits 10..15 select between U_hi and U_hi + 1.
__device__ __forceinline__ void bs_ctr_planes(uint32_t (&st)[128], const uint32_t* ja,
                                              const uint32_t* jb, uint32_t u) {
#pragma unroll
  for (int w = 0; w < 3; w++)
#pragma unroll
    for (int bit = 0; bit < 32; bit++) {
      const uint32_t ma = 0u - ((ja[w] >> bit) & 1u), mb = 0u - ((jb[w] >> bit) & 1u);
      st[32 * w + bit] = (ma & 0x0000FFFFu) | (mb & 0xFFFF0000u);
    }
#pragma unroll
  for (int k = 0; k < 16; k++) st[96 + k] = 0u;
#pragma unroll
  for (int k = 0; k < 6; k++) st[120 + k] = 0u - ((u >> k) & 1u);
  const uint32_t U = u >> 6, ulo = U & 15u, uhi = U >> 4;
  st[126] = __builtin_amdgcn_alignbit(0xAAAAAAAAu, 0xAAAAAAAAu, ulo);
  st[127] = __builtin_amdgcn_alignbit(0xCCCCCCCCu, 0xCCCCCCCCu, ulo);
  st[112] = __builtin_amdgcn_alignbit(0xF0F0F0F0u, 0xF0F0F0F0u, ulo);
  st[113] = __builtin_amdgcn_alignbit(0xFF00FF00u, 0xFF00FF00u, ulo);
  const uint32_t cm = ((0xFFFF0000u >> ulo) & 0xFFFFu) * 0x10001u;  // slots that carry
  const uint32_t h1 = uhi + 1u;
#pragma unroll
  for (int q = 0; q < 6; q++)
    st[114 + q] = (cm & (0u - ((h1 >> q) & 1u))) | (~cm & (0u - ((uhi >> q) & 1u)));
}

// One consume step of gcm_pair_hy (see there).
template <bool SEAL, int T>
__device__ __forceinline__ void bs_consume(const uint32_t (&st)[128], uint32_t (&ring)[4][2][4],
                                           uint32_t (&x)[2][4], const RecCtx (&rc)[2],
                                           const uint32_t (&rkl)[4], uint32_t pb, uint32_t lane,
                                           const GhLane& gl) {
  const uint32_t i = pb + 64u * T + lane;
  uint32_t c[2][4], g[2][4];
#pragma unroll
  for (int q = 0; q < 2; q++)
#pragma unroll
    for (int w = 0; w < 4; w++) c[q][w] = ring[T & 3][q][w];
  if (T + 4 < 16) {
#pragma unroll
    for (int q = 0; q < 2; q++) {
      const uint4 v = *reinterpret_cast<const uint4*>(rc[q].src + 16u * (i + 256u));
      ring[T & 3][q][0] = v.x; ring[T & 3][q][1] = v.y; ring[T & 3][q][2] = v.z; ring[T & 3][q][3] = v.w;
    }
  }
#pragma unroll
  for (int q = 0; q < 2; q++) {
    uint32_t o[4];
#pragma unroll
    for (int w = 0; w < 4; w++) o[w] = xor3s(c[q][w], st[32 * w + 16 * q + T], rkl[w]);
    *reinterpret_cast<uint4*>(rc[q].dst + 16u * i) = make_uint4(o[0], o[1], o[2], o[3]);
#pragma unroll
    for (int w = 0; w < 4; w++) g[q][w] = SEAL ? o[w] : c[q][w];
  }
  uint32_t xa[4], xb[4];
  mul_k2(x[0], x[1], xa, xb, gl);
#pragma unroll
  for (int w = 0; w < 4; w++) { x[0][w] = xa[w] ^ g[0][w]; x[1][w] = xb[w] ^ g[1][w]; }
}

template <bool SEAL, int... T>
__device__ __forceinline__ void bs_consume_all(const uint32_t (&st)[128], uint32_t (&ring)[4][2][4],
                                               uint32_t (&x)[2][4], const RecCtx (&rc)[2],
                                               const uint32_t (&rkl)[4], uint32_t pb,
                                               uint32_t lane, const GhLane& gl,
                                               std::integer_sequence<int, T...>) {
  (bs_consume<SEAL, T>(st, ring, x, rc, rkl, pb, lane, gl), ...);
}

// Two records of one session, both 16-B aligned with >= 1024 full blocks.
// Whole 1024-block passes run bitsliced; any remainder of either record

// ---------------------------------------------------------------------------
// Hybrid kernel.  The T-table path is bound by LDS (16
// lookups per block-round), the bitsliced path by VALU issue; one CU has both.
// A 512-thread workgroup runs 8 waves, two per SIMD: waves 0-3 are "bitsliced"
// waves (record pairs through bs_encrypt_ctr, VALU-only AES), waves 4-7 are
// "T-table" waves (single records, 4 blocks per lane in flight, raised issue
// priority so the LDS pipe stays fed).  Inside a session run the waves pull
// records from an LDS counter, so the split follows the measured rates; a
// bitsliced wave stops taking pairs when fewer than a.bs_reserve records of
// the run remain (a pair is the coarsest unit; the run ends at a barrier).
constexpr int kHyThreads = 512;
constexpr int kHyBsWaves = 4;

// Round-1/2 shortcut for TLS counters (< 2^16): bytes 0..13 of
// every counter block of a record are the same, so after round 1 columns 2, 3
// are per-record constants and columns 0, 1 differ only through
// S(ctr byte 15 ^ rk0) and S(ctr byte 14 ^ rk0):
//   col 0 = k1a ^ (s, s, 3s, 2s),  col 1 = k1b ^ (s', 3s', 2s', s')
// (the MixColumns images of one non-zero byte in row 3 / row 2).  Round 2 then
// needs 8 S-boxes on the VALU; the other 8 are the per-record constants sb2.
// Slots 0..15 hold record A, 16..31 record B (half-word planes).
__device__ __forceinline__ uint32_t half_plane(uint32_t wa, uint32_t wb, int bit) {
  const uint32_t ma = (uint32_t)__builtin_amdgcn_sbfe((int32_t)wa, (uint32_t)bit, 1u);
  const uint32_t mb = (uint32_t)__builtin_amdgcn_sbfe((int32_t)wb, (uint32_t)bit, 1u);
  return (ma & 0x0000FFFFu) | (mb & 0xFFFF0000u);
}

// xtime on 8 planes (p[k] = bit k): {p7, p0^p7, p1, p2^p7, p3^p7, p4, p5, p6}
__device__ __forceinline__ void bs_xtime(const uint32_t (&p)[8], uint32_t (&o)[8]) {
  o[0] = p[7]; o[1] = p[0] ^ p[7]; o[2] = p[1]; o[3] = p[2] ^ p[7];
  o[4] = p[3] ^ p[7]; o[5] = p[4]; o[6] = p[5]; o[7] = p[6];
}

#define TG_SBOX8(in, out) \
  TG_BS_SBOX(in[7], in[6], in[5], in[4], in[3], in[2], in[1], in[0], out[7], out[6], out[5], \
             out[4], out[3], out[2], out[1], out[0])

// Planes of counter bytes 14 (c14) and 15 (c15) of slot j (bit j, both
// half-words alike): the big-endian counter u + 64 (j mod 16) < 2^16.
__device__ __forceinline__ void bs_ctr_c14c15(uint32_t u, uint32_t (&c14)[8], uint32_t (&c15)[8]) {
#pragma unroll
  for (int k = 0; k < 6; k++) c15[k] = 0u - ((u >> k) & 1u);
  const uint32_t U = u >> 6, ulo = U & 15u, uhi = U >> 4;
  c15[6] = __builtin_amdgcn_alignbit(0xAAAAAAAAu, 0xAAAAAAAAu, ulo);
  c15[7] = __builtin_amdgcn_alignbit(0xCCCCCCCCu, 0xCCCCCCCCu, ulo);
  c14[0] = __builtin_amdgcn_alignbit(0xF0F0F0F0u, 0xF0F0F0F0u, ulo);
  c14[1] = __builtin_amdgcn_alignbit(0xFF00FF00u, 0xFF00FF00u, ulo);
  const uint32_t cm = ((0xFFFF0000u >> ulo) & 0xFFFFu) * 0x10001u;  // slots that carry
  const uint32_t h1 = uhi + 1u;
#pragma unroll
  for (int q = 0; q < 6; q++)
    c14[2 + q] = (cm & (0u - ((h1 >> q) & 1u))) | (~cm & (0u - ((uhi >> q) & 1u)));
}

// Keystream planes of pass p (blocks 1024p .. 1024p + 1023 of records A and B,
// u = 2 + lane + 1024p) without the final AddRoundKey.
// Rounds 1 and 2 (through round 2's AddRoundKey).
template <int ROUNDS>
__device__ __forceinline__ void bs_encrypt_r2(uint32_t (&st)[128], const RecPre* pa,
                                              const RecPre* pb, uint32_t u, cu32* rk) {
  const SgprMasks km{rk};
  uint32_t c14[8], c15[8];
  bs_ctr_c14c15(u, c14, c15);
#pragma unroll
  for (int k = 0; k < 8; k++) {
    c14[k] ^= km.mask(0, 8 * 14 + k);
    c15[k] ^= km.mask(0, 8 * 15 + k);
  }
  uint32_t s14[8], s15[8], x14[8], x15[8];
  TG_SBOX8(c14, s14);
  TG_SBOX8(c15, s15);
  bs_xtime(s14, x14);
  bs_xtime(s15, x15);
  cu32* A = as_const(pa);
  cu32* B = as_const(pb);
  const uint32_t k1aA = A[4], k1aB = B[4], k1bA = A[5], k1bB = B[5];
#pragma unroll
  for (int k = 0; k < 8; k++) {
    st[8 * 0 + k] = half_plane(k1aA, k1aB, k) ^ s15[k];
    st[8 * 1 + k] = half_plane(k1aA, k1aB, 8 + k) ^ s15[k];
    st[8 * 2 + k] = half_plane(k1aA, k1aB, 16 + k) ^ x15[k] ^ s15[k];
    st[8 * 3 + k] = half_plane(k1aA, k1aB, 24 + k) ^ x15[k];
    st[8 * 4 + k] = half_plane(k1bA, k1bB, k) ^ s14[k];
    st[8 * 5 + k] = half_plane(k1bA, k1bB, 8 + k) ^ x14[k] ^ s14[k];
    st[8 * 6 + k] = half_plane(k1bA, k1bB, 16 + k) ^ x14[k];
    st[8 * 7 + k] = half_plane(k1bA, k1bB, 24 + k) ^ s14[k];
  }
  // round 2: SubBytes of columns 0, 1 on the VALU, columns 2, 3 from sb2
#pragma unroll
  for (int b = 0; b < 8; b++) {
    uint32_t* p = st + 8 * b;
    uint32_t o7, o6, o5, o4, o3, o2, o1, o0;
    TG_BS_SBOX(p[7], p[6], p[5], p[4], p[3], p[2], p[1], p[0], o7, o6, o5, o4, o3, o2, o1, o0);
    p[7] = o7; p[6] = o6; p[5] = o5; p[4] = o4; p[3] = o3; p[2] = o2; p[1] = o1; p[0] = o0;
    __builtin_amdgcn_sched_barrier(0);
  }
  const uint32_t sbA[2] = {A[10], A[11]}, sbB[2] = {B[10], B[11]};
#pragma unroll
  for (int b = 8; b < 16; b++)
#pragma unroll
    for (int k = 0; k < 8; k++)
      st[8 * b + k] = half_plane(sbA[(b - 8) >> 2], sbB[(b - 8) >> 2], 8 * ((b - 8) & 3) + k);
  bs_shiftrows(st);
  bs_mixcolumn<0>(st, km, 2);
  bs_mixcolumn<1>(st, km, 2);
  bs_mixcolumn<2>(st, km, 2);
  bs_mixcolumn<3>(st, km, 2);
}

template <int ROUNDS>
__device__ __forceinline__ void bs_encrypt_ctr(uint32_t (&st)[128], const RecPre* pa,
                                               const RecPre* pb, uint32_t u, cu32* rk) {
  const SgprMasks km{rk};
  bs_encrypt_r2<ROUNDS>(st, pa, pb, u, rk);
#pragma unroll 1
  for (int r = 3; r < ROUNDS; r++) {
    bs_subbytes(st);
    bs_shiftrows(st);
    bs_mixcolumn<0>(st, km, r);
    bs_mixcolumn<1>(st, km, r);
    bs_mixcolumn<2>(st, km, r);
    bs_mixcolumn<3>(st, km, r);
  }
  bs_subbytes(st);
  bs_shiftrows(st);
}

__device__ __forceinline__ RecConsts rec_consts_of(const RecPre* p) {
  cu32* w = as_const(p);
  RecConsts c;
#pragma unroll
  for (int i = 0; i < 4; i++) c.ek0[i] = w[i];
  c.k1a = w[4];
  c.k1b = w[5];
#pragma unroll
  for (int i = 0; i < 4; i++) c.k2[i] = w[6 + i];
  return c;
}

// Two 16-B-aligned records of one session with >= 1024 full blocks each:
// whole 1024-block passes bitsliced, any remainder through gcm_blocks.
template <bool SEAL, int ROUNDS>
__device__ void gcm_pair_hy(const RecCtx (&rc)[2], const RecPre* pa, const RecPre* pb,
                            int32_t* slot_a, int32_t* slot_b, const DevSession* __restrict__ S,
                            uint32_t lane, uint32_t laneoff, const GhLane& gl,
                            unsigned long long* dbg) {
  PhaseClock pc(dbg);
  cu32* rk = as_const(S->rk);
  const uint32_t rkl[4] = {rk[4 * ROUNDS], rk[4 * ROUNDS + 1], rk[4 * ROUNDS + 2],
                           rk[4 * ROUNDS + 3]};
  uint32_t x[2][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
  if (lane == 63) {  // AAD' at j = -1 (TLS always has the 13-byte AAD)
#pragma unroll
    for (int q = 0; q < 2; q++)
#pragma unroll
      for (int w = 0; w < 4; w++) x[q][w] = bswap32(rc[q].aad_be[w]);
  }
  const uint32_t passes = min(rc[0].n, rc[1].n) >> 14;
  for (uint32_t p = 0; p < passes; p++) {
    const uint32_t pb0 = p << 10;
    // this pass's 2 x 16 KiB to L2 ahead of the ~15K-instruction AES phase
    const Prefetch<2> pfa = l2_prefetch<2>(rc[0].src + 16u * pb0, rc[0].n - 16u * pb0, lane);
    const Prefetch<2> pfb = l2_prefetch<2>(rc[1].src + 16u * pb0, rc[1].n - 16u * pb0, lane);
    uint32_t st[128];
    bs_encrypt_ctr<ROUNDS>(st, pa, pb, 2u + lane + pb0, rk);
    pc.lap(1, lane);
    uint32_t ring[4][2][4];
#pragma unroll
    for (int t = 0; t < 4; t++)
#pragma unroll
      for (int q = 0; q < 2; q++) {
        const uint4 v = *reinterpret_cast<const uint4*>(rc[q].src + 16u * (pb0 + 64u * t + lane));
        ring[t][q][0] = v.x; ring[t][q][1] = v.y; ring[t][q][2] = v.z; ring[t][q][3] = v.w;
      }
    prefetch_done(pfa);
    prefetch_done(pfb);
    transpose_all(st);
    bs_consume_all<SEAL>(st, ring, x, rc, rkl, pb0, lane, gl,
                         std::make_integer_sequence<int, 16>{});
    pc.lap(2, lane);
  }
#pragma unroll
  for (int q = 0; q < 2; q++) {
    if (((rc[q].n + 15) >> 4) > (passes << 10)) {
      const RecConsts rcc = rec_consts_of(q ? pb : pa);
      const CtrConst none = {};
      gcm_blocks<SEAL, ROUNDS, true>(rc[q], S, rcc, none, x[q], passes << 10, lane, laneoff, gl);
    }
  }
  uint32_t ek[2][4];
#pragma unroll
  for (int w = 0; w < 4; w++) {
    ek[0][w] = as_const(pa)[w];
    ek[1][w] = as_const(pb)[w];
  }
  gcm_finish2<SEAL>(rc, x, ek, S, slot_a, slot_b, lane, gl);
  pc.lap(3, lane);
}

}  // namespace tg

#ifdef TG_EXPERIMENTAL  // the packed bitsliced record path (talos_amd/experimental/)
#include "../experimental/gcm_bs16.h"
#endif

namespace tg {

// The bounds rule of check_record_bounds (session_kernels.hip): the record's
// input span and output span lie inside the caller's buffers.
__device__ __forceinline__ bool rec_in_bounds(const tlsgpu_record& d, const DevSession* S,
                                              uint64_t in_bytes, uint64_t out_bytes, bool seal) {
  const uint64_t eiv = as_const(&S->nonce_in_record)[0] ? 8u : 0u, tag = as_const(&S->tag_len)[0];
  const uint64_t len = d.len_type & 0xFFFFFFu;
  const uint64_t out_len = seal ? len + eiv + tag : (len >= eiv + tag ? len - eiv - tag : 0);
  return !(d.in_off > in_bytes || len > in_bytes - d.in_off || d.out_off > out_bytes ||
           out_len > out_bytes - d.out_off);
}

// RecPre written by this kernel's own prologue (fused): vector loads (the
// scalar cache, shared by neighbouring CUs, could hold a line of it from
// before the prologue's stores), made wave-uniform.
__device__ __forceinline__ RecConsts rec_consts_fresh(const RecPre* p) {
  const uint4* q = reinterpret_cast<const uint4*>(p);
  const uint4 a = q[0], b = q[1], c = q[2];
  RecConsts rc;
  rc.ek0[0] = __builtin_amdgcn_readfirstlane(a.x);
  rc.ek0[1] = __builtin_amdgcn_readfirstlane(a.y);
  rc.ek0[2] = __builtin_amdgcn_readfirstlane(a.z);
  rc.ek0[3] = __builtin_amdgcn_readfirstlane(a.w);
  rc.k1a = __builtin_amdgcn_readfirstlane(b.x);
  rc.k1b = __builtin_amdgcn_readfirstlane(b.y);
  rc.k2[0] = __builtin_amdgcn_readfirstlane(b.z);
  rc.k2[1] = __builtin_amdgcn_readfirstlane(b.w);
  rc.k2[2] = __builtin_amdgcn_readfirstlane(c.x);
  rc.k2[3] = __builtin_amdgcn_readfirstlane(c.y);
  return rc;
}

template <bool SEAL, int ROUNDS, int NB = 4>
__device__ __forceinline__ void hy_tt_record(const BatchArgs& a, const RecPre* __restrict__ pre,
                                             uint32_t r, const DevSession* __restrict__ S,
                                             uint32_t lane, uint32_t laneoff, const GhLane& gl) {
  const tlsgpu_record* D = reinterpret_cast<const tlsgpu_record*>(a.descs);
  RecCtx rc;
  const tlsgpu_record d = load_desc(D + r);
  // fused: an out-of-bounds record's status was written by the prologue
  if (a.fused && !rec_in_bounds(d, S, a.in_bytes, a.out_bytes, SEAL)) return;
  if (!parse_tls<SEAL>(d, S, a.in, a.out, a.status + r, lane, rc)) return;
#ifdef TG_BS16  // packed bitsliced path (experimental build)
  if (a.bs16_min != 0 && rc.n >= a.bs16_min && rc.n <= 16384u &&
      ((((uintptr_t)rc.src) | ((uintptr_t)rc.dst)) & 15) == 0) {
    gcm_record_bs16<SEAL, ROUNDS>(rc, pre + r, S, a.status + r, lane, gl, a.dbg);
    return;
  }
#endif
  const RecConsts rcc = rec_consts_fresh(pre + r);
  gcm_record_x4<SEAL, ROUNDS, NB>(rc, S, rcc, a.status + r, lane, laneoff, gl, a.dbg);
}

// Packed bitsliced wave role: a record of a_min..16384
// bytes, 16-B aligned, with more than `reserve` records of its session run
// still unclaimed runs through gcm_record_bs16 (AES-CTR on the VALU, GHASH on
// the shared LDS table); anything else through the T-table path.  The reserve
// keeps the run's last records on T-table waves, so the run-end barrier does
// not wait for a bitsliced record started late.
#ifndef TG_EXPERIMENTAL
// default build: no bitsliced role (B16W = 0 everywhere), never instantiated
template <bool SEAL, int ROUNDS>
__device__ __forceinline__ bool hy_b16_record(const BatchArgs&, const RecPre* __restrict__,
                                              uint32_t, uint32_t, const DevSession* __restrict__,
                                              uint32_t, uint32_t, const GhLane&) {
  return false;
}
#else
template <bool SEAL, int ROUNDS>
__device__ __forceinline__ bool hy_b16_record(const BatchArgs& a, const RecPre* __restrict__ pre,
                                              uint32_t r, uint32_t left,
                                              const DevSession* __restrict__ S, uint32_t lane,
                                              uint32_t laneoff, const GhLane& gl) {
  const tlsgpu_record* D = reinterpret_cast<const tlsgpu_record*>(a.descs);
  const tlsgpu_record d = load_desc(D + r);
  if (left <= a.bs_reserve) return false;
  RecCtx rc;
  if (!parse_tls<SEAL>(d, S, a.in, a.out, a.status + r, lane, rc)) return true;
  if (rc.n >= a.bs16_min && rc.n >= 1024u && rc.n <= 16384u &&
      ((((uintptr_t)rc.src) | ((uintptr_t)rc.dst)) & 15) == 0) {
    gcm_record_bs16f<SEAL, ROUNDS>(rc, pre + r, S, a.status + r, lane, laneoff, gl);
    return true;
  }
  return false;  // the caller's T-table path (one call site of gcm_record_x4: inlined)
}
#endif

// ---------------------------------------------------------------------------
// Short-record packs.  A record's GHASH sequence is
// [AAD, C_0..C_{nb-1}, lengths] (gcm128.c:826-881,1356-1500): nb + 2 elements.
// When that fits in the wave, consecutive records of one session are laid side
// by side across the lanes, record i at lanes [base_i, base_i + nb_i + 2).  Each
// lane then holds ONE element E_j and GHASH = XOR_j E_j * H^(nb + 1 - j)
// (j = -1 for the AAD, nb for the lengths block): one Shoup multiply per lane
// and a segmented XOR scan, so the per-record finish (the dominant cost of a
// record of a few blocks) is paid once per pack instead of once per record.
constexpr uint32_t kPackMaxNeed = 64;  // lanes; nb + 2 <= 64 keeps H^e within H^1..H^65
constexpr uint32_t kPackNone = 0xFFu;

// Lanes record descriptor word len_type needs in a pack, or kPackNone when it
// takes the single-record path (too long, or publicly invalid: parse_tls).
template <bool SEAL>
__device__ __forceinline__ uint32_t pack_need(uint32_t len_type, uint32_t tag_len) {
  const uint32_t len = len_type & 0xFFFFFFu;
  if (!SEAL && len < 8 + tag_len) return kPackNone;
  const uint32_t n = SEAL ? len : len - 8 - tag_len;
  const uint32_t nb = (n + 15) >> 4;
  return nb + 2 <= kPackMaxNeed ? nb + 2 : kPackNone;
}

// k records of one session S (each pack_need() <= 64, sum <= 64 lanes): lane
// i < k holds record index `rec` and its pack_need `need`.  Same outputs, status and
// zero-fill as parse_tls + gcm_record_x4 record by record (t1_enc.c:832-975).
template <bool SEAL, int ROUNDS>
__device__ void gcm_pack(const BatchArgs& a, const RecPre* __restrict__ pre, uint32_t rec, uint32_t k,
                         const DevSession* __restrict__ S, uint32_t lane, uint32_t laneoff,
                         uint32_t need) {
  const tlsgpu_record* D = reinterpret_cast<const tlsgpu_record*>(a.descs);
  cu32* rk = as_const(S->rk);
  cu32* rkr = as_const(S->rk_rot);
  const uint32_t tag_len = as_const(&S->tag_len)[0];
  const uint32_t version = as_const(&S->version)[0];
  // lane layout: exclusive prefix sum of the needs
  const uint32_t own = lane < k ? need : 0u;
#ifndef TG_PACK_SHFL_SCAN
  const uint32_t incl = wave_scan_add(own);  // DPP (aes_common.h)
#else
  uint32_t incl = own;
#pragma unroll
  for (int d = 1; d < kWave; d <<= 1) {
    const uint32_t t = __shfl_up(incl, d);
    if (lane >= (uint32_t)d) incl += t;
  }
#endif
  const uint32_t base_of = incl - own;  // lane i < k: first lane of record r0 + i
  uint32_t ri = 0;
  for (uint32_t i = 1; i < k; i++) ri += __builtin_amdgcn_readlane(base_of, i) <= lane ? 1u : 0u;
  const uint32_t total = __builtin_amdgcn_readlane(incl, k - 1);
  const bool used = lane < total;
  const uint32_t base = __shfl(base_of, (int)ri);
  const uint32_t rneed = __shfl(need, (int)ri);
  const uint32_t nb = rneed - 2;
  const int32_t j = (int32_t)lane - (int32_t)base - 1;  // -1: AAD, nb: lengths block
  const uint32_t r = __shfl(rec, (int)ri);  // ri < k: always a record of the pack

  const tlsgpu_record d = D[r];
  const uint32_t len = d.len_type & 0xFFFFFFu;
  const uint8_t* ip = a.in + d.in_off;
  uint8_t* op = a.out + d.out_off;
  const uint32_t n = SEAL ? len : len - 8 - tag_len;
  const uint8_t* src = SEAL ? ip : ip + 8;
  uint8_t* dst = SEAL ? op + 8 : op;
  const uint4* P = reinterpret_cast<const uint4*>(pre + r);
  const uint4 p0 = P[0], p1 = P[1], p2 = P[2];
  RecConsts rcc;
  rcc.ek0[0] = p0.x; rcc.ek0[1] = p0.y; rcc.ek0[2] = p0.z; rcc.ek0[3] = p0.w;
  rcc.k1a = p1.x; rcc.k1b = p1.y;
  rcc.k2[0] = p1.z; rcc.k2[1] = p1.w; rcc.k2[2] = p2.x; rcc.k2[3] = p2.y;

  // this lane's element (BE words) and, for a data block, its output block
  const bool blk = used && j >= 0 && (uint32_t)j < nb;
  const uint32_t jb = blk ? (uint32_t)j : 0u;
  const uint32_t nbytes = blk ? min(16u, n - 16u * jb) : 0u;
  const bool aligned = ((((uintptr_t)(src + 16u * jb)) | ((uintptr_t)(dst + 16u * jb))) & 15) == 0;
  uint32_t in[4] = {0, 0, 0, 0}, ks[4];
  if (blk) load_block(src + 16u * jb, nbytes, aligned, in);
  uint32_t tagw[4] = {0, 0, 0, 0};  // open: received tag (lengths lane)
  const bool last = used && j == (int32_t)nb;
  if (!SEAL && last) {
    const uint8_t* t = src + n;
    if (tag_len == 16) {
      load16_any(t, tagw);
    } else {
      for (uint32_t b = 0; b < tag_len; b++) tagw[b >> 2] |= (uint32_t)t[b] << (8 * (b & 3));
    }
  }
  aes_ctr16<ROUNDS>(ks, 2u + jb, rcc, rk[3], rk, rkr, laneoff);  // inc32(J0) = 2 (TLS J0)
#pragma unroll
  for (int w = 0; w < 4; w++) {
    const int32_t b = (int32_t)nbytes - 4 * w;
    ks[w] &= b >= 4 ? 0xFFFFFFFFu : (b <= 0 ? 0u : ((1u << (8 * b)) - 1u));
  }
  const uint32_t ob[4] = {in[0] ^ ks[0], in[1] ^ ks[1], in[2] ^ ks[2], in[3] ^ ks[3]};
  uint32_t e[4];
  if (blk) {
    const uint32_t* c = SEAL ? ob : in;
    e[0] = bswap32(c[0]); e[1] = bswap32(c[1]); e[2] = bswap32(c[2]); e[3] = bswap32(c[3]);
  } else if (j == -1) {  // AAD = seq || type || version || length (t1_enc.c:841-847,961-962)
    e[0] = (uint32_t)(d.seq >> 32);
    e[1] = (uint32_t)d.seq;
    e[2] = ((d.len_type >> 24) << 24) | ((version & 0xFFFF) << 8) | ((n >> 8) & 0xFF);
    e[3] = (n & 0xFF) << 24;
  } else {  // lengths block: BE64(13 * 8) || BE64(n * 8)
    e[0] = 0; e[1] = 13u * 8u;
    e[2] = (uint32_t)(((uint64_t)n * 8) >> 32); e[3] = (uint32_t)((uint64_t)n * 8);
  }
  // open stores its plaintext now too and overwrites it with zeros below when
  // the record's tag fails (as gcm_record's zero_len fill): ob is not held
  // live through the multiply
  if (blk) store_block(dst + 16u * jb, nbytes, aligned, ob);
  if (SEAL && used && j == -1) {
    for (int b = 0; b < 8; b++) op[b] = (uint8_t)(d.seq >> (56 - 8 * b));  // explicit nonce
  }
  // y = E_j * H^(nb + 1 - j), then the per-record XOR: inclusive scan, minus
  // the scan value just before the record's first lane
  uint32_t y[4];
  mul_shoup(e, used ? (uint32_t)((int32_t)nb + 1 - j) : 1u, y);
#pragma unroll
  for (int w = 0; w < 4; w++) y[w] = used ? y[w] : 0u;
#ifndef TG_PACK_SHFL_SCAN
#pragma unroll
  for (int w = 0; w < 4; w++) y[w] = wave_scan_xor(y[w]);
#else
#pragma unroll
  for (int dd = 1; dd < kWave; dd <<= 1) {
#pragma unroll
    for (int w = 0; w < 4; w++) {
      const uint32_t t = __shfl_up(y[w], dd);
      if (lane >= (uint32_t)dd) y[w] ^= t;
    }
  }
#endif
  uint32_t tag[4];
#pragma unroll
  for (int w = 0; w < 4; w++) {
    const uint32_t before = __shfl(y[w], (int)(base == 0 ? 0 : base - 1));
    tag[w] = bswap32(y[w] ^ (base == 0 ? 0u : before)) ^ rcc.ek0[w];
  }
  uint32_t bad = 0;
  if (last) {
    int32_t* slot = a.status + r;
    if (SEAL) {
      uint8_t* to = dst + n;
      if (tag_len == 16) {
        store16_any(to, tag);
      } else {
        for (uint32_t b = 0; b < tag_len; b++) to[b] = (uint8_t)(tag[b >> 2] >> (8 * (b & 3)));
      }
      *slot = (int32_t)(len + 8 + tag_len);
    } else {
      uint32_t diff = 0;
#pragma unroll
      for (int w = 0; w < 4; w++) {
        const int32_t b = (int32_t)tag_len - 4 * w;
        const uint32_t keep = b >= 4 ? 0xFFFFFFFFu : (b <= 0 ? 0u : ((1u << (8 * b)) - 1u));
        diff |= (tag[w] ^ tagw[w]) & keep;  // every byte compared (timingsafe_memcmp)
      }
      bad = diff != 0 ? 1u : 0u;
      *slot = bad ? TLSGPU_REC_BAD_MAC : (int32_t)n;
    }
  }
  if (!SEAL) {  // plaintext, or zeros when the record's tag failed (evp_aead.c:137-143)
    const uint32_t rbad = __shfl(bad, (int)(base + rneed - 1));
    if (blk && rbad) {
      const uint32_t z[4] = {0, 0, 0, 0};
      store_block(dst + 16u * jb, nbytes, aligned, z);
    }
  }
}

__device__ __forceinline__ uint32_t queue_take(uint32_t* q, uint32_t k, uint32_t lane) {
  uint32_t r = 0;
  if (lane == 0) r = atomicAdd(q, k);
  return __builtin_amdgcn_readfirstlane(r);
}

// The prep pass's selection words, summed over the kSelSlots cache lines
// (s_load: wave-uniform).
struct SelSums {
  uint32_t pack, runs, recs;
};
__device__ __forceinline__ SelSums sel_sums(const uint32_t* sel) {
  cu32* f = as_const(sel);
  SelSums t = {0, 0, 0};
#pragma unroll
  for (int i = 0; i < kSelSlots; i++) {
    t.pack |= f[kSelWords * i];
    t.runs += f[kSelWords * i + 1];
    t.recs += f[kSelWords * i + 2];
  }
  return t;
}

// Per-record constants of one record (the body of gcm_prep_kernel; rec_consts
// in gcm_device.h): E_K(J0), the round-1 columns 0, 1 and the round-2
// constants.  T0 / T1 / SB: Te0, Te1 and S-box lookups of byte b of w.
template <bool SEAL, int ROUNDS, typename RK, typename T0F, typename T1F, typename SBF>
__device__ __forceinline__ RecPre rec_pre(const uint32_t j0[4], RK rk, T0F T0, T1F T1, SBF SB) {
  uint32_t s[4] = {j0[0] ^ rk[0], j0[1] ^ rk[1], j0[2] ^ rk[2], j0[3] ^ rk[3]};
#pragma unroll
  for (int rr = 1; rr < ROUNDS; rr++) {
    uint32_t t[4];
#pragma unroll
    for (int c = 0; c < 4; c++)
      t[c] = T0(s[c], 0) ^ T1(s[(c + 1) & 3], 1) ^
             rotl32(T0(s[(c + 2) & 3], 2) ^ T1(s[(c + 3) & 3], 3), 16) ^ rk[4 * rr + c];
#pragma unroll
    for (int c = 0; c < 4; c++) s[c] = t[c];
  }
  RecPre o;
#pragma unroll
  for (int c = 0; c < 4; c++)
    o.ek0[c] = (SB(s[c], 0) | (SB(s[(c + 1) & 3], 1) << 8) | (SB(s[(c + 2) & 3], 2) << 16) |
                (SB(s[(c + 3) & 3], 3) << 24)) ^ rk[4 * ROUNDS + c];
  const uint32_t s0 = j0[0] ^ rk[0], s1 = j0[1] ^ rk[1], s2 = j0[2] ^ rk[2];
  uint32_t k1[4];
  k1[0] = T0(s0, 0) ^ T1(s1, 1) ^ rotl32(T0(s2, 2), 16) ^ rk[4];
  k1[1] = T0(s1, 0) ^ T1(s2, 1) ^ rotl32(T1(s0, 3), 16) ^ rk[5];
  k1[2] = T0(s2, 0) ^ rotl32(T0(s0, 2) ^ T1(s1, 3), 16) ^ rk[6];
  k1[3] = T1(s0, 1) ^ rotl32(T0(s1, 2) ^ T1(s2, 3), 16) ^ rk[7];
  const uint32_t v0 = rk[3];
  const uint32_t c2 = k1[2] ^ T1(v0, 1), c3 = k1[3] ^ T0(v0, 0);  // round-1 columns 2, 3
  o.k1a = k1[0];
  o.k1b = k1[1];
  o.k2[0] = rotl32(T0(c2, 2) ^ T1(c3, 3), 16) ^ rk[8];
  o.k2[1] = T1(c2, 1) ^ rotl32(T0(c3, 2), 16) ^ rk[9];
  o.k2[2] = T0(c2, 0) ^ T1(c3, 1) ^ rk[10];
  o.k2[3] = T0(c3, 0) ^ rotl32(T1(c2, 3), 16) ^ rk[11];
  o.sb2[0] = SB(c2, 0) | (SB(c2, 1) << 8) | (SB(c2, 2) << 16) | (SB(c2, 3) << 24);
  o.sb2[1] = SB(c3, 0) | (SB(c3, 1) << 8) | (SB(c3, 2) << 16) | (SB(c3, 3) << 24);
  return o;
}

// Fused prologue (round 5): what check_record_bounds
// and gcm_prep_kernel did in two launches before this kernel, for the
// workgroup's own records [rlo, rhi), one thread per record: the bounds check
// and initial status (TLSGPU_REC_OUT_OF_BOUNDS / _PUBLIC_INVALID, the status of
// a record no kernel takes), and the per-record constants of every record this
// kernel will run, into `pre`.  The T-tables are already in LDS (fill_aes_lds:
// row x = 32 bank copies of Te0[x], then 32 of Te1[x]).  Only used when this
// kernel is the batch's only one (one AES key size installed, no ChaCha, no
// pack / per-wave-session variants: engine.cpp run_batch), so every status
// write here precedes this workgroup's own final one (barrier below).
// `nrec` records, the L-th of them record map(L) (one range, or the
// workgroup's whole pieces: one pass over all of them).
template <bool SEAL, int ROUNDS, int NT, typename MAP>
__device__ void fused_prologue_map(const BatchArgs& a, RecPre* __restrict__ pre, uint32_t nrec,
                                   MAP map) {
  const tlsgpu_record* D = reinterpret_cast<const tlsgpu_record*>(a.descs);
  const uint32_t* te = reinterpret_cast<const uint32_t*>(s_lds + AES_OFF);
  const uint32_t l32 = threadIdx.x & 31;
  auto T0 = [&](uint32_t w, int b) { return te[(((w >> (8 * b)) & 0xFF) << 6) | l32]; };
  auto T1 = [&](uint32_t w, int b) { return te[(((w >> (8 * b)) & 0xFF) << 6) | 32 | l32]; };
  auto SB = [&](uint32_t w, int b) { return (T0(w, b) >> 8) & 0xFF; };
  for (uint32_t base = 0; base < nrec; base += NT) {  // wave-uniform trip count
    const uint32_t L = base + threadIdx.x;
    const uint32_t r = L < nrec ? map(L) : 0u;
    bool mine = false;
    tlsgpu_record d = {};
    const DevSession* S = nullptr;
    if (L < nrec) {
      d = D[r];
      int32_t st = TLSGPU_REC_PUBLIC_INVALID;
      if (d.session < a.n_sessions) {
        S = a.sessions + d.session;
        if (!rec_in_bounds(d, S, a.in_bytes, a.out_bytes, SEAL)) st = TLSGPU_REC_OUT_OF_BOUNDS;
        else mine = is_gcm(S->kind) && (int)S->rounds == ROUNDS;
      }
      a.status[r] = st;
    }
    const uint32_t sid0 = __builtin_amdgcn_readfirstlane(mine ? d.session : 0xFFFFFFFFu);
    const bool uniform = !__any(mine && d.session != sid0);
    if (!mine) continue;
    uint32_t j0[4];
    j0[0] = *reinterpret_cast<const uint32_t*>(S->fixed_nonce);
    j0[1] = j0[2] = 0;
    j0[3] = 0x01000000u;
    if (SEAL) {
      j0[1] = bswap32((uint32_t)(d.seq >> 32));
      j0[2] = bswap32((uint32_t)d.seq);
    } else if ((d.len_type & 0xFFFFFFu) >= 8) {
      const uint8_t* p = a.in + d.in_off;
      j0[1] = load_u32_bytes(p);
      j0[2] = load_u32_bytes(p + 4);
    }
    pre[r] = uniform ? rec_pre<SEAL, ROUNDS>(j0, as_const(a.sessions[sid0].rk), T0, T1, SB)
                     : rec_pre<SEAL, ROUNDS>(j0, S->rk, T0, T1, SB);
  }
  __threadfence_block();  // the statuses and constants before this workgroup's main loop
}

template <bool SEAL, int ROUNDS, int NT>
__device__ __forceinline__ void fused_prologue(const BatchArgs& a, RecPre* __restrict__ pre,
                                               uint32_t rlo, uint32_t rhi) {
  fused_prologue_map<SEAL, ROUNDS, NT>(a, pre, rhi > rlo ? rhi - rlo : 0u,
                                       [&](uint32_t L) { return rlo + L; });
}

// Inclusive prefix sum of one value per thread over the workgroup, and the
// total; `tmp` holds NT/64 words of LDS.  Every thread calls it.
template <int NT>
__device__ uint64_t block_scan_incl(uint64_t v, uint64_t* tmp, uint64_t* total) {
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (uint32_t d = 1; d < 64; d <<= 1) {
    const uint64_t u = __shfl_up(v, d);
    if (lane >= d) v += u;
  }
  if (lane == 63) tmp[wave] = v;
  __syncthreads();
  uint64_t off = 0, tot = 0;
  for (uint32_t w = 0; w < (uint32_t)NT / 64; w++) {
    const uint64_t t = tmp[w];
    off += w < wave ? t : 0;
    tot += t;
  }
  __syncthreads();  // tmp is reused by the next scan
  *total = tot;
  return v + off;
}

// Work-balanced ranges (round 5, a.cut_work): cut k of gridDim.x is the first
// record i whose work prefix W(i) = sum_{j<i} cut_work_of(D[j]) reaches
// total * k / G.  W is strictly increasing (every weight > 0), so the cuts are
// non-decreasing with cut(0) = 0 and cut(G) = n, and the two workgroups that
// share a cut compute it from the same sums: the ranges partition the batch.
// The count-range sums (range_work_kernel) locate the range the cut falls in;
// a scan of that range's records finds the record.  LDS: PLAN_OFF (free
// until the main loop).
template <int NT>
__device__ uint32_t work_cut(const BatchArgs& a, uint32_t k) {
  const uint32_t G = gridDim.x;
  if (k == 0) return 0;
  if (k >= G) return a.n;
  const tlsgpu_record* D = reinterpret_cast<const tlsgpu_record*>(a.descs);
  uint64_t* tmp = reinterpret_cast<uint64_t*>(s_lds + PLAN_OFF);
  uint64_t* res = tmp + NT / 64;  // [0] range, [1] work before it, [2] the cut
  const uint64_t v = threadIdx.x < G ? a.cut_work[threadIdx.x] : 0;
  uint64_t total;
  const uint64_t incl = block_scan_incl<NT>(v, tmp, &total);
  const uint64_t target = total * k / G;  // >= 1: total >= 256 n >= G
  if (threadIdx.x < G && incl - v < target && target <= incl) {
    res[0] = threadIdx.x;
    res[1] = incl - v;
  }
  __syncthreads();
  const uint32_t q = (uint32_t)res[0];
  uint64_t base = res[1];
  const uint32_t lo = q * a.records_per_group, hi = min(a.n, lo + a.records_per_group);
  for (uint32_t c = lo; c < hi; c += NT) {  // workgroup-uniform trip count
    const uint32_t i = c + threadIdx.x;
    const uint64_t w = i < hi ? cut_work_of(D[i].len_type) : 0;
    uint64_t tot;
    const uint64_t in = block_scan_incl<NT>(w, tmp, &tot);
    if (i < hi && base + in - w < target && target <= base + in) res[2] = i + 1;
    base += tot;
  }
  __syncthreads();
  uint32_t cut = (uint32_t)res[2];
  if (a.cut_snap != 0 && cut > 0 && cut < a.n) {
    // Snap to the nearest session-run boundary when one lies within
    // a.cut_snap / 1024 of a workgroup's share of the work (a split run costs
    // both workgroups a table build, a plan and a run-end wait): rs = the last
    // boundary <= cut, re = the first >= cut, each looked for within NT
    // records.  Monotone in the target — two targets in one run find the same
    // boundaries and the nearer-boundary rule never crosses them over — so
    // the cuts still partition the batch.
    const uint32_t i = cut;
    uint32_t* bnd = reinterpret_cast<uint32_t*>(res + 3);  // [0] i - rs, [1] re - i
    if (threadIdx.x < 2) bnd[threadIdx.x] = 0xFFFFFFFFu;
    __syncthreads();
    const uint32_t t = threadIdx.x;
    if (t < i) {  // p = i - t; a boundary at p: D[p - 1] and D[p] in different sessions
      const uint32_t p = i - t;
      if (D[p].session != D[p - 1].session) atomicMin(bnd, t);
    } else if (t == i) {
      atomicMin(bnd, t);  // p = 0
    }
    if (i + t <= a.n) {
      const uint32_t p = i + t;
      if (p == a.n || D[p].session != D[p - 1].session) atomicMin(bnd + 1, t);
    }
    __syncthreads();
    const uint32_t dlr = bnd[0], drr = bnd[1];
    const uint64_t wl = t < dlr && dlr != 0xFFFFFFFFu ? cut_work_of(D[i - 1 - t].len_type) : 0;
    const uint64_t wr = t < drr && drr != 0xFFFFFFFFu ? cut_work_of(D[i + t].len_type) : 0;
    uint64_t dl, dr;
    (void)block_scan_incl<NT>(wl, tmp, &dl);
    (void)block_scan_incl<NT>(wr, tmp, &dr);
    const uint64_t thr = total / G * a.cut_snap / 1024;
    const bool has_l = dlr != 0xFFFFFFFFu, has_r = drr != 0xFFFFFFFFu;
    if (dlr != 0 && drr != 0) {  // not on a boundary already
      if (has_l && dl < thr && (!has_r || dl <= dr)) cut = i - dlr;
      else if (has_r && dr < thr && (!has_l || dr < dl)) cut = i + drr;
    }
  }
  __syncthreads();  // res is rewritten by the next call
  return cut;
}

// NT threads, the first BSW waves bitsliced (0: a pure T-table queue kernel,
// 16 waves of <= 128 VGPRs), T-table waves NB blocks wide; B16W > 0: the first
// B16W waves take the packed bitsliced role (hy_b16_record, one per SIMD for
// B16W = 4: waves go to the SIMDs in turn).
template <bool SEAL, int ROUNDS, int NT, int BSW, int NB, bool PACK = false, int B16W = 0>
__global__ __launch_bounds__(NT, 1) void gcm_hy_kernel(BatchArgs a,
                                                       const RecPre* __restrict__ pre) {
  // pack and no-pack variants are separate kernels (the pack code costs the
  // long-record loop SGPR spills), and the per-wave-session kernel replaces both
  // when session runs are short; the prep pass's selection words pick one
  if (a.sel) {
    const SelSums f = sel_sums(a.sel);
    if (pws_selected(a.pws, f.runs, f.recs)) return;
    if ((a.pack != 0 && f.pack != 0) != PACK) return;
  } else if (PACK != (a.fused != 0 && a.pack != 0)) {
    // no selection words: the no-pack variant, or (fused, packs allowed by the
    // hints) only the pack variant is launched
    return;
  }
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t laneoff = aes_laneoff(lane);
  const GhLane gl = gh_lane(lane);
  const tlsgpu_record* D = reinterpret_cast<const tlsgpu_record*>(a.descs);
  const bool bs_role = wave < (uint32_t)BSW;
  if (BSW && !bs_role) __builtin_amdgcn_s_setprio(1);
  const bool b16_role = B16W > 0 && wave < (uint32_t)B16W;
  if (B16W > 0 && !b16_role && !(a.hy_flags & 8u)) __builtin_amdgcn_s_setprio(1);
  uint32_t* q = reinterpret_cast<uint32_t*>(s_lds + Q_OFF);

  if (a.wg_times && threadIdx.x == 0) a.wg_times[4 * blockIdx.x] = __builtin_amdgcn_s_memrealtime();
  fill_aes_lds<NT>();
  if (a.dbg && threadIdx.x < 32) reinterpret_cast<unsigned long long*>(s_lds + DBG_OFF)[threadIdx.x] = 0;

  // whole pieces sorted by work (a.pieces, written by piece_sort_kernel: a
  // vector load), else this workgroup's count range (or work cuts)
  const uint32_t n_pieces =
      a.pieces ? __builtin_amdgcn_readfirstlane(*reinterpret_cast<const volatile uint32_t*>(a.n_pieces))
               : 0u;
  // piece m of this workgroup: false when it has no more
  auto piece = [&](uint32_t m, uint32_t& rlo, uint32_t& rhi) -> bool {
    if (n_pieces != 0) {
      const uint32_t G = gridDim.x;
      const uint32_t idx = m * G + ((m & 1u) ? G - 1u - blockIdx.x : blockIdx.x);
      if (idx >= n_pieces) return false;
      // vector loads (the plan was written by the previous kernel)
      const volatile uint32_t* pw = reinterpret_cast<const volatile uint32_t*>(a.pieces + idx);
      rlo = __builtin_amdgcn_readfirstlane(pw[0]);
      rhi = __builtin_amdgcn_readfirstlane(pw[1]);
      return true;
    }
    if (m != 0) return false;
    rlo = blockIdx.x * a.records_per_group;
    rhi = min(a.n, rlo + a.records_per_group);
    return true;
  };
  uint32_t rlo = 0, rhi = 0;
  if (BSW == 0 && B16W == 0 && a.fused) {
    __syncthreads();  // the T-tables
    if (a.cut_work) {  // work-balanced ranges (engine.cpp run_batch)
      rlo = work_cut<NT>(a, blockIdx.x);
      rhi = work_cut<NT>(a, blockIdx.x + 1);
      fused_prologue<SEAL, ROUNDS, NT>(a, const_cast<RecPre*>(pre), rlo, rhi);
    } else if (n_pieces == 0) {
      piece(0, rlo, rhi);
      fused_prologue<SEAL, ROUNDS, NT>(a, const_cast<RecPre*>(pre), rlo, rhi);
    } else {
      // the workgroup's pieces (at most kPiecesPerRange: n_pieces <= that
      // many per workgroup) into LDS, then one prologue pass over all of them
      uint32_t* pl = reinterpret_cast<uint32_t*>(s_lds + PLAN_OFF + 512);
      if (threadIdx.x < kPiecesPerRange) {
        const uint32_t t = threadIdx.x, G = gridDim.x;
        const uint32_t idx = t * G + ((t & 1u) ? G - 1u - blockIdx.x : blockIdx.x);
        uint32_t lo = 0, hi = 0;
        if (idx < n_pieces) {
          const volatile uint32_t* pw = reinterpret_cast<const volatile uint32_t*>(a.pieces + idx);
          lo = pw[0];
          hi = pw[1];
        }
        pl[2 * t] = lo;
        pl[2 * t + 1] = hi;
      }
      __syncthreads();
      uint32_t nrec = 0;
      for (uint32_t k = 0; k < kPiecesPerRange; k++) nrec += pl[2 * k + 1] - pl[2 * k];
      fused_prologue_map<SEAL, ROUNDS, NT>(a, const_cast<RecPre*>(pre), nrec, [&](uint32_t L) {
        uint32_t k = 0;
        for (; k + 1 < kPiecesPerRange; k++) {
          const uint32_t len = pl[2 * k + 1] - pl[2 * k];
          if (L < len) break;
          L -= len;
        }
        return pl[2 * k] + L;
      });
    }
  }
  if (a.wg_times) {  // diagnostic: the workgroup's records and work
    uint64_t recs = 0, work = 0;
    for (uint32_t m = 0; a.cut_work ? m == 0 : piece(m, rlo, rhi); m++) {
      for (uint32_t c = rlo; c < rhi; c += NT) {
        const uint32_t i = c + threadIdx.x;
        uint64_t t;
        (void)block_scan_incl<NT>(i < rhi ? cut_work_of(D[i].len_type) : 0u,
                                  reinterpret_cast<uint64_t*>(s_lds + PLAN_OFF), &t);
        work += t;
      }
      recs += rhi - rlo;
    }
    if (threadIdx.x == 0) {
      a.wg_times[4 * blockIdx.x + 2] = recs;
      a.wg_times[4 * blockIdx.x + 3] = work;
    }
  }
  uint32_t cur = 0xFFFFFFFFu;
  // one loop over the workgroup's pieces and their session runs
  uint32_t m = 0;
  if (!a.cut_work && !piece(0, rlo, rhi)) rlo = rhi = 0;
  uint32_t pos = rlo;
  // short-record packs (gcm_pack): T-table waves only, planned per run in LDS
  const bool packing = PACK && BSW == 0 && a.pack != 0;
  // the run in claim order: long records first (run-relative index order[t]),
  // then the short ones, packed greedily (plan_k[t] records from position t)
  uint16_t* order = reinterpret_cast<uint16_t*>(s_lds + PLAN_OFF);
  uint8_t* plan_need = s_lds + PLAN_OFF + 2 * kPlanCap;  // pack_need of order[t]
  uint8_t* plan_k = plan_need + kPlanCap;
  uint32_t* ends = q + 1;  // [0]: next long slot (from the front), [1]: short slots (from the back)
  for (;;) {
    if (pos >= rhi) {  // the next piece
      if (a.cut_work || !piece(++m, rlo, rhi)) break;
      pos = rlo;
      continue;
    }
    const uint32_t sid = __builtin_amdgcn_readfirstlane(D[pos].session);
    const bool in_range = sid < a.n_sessions;
    const DevSession* __restrict__ S = a.sessions + (in_range ? sid : 0);
    const uint32_t tag_len = as_const(&S->tag_len)[0];
    const uint32_t run_cap = packing ? min(rhi, pos + kPlanCap) : rhi;
    bool has_short = packing && pack_need<SEAL>(as_const(&D[pos].len_type)[0], tag_len) <= kPackMaxNeed;
    uint32_t run_end = pos + 1;
    // the run's end: 4 x 64 descriptors per memory round trip (the scan is
    // on the run-to-run critical path of the wave that finished last; round 5,
    // same-box A/B against one 64-record step per trip: B +0.3 %, D +0.2 %,
    // profiles/r05j_ab_run_scan.txt)
    while (run_end < run_cap) {
      uint32_t s[4], lt[4];
#pragma unroll
      for (uint32_t u = 0; u < 4; u++) {
        const uint32_t p = run_end + 64u * u + lane;
        s[u] = p < run_cap ? D[p].session : sid;
        lt[u] = packing && p < run_cap ? D[p].len_type : 0u;
      }
      uint32_t found = 0xFFFFFFFFu;
#pragma unroll
      for (uint32_t u = 0; u < 4; u++) {
        const uint32_t p = run_end + 64u * u + lane;
        if (packing)  // a hint only: records past the run's end may count
          has_short |= __ballot(p < run_cap && s[u] == sid &&
                                pack_need<SEAL>(lt[u], tag_len) <= kPackMaxNeed) != 0;
        const uint64_t diff = __ballot(p < run_cap && s[u] != sid);
        if (diff && found == 0xFFFFFFFFu)
          found = 64u * u + __builtin_amdgcn_readfirstlane((uint32_t)__builtin_ctzll(diff));
      }
      if (found != 0xFFFFFFFFu) { run_end += found; break; }
      run_end = min(run_cap, run_end + 256);
    }
    const uint32_t kind = as_const(&S->kind)[0];
    const bool usable = in_range && is_gcm(kind) && (int)as_const(&S->rounds)[0] == ROUNDS;
    if (usable) {
      PhaseClock pc(a.dbg);
      __syncthreads();  // every wave is done with the previous run (queue, tables, plan)
      pc.lap(bs_role ? 4 : 12, lane);
      if (threadIdx.x == 0) *q = pos;
      if (sid != cur) load_session_tables<NT>(a.gcm_tables + sid);
      cur = sid;
      const uint32_t run_len = run_end - pos;
      if (has_short) {  // the plan: greedy pack from every start, <= 64 lanes, <= 32 records
        if (threadIdx.x == 0) { ends[0] = 0; ends[1] = run_len; }
        __syncthreads();
        for (uint32_t c = wave * kWave; c < run_len; c += NT) {  // ballot compaction per wave
          const uint32_t t = c + lane;
          const uint32_t nd = t < run_len ? pack_need<SEAL>(D[pos + t].len_type, tag_len) : 0u;
          // fused: an out-of-bounds record takes the long-record path, which
          // skips it (its status was written by the prologue)
          const bool sh = t < run_len && nd <= kPackMaxNeed &&
                          (!a.fused || rec_in_bounds(D[pos + t], S, a.in_bytes, a.out_bytes, SEAL));
          const uint64_t lm = __ballot(t < run_len && !sh), sm = __ballot(sh);
          uint32_t fb = 0, bb = 0;
          if (lane == 0) {
            fb = atomicAdd(ends, (uint32_t)__builtin_popcountll(lm));
            bb = atomicSub(ends + 1, (uint32_t)__builtin_popcountll(sm)) -
                 (uint32_t)__builtin_popcountll(sm);
          }
          fb = __builtin_amdgcn_readfirstlane(fb);
          bb = __builtin_amdgcn_readfirstlane(bb);
          const uint64_t below = (1ull << lane) - 1ull;
          if (t < run_len) {
            const uint32_t at = sh ? bb + (uint32_t)__builtin_popcountll(sm & below)
                                   : fb + (uint32_t)__builtin_popcountll(lm & below);
            order[at] = (uint16_t)t;
            // a record left out of the packs (long, or fused and out of
            // bounds) never starts or joins one: kPackNone stops plan_k
            plan_need[at] = (uint8_t)(sh ? nd : kPackNone);
          }
        }
        __syncthreads();
        for (uint32_t t = threadIdx.x; t < run_len; t += NT) {
          uint32_t k = 0, sum = 0;
          for (; k < 32 && t + k < run_len; k++) {
            const uint32_t nd = plan_need[t + k];
            if (sum + nd > kPackMaxNeed) break;
            sum += nd;
          }
          plan_k[t] = (uint8_t)k;
        }
        pc.lap(15, lane);
      }
      __syncthreads();
      pc.lap(5, lane);
      const bool idle = (a.hy_flags & (bs_role ? 4u : 2u)) != 0;
      for (; !idle;) {
        if (BSW && bs_role) {
          const uint32_t r = queue_take(q, 2, lane);
          if (r >= run_end) break;
          const uint32_t rb = r + 1;
          if (rb < run_end && run_end - r >= a.bs_reserve && !(a.hy_flags & 1u)) {
            RecCtx rc[2];
            const bool oka = parse_tls<SEAL>(load_desc(D + r), S, a.in, a.out, a.status + r, lane,
                                             rc[0]);
            const bool okb = parse_tls<SEAL>(load_desc(D + rb), S, a.in, a.out, a.status + rb,
                                             lane, rc[1]);
            if (oka && okb && rc[0].n >= 16384 && rc[1].n >= 16384 &&
                (((uintptr_t)rc[0].src | (uintptr_t)rc[0].dst | (uintptr_t)rc[1].src |
                  (uintptr_t)rc[1].dst) & 15) == 0) {
              gcm_pair_hy<SEAL, ROUNDS>(rc, pre + r, pre + rb, a.status + r, a.status + rb, S,
                                        lane, laneoff, gl, a.dbg);
            } else {
              for (uint32_t m = 0; m < 2; m++) {
                if (!(m ? okb : oka)) continue;
                const RecConsts rcc = rec_consts_of(pre + r + m);
                gcm_record_x4<SEAL, ROUNDS, NB>(m ? rc[1] : rc[0], S, rcc, a.status + r + m, lane,
                                            laneoff, gl);
              }
            }
          } else {
            hy_tt_record<SEAL, ROUNDS, NB>(a, pre, r, S, lane, laneoff, gl);
            if (rb < run_end) hy_tt_record<SEAL, ROUNDS, NB>(a, pre, rb, S, lane, laneoff, gl);
          }
        } else {
          uint32_t r;
          if (B16W > 0 && b16_role) {
            r = queue_take(q, 1, lane);
            if (r >= run_end) break;
            if (hy_b16_record<SEAL, ROUNDS>(a, pre, r, run_end - r, S, lane, laneoff, gl)) continue;
          } else if (has_short) {
            // claim the pack the plan starts at the queue head (k = 0: a long
            // record alone); the CAS window is two LDS operations
            uint32_t k = 0;
            for (;;) {
              r = __builtin_amdgcn_readfirstlane(__atomic_load_n(q, __ATOMIC_RELAXED));
              if (r >= run_end) break;
              k = plan_k[r - pos];
              uint32_t got = 0;
              if (lane == 0) got = atomicCAS(q, r, r + (k ? k : 1u));
              if (__builtin_amdgcn_readfirstlane(got) == r) break;
            }
            if (r >= run_end) break;
            if (k != 0) {
              PhaseClock pp(a.dbg);
              const uint32_t li = r - pos + min(lane, k - 1);
              const uint32_t need = lane < k ? (uint32_t)plan_need[li] : kPackNone;
              gcm_pack<SEAL, ROUNDS>(a, pre, pos + order[li], k, S, lane, laneoff, need);
              pp.lap(13, lane);
              if (a.dbg && lane == 0) {  // phase slot 14: records per pack (diagnostic)
                unsigned long long* c = reinterpret_cast<unsigned long long*>(s_lds + DBG_OFF);
                atomicAdd(c + 28, (unsigned long long)k);
                atomicAdd(c + 29, 1ull);
              }
              continue;
            }
            r = pos + order[r - pos];
          } else {
            r = queue_take(q, 1, lane);
            if (r >= run_end) break;
          }
#ifndef TG_NO_TAIL_PRIO
          // the run's last claims finish last: issue priority by claim order
          // over the final records, so the run's tail ends together instead of
          // one straggler per SIMD running alone before the barrier
          const uint32_t left = run_end - r;
#ifndef TG_TAIL_WIN
#define TG_TAIL_WIN 3  // tail window in claims of kWaves records (A/B: TG_TAIL_WIN=2/4)
#endif
          if (!BSW && !PACK && left <= TG_TAIL_WIN * kWaves) {
            if (left <= kWaves) __builtin_amdgcn_s_setprio(3);
            else if (left <= 2 * kWaves) __builtin_amdgcn_s_setprio(2);
            else __builtin_amdgcn_s_setprio(1);
          }
#endif
          hy_tt_record<SEAL, ROUNDS, NB>(a, pre, r, S, lane, laneoff, gl);
#ifndef TG_NO_TAIL_PRIO
          if (!BSW && !PACK) __builtin_amdgcn_s_setprio(0);
#endif
        }
      }
    }
    pos = run_end;
  }
  if (a.dbg) {
    __syncthreads();
    if (threadIdx.x < 32)
      atomicAdd(a.dbg + threadIdx.x, reinterpret_cast<unsigned long long*>(s_lds + DBG_OFF)[threadIdx.x]);
  }
  if (a.wg_times) {  // diagnostic: when the workgroup's last wave is done, its records and work
    __syncthreads();
    if (threadIdx.x == 0) a.wg_times[4 * blockIdx.x + 1] = __builtin_amdgcn_s_memrealtime();
  }
}

// Per-record constants (RecPre) for the queue kernels, one thread per record.
// Follows rec_consts (gcm_device.h).  Te0 sits in LDS replicated over the 32
// banks of ds_read_b32 (row x, copy = lane % 32: conflict-free, 32 KiB; Te1 =
// rotl8(Te0)); the round keys come through s_load when the wave's records all
// belong to one session (the common case: sessions form runs), else per lane.
constexpr int kPrepThreads = 512;
template <bool SEAL, int ROUNDS>
__global__ __launch_bounds__(kPrepThreads) void gcm_prep_kernel(BatchArgs a,
                                                                RecPre* __restrict__ pre) {
  __shared__ uint32_t te[256 * 32];
  __shared__ uint32_t cnt[3];  // packable flag, run starts, records of this key size
  for (uint32_t q = threadIdx.x; q < 256 * 8; q += kPrepThreads) {
    const uint32_t v = g_te0.v[q >> 3];
    reinterpret_cast<uint4*>(te)[q] = make_uint4(v, v, v, v);
  }
  if (threadIdx.x < 3) cnt[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t r = blockIdx.x * kPrepThreads + threadIdx.x;
  const uint32_t l32 = threadIdx.x & 31;
  const tlsgpu_record* D = reinterpret_cast<const tlsgpu_record*>(a.descs);
  bool mine = false, run_start = false, packable = false;
  tlsgpu_record d = {};
  const DevSession* S = nullptr;
  if (r < a.n) {
    d = D[r];
    if (d.session < a.n_sessions) {
      S = a.sessions + d.session;
      mine = is_gcm(S->kind) && (int)S->rounds == ROUNDS;
      run_start = mine && (r == 0 || D[r - 1].session != d.session);
      packable = mine && pack_need<SEAL>(d.len_type, S->tag_len) <= kPackMaxNeed;
    }
  }
  // selection words (a.sel, SelSums): summed per wave (ballot), per workgroup
  // (LDS) and then added to one of kSelSlots cache lines — one global atomic
  // per workgroup and counter, spread over 16 addresses (same-address atomics
  // from every wave serialised at one L2 channel: 115 us of config D's step)
  if (a.sel) {
    const uint64_t m = __ballot(mine), rs = __ballot(run_start), pk = __ballot(packable);
    if ((threadIdx.x & 63) == 0 && m) {
      atomicAdd(&cnt[2], (uint32_t)__builtin_popcountll(m));
      atomicAdd(&cnt[1], (uint32_t)__builtin_popcountll(rs));
      if (pk) cnt[0] = 1u;
    }
    __syncthreads();
    if (threadIdx.x == 0 && cnt[2]) {
      uint32_t* slot = a.sel + kSelWords * (blockIdx.x % kSelSlots);
      atomicAdd(slot + 2, cnt[2]);
      atomicAdd(slot + 1, cnt[1]);
      if (cnt[0]) atomicOr(slot, 1u);
    }
  }
  const uint32_t sid0 = __builtin_amdgcn_readfirstlane(mine ? d.session : 0xFFFFFFFFu);
  const bool uniform = !__any(mine && d.session != sid0);
  if (!mine) return;
  auto T0 = [&](uint32_t w, int b) { return te[(((w >> (8 * b)) & 0xFF) << 5) | l32]; };
  auto T1 = [&](uint32_t w, int b) { return rotl32(T0(w, b), 8); };
  auto SB = [&](uint32_t w, int b) { return (T0(w, b) >> 8) & 0xFF; };
  uint32_t j0[4];
  j0[0] = *reinterpret_cast<const uint32_t*>(S->fixed_nonce);
  j0[1] = j0[2] = 0;
  j0[3] = 0x01000000u;
  if (SEAL) {
    j0[1] = bswap32((uint32_t)(d.seq >> 32));
    j0[2] = bswap32((uint32_t)d.seq);
  } else if ((d.len_type & 0xFFFFFFu) >= 8) {
    const uint8_t* p = a.in + d.in_off;
    j0[1] = load_u32_bytes(p);
    j0[2] = load_u32_bytes(p + 4);
  }
  auto body = [&](auto rk) { pre[r] = rec_pre<SEAL, ROUNDS>(j0, rk, T0, T1, SB); };
  if (uniform)
    body(as_const(a.sessions[sid0].rk));  // wave-uniform: round keys in SGPRs
  else
    body(S->rk);
}


}  // namespace tg
