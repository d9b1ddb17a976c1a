// gcm_fused.h — the fused AES-GCM TLS kernel.
//
// Every wave runs two pipelines in one instruction stream:
//   * a bitsliced record pair (gcm_hybrid.h: AES-CTR keystream of 2 x 1024
//     blocks as 128 bit planes, VALU only), and
//   * a T-table record ("TT record"), 1 block per lane per group, whose
//     AES rounds and GHASH steps are cut into phases: phase K runs after
//     S-box K of a bitsliced round, issues its LDS lookups there and combines
//     them one S-box (~85 VALU ops) later, so the LDS latency hides behind the
//     bitsliced work and the LDS pipe (idle in a pure bitsliced wave) and the
//     VALU (two thirds idle in a pure T-table wave) are both used.
// One TT group (64 blocks, one per lane) per bitsliced round: for AES-128 the
// 8 fused rounds of a pass (rounds 3..9 and the final round) carry half of a
// 16 KiB TT record per record pair.  TT record boundaries are handled after a pass's
// consume step, where the bitsliced state is dead.
#pragma once
#include "../csrc/gcm_hybrid.h"

namespace tg {

// TT record state carried across fused rounds and passes.
struct TtRec {
  RecCtx rc;
  RecConsts rcc;       // wave-uniform
  int32_t* slot;
  uint32_t ctr0;       // inc32(J0)
  uint32_t g, ng;      // next 2-step group, number of full groups (uniform)
  uint32_t x[4];       // this lane's GHASH chain (LE words)
  uint32_t c[4];       // ciphertext (open) / plaintext (seal) of group g (one block per lane)
  bool on;             // uniform: a TT record is in flight
};

// Per-round temporaries of the TT group (live between phases).  One block per
// lane and quarter-width GHASH steps keep this at ~40 VGPRs beside the 128
// bit planes (two blocks and half-width steps spilled in the round loop).
struct TtTmp {
  uint32_t A[4];       // AES state of the lane's block
  uint32_t t[16];      // lookups in flight
  uint32_t cn[4];      // next group's input, loaded at phase 0
  uint32_t gin[4];     // GHASH input of this group
  uint32_t y[4];       // rotated chain value for the GHASH lookups
  uint4 h[4];          // GHASH lookups in flight (a quarter of mul_k)
  uint32_t acc[4];
};

__device__ __forceinline__ void gh_rot(const uint32_t x[4], uint32_t y[4], const GhLane& g) {
  uint32_t a0 = g.c2 ? x[2] : x[0], a1 = g.c2 ? x[3] : x[1];
  uint32_t a2 = g.c2 ? x[0] : x[2], a3 = g.c2 ? x[1] : x[3];
  uint32_t b0 = g.c1 ? a1 : a0, b1 = g.c1 ? a2 : a1, b2 = g.c1 ? a3 : a2, b3 = g.c1 ? a0 : a3;
  y[0] = __builtin_amdgcn_alignbyte(b1, b0, g.r);
  y[1] = __builtin_amdgcn_alignbyte(b2, b1, g.r);
  y[2] = __builtin_amdgcn_alignbyte(b3, b2, g.r);
  y[3] = __builtin_amdgcn_alignbyte(b0, b3, g.r);
}

// quarter Q (positions of y[Q]) of x * H^64 (mul_k)
template <int Q>
__device__ __forceinline__ void gh_issue(TtTmp& w, const GhLane& g) {
  w.h[0] = lds_u128(KT_OFF + kaddr<0>(w.y[Q], g.cq[Q]));
  w.h[1] = lds_u128(KT_OFF + kaddr<1>(w.y[Q], g.cq[Q]));
  w.h[2] = lds_u128(KT_OFF + kaddr<2>(w.y[Q], g.cq[Q]));
  w.h[3] = lds_u128(KT_OFF + kaddr<3>(w.y[Q], g.cq[Q]));
}
template <bool FIRST>
__device__ __forceinline__ void gh_combine(TtTmp& w) {
  uint32_t a[4];
  a[0] = xor3(w.h[0].x, w.h[1].x, w.h[2].x);
  a[1] = xor3(w.h[0].y, w.h[1].y, w.h[2].y);
  a[2] = xor3(w.h[0].z, w.h[1].z, w.h[2].z);
  a[3] = xor3(w.h[0].w, w.h[1].w, w.h[2].w);
  if (FIRST) {
    w.acc[0] = a[0] ^ w.h[3].x; w.acc[1] = a[1] ^ w.h[3].y;
    w.acc[2] = a[2] ^ w.h[3].z; w.acc[3] = a[3] ^ w.h[3].w;
  } else {
    w.acc[0] = xor3(w.acc[0], a[0], w.h[3].x); w.acc[1] = xor3(w.acc[1], a[1], w.h[3].y);
    w.acc[2] = xor3(w.acc[2], a[2], w.h[3].z); w.acc[3] = xor3(w.acc[3], a[3], w.h[3].w);
  }
}

// T-table round lookups of the lane's block (LAST: final-round pattern)
template <bool LAST>
__device__ __forceinline__ void tt_issue_round(TtTmp& w, uint32_t laneoff) {
#pragma unroll
  for (int c = 0; c < 4; c++) {
    w.t[4 * c + 0] = TE0(w.A[c], 0);
    w.t[4 * c + 1] = LAST ? TE0(w.A[(c + 1) & 3], 1) : TE1(w.A[(c + 1) & 3], 1);
    w.t[4 * c + 2] = TE0(w.A[(c + 2) & 3], 2);
    w.t[4 * c + 3] = TE1(w.A[(c + 3) & 3], 3);
  }
}
__device__ __forceinline__ void tt_combine_round(TtTmp& w, cu32* rkr, int r) {
#pragma unroll
  for (int c = 0; c < 4; c++)
    w.A[c] = xor3(w.t[4 * c], w.t[4 * c + 1],
                  rotl16(xor3(w.t[4 * c + 2], w.t[4 * c + 3], rkr[4 * r + c])));
}

// Phase K of a TT group (see the file comment).  Phases: 0 round-1 lookups
// (+ next group's input loads), 1 round 2, 2 .. ROUNDS-1 rounds 3 .. ROUNDS
// (the last of them issues the final-round lookups), ROUNDS: keystream, output
// store, first GHASH half, then four GHASH half-steps.
template <bool SEAL, int ROUNDS, int K>
__device__ __forceinline__ void tt_phase(TtRec& tt, TtTmp& w, const DevSession* __restrict__ S,
                                         uint32_t lane, uint32_t laneoff, const GhLane& gl) {
  cu32* rk = as_const(S->rk);
  cu32* rkr = as_const(S->rk_rot);
  const uint32_t base = tt.g * 64u;
  if constexpr (K == 0) {
    const uint32_t v = bswap32(tt.ctr0 + base + lane) ^ rk[3];
    w.t[0] = TE1(v, 3);
    w.t[1] = TE0(v, 2);
    if (tt.g + 1 < tt.ng) {
      const uint4 c = *reinterpret_cast<const uint4*>(tt.rc.src + 16u * (base + 64u + lane));
      w.cn[0] = c.x; w.cn[1] = c.y; w.cn[2] = c.z; w.cn[3] = c.w;
    }
  } else if constexpr (K == 1) {
    const uint32_t s0 = tt.rcc.k1a ^ rotl16(w.t[0]), s1 = tt.rcc.k1b ^ rotl16(w.t[1]);
    w.t[0] = TE0(s0, 0); w.t[1] = TE1(s1, 1);
    w.t[2] = TE0(s1, 0); w.t[3] = TE1(s0, 3);
    w.t[4] = TE0(s0, 2); w.t[5] = TE1(s1, 3);
    w.t[6] = TE1(s0, 1); w.t[7] = TE0(s1, 2);
  } else if constexpr (K == 2) {
    w.A[0] = xor3(tt.rcc.k2[0], w.t[0], w.t[1]);
    w.A[1] = xor3(tt.rcc.k2[1], w.t[2], rotl16(w.t[3]));
    w.A[2] = tt.rcc.k2[2] ^ rotl16(w.t[4] ^ w.t[5]);
    w.A[3] = xor3(tt.rcc.k2[3], w.t[6], rotl16(w.t[7]));
    tt_issue_round<ROUNDS == 3>(w, laneoff);
  } else if constexpr (K < ROUNDS) {
    tt_combine_round(w, rkr, K);              // round K (3 .. ROUNDS-1)
    tt_issue_round<K + 1 == ROUNDS>(w, laneoff);
  } else if constexpr (K == ROUNDS) {
    uint32_t o[4];
#pragma unroll
    for (int c = 0; c < 4; c++) {
      const uint32_t lo = __builtin_amdgcn_perm(w.t[4 * c + 1], w.t[4 * c + 0], 0x0C0C0501u);
      const uint32_t hi = __builtin_amdgcn_perm(w.t[4 * c + 3], w.t[4 * c + 2], 0x07020C0Cu);
      o[c] = tt.c[c] ^ xor3(lo, hi, rk[4 * ROUNDS + c]);
      w.gin[c] = SEAL ? o[c] : tt.c[c];
    }
    *reinterpret_cast<uint4*>(tt.rc.dst + 16u * (base + lane)) = make_uint4(o[0], o[1], o[2], o[3]);
    gh_rot(tt.x, w.y, gl);
    gh_issue<0>(w, gl);
  } else if constexpr (K == ROUNDS + 1) {
    gh_combine<true>(w);
    gh_issue<1>(w, gl);
  } else if constexpr (K == ROUNDS + 2) {
    gh_combine<false>(w);
    gh_issue<2>(w, gl);
  } else if constexpr (K == ROUNDS + 3) {
    gh_combine<false>(w);
    gh_issue<3>(w, gl);
  } else if constexpr (K == ROUNDS + 4) {
    gh_combine<false>(w);
#pragma unroll
    for (int c = 0; c < 4; c++) {
      tt.x[c] = w.acc[c] ^ w.gin[c];
      tt.c[c] = w.cn[c];
    }
    tt.g++;
  }
}
constexpr int tt_phases(int rounds) { return rounds + 5; }

// One S-box of a bitsliced round (bs_subbytes, one byte)
template <int B>
__device__ __forceinline__ void bs_sbox_one(uint32_t (&st)[128]) {
  uint32_t* p = st + 8 * B;
  uint32_t o7, o6, o5, o4, o3, o2, o1, o0;
  TG_BS_SBOX(p[7], p[6], p[5], p[4], p[3], p[2], p[1], p[0], o7, o6, o5, o4, o3, o2, o1, o0);
  p[7] = o7; p[6] = o6; p[5] = o5; p[4] = o4; p[3] = o3; p[2] = o2; p[1] = o1; p[0] = o0;
  __builtin_amdgcn_sched_barrier(0);  // one S-box at a time (register pressure)
}

template <bool SEAL, int ROUNDS, int K>
__device__ __forceinline__ void tt_slot(bool run, TtRec& tt, TtTmp& w, const DevSession* __restrict__ S,
                                        uint32_t lane, uint32_t laneoff, const GhLane& gl) {
  if constexpr (K < tt_phases(ROUNDS)) {
    if (run) tt_phase<SEAL, ROUNDS, K>(tt, w, S, lane, laneoff, gl);
    __builtin_amdgcn_sched_barrier(0);  // the phase stays between its two S-boxes
  }
}

// A bitsliced round (MC: with MixColumns + AddRoundKey r; else the final
// round's SubBytes + ShiftRows) carrying one TT group when `run`.
template <bool SEAL, int ROUNDS, bool MC, int... B>
__device__ __forceinline__ void fused_round(uint32_t (&st)[128], const SgprMasks& km, int r, bool run,
                                            TtRec& tt, const DevSession* __restrict__ S, uint32_t lane,
                                            uint32_t laneoff, const GhLane& gl,
                                            std::integer_sequence<int, B...>) {
  TtTmp w;
  ((bs_sbox_one<B>(st), tt_slot<SEAL, ROUNDS, B>(run, tt, w, S, lane, laneoff, gl)), ...);
  bs_shiftrows(st);
  if (MC) bs_mixcolumn<0>(st, km, r);
  tt_slot<SEAL, ROUNDS, 16>(run, tt, w, S, lane, laneoff, gl);
  if (MC) bs_mixcolumn<1>(st, km, r);
  tt_slot<SEAL, ROUNDS, 17>(run, tt, w, S, lane, laneoff, gl);
  if (MC) bs_mixcolumn<2>(st, km, r);
  tt_slot<SEAL, ROUNDS, 18>(run, tt, w, S, lane, laneoff, gl);
  if (MC) bs_mixcolumn<3>(st, km, r);
}

// Start the next TT record of the run (claimed from the queue), or none.
template <bool SEAL, int ROUNDS>
__device__ __forceinline__ void tt_begin(TtRec& tt, const BatchArgs& a, const RecPre* __restrict__ pre,
                                         uint32_t* q, uint32_t run_end, const DevSession* __restrict__ S,
                                         uint32_t lane) {
  const tlsgpu_record* D = reinterpret_cast<const tlsgpu_record*>(a.descs);
  tt.on = false;
  for (;;) {
    const uint32_t r = queue_take(q, 1, lane);
    if (r >= run_end) return;
    if (!parse_tls<SEAL>(load_desc(D + r), S, a.in, a.out, a.status + r, lane, tt.rc)) continue;
    tt.rcc = rec_consts_of(pre + r);
    tt.slot = a.status + r;
    tt.ctr0 = bswap32(tt.rc.j0[3]) + 1u;
    const bool aligned = ((((uintptr_t)tt.rc.src) | ((uintptr_t)tt.rc.dst)) & 15) == 0;
    tt.ng = aligned ? (tt.rc.n >> 4) / 64u : 0u;
    tt.g = 0;
#pragma unroll
    for (int c = 0; c < 4; c++) tt.x[c] = (lane == 63) ? bswap32(tt.rc.aad_be[c]) : 0u;
    if (tt.ng) {
      const uint4 v = *reinterpret_cast<const uint4*>(tt.rc.src + 16u * lane);
      tt.c[0] = v.x; tt.c[1] = v.y; tt.c[2] = v.z; tt.c[3] = v.w;
    }
    tt.on = true;
    return;
  }
}

// Finish the TT record if its full groups are done (remainder on the plain
// T-table path, then the tag).
template <bool SEAL, int ROUNDS>
__device__ __forceinline__ bool tt_end_if_done(TtRec& tt, const DevSession* __restrict__ S, uint32_t lane,
                                               uint32_t laneoff, const GhLane& gl, bool force) {
  if (!tt.on || (!force && tt.g < tt.ng)) return false;
  const CtrConst none = {};
  gcm_blocks<SEAL, ROUNDS, true>(tt.rc, S, tt.rcc, none, tt.x, tt.g * 64u, lane, laneoff, gl);
  gcm_finish<SEAL>(tt.rc, tt.x, tt.rcc.ek0, S, tt.slot, lane, gl);
  tt.on = false;
  return true;
}

// Bitsliced pair (gcm_pair_hy) with the TT record riding in its rounds.
template <bool SEAL, int ROUNDS>
__device__ __forceinline__ void gcm_pair_fused(const RecCtx (&rc)[2], const RecPre* pa, const RecPre* pb,
                               int32_t* slot_a, int32_t* slot_b, const DevSession* __restrict__ S,
                               TtRec& tt, const BatchArgs& a, const RecPre* __restrict__ pre,
                               uint32_t* q, uint32_t run_end, uint32_t lane, uint32_t laneoff,
                               const GhLane& gl) {
  PhaseClock pc(a.dbg);
  cu32* rk = as_const(S->rk);
  const SgprMasks km{rk};
  const uint32_t rkl[4] = {rk[4 * ROUNDS], rk[4 * ROUNDS + 1], rk[4 * ROUNDS + 2],
                           rk[4 * ROUNDS + 3]};
  uint32_t x[2][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
  if (lane == 63) {
#pragma unroll
    for (int qq = 0; qq < 2; qq++)
#pragma unroll
      for (int w = 0; w < 4; w++) x[qq][w] = bswap32(rc[qq].aad_be[w]);
  }
  const uint32_t passes = min(rc[0].n, rc[1].n) >> 14;
  for (uint32_t p = 0; p < passes; p++) {
    const uint32_t pb0 = p << 10;
    uint32_t st[128];
    bs_encrypt_r2<ROUNDS>(st, pa, pb, 2u + lane + pb0, rk);  // rounds 1, 2
#pragma unroll 1
    for (int r = 3; r < ROUNDS; r++) {
      const bool run = tt.on && tt.g < tt.ng;
      fused_round<SEAL, ROUNDS, true>(st, km, r, run, tt, S, lane, laneoff, gl,
                                      std::make_integer_sequence<int, 16>{});
    }
    {
      const bool run = tt.on && tt.g < tt.ng;
      fused_round<SEAL, ROUNDS, false>(st, km, ROUNDS, run, tt, S, lane, laneoff, gl,
                                       std::make_integer_sequence<int, 16>{});
    }
    pc.lap(1, lane);
    uint32_t ring[4][2][4];
#pragma unroll
    for (int t = 0; t < 4; t++)
#pragma unroll
      for (int qq = 0; qq < 2; qq++) {
        const uint4 v = *reinterpret_cast<const uint4*>(rc[qq].src + 16u * (pb0 + 64u * t + lane));
        ring[t][qq][0] = v.x; ring[t][qq][1] = v.y; ring[t][qq][2] = v.z; ring[t][qq][3] = v.w;
      }
    transpose_all(st);
    bs_consume_all<SEAL>(st, ring, x, rc, rkl, pb0, lane, gl,
                         std::make_integer_sequence<int, 16>{});
    pc.lap(2, lane);
    if (tt_end_if_done<SEAL, ROUNDS>(tt, S, lane, laneoff, gl, false))
      tt_begin<SEAL, ROUNDS>(tt, a, pre, q, run_end, S, lane);
    pc.lap(6, lane);
  }
#pragma unroll
  for (int qq = 0; qq < 2; qq++) {
    if (((rc[qq].n + 15) >> 4) > (passes << 10)) {
      const RecConsts rcc = rec_consts_of(qq ? pb : pa);
      const CtrConst none = {};
      gcm_blocks<SEAL, ROUNDS, true>(rc[qq], S, rcc, none, x[qq], passes << 10, lane, laneoff, gl);
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

// 8 fused waves per CU (two per SIMD, 256 VGPRs each).
constexpr int kFuThreads = 512;

template <bool SEAL, int ROUNDS>
__global__ __launch_bounds__(kFuThreads, 1) void gcm_fused_kernel(BatchArgs a,
                                                                 const RecPre* __restrict__ pre) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t laneoff = aes_laneoff(lane);
  const GhLane gl = gh_lane(lane);
  const tlsgpu_record* D = reinterpret_cast<const tlsgpu_record*>(a.descs);
  uint32_t* q = reinterpret_cast<uint32_t*>(s_lds + Q_OFF);

  fill_aes_lds<kFuThreads>();
  if (a.dbg && threadIdx.x < 32) reinterpret_cast<unsigned long long*>(s_lds + DBG_OFF)[threadIdx.x] = 0;

  const uint32_t rlo = blockIdx.x * a.records_per_group;
  const uint32_t rhi = min(a.n, rlo + a.records_per_group);
  uint32_t cur = 0xFFFFFFFFu;
  uint32_t pos = rlo;
  while (pos < rhi) {
    const uint32_t sid = __builtin_amdgcn_readfirstlane(D[pos].session);
    uint32_t run_end = pos + 1;
    while (run_end < rhi) {
      uint32_t p = run_end + lane;
      uint32_t s = p < rhi ? D[p].session : sid;
      uint64_t diff = __ballot(p < rhi && s != sid);
      if (diff) { run_end += __builtin_amdgcn_readfirstlane((uint32_t)__builtin_ctzll(diff)); break; }
      run_end = min(rhi, run_end + 64);
    }
    const bool in_range = sid < a.n_sessions;
    const DevSession* __restrict__ S = a.sessions + (in_range ? sid : 0);
    const uint32_t kind = as_const(&S->kind)[0];
    const bool usable = in_range && is_gcm(kind) && (int)as_const(&S->rounds)[0] == ROUNDS;
    if (usable) {
      PhaseClock pc(a.dbg);
      __syncthreads();
      pc.lap(4, lane);
      if (threadIdx.x == 0) *q = pos;
      if (sid != cur) load_session_tables<kFuThreads>(a.gcm_tables + sid);
      cur = sid;
      __syncthreads();
      pc.lap(5, lane);
      TtRec tt;
      tt.on = false;
      for (;;) {
        const uint32_t r = queue_take(q, 2, lane);
        if (r >= run_end) break;
        const uint32_t rb = r + 1;
        bool paired = false;
        if (rb < run_end && run_end - r >= a.bs_reserve) {
          RecCtx rc[2];
          const bool oka = parse_tls<SEAL>(load_desc(D + r), S, a.in, a.out, a.status + r, lane, rc[0]);
          const bool okb = parse_tls<SEAL>(load_desc(D + rb), S, a.in, a.out, a.status + rb, lane, rc[1]);
          if (oka && okb && rc[0].n >= 16384 && rc[1].n >= 16384 &&
              (((uintptr_t)rc[0].src | (uintptr_t)rc[0].dst | (uintptr_t)rc[1].src |
                (uintptr_t)rc[1].dst) & 15) == 0) {
            if (!tt.on) tt_begin<SEAL, ROUNDS>(tt, a, pre, q, run_end, S, lane);
            gcm_pair_fused<SEAL, ROUNDS>(rc, pre + r, pre + rb, a.status + r, a.status + rb, S, tt,
                                         a, pre, q, run_end, lane, laneoff, gl);
            paired = true;
          } else {
            for (uint32_t m = 0; m < 2; m++) {
              if (!(m ? okb : oka)) continue;
              gcm_record_x4<SEAL, ROUNDS, 2>(m ? rc[1] : rc[0], S, rec_consts_of(pre + r + m),
                                             a.status + r + m, lane, laneoff, gl);
            }
            paired = true;
          }
        }
        if (!paired) {
          hy_tt_record<SEAL, ROUNDS, 2>(a, pre, r, S, lane, laneoff, gl);
          if (rb < run_end) hy_tt_record<SEAL, ROUNDS, 2>(a, pre, rb, S, lane, laneoff, gl);
        }
      }
      tt_end_if_done<SEAL, ROUNDS>(tt, S, lane, laneoff, gl, true);
    }
    pos = run_end;
  }
  if (a.dbg) {
    __syncthreads();
    if (threadIdx.x < 32)
      atomicAdd(a.dbg + threadIdx.x, reinterpret_cast<unsigned long long*>(s_lds + DBG_OFF)[threadIdx.x]);
  }
}

}  // namespace tg
