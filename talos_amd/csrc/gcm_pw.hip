// gcm_pw.hip — the per-wave-session AES-GCM TLS kernel.
//
// The queue kernel (gcm_hybrid.h) shares one session's 64 KiB GHASH byte table
// and 16.6 KiB of Shoup tables in LDS across its 16 waves, so it works through
// a batch one session run at a time with a workgroup barrier between runs.
// When runs are short — many connections with a few records each, or records
// of different connections interleaved, as a server's batch arrives — most of
// the 16 waves idle at every run boundary (1 record per session: 1 busy wave of
// 16, measured 9x slower).  Here every wave is independent:
//   * the AES T-tables (64 KiB, session independent) stay shared;
//   * each of the 12 waves owns an 8 KiB nibble-position table of its current
//     session's H^64 (T[h][v][p] = nibble v at nibble p of half h, times H^64),
//     rebuilt from the session's 2 KiB basis (DevGcmTables::basis, L2) when the
//     wave's next record belongs to another session: 32 conflict-free
//     ds_read_b128 per Horner step instead of the byte table's 16;
//   * the chain weights H^1..H^65 come from the session's Shoup tables in HBM
//     (one 256-B table per lane, L2-resident), the rem_4bit reduction is done
//     on the VALU (rem * 0xE1 carry-less, gcm128.c:327-331);
//   * waves pull single records from a per-workgroup counter in global memory.
// LDS: 64 KiB AES + 16 x 4 KiB (TG_PW_HALF) or 12 x 8 KiB, one workgroup per CU.
//
// TG_PW_HALF (default): the table covers one 64-bit half only (4 KiB: the high
// half's nibble p is the low half's nibble p times x^64, so its sum is
// multiplied by x^64 on the VALU, mulx64), which fits 16 waves x 4 KiB + the
// AES tables in LDS: a 1024-thread workgroup at <= 128 VGPRs, as the queue
// kernel.  TG_PW_HALF=0: the round-2 form, 12 waves x 8 KiB.
#ifndef TG_PW_HALF
#define TG_PW_HALF 1
#endif
#if TG_PW_HALF
#define TG_LDS_BYTES 131072
#else
// 12 x 8 KiB tables + the T-tables at 64 KiB (gcm_device.h AES_OFF) exceed the LDS
#error "TG_PW_HALF=0 (12 waves x 8 KiB tables) no longer fits the LDS plan"
#endif
#define TG_XOR3_ASM  // xor3 as inline asm here: the builtin's freer schedule spills this kernel
#include "gcm_hybrid.h"

namespace tg {

#if TG_PW_HALF
constexpr int kPwThreads = 1024;
constexpr uint32_t PW_TAB_BYTES = 4096;  // 16 values x 16 positions x 16 B
#else
constexpr int kPwThreads = 768;
constexpr uint32_t PW_TAB_BYTES = 8192;  // 2 halves x 16 values x 16 positions x 16 B
#endif
constexpr int kPwWaves = kPwThreads / kWave;
// per-wave tables at 0 .. 64 KiB, below the T-tables (AES_OFF): a lookup address
// is the table's [0, 0, wave * 16 + nibble, position * 16], one v_perm
constexpr uint32_t PW_TAB_OFF = 0;
static_assert(PW_TAB_OFF + kPwWaves * PW_TAB_BYTES <= AES_OFF, "per-wave tables overlap the T-tables");
static_assert(PW_TAB_OFF + kPwWaves * PW_TAB_BYTES <= LDS_BYTES, "per-wave tables exceed LDS");

#ifndef TG_PW_NB
#define TG_PW_NB 2
#endif
#ifndef TG_PW_QGROUP  // nibble-plane groups of 4 lookups per batch (1, 2 or 4)
#define TG_PW_QGROUP (TG_PW_HALF ? 2 : 4)
#endif
#ifndef TG_PW_SHOUP_BATCH
#define TG_PW_SHOUP_BATCH 16
#endif

// Reverse the bits of every byte of w (GCM's bit order <-> integer bit order).
__device__ __forceinline__ uint32_t rbyte(uint32_t w) {
  return __builtin_bitreverse32(__builtin_amdgcn_perm(w, w, 0x00010203u));
}

// b * x^64 in GF(2^128) (LE words: bytes 8..15 of the result are bytes 0..7
// of b; bytes 8..15 of b, times x^128 = x^7 + x^2 + x + 1, fold into bytes
// 0..8: gcm128.c's reduction, 64 bits at once).
__device__ __forceinline__ void mulx64(const uint32_t b[4], uint32_t r[4]) {
  const uint32_t s0 = rbyte(b[2]), s1 = rbyte(b[3]);  // x^0..x^63 of the overflow, integer order
  const uint32_t q0 = xor3(s0, s0 << 1, s0 << 2) ^ (s0 << 7);
  const uint32_t q1 = xor3(s1, __builtin_amdgcn_alignbit(s1, s0, 31),
                           __builtin_amdgcn_alignbit(s1, s0, 30)) ^
                      __builtin_amdgcn_alignbit(s1, s0, 25);
  const uint32_t q2 = xor3(s1 >> 31, s1 >> 30, s1 >> 25);  // x^64..x^70
  r[0] = rbyte(q0);
  r[1] = rbyte(q1);
  r[2] = b[0] ^ rbyte(q2);
  r[3] = b[1];
}

struct GhNib {
  uint32_t base;     // LDS byte offset of this wave's table
  uint32_t wb;       // (base >> 8) in every byte: the table's 256-B row index, ORed
                     // into the nibble planes so the address needs no base add
  uint32_t sw;       // m >= 8 (m = lane % 16): swap the words of each 64-bit half
  uint32_t s;        // then rotate each half right by 4 * (m & 7) bits
  uint32_t cq[4];    // cq[pl].byte[b] = ((k + m) & 15) * 16, k = 8(pl>>1) + 2b + (pl&1)
  const DevGcmTables* tab;  // the session's tables in HBM

  // o = x * H^64 (LE words).  Half h of x rotated right by m nibbles puts
  // nibble (k + m) % 16 at nibble k; the nibbles are split into byte planes so
  // one v_perm forms [0, 0, nibble, position * 16] = the entry's address.
  // Lanes of a ds_read_b128 lane group have distinct m, so distinct positions,
  // so distinct quad-banks: conflict-free.
  __device__ __forceinline__ void mul64(const uint32_t x[4], uint32_t o[4]) const {
    uint32_t acc[2][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}};
#pragma unroll
    for (int h = 0; h < 2; h++) {  // 16 lookups in flight per half
      const uint32_t lo = x[2 * h], hi = x[2 * h + 1];
      const uint32_t a = sw ? hi : lo, b = sw ? lo : hi;
      const uint32_t ylo = __builtin_amdgcn_alignbit(b, a, s);
      const uint32_t yhi = __builtin_amdgcn_alignbit(a, b, s);
      const uint32_t pl[4] = {(ylo & 0x0F0F0F0Fu) | wb, ((ylo >> 4) & 0x0F0F0F0Fu) | wb,
                              (yhi & 0x0F0F0F0Fu) | wb, ((yhi >> 4) & 0x0F0F0F0Fu) | wb};
      const uint32_t hb = 0;
      const int d = TG_PW_HALF ? h : 0;
#pragma unroll
      for (int q0 = 0; q0 < 4; q0 += TG_PW_QGROUP) {  // 4 * TG_PW_QGROUP lookups in flight
        uint4 v[4 * TG_PW_QGROUP];
#pragma unroll
        for (int q = 0; q < TG_PW_QGROUP; q++)
#pragma unroll
          for (int bb = 0; bb < 4; bb++)
            v[4 * q + bb] = lds_u128(hb + __builtin_amdgcn_perm(pl[q0 + q], cq[q0 + q],
                                                                0x0C0C0000u | ((4u + bb) << 8) | bb));
#pragma unroll
        for (int k = 0; k < 4 * TG_PW_QGROUP; k += 2) {
          acc[d][0] = xor3(acc[d][0], v[k].x, v[k + 1].x);
          acc[d][1] = xor3(acc[d][1], v[k].y, v[k + 1].y);
          acc[d][2] = xor3(acc[d][2], v[k].z, v[k + 1].z);
          acc[d][3] = xor3(acc[d][3], v[k].w, v[k + 1].w);
        }
      }
    }
    if (TG_PW_HALF) {
      uint32_t t[4];
      mulx64(acc[1], t);
      o[0] = acc[0][0] ^ t[0]; o[1] = acc[0][1] ^ t[1]; o[2] = acc[0][2] ^ t[2]; o[3] = acc[0][3] ^ t[3];
    } else {
      o[0] = acc[0][0]; o[1] = acc[0][1]; o[2] = acc[0][2]; o[3] = acc[0][3];
    }
  }

  // Z = X * H^e (Shoup 4-bit, gcm128.c:333-393), BE words, table from HBM
  // (L2 after the kernel's prefetch at record start).  The 32 table entries
  // depend only on X's nibbles: loaded PWS_SHOUP_BATCH at a time ahead of the
  // serial shift/reduce chain.
  __device__ __forceinline__ void shoup(const uint32_t X[4], uint32_t e, uint32_t Z[4]) const {
    constexpr int kB = TG_PW_SHOUP_BATCH;
    const uint8_t* T = reinterpret_cast<const uint8_t*>(&tab->shoup[e - 1][0][0]);
    uint32_t z0 = 0, z1 = 0, z2 = 0, z3 = 0;
#pragma unroll
    for (int g = 0; g < 32 / kB; g++) {
      uint4 m[kB];
#pragma unroll
      for (int i = 0; i < kB; i++) {
        const int k = kB * g + i;
        const uint32_t nib = (X[3 - k / 8] >> (4 * (k % 8))) & 0xF;
        m[i] = gload16(T + nib * 16);
      }
#pragma unroll
      for (int i = 0; i < kB; i++) {
        if (g != 0 || i != 0) {
          const uint32_t rem = z3 & 0xF;
          z3 = __builtin_amdgcn_alignbit(z2, z3, 4);
          z2 = __builtin_amdgcn_alignbit(z1, z2, 4);
          z1 = __builtin_amdgcn_alignbit(z0, z1, 4);
          z0 = (z0 >> 4) ^ rem4(rem);
        }
        z0 ^= m[i].x; z1 ^= m[i].y; z2 ^= m[i].z; z3 ^= m[i].w;
      }
    }
    Z[0] = z0; Z[1] = z1; Z[2] = z2; Z[3] = z3;
  }

  // This wave's table for session tables `t` (from basis[q] = H^64 * x^q, LE
  // words; bit t of the byte at position j is x^(8j + 7 - t), load_session_tables).
  // Half form: lane l builds position p = l % 16, values 4g .. 4g + 3 with
  // g = l / 16.  Full form: position p = l % 16 of half h = (l / 16) % 2,
  // values 8g .. 8g + 7 with g = l / 32.
  __device__ __forceinline__ void build(uint32_t lane) const {
#if TG_PW_HALF
    const uint32_t p = lane & 15, h = 0, g = lane >> 4;
    constexpr int kVals = 4;
#else
    const uint32_t p = lane & 15, h = (lane >> 4) & 1, g = lane >> 5;
    constexpr int kVals = 8;
#endif
    const uint32_t i = 16 * h + p, j = i >> 1, sh = 4 * (i & 1);
    uint4 B[4];
#pragma unroll
    for (int t = 0; t < 4; t++) B[t] = gload16(&tab->basis[8 * j + 7 - sh - t][0]);
#pragma unroll
    for (int u = 0; u < kVals; u++) {
      const uint32_t v = kVals * g + u;
      const uint32_t m0 = (v & 1) ? 0xFFFFFFFFu : 0u, m1 = (v & 2) ? 0xFFFFFFFFu : 0u;
      const uint32_t m2 = (v & 4) ? 0xFFFFFFFFu : 0u, m3 = (v & 8) ? 0xFFFFFFFFu : 0u;
      const uint4 e = make_uint4((B[0].x & m0) ^ (B[1].x & m1) ^ (B[2].x & m2) ^ (B[3].x & m3),
                                 (B[0].y & m0) ^ (B[1].y & m1) ^ (B[2].y & m2) ^ (B[3].y & m3),
                                 (B[0].z & m0) ^ (B[1].z & m1) ^ (B[2].z & m2) ^ (B[3].z & m3),
                                 (B[0].w & m0) ^ (B[1].w & m1) ^ (B[2].w & m2) ^ (B[3].w & m3));
      *reinterpret_cast<uint4*>(s_lds + base + 4096u * h + v * 256u + p * 16u) = e;
    }
    // the wave's own later lookups read what its lanes just wrote
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
};

__device__ __forceinline__ GhNib gh_nib(uint32_t lane, uint32_t base) {
  GhNib g;
  const uint32_t m = lane & 15;
  g.base = base;
  g.wb = (base >> 8) * 0x01010101u;
  g.sw = m >> 3;
  g.s = 4 * (m & 7);
#pragma unroll
  for (int q = 0; q < 4; q++) {
    uint32_t v = 0;
#pragma unroll
    for (int b = 0; b < 4; b++) {
      const uint32_t k = 8 * (q >> 1) + 2 * b + (q & 1);
      v |= (((k + m) & 15u) << 4) << (8 * b);
    }
    g.cq[q] = v;
  }
  g.tab = nullptr;
  return g;
}

template <bool SEAL, int ROUNDS>
__global__ __launch_bounds__(kPwThreads, 1) void gcm_pw_kernel(BatchArgs a,
                                                               const RecPre* __restrict__ pre) {
  const SelSums f = sel_sums(a.sel);
  if (!pws_selected(a.pws, f.runs, f.recs)) return;  // the queue kernel runs this batch
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t laneoff = aes_laneoff(lane);
  const tlsgpu_record* D = reinterpret_cast<const tlsgpu_record*>(a.descs);
  fill_aes_lds<kPwThreads, false>();
  __syncthreads();
  GhNib g = gh_nib(lane, PW_TAB_OFF + wave * PW_TAB_BYTES);
  const uint32_t rlo = blockIdx.x * a.records_per_group;
  const uint32_t rhi = min(a.n, rlo + a.records_per_group);
  uint32_t* next = a.wg_next + blockIdx.x;
  uint32_t cur = 0xFFFFFFFFu;
  for (;;) {
    const uint32_t r = rlo + queue_take(next, 1, lane);
    if (r >= rhi) break;
    const tlsgpu_record d = load_desc(D + r);
    if (d.session >= a.n_sessions) continue;
    const DevSession* __restrict__ S = a.sessions + d.session;
    if (!is_gcm(as_const(&S->kind)[0]) || (int)as_const(&S->rounds)[0] != ROUNDS) continue;
    if (d.session != cur) {
      g.tab = a.gcm_tables + d.session;
      g.build(lane);
      cur = d.session;
    }
    RecCtx rc;
    if (!parse_tls<SEAL>(d, S, a.in, a.out, a.status + r, lane, rc)) continue;
    // this lane's chain weight H^e, e = 1 + ((nb - lane) mod 64) (gcm_close_chain):
    // its 256-B Shoup table towards L2 now, read at the record's finish
    const uint32_t e = 1u + ((((rc.n + 15) >> 4) - lane) & 63u);
    Prefetch<2> pf;
    pf.v[0] = *gld<uint32_t>(&g.tab->shoup[e - 1][0][0]);
    pf.v[1] = *gld<uint32_t>(&g.tab->shoup[e - 1][8][0]);
    const RecConsts rcc = rec_consts_of(pre + r);
    gcm_record_x4<SEAL, ROUNDS, TG_PW_NB>(rc, S, rcc, a.status + r, lane, laneoff, g);
    prefetch_done(pf);
  }
}

int launch_gcm_pw(const BatchArgs& a, const RecPre* pre, bool seal, int rounds, int groups,
                  hipStream_t s) {
  if (a.n == 0 || !a.sel || !a.wg_next) return 0;
  const dim3 g(groups), b(kPwThreads);
  if (rounds == 10) {
    if (seal) hipLaunchKernelGGL((gcm_pw_kernel<true, 10>), g, b, 0, s, a, pre);
    else hipLaunchKernelGGL((gcm_pw_kernel<false, 10>), g, b, 0, s, a, pre);
  } else {
    if (seal) hipLaunchKernelGGL((gcm_pw_kernel<true, 14>), g, b, 0, s, a, pre);
    else hipLaunchKernelGGL((gcm_pw_kernel<false, 14>), g, b, 0, s, a, pre);
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace tg
