// gcm_device.h — device-side building blocks shared by the AES-GCM kernels
// (gcm_kernels.hip: T-table batch kernel; gcm_bs_kernels.hip: bitsliced and
// hybrid kernels).  Layout and mapping notes: gcm_kernels.hip header and
// DESIGN.md §4.  Each translation unit gets its own copy of the LDS array.
#pragma once
#include <utility>

#include "aes_common.h"
#include "bs_aes.h"
#include "tlsgpu_internal.h"

namespace tg {

static __device__ const WordTable g_te0 = kTe0;

constexpr int kThreads = 1024;
constexpr int kWaves = kThreads / kWave;
// The GHASH byte-position table sits at LDS offset 0 and the AES T-tables at
// 64 KiB: a table address is then a single v_perm with no base add — the
// KT lookups' base is 0, and the T-table base 0x10000 rides in byte 2 of the
// lane's `laneoff` operand, which taddr's selector copies (aes_laneoff).
constexpr uint32_t KT_OFF = 0;
constexpr uint32_t AES_OFF = 0x10000;
static_assert(AES_OFF == 0x10000, "taddr takes the T-table base from byte 2 of laneoff");
constexpr uint32_t SH_OFF = 131072;
// Shoup tables: entry (e, v) of H^e (e = 1..65, nibble v) at
// SH_OFF + ((e-1)/16) * 4 KiB + v * 256 + ((e-1) % 16) * 16 (sh_base), i.e. the
// power picks the 16-B column: the lanes of a ds_read_b128 group (distinct lane
// % 16) need powers with distinct (e-1) % 16 in the per-lane chain weights, so
// their lookups are conflict-free whatever the nibbles.
constexpr uint32_t SH_BYTES = ((kPowMax + 15) / 16) * 4096;
constexpr uint32_t R4_OFF = SH_OFF + SH_BYTES;
constexpr uint32_t Q_OFF = R4_OFF + 64;      // hybrid kernel: per-run record queue
constexpr uint32_t DBG_OFF = Q_OFF + 16;     // hybrid kernel: phase counters (diagnostic)
constexpr uint32_t PLAN_OFF = DBG_OFF + 32 * 8;  // queue kernel: per-run pack plan
constexpr uint32_t kPlanCap = 2048;                // records planned per run (runs split)
#ifdef TG_LDS_BYTES  // a translation unit with its own LDS plan (gcm_pw.hip)
constexpr uint32_t LDS_BYTES = TG_LDS_BYTES;
#else
constexpr uint32_t LDS_BYTES = PLAN_OFF + 4 * kPlanCap;
#endif

__shared__ __attribute__((aligned(16))) uint8_t s_lds[LDS_BYTES];

// Wave-uniform data (session header, round keys, descriptors) is read through
// the constant address space so it lands in SGPRs via s_load.  A persistent
// kernel (evp_server.hip: TG_VECTOR_SESSION_LOADS) reads the same data as
// plain global loads instead: a kernel launch invalidates the scalar cache, a
// long-running kernel never gets that, and session slots are re-keyed while it
// runs; its per-job acquire fence invalidates only the vector caches.
#ifdef TG_VECTOR_SESSION_LOADS
// a uniform word read by a vector load and moved to an SGPR (readfirstlane)
struct cu32_word {
  uint32_t raw;
  __device__ __forceinline__ operator uint32_t() const {
    return __builtin_amdgcn_readfirstlane(raw);
  }
};
typedef const cu32_word cu32;
#else
typedef __attribute__((address_space(4))) const uint32_t cu32;
#endif
template <typename T>
__device__ __forceinline__ cu32* as_const(const T* p) { return (cu32*)(p); }

// ---------------------------------------------------------------------------
// LDS access helpers
__device__ __forceinline__ uint32_t lds_u32(uint32_t off) {
  return *reinterpret_cast<const uint32_t*>(s_lds + off);
}
__device__ __forceinline__ uint4 lds_u128(uint32_t off) {
  return *reinterpret_cast<const uint4*>(s_lds + off);
}

// The lane's T-table operand: its bank offset (lane % 32) * 4 in byte 0 and
// the table base AES_OFF >> 16 in byte 2.
__device__ __forceinline__ uint32_t aes_laneoff(uint32_t lane) { return ((lane & 31) * 4) | AES_OFF; }
// address of Te0[byte r of w] for this lane: [0, AES_OFF >> 16, byte, lane bank].
// Byte 1 already sits where the address wants it: (w & 0xFF00) | laneoff in one
// full-rate v_bitop3_b32 (truth table 0xEA = (a & b) | c) instead of a
// v_perm_b32, which measured 3.4 cycles per wave64 instruction at 4 waves/SIMD
// against 2.1 (tools/ubench.hip); VALU issue adds to the T-table waves' LDS
// lookup time nearly 1:1 (profiles/r03b_ubench_set2.jsonl).
template <int R>
__device__ __forceinline__ uint32_t taddr(uint32_t w, uint32_t laneoff) {
  if constexpr (R == 1) return __builtin_amdgcn_bitop3_b32(w, 0xFF00u, laneoff, 0xEA);
  return __builtin_amdgcn_perm(w, laneoff, 0x0C020000u | ((4u + R) << 8));
}
__device__ __forceinline__ uint32_t rotl16(uint32_t x) { return __builtin_amdgcn_alignbit(x, x, 16); }
// three-input XOR in one VALU op: v_bitop3_b32 with truth table 0x96 (gfx950
// has no v_xor3_b32; hipcc does not form bitop3 from these ^ chains).  The
// builtin, not inline asm: a wave-uniform operand (round-key word) stays in
// its SGPR instead of being copied to a VGPR first, and the scheduler sees it.
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
#ifdef TG_XOR3_ASM  // opaque to the scheduler: gcm_pw.hip (the builtin's schedule spills there)
  uint32_t d;
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(d) : "v"(a), "v"(b), "v"(c));
  return d;
#else
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
#endif
}

#define TE0(w, r) lds_u32(taddr<r>((w), laneoff))
#define TE1(w, r) lds_u32(128 + taddr<r>((w), laneoff))

// One full AES round on little-endian columns (ShiftRows: row r of output
// column c comes from input column c+r).  kr_c = rotr16(k_c) is folded into the
// rotated half so a column costs xor3 + alignbit + xor3:
//   t = Te0[a] ^ Te1[b] ^ rotl16(Te0[c] ^ Te1[d] ^ rotr16(k))
__device__ __forceinline__ void aes_round(uint32_t& s0, uint32_t& s1, uint32_t& s2, uint32_t& s3,
                                          uint32_t k0, uint32_t k1, uint32_t k2, uint32_t k3,
                                          uint32_t laneoff) {
  uint32_t t0 = xor3(TE0(s0, 0), TE1(s1, 1), rotl16(xor3(TE0(s2, 2), TE1(s3, 3), k0)));
  uint32_t t1 = xor3(TE0(s1, 0), TE1(s2, 1), rotl16(xor3(TE0(s3, 2), TE1(s0, 3), k1)));
  uint32_t t2 = xor3(TE0(s2, 0), TE1(s3, 1), rotl16(xor3(TE0(s0, 2), TE1(s1, 3), k2)));
  uint32_t t3 = xor3(TE0(s3, 0), TE1(s0, 1), rotl16(xor3(TE0(s1, 2), TE1(s2, 3), k3)));
  s0 = t0; s1 = t1; s2 = t2; s3 = t3;
}

// Two independent blocks per call, written so the 32 lookups of a round are
// issued together and the scheduler is told to keep them together: 32 address
// perms, 32 DS reads, then the 24 combining ops (T19 sched_group_barrier).
__device__ __forceinline__ void aes_round2(uint32_t (&a)[4], uint32_t (&b)[4], uint32_t k0,
                                           uint32_t k1, uint32_t k2, uint32_t k3,
                                           uint32_t laneoff) {
  uint32_t ta[16], tb[16];
#pragma unroll
  for (int c = 0; c < 4; c++) {
    ta[4 * c + 0] = TE0(a[c], 0);
    ta[4 * c + 1] = TE1(a[(c + 1) & 3], 1);
    ta[4 * c + 2] = TE0(a[(c + 2) & 3], 2);
    ta[4 * c + 3] = TE1(a[(c + 3) & 3], 3);
  }
#pragma unroll
  for (int c = 0; c < 4; c++) {
    tb[4 * c + 0] = TE0(b[c], 0);
    tb[4 * c + 1] = TE1(b[(c + 1) & 3], 1);
    tb[4 * c + 2] = TE0(b[(c + 2) & 3], 2);
    tb[4 * c + 3] = TE1(b[(c + 3) & 3], 3);
  }
  const uint32_t k[4] = {k0, k1, k2, k3};
#pragma unroll
  for (int c = 0; c < 4; c++)
    a[c] = xor3(ta[4 * c], ta[4 * c + 1], rotl16(xor3(ta[4 * c + 2], ta[4 * c + 3], k[c])));
#pragma unroll
  for (int c = 0; c < 4; c++)
    b[c] = xor3(tb[4 * c], tb[4 * c + 1], rotl16(xor3(tb[4 * c + 2], tb[4 * c + 3], k[c])));
  __builtin_amdgcn_sched_group_barrier(0x002, 16, 0);  // A addresses
  __builtin_amdgcn_sched_group_barrier(0x100, 16, 0);  // A lookups
  __builtin_amdgcn_sched_group_barrier(0x002, 16, 0);  // B addresses
  __builtin_amdgcn_sched_group_barrier(0x100, 16, 0);  // B lookups
  __builtin_amdgcn_sched_group_barrier(0x002, 24, 0);  // combine
}

// Final round: SubBytes/ShiftRows only.  S[x] is byte 1 (and 2) of Te0_le[x]
// and byte 3 of Te1_le[x].
__device__ __forceinline__ uint32_t last_col(uint32_t a, uint32_t b, uint32_t c, uint32_t d,
                                             uint32_t k, uint32_t laneoff) {
  uint32_t lo = __builtin_amdgcn_perm(TE0(b, 1), TE0(a, 0), 0x0C0C0501u);
  uint32_t hi = __builtin_amdgcn_perm(TE1(d, 3), TE0(c, 2), 0x07020C0Cu);
  return lo ^ hi ^ k;
}
__device__ __forceinline__ void aes_last(uint32_t& s0, uint32_t& s1, uint32_t& s2, uint32_t& s3,
                                         cu32* rk, uint32_t laneoff) {
  uint32_t t0 = last_col(s0, s1, s2, s3, rk[0], laneoff);
  uint32_t t1 = last_col(s1, s2, s3, s0, rk[1], laneoff);
  uint32_t t2 = last_col(s2, s3, s0, s1, rk[2], laneoff);
  uint32_t t3 = last_col(s3, s0, s1, s2, rk[3], laneoff);
  s0 = t0; s1 = t1; s2 = t2; s3 = t3;
}

// Full block encryption (used for E_K(J0)).
template <int ROUNDS>
__device__ __forceinline__ void aes_block(uint32_t s[4], cu32* rk, cu32* rkr,
                                          uint32_t laneoff) {
  s[0] ^= rk[0]; s[1] ^= rk[1]; s[2] ^= rk[2]; s[3] ^= rk[3];
#pragma unroll
  for (int r = 1; r < ROUNDS; r++)
    aes_round(s[0], s[1], s[2], s[3], rkr[4 * r], rkr[4 * r + 1], rkr[4 * r + 2], rkr[4 * r + 3],
              laneoff);
  aes_last(s[0], s[1], s[2], s[3], rk + 4 * ROUNDS, laneoff);
}

// Per-record CTR constants: J0 columns 0..2 through AddRoundKey 0 and the
// constant three quarters of round 1 (only column 3 carries the counter).
struct CtrConst { uint32_t k1[4]; uint32_t rk03; };

__device__ __forceinline__ CtrConst ctr_setup(const uint32_t j0[4], cu32* rk,
                                              uint32_t laneoff) {
  uint32_t s0 = j0[0] ^ rk[0], s1 = j0[1] ^ rk[1], s2 = j0[2] ^ rk[2];
  CtrConst c;
  c.k1[0] = TE0(s0, 0) ^ TE1(s1, 1) ^ rotl16(TE0(s2, 2)) ^ rk[4];
  c.k1[1] = TE0(s1, 0) ^ TE1(s2, 1) ^ rotl16(TE1(s0, 3)) ^ rk[5];
  c.k1[2] = TE0(s2, 0) ^ rotl16(TE0(s0, 2) ^ TE1(s1, 3)) ^ rk[6];
  c.k1[3] = TE1(s0, 1) ^ rotl16(TE0(s1, 2) ^ TE1(s2, 3)) ^ rk[7];
  c.rk03 = rk[3];
  return c;
}

// Keystream block for 32-bit counter value ctr (big-endian in bytes 12..15),
// general form: only round 1 is shortened.
template <int ROUNDS>
__device__ __forceinline__ void aes_ctr(uint32_t ks[4], uint32_t ctr, const CtrConst& c,
                                        cu32* rk, cu32* rkr, uint32_t laneoff) {
  uint32_t v = bswap32(ctr) ^ c.rk03;
  uint32_t s0 = c.k1[0] ^ rotl16(TE1(v, 3));
  uint32_t s1 = c.k1[1] ^ rotl16(TE0(v, 2));
  uint32_t s2 = c.k1[2] ^ TE1(v, 1);
  uint32_t s3 = c.k1[3] ^ TE0(v, 0);
#pragma unroll
  for (int r = 2; r < ROUNDS; r++)
    aes_round(s0, s1, s2, s3, rkr[4 * r], rkr[4 * r + 1], rkr[4 * r + 2], rkr[4 * r + 3], laneoff);
  aes_last(s0, s1, s2, s3, rk + 4 * ROUNDS, laneoff);
  ks[0] = s0; ks[1] = s1; ks[2] = s2; ks[3] = s3;
}

// Per-record constants for counters below 2^16 (every TLS record: the counter
// runs 2..nb+1 with nb <= 65534).  Counter bytes 12-13 are then zero, so after
// round 1 only columns 0 and 1 depend on the counter and round 2 needs 8
// lookups instead of 16; E_K(J0) rides along.  Computed for 64 records at a
// time (one per lane) and broadcast with readlane when a record is processed.
struct RecConsts {
  uint32_t ek0[4];   // E_K(J0)
  uint32_t k1a, k1b; // round-1 constants of columns 0, 1
  uint32_t k2[4];    // round-2 constants
};

template <int ROUNDS>
__device__ __forceinline__ RecConsts rec_consts(const uint32_t j0[4], cu32* rk, cu32* rkr,
                                                uint32_t laneoff) {
  RecConsts r;
  uint32_t e[4] = {j0[0], j0[1], j0[2], j0[3]};
  aes_block<ROUNDS>(e, rk, rkr, laneoff);
  r.ek0[0] = e[0]; r.ek0[1] = e[1]; r.ek0[2] = e[2]; r.ek0[3] = e[3];
  CtrConst c = ctr_setup(j0, rk, laneoff);
  const uint32_t v0 = c.rk03;           // counter bytes 12..15 = 0 (bytes 12,13 stay 0)
  const uint32_t s2 = c.k1[2] ^ TE1(v0, 1);
  const uint32_t s3 = c.k1[3] ^ TE0(v0, 0);
  r.k1a = c.k1[0];
  r.k1b = c.k1[1];
  r.k2[0] = rotl16(TE0(s2, 2) ^ TE1(s3, 3)) ^ rk[8];
  r.k2[1] = TE1(s2, 1) ^ rotl16(TE0(s3, 2)) ^ rk[9];
  r.k2[2] = TE0(s2, 0) ^ TE1(s3, 1) ^ rk[10];
  r.k2[3] = TE0(s3, 0) ^ rotl16(TE1(s2, 3)) ^ rk[11];
  return r;
}

// Fast keystream for ctr < 2^16: round 1 = 2 lookups, round 2 = 8 lookups.
template <int ROUNDS>
__device__ __forceinline__ void aes_ctr16(uint32_t ks[4], uint32_t ctr, const RecConsts& c,
                                          uint32_t rk03, cu32* rk, cu32* rkr, uint32_t laneoff) {
  const uint32_t v = bswap32(ctr) ^ rk03;
  const uint32_t s0 = c.k1a ^ rotl16(TE1(v, 3));
  const uint32_t s1 = c.k1b ^ rotl16(TE0(v, 2));
  uint32_t t0 = xor3(c.k2[0], TE0(s0, 0), TE1(s1, 1));
  uint32_t t1 = xor3(c.k2[1], TE0(s1, 0), rotl16(TE1(s0, 3)));
  uint32_t t2 = c.k2[2] ^ rotl16(TE0(s0, 2) ^ TE1(s1, 3));
  uint32_t t3 = xor3(c.k2[3], TE1(s0, 1), rotl16(TE0(s1, 2)));
#pragma unroll
  for (int r = 3; r < ROUNDS; r++)
    aes_round(t0, t1, t2, t3, rkr[4 * r], rkr[4 * r + 1], rkr[4 * r + 2], rkr[4 * r + 3], laneoff);
  aes_last(t0, t1, t2, t3, rk + 4 * ROUNDS, laneoff);
  ks[0] = t0; ks[1] = t1; ks[2] = t2; ks[3] = t3;
}

// Two keystream blocks (counters c0, c1) with interleaved rounds.
template <int ROUNDS>
__device__ __forceinline__ void aes_ctr16x2(uint32_t ka[4], uint32_t kb[4], uint32_t c0,
                                            uint32_t c1, const RecConsts& c, uint32_t rk03,
                                            cu32* rk, cu32* rkr, uint32_t laneoff) {
  const uint32_t va = bswap32(c0) ^ rk03, vb = bswap32(c1) ^ rk03;
  const uint32_t a0 = c.k1a ^ rotl16(TE1(va, 3)), a1 = c.k1b ^ rotl16(TE0(va, 2));
  const uint32_t b0 = c.k1a ^ rotl16(TE1(vb, 3)), b1 = c.k1b ^ rotl16(TE0(vb, 2));
  uint32_t A[4], B[4];
  A[0] = xor3(c.k2[0], TE0(a0, 0), TE1(a1, 1));
  A[1] = xor3(c.k2[1], TE0(a1, 0), rotl16(TE1(a0, 3)));
  A[2] = c.k2[2] ^ rotl16(TE0(a0, 2) ^ TE1(a1, 3));
  A[3] = xor3(c.k2[3], TE1(a0, 1), rotl16(TE0(a1, 2)));
  B[0] = xor3(c.k2[0], TE0(b0, 0), TE1(b1, 1));
  B[1] = xor3(c.k2[1], TE0(b1, 0), rotl16(TE1(b0, 3)));
  B[2] = c.k2[2] ^ rotl16(TE0(b0, 2) ^ TE1(b1, 3));
  B[3] = xor3(c.k2[3], TE1(b0, 1), rotl16(TE0(b1, 2)));
#pragma unroll
  for (int r = 3; r < ROUNDS; r++)
    aes_round2(A, B, rkr[4 * r], rkr[4 * r + 1], rkr[4 * r + 2], rkr[4 * r + 3], laneoff);
  aes_last(A[0], A[1], A[2], A[3], rk + 4 * ROUNDS, laneoff);
  aes_last(B[0], B[1], B[2], B[3], rk + 4 * ROUNDS, laneoff);
#pragma unroll
  for (int w = 0; w < 4; w++) { ka[w] = A[w]; kb[w] = B[w]; }
}

// ---------------------------------------------------------------------------
// GHASH helpers.  The record code (gcm_blocks*, gcm_finish, gcm_record_x4) is
// generic in a GHASH policy G with two members:
//   G::mul64(x, o)      o = x * H^64 (LE words), the per-lane Horner step;
//   G::shoup(X, e, Z)   Z = X * H^e, e = 1..65 (BE words), the chain weights.
// GhLane: the session's 64 KiB byte-position table and Shoup tables in LDS,
// shared by the workgroup (queue kernel, one session per run).  GhNib
// (gcm_pw.hip): a per-wave 8 KiB nibble-position table and Shoup tables read
// from HBM/L2 (per-wave-session kernel, any session per wave).
struct GhLane {
  bool c2, c1;       // word-rotation selects for m = lane % 16
  uint32_t r;        // byte rotation
  uint32_t cq[4];    // slot bytes: cq[q].byte[i] = ((4q + i + m) & 15) * 16
  __device__ __forceinline__ void mul64(const uint32_t x[4], uint32_t o[4]) const;
  __device__ __forceinline__ void shoup(const uint32_t X[4], uint32_t e, uint32_t Z[4]) const;
};

__device__ __forceinline__ GhLane gh_lane(uint32_t lane) {
  GhLane g;
  uint32_t m = lane & 15;
  g.c2 = (m >> 3) & 1;
  g.c1 = (m >> 2) & 1;
  g.r = m & 3;
#pragma unroll
  for (int q = 0; q < 4; q++) {
    uint32_t v = 0;
#pragma unroll
    for (int i = 0; i < 4; i++) v |= (((4 * q + i + m) & 15) << 4) << (8 * i);
    g.cq[q] = v;
  }
  return g;
}

template <int K>
__device__ __forceinline__ uint32_t kaddr(uint32_t y, uint32_t cq) {
  return __builtin_amdgcn_perm(y, cq, 0x0C0C0000u | ((4u + K) << 8) | K);
}

// out = x * H^64 using the LDS byte-position table (LE words).
__device__ __forceinline__ void mul_k(const uint32_t x[4], uint32_t o[4], const GhLane& g) {
  uint32_t a0 = g.c2 ? x[2] : x[0], a1 = g.c2 ? x[3] : x[1];
  uint32_t a2 = g.c2 ? x[0] : x[2], a3 = g.c2 ? x[1] : x[3];
  uint32_t b0 = g.c1 ? a1 : a0, b1 = g.c1 ? a2 : a1, b2 = g.c1 ? a3 : a2, b3 = g.c1 ? a0 : a3;
  uint32_t y[4];
  y[0] = __builtin_amdgcn_alignbyte(b1, b0, g.r);
  y[1] = __builtin_amdgcn_alignbyte(b2, b1, g.r);
  y[2] = __builtin_amdgcn_alignbyte(b3, b2, g.r);
  y[3] = __builtin_amdgcn_alignbyte(b0, b3, g.r);
  uint4 acc = make_uint4(0, 0, 0, 0);
#pragma unroll
  for (int q = 0; q < 4; q++) {
    uint4 v0 = lds_u128(KT_OFF + kaddr<0>(y[q], g.cq[q]));
    uint4 v1 = lds_u128(KT_OFF + kaddr<1>(y[q], g.cq[q]));
    uint4 v2 = lds_u128(KT_OFF + kaddr<2>(y[q], g.cq[q]));
    uint4 v3 = lds_u128(KT_OFF + kaddr<3>(y[q], g.cq[q]));
    acc.x = xor3(acc.x, xor3(v0.x, v1.x, v2.x), v3.x);
    acc.y = xor3(acc.y, xor3(v0.y, v1.y, v2.y), v3.y);
    acc.z = xor3(acc.z, xor3(v0.z, v1.z, v2.z), v3.z);
    acc.w = xor3(acc.w, xor3(v0.w, v1.w, v2.w), v3.w);
  }
  o[0] = acc.x; o[1] = acc.y; o[2] = acc.z; o[3] = acc.w;
}

// Two independent chains at once: o_a = x_a * H^64, o_b = x_b * H^64, with all
// 32 lookups issued before any is combined (the chains' latencies overlap).
__device__ __forceinline__ void mul_k2(const uint32_t xa[4], const uint32_t xb[4], uint32_t oa[4],
                                       uint32_t ob[4], const GhLane& g) {
  uint32_t addr[2][16];
  const uint32_t* xs[2] = {xa, xb};
#pragma unroll
  for (int c = 0; c < 2; c++) {
    const uint32_t* x = xs[c];
    uint32_t a0 = g.c2 ? x[2] : x[0], a1 = g.c2 ? x[3] : x[1];
    uint32_t a2 = g.c2 ? x[0] : x[2], a3 = g.c2 ? x[1] : x[3];
    uint32_t b0 = g.c1 ? a1 : a0, b1 = g.c1 ? a2 : a1, b2 = g.c1 ? a3 : a2, b3 = g.c1 ? a0 : a3;
    uint32_t y[4];
    y[0] = __builtin_amdgcn_alignbyte(b1, b0, g.r);
    y[1] = __builtin_amdgcn_alignbyte(b2, b1, g.r);
    y[2] = __builtin_amdgcn_alignbyte(b3, b2, g.r);
    y[3] = __builtin_amdgcn_alignbyte(b0, b3, g.r);
#pragma unroll
    for (int q = 0; q < 4; q++) {
      addr[c][4 * q + 0] = KT_OFF + kaddr<0>(y[q], g.cq[q]);
      addr[c][4 * q + 1] = KT_OFF + kaddr<1>(y[q], g.cq[q]);
      addr[c][4 * q + 2] = KT_OFF + kaddr<2>(y[q], g.cq[q]);
      addr[c][4 * q + 3] = KT_OFF + kaddr<3>(y[q], g.cq[q]);
    }
  }
  // two halves of 8 lookups per chain: at most 16 reads (64 VGPRs) in flight
  uint4 acc[2];
#pragma unroll
  for (int h = 0; h < 2; h++) {
    uint4 v[2][8];
#pragma unroll
    for (int m = 0; m < 8; m++) {
      v[0][m] = lds_u128(addr[0][8 * h + m]);
      v[1][m] = lds_u128(addr[1][8 * h + m]);
    }
#pragma unroll
    for (int c = 0; c < 2; c++) {
      uint4 t;
      t.x = xor3(v[c][0].x, v[c][1].x, v[c][2].x);
      t.y = xor3(v[c][0].y, v[c][1].y, v[c][2].y);
      t.z = xor3(v[c][0].z, v[c][1].z, v[c][2].z);
      t.w = xor3(v[c][0].w, v[c][1].w, v[c][2].w);
#pragma unroll
      for (int m = 3; m < 7; m += 2) {
        t.x = xor3(t.x, v[c][m].x, v[c][m + 1].x);
        t.y = xor3(t.y, v[c][m].y, v[c][m + 1].y);
        t.z = xor3(t.z, v[c][m].z, v[c][m + 1].z);
        t.w = xor3(t.w, v[c][m].w, v[c][m + 1].w);
      }
      if (h == 0) {
        acc[c].x = t.x ^ v[c][7].x; acc[c].y = t.y ^ v[c][7].y;
        acc[c].z = t.z ^ v[c][7].z; acc[c].w = t.w ^ v[c][7].w;
      } else {
        acc[c].x = xor3(acc[c].x, t.x, v[c][7].x); acc[c].y = xor3(acc[c].y, t.y, v[c][7].y);
        acc[c].z = xor3(acc[c].z, t.z, v[c][7].z); acc[c].w = xor3(acc[c].w, t.w, v[c][7].w);
      }
    }
  }
  oa[0] = acc[0].x; oa[1] = acc[0].y; oa[2] = acc[0].z; oa[3] = acc[0].w;
  ob[0] = acc[1].x; ob[1] = acc[1].y; ob[2] = acc[1].z; ob[3] = acc[1].w;
}

// LDS address of the Shoup table of H^e (e = 1..65); entry v at + v * 256.
__device__ __forceinline__ uint32_t sh_base(uint32_t e) {
  const uint32_t i = e - 1;
  return SH_OFF + (i >> 4) * 4096u + (i & 15u) * 16u;
}

// rem_4bit[r] >> 32 (gcm128.c:327-331) on the VALU: (r * 0xE1, carry-less) << 21,
// 0xE1 = x^0 + x^5 + x^6 + x^7, so r*0xE1 = r ^ ((r ^ r<<1 ^ r<<2) << 5).  (A
// 16-entry LDS table read with a random index costs 3-4-way bank conflicts.)
__device__ __forceinline__ uint32_t rem4(uint32_t r) {
  const uint32_t a = xor3(r, r << 1, r << 2);
  return (r << 21) ^ (a << 26);
}

// z = x * H^e (Shoup 4-bit, gcm128.c:333-393), all in big-endian words.
__device__ __forceinline__ void mul_shoup(const uint32_t X[4], uint32_t e, uint32_t Z[4]) {
  const uint32_t base = sh_base(e);
  uint32_t n0 = X[3] & 0xF;
  uint4 m = lds_u128(base + n0 * 256);
  uint32_t z0 = m.x, z1 = m.y, z2 = m.z, z3 = m.w;
#pragma unroll
  for (int k = 1; k < 32; k++) {
    uint32_t nib = (X[3 - k / 8] >> (4 * (k % 8))) & 0xF;
    uint32_t rem = z3 & 0xF;
    z3 = __builtin_amdgcn_alignbit(z2, z3, 4);
    z2 = __builtin_amdgcn_alignbit(z1, z2, 4);
    z1 = __builtin_amdgcn_alignbit(z0, z1, 4);
    z0 = (z0 >> 4) ^ rem4(rem);
    uint4 t = lds_u128(base + nib * 256);
    z0 ^= t.x; z1 ^= t.y; z2 ^= t.z; z3 ^= t.w;
  }
  Z[0] = z0; Z[1] = z1; Z[2] = z2; Z[3] = z3;
}

// The same product with its table reads issued ahead of the chain (round 3):
// the reads depend only on x's nibbles, but the compiler waited for each read
// right after issuing it, so a multiply cost 32 LDS round trips in series.
// Used by the per-record finish (GhLane::shoup); the pack path keeps
// mul_shoup, whose lanes hold their plaintext through the multiply (the
// look-ahead registers made that kernel spill 60 VGPRs).
constexpr int kShoupAhead = 4;
__device__ __forceinline__ void mul_shoup_ahead(const uint32_t X[4], uint32_t e, uint32_t Z[4]) {
  const uint32_t base = sh_base(e);
  uint4 t[32];
#pragma unroll
  for (int k = 0; k < 32; k++) t[k] = lds_u128(base + ((X[3 - k / 8] >> (4 * (k % 8))) & 0xF) * 256);
  uint32_t z0 = t[0].x, z1 = t[0].y, z2 = t[0].z, z3 = t[0].w;
#pragma unroll
  for (int k = 1; k < 32; k++) {
    const uint32_t rem = z3 & 0xF;
    z3 = __builtin_amdgcn_alignbit(z2, z3, 4);
    z2 = __builtin_amdgcn_alignbit(z1, z2, 4);
    z1 = __builtin_amdgcn_alignbit(z0, z1, 4);
    z0 = (z0 >> 4) ^ rem4(rem);
    z0 ^= t[k].x; z1 ^= t[k].y; z2 ^= t[k].z; z3 ^= t[k].w;
  }
  // schedule: kShoupAhead reads first, then one read per chain step
  __builtin_amdgcn_sched_group_barrier(0x100, kShoupAhead, 0);
#pragma unroll
  for (int k = 0; k < 32 - kShoupAhead; k++) {
    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    __builtin_amdgcn_sched_group_barrier(0x002, 10, 0);
  }
  Z[0] = z0; Z[1] = z1; Z[2] = z2; Z[3] = z3;
}

__device__ __forceinline__ void GhLane::mul64(const uint32_t x[4], uint32_t o[4]) const {
  mul_k(x, o, *this);
}
__device__ __forceinline__ void GhLane::shoup(const uint32_t X[4], uint32_t e, uint32_t Z[4]) const {
  mul_shoup_ahead(X, e, Z);
}

// Two independent Shoup multiplies, interleaved; e == 0 gives zero.
__device__ __forceinline__ void mul_shoup2(const uint32_t A[4], uint32_t ea, uint32_t ZA[4],
                                           const uint32_t B[4], uint32_t eb, uint32_t ZB[4]) {
  // empty chains (e == 0) read the H^1 table and are masked to zero at the end
  const uint32_t base_a = sh_base(ea ? ea : 1), base_b = sh_base(eb ? eb : 1);
  const uint32_t ma = ea ? 0xFFFFFFFFu : 0u, mb = eb ? 0xFFFFFFFFu : 0u;
  uint4 m = lds_u128(base_a + (A[3] & 0xF) * 256);
  uint4 n = lds_u128(base_b + (B[3] & 0xF) * 256);
  uint32_t a0 = m.x, a1 = m.y, a2 = m.z, a3 = m.w;
  uint32_t b0 = n.x, b1 = n.y, b2 = n.z, b3 = n.w;
#pragma unroll
  for (int k = 1; k < 32; k++) {
    const uint32_t na = (A[3 - k / 8] >> (4 * (k % 8))) & 0xF;
    const uint32_t nb = (B[3 - k / 8] >> (4 * (k % 8))) & 0xF;
    const uint32_t ra = a3 & 0xF, rb = b3 & 0xF;
    const uint4 ta = lds_u128(base_a + na * 256), tb = lds_u128(base_b + nb * 256);
    const uint32_t qa = rem4(ra), qb = rem4(rb);
    a3 = __builtin_amdgcn_alignbit(a2, a3, 4);
    a2 = __builtin_amdgcn_alignbit(a1, a2, 4);
    a1 = __builtin_amdgcn_alignbit(a0, a1, 4);
    a0 = (a0 >> 4) ^ qa;
    b3 = __builtin_amdgcn_alignbit(b2, b3, 4);
    b2 = __builtin_amdgcn_alignbit(b1, b2, 4);
    b1 = __builtin_amdgcn_alignbit(b0, b1, 4);
    b0 = (b0 >> 4) ^ qb;
    a0 ^= ta.x; a1 ^= ta.y; a2 ^= ta.z; a3 ^= ta.w;
    b0 ^= tb.x; b1 ^= tb.y; b2 ^= tb.z; b3 ^= tb.w;
  }
  ZA[0] = a0 & ma; ZA[1] = a1 & ma; ZA[2] = a2 & ma; ZA[3] = a3 & ma;
  ZB[0] = b0 & mb; ZB[1] = b1 & mb; ZB[2] = b2 & mb; ZB[3] = b3 & mb;
}

// Serial GHASH over a byte string with H (all lanes redundantly, rare path:
// non-96-bit IVs and RAW-mode AAD).  x is big-endian words.  When final_mul
// is false the last block is only XORed in (no trailing multiply).
__device__ void ghash_serial(uint32_t x[4], const uint8_t* p, uint64_t len, bool final_mul) {
  const bool al4 = ((uintptr_t)p & 3) == 0;
  for (uint64_t off = 0; off < len; off += 16) {
    uint32_t b[4] = {0, 0, 0, 0};
    if (al4) {  // whole words (a 4-B aligned word cannot cross a page), tail bytes masked
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const int64_t nb = (int64_t)(len - off) - 4 * k;
        if (nb > 0) {
          const uint32_t w = reinterpret_cast<const uint32_t*>(p + off)[k];
          b[k] = bswap32(nb >= 4 ? w : (w & ((1u << (8 * nb)) - 1u)));
        }
      }
    } else {
#pragma unroll
      for (int k = 0; k < 16; k++)
        if (off + k < len) b[k >> 2] |= (uint32_t)p[off + k] << (24 - 8 * (k & 3));
    }
    x[0] ^= b[0]; x[1] ^= b[1]; x[2] ^= b[2]; x[3] ^= b[3];
    if (off + 16 < len || final_mul) {
      uint32_t z[4];
      mul_shoup(x, 1, z);
      x[0] = z[0]; x[1] = z[1]; x[2] = z[2]; x[3] = z[3];
    }
  }
}

__device__ __forceinline__ void be_from_le(const uint32_t* l, uint32_t* b) {
  b[0] = bswap32(l[0]); b[1] = bswap32(l[1]); b[2] = bswap32(l[2]); b[3] = bswap32(l[3]);
}

// ---------------------------------------------------------------------------
// Memory helpers (records are byte-aligned in general).
__device__ __forceinline__ uint32_t load_u32_bytes(const uint8_t* p) {
  if (((uintptr_t)p & 3) == 0) return *reinterpret_cast<const uint32_t*>(p);  // one load, not four
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

// (load16_any / store16_any: tlsgpu_internal.h)
__device__ __forceinline__ void load_block(const uint8_t* p, uint32_t nbytes, bool aligned,
                                           uint32_t v[4]) {
  if (aligned && nbytes == 16) {
    uint4 t = *reinterpret_cast<const uint4*>(p);
    v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
  } else if (nbytes == 16) {
    load16_any(p, v);
  } else if (nbytes != 0 && ((uintptr_t)p & 15) == 0) {
    // a partial last block at a 16-B aligned address: one 16-B load (it cannot
    // cross a page) with the bytes past the end masked, not up to 15 byte loads
    const uint4 t = *reinterpret_cast<const uint4*>(p);
    const uint32_t w[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const int32_t b = (int32_t)nbytes - 4 * k;
      v[k] = w[k] & (b >= 4 ? 0xFFFFFFFFu : (b <= 0 ? 0u : ((1u << (8 * b)) - 1u)));
    }
  } else {
    v[0] = v[1] = v[2] = v[3] = 0;
#pragma unroll
    for (uint32_t k = 0; k < 16; k++)
      if (k < nbytes) v[k >> 2] |= (uint32_t)p[k] << (8 * (k & 3));
  }
}

__device__ __forceinline__ void store_block(uint8_t* p, uint32_t nbytes, bool aligned,
                                            const uint32_t v[4]) {
  if (nbytes == 16 && aligned) {
    *reinterpret_cast<uint4*>(p) = make_uint4(v[0], v[1], v[2], v[3]);
  } else if (nbytes == 16) {
    store16_any(p, v);
  } else {
#pragma unroll
    for (uint32_t k = 0; k < 16; k++)
      if (k < nbytes) p[k] = (uint8_t)(v[k >> 2] >> (8 * (k & 3)));
  }
}


// ---------------------------------------------------------------------------
// Per-record context after parsing (TLS descriptor or raw job).
struct RecCtx {
  const uint8_t* src;     // open: ciphertext ; seal: plaintext
  uint8_t* dst;           // open: plaintext  ; seal: ciphertext
  const uint8_t* tag_in;  // open: received tag (tag_len bytes)
  uint32_t tag_byte;      // open: tag_in[lane] for lane < tag_len, loaded at parse
                          // time so the tag check never waits on HBM
  uint8_t* tag_out;       // seal: where the tag goes
  uint32_t n;             // plaintext length
  uint32_t j0[4];         // J0 (LE words)
  uint32_t aad_be[4];     // AAD' = Horner of the AAD blocks without the final
                          // multiply (gcm128.c:826-881 folded), BE words
  uint64_t aad_len;       // bytes of AAD (for the lengths block)
  uint64_t zero_len;      // bytes of dst zero-filled on failure
  int32_t ok_status;      // status written on success
};

// Close the lane chains of a record: the lengths block BE64(aad bits) ||
// BE64(ct bits) joins lane (nb % 64)'s chain at j = nb (gcm128.c:1477-1500),
// then each lane's value still needs the weight H^e, e = nb + 1 - (index of
// the chain's last element).  Returns the BE chain value and e (0 = empty).
template <class G>
__device__ __forceinline__ uint32_t gcm_close_chain(const RecCtx& rc, uint32_t (&x)[4],
                                                    uint32_t (&xb)[4], uint32_t lane,
                                                    const G& gl) {
  const uint32_t n = rc.n;
  const uint32_t nb = (n + 15) >> 4;
  const uint32_t lstar = nb & 63;
  uint32_t xk[4];
  gl.mul64(x, xk);
  if (lane == lstar) {
    uint64_t ab = rc.aad_len * 8, cb = (uint64_t)n * 8;
    x[0] = xk[0] ^ bswap32((uint32_t)(ab >> 32));
    x[1] = xk[1] ^ bswap32((uint32_t)ab);
    x[2] = xk[2] ^ bswap32((uint32_t)(cb >> 32));
    x[3] = xk[3] ^ bswap32((uint32_t)cb);
  }
  int32_t jlast;
  if (lane == lstar) {
    jlast = (int32_t)nb;
  } else if (lane < nb) {
    jlast = (int32_t)(lane + ((nb - 1 - lane) & ~63u));
  } else {
    jlast = (rc.aad_len != 0 && lane == 63) ? -1 : -2;  // -2: empty chain
  }
  be_from_le(x, xb);
  return jlast == -2 ? 0u : (uint32_t)((int32_t)nb + 1 - jlast);
}

// Zero n bytes at d (the plaintext of a record whose tag failed,
// evp_aead.c:137-143): the whole wave, 16-B stores for the aligned bulk (a
// byte loop made a tampered 16 KiB record's wave 256 store rounds long).
__device__ __forceinline__ void zero_fill_wave(uint8_t* d, uint64_t n, uint32_t lane) {
  const uint64_t head = min(n, (uint64_t)((16u - ((uintptr_t)d & 15u)) & 15u));
  if (lane < head) d[lane] = 0;
  uint4* b = reinterpret_cast<uint4*>(d + head);
  const uint64_t nb = (n - head) >> 4;
  for (uint64_t k = lane; k < nb; k += kWave) b[k] = make_uint4(0, 0, 0, 0);
  const uint64_t done = head + 16 * nb;
  if (lane < n - done) d[done + lane] = 0;
}

// Sum the weighted lane values across the wave, form the tag (GHASH ^ E_K(J0))
// and check it (open, constant time over the tag bytes, zero-fill on failure:
// e_aes.c:1492-1506, evp_aead.c:137-143) or write it (seal, e_aes.c:1452-1456).
template <bool SEAL>
__device__ __forceinline__ void gcm_tag(const RecCtx& rc, uint32_t (&y)[4], const uint32_t ek0[4],
                                        const DevSession* __restrict__ S, int32_t* status_slot,
                                        uint32_t lane) {
  y[0] = wave_xor_total(y[0]);
  y[1] = wave_xor_total(y[1]);
  y[2] = wave_xor_total(y[2]);
  y[3] = wave_xor_total(y[3]);
  // tag = GHASH ^ E_K(J0)  (y is BE words, ek0 LE words)
  uint32_t tag[4] = {bswap32(y[0]) ^ ek0[0], bswap32(y[1]) ^ ek0[1], bswap32(y[2]) ^ ek0[2],
                     bswap32(y[3]) ^ ek0[3]};
  const uint32_t tag_len = as_const(&S->tag_len)[0];
  const uint32_t tw = lane >> 2;
  const uint32_t tword = tw == 0 ? tag[0] : tw == 1 ? tag[1] : tw == 2 ? tag[2] : tag[3];
  const uint32_t tbyte = (tword >> (8 * (lane & 3))) & 0xFF;
  if (SEAL) {
    if (lane < tag_len) rc.tag_out[lane] = (uint8_t)tbyte;
    if (lane == 0) *status_slot = rc.ok_status;
  } else {
    uint32_t diff = 0;
    if (lane < tag_len) diff = rc.tag_byte ^ tbyte;
    bool bad = __any(diff != 0);  // constant-time in the data: every lane compares
    if (bad) {
      zero_fill_wave(rc.dst, rc.zero_len, lane);
    }
    if (lane == 0) *status_slot = bad ? TLSGPU_REC_BAD_MAC : rc.ok_status;
  }
}

// Finish one record (chains -> weights -> tag).
template <bool SEAL, class G>
__device__ __forceinline__ void gcm_finish(const RecCtx& rc, uint32_t (&x)[4], const uint32_t ek0[4],
                                           const DevSession* __restrict__ S, int32_t* status_slot,
                                           uint32_t lane, const G& gl) {
  uint32_t xb[4], y[4] = {0, 0, 0, 0};
  const uint32_t e = gcm_close_chain(rc, x, xb, lane, gl);
  if (e != 0) gl.shoup(xb, e, y);
  gcm_tag<SEAL>(rc, y, ek0, S, status_slot, lane);
}

// Finish two records with their Shoup multiplies interleaved (two independent
// 32-step LDS chains per lane instead of two back-to-back ones).
template <bool SEAL>
__device__ __forceinline__ void gcm_finish2(const RecCtx (&rc)[2], uint32_t (&x)[2][4],
                                            const uint32_t (&ek)[2][4],
                                            const DevSession* __restrict__ S, int32_t* slot_a,
                                            int32_t* slot_b, uint32_t lane, const GhLane& gl) {
  uint32_t xb[2][4], y[2][4];
  const uint32_t ea = gcm_close_chain(rc[0], x[0], xb[0], lane, gl);
  const uint32_t eb = gcm_close_chain(rc[1], x[1], xb[1], lane, gl);
  mul_shoup2(xb[0], ea, y[0], xb[1], eb, y[1]);
  gcm_tag<SEAL>(rc[0], y[0], ek[0], S, slot_a, lane);
  gcm_tag<SEAL>(rc[1], y[1], ek[1], S, slot_b, lane);
}

// CTR en/decryption of blocks [start, nb) fused with the lane GHASH chains x
// (start is a multiple of 64: block i belongs to lane i % 64's chain).
// FAST: counters < 2^16 and the per-record constants `rcc` were precomputed
// (wave-uniform values); otherwise `cc` (ctr_setup) is used.
template <bool SEAL, int ROUNDS, bool FAST, class G>
__device__ __forceinline__ void gcm_blocks(const RecCtx& rc, const DevSession* __restrict__ S,
                                           const RecConsts& rcc, const CtrConst& cc,
                                           uint32_t (&x)[4], uint32_t start, uint32_t lane,
                                           uint32_t laneoff, const G& gl) {
  cu32* rk = as_const(S->rk);
  cu32* rkr = as_const(S->rk_rot);
  const uint32_t n = rc.n;
  const uint32_t nb = (n + 15) >> 4;
  const uint32_t rk03 = rk[3];
  auto keystream = [&](uint32_t ks[4], uint32_t ctr) {
    if (FAST)
      aes_ctr16<ROUNDS>(ks, ctr, rcc, rk03, rk, rkr, laneoff);
    else
      aes_ctr<ROUNDS>(ks, ctr, cc, rk, rkr, laneoff);
  };
  const uint32_t ctr0 = bswap32(rc.j0[3]) + 1u;  // inc32(J0), gcm128.c:815-823
  const bool aligned = ((((uintptr_t)rc.src) | ((uintptr_t)rc.dst)) & 15) == 0;

  // Full-block steps, two per iteration (two independent AES chains per lane
  // keep twice as many LDS lookups in flight), with the next iteration's
  // ciphertext loads issued before this iteration's AES.
  const uint32_t nfull_steps = (n >> 4) / kWave;
  uint32_t base = start;
  if (nfull_steps >= start / kWave + 2) {
    uint32_t c0[4], c1[4];
    load_block(rc.src + 16u * (start + lane), 16, aligned, c0);
    load_block(rc.src + 16u * (start + lane + kWave), 16, aligned, c1);
    uint32_t t = start / kWave;
    for (; t + 2 <= nfull_steps; t += 2, base += 2 * kWave) {
      const uint32_t i = base + lane;
      uint32_t n0[4] = {0, 0, 0, 0}, n1[4] = {0, 0, 0, 0};
      if (t + 4 <= nfull_steps) {
        load_block(rc.src + 16u * (i + 2 * kWave), 16, aligned, n0);
        load_block(rc.src + 16u * (i + 3 * kWave), 16, aligned, n1);
      }
      uint32_t k0[4], k1[4];
      if (FAST) {
        aes_ctr16x2<ROUNDS>(k0, k1, ctr0 + i, ctr0 + i + kWave, rcc, rk03, rk, rkr, laneoff);
      } else {
        keystream(k0, ctr0 + i);
        keystream(k1, ctr0 + i + kWave);
      }
      uint32_t o0[4] = {c0[0] ^ k0[0], c0[1] ^ k0[1], c0[2] ^ k0[2], c0[3] ^ k0[3]};
      uint32_t o1[4] = {c1[0] ^ k1[0], c1[1] ^ k1[1], c1[2] ^ k1[2], c1[3] ^ k1[3]};
      store_block(rc.dst + 16u * i, 16, aligned, o0);
      store_block(rc.dst + 16u * (i + kWave), 16, aligned, o1);
      uint32_t xk[4];
      gl.mul64(x, xk);
      const uint32_t* g0 = SEAL ? o0 : c0;
      const uint32_t* g1 = SEAL ? o1 : c1;
      x[0] = xk[0] ^ g0[0]; x[1] = xk[1] ^ g0[1]; x[2] = xk[2] ^ g0[2]; x[3] = xk[3] ^ g0[3];
      gl.mul64(x, xk);
      x[0] = xk[0] ^ g1[0]; x[1] = xk[1] ^ g1[1]; x[2] = xk[2] ^ g1[2]; x[3] = xk[3] ^ g1[3];
#pragma unroll
      for (int w = 0; w < 4; w++) { c0[w] = n0[w]; c1[w] = n1[w]; }
    }
  }
  // Two remaining steps at a time when the first is full (short records have
  // no full step pairs; this halves their serial AES latency), masked second.
  if (FAST) {
    for (; base + kWave < nb; base += 2 * kWave) {
      const uint32_t i0 = base + lane, i1 = i0 + kWave;  // i0 < nb always
      const bool a1 = i1 < nb;
      const uint32_t nb0 = min(16u, n - 16u * i0), nb1 = a1 ? min(16u, n - 16u * i1) : 0u;
      uint32_t in0[4], in1[4], k0[4], k1[4];
      load_block(rc.src + 16u * i0, nb0, aligned, in0);
      load_block(rc.src + 16u * i1, nb1, aligned, in1);
      aes_ctr16x2<ROUNDS>(k0, k1, ctr0 + i0, ctr0 + i1, rcc, rk[3], rk, as_const(S->rk_rot), laneoff);
#pragma unroll
      for (int w = 0; w < 4; w++) {
        const int32_t b0 = (int32_t)nb0 - 4 * w, b1 = (int32_t)nb1 - 4 * w;
        k0[w] &= b0 >= 4 ? 0xFFFFFFFFu : (b0 <= 0 ? 0u : ((1u << (8 * b0)) - 1u));
        k1[w] &= b1 >= 4 ? 0xFFFFFFFFu : (b1 <= 0 ? 0u : ((1u << (8 * b1)) - 1u));
      }
      uint32_t o0[4] = {in0[0] ^ k0[0], in0[1] ^ k0[1], in0[2] ^ k0[2], in0[3] ^ k0[3]};
      uint32_t o1[4] = {in1[0] ^ k1[0], in1[1] ^ k1[1], in1[2] ^ k1[2], in1[3] ^ k1[3]};
      store_block(rc.dst + 16u * i0, nb0, aligned, o0);
      if (a1) store_block(rc.dst + 16u * i1, nb1, aligned, o1);
      uint32_t xk[4];
      gl.mul64(x, xk);
      const uint32_t* g0 = SEAL ? o0 : in0;
      x[0] = xk[0] ^ g0[0]; x[1] = xk[1] ^ g0[1]; x[2] = xk[2] ^ g0[2]; x[3] = xk[3] ^ g0[3];
      gl.mul64(x, xk);
      if (a1) {
        const uint32_t* g1 = SEAL ? o1 : in1;
        x[0] = xk[0] ^ g1[0]; x[1] = xk[1] ^ g1[1]; x[2] = xk[2] ^ g1[2]; x[3] = xk[3] ^ g1[3];
      }
    }
  }
  // Remaining steps (odd full step, partial wave, partial last block).
  for (; base < nb; base += kWave) {
    const uint32_t i = base + lane;
    const bool active = i < nb;
    const uint32_t nbytes = active ? min(16u, n - 16u * i) : 0u;
    uint32_t in[4];
    load_block(rc.src + 16u * i, nbytes, aligned, in);
    uint32_t ks[4];
    keystream(ks, ctr0 + i);
#pragma unroll
    for (int w = 0; w < 4; w++) {  // zero-padded GHASH block for the partial tail
      int32_t b = (int32_t)nbytes - 4 * w;
      uint32_t keep = b >= 4 ? 0xFFFFFFFFu : (b <= 0 ? 0u : ((1u << (8 * b)) - 1u));
      ks[w] &= keep;
    }
    uint32_t ob[4] = {in[0] ^ ks[0], in[1] ^ ks[1], in[2] ^ ks[2], in[3] ^ ks[3]};
    if (active) store_block(rc.dst + 16u * i, nbytes, aligned, ob);
    uint32_t xk[4];
    gl.mul64(x, xk);
    if (active) {
      const uint32_t* c = SEAL ? ob : in;
      x[0] = xk[0] ^ c[0]; x[1] = xk[1] ^ c[1]; x[2] = xk[2] ^ c[2]; x[3] = xk[3] ^ c[3];
    }
  }

}

// GHASH(AAD || C || lengths) with the lane chains described in the header,
// fused with CTR en/decryption.  Checks the tag (open) or writes it (seal).
template <bool SEAL, int ROUNDS, bool FAST>
__device__ void gcm_record(const RecCtx& rc, const DevSession* __restrict__ S,
                           const RecConsts& rcc, int32_t* status_slot, uint32_t lane,
                           uint32_t laneoff, const GhLane& gl) {
  cu32* rk = as_const(S->rk);
  cu32* rkr = as_const(S->rk_rot);
  uint32_t ek0[4];
  CtrConst cc;
  if (FAST) {
    ek0[0] = rcc.ek0[0]; ek0[1] = rcc.ek0[1]; ek0[2] = rcc.ek0[2]; ek0[3] = rcc.ek0[3];
  } else {
    ek0[0] = rc.j0[0]; ek0[1] = rc.j0[1]; ek0[2] = rc.j0[2]; ek0[3] = rc.j0[3];
    aes_block<ROUNDS>(ek0, rk, rkr, laneoff);
    cc = ctr_setup(rc.j0, rk, laneoff);
  }
  // Horner chain state (LE words).  The AAD' element sits at j = -1, i.e. in
  // lane 63's chain one H^64 step before C_63.
  uint32_t x[4] = {0, 0, 0, 0};
  if (rc.aad_len != 0 && lane == 63) {
    x[0] = bswap32(rc.aad_be[0]); x[1] = bswap32(rc.aad_be[1]);
    x[2] = bswap32(rc.aad_be[2]); x[3] = bswap32(rc.aad_be[3]);
  }
  gcm_blocks<SEAL, ROUNDS, FAST>(rc, S, rcc, cc, x, 0, lane, laneoff, gl);
  gcm_finish<SEAL>(rc, x, ek0, S, status_slot, lane, gl);
}

// ---------------------------------------------------------------------------
// L2 prefetch: one dword of each 128-B line of [p, p + bytes), N lines per
// lane.  Ordinary (cached) loads whose values are handed to an empty asm at
// prefetch_done(), so the compiler counts them in vmcnt and waits for them
// only there; as the wave's oldest loads they have long completed by then.
template <int N>
struct Prefetch {
  uint32_t v[N];
};
template <int N>
__device__ __forceinline__ Prefetch<N> l2_prefetch(const uint8_t* p, uint32_t bytes, uint32_t lane) {
  Prefetch<N> f;
#pragma unroll
  for (int k = 0; k < N; k++) {
    const uint32_t off = (uint32_t)(k * 64 + lane) * 128u;
    f.v[k] = off < bytes ? *reinterpret_cast<const uint32_t*>(p + off) : 0u;
  }
  return f;
}
template <int N>
__device__ __forceinline__ void prefetch_done(const Prefetch<N>& f) {
#pragma unroll
  for (int k = 0; k < N; k++) asm volatile("" ::"v"(f.v[k]));
}

// ---------------------------------------------------------------------------
// Phase timing (diagnostic, BatchArgs::dbg != null, env TLSGPU_PHASE_STATS):
// shader-clock cycles per phase summed over waves, dbg[2i] = cycles,
// dbg[2i+1] = events.
struct PhaseClock {
  unsigned long long* dbg;
  uint64_t t;
  __device__ __forceinline__ PhaseClock(unsigned long long* d) : dbg(d), t(d ? __builtin_amdgcn_s_memtime() : 0) {}
  // counters live in LDS (DBG_OFF) during the launch; the kernel flushes them
  __device__ __forceinline__ void lap(int i, uint32_t lane) {
    if (dbg) {
      const uint64_t n = __builtin_amdgcn_s_memtime();
      if (lane == 0) {
        unsigned long long* c = reinterpret_cast<unsigned long long*>(s_lds + DBG_OFF);
        atomicAdd(c + 2 * i, (unsigned long long)(n - t));
        atomicAdd(c + 2 * i + 1, 1ull);
      }
      t = __builtin_amdgcn_s_memtime();
    }
  }
};

// ---------------------------------------------------------------------------
// NB-block T-table keystream (the hybrid kernel's T-table waves run alone on
// their SIMD's LDS share, so they keep 16 * NB lookups in flight per round).
template <int NB>
__device__ __forceinline__ void aes_roundN(uint32_t (&s)[NB][4], uint32_t k0, uint32_t k1,
                                           uint32_t k2, uint32_t k3, uint32_t laneoff) {
  uint32_t t[NB][16];
#pragma unroll
  for (int b = 0; b < NB; b++)
#pragma unroll
    for (int c = 0; c < 4; c++) {
      t[b][4 * c + 0] = TE0(s[b][c], 0);
      t[b][4 * c + 1] = TE1(s[b][(c + 1) & 3], 1);
      t[b][4 * c + 2] = TE0(s[b][(c + 2) & 3], 2);
      t[b][4 * c + 3] = TE1(s[b][(c + 3) & 3], 3);
    }
  const uint32_t k[4] = {k0, k1, k2, k3};
#pragma unroll
  for (int b = 0; b < NB; b++)
#pragma unroll
    for (int c = 0; c < 4; c++)
      s[b][c] = xor3(t[b][4 * c], t[b][4 * c + 1], rotl16(xor3(t[b][4 * c + 2], t[b][4 * c + 3], k[c])));
#ifdef TG_SCHED_HINTS  // measured 3 % slower than the compiler schedule (queue kernel)
#pragma unroll
  for (int b = 0; b < NB; b++) {
    __builtin_amdgcn_sched_group_barrier(0x002, 16, 0);  // addresses of block b
    __builtin_amdgcn_sched_group_barrier(0x100, 16, 0);  // its lookups
  }
  __builtin_amdgcn_sched_group_barrier(0x002, 12 * NB, 0);  // combine
#endif
}

// NB keystream blocks for counters ctr[b] < 2^16 (aes_ctr16 generalised).
template <int NB, int ROUNDS, class Hook>
__device__ __forceinline__ void aes_ctr16xN(uint32_t (&ks)[NB][4], const uint32_t (&ctr)[NB],
                                            const RecConsts& c, uint32_t rk03, cu32* rk,
                                            cu32* rkr, uint32_t laneoff, Hook&& hook) {
  uint32_t A[NB][4];
#pragma unroll
  for (int b = 0; b < NB; b++) {
    const uint32_t v = bswap32(ctr[b]) ^ rk03;
    const uint32_t s0 = c.k1a ^ rotl16(TE1(v, 3)), s1 = c.k1b ^ rotl16(TE0(v, 2));
    A[b][0] = xor3(c.k2[0], TE0(s0, 0), TE1(s1, 1));
    A[b][1] = xor3(c.k2[1], TE0(s1, 0), rotl16(TE1(s0, 3)));
    A[b][2] = c.k2[2] ^ rotl16(TE0(s0, 2) ^ TE1(s1, 3));
    A[b][3] = xor3(c.k2[3], TE1(s0, 1), rotl16(TE0(s1, 2)));
  }
#pragma unroll
  for (int r = 3; r < ROUNDS; r++) {
    aes_roundN<NB>(A, rkr[4 * r], rkr[4 * r + 1], rkr[4 * r + 2], rkr[4 * r + 3], laneoff);
    hook(r);  // work independent of A (GHASH of the previous group) between rounds
  }
#pragma unroll
  for (int b = 0; b < NB; b++) {
    aes_last(A[b][0], A[b][1], A[b][2], A[b][3], rk + 4 * ROUNDS, laneoff);
#pragma unroll
    for (int w = 0; w < 4; w++) ks[b][w] = A[b][w];
  }
}
template <int NB, int ROUNDS>
__device__ __forceinline__ void aes_ctr16xN(uint32_t (&ks)[NB][4], const uint32_t (&ctr)[NB],
                                            const RecConsts& c, uint32_t rk03, cu32* rk,
                                            cu32* rkr, uint32_t laneoff) {
  aes_ctr16xN<NB, ROUNDS>(ks, ctr, c, rk03, rk, rkr, laneoff, [](int) {});
}

// Full NB-step groups of a record (any alignment) from block `start` on (FAST
// constants only): NB keystream blocks per lane in flight, the next group's
// input loads issued first, and the GHASH of each group's NB blocks folded
// into the AES rounds of the following group (the chain's LDS round trips then
// overlap the AES lookups instead of trailing them).  Advances `start` past
// the groups done; the caller finishes the record with gcm_blocks.
template <bool SEAL, int ROUNDS, int NB, class G>
__device__ __forceinline__ void gcm_blocks_xN(const RecCtx& rc, const DevSession* __restrict__ S,
                                              const RecConsts& rcc, uint32_t (&x)[4],
                                              uint32_t& start, uint32_t lane, uint32_t laneoff,
                                              const G& gl) {
  const bool aligned = ((((uintptr_t)rc.src) | ((uintptr_t)rc.dst)) & 15) == 0;
#ifndef TG_XN_UNALIGNED
  if (!aligned) return;
#endif
  cu32* rk = as_const(S->rk);
  cu32* rkr = as_const(S->rk_rot);
  const uint32_t rk03 = rk[3];
  const uint32_t ctr0 = bswap32(rc.j0[3]) + 1u;
  const uint32_t nfull_steps = (rc.n >> 4) / kWave;
  uint32_t t = start / kWave;
  if (t + NB > nfull_steps) return;
  uint32_t c[NB][4], gp[NB][4];
#pragma unroll
  for (int b = 0; b < NB; b++) load_block(rc.src + 16u * (start + kWave * b + lane), 16, aligned, c[b]);
  auto ghash_step = [&](int b) {
    uint32_t xk[4];
    gl.mul64(x, xk);
    x[0] = xk[0] ^ gp[b][0]; x[1] = xk[1] ^ gp[b][1]; x[2] = xk[2] ^ gp[b][2]; x[3] = xk[3] ^ gp[b][3];
  };
  // GHASH step b of the previous group after AES round 3 + 2b (all NB steps
  // fall inside rounds 3 .. ROUNDS-1)
  static_assert(3 + 2 * (NB - 1) < ROUNDS, "GHASH steps must fit between the AES rounds");
  auto hook = [&](int r) {
#pragma unroll
    for (int b = 0; b < NB; b++)
      if (r == 3 + 2 * b) ghash_step(b);
  };
  bool first = true;
  for (; t + NB <= nfull_steps; t += NB, start += NB * kWave) {
    const uint32_t i = start + lane;
    uint32_t nx[NB][4];
    if (t + 2 * NB <= nfull_steps) {
#pragma unroll
      for (int b = 0; b < NB; b++) load_block(rc.src + 16u * (i + kWave * (NB + b)), 16, aligned, nx[b]);
    }
    uint32_t ctr[NB], k[NB][4];
#pragma unroll
    for (int b = 0; b < NB; b++) ctr[b] = ctr0 + i + kWave * b;
    if (first)
      aes_ctr16xN<NB, ROUNDS>(k, ctr, rcc, rk03, rk, rkr, laneoff);
    else
      aes_ctr16xN<NB, ROUNDS>(k, ctr, rcc, rk03, rk, rkr, laneoff, hook);
    first = false;
#pragma unroll
    for (int b = 0; b < NB; b++) {
      uint32_t o[4] = {c[b][0] ^ k[b][0], c[b][1] ^ k[b][1], c[b][2] ^ k[b][2], c[b][3] ^ k[b][3]};
      store_block(rc.dst + 16u * (i + kWave * b), 16, aligned, o);
#pragma unroll
      for (int w = 0; w < 4; w++) gp[b][w] = SEAL ? o[w] : c[b][w];
    }
#pragma unroll
    for (int b = 0; b < NB; b++)
#pragma unroll
      for (int w = 0; w < 4; w++) c[b][w] = nx[b][w];
  }
#pragma unroll
  for (int b = 0; b < NB; b++) ghash_step(b);  // the last group's GHASH
}

// gcm_record<SEAL, ROUNDS, true> with the NB-wide full-block loop first.
template <bool SEAL, int ROUNDS, int NB = 4, class G = GhLane>
__device__ void gcm_record_x4(const RecCtx& rc, const DevSession* __restrict__ S,
                              const RecConsts& rcc, int32_t* status_slot, uint32_t lane,
                              uint32_t laneoff, const G& gl,
                              unsigned long long* dbg = nullptr) {
  PhaseClock pc(dbg);
  uint32_t x[4] = {0, 0, 0, 0};
  if (rc.aad_len != 0 && lane == 63) {
    x[0] = bswap32(rc.aad_be[0]); x[1] = bswap32(rc.aad_be[1]);
    x[2] = bswap32(rc.aad_be[2]); x[3] = bswap32(rc.aad_be[3]);
  }
  uint32_t start = 0;
  gcm_blocks_xN<SEAL, ROUNDS, NB>(rc, S, rcc, x, start, lane, laneoff, gl);
#ifdef TG_XN_ODD_STEP
  // an odd full step left by the NB-wide loop: the pipelined one-step loop
  if (NB > 1) gcm_blocks_xN<SEAL, ROUNDS, 1>(rc, S, rcc, x, start, lane, laneoff, gl);
#endif
  pc.lap(9, lane);
  const CtrConst none = {};
  gcm_blocks<SEAL, ROUNDS, true>(rc, S, rcc, none, x, start, lane, laneoff, gl);
  pc.lap(10, lane);
  gcm_finish<SEAL>(rc, x, rcc.ek0, S, status_slot, lane, gl);
  pc.lap(11, lane);
}

__device__ __forceinline__ uint64_t uni64(uint64_t v) {
  return ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32)) << 32) |
         __builtin_amdgcn_readfirstlane((uint32_t)v);
}
__device__ __forceinline__ tlsgpu_record load_desc(const tlsgpu_record* p) {
  cu32* w = as_const(p);
  tlsgpu_record d;
  d.in_off = ((uint64_t)w[1] << 32) | w[0];
  d.out_off = ((uint64_t)w[3] << 32) | w[2];
  d.seq = ((uint64_t)w[5] << 32) | w[4];
  d.session = w[6];
  d.len_type = w[7];
  return d;
}

// J0 of record r for this lane (the batched constant pass): fixed IV(4) ||
// explicit nonce(8) || 0x00000001 — the explicit nonce is the record's first
// 8 bytes on open and the sequence number on seal (t1_enc.c:887-892, 941-948).
template <bool SEAL>
__device__ __forceinline__ void lane_j0(const tlsgpu_record* D, uint32_t r, uint32_t run_end,
                                        const DevSession* __restrict__ S, const uint8_t* in,
                                        uint32_t j0[4]) {
  j0[0] = as_const(S->fixed_nonce)[0];
  j0[1] = j0[2] = 0;
  j0[3] = 0x01000000u;
  if (r >= run_end) return;
  const tlsgpu_record d = D[r];
  if (SEAL) {
    j0[1] = bswap32((uint32_t)(d.seq >> 32));
    j0[2] = bswap32((uint32_t)d.seq);
  } else if ((d.len_type & 0xFFFFFFu) >= 8) {
    const uint8_t* p = in + d.in_off;
    j0[1] = load_u32_bytes(p);
    j0[2] = load_u32_bytes(p + 4);
  }
}

// Build the per-record context from a TLS descriptor (t1_enc.c:832-975).
// Returns false (and writes the status) when tls1_enc would return 0.
template <bool SEAL>
__device__ __forceinline__ bool parse_tls(const tlsgpu_record& d, const DevSession* __restrict__ S,
                                          const uint8_t* in, uint8_t* out, int32_t* status_slot,
                                          uint32_t lane, RecCtx& rc) {
  uint32_t len = d.len_type & 0xFFFFFFu;
  uint32_t type = d.len_type >> 24;
  const uint8_t* ip = in + d.in_off;
  uint8_t* op = out + d.out_off;
  uint8_t explicit_nonce[8];
  uint32_t tag_len = as_const(&S->tag_len)[0];
  if (SEAL ? len > TLSGPU_MAX_RECORD : (len < 8 || len - 8 < tag_len ||
                                          len - 8 - tag_len > TLSGPU_MAX_RECORD)) {
    if (lane == 0) *status_slot = TLSGPU_REC_PUBLIC_INVALID;
    return false;
  }
  if (SEAL) {
    rc.n = len;
    rc.src = ip;
    rc.dst = op + 8;
    rc.tag_out = op + 8 + len;
    rc.tag_in = nullptr;
    for (int k = 0; k < 8; k++) explicit_nonce[k] = (uint8_t)(d.seq >> (56 - 8 * k));
    if (lane < 8) op[lane] = (uint8_t)(d.seq >> (56 - 8 * lane));  // explicit nonce into the record
    rc.ok_status = (int32_t)(len + 8 + tag_len);
    rc.zero_len = 0;
  } else {
    for (int k = 0; k < 8; k++) explicit_nonce[k] = ip[k];
    rc.n = len - 8 - tag_len;
    rc.src = ip + 8;
    rc.dst = op;
    rc.tag_in = ip + 8 + rc.n;
    rc.tag_byte = lane < tag_len ? rc.tag_in[lane] : 0u;
    rc.tag_out = nullptr;
    rc.ok_status = (int32_t)rc.n;
    rc.zero_len = rc.n;
  }
  // nonce = fixed_iv(4) || explicit(8); J0 = nonce || 0x00000001
  rc.j0[0] = as_const(S->fixed_nonce)[0];
  rc.j0[1] = (uint32_t)explicit_nonce[0] | ((uint32_t)explicit_nonce[1] << 8) |
             ((uint32_t)explicit_nonce[2] << 16) | ((uint32_t)explicit_nonce[3] << 24);
  rc.j0[2] = (uint32_t)explicit_nonce[4] | ((uint32_t)explicit_nonce[5] << 8) |
             ((uint32_t)explicit_nonce[6] << 16) | ((uint32_t)explicit_nonce[7] << 24);
  rc.j0[3] = 0x01000000u;
  // AAD = seq(8) || type || version(2) || length(2), one zero-padded block
  uint32_t v = as_const(&S->version)[0];
  rc.aad_be[0] = (uint32_t)(d.seq >> 32);
  rc.aad_be[1] = (uint32_t)d.seq;
  rc.aad_be[2] = (type << 24) | ((v & 0xFFFF) << 8) | ((rc.n >> 8) & 0xFF);
  rc.aad_be[3] = (rc.n & 0xFF) << 24;
  rc.aad_len = 13;
  return true;
}

// Raw EVP_AEAD job (arbitrary nonce and AAD; e_aes.c:1424-1510).  The host
// already applied the argument checks of evp_aead.c / e_aes.c.
template <bool SEAL>
__device__ __forceinline__ void parse_raw(const RawJob& j, const DevSession* __restrict__ S,
                                          RecCtx& rc) {
  const uint8_t* ip = (const uint8_t*)j.in;
  uint8_t* op = (uint8_t*)j.out;
  const uint8_t* nonce = (const uint8_t*)j.nonce;
  uint32_t tag_len = as_const(&S->tag_len)[0];
  if (SEAL) {
    rc.n = j.in_len;
    rc.src = ip;
    rc.dst = op;
    rc.tag_out = op + j.in_len;
    rc.tag_in = nullptr;
    rc.ok_status = (int32_t)(j.in_len + tag_len);
  } else {
    rc.n = j.in_len - tag_len;
    rc.src = ip;
    rc.dst = op;
    rc.tag_in = ip + rc.n;
    const uint32_t ln = threadIdx.x & 63;
    rc.tag_byte = ln < tag_len ? rc.tag_in[ln] : 0u;
    rc.tag_out = nullptr;
    rc.ok_status = (int32_t)rc.n;
  }
  rc.zero_len = j.max_out;
  if (j.nonce_len == 12) {
    rc.j0[0] = load_u32_bytes(nonce);
    rc.j0[1] = load_u32_bytes(nonce + 4);
    rc.j0[2] = load_u32_bytes(nonce + 8);
    rc.j0[3] = 0x01000000u;
  } else {  // J0 = GHASH(IV || pad || 0^64 || [len(IV)]_64)  (gcm128.c:770-812)
    uint32_t xb[4] = {0, 0, 0, 0};
    ghash_serial(xb, nonce, j.nonce_len, true);
    uint64_t bits = (uint64_t)j.nonce_len * 8;
    xb[2] ^= (uint32_t)(bits >> 32);
    xb[3] ^= (uint32_t)bits;
    uint32_t z[4];
    mul_shoup(xb, 1, z);
    rc.j0[0] = bswap32(z[0]); rc.j0[1] = bswap32(z[1]);
    rc.j0[2] = bswap32(z[2]); rc.j0[3] = bswap32(z[3]);
  }
  rc.aad_be[0] = rc.aad_be[1] = rc.aad_be[2] = rc.aad_be[3] = 0;
  rc.aad_len = j.aad_len;
  if (j.aad_len) ghash_serial(rc.aad_be, (const uint8_t*)j.aad, j.aad_len, false);
}

// ---------------------------------------------------------------------------
// Workgroup prologue / session table staging
template <int NT, bool R4 = true>
__device__ void fill_aes_lds() {
  for (uint32_t t = threadIdx.x; t < 1024; t += NT) {  // 1024 x 64 B = 64 KiB
    const uint32_t row = t >> 2, part = t & 3;
    uint32_t v = g_te0.v[row];
    if (part >= 2) v = rotl32(v, 8);  // Te1 = rotl8(Te0)
    uint4 w = make_uint4(v, v, v, v);
    uint4* dst = reinterpret_cast<uint4*>(s_lds + AES_OFF + row * 256 + part * 64);
    dst[0] = w; dst[1] = w; dst[2] = w; dst[3] = w;
  }
  const uint32_t t = threadIdx.x;
  if (R4 && t < 16) {  // rem_4bit >> 32 (gcm128.c:327-331), derived by four x-shifts
    uint64_t hi = 0, lo = t;
    for (int k = 0; k < 4; k++) {
      uint64_t c = lo & 1;
      lo = (lo >> 1) | (hi << 63);
      hi = (hi >> 1) ^ (c ? 0xE100000000000000ull : 0);
    }
    *reinterpret_cast<uint32_t*>(s_lds + R4_OFF + t * 4) = (uint32_t)(hi >> 32);
  }
}

// Expand the session's 128 basis vectors K*x^p into T[j][b] and copy the
// Shoup tables of H^1..H^65.
template <int NT>
__device__ void load_session_tables(const DevGcmTables* __restrict__ tab) {
  const uint32_t bl = threadIdx.x & 63;
  for (uint32_t jj = threadIdx.x >> 6; jj < 16; jj += NT / kWave) {
    const uint32_t j = __builtin_amdgcn_readfirstlane(jj);  // byte position
    uint32_t lo[4] = {0, 0, 0, 0};
#ifdef TG_VECTOR_SESSION_LOADS
    // the persistent server: the wave's 8 basis entries in one lane-parallel
    // load (lane k < 8: x^(8j + 7 - k)), then lane reads — one memory round
    // trip instead of eight serialised uniform loads (round-4 trace: a key
    // change cost 4.3 µs)
    uint4 own = make_uint4(0, 0, 0, 0);
    if (bl < 8) own = *reinterpret_cast<const uint4*>(tab->basis[8 * j + 7 - bl]);
    struct LaneWord {
      uint4 v;
      __device__ __forceinline__ uint32_t operator()(int k, int c) const {
        const uint32_t w = c == 0 ? v.x : c == 1 ? v.y : c == 2 ? v.z : v.w;
        return (uint32_t)__builtin_amdgcn_readlane((int)w, k);
      }
    } bw{own};
#pragma unroll
    for (int k = 0; k < 6; k++) {   // bit k of the byte <-> x^(8j + 7 - k)
      uint32_t msk = 0u - ((bl >> k) & 1u);
      lo[0] ^= bw(k, 0) & msk; lo[1] ^= bw(k, 1) & msk; lo[2] ^= bw(k, 2) & msk; lo[3] ^= bw(k, 3) & msk;
    }
    const uint32_t b6[4] = {bw(6, 0), bw(6, 1), bw(6, 2), bw(6, 3)};  // x^(8j + 1)
    const uint32_t b7[4] = {bw(7, 0), bw(7, 1), bw(7, 2), bw(7, 3)};  // x^(8j)
#else
#pragma unroll
    for (int k = 0; k < 6; k++) {   // bit k of the byte <-> x^(8j + 7 - k)
      uint32_t msk = 0u - ((bl >> k) & 1u);
      cu32* bv = as_const(tab->basis[8 * j + 7 - k]);
      lo[0] ^= bv[0] & msk; lo[1] ^= bv[1] & msk; lo[2] ^= bv[2] & msk; lo[3] ^= bv[3] & msk;
    }
    cu32* b6 = as_const(tab->basis[8 * j + 1]);
    cu32* b7 = as_const(tab->basis[8 * j + 0]);
#endif
#pragma unroll
    for (int q = 0; q < 4; q++) {
      uint32_t m6 = (q & 1) ? 0xFFFFFFFFu : 0u, m7 = (q & 2) ? 0xFFFFFFFFu : 0u;
      uint4 v = make_uint4(lo[0] ^ (b6[0] & m6) ^ (b7[0] & m7), lo[1] ^ (b6[1] & m6) ^ (b7[1] & m7),
                           lo[2] ^ (b6[2] & m6) ^ (b7[2] & m7), lo[3] ^ (b6[3] & m6) ^ (b7[3] & m7));
      uint32_t b = bl + 64u * q;
      *reinterpret_cast<uint4*>(s_lds + KT_OFF + b * 256 + j * 16) = v;
    }
  }
  const uint4* sh = reinterpret_cast<const uint4*>(&tab->shoup[0][0][0]);
  for (uint32_t k = threadIdx.x; k < kPowMax * 16; k += NT)  // k = 16 (e - 1) + v
    *reinterpret_cast<uint4*>(s_lds + sh_base(1 + (k >> 4)) + (k & 15u) * 256u) = sh[k];
}

// Bitsliced round-key masks from the round-key words (SGPRs): s_bfe_i32
// sign-extends the key bit into 0 / ~0.
struct SgprMasks {
  cu32* rk;
  __device__ __forceinline__ uint32_t mask(int r, int i) const {
    return (uint32_t)__builtin_amdgcn_sbfe((int32_t)rk[4 * r + (i >> 5)], (uint32_t)(i & 31), 1u);
  }
};

__device__ __forceinline__ bool is_gcm(uint32_t kind) {
  return kind == TLSGPU_AES_128_GCM || kind == TLSGPU_AES_256_GCM;
}

}  // namespace tg
