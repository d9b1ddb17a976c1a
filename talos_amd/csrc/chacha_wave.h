// chacha_wave.h — one ChaCha20-Poly1305 EVP job (RFC 7539 layout) on one
// wave, for latency-bound per-call jobs: the launched raw path
// (chacha_raw_wave_kernel) and the doorbell server (evp_server.hip).
//
// Replaces aead_chacha20_poly1305_seal/open (e_chacha20poly1305.c:124-286)
// for the 12-byte-nonce AEAD.  The per-lane kernels run a job's keystream
// blocks and its Poly1305 Horner chain serially on one lane; here the job is
// spread over the 64 lanes of a wave:
//
//   * keystream: lane l computes block counter 64t + l in pass t (counter 0 is
//     the one-time Poly1305 key, chacha20poly1305.c:178-180), XORs its 64
//     bytes and stages the ciphertext of the pass in LDS (4 KiB);
//   * Poly1305 over the N = ceil(|AD|/16) + ceil(|CT|/16) + 1 blocks
//     c_0..c_{N-1} of AD || pad16 || CT || pad16 || le64 || le64 (:182-190):
//     tag = (sum_b c_b r^(N-b) mod 2^130-5) + s.  Lane l takes the blocks
//     b = l (mod 64) in order, Horner with r^64, and multiplies its sum by
//     r^(N - b_last); the 64 lane sums are added across the wave (DPP row
//     shifts and broadcasts, p5_wave_sum).  The powers
//     r^1..r^64 are built by doubling (6 multiplies per lane).
//
// The arithmetic is poly1305-donna's 26-bit limbs (chacha_common.h); the
// result is the same field element as the serial chain's, so the tag is
// identical (tests/test_evp*.py against the oracle).  Session words are read
// by vector loads (the server's coherence rule, evp_server.hip).
#pragma once
#include "chacha_common.h"

namespace tg {

constexpr uint32_t kM26 = 0x3ffffff;

// An element of GF(2^130-5) in five 26-bit limbs (limbs may exceed 2^26
// slightly between carries, as in poly1305-donna).
struct P5 {
  uint32_t v0, v1, v2, v3, v4;
};

__device__ __forceinline__ P5 p5_block(uint32_t m0, uint32_t m1, uint32_t m2, uint32_t m3,
                                       uint32_t hibit) {
  return {m0 & kM26, ((m0 >> 26) | (m1 << 6)) & kM26, ((m1 >> 20) | (m2 << 12)) & kM26,
          ((m2 >> 14) | (m3 << 18)) & kM26, (m3 >> 8) | hibit};
}

__device__ __forceinline__ P5 p5_add(const P5& a, const P5& b) {
  return {a.v0 + b.v0, a.v1 + b.v1, a.v2 + b.v2, a.v3 + b.v3, a.v4 + b.v4};
}

// One serial carry pass (limbs < 2^31 in, donna's invariant out).
__device__ __forceinline__ P5 p5_carry(P5 a) {
  uint32_t c = a.v0 >> 26; a.v0 &= kM26;
  a.v1 += c; c = a.v1 >> 26; a.v1 &= kM26;
  a.v2 += c; c = a.v2 >> 26; a.v2 &= kM26;
  a.v3 += c; c = a.v3 >> 26; a.v3 &= kM26;
  a.v4 += c; c = a.v4 >> 26; a.v4 &= kM26;
  a.v0 += c * 5; c = a.v0 >> 26; a.v0 &= kM26;
  a.v1 += c;
  return a;
}

// a * b mod 2^130-5 (poly1305-donna.c:135-172 with a general second operand).
// Bounds: a's limbs < 2^27.1 (an accumulator plus a block), b's < 2^26.1 (a
// product of this function or the clamped key): every column sum stays below
// 2^57.5, the top column (no *5 terms) below 2^55.4, so each carry fits 32 bits.
__device__ __forceinline__ P5 p5_mul(const P5& a, const P5& b) {
  const uint32_t s1 = b.v1 * 5, s2 = b.v2 * 5, s3 = b.v3 * 5, s4 = b.v4 * 5;
  uint64_t d0 = (uint64_t)a.v0 * b.v0 + (uint64_t)a.v1 * s4 + (uint64_t)a.v2 * s3 +
                (uint64_t)a.v3 * s2 + (uint64_t)a.v4 * s1;
  uint64_t d1 = (uint64_t)a.v0 * b.v1 + (uint64_t)a.v1 * b.v0 + (uint64_t)a.v2 * s4 +
                (uint64_t)a.v3 * s3 + (uint64_t)a.v4 * s2;
  uint64_t d2 = (uint64_t)a.v0 * b.v2 + (uint64_t)a.v1 * b.v1 + (uint64_t)a.v2 * b.v0 +
                (uint64_t)a.v3 * s4 + (uint64_t)a.v4 * s3;
  uint64_t d3 = (uint64_t)a.v0 * b.v3 + (uint64_t)a.v1 * b.v2 + (uint64_t)a.v2 * b.v1 +
                (uint64_t)a.v3 * b.v0 + (uint64_t)a.v4 * s4;
  uint64_t d4 = (uint64_t)a.v0 * b.v4 + (uint64_t)a.v1 * b.v3 + (uint64_t)a.v2 * b.v2 +
                (uint64_t)a.v3 * b.v1 + (uint64_t)a.v4 * b.v0;
  P5 h;
  uint32_t c = (uint32_t)(d0 >> 26); h.v0 = (uint32_t)d0 & kM26;
  d1 += c; c = (uint32_t)(d1 >> 26); h.v1 = (uint32_t)d1 & kM26;
  d2 += c; c = (uint32_t)(d2 >> 26); h.v2 = (uint32_t)d2 & kM26;
  d3 += c; c = (uint32_t)(d3 >> 26); h.v3 = (uint32_t)d3 & kM26;
  d4 += c; c = (uint32_t)(d4 >> 26); h.v4 = (uint32_t)d4 & kM26;
  h.v0 += c * 5; c = h.v0 >> 26; h.v0 &= kM26;
  h.v1 += c;
  return h;
}

__device__ __forceinline__ P5 p5_shfl(const P5& a, int src) {
  return {(uint32_t)__shfl((int)a.v0, src), (uint32_t)__shfl((int)a.v1, src),
          (uint32_t)__shfl((int)a.v2, src), (uint32_t)__shfl((int)a.v3, src),
          (uint32_t)__shfl((int)a.v4, src)};
}

__device__ __forceinline__ P5 p5_readlane(const P5& a, int src) {
  return {(uint32_t)__builtin_amdgcn_readlane((int)a.v0, src),
          (uint32_t)__builtin_amdgcn_readlane((int)a.v1, src),
          (uint32_t)__builtin_amdgcn_readlane((int)a.v2, src),
          (uint32_t)__builtin_amdgcn_readlane((int)a.v3, src),
          (uint32_t)__builtin_amdgcn_readlane((int)a.v4, src)};
}

// One DPP step of a wave reduction on all five limbs (update_dpp with old = 0:
// lanes without a source, or outside row_mask / bank_mask, add nothing).
template <int CTRL, int ROWS, int BANKS, bool BOUND>
__device__ __forceinline__ P5 p5_dpp(const P5& a) {
  return {(uint32_t)__builtin_amdgcn_update_dpp(0, (int)a.v0, CTRL, ROWS, BANKS, BOUND),
          (uint32_t)__builtin_amdgcn_update_dpp(0, (int)a.v1, CTRL, ROWS, BANKS, BOUND),
          (uint32_t)__builtin_amdgcn_update_dpp(0, (int)a.v2, CTRL, ROWS, BANKS, BOUND),
          (uint32_t)__builtin_amdgcn_update_dpp(0, (int)a.v3, CTRL, ROWS, BANKS, BOUND),
          (uint32_t)__builtin_amdgcn_update_dpp(0, (int)a.v4, CTRL, ROWS, BANKS, BOUND)};
}

// Sum of a over the 64 lanes (all active) mod 2^130-5, uniform: the row
// shift / row broadcast pattern of wave_xor_total (aes_common.h) with a
// carry pass after each level (4 terms < 2^28.1, then 2 terms < 2^27.1 per
// limb going in; p5_carry takes < 2^31).
__device__ __forceinline__ P5 p5_wave_sum(const P5& v) {
  P5 a = p5_carry(p5_add(p5_add(v, p5_dpp<0x111, 0xf, 0xf, true>(v)),
                         p5_add(p5_dpp<0x112, 0xf, 0xf, true>(v), p5_dpp<0x113, 0xf, 0xf, true>(v))));
  a = p5_carry(p5_add(a, p5_dpp<0x114, 0xf, 0xe, false>(a)));
  a = p5_carry(p5_add(a, p5_dpp<0x118, 0xf, 0xc, false>(a)));
  a = p5_carry(p5_add(a, p5_dpp<0x142, 0xa, 0xf, false>(a)));
  a = p5_carry(p5_add(a, p5_dpp<0x143, 0xc, 0xf, false>(a)));
  return p5_readlane(a, 63);
}

// Up to 16 bytes at p (nb < 16: zero padded) as little-endian words.
__device__ __forceinline__ void cw_load16(const uint8_t* p, uint32_t nb, bool aligned,
                                          uint32_t w[4]) {
  if (nb >= 16 && aligned) {
    const uint4 t = *reinterpret_cast<const uint4*>(p);
    w[0] = t.x; w[1] = t.y; w[2] = t.z; w[3] = t.w;
    return;
  }
  w[0] = w[1] = w[2] = w[3] = 0;
#pragma unroll
  for (int k = 0; k < 16; k++)
    if ((uint32_t)k < nb) w[k >> 2] |= (uint32_t)p[k] << (8 * (k & 3));
}

__device__ __forceinline__ void cw_store16(uint8_t* p, uint32_t nb, bool aligned,
                                           const uint32_t w[4]) {
  if (nb >= 16 && aligned) {
    *reinterpret_cast<uint4*>(p) = make_uint4(w[0], w[1], w[2], w[3]);
    return;
  }
#pragma unroll
  for (int k = 0; k < 16; k++)
    if ((uint32_t)k < nb) p[k] = (uint8_t)(w[k >> 2] >> (8 * (k & 3)));
}

__device__ __forceinline__ uint32_t cw_mac_byte(const uint32_t mac[4], uint32_t k) {
  const uint32_t w = k < 4 ? mac[0] : k < 8 ? mac[1] : k < 12 ? mac[2] : mac[3];
  return (w >> (8 * (k & 3))) & 0xFF;
}

// Run raw job j of the RFC 7539 AEAD on the calling wave (all 64 lanes).
// S: the job's session (kind already checked); stage: 4 KiB of LDS, 16-B
// aligned, owned by this wave.  Writes the output, the tag (seal) and
// *status (lane 0); on a tag mismatch zero-fills j.max_out bytes
// (evp_aead.c:137-143).  Host-side checks (nonce_len == 12, open in_len >=
// tag_len, output room) are the caller's, as for the per-lane kernel.
template <bool SEAL>
__device__ void cc_wave_job(const RawJob& j, const DevSession* S, int32_t* status,
                            uint8_t* stage) {
  const uint32_t lane = threadIdx.x & 63;
  // session words 0..7 (kind, rounds, tag_len, ...) and 72..79 (chacha_key)
  const uint32_t* sw = reinterpret_cast<const uint32_t*>(S);
  static_assert(offsetof(DevSession, chacha_key) == 72 * 4, "DevSession layout");
  const uint32_t sv = sw[lane < 8 ? lane : 64 + (lane & 15)];
  const uint32_t tag_len = __builtin_amdgcn_readlane(sv, 2);
  uint32_t in[16];
  in[0] = 0x61707865u; in[1] = 0x3320646eu; in[2] = 0x79622d32u; in[3] = 0x6b206574u;
#pragma unroll
  for (int i = 0; i < 8; i++) in[4 + i] = __builtin_amdgcn_readlane(sv, 8 + i);
  // 12-byte nonce: 64-bit counter words 12-13 = 0 || LE32(nonce[0..3]),
  // iv = nonce[4..11] (e_chacha20poly1305.c:140-150)
  const uint8_t* nonce = reinterpret_cast<const uint8_t*>(j.nonce);
  in[13] = ld_le32(nonce);
  in[14] = ld_le32(nonce + 4);
  in[15] = ld_le32(nonce + 8);

  const uint32_t n = SEAL ? j.in_len : j.in_len - tag_len;
  const uint32_t ad_len = j.aad_len;
  const uint8_t* src = reinterpret_cast<const uint8_t*>(j.in);
  uint8_t* dst = reinterpret_cast<uint8_t*>(j.out);
  const uint8_t* aad = reinterpret_cast<const uint8_t*>(j.aad);
  const bool aligned = ((((uintptr_t)src) | ((uintptr_t)dst)) & 15) == 0;
  const uint32_t na = (ad_len + 15) >> 4, nc = (n + 15) >> 4, N = na + nc + 1;
  const uint32_t nkb = (n + 63) >> 6;            // keystream blocks of data
  const uint32_t passes = (nkb + 1 + 63) >> 6;   // counters 0..nkb

  P5 acc = {0, 0, 0, 0, 0}, pw = {0, 0, 0, 0, 0}, r64 = {0, 0, 0, 0, 0};
  uint32_t pad[4] = {0, 0, 0, 0};
  for (uint32_t t = 0; t < passes; t++) {
    const uint32_t ctr = 64 * t + lane;
    uint32_t ks[16];
    in[12] = ctr;
    chacha_block(in, ks);
    if (t == 0) {
      // one-time key from lane 0's block 0: r (clamped) and s
      uint32_t k[8];
#pragma unroll
      for (int i = 0; i < 8; i++) k[i] = __builtin_amdgcn_readlane(ks[i], 0);
      Poly p;
      poly_init(p, k);
      pad[0] = k[4]; pad[1] = k[5]; pad[2] = k[6]; pad[3] = k[7];
      // lane l: r^(l+1), by doubling
      pw = {p.r0, p.r1, p.r2, p.r3, p.r4};
#pragma unroll
      for (int lev = 0; lev < 6; lev++) {
        const int step = 1 << lev;
        const P5 base = p5_readlane(pw, step - 1);          // r^step
        const P5 lo = p5_shfl(pw, (int)lane - step);        // r^(l-step+1)
        const P5 m = p5_mul(lo, base);
        if ((int)lane >= step && (int)lane < 2 * step) pw = m;
      }
      r64 = p5_readlane(pw, 63);
      // AD blocks b = lane, lane + 64, ... (zero padded to 16)
      for (uint32_t b = lane; b < na; b += 64) {
        uint32_t w[4];
        const uint32_t o = 16 * b;
        cw_load16(aad + o, min(16u, ad_len - o), false, w);
        acc = p5_add(p5_mul(acc, r64), p5_block(w[0], w[1], w[2], w[3], 1u << 24));
      }
    }
    // data: keystream block kb = ctr - 1 covers bytes [64 kb, 64 kb + 64);
    // its ciphertext goes to stage[64 lane ..] (data block i at
    // 16 (i - 256 t + 4))
    if (ctr >= 1 && ctr - 1 < nkb) {
      const uint32_t kb = ctr - 1;
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const uint32_t o = 64 * kb + 16 * q;
        if (o < n) {
          const uint32_t nb = min(16u, n - o);
          uint32_t x[4], y[4];
          cw_load16(src + o, nb, aligned, x);
#pragma unroll
          for (int w = 0; w < 4; w++) y[w] = x[w] ^ ks[4 * q + w];
          if (nb < 16) {  // the MAC sees zero padding
#pragma unroll
            for (int w = 0; w < 4; w++) {
              const int32_t b = (int32_t)nb - 4 * w;
              y[w] &= b >= 4 ? 0xFFFFFFFFu : (b <= 0 ? 0u : ((1u << (8 * b)) - 1u));
            }
          }
          cw_store16(dst + o, nb, aligned, y);
          const uint32_t* c = SEAL ? y : x;
          *reinterpret_cast<uint4*>(stage + 64 * lane + 16 * q) = make_uint4(c[0], c[1], c[2], c[3]);
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // this pass's data blocks [lo, hi) in Poly1305 order: block b = na + i
    // belongs to lane b mod 64
    const uint32_t lo = t == 0 ? 0u : 256 * t - 4, hi = min(nc, 256 * t + 252);
    const uint32_t i0 = lo + ((lane - na - lo) & 63);
#pragma unroll
    for (int s = 0; s < 4; s++) {
      const uint32_t i = i0 + 64 * s;
      if (i < hi) {
        const uint4 c = *reinterpret_cast<const uint4*>(stage + 16 * (i - 256 * t + 4));
        acc = p5_add(p5_mul(acc, r64), p5_block(c.x, c.y, c.z, c.w, 1u << 24));
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  // le64(|AD|) || le64(|CT|) is block N-1
  if (lane == ((N - 1) & 63)) acc = p5_add(p5_mul(acc, r64), p5_block(ad_len, 0, n, 0, 1u << 24));
  // weight r^(N - b_last) for the lane's last block
  const uint32_t w = lane < N ? N - (lane + 64 * ((N - 1 - lane) >> 6)) : 1u;
  acc = p5_mul(acc, p5_shfl(pw, (int)w - 1));
  acc = p5_wave_sum(acc);
  Poly p = {};
  p.h0 = acc.v0; p.h1 = acc.v1; p.h2 = acc.v2; p.h3 = acc.v3; p.h4 = acc.v4;
  p.pad0 = pad[0]; p.pad1 = pad[1]; p.pad2 = pad[2]; p.pad3 = pad[3];
  uint32_t mac[4];
  poly_finish(p, mac);
  if (SEAL) {
    if (lane < tag_len) dst[n + lane] = (uint8_t)cw_mac_byte(mac, lane);
    if (lane == 0) *status = (int32_t)(n + tag_len);
    return;
  }
  const uint8_t* tag_in = src + n;
  const bool bad = lane < tag_len && (tag_in[lane] ^ cw_mac_byte(mac, lane)) != 0;
  if (__ballot(bad) == 0) {
    if (lane == 0) *status = (int32_t)n;
    return;
  }
  // the plaintext stores are ordered before the zero-fill
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  const uint64_t z = j.max_out;
  const bool zal = (((uintptr_t)dst) & 15) == 0;
  for (uint64_t o = 16 * (uint64_t)lane; o < z; o += 1024) {
    const uint32_t zero[4] = {0, 0, 0, 0};
    cw_store16(dst + o, z - o < 16 ? (uint32_t)(z - o) : 16u, zal, zero);
  }
  if (lane == 0) *status = TLSGPU_REC_BAD_MAC;
}

// Bytes [off, off + 16) of the segment p[0, len) as little-endian words,
// zero outside it; off may be negative.  A window inside the segment takes
// dword loads (load16_any, global memory); an edge window goes byte by byte
// through the generic pointer (the server's inline AAD lives in LDS).
__device__ __forceinline__ void cw_seg16(const uint8_t* p, int64_t len, int64_t off, bool global,
                                         uint32_t w[4]) {
  w[0] = w[1] = w[2] = w[3] = 0;
  if (off >= len || off + 16 <= 0) return;
  if (global && off >= 0 && off + 16 <= len) {
    load16_any(p + off, w);
    return;
  }
#pragma unroll
  for (int k = 0; k < 16; k++) {
    const int64_t q = off + k;
    if (q >= 0 && q < len) w[k >> 2] |= (uint32_t)p[q] << (8 * (k & 3));
  }
}

// The same window of the 8-byte little-endian encoding of v.
__device__ __forceinline__ void cw_le64_16(uint64_t v, int64_t off, uint32_t w[4]) {
  w[0] = w[1] = w[2] = w[3] = 0;
#pragma unroll
  for (int k = 0; k < 16; k++) {
    const int64_t q = off + k;
    if (q >= 0 && q < 8) w[k >> 2] |= (uint32_t)((v >> (8 * q)) & 0xFF) << (8 * (k & 3));
  }
}

// Poly1305 tag of the draft AEAD's byte stream AD || le64(|AD|) || CT ||
// le64(|CT|) (e_chacha20poly1305.c:160-170, poly1305_update over
// unpadded pieces), with the lane split of cc_wave_job: lane l takes stream
// blocks b = l (mod 64), Horner with r^64, weight r^(N - b_last), wave sum.
// The last block, if partial, carries the 0x01 byte after its data and no
// 2^128 bit (poly1305-donna's final block).  pw: r^(l+1) on lane l.
__device__ __forceinline__ void cw_old_mac(const uint8_t* aad, uint32_t ad_len, bool aad_global,
                                           const uint8_t* ct, uint32_t n, bool ct_global,
                                           const P5& pw, const uint32_t pad[4], uint32_t mac[4]) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t M = (uint64_t)ad_len + 8 + n + 8;
  const uint32_t N = (uint32_t)((M + 15) >> 4);
  const P5 r64 = p5_readlane(pw, 63);
  P5 acc = {0, 0, 0, 0, 0};
  for (uint32_t b = lane; b < N; b += 64) {
    const int64_t o = 16 * (int64_t)b;
    uint32_t w[4], t[4];
    cw_seg16(aad, ad_len, o, aad_global, w);
    cw_le64_16(ad_len, o - ad_len, t);
    w[0] |= t[0]; w[1] |= t[1]; w[2] |= t[2]; w[3] |= t[3];
    cw_seg16(ct, n, o - ad_len - 8, ct_global, t);
    w[0] |= t[0]; w[1] |= t[1]; w[2] |= t[2]; w[3] |= t[3];
    cw_le64_16(n, o - ad_len - 8 - n, t);
    w[0] |= t[0]; w[1] |= t[1]; w[2] |= t[2]; w[3] |= t[3];
    uint32_t hibit = 1u << 24;
    const uint64_t left = M - (uint64_t)o;
    if (left < 16) {  // poly1305 final block: 0x01 after the data, no 2^128
      w[left >> 2] |= 1u << (8 * (left & 3));
      hibit = 0;
    }
    acc = p5_add(p5_mul(acc, r64), p5_block(w[0], w[1], w[2], w[3], hibit));
  }
  const uint32_t wgt = lane < N ? N - (lane + 64 * ((N - 1 - lane) >> 6)) : 1u;
  acc = p5_mul(acc, p5_shfl(pw, (int)wgt - 1));
  acc = p5_wave_sum(acc);
  Poly p = {};
  p.h0 = acc.v0; p.h1 = acc.v1; p.h2 = acc.v2; p.h3 = acc.v3; p.h4 = acc.v4;
  p.pad0 = pad[0]; p.pad1 = pad[1]; p.pad2 = pad[2]; p.pad3 = pad[3];
  poly_finish(p, mac);
}

// Run raw job j of the draft ("old") ChaCha20-Poly1305 AEAD on the calling
// wave (round 5: the doorbell server's op 21 and chacha_raw_wave_kernel).
// e_chacha20poly1305.c:124-286 with the 8-byte nonce: ChaCha20 with a 64-bit
// block counter in words 12-13 and the nonce in words 14-15 (counter 0: the
// one-time Poly1305 key, data from counter 1); the MAC over the byte stream
// of cw_old_mac.  Open checks the tag before it writes any plaintext (the
// reference's order), seal MACs the ciphertext it wrote.  Same contract as
// cc_wave_job (host-side checks are the caller's).
template <bool SEAL>
__device__ void cc_wave_job_old(const RawJob& j, const DevSession* S, int32_t* status,
                                bool aad_global, uint8_t* stage) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t* sw = reinterpret_cast<const uint32_t*>(S);
  static_assert(offsetof(DevSession, chacha_key) == 72 * 4, "DevSession layout");
  const uint32_t sv = sw[lane < 8 ? lane : 64 + (lane & 15)];
  const uint32_t tag_len = __builtin_amdgcn_readlane(sv, 2);
  uint32_t in[16];
  in[0] = 0x61707865u; in[1] = 0x3320646eu; in[2] = 0x79622d32u; in[3] = 0x6b206574u;
#pragma unroll
  for (int i = 0; i < 8; i++) in[4 + i] = __builtin_amdgcn_readlane(sv, 8 + i);
  const uint8_t* nonce = reinterpret_cast<const uint8_t*>(j.nonce);
  in[13] = 0;
  in[14] = ld_le32(nonce);
  in[15] = ld_le32(nonce + 4);
  const uint32_t n = SEAL ? j.in_len : j.in_len - tag_len;
  const uint8_t* src = reinterpret_cast<const uint8_t*>(j.in);
  uint8_t* dst = reinterpret_cast<uint8_t*>(j.out);
  const uint8_t* aad = reinterpret_cast<const uint8_t*>(j.aad);
  const bool aligned = ((((uintptr_t)src) | ((uintptr_t)dst)) & 15) == 0;

  // the one-time key (counter 0, lane 0's block) and r^1..r^64 by doubling
  uint32_t ks[16];
  in[12] = 0;
  chacha_block(in, ks);
  uint32_t k[8];
#pragma unroll
  for (int i = 0; i < 8; i++) k[i] = __builtin_amdgcn_readfirstlane(ks[i]);
  Poly p0;
  poly_init(p0, k);
  const uint32_t pad[4] = {k[4], k[5], k[6], k[7]};
  P5 pw = {p0.r0, p0.r1, p0.r2, p0.r3, p0.r4};
#pragma unroll
  for (int lev = 0; lev < 6; lev++) {
    const int step = 1 << lev;
    const P5 base = p5_readlane(pw, step - 1);
    const P5 lo = p5_shfl(pw, (int)lane - step);
    const P5 m = p5_mul(lo, base);
    if ((int)lane >= step && (int)lane < 2 * step) pw = m;
  }
  // a job whose data fits the 4 KiB LDS stage (one pass: every TLS record of
  // up to 4,032 B) MACs from there: open copies its ciphertext in once (the
  // MAC and the decryption read it from LDS), seal stages what it writes —
  // the input and output live in pinned host memory, where every re-read is
  // a PCIe round trip
  const bool staged = n <= 4096u - 64u;
  uint32_t mac[4];
  if (!SEAL) {
    if (staged) {
      for (uint32_t o = 16 * lane; o < n; o += 1024) {
        uint32_t x[4];
        cw_load16(src + o, min(16u, n - o), aligned, x);
        *reinterpret_cast<uint4*>(stage + o) = make_uint4(x[0], x[1], x[2], x[3]);
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    cw_old_mac(aad, j.aad_len, aad_global, staged ? stage : src, n, !staged, pw, pad, mac);
  }
  bool bad = false;
  if (!SEAL) {
    const uint8_t* tag_in = src + n;
    bad = __ballot(lane < tag_len && (tag_in[lane] ^ cw_mac_byte(mac, lane)) != 0) != 0;
  }
  if (!bad) {
    // data: lane l of pass t runs counter 64 t + l + 1 over bytes [64 kb, 64 kb + 64)
    const uint32_t nkb = (n + 63) >> 6;
    for (uint32_t kb = lane; kb - lane < nkb; kb += 64) {  // wave-uniform trip count
      if (kb >= nkb) continue;
      in[12] = kb + 1;  // < 2^26 blocks per job: word 13 stays 0
      chacha_block(in, ks);
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const uint32_t o = 64 * kb + 16 * q;
        if (o < n) {
          const uint32_t nb = min(16u, n - o);
          uint32_t x[4], y[4];
          if (!SEAL && staged) {
            const uint4 t = *reinterpret_cast<const uint4*>(stage + o);
            x[0] = t.x; x[1] = t.y; x[2] = t.z; x[3] = t.w;
          } else {
            cw_load16(src + o, nb, aligned, x);
          }
#pragma unroll
          for (int w = 0; w < 4; w++) y[w] = x[w] ^ ks[4 * q + w];
          cw_store16(dst + o, nb, aligned, y);
          if (SEAL && staged) {  // the MAC's copy (bytes past n are never read)
            *reinterpret_cast<uint4*>(stage + o) = make_uint4(y[0], y[1], y[2], y[3]);
          }
        }
      }
    }
  }
  if (SEAL) {
    // the ciphertext other lanes stored, before the MAC reads it
    if (staged) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    } else {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    cw_old_mac(aad, j.aad_len, aad_global, staged ? stage : dst, n, !staged, pw, pad, mac);
    if (lane < tag_len) dst[n + lane] = (uint8_t)cw_mac_byte(mac, lane);
    if (lane == 0) *status = (int32_t)(n + tag_len);
    return;
  }
  if (!bad) {
    if (lane == 0) *status = (int32_t)n;
    return;
  }
  const uint64_t z = j.max_out;  // evp_aead.c:137-143
  const bool zal = (((uintptr_t)dst) & 15) == 0;
  for (uint64_t o = 16 * (uint64_t)lane; o < z; o += 1024) {
    const uint32_t zero[4] = {0, 0, 0, 0};
    cw_store16(dst + o, z - o < 16 ? (uint32_t)(z - o) : 16u, zal, zero);
  }
  if (lane == 0) *status = TLSGPU_REC_BAD_MAC;
}

}  // namespace tg
