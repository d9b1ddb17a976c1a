// chacha_common.h — ChaCha20 block function and Poly1305-donna primitives
// shared by the batch kernels (chacha_kernels.hip) and the per-job wave path
// (chacha_wave.h: launched raw EVP jobs and the doorbell server).
//
// ChaCha20: chacha/chacha-merged.c:113-270 (64-bit block counter in words
// 12-13).  Poly1305: poly1305-donna.c:54-321, 26-bit limbs.
#pragma once
#include "aes_common.h"
#include "tlsgpu_internal.h"

namespace tg {

__device__ __forceinline__ uint32_t ld_le32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

// Zero n bytes at d from one lane (a record whose tag failed,
// e_chacha20poly1305.c:276-283 + evp_aead.c:137-143): 16-B stores for the
// aligned bulk instead of one store per byte.
__device__ __forceinline__ void zero_fill_lane(uint8_t* d, uint64_t n) {
  uint64_t o = 0;
  for (; o < n && (((uintptr_t)(d + o)) & 15); o++) d[o] = 0;
  for (; o + 16 <= n; o += 16) *reinterpret_cast<uint4*>(d + o) = make_uint4(0, 0, 0, 0);
  for (; o < n; o++) d[o] = 0;
}

#define CC_QR(a, b, c, d)            \
  a += b; d = rotl32(d ^ a, 16);     \
  c += d; b = rotl32(b ^ c, 12);     \
  a += b; d = rotl32(d ^ a, 8);      \
  c += d; b = rotl32(b ^ c, 7);

__device__ __forceinline__ void chacha_block(const uint32_t in[16], uint32_t x[16]) {
#pragma unroll
  for (int i = 0; i < 16; i++) x[i] = in[i];
#pragma unroll
  for (int i = 0; i < 10; i++) {
    CC_QR(x[0], x[4], x[8], x[12]);
    CC_QR(x[1], x[5], x[9], x[13]);
    CC_QR(x[2], x[6], x[10], x[14]);
    CC_QR(x[3], x[7], x[11], x[15]);
    CC_QR(x[0], x[5], x[10], x[15]);
    CC_QR(x[1], x[6], x[11], x[12]);
    CC_QR(x[2], x[7], x[8], x[13]);
    CC_QR(x[3], x[4], x[9], x[14]);
  }
#pragma unroll
  for (int i = 0; i < 16; i++) x[i] += in[i];
}

struct Poly {
  uint32_t r0, r1, r2, r3, r4, s1, s2, s3, s4;
  uint32_t h0, h1, h2, h3, h4;
  uint32_t pad0, pad1, pad2, pad3;
};

__device__ __forceinline__ void poly_init(Poly& p, const uint32_t k[8]) {
  // clamp r (poly1305-donna.c:59-64) on the key words
  uint32_t t0 = k[0], t1 = k[1], t2 = k[2], t3 = k[3];
  p.r0 = t0 & 0x3ffffff;
  p.r1 = ((t0 >> 26) | (t1 << 6)) & 0x3ffff03;
  p.r2 = ((t1 >> 20) | (t2 << 12)) & 0x3ffc0ff;
  p.r3 = ((t2 >> 14) | (t3 << 18)) & 0x3f03fff;
  p.r4 = (t3 >> 8) & 0x00fffff;
  p.s1 = p.r1 * 5; p.s2 = p.r2 * 5; p.s3 = p.r3 * 5; p.s4 = p.r4 * 5;
  p.h0 = p.h1 = p.h2 = p.h3 = p.h4 = 0;
  p.pad0 = k[4]; p.pad1 = k[5]; p.pad2 = k[6]; p.pad3 = k[7];
}

// One 16-byte block m (LE words) with the 2^128 bit given by hibit.
__device__ __forceinline__ void poly_block(Poly& p, uint32_t m0, uint32_t m1, uint32_t m2,
                                           uint32_t m3, uint32_t hibit) {
  uint32_t h0 = p.h0 + (m0 & 0x3ffffff);
  uint32_t h1 = p.h1 + (((m0 >> 26) | (m1 << 6)) & 0x3ffffff);
  uint32_t h2 = p.h2 + (((m1 >> 20) | (m2 << 12)) & 0x3ffffff);
  uint32_t h3 = p.h3 + (((m2 >> 14) | (m3 << 18)) & 0x3ffffff);
  uint32_t h4 = p.h4 + ((m3 >> 8) | hibit);
  uint64_t d0 = (uint64_t)h0 * p.r0 + (uint64_t)h1 * p.s4 + (uint64_t)h2 * p.s3 +
                (uint64_t)h3 * p.s2 + (uint64_t)h4 * p.s1;
  uint64_t d1 = (uint64_t)h0 * p.r1 + (uint64_t)h1 * p.r0 + (uint64_t)h2 * p.s4 +
                (uint64_t)h3 * p.s3 + (uint64_t)h4 * p.s2;
  uint64_t d2 = (uint64_t)h0 * p.r2 + (uint64_t)h1 * p.r1 + (uint64_t)h2 * p.r0 +
                (uint64_t)h3 * p.s4 + (uint64_t)h4 * p.s3;
  uint64_t d3 = (uint64_t)h0 * p.r3 + (uint64_t)h1 * p.r2 + (uint64_t)h2 * p.r1 +
                (uint64_t)h3 * p.r0 + (uint64_t)h4 * p.s4;
  uint64_t d4 = (uint64_t)h0 * p.r4 + (uint64_t)h1 * p.r3 + (uint64_t)h2 * p.r2 +
                (uint64_t)h3 * p.r1 + (uint64_t)h4 * p.r0;
  uint32_t c = (uint32_t)(d0 >> 26); h0 = (uint32_t)d0 & 0x3ffffff;
  d1 += c; c = (uint32_t)(d1 >> 26); h1 = (uint32_t)d1 & 0x3ffffff;
  d2 += c; c = (uint32_t)(d2 >> 26); h2 = (uint32_t)d2 & 0x3ffffff;
  d3 += c; c = (uint32_t)(d3 >> 26); h3 = (uint32_t)d3 & 0x3ffffff;
  d4 += c; c = (uint32_t)(d4 >> 26); h4 = (uint32_t)d4 & 0x3ffffff;
  h0 += c * 5; c = h0 >> 26; h0 &= 0x3ffffff;
  h1 += c;
  p.h0 = h0; p.h1 = h1; p.h2 = h2; p.h3 = h3; p.h4 = h4;
}

// poly1305-donna.c:231-321: full carry, conditional subtract, + pad.
__device__ __forceinline__ void poly_finish(const Poly& p, uint32_t mac[4]) {
  uint32_t h0 = p.h0, h1 = p.h1, h2 = p.h2, h3 = p.h3, h4 = p.h4, c;
  c = h1 >> 26; h1 &= 0x3ffffff;
  h2 += c; c = h2 >> 26; h2 &= 0x3ffffff;
  h3 += c; c = h3 >> 26; h3 &= 0x3ffffff;
  h4 += c; c = h4 >> 26; h4 &= 0x3ffffff;
  h0 += c * 5; c = h0 >> 26; h0 &= 0x3ffffff;
  h1 += c;
  uint32_t g0 = h0 + 5; c = g0 >> 26; g0 &= 0x3ffffff;
  uint32_t g1 = h1 + c; c = g1 >> 26; g1 &= 0x3ffffff;
  uint32_t g2 = h2 + c; c = g2 >> 26; g2 &= 0x3ffffff;
  uint32_t g3 = h3 + c; c = g3 >> 26; g3 &= 0x3ffffff;
  uint32_t g4 = h4 + c - (1u << 26);
  uint32_t mask = (g4 >> 31) - 1;
  h0 = (h0 & ~mask) | (g0 & mask);
  h1 = (h1 & ~mask) | (g1 & mask);
  h2 = (h2 & ~mask) | (g2 & mask);
  h3 = (h3 & ~mask) | (g3 & mask);
  h4 = (h4 & ~mask) | (g4 & mask);
  uint32_t w0 = h0 | (h1 << 26), w1 = (h1 >> 6) | (h2 << 20), w2 = (h2 >> 12) | (h3 << 14),
           w3 = (h3 >> 18) | (h4 << 8);
  uint64_t f = (uint64_t)w0 + p.pad0; mac[0] = (uint32_t)f;
  f = (uint64_t)w1 + p.pad1 + (f >> 32); mac[1] = (uint32_t)f;
  f = (uint64_t)w2 + p.pad2 + (f >> 32); mac[2] = (uint32_t)f;
  f = (uint64_t)w3 + p.pad3 + (f >> 32); mac[3] = (uint32_t)f;
}

}  // namespace tg
