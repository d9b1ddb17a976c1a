// chacha_kernels.hip — ChaCha20-Poly1305 TLS record open/seal for gfx950.
//
// Replaces, per record, aead_chacha20_poly1305_seal/open
// (crypto/evp/e_chacha20poly1305.c:124-286) driven by tls1_enc
// (ssl/t1_enc.c:832-975): ChaCha20 with a 64-bit block counter
// (chacha/chacha.c:59-77, chacha-merged.c:113-270), the Poly1305 one-time key
// from block 0 (:178-180), Poly1305-donna with 26-bit limbs
// (poly1305-donna.c:54-321) over the RFC 7539 layout
// AD || pad16 || CT || pad16 || le64(|AD|) || le64(|CT|) (:182-190), or the
// draft layout AD || le64(|AD|) || CT || le64(|CT|) for the 8-byte-nonce "old"
// AEAD (:160-170).  Open computes the MAC over the ciphertext while it
// decrypts and zero-fills the plaintext on a tag mismatch, which yields the
// same output as the reference's MAC-then-decrypt order (:276-283).
//
// Mapping: one record per lane.  Poly1305 is a serial Horner chain with a
// per-record key r, so a lane owns the whole chain (no cross-lane combine);
// the VALU does ARX + 32x32->64 multiplies only, no LDS.
#include "chacha_wave.h"

namespace tg {

typedef __attribute__((address_space(4))) const uint32_t cu32c;

// Byte-stream Poly1305 (poly1305-donna.c:176-212 buffering) for the draft
// layout, whose segments are not 16-byte aligned.
struct PolyStream {
  uint32_t buf[4];
  uint32_t fill;
};
__device__ __forceinline__ void ps_byte(Poly& p, PolyStream& s, uint32_t b) {
  uint32_t w = s.fill >> 2, sh = 8 * (s.fill & 3);
  if (w == 0) s.buf[0] |= b << sh;
  else if (w == 1) s.buf[1] |= b << sh;
  else if (w == 2) s.buf[2] |= b << sh;
  else s.buf[3] |= b << sh;
  if (++s.fill == 16) {
    poly_block(p, s.buf[0], s.buf[1], s.buf[2], s.buf[3], 1u << 24);
    s.buf[0] = s.buf[1] = s.buf[2] = s.buf[3] = 0;
    s.fill = 0;
  }
}
__device__ __forceinline__ void ps_u64(Poly& p, PolyStream& s, uint64_t v) {
  for (int k = 0; k < 8; k++) ps_byte(p, s, (uint32_t)(v >> (8 * k)) & 0xFF);
}
__device__ __forceinline__ void ps_final(Poly& p, PolyStream& s) {
  if (s.fill) {  // 0x01 terminator, zero pad, no 2^128 bit (:214-230)
    uint32_t w = s.fill >> 2, bit = 1u << (8 * (s.fill & 3));
    s.buf[0] |= w == 0 ? bit : 0u;
    s.buf[1] |= w == 1 ? bit : 0u;
    s.buf[2] |= w == 2 ? bit : 0u;
    s.buf[3] |= w == 3 ? bit : 0u;
    poly_block(p, s.buf[0], s.buf[1], s.buf[2], s.buf[3], 0);
  }
}

struct CcRec {
  const uint8_t* src;
  uint8_t* dst;
  const uint8_t* tag_in;
  uint8_t* tag_out;
  const uint8_t* aad_ptr;  // raw mode
  uint32_t ad[4];          // TLS mode 13-byte AAD (LE words, zero padded)
  uint32_t ad_len;
  uint32_t n;
  uint32_t st[16];         // ChaCha input block with counter 0
  bool old;
  uint64_t zero_len;
  int32_t ok_status;
  bool valid;
};

template <bool SEAL>
__device__ void cc_record(const CcRec& rc, uint32_t tag_len, int32_t* status_slot) {
  uint32_t st[16], ks[16];
#pragma unroll
  for (int i = 0; i < 16; i++) st[i] = rc.st[i];
  chacha_block(st, ks);  // counter 0 block -> one-time Poly1305 key
  Poly p;
  poly_init(p, ks);
  PolyStream ps = {{0, 0, 0, 0}, 0};
  const uint32_t n = rc.n;

  // AD
  if (!rc.old) {
    for (uint32_t o = 0; o < rc.ad_len; o += 16) {
      uint32_t b[4] = {0, 0, 0, 0};
      if (rc.aad_ptr) {
#pragma unroll
        for (int k = 0; k < 16; k++)
          if (o + k < rc.ad_len) b[k >> 2] |= (uint32_t)rc.aad_ptr[o + k] << (8 * (k & 3));
      } else {
        b[0] = rc.ad[0]; b[1] = rc.ad[1]; b[2] = rc.ad[2]; b[3] = rc.ad[3];
      }
      poly_block(p, b[0], b[1], b[2], b[3], 1u << 24);  // pad16
    }
  } else {
    for (uint32_t o = 0; o < rc.ad_len; o++)
      ps_byte(p, ps, rc.aad_ptr ? rc.aad_ptr[o] : (rc.ad[o >> 2] >> (8 * (o & 3))) & 0xFF);
    ps_u64(p, ps, rc.ad_len);
  }

  const bool aligned = ((((uintptr_t)rc.src) | ((uintptr_t)rc.dst)) & 15) == 0;
  // data: counter 1.. (64-bit counter in words 12-13, chacha-merged.c:230-236)
  uint64_t ctr = ((uint64_t)st[13] << 32) | st[12];
  for (uint32_t off = 0; off < n; off += 64) {
    ctr += 1;
    st[12] = (uint32_t)ctr;
    st[13] = (uint32_t)(ctr >> 32);
    chacha_block(st, ks);
#pragma unroll
    for (int q = 0; q < 4; q++) {
      uint32_t o = off + 16 * q;
      if (o >= n) break;
      uint32_t nb = min(16u, n - o);
      uint32_t in[4] = {0, 0, 0, 0};
      if (nb == 16 && aligned) {
        uint4 t = *reinterpret_cast<const uint4*>(rc.src + o);
        in[0] = t.x; in[1] = t.y; in[2] = t.z; in[3] = t.w;
      } else {
#pragma unroll
        for (int k = 0; k < 16; k++)
          if ((uint32_t)k < nb) in[k >> 2] |= (uint32_t)rc.src[o + k] << (8 * (k & 3));
      }
      uint32_t ob[4] = {in[0] ^ ks[4 * q], in[1] ^ ks[4 * q + 1], in[2] ^ ks[4 * q + 2],
                        in[3] ^ ks[4 * q + 3]};
      if (nb < 16) {  // zero the pad bytes so the MAC sees pad16 zeros
#pragma unroll
        for (int w = 0; w < 4; w++) {
          int32_t b = (int32_t)nb - 4 * w;
          uint32_t keep = b >= 4 ? 0xFFFFFFFFu : (b <= 0 ? 0u : ((1u << (8 * b)) - 1u));
          ob[w] &= keep;
        }
      }
      if (nb == 16 && aligned) {
        *reinterpret_cast<uint4*>(rc.dst + o) = make_uint4(ob[0], ob[1], ob[2], ob[3]);
      } else {
#pragma unroll
        for (int k = 0; k < 16; k++)
          if ((uint32_t)k < nb) rc.dst[o + k] = (uint8_t)(ob[k >> 2] >> (8 * (k & 3)));
      }
      const uint32_t* c = SEAL ? ob : in;
      if (!rc.old) {
        poly_block(p, c[0], c[1], c[2], c[3], 1u << 24);
      } else {
        for (uint32_t k = 0; k < nb; k++) ps_byte(p, ps, (c[k >> 2] >> (8 * (k & 3))) & 0xFF);
      }
    }
  }
  if (!rc.old) {
    poly_block(p, rc.ad_len, 0, n, 0, 1u << 24);  // le64(ad_len) || le64(ct_len)
  } else {
    ps_u64(p, ps, n);
    ps_final(p, ps);
  }
  uint32_t mac[4];
  poly_finish(p, mac);
  if (SEAL) {  // 16-B tags through dword accesses (as cc_tls_wave)
    if (tag_len == 16) {
      store16_any(rc.tag_out, mac);
    } else {
      for (uint32_t k = 0; k < tag_len; k++) rc.tag_out[k] = (uint8_t)(mac[k >> 2] >> (8 * (k & 3)));
    }
    *status_slot = rc.ok_status;
  } else {
    uint32_t diff = 0;
    if (tag_len == 16) {  // every byte compared (timingsafe_memcmp)
      uint32_t t[4];
      load16_any(rc.tag_in, t);
      diff = (t[0] ^ mac[0]) | (t[1] ^ mac[1]) | (t[2] ^ mac[2]) | (t[3] ^ mac[3]);
    } else {
      for (uint32_t k = 0; k < tag_len; k++)
        diff |= rc.tag_in[k] ^ ((mac[k >> 2] >> (8 * (k & 3))) & 0xFF);
    }
    if (diff) {
      zero_fill_lane(rc.dst, rc.zero_len);
      *status_slot = TLSGPU_REC_BAD_MAC;
    } else {
      *status_slot = rc.ok_status;
    }
  }
}

// ---------------------------------------------------------------------------
// LDS-staged data path (TLS batches).  With one record per lane a wave's
// 16-B accesses touch 64 records (64 cache lines per instruction).  Here the
// data moves in 128-B steps through a per-wave LDS tile of 64 rows: lane l
// serves pieces of records 8k + l/8 (k = 0..7), so each load/store instruction
// covers 8 records x 128 contiguous bytes; each lane then en/decrypts and MACs
// its own record's row.  Rows are 128 B with no padding: the 16-B pieces of
// row r are stored rotated by r/2 (cc_slot), so the row-wise ds_read_b128 of
// the 64 lanes (same piece, different rows) is bank-conflict-free while the
// gather/scatter still write and read each 1 KiB slot group contiguously.
// Register budget (round 3): the ChaCha key words sit in LDS (read per block),
// the record's tag/status fields are re-derived at the end, so the kernel fits
// 128 VGPRs = 4 waves per SIMD (round 2: 146 VGPRs, 3 waves per SIMD).
constexpr uint32_t kCcStep = 128;
constexpr int kCcP = kCcStep / 16;           // 16-B pieces of a record per step = loads per lane
constexpr int kCcR = kWave / kCcP;           // records covered by one load instruction
constexpr int kCcThreads = 256;
constexpr uint32_t kCcTile = kWave * kCcStep;  // 8 KiB of rows per wave
constexpr uint32_t kCcKeys = kWave * 32;       // the lanes' ChaCha keys, 2 KiB per wave
// Diagnostic bits (TLSGPU_CC_DIAG, BatchArgs::hy_flags of the staged launch;
// tools/cc_diag.py): drop the gather's global loads, the scatter's global
// stores, or the ChaCha / Poly1305 work, to split the kernel's time.  The
// results are then wrong; never set outside that harness.
constexpr uint32_t kCcDiagNoLoads = 1, kCcDiagNoStores = 2, kCcDiagNoCompute = 4;
// TLSGPU_CC_NARROW=0 (A/B): 64-bit pointer shuffles even when NARROW applies
constexpr uint32_t kCcNoNarrow = 8;  // (host-side only)
// TLSGPU_CC_UKEY=0 (A/B): keys from LDS even for one-session waves
constexpr uint32_t kCcNoUkey = 16;

// tile offset of piece q (0..7) of row r
__device__ __forceinline__ uint32_t cc_slot(uint32_t r, uint32_t q) {
  return r * kCcStep + (((q + (r >> 1)) & 7u) << 4);
}

__device__ __forceinline__ uint64_t shfl64(uint64_t v, uint32_t src) {
  const uint32_t lo = __shfl((uint32_t)v, (int)src), hi = __shfl((uint32_t)(v >> 32), (int)src);
  return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ void lds_wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// ChaCha20 block (chacha-merged.c:113-270) with the key words read from LDS
// at the start and again for the feed-forward (not held across the rounds).
__device__ __forceinline__ void cc_block_lds(uint32_t x[16], const uint8_t* key, uint32_t c12,
                                             uint32_t c13, uint32_t c14, uint32_t c15) {
  const volatile u32x4* kp = reinterpret_cast<const volatile u32x4*>(key);
  {
    const u32x4 ka = kp[0], kb = kp[kWave];
    x[0] = 0x61707865u; x[1] = 0x3320646eu; x[2] = 0x79622d32u; x[3] = 0x6b206574u;
    x[4] = ka.x; x[5] = ka.y; x[6] = ka.z; x[7] = ka.w;
    x[8] = kb.x; x[9] = kb.y; x[10] = kb.z; x[11] = kb.w;
    x[12] = c12; x[13] = c13; x[14] = c14; x[15] = c15;
  }
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
  const u32x4 ka = kp[0], kb = kp[kWave];
  x[0] += 0x61707865u; x[1] += 0x3320646eu; x[2] += 0x79622d32u; x[3] += 0x6b206574u;
  x[4] += ka.x; x[5] += ka.y; x[6] += ka.z; x[7] += ka.w;
  x[8] += kb.x; x[9] += kb.y; x[10] += kb.z; x[11] += kb.w;
  x[12] += c12; x[13] += c13; x[14] += c14; x[15] += c15;
}

// The same block with the key words of a wave-uniform session read through
// the constant address space (s_load: SGPRs, no LDS reads; UKEY below).
__device__ __forceinline__ void cc_block_sk(uint32_t x[16], cu32c* k, uint32_t c12, uint32_t c13,
                                            uint32_t c14, uint32_t c15) {
  x[0] = 0x61707865u; x[1] = 0x3320646eu; x[2] = 0x79622d32u; x[3] = 0x6b206574u;
#pragma unroll
  for (int i = 0; i < 8; i++) x[4 + i] = k[i];
  x[12] = c12; x[13] = c13; x[14] = c14; x[15] = c15;
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
  x[0] += 0x61707865u; x[1] += 0x3320646eu; x[2] += 0x79622d32u; x[3] += 0x6b206574u;
#pragma unroll
  for (int i = 0; i < 8; i++) x[4 + i] += k[i];
  x[12] += c12; x[13] += c13; x[14] += c14; x[15] += c15;
}

// One wave: records r = (first record of the wave) + lane, one per lane
// (t1_enc.c:832-975 for the ChaCha suites, e_chacha20poly1305.c:124-286).
// The staged loop and the record's end.  NARROW (round 5): every record's
// offset in its buffer fits 32 bits, so a piece's pointer is one ds_bpermute
// of that offset (plus the buffer base) instead of two of the 64-bit pointer.
template <bool SEAL, bool LATE_STORES, bool NARROW, bool UKEY = false>
__device__ __forceinline__ void cc_tls_body(const BatchArgs& a, uint32_t r, uint32_t lane, uint8_t* tile,
                                            uint8_t* key, cu32c* ukey, bool active, uint32_t n,
                                            uint32_t tag_len,
                                            uint32_t c13, uint32_t c14, uint32_t c15,
                                            uint64_t src_v, uint64_t dst_v, Poly& p) {
  // src_v / dst_v: the record's pointers, or with NARROW its 32-bit offsets in
  // the caller's buffers (an active record lies inside them, each at most
  // 4 GiB; an inactive lane's value is never used: its length shuffles as 0)
  auto ptr_of = [&](uint64_t v, const void* base, uint32_t rr) -> uint64_t {
    if (NARROW) return (uint64_t)(uintptr_t)base + (uint32_t)__shfl((int)(uint32_t)v, (int)rr);
    return shfl64(v, rr);
  };
  // pieces this lane moves: records 8k + lane/8, piece (lane % 8 - record/2) % 8
  // of each step; the records' pointers and lengths are fetched with ds_bpermute
  // per step (keeping 8 x 5 of them in VGPRs would cost a wave per SIMD)
  uint32_t steps = (n + kCcStep - 1) / kCcStep;
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) steps = max(steps, (uint32_t)__shfl_xor((int)steps, m));
  uint32_t ctr = 0;
  // gather of step s: 8 records x 128 B per load instruction, into registers
  // (issued one step ahead, so the loads fly during the previous step's math)
  auto gather = [&](uint32_t base, uint4 (&v)[kCcP]) {
#pragma unroll
    for (int k = 0; k < kCcP; k++) {
      const uint32_t rr = kCcR * k + lane / kCcP;
      const uint32_t off = base + 16u * (((lane % kCcP) - (rr >> 1)) & 7u);
      const uint32_t snk = __shfl(n, (int)rr);
      // ds_bpermute outside the branch: an inactive source lane reads as 0
      const uint64_t srck = ptr_of(src_v, a.in, rr);
      v[k] = make_uint4(0, 0, 0, 0);
      if (off < snk && !(a.hy_flags & kCcDiagNoLoads)) {
        const uint8_t* sp = (const uint8_t*)(uintptr_t)srck + off;
        if (((uintptr_t)sp & 15) == 0) {
          v[k] = gload16(sp);  // full or last piece: an aligned 16 B never crosses a page
        } else {  // wire fragments (misaligned): only dwords that hold a record byte
          uint32_t w[4];
          load16_upto(sp, min(16u, snk - off), w);
          v[k] = make_uint4(w[0], w[1], w[2], w[3]);
        }
      }
    }
  };
  // Step order.  LATE_STORES (round 5): the scatter of step s reads its pieces
  // from the tile into registers, the tile takes step s + 1's gathered pieces
  // in the same pass (the lane's own slots, so no wave sync between), and only
  // then are step s's stores and step s + 2's loads issued.  vmcnt counts loads
  // and stores together and the compiler waits for zero when both are pending,
  // so a tile fill right after the stores (the other order) makes every step
  // wait for its previous step's write acknowledgements, which are slow for the
  // partial lines a straddling window writes; with LATE_STORES everything the
  // fill waits for was issued before the step's compute.
  uint4 pf[kCcP];
  gather(0, pf);
  if (LATE_STORES) {
#pragma unroll
    for (int k = 0; k < kCcP; k++) *reinterpret_cast<uint4*>(tile + 1024u * k + 16u * lane) = pf[k];
    if (steps > 1) gather(kCcStep, pf);
  }
  for (uint32_t s = 0; s < steps; s++) {
    const uint32_t base = s * kCcStep;
    if (!LATE_STORES) {
#pragma unroll
      for (int k = 0; k < kCcP; k++) *reinterpret_cast<uint4*>(tile + 1024u * k + 16u * lane) = pf[k];
      if (s + 1 < steps) gather(base + kCcStep, pf);
    }
    lds_wave_sync();
    // en/decrypt + MAC this lane's row: 2 ChaCha blocks
    if (base < n && !(a.hy_flags & kCcDiagNoCompute)) {
#pragma unroll 1
      for (int h = 0; h < (int)(kCcStep / 64); h++) {
        const uint32_t o64 = base + 64u * h;
        if (o64 >= n) break;
        ctr += 1;  // data blocks count from 1 (chacha-merged.c:230-236; TLS records < 2^32 blocks)
        uint32_t ks[16];
        if (UKEY) cc_block_sk(ks, ukey, ctr, c13, c14, c15);
        else cc_block_lds(ks, key, ctr, c13, c14, c15);
#pragma unroll
        for (int q = 0; q < 4; q++) {
          const uint32_t o = o64 + 16 * q;
          if (o >= n) break;
          const uint32_t nb = min(16u, n - o);
          uint4* slot = reinterpret_cast<uint4*>(tile + cc_slot(lane, 4 * h + q));
          const uint4 t = *slot;
          uint32_t in[4] = {t.x, t.y, t.z, t.w};
          uint32_t ob[4] = {in[0] ^ ks[4 * q], in[1] ^ ks[4 * q + 1], in[2] ^ ks[4 * q + 2],
                            in[3] ^ ks[4 * q + 3]};
          if (nb < 16) {  // zero the bytes past the record (MAC pad16 / staged garbage)
#pragma unroll
            for (int w = 0; w < 4; w++) {
              int32_t b = (int32_t)nb - 4 * w;
              uint32_t keep = b >= 4 ? 0xFFFFFFFFu : (b <= 0 ? 0u : ((1u << (8 * b)) - 1u));
              ob[w] &= keep;
              in[w] &= keep;
            }
          }
          *slot = make_uint4(ob[0], ob[1], ob[2], ob[3]);
          const uint32_t* c = SEAL ? ob : in;
          poly_block(p, c[0], c[1], c[2], c[3], 1u << 24);
        }
      }
    }
    lds_wave_sync();
    // scatter.  LATE_STORES: one wait for everything issued before the compute
    // (step s + 1's loads, step s - 1's stores), then per piece: read the slot,
    // refill it with step s + 1's piece, store the read piece
    const bool refill = LATE_STORES && s + 1 < steps;
    if (LATE_STORES) __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0) only
#pragma unroll
    for (int k = 0; k < kCcP; k++) {
      const uint32_t rr = kCcR * k + lane / kCcP;
      const uint32_t off = base + 16u * (((lane % kCcP) - (rr >> 1)) & 7u);
      const uint32_t snk = __shfl(n, (int)rr);
      const uint64_t dstk = ptr_of(dst_v, a.out, rr);
      uint4* tslot = reinterpret_cast<uint4*>(tile + 1024u * k + 16u * lane);
      uint4 v = make_uint4(0, 0, 0, 0);
      if (LATE_STORES) {
        v = *tslot;
        if (refill) *tslot = pf[k];
      }
      if (off < snk && !(a.hy_flags & kCcDiagNoStores)) {
        uint8_t* dp = (uint8_t*)(uintptr_t)dstk + off;
        if (!LATE_STORES) v = *tslot;
        if (off + 16 <= snk && ((uintptr_t)dp & 15) == 0) {
          gstore16(dp, v);
        } else if (off + 16 <= snk) {
          const uint32_t w[4] = {v.x, v.y, v.z, v.w};
          store16_any(dp, w);
        } else {
          const uint32_t w[4] = {v.x, v.y, v.z, v.w};
          const uint32_t nb = min(16u, snk - off);
          for (uint32_t b = 0; b < nb; b++) gst<uint8_t>(dp)[b] = (uint8_t)(w[b >> 2] >> (8 * (b & 3)));
        }
      }
    }
    if (LATE_STORES) {
      if (s + 2 < steps) gather(base + 2 * kCcStep, pf);
    } else {
      lds_wave_sync();
    }
  }
  if (!active) return;
  const uint8_t* src = NARROW ? a.in + (uint32_t)src_v : (const uint8_t*)(uintptr_t)src_v;
  uint8_t* dst = NARROW ? a.out + (uint32_t)dst_v : (uint8_t*)(uintptr_t)dst_v;
  poly_block(p, 13u, 0, n, 0, 1u << 24);  // le64(ad_len) || le64(ct_len)
  uint32_t mac[4];
  poly_finish(p, mac);
  int32_t* slot = a.status + r;
  // full 16-B tags through dword accesses (one instruction per dword instead
  // of one per byte: each lane's tag is in another record); truncated tags
  // byte by byte
  if (SEAL) {
    uint8_t* tag_out = dst + n;
    if (tag_len == 16) {
      store16_any(tag_out, mac);
    } else {
      for (uint32_t k = 0; k < tag_len; k++) tag_out[k] = (uint8_t)(mac[k >> 2] >> (8 * (k & 3)));
    }
    *slot = (int32_t)(n + tag_len);
  } else {
    const uint8_t* tag_in = src + n;
    uint32_t diff = 0;
    if (tag_len == 16) {  // every byte compared (timingsafe_memcmp)
      uint32_t t[4];
      load16_any(tag_in, t);
      diff = (t[0] ^ mac[0]) | (t[1] ^ mac[1]) | (t[2] ^ mac[2]) | (t[3] ^ mac[3]);
    } else {
      for (uint32_t k = 0; k < tag_len; k++) diff |= tag_in[k] ^ ((mac[k >> 2] >> (8 * (k & 3))) & 0xFF);
    }
    if (diff) {
      zero_fill_lane(dst, n);
      *slot = TLSGPU_REC_BAD_MAC;
    } else {
      *slot = (int32_t)n;
    }
  }
}

template <bool SEAL, bool LATE_STORES, bool NARROW = false>
__device__ void cc_tls_wave(const BatchArgs& a, uint32_t r, uint32_t lane, uint8_t* tile,
                            uint8_t* keys) {
  // --- parse (the fields the end of the record needs are re-derived there)
  bool active = false;
  uint32_t n = 0, tag_len = 16, c13 = 0, c14 = 0, c15 = 0;
  uint32_t ad2 = 0;  // AD word 2 (type, version, length high byte); words 0-1 = c14/c15 (RFC)
  const uint8_t* src = nullptr;
  uint8_t* dst = nullptr;
  uint32_t sq_hi = 0, sq_lo = 0;
  uint32_t sess = 0xFFFFFFFFu;
  if (r < a.n) {
    const tlsgpu_record d = reinterpret_cast<const tlsgpu_record*>(a.descs)[r];
    // fused (round 5, engine.cpp run_batch: a batch of RFC ChaCha sessions
    // only): the caller's descriptors, checked here by check_record_bounds's
    // rule, and the initial status of a record this kernel does not run
    int32_t st0 = TLSGPU_REC_PUBLIC_INVALID;
    if (d.session < a.n_sessions) {  // else the status stays PUBLIC_INVALID
      const DevSession* S = a.sessions + d.session;
      const uint32_t kind = S->kind;
      bool in_bounds = true;
      if (a.fused) {
        const uint64_t len = d.len_type & 0xFFFFFFu, tag = S->tag_len;
        const uint64_t eiv = S->nonce_in_record ? 8u : 0u;
        const uint64_t out_len = SEAL ? len + eiv + tag : (len >= eiv + tag ? len - eiv - tag : 0);
        in_bounds = !(d.in_off > a.in_bytes || len > a.in_bytes - d.in_off ||
                      d.out_off > a.out_bytes || out_len > a.out_bytes - d.out_off);
        if (!in_bounds) st0 = TLSGPU_REC_OUT_OF_BOUNDS;
      }
      if (kind == TLSGPU_CHACHA20_POLY1305 && in_bounds) {  // the draft ("old") suite: chacha_batch_kernel
        tag_len = S->tag_len;
        const uint32_t len = d.len_type & 0xFFFFFFu, type = d.len_type >> 24;
        if (!SEAL && len < tag_len) {  // t1_enc.c:958-959 (no explicit nonce for ChaCha)
          a.status[r] = TLSGPU_REC_PUBLIC_INVALID;
        } else {
          active = true;
          sess = d.session;
          n = SEAL ? len : len - tag_len;
          src = a.in + d.in_off;
          dst = a.out + d.out_off;
          // nonce: RFC 7905 fixed(12) XOR (0^4 || seq)
          sq_hi = bswap32((uint32_t)(d.seq >> 32));
          sq_lo = bswap32((uint32_t)d.seq);
          const uint32_t* fx = reinterpret_cast<const uint32_t*>(S->fixed_nonce);
          c13 = fx[0];
          c14 = fx[1] ^ sq_hi;
          c15 = fx[2] ^ sq_lo;
          const uint32_t v = S->version;
          ad2 = type | (((v >> 8) & 0xFF) << 8) | ((v & 0xFF) << 16) | (((n >> 8) & 0xFF) << 24);
          const uint4* kw = reinterpret_cast<const uint4*>(S->chacha_key);
          reinterpret_cast<uint4*>(keys)[lane] = kw[0];
          reinterpret_cast<uint4*>(keys)[kWave + lane] = kw[1];
        }
      }
    }
    if (a.fused && !active) a.status[r] = st0;
  }
  uint8_t* key = keys + 16u * lane;
  lds_wave_sync();
  Poly p;
  if (active) {
    uint32_t ks[16];
    cc_block_lds(ks, key, 0u, c13, c14, c15);  // counter 0 block -> one-time Poly1305 key
    poly_init(p, ks);
    poly_block(p, sq_hi, sq_lo, ad2, n & 0xFF, 1u << 24);  // 13-B AD, pad16
  }
  // NARROW (the launch's choice, launch_chacha): a fused batch whose buffers
  // are at most 4 GiB each, so a record's offset fits 32 bits
  const uint64_t sv = NARROW ? (uint64_t)(uint32_t)(src - a.in) : (uint64_t)(uintptr_t)src;
  const uint64_t dv = NARROW ? (uint64_t)(uint32_t)(dst - a.out) : (uint64_t)(uintptr_t)dst;
  // UKEY: every active lane's record is of one session, so
  // the key words come from that session through s_load, not from LDS
  const uint64_t act = __ballot(active);
  const int l0 = act ? __ffsll((long long)act) - 1 : 0;
  const uint32_t sid0 = __builtin_amdgcn_readlane(sess, l0);
  const bool ukey = act != 0 && !__any(active && sess != sid0) &&
                    !(a.hy_flags & kCcNoUkey);
  if (ukey) {
    cu32c* k = (cu32c*)(const uint32_t*)a.sessions[sid0].chacha_key;
    cc_tls_body<SEAL, LATE_STORES, NARROW, true>(a, r, lane, tile, key, k, active, n, tag_len, c13,
                                                 c14, c15, sv, dv, p);
  } else {
    cc_tls_body<SEAL, LATE_STORES, NARROW, false>(a, r, lane, tile, key, nullptr, active, n,
                                                  tag_len, c13, c14, c15, sv, dv, p);
  }
}

__device__ __forceinline__ void cc_state(uint32_t st[16], const DevSession* S) {
  st[0] = 0x61707865u; st[1] = 0x3320646eu; st[2] = 0x79622d32u; st[3] = 0x6b206574u;
  const uint32_t* kw = reinterpret_cast<const uint32_t*>(S->chacha_key);
#pragma unroll
  for (int i = 0; i < 8; i++) st[4 + i] = kw[i];
}

// TLS descriptor -> CcRec (t1_enc.c:832-975 for the ChaCha suites).  Returns
// false when the record is not this kernel's (other kind / bad session: status
// untouched) or publicly invalid (status written).
template <bool SEAL>
__device__ __forceinline__ bool cc_parse_tls(const BatchArgs& a, uint32_t r, CcRec& rc,
                                             uint32_t& tag_len) {
  int32_t* slot = a.status + r;
  const DevSession* S;
  const tlsgpu_record d = reinterpret_cast<const tlsgpu_record*>(a.descs)[r];
  if (d.session >= a.n_sessions) return false;  // status stays PUBLIC_INVALID
  S = a.sessions + d.session;
  uint32_t kind = S->kind;
  if (kind != TLSGPU_CHACHA20_POLY1305 && kind != TLSGPU_CHACHA20_POLY1305_OLD) return false;
  tag_len = S->tag_len;
  rc.old = kind == TLSGPU_CHACHA20_POLY1305_OLD;
  uint32_t len = d.len_type & 0xFFFFFFu, type = d.len_type >> 24;
  const uint8_t* ip = a.in + d.in_off;
  uint8_t* op = a.out + d.out_off;
  if (SEAL) {
    rc.n = len;
    rc.src = ip;
    rc.dst = op;
    rc.tag_out = op + len;
    rc.ok_status = (int32_t)(len + tag_len);
    rc.zero_len = 0;
  } else {
    if (len < tag_len) {  // t1_enc.c:958-959 (no explicit nonce for ChaCha)
      *slot = TLSGPU_REC_PUBLIC_INVALID;
      return false;
    }
    rc.n = len - tag_len;
    rc.src = ip;
    rc.dst = op;
    rc.tag_in = ip + rc.n;
    rc.ok_status = (int32_t)rc.n;
    rc.zero_len = rc.n;
  }
  // nonce: RFC 7905 fixed(12) XOR (0^4 || seq) ; old: fixed(0) || seq
  uint32_t sq_hi = bswap32((uint32_t)(d.seq >> 32)), sq_lo = bswap32((uint32_t)d.seq);
  cc_state(rc.st, S);
  const uint32_t* fx = reinterpret_cast<const uint32_t*>(S->fixed_nonce);
  rc.st[12] = 0;
  if (!rc.old) {
    rc.st[13] = fx[0];
    rc.st[14] = fx[1] ^ sq_hi;
    rc.st[15] = fx[2] ^ sq_lo;
  } else {
    rc.st[13] = 0;
    rc.st[14] = sq_hi;
    rc.st[15] = sq_lo;
  }
  uint32_t v = S->version;
  rc.aad_ptr = nullptr;
  rc.ad_len = 13;
  rc.ad[0] = sq_hi;
  rc.ad[1] = sq_lo;
  rc.ad[2] = type | (((v >> 8) & 0xFF) << 8) | ((v & 0xFF) << 16) | (((rc.n >> 8) & 0xFF) << 24);
  rc.ad[3] = rc.n & 0xFF;
  return true;
}

// Raw EVP job -> CcRec (e_chacha20poly1305.c:124-286; the host checked
// nonce_len, in_len >= tag_len and the output room).
template <bool SEAL>
__device__ __forceinline__ void cc_parse_raw(const RawJob& j, const DevSession* S, CcRec& rc,
                                             uint32_t& tag_len) {
  const uint32_t kind = S->kind;
  tag_len = S->tag_len;
  rc.old = kind == TLSGPU_CHACHA20_POLY1305_OLD;
  const uint8_t* nonce = (const uint8_t*)j.nonce;
  cc_state(rc.st, S);
  if (!rc.old) {  // ctr = LE32(nonce[0..3]) << 32 ; iv = nonce + 4
    rc.st[12] = 0;
    rc.st[13] = ld_le32(nonce);
    rc.st[14] = ld_le32(nonce + 4);
    rc.st[15] = ld_le32(nonce + 8);
  } else {
    rc.st[12] = 0; rc.st[13] = 0;
    rc.st[14] = ld_le32(nonce);
    rc.st[15] = ld_le32(nonce + 4);
  }
  rc.src = (const uint8_t*)j.in;
  rc.dst = (uint8_t*)j.out;
  rc.aad_ptr = (const uint8_t*)j.aad;
  rc.ad_len = j.aad_len;
  if (SEAL) {
    rc.n = j.in_len;
    rc.tag_out = rc.dst + j.in_len;
    rc.ok_status = (int32_t)(j.in_len + tag_len);
  } else {
    rc.n = j.in_len - tag_len;
    rc.tag_in = rc.src + rc.n;
    rc.ok_status = (int32_t)rc.n;
  }
  rc.zero_len = j.max_out;
}

// TLS batches: LDS-staged coalesced data path (cc_tls_wave), 4 waves per SIMD.
template <bool SEAL>
__global__ __launch_bounds__(kCcThreads) void chacha_tls_wide_kernel(BatchArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t tiles[kCcThreads / kWave][kCcTile];
  __shared__ __attribute__((aligned(16))) uint8_t keys[kCcThreads / kWave][kCcKeys];
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  cc_tls_wave<SEAL, false>(a, blockIdx.x * blockDim.x + threadIdx.x, lane, tiles[wave], keys[wave]);
}
// the same with 32-bit pointer shuffles (NARROW: cc_tls_body) — what a fused
// batch (bounds known, buffers of at most 4 GiB) runs: C +0.6 %
// (profiles/r05ap_ab_cc_narrow.txt); 64-bit shuffles otherwise
template <bool SEAL>
__global__ __launch_bounds__(kCcThreads) void chacha_tls_kernel(BatchArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t tiles[kCcThreads / kWave][kCcTile];
  __shared__ __attribute__((aligned(16))) uint8_t keys[kCcThreads / kWave][kCcKeys];
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  cc_tls_wave<SEAL, false, true>(a, blockIdx.x * blockDim.x + threadIdx.x, lane, tiles[wave],
                                 keys[wave]);
}
// the LATE_STORES order (A/B only, TLSGPU_CC_ORDER): at 3 waves per SIMD (131
// VGPRs), and held to 128 VGPRs (4 waves per SIMD, 5 spilled)
template <bool SEAL>
__global__ __launch_bounds__(kCcThreads) void chacha_tls_late3_kernel(BatchArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t tiles[kCcThreads / kWave][kCcTile];
  __shared__ __attribute__((aligned(16))) uint8_t keys[kCcThreads / kWave][kCcKeys];
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  cc_tls_wave<SEAL, true>(a, blockIdx.x * blockDim.x + threadIdx.x, lane, tiles[wave], keys[wave]);
}
template <bool SEAL>
__global__ __launch_bounds__(kCcThreads) __attribute__((amdgpu_waves_per_eu(4, 4))) void chacha_tls_late4_kernel(BatchArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t tiles[kCcThreads / kWave][kCcTile];
  __shared__ __attribute__((aligned(16))) uint8_t keys[kCcThreads / kWave][kCcKeys];
  const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  cc_tls_wave<SEAL, true>(a, blockIdx.x * blockDim.x + threadIdx.x, lane, tiles[wave], keys[wave]);
}

// Per-lane data path: raw EVP jobs, TLS records of the draft suite (OLD_ONLY:
// beside chacha_tls_kernel, which takes the RFC 7905 suite), and
// TLSGPU_CHACHA_LEGACY=1 TLS batches.
template <bool SEAL, bool RAW, bool OLD_ONLY = false>
__global__ __launch_bounds__(256) void chacha_batch_kernel(BatchArgs a) {
  const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= a.n) return;
  CcRec rc;
  int32_t* slot = a.status + r;
  const DevSession* S;
  uint32_t tag_len;
  if (RAW) {
    const RawJob j = reinterpret_cast<const RawJob*>(a.descs)[r];
    // no per-batch status memset for raw jobs (run_batch): a bad or empty
    // session is publicly invalid here (the GCM raw kernel writes the same)
    if (j.session >= a.n_sessions) { *slot = TLSGPU_REC_PUBLIC_INVALID; return; }
    S = a.sessions + j.session;
    uint32_t kind = S->kind;
    if (kind < TLSGPU_AES_128_GCM || kind > TLSGPU_CHACHA20_POLY1305_OLD) {
      *slot = TLSGPU_REC_PUBLIC_INVALID;
      return;
    }
    if (kind != TLSGPU_CHACHA20_POLY1305 && kind != TLSGPU_CHACHA20_POLY1305_OLD) return;
    cc_parse_raw<SEAL>(j, S, rc, tag_len);
  } else {
    if (OLD_ONLY) {  // the staged kernel leaves these records' statuses alone
      const tlsgpu_record d = reinterpret_cast<const tlsgpu_record*>(a.descs)[r];
      if (d.session >= a.n_sessions || a.sessions[d.session].kind != TLSGPU_CHACHA20_POLY1305_OLD)
        return;
    }
    if (!cc_parse_tls<SEAL>(a, r, rc, tag_len)) return;
  }
  cc_record<SEAL>(rc, tag_len, slot);
}

// Raw EVP jobs, one wave per job: the RFC 7539 AEAD on the whole wave
// (chacha_wave.h: per-call latency), the draft AEAD too (cc_wave_job_old, round 5).
template <bool SEAL>
__global__ __launch_bounds__(kWave) void chacha_raw_wave_kernel(BatchArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t stage[4096];
  const uint32_t r = blockIdx.x;
  const RawJob j = reinterpret_cast<const RawJob*>(a.descs)[r];
  int32_t* slot = a.status + r;
  // no per-batch status memset for raw jobs (run_batch): as chacha_batch_kernel
  if (j.session >= a.n_sessions) {
    if (threadIdx.x == 0) *slot = TLSGPU_REC_PUBLIC_INVALID;
    return;
  }
  const DevSession* S = a.sessions + j.session;
  const uint32_t kind = S->kind;
  if (kind < TLSGPU_AES_128_GCM || kind > TLSGPU_CHACHA20_POLY1305_OLD) {
    if (threadIdx.x == 0) *slot = TLSGPU_REC_PUBLIC_INVALID;
    return;
  }
  if (kind == TLSGPU_CHACHA20_POLY1305) {
    cc_wave_job<SEAL>(j, S, slot, stage);
  } else if (kind == TLSGPU_CHACHA20_POLY1305_OLD) {
    cc_wave_job_old<SEAL>(j, S, slot, true, stage);
  }
}

// TLSGPU_CHACHA_LEGACY=1 selects the per-lane data path for TLS batches too
// (A/B measurement of the staged kernel).
static bool getenv_legacy_chacha() {
  static const bool v = [] {
    const char* e = getenv("TLSGPU_CHACHA_LEGACY");
    return e && *e && *e != '0';
  }();
  return v;
}

// rfc / old: the batch may hold records of the RFC 7905 / draft suite.
int launch_chacha(const BatchArgs& a, bool seal, bool raw, bool rfc, bool old, hipStream_t s) {
  if (a.n == 0) return 0;
  dim3 grid((a.n + 255) / 256), block(256);
  const bool staged = !raw && !getenv_legacy_chacha();
  if (raw && !getenv_legacy_chacha()) {  // one wave per job
    if (seal) hipLaunchKernelGGL((chacha_raw_wave_kernel<true>), dim3(a.n), dim3(kWave), 0, s, a);
    else hipLaunchKernelGGL((chacha_raw_wave_kernel<false>), dim3(a.n), dim3(kWave), 0, s, a);
    return hipGetLastError() == hipSuccess ? 0 : -1;
  }
  if (raw || !staged) {
    if (seal) {
      if (raw) hipLaunchKernelGGL((chacha_batch_kernel<true, true>), grid, block, 0, s, a);
      else hipLaunchKernelGGL((chacha_batch_kernel<true, false>), grid, block, 0, s, a);
    } else {
      if (raw) hipLaunchKernelGGL((chacha_batch_kernel<false, true>), grid, block, 0, s, a);
      else hipLaunchKernelGGL((chacha_batch_kernel<false, false>), grid, block, 0, s, a);
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
  }
  if (rfc) {
    // TLSGPU_CC_LDS_PAD=<bytes> (A/B only): unused dynamic LDS per 4-wave
    // workgroup, which lowers the waves per SIMD (40 KiB static: 1 B more = 3)
    static const unsigned pad_all = [] {
      const char* e = getenv("TLSGPU_CC_LDS_PAD");
      return e ? (unsigned)strtoul(e, nullptr, 10) : 0u;
    }();
    // per direction (A/B): TLSGPU_CC_LDS_PAD_OPEN / _SEAL
    static const unsigned pad_dir[2] = {[] {
      const char* e = getenv("TLSGPU_CC_LDS_PAD_OPEN");
      return e ? (unsigned)strtoul(e, nullptr, 10) : 0u;
    }(), [] {
      const char* e = getenv("TLSGPU_CC_LDS_PAD_SEAL");
      return e ? (unsigned)strtoul(e, nullptr, 10) : 0u;
    }()};
    const unsigned pad = pad_all ? pad_all : pad_dir[seal ? 1 : 0];
    static const uint32_t diag = [] {
      const char* e = getenv("TLSGPU_CC_DIAG");
      return e ? (uint32_t)strtoul(e, nullptr, 0) & 7u : 0u;
    }();
    static const uint32_t no_narrow = [] {
      const char* e = getenv("TLSGPU_CC_NARROW");
      return e && *e == '0' ? kCcNoNarrow : 0u;
    }();
    static const uint32_t no_ukey = [] {
      const char* e = getenv("TLSGPU_CC_UKEY");
      return e && *e == '0' ? kCcNoUkey : 0u;
    }();
    BatchArgs b = a;
    b.hy_flags = diag | no_ukey;
    // NARROW needs the buffer sizes (a fused batch: run_batch passes them, and
    // the kernel runs only records inside them): a piece's pointer is then the
    // buffer base + a 32-bit offset
    const bool narrow = !no_narrow && a.fused && a.in_bytes <= (1ull << 32) &&
                        a.out_bytes <= (1ull << 32);
    // TLSGPU_CC_ORDER (A/B): 0 (default) tile fill after the stores, 1
    // LATE_STORES (131 VGPRs, 3 waves per SIMD), 2 LATE_STORES held to 4 waves
    // per SIMD (5 spilled VGPRs).  2 measured +0.6 % on C in the clock dip of
    // the old bench order, then -0.9 % with the warm-start bench
    // (profiles/r05w_ab_cc_order.txt, r05am_ab_warm.txt)
    static const int order = [] {
      const char* e = getenv("TLSGPU_CC_ORDER");
      return e ? atoi(e) : 0;
    }();
    if (order == 1) {
      if (seal) hipLaunchKernelGGL((chacha_tls_late3_kernel<true>), grid, block, pad, s, b);
      else hipLaunchKernelGGL((chacha_tls_late3_kernel<false>), grid, block, pad, s, b);
    } else if (order == 2) {
      if (seal) hipLaunchKernelGGL((chacha_tls_late4_kernel<true>), grid, block, pad, s, b);
      else hipLaunchKernelGGL((chacha_tls_late4_kernel<false>), grid, block, pad, s, b);
    } else if (narrow) {
      if (seal) hipLaunchKernelGGL((chacha_tls_kernel<true>), grid, block, pad, s, b);
      else hipLaunchKernelGGL((chacha_tls_kernel<false>), grid, block, pad, s, b);
    } else {
      if (seal) hipLaunchKernelGGL((chacha_tls_wide_kernel<true>), grid, block, pad, s, b);
      else hipLaunchKernelGGL((chacha_tls_wide_kernel<false>), grid, block, pad, s, b);
    }
  }
  if (old) {
    if (seal) hipLaunchKernelGGL((chacha_batch_kernel<true, false, true>), grid, block, 0, s, a);
    else hipLaunchKernelGGL((chacha_batch_kernel<false, false, true>), grid, block, 0, s, a);
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace tg
