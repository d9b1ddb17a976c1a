// session_kernels.hip — device session install and synthetic-data kernels.
//
// tlsgpu_sessions_install() runs install_sessions: one wave per session does
// what aead_aes_gcm_init / CRYPTO_gcm128_init (crypto/evp/e_aes.c:1372-1413,
// crypto/modes/gcm128.c:681-747) and aead_chacha20_poly1305_init
// (e_chacha20poly1305.c:52-79) do at ChangeCipherSpec, plus the GHASH power
// tables the batch kernels need.  Cold path: bit-serial GF(2^128) arithmetic.
#include "aes_common.h"
#include "tlsgpu_internal.h"

namespace tg {

__device__ const ByteTable g_sbox = kSbox;

struct U128 { uint64_t hi, lo; };  // big-endian halves, x^0 = MSB of hi

__device__ inline U128 gf_mulx(U128 v) {
  uint64_t carry = v.lo & 1;
  v.lo = (v.lo >> 1) | (v.hi << 63);
  v.hi = (v.hi >> 1) ^ (carry ? 0xE100000000000000ull : 0);
  return v;
}

__device__ inline U128 gf_mul(U128 a, U128 b) {  // SP 800-38D Algorithm 1
  U128 z{0, 0};
  for (int i = 0; i < 128; i++) {
    uint64_t bit = (i < 64) ? (a.hi >> (63 - i)) & 1 : (a.lo >> (127 - i)) & 1;
    if (bit) { z.hi ^= b.hi; z.lo ^= b.lo; }
    b = gf_mulx(b);
  }
  return z;
}

__device__ inline uint32_t sub_word(uint32_t w) {
  return ((uint32_t)g_sbox.v[w >> 24] << 24) | ((uint32_t)g_sbox.v[(w >> 16) & 0xff] << 16) |
         ((uint32_t)g_sbox.v[(w >> 8) & 0xff] << 8) | g_sbox.v[w & 0xff];
}

// FIPS-197 key expansion (aes_core.c:628-723); big-endian words.
__device__ inline int expand_key(const uint8_t* key, int key_len, uint32_t* rk_be) {
  int nk = key_len / 4, rounds = nk + 6, total = 4 * (rounds + 1);
  uint32_t rcon = 1;
  for (int i = 0; i < nk; i++)
    rk_be[i] = ((uint32_t)key[4 * i] << 24) | ((uint32_t)key[4 * i + 1] << 16) |
               ((uint32_t)key[4 * i + 2] << 8) | key[4 * i + 3];
  for (int i = nk; i < total; i++) {
    uint32_t t = rk_be[i - 1];
    if (i % nk == 0) {
      t = sub_word((t << 8) | (t >> 24)) ^ (rcon << 24);
      rcon = xtime8((uint8_t)rcon);
    } else if (nk > 6 && i % nk == 4) {
      t = sub_word(t);
    }
    rk_be[i] = rk_be[i - nk] ^ t;
  }
  return rounds;
}

// Byte-wise AES encryption of one block (aes_core.c:789-972), cold path only.
__device__ inline void aes_encrypt_bytes(const uint32_t* rk_be, int rounds, uint8_t s[16]) {
  uint8_t t[16];
  for (int i = 0; i < 16; i++) s[i] ^= (uint8_t)(rk_be[i / 4] >> (24 - 8 * (i % 4)));
  for (int r = 1; r <= rounds; r++) {
    for (int c = 0; c < 4; c++)
      for (int i = 0; i < 4; i++) t[c * 4 + i] = g_sbox.v[s[((c + i) & 3) * 4 + i]];
    for (int c = 0; c < 4; c++) {
      uint8_t a0 = t[4 * c], a1 = t[4 * c + 1], a2 = t[4 * c + 2], a3 = t[4 * c + 3];
      if (r != rounds) {
        uint8_t all = a0 ^ a1 ^ a2 ^ a3;
        s[4 * c + 0] = a0 ^ all ^ xtime8(a0 ^ a1);
        s[4 * c + 1] = a1 ^ all ^ xtime8(a1 ^ a2);
        s[4 * c + 2] = a2 ^ all ^ xtime8(a2 ^ a3);
        s[4 * c + 3] = a3 ^ all ^ xtime8(a3 ^ a0);
      } else {
        s[4 * c] = a0; s[4 * c + 1] = a1; s[4 * c + 2] = a2; s[4 * c + 3] = a3;
      }
    }
    for (int i = 0; i < 16; i++) s[i] ^= (uint8_t)(rk_be[4 * r + i / 4] >> (24 - 8 * (i % 4)));
  }
}

__device__ inline void store_le(uint32_t* w, U128 v) {  // 16-byte string -> LE words
  w[0] = bswap32((uint32_t)(v.hi >> 32));
  w[1] = bswap32((uint32_t)v.hi);
  w[2] = bswap32((uint32_t)(v.lo >> 32));
  w[3] = bswap32((uint32_t)v.lo);
}
__device__ inline void store_be(uint32_t* w, U128 v) {
  w[0] = (uint32_t)(v.hi >> 32);
  w[1] = (uint32_t)v.hi;
  w[2] = (uint32_t)(v.lo >> 32);
  w[3] = (uint32_t)v.lo;
}

// One wave per session (blockIdx.x = session index): the key schedule and H
// are computed by every lane (wave-uniform), then the 65 GHASH powers, their
// Shoup tables, the H^64 basis and the bitsliced round-key masks are split
// over the lanes.  Lane e gets H^(e+1) by square-and-multiply from the seven
// squarings H^(2^k), so the longest chain is 6 squarings + 6 products instead
// of the 64 serial products of a one-thread-per-session form (487 us per
// session on MI355X, which was the EVP_AEAD_CTX_init latency).
__global__ __launch_bounds__(64) void install_sessions(DevSession* __restrict__ sessions,
                                                       DevGcmTables* __restrict__ tables,
                                                       const tlsgpu_session_params* __restrict__ params,
                                                       uint32_t first, uint32_t n) {
  const uint32_t i = blockIdx.x;
  const uint32_t lane = threadIdx.x;
  if (i >= n) return;
  const tlsgpu_session_params p = params[i];
  DevSession s = {};
  uint32_t id = first + i;
  bool gcm = p.aead == TLSGPU_AES_128_GCM || p.aead == TLSGPU_AES_256_GCM;
  bool cc = p.aead == TLSGPU_CHACHA20_POLY1305 || p.aead == TLSGPU_CHACHA20_POLY1305_OLD;
  uint32_t want_key = p.aead == TLSGPU_AES_128_GCM ? 16 : 32;
  uint32_t tag = p.tag_len == 0 ? 16 : p.tag_len;
  if ((!gcm && !cc) || p.key_len != want_key || tag > 16 || p.fixed_iv_len > 12) {
    if (lane == 0) sessions[id] = s;  // kind 0: empty / invalid
    return;
  }
  s.kind = (uint32_t)p.aead;
  s.tag_len = tag;
  s.key_len = p.key_len;
  s.fixed_nonce_len = p.fixed_iv_len;
  s.xor_fixed_nonce = p.aead == TLSGPU_CHACHA20_POLY1305;
  s.nonce_in_record = gcm;
  s.version = p.version;
  for (uint32_t k = 0; k < p.fixed_iv_len; k++) s.fixed_nonce[k] = p.fixed_iv[k];
  if (cc) {
    for (int k = 0; k < 32; k++) s.chacha_key[k] = p.key[k];
    if (lane == 0) sessions[id] = s;
    return;
  }
  uint32_t rk_be[60];
  s.rounds = (uint32_t)expand_key(p.key, (int)p.key_len, rk_be);
  for (int k = 0; k < 4 * ((int)s.rounds + 1); k++) {
    s.rk[k] = bswap32(rk_be[k]);
    s.rk_rot[k] = __builtin_amdgcn_alignbit(s.rk[k], s.rk[k], 16);
  }
  uint8_t hb[16] = {};
  aes_encrypt_bytes(rk_be, (int)s.rounds, hb);  // H = E_K(0^128)
  U128 H{0, 0};
  for (int k = 0; k < 8; k++) {
    H.hi = (H.hi << 8) | hb[k];
    H.lo = (H.lo << 8) | hb[8 + k];
  }
  store_le(s.h_le, H);
  if (lane == 0) sessions[id] = s;

  DevGcmTables* t = &tables[id];
  // bitsliced AddRoundKey masks: (rounds + 1) x 128 words over the lanes
  for (uint32_t w = lane; w < 128u * (s.rounds + 1); w += 64) {
    const uint32_t r = w / 128, b = (w % 128) / 8, k = w % 8;
    t->bsrk[r][8 * b + k] = 0u - ((s.rk[4 * r + b / 4] >> (8 * (b % 4) + k)) & 1u);
  }
  U128 sq[7];  // H^(2^k)
  sq[0] = H;
  for (int k = 1; k < 7; k++) sq[k] = gf_mul(sq[k - 1], sq[k - 1]);
  for (uint32_t e = lane + 1; e <= (uint32_t)kPowMax; e += 64) {
    U128 pw{0, 0};
    bool have = false;
    for (int k = 0; k < 7; k++) {
      if (!((e >> k) & 1)) continue;
      pw = have ? gf_mul(pw, sq[k]) : sq[k];
      have = true;
    }
    U128 m[16];
    m[0] = U128{0, 0};
    m[8] = pw;
    m[4] = gf_mulx(m[8]);
    m[2] = gf_mulx(m[4]);
    m[1] = gf_mulx(m[2]);
    for (int a = 2; a < 16; a <<= 1)
      for (int b = 1; b < a; b++) m[a + b] = U128{m[a].hi ^ m[b].hi, m[a].lo ^ m[b].lo};
    for (int v = 0; v < 16; v++) store_be(t->shoup[e - 1][v], m[v]);
  }
  // basis[q] = K * x^q, K = H^64 = sq[6]; lanes q and q + 64
  for (uint32_t q = lane; q < 128; q += 64) {
    U128 b = sq[6];
    for (uint32_t k = 0; k < q; k++) b = gf_mulx(b);
    store_le(t->basis[q], b);
  }
}

// Counter-based SplitMix64 bytes (identical to oracle_fill_bytes).
__global__ void fill_synthetic(uint8_t* __restrict__ out, uint64_t stride, uint32_t span_len,
                               uint32_t n, uint64_t seed, uint64_t index0) {
  uint32_t words = (span_len + 7) / 8;
  uint64_t total = (uint64_t)words * n;
  for (uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; g < total;
       g += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t span = g / words, w = g % words;
    uint64_t st = seed ^ ((index0 + span) * 0xD1B54A32D192ED03ull);
    uint64_t z = st + (w + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    uint8_t* p = out + span * stride + w * 8;
    uint32_t left = span_len - (uint32_t)(w * 8);
    if (left >= 8 && ((uintptr_t)p & 7) == 0) {
      *(uint64_t*)p = z;
    } else {
      for (uint32_t k = 0; k < 8 && k < left; k++) p[k] = (uint8_t)(z >> (8 * k));
    }
  }
}

// Variable-length spans in one launch: span i (offs[i], lens[i]) keyed index0 + i.
// One workgroup per span (grid-strided), 8 B per thread-step.
__global__ void fill_synthetic_spans(uint8_t* __restrict__ out, const uint64_t* __restrict__ offs,
                                     const uint32_t* __restrict__ lens, uint32_t n, uint64_t seed,
                                     uint64_t index0) {
  for (uint32_t span = blockIdx.x; span < n; span += gridDim.x) {
    const uint32_t len = lens[span];
    uint8_t* base = out + offs[span];
    const uint64_t st = seed ^ ((index0 + span) * 0xD1B54A32D192ED03ull);
    for (uint32_t w = threadIdx.x; w * 8 < len; w += blockDim.x) {
      uint64_t z = st + (uint64_t)(w + 1) * 0x9E3779B97F4A7C15ull;
      z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
      z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
      z ^= z >> 31;
      uint8_t* p = base + (uint64_t)w * 8;
      const uint32_t left = len - w * 8;
      if (left >= 8 && ((uintptr_t)p & 7) == 0) {
        *(uint64_t*)p = z;
      } else {
        for (uint32_t k = 0; k < 8 && k < left; k++) p[k] = (uint8_t)(z >> (8 * k));
      }
    }
  }
}

int launch_fill_synthetic_spans(uint8_t* d_out, const uint64_t* d_offs, const uint32_t* d_lens,
                                uint32_t n, uint64_t seed, uint64_t index0, hipStream_t s) {
  if (n == 0) return 0;
  const uint32_t blocks = n < 65536 ? n : 65536;
  hipLaunchKernelGGL(fill_synthetic_spans, dim3(blocks), dim3(256), 0, s, d_out, d_offs, d_lens, n,
                     seed, index0);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// Batch ABI bounds (tlsgpu_open_batch / _seal_batch take the sizes of d_in and
// d_out): a record whose input or output span leaves its buffer is dropped
// from the kernels' copy of the descriptors (session 0xFFFFFFFF, which every
// batch kernel skips) and gets TLSGPU_REC_OUT_OF_BOUNDS.  Output span = the
// plaintext on open (fragment - explicit nonce - tag), the fragment on seal.
__global__ void check_record_bounds(const tlsgpu_record* __restrict__ recs,
                                    tlsgpu_record* __restrict__ safe, uint32_t n,
                                    const DevSession* __restrict__ sessions, uint32_t n_sessions,
                                    uint64_t in_bytes, uint64_t out_bytes, int seal,
                                    int32_t* __restrict__ status) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  tlsgpu_record r = recs[i];
  if (r.session < n_sessions) {
    const DevSession& S = sessions[r.session];
    const uint64_t eiv = S.nonce_in_record ? 8u : 0u, tag = S.tag_len;
    const uint64_t len = r.len_type & 0xFFFFFFu;
    const uint64_t in_len = len;
    const uint64_t out_len = seal ? len + eiv + tag : (len >= eiv + tag ? len - eiv - tag : 0);
    if (r.in_off > in_bytes || in_len > in_bytes - r.in_off || r.out_off > out_bytes ||
        out_len > out_bytes - r.out_off) {
      r.session = 0xFFFFFFFFu;
      status[i] = TLSGPU_REC_OUT_OF_BOUNDS;
    }
  }
  safe[i] = r;
}

int launch_check_bounds(const tlsgpu_record* recs, tlsgpu_record* safe, uint32_t n,
                        const DevSession* sessions, uint32_t n_sessions, uint64_t in_bytes,
                        uint64_t out_bytes, bool seal, int32_t* status, hipStream_t s) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(check_record_bounds, dim3((n + 255) / 256), dim3(256), 0, s, recs, safe, n,
                     sessions, n_sessions, in_bytes, out_bytes, seal ? 1 : 0, status);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_session_install(DevSession* sessions, DevGcmTables* tables,
                           const tlsgpu_session_params* d_params, uint32_t first, uint32_t n,
                           hipStream_t s) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(install_sessions, dim3(n), dim3(64), 0, s, sessions, tables,
                     d_params, first, n);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_fill_synthetic(uint8_t* d_out, uint64_t stride, uint32_t span_len, uint32_t n,
                          uint64_t seed, uint64_t index0, hipStream_t s) {
  if (n == 0 || span_len == 0) return 0;
  uint64_t words = (uint64_t)((span_len + 7) / 8) * n;
  uint64_t blocks = (words + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(fill_synthetic, dim3((uint32_t)blocks), dim3(256), 0, s, d_out, stride,
                     span_len, n, seed, index0);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace tg
