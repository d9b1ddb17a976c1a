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

__device__ const ByteTable g_sbox __attribute__((aligned(16))) = kSbox;

struct U128 { uint64_t hi, lo; };  // big-endian halves, x^0 = MSB of hi

__device__ inline U128 gf_mulx(U128 v) {
  uint64_t carry = v.lo & 1;
  v.lo = (v.lo >> 1) | (v.hi << 63);
  v.hi = (v.hi >> 1) ^ (carry ? 0xE100000000000000ull : 0);
  return v;
}

// S-box lookups from the workgroup's LDS copy (a global-memory table costs a
// dependent L2 round trip per round of the serial key schedule)
__device__ inline uint32_t sub_word(const uint8_t* sb, uint32_t w) {
  return ((uint32_t)sb[w >> 24] << 24) | ((uint32_t)sb[(w >> 16) & 0xff] << 16) |
         ((uint32_t)sb[(w >> 8) & 0xff] << 8) | sb[w & 0xff];
}

// FIPS-197 key expansion (aes_core.c:628-723); big-endian words.
__device__ inline int expand_key(const uint8_t* sb, const uint8_t* key, int key_len,
                                 uint32_t* rk_be) {
  int nk = key_len / 4, rounds = nk + 6, total = 4 * (rounds + 1);
  uint32_t rcon = 1;
  for (int i = 0; i < nk; i++)
    rk_be[i] = ((uint32_t)key[4 * i] << 24) | ((uint32_t)key[4 * i + 1] << 16) |
               ((uint32_t)key[4 * i + 2] << 8) | key[4 * i + 3];
  uint32_t prev = rk_be[nk - 1];
  for (int i = nk; i < total; i++) {
    uint32_t t = prev;
    if (i % nk == 0) {
      t = sub_word(sb, (t << 8) | (t >> 24)) ^ (rcon << 24);
      rcon = xtime8((uint8_t)rcon);
    } else if (nk > 6 && i % nk == 4) {
      t = sub_word(sb, t);
    }
    prev = rk_be[i] = rk_be[i - nk] ^ t;
  }
  return rounds;
}

// Byte-wise AES encryption of one block (aes_core.c:789-972), cold path only.
__device__ inline void aes_encrypt_bytes(const uint8_t* sb, const uint32_t* rk_be, int rounds,
                                         uint8_t s[16]) {
  uint8_t t[16];
  for (int i = 0; i < 16; i++) s[i] ^= (uint8_t)(rk_be[i / 4] >> (24 - 8 * (i % 4)));
  for (int r = 1; r <= rounds; r++) {
    for (int c = 0; c < 4; c++)
      for (int i = 0; i < 4; i++) t[c * 4 + i] = sb[s[((c + i) & 3) * 4 + i]];
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
__device__ inline uint4 be_words(U128 v) {
  return make_uint4((uint32_t)(v.hi >> 32), (uint32_t)v.hi, (uint32_t)(v.lo >> 32), (uint32_t)v.lo);
}

// Shoup 4-bit table of y (gcm128.c:255-324 layout, big-endian words):
// m[8] = y, m[4] = y.x, m[2] = y.x^2, m[1] = y.x^3, m[a ^ b] = m[a] ^ m[b].
__device__ inline void shoup_table(U128 y, U128 (&m)[16]) {
  m[0] = U128{0, 0};
  m[8] = y;
  m[4] = gf_mulx(m[8]);
  m[2] = gf_mulx(m[4]);
  m[1] = gf_mulx(m[2]);
  for (int a = 2; a < 16; a <<= 1)
    for (int b = 1; b < a; b++) m[a + b] = U128{m[a].hi ^ m[b].hi, m[a].lo ^ m[b].lo};
}

// Entry v of y's Shoup table without building the others (a lane-indexed
// array would live in scratch memory): the XOR of m[8], m[4], m[2], m[1]
// selected by v's bits.
__device__ inline U128 shoup_entry(U128 y, uint32_t v) {
  const U128 y1 = gf_mulx(y), y2 = gf_mulx(y1), y3 = gf_mulx(y2);
  U128 r{0, 0};
  if (v & 8) { r.hi ^= y.hi; r.lo ^= y.lo; }
  if (v & 4) { r.hi ^= y1.hi; r.lo ^= y1.lo; }
  if (v & 2) { r.hi ^= y2.hi; r.lo ^= y2.lo; }
  if (v & 1) { r.hi ^= y3.hi; r.lo ^= y3.lo; }
  return r;
}

// rem_4bit[r] >> 32 (gcm128.c:327-331) on the VALU: (r * 0xE1) << 21, carry-less
__device__ inline uint32_t rem4v(uint32_t r) {
  return (r << 21) ^ ((r ^ (r << 1) ^ (r << 2)) << 26);
}

// z = x * y with y's Shoup table in LDS (16 x 16 B = all 64 banks: lanes with
// different nibbles never conflict, equal ones broadcast) — gcm_gmult_4bit
// (gcm128.c:333-393); 32 nibble steps instead of the 128 of a bit-serial product.
__device__ inline U128 gf_mul_tab(U128 x, const uint4* tab) {
  const uint32_t X[4] = {(uint32_t)(x.hi >> 32), (uint32_t)x.hi, (uint32_t)(x.lo >> 32),
                         (uint32_t)x.lo};
  // the 32 table reads depend on x only: issued ahead of the chain (round 3)
  uint4 t[32];
#pragma unroll
  for (int k = 0; k < 32; k++) t[k] = tab[(X[3 - k / 8] >> (4 * (k % 8))) & 0xF];
  uint32_t z0 = t[0].x, z1 = t[0].y, z2 = t[0].z, z3 = t[0].w;
#pragma unroll
  for (int k = 1; k < 32; k++) {
    const uint32_t rem = z3 & 0xF;
    z3 = __builtin_amdgcn_alignbit(z2, z3, 4);
    z2 = __builtin_amdgcn_alignbit(z1, z2, 4);
    z1 = __builtin_amdgcn_alignbit(z0, z1, 4);
    z0 = (z0 >> 4) ^ rem4v(rem);
    z0 ^= t[k].x; z1 ^= t[k].y; z2 ^= t[k].z; z3 ^= t[k].w;
  }
  __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);
#pragma unroll
  for (int k = 0; k < 24; k++) {
    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    __builtin_amdgcn_sched_group_barrier(0x002, 10, 0);
  }
  return U128{((uint64_t)z0 << 32) | z1, ((uint64_t)z2 << 32) | z3};
}

__device__ inline U128 shfl128(U128 v, uint32_t src) {
  const uint32_t a = __shfl((uint32_t)(v.hi >> 32), (int)src), b = __shfl((uint32_t)v.hi, (int)src);
  const uint32_t c = __shfl((uint32_t)(v.lo >> 32), (int)src), d = __shfl((uint32_t)v.lo, (int)src);
  return U128{((uint64_t)a << 32) | b, ((uint64_t)c << 32) | d};
}

// One wave per session (blockIdx.x = session index), the work of
// aead_aes_gcm_init / CRYPTO_gcm128_init (e_aes.c:1372-1413, gcm128.c:681-747)
// plus the tables of the batch kernels.  The latency of one install is the
// latency of EVP_AEAD_CTX_init and of a connection's key install, so it is
// written for latency: the S-box and the session header are built in LDS (no
// scratch memory, one 16-B store per lane), the key schedule and H = E_K(0)
// run on one lane from LDS, the seven squarings H^(2^k) and the per-lane powers
// H^e (lane e, square-and-multiply over them) use 4-bit products against
// Shoup tables shared in LDS.  Round 2 measured 104 us per install with
// global-memory S-box lookups, a scratch DevSession and bit-serial products.
__device__ __forceinline__ void install_body(DevSession* __restrict__ sessions,
                                             DevGcmTables* __restrict__ tables,
                                             const tlsgpu_session_params& p, uint32_t id);

__global__ __launch_bounds__(64) void install_sessions(DevSession* __restrict__ sessions,
                                                       DevGcmTables* __restrict__ tables,
                                                       const tlsgpu_session_params* __restrict__ params,
                                                       uint32_t first, uint32_t n) {
  if (blockIdx.x >= n) return;
  install_body(sessions, tables, params[blockIdx.x], first + blockIdx.x);
}

// One session with its parameters as a kernel argument (EVP_AEAD_CTX_init):
// no staging buffer and no copy, so the caller need not wait for the install
// before it reuses its memory (round 3, asynchronous context init).
__global__ __launch_bounds__(64) void install_session_arg(DevSession* __restrict__ sessions,
                                                          DevGcmTables* __restrict__ tables,
                                                          tlsgpu_session_params p, uint32_t id) {
  install_body(sessions, tables, p, id);
}

__device__ __forceinline__ void install_body(DevSession* __restrict__ sessions,
                                             DevGcmTables* __restrict__ tables,
                                             const tlsgpu_session_params& p, uint32_t id) {
  __shared__ __attribute__((aligned(16))) uint8_t sb[256];
  __shared__ uint32_t rk_be[60];
  __shared__ uint8_t hb[16];
  __shared__ uint4 hdr[sizeof(DevSession) / 16];
  __shared__ uint4 sqtab[7][16];  // Shoup tables of H^(2^k), k = 0..6
  const uint32_t lane = threadIdx.x;
  static_assert(sizeof(DevSession) / 16 == 64, "one 16-B chunk of the header per lane");
  reinterpret_cast<uint32_t*>(sb)[lane] = reinterpret_cast<const uint32_t*>(g_sbox.v)[lane];
  hdr[lane] = make_uint4(0, 0, 0, 0);
  const bool gcm = p.aead == TLSGPU_AES_128_GCM || p.aead == TLSGPU_AES_256_GCM;
  const bool cc = p.aead == TLSGPU_CHACHA20_POLY1305 || p.aead == TLSGPU_CHACHA20_POLY1305_OLD;
  const uint32_t want_key = p.aead == TLSGPU_AES_128_GCM ? 16 : 32;
  const uint32_t tag = p.tag_len == 0 ? 16 : p.tag_len;
  const bool valid = (gcm || cc) && p.key_len == want_key && tag <= 16 && p.fixed_iv_len <= 12;
  __syncthreads();
  DevSession& s = *reinterpret_cast<DevSession*>(hdr);
  uint32_t rounds = 0;
  if (valid && lane == 0) {  // header fields; kind stays 0 for an invalid slot
    s.kind = (uint32_t)p.aead;
    s.tag_len = tag;
    s.key_len = p.key_len;
    s.fixed_nonce_len = p.fixed_iv_len;
    s.xor_fixed_nonce = p.aead == TLSGPU_CHACHA20_POLY1305;
    s.nonce_in_record = gcm;
    s.version = p.version;
    for (uint32_t k = 0; k < p.fixed_iv_len; k++) s.fixed_nonce[k] = p.fixed_iv[k];
    if (cc)
      for (int k = 0; k < 32; k++) s.chacha_key[k] = p.key[k];
    if (gcm) {
      s.rounds = (uint32_t)expand_key(sb, p.key, (int)p.key_len, rk_be);
      for (int k = 0; k < 16; k++) hb[k] = 0;
      aes_encrypt_bytes(sb, rk_be, (int)s.rounds, hb);  // H = E_K(0^128)
    }
  }
  __syncthreads();
  if (valid && gcm) {
    rounds = s.rounds;
    if (lane < 4 * (rounds + 1)) {
      const uint32_t w = bswap32(rk_be[lane]);
      s.rk[lane] = w;
      s.rk_rot[lane] = __builtin_amdgcn_alignbit(w, w, 16);
    }
  }
  U128 H{0, 0};
  for (int k = 0; k < 8; k++) {
    H.hi = (H.hi << 8) | hb[k];
    H.lo = (H.lo << 8) | hb[8 + k];
  }
  if (valid && gcm && lane == 0) store_le(s.h_le, H);
  __syncthreads();
  reinterpret_cast<uint4*>(sessions + id)[lane] = hdr[lane];
  if (!valid || !gcm) return;

  DevGcmTables* t = &tables[id];
  // bitsliced AddRoundKey masks: (rounds + 1) x 128 words over the lanes
  for (uint32_t w = lane; w < 128u * (rounds + 1); w += 64) {
    const uint32_t r = w / 128, b = (w % 128) / 8, k = w % 8;
    t->bsrk[r][8 * b + k] = 0u - ((s.rk[4 * r + b / 4] >> (8 * (b % 4) + k)) & 1u);
  }
  // H^(lane + 1) by doubling (round 3): after level k, lanes [0, 2^(k+1))
  // hold their powers; level k multiplies lane (l - 2^k)'s power by H^(2^k)
  // for lanes l in [2^k, 2^(k+1)), against the Shoup table 16 lanes build from
  // lane 2^k - 1.  Seven products deep in all (round 2: seven squarings, then
  // up to five square-and-multiply products per lane).
  U128 pw = lane == 0 ? H : U128{0, 0};
  for (int k = 0; k < 6; k++) {
    const uint32_t step = 1u << k;
    const U128 b = shfl128(pw, step - 1);
    if (lane < 16) sqtab[k][lane] = be_words(shoup_entry(b, lane));
    __syncthreads();
    const U128 src = shfl128(pw, lane >= step ? lane - step : 0);
    if (lane >= step && lane < 2 * step) pw = gf_mul_tab(src, sqtab[k]);
  }
  // H^64 (lane 63): its table gives H^65 and the basis
  const U128 h64 = shfl128(pw, 63);
  if (lane < 16) sqtab[6][lane] = be_words(shoup_entry(h64, lane));
  __syncthreads();
  // Shoup tables of H^e: lane e - 1, and lane 0 for e = 65
  {
    U128 m[16];
    shoup_table(pw, m);
    for (int v = 0; v < 16; v++) *reinterpret_cast<uint4*>(t->shoup[lane][v]) = be_words(m[v]);
    if (lane == 0) {
      shoup_table(gf_mul_tab(H, sqtab[6]), m);
      for (int v = 0; v < 16; v++) *reinterpret_cast<uint4*>(t->shoup[kPowMax - 1][v]) = be_words(m[v]);
    }
  }
  // basis[q] = H^64 * x^q: the product of the one-hot x^q (bit q from the
  // MSB, gcm128.c's bit order) with H^64's table; lanes q and q + 64
  for (uint32_t q = lane; q < 128; q += 64) {
    const U128 xq = q < 64 ? U128{1ull << (63 - q), 0} : U128{0, 1ull << (127 - q)};
    store_le(t->basis[q], gf_mul_tab(xq, sqtab[6]));
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
// Also the batch's setup (one launch instead of three): every record's
// initial status (TLSGPU_REC_PUBLIC_INVALID, the status of a record no kernel
// takes, or TLSGPU_REC_OUT_OF_BOUNDS) and, from block 0, the zeroed control
// words of the queue kernels (ctl_words uint32s, may be 0).
__global__ void check_record_bounds(const tlsgpu_record* __restrict__ recs,
                                    tlsgpu_record* __restrict__ safe, uint32_t n,
                                    const DevSession* __restrict__ sessions, uint32_t n_sessions,
                                    uint64_t in_bytes, uint64_t out_bytes, int seal,
                                    int32_t* __restrict__ status, uint32_t* __restrict__ ctl,
                                    uint32_t ctl_words) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (blockIdx.x == 0)
    for (uint32_t w = threadIdx.x; w < ctl_words; w += blockDim.x) ctl[w] = 0;
  if (i >= n) return;
  tlsgpu_record r = recs[i];
  int32_t st = TLSGPU_REC_PUBLIC_INVALID;
  if (r.session < n_sessions) {
    const DevSession& S = sessions[r.session];
    const uint64_t eiv = S.nonce_in_record ? 8u : 0u, tag = S.tag_len;
    const uint64_t len = r.len_type & 0xFFFFFFu;
    const uint64_t in_len = len;
    const uint64_t out_len = seal ? len + eiv + tag : (len >= eiv + tag ? len - eiv - tag : 0);
    if (r.in_off > in_bytes || in_len > in_bytes - r.in_off || r.out_off > out_bytes ||
        out_len > out_bytes - r.out_off) {
      r.session = 0xFFFFFFFFu;
      st = TLSGPU_REC_OUT_OF_BOUNDS;
    }
  }
  status[i] = st;
  safe[i] = r;
}

int launch_check_bounds(const tlsgpu_record* recs, tlsgpu_record* safe, uint32_t n,
                        const DevSession* sessions, uint32_t n_sessions, uint64_t in_bytes,
                        uint64_t out_bytes, bool seal, int32_t* status, uint32_t* ctl,
                        uint32_t ctl_words, hipStream_t s) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(check_record_bounds, dim3((n + 255) / 256), dim3(256), 0, s, recs, safe, n,
                     sessions, n_sessions, in_bytes, out_bytes, seal ? 1 : 0, status, ctl,
                     ctl_words);
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

int launch_session_install_arg(DevSession* sessions, DevGcmTables* tables,
                               const tlsgpu_session_params& p, uint32_t id, hipStream_t s) {
  hipLaunchKernelGGL(install_session_arg, dim3(1), dim3(64), 0, s, sessions, tables, p, id);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// EVP_AEAD_CTX_init's install (round 5): the calling thread built the slot's
// image on the host (session_host.cpp) in its pinned key area; one 256-thread
// workgroup copies it into the slot (zero-copy reads of the pinned image), the
// GCM tables only when `table_bytes` != 0.  Kernel arguments carry pointers
// only — no key material.
__global__ __launch_bounds__(256) void upload_session(const uint4* __restrict__ img,
                                                      DevSession* __restrict__ sess,
                                                      DevGcmTables* __restrict__ tab,
                                                      uint32_t table_bytes) {
  constexpr uint32_t kS = sizeof(DevSession) / 16;
  const uint32_t n = kS + table_bytes / 16;
  for (uint32_t i = threadIdx.x; i < n; i += 256) {
    const uint4 v = img[i];
    if (i < kS) reinterpret_cast<uint4*>(sess)[i] = v;
    else reinterpret_cast<uint4*>(tab)[i - kS] = v;
  }
}

// EVP_AEAD_CTX_cleanup's scrub (e_aes.c:1415-1422 explicit_bzero analogue):
// the slot's DevSession and GCM tables zeroed in one launch.
__global__ __launch_bounds__(256) void scrub_session(DevSession* __restrict__ sess,
                                                     DevGcmTables* __restrict__ tab) {
  constexpr uint32_t kS = sizeof(DevSession) / 16, kT = sizeof(DevGcmTables) / 16;
  for (uint32_t i = threadIdx.x; i < kS + kT; i += 256) {
    if (i < kS) reinterpret_cast<uint4*>(sess)[i] = make_uint4(0, 0, 0, 0);
    else reinterpret_cast<uint4*>(tab)[i - kS] = make_uint4(0, 0, 0, 0);
  }
}

int launch_upload_session(const void* img, DevSession* sess, DevGcmTables* tab,
                          uint32_t table_bytes, hipStream_t s) {
  hipLaunchKernelGGL(upload_session, dim3(1), dim3(256), 0, s,
                     reinterpret_cast<const uint4*>(img), sess, tab, table_bytes);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_scrub_session(DevSession* sess, DevGcmTables* tab, hipStream_t s) {
  hipLaunchKernelGGL(scrub_session, dim3(1), dim3(256), 0, s, sess, tab);
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
