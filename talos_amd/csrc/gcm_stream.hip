// gcm_stream.hip — streaming AES-GCM state machine on the GPU for the legacy
// EVP_CIPHER GCM surface (EVP_aes_{128,256}_gcm, crypto/evp/e_aes.c:715-1059),
// SURVEY.md §8f-4.  The EVP_AEAD / TLS paths seal whole records; EVP_CIPHER
// callers instead feed CRYPTO_gcm128_{setiv,aad,encrypt,decrypt,finish}
// (crypto/modes/gcm128.c:749-1521) piecewise, with partial blocks carried
// between calls (ares / mres).  This kernel keeps a GCM128_CONTEXT equivalent
// (modes_lcl.h:79-95) in device memory and runs a short program of such
// operations per launch in one 64-lane workgroup:
//   * byte-level prefixes, tails, AAD and IV hashing on lane 0 (exact gcm128.c
//     carry semantics);
//   * whole blocks on all lanes: counter blocks E_K(Yi + b) in parallel, GHASH
//     as 64 lane chains x <- x * H^64 + C_j (the running Xi joins C_0), each
//     weighted by H^(n - j_last) and XORed together.
// AES is the T-table cipher with Te0 staged in LDS; H-powers come from the
// session's Shoup tables (DevGcmTables::shoup, HBM).  Not a throughput path:
// the TLS record layer of LibreSSL 2.4.1 uses EVP_AEAD (s3_lib.c:1747-1749).
#include "aes_common.h"
#include "tlsgpu_internal.h"

namespace tg {

static __device__ const WordTable g_te0_s = kTe0;

__device__ __forceinline__ uint32_t rem4s(uint32_t r) {  // rem_4bit[r] >> 32 (gcm128.c:327-331)
  const uint32_t a = r ^ (r << 1) ^ (r << 2);
  return (r << 21) ^ (a << 26);
}

// Z = X * H^e, BE words (Shoup 4-bit, gcm128.c:333-393) from the HBM table
__device__ void gmul(const DevGcmTables* tab, uint32_t e, const uint32_t X[4], uint32_t Z[4]) {
  const uint32_t* T = &tab->shoup[e - 1][0][0];
  uint32_t z0 = 0, z1 = 0, z2 = 0, z3 = 0;
  for (int k = 0; k < 32; k++) {
    if (k) {
      const uint32_t rem = z3 & 0xF;
      z3 = __builtin_amdgcn_alignbit(z2, z3, 4);
      z2 = __builtin_amdgcn_alignbit(z1, z2, 4);
      z1 = __builtin_amdgcn_alignbit(z0, z1, 4);
      z0 = (z0 >> 4) ^ rem4s(rem);
    }
    const uint32_t nib = (X[3 - k / 8] >> (4 * (k % 8))) & 0xF;
    z0 ^= T[4 * nib]; z1 ^= T[4 * nib + 1]; z2 ^= T[4 * nib + 2]; z3 ^= T[4 * nib + 3];
  }
  Z[0] = z0; Z[1] = z1; Z[2] = z2; Z[3] = z3;
}

// E_K(block), 16 bytes as BE words in and out; T-table AES (aes_core.c:789-972)
// with the session's little-endian column round keys.
__device__ void aes_be(const uint32_t* te, const DevSession* S, const uint32_t in[4], uint32_t o[4]) {
  const uint32_t* rk = S->rk;
  const int R = (int)S->rounds;
  auto T0 = [&](uint32_t w, int b) { return te[(w >> (8 * b)) & 0xFF]; };
  auto T1 = [&](uint32_t w, int b) { return rotl32(te[(w >> (8 * b)) & 0xFF], 8); };
  auto SB = [&](uint32_t w, int b) { return (te[(w >> (8 * b)) & 0xFF] >> 8) & 0xFF; };
  uint32_t s[4];
  for (int c = 0; c < 4; c++) s[c] = bswap32(in[c]) ^ rk[c];
  for (int r = 1; r < R; r++) {
    uint32_t t[4];
    for (int c = 0; c < 4; c++)
      t[c] = T0(s[c], 0) ^ T1(s[(c + 1) & 3], 1) ^
             rotl32(T0(s[(c + 2) & 3], 2) ^ T1(s[(c + 3) & 3], 3), 16) ^ rk[4 * r + c];
    for (int c = 0; c < 4; c++) s[c] = t[c];
  }
  for (int c = 0; c < 4; c++)
    o[c] = bswap32((SB(s[c], 0) | (SB(s[(c + 1) & 3], 1) << 8) | (SB(s[(c + 2) & 3], 2) << 16) |
                    (SB(s[(c + 3) & 3], 3) << 24)) ^ rk[4 * R + c]);
}

__device__ __forceinline__ uint32_t getb(const uint32_t X[4], uint32_t i) {
  return (X[i >> 2] >> (24 - 8 * (i & 3))) & 0xFF;
}
__device__ __forceinline__ void xorb(uint32_t X[4], uint32_t i, uint32_t v) {
  X[i >> 2] ^= (v & 0xFF) << (24 - 8 * (i & 3));
}
__device__ __forceinline__ void load_be(const uint8_t* p, uint32_t X[4]) {
  for (int w = 0; w < 4; w++)
    X[w] = ((uint32_t)p[4 * w] << 24) | ((uint32_t)p[4 * w + 1] << 16) |
           ((uint32_t)p[4 * w + 2] << 8) | p[4 * w + 3];
}

__global__ __launch_bounds__(64) void gcm_stream_kernel(const DevSession* __restrict__ sessions,
                                                        const DevGcmTables* __restrict__ tables,
                                                        uint32_t session, GcmStream* __restrict__ st,
                                                        const GcmStreamOp* __restrict__ ops,
                                                        uint32_t nops) {
  __shared__ uint32_t te[256];
  __shared__ GcmStream g;
  __shared__ uint32_t xl[64][4];
  const uint32_t lane = threadIdx.x;
  for (uint32_t i = lane; i < 256; i += 64) te[i] = g_te0_s.v[i];
  if (lane == 0) g = *st;
  __syncthreads();
  const DevSession* S = sessions + session;
  const DevGcmTables* tab = tables + session;
  auto mulH = [&](uint32_t X[4]) { uint32_t z[4]; gmul(tab, 1, X, z); for (int w = 0; w < 4; w++) X[w] = z[w]; };
  for (uint32_t k = 0; k < nops; k++) {
    const GcmStreamOp op = ops[k];
    const uint8_t* in = reinterpret_cast<const uint8_t*>(op.in);
    uint8_t* out = reinterpret_cast<uint8_t*>(op.out);
    uint64_t len = op.len;
    if (op.kind == GCM_OP_SETIV) {  // CRYPTO_gcm128_setiv (gcm128.c:749-824)
      if (lane == 0) {
        for (int w = 0; w < 4; w++) g.Yi[w] = g.Xi[w] = 0;
        g.len_aad = g.len_data = 0;
        g.ares = g.mres = 0;
        uint32_t ctr;
        if (len == 12) {
          uint8_t b[16] = {};
          for (int i = 0; i < 12; i++) b[i] = in[i];
          b[15] = 1;
          load_be(b, g.Yi);
          ctr = 1;
        } else {
          uint64_t off = 0;
          for (; off + 16 <= len; off += 16) {
            for (uint32_t i = 0; i < 16; i++) xorb(g.Yi, i, in[off + i]);
            mulH(g.Yi);
          }
          if (off < len) {
            for (uint32_t i = 0; off + i < len; i++) xorb(g.Yi, i, in[off + i]);
            mulH(g.Yi);
          }
          const uint64_t bits = len << 3;
          g.Yi[2] ^= (uint32_t)(bits >> 32);
          g.Yi[3] ^= (uint32_t)bits;
          mulH(g.Yi);
          ctr = g.Yi[3];
        }
        aes_be(te, S, g.Yi, g.EK0);
        g.Yi[3] = ctr + 1;
        g.rc = 0;
      }
    } else if (op.kind == GCM_OP_AAD) {  // CRYPTO_gcm128_aad (gcm128.c:826-881)
      if (lane == 0) {
        g.rc = 0;
        const uint64_t alen = g.len_aad + len;
        if (g.len_data) {
          g.rc = -2;
        } else if (alen > (1ull << 61) || alen < len) {
          g.rc = -1;
        } else {
          g.len_aad = alen;
          uint32_t n = g.ares;
          uint64_t p = 0;
          bool done = false;
          if (n) {
            while (n && p < len) {
              xorb(g.Xi, n, in[p++]);
              n = (n + 1) % 16;
            }
            if (n == 0) mulH(g.Xi);
            else { g.ares = n; done = true; }
          }
          if (!done) {
            for (; p + 16 <= len; p += 16) {
              for (uint32_t i = 0; i < 16; i++) xorb(g.Xi, i, in[p + i]);
              mulH(g.Xi);
            }
            n = (uint32_t)(len - p);
            for (uint32_t i = 0; i < n; i++) xorb(g.Xi, i, in[p + i]);
            g.ares = n;
          }
        }
      }
    } else if (op.kind == GCM_OP_ENCRYPT || op.kind == GCM_OP_DECRYPT) {
      // CRYPTO_gcm128_encrypt / _decrypt (gcm128.c:883-1240)
      const bool enc = op.kind == GCM_OP_ENCRYPT;
      __shared__ uint64_t p0, nblk;
      __shared__ uint32_t ctr0;
      __shared__ int go;
      if (lane == 0) {
        g.rc = 0;
        go = 0;
        const uint64_t mlen = g.len_data + len;
        if (mlen > (1ull << 36) - 32 || mlen < len) {
          g.rc = -1;
        } else {
          g.len_data = mlen;
          if (g.ares) {  // first data finalizes GHASH(AAD)
            mulH(g.Xi);
            g.ares = 0;
          }
          uint32_t n = g.mres;
          uint64_t p = 0;
          if (n) {
            while (n && p < len) {
              const uint32_t v = in[p], c = v ^ getb(g.EKi, n);  // in may be out
              out[p] = (uint8_t)c;
              xorb(g.Xi, n, enc ? c : v);
              p++;
              n = (n + 1) % 16;
            }
            if (n == 0) mulH(g.Xi);
            else g.mres = n;
          }
          if (n == 0) {
            p0 = p;
            nblk = (len - p) / 16;
            ctr0 = g.Yi[3];
            go = 1;
          }
        }
      }
      __syncthreads();
      if (go) {
        // whole blocks: keystream and output on every lane; GHASH over the
        // ciphertext, so before the writes on decrypt (in place: out == in)
        // and after them on encrypt
        auto crypt = [&]() {
          for (uint64_t b = lane; b < nblk; b += 64) {
            uint32_t y[4] = {g.Yi[0], g.Yi[1], g.Yi[2], ctr0 + (uint32_t)b}, ks[4];
            aes_be(te, S, y, ks);
            const uint8_t* ip = in + p0 + 16 * b;
            uint8_t* opp = out + p0 + 16 * b;
            for (int i = 0; i < 16; i++) opp[i] = ip[i] ^ (uint8_t)(ks[i >> 2] >> (24 - 8 * (i & 3)));
          }
        };
        if (enc) {
          crypt();
          __syncthreads();
        }
        // GHASH: lane chains in H^64, the running Xi joined to block 0
        uint32_t x[4] = {0, 0, 0, 0};
        int64_t jlast = -1;
        for (uint64_t j = lane; j < nblk; j += 64) {
          uint32_t c[4];
          load_be((enc ? out : in) + p0 + 16 * j, c);
          if (j == 0)
            for (int w = 0; w < 4; w++) c[w] ^= g.Xi[w];
          if (jlast >= 0) {
            uint32_t z[4];
            gmul(tab, 64, x, z);
            for (int w = 0; w < 4; w++) x[w] = z[w];
          }
          for (int w = 0; w < 4; w++) x[w] ^= c[w];
          jlast = (int64_t)j;
        }
        if (jlast >= 0) {
          uint32_t z[4];
          gmul(tab, (uint32_t)(nblk - (uint64_t)jlast), x, z);
          for (int w = 0; w < 4; w++) x[w] = z[w];
        }
        for (int w = 0; w < 4; w++) xl[lane][w] = x[w];
        __syncthreads();
        if (!enc) {
          crypt();
          __syncthreads();
        }
        if (lane == 0) {
          if (nblk) {
            uint32_t acc[4] = {0, 0, 0, 0};
            for (int l = 0; l < 64; l++)
              for (int w = 0; w < 4; w++) acc[w] ^= xl[l][w];
            for (int w = 0; w < 4; w++) g.Xi[w] = acc[w];
          }
          uint32_t ctr = ctr0 + (uint32_t)nblk;
          uint64_t p = p0 + 16 * nblk;
          uint32_t n = 0;
          if (p < len) {  // partial tail: keystream block kept in EKi (mres)
            uint32_t y[4] = {g.Yi[0], g.Yi[1], g.Yi[2], ctr};
            aes_be(te, S, y, g.EKi);
            ctr++;
            for (; p < len; p++, n++) {
              const uint32_t v = in[p], c = v ^ getb(g.EKi, n);
              out[p] = (uint8_t)c;
              xorb(g.Xi, n, enc ? c : v);
            }
          }
          g.Yi[3] = ctr;
          g.mres = n;
        }
      }
    } else {  // GCM_OP_FINISH / GCM_OP_TAG: CRYPTO_gcm128_finish / _tag (gcm128.c:1477-1521)
      if (lane == 0) {
        if (g.mres || g.ares) mulH(g.Xi);
        const uint64_t ab = g.len_aad << 3, cb = g.len_data << 3;
        g.Xi[0] ^= (uint32_t)(ab >> 32);
        g.Xi[1] ^= (uint32_t)ab;
        g.Xi[2] ^= (uint32_t)(cb >> 32);
        g.Xi[3] ^= (uint32_t)cb;
        mulH(g.Xi);
        for (int w = 0; w < 4; w++) g.Xi[w] ^= g.EK0[w];
        if (op.kind == GCM_OP_TAG) {
          for (uint64_t i = 0; i < len && i < 16; i++) out[i] = (uint8_t)getb(g.Xi, (uint32_t)i);
          g.rc = 0;
        } else if (in && len <= 16) {
          uint32_t diff = 0;
          for (uint64_t i = 0; i < len; i++) diff |= getb(g.Xi, (uint32_t)i) ^ in[i];
          g.rc = diff ? 1 : 0;
        } else {
          g.rc = -1;
        }
      }
    }
    __syncthreads();
    if (g.rc != 0) break;  // a failed step ends the program (the caller reads rc)
  }
  if (lane == 0) *st = g;
}

int launch_gcm_stream(const DevSession* sessions, const DevGcmTables* tables, uint32_t session,
                      GcmStream* st, const GcmStreamOp* ops, uint32_t nops, hipStream_t s) {
  if (nops == 0) return 0;
  hipLaunchKernelGGL(gcm_stream_kernel, dim3(1), dim3(64), 0, s, sessions, tables, session, st, ops,
                     nops);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace tg
