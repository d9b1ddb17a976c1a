// tlsgpu_internal.h — layouts shared by the host engine (engine.cpp) and the
// HIP kernels (gcm_kernels.hip, chacha_kernels.hip, session_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstddef>

#include "../../include/tlsgpu.h"

namespace tg {

constexpr int kWave = 64;

// Device session header (one per session id, 1 KiB, in HBM).  Mirrors the
// per-direction state LibreSSL keeps in SSL_AEAD_CTX (ssl/ssl_locl.h:527-543)
// plus the expanded key material aead_aes_gcm_init / _chacha20_poly1305_init
// derive (e_aes.c:1372-1413, e_chacha20poly1305.c:52-79).
struct alignas(16) DevSession {
  uint32_t kind;              // enum tlsgpu_aead, 0 = empty slot
  uint32_t rounds;            // 10 / 14 (AES)
  uint32_t tag_len;           // 1..16
  uint32_t key_len;
  uint32_t fixed_nonce_len;   // 4 / 12 / 0
  uint32_t xor_fixed_nonce;   // ChaCha RFC 7905
  uint32_t nonce_in_record;   // GCM explicit nonce
  uint32_t version;           // TLS version for the AAD
  uint8_t fixed_nonce[16];
  uint32_t rk[60];            // AES round keys, little-endian column words
  uint8_t chacha_key[32];
  uint32_t h_le[4];           // H = E_K(0), little-endian words
  uint32_t rk_rot[60];        // rotr16(rk[i]): round keys pre-rotated for the
                              // xor3 + alignbit + xor3 column form
  uint32_t reserved[112];
};
static_assert(sizeof(DevSession) == 1024, "DevSession layout");

// Per-session GHASH tables (GCM sessions only), 16-B aligned, in HBM.
//   basis[p]      = K * x^p, K = H^64, p = 0..127 (little-endian words); a
//                   workgroup expands these into the 64 KiB byte-position table
//                   T[j][b] = (b at byte j) * K in LDS.
//   shoup[e-1][v] = v * H^e for nibble v (Shoup 4-bit, gcm128.c:255-324
//                   layout: v's MSB is x^0), e = 1..65, big-endian words.
//   bsrk[r][8b+k] = 0 or ~0: bit k of byte b of round key r, the AddRoundKey
//                   masks of the bitsliced AES path (bs_aes.h), read by s_load.
constexpr int kPowMax = 65;
struct alignas(16) DevGcmTables {
  uint32_t basis[128][4];
  uint32_t shoup[kPowMax][16][4];
  uint32_t bsrk[15][128];
};
static_assert(sizeof(DevGcmTables) == 2048 + kPowMax * 256 + 15 * 512, "DevGcmTables layout");

// Raw AEAD job: one EVP_AEAD_CTX_seal/open call (arbitrary nonce / AAD), used
// by the per-call drop-in path.  Pointers are device pointers.
struct RawJob {
  uint64_t in, out, nonce, aad;
  uint32_t in_len;     // open: ct||tag length ; seal: plaintext length
  uint32_t nonce_len;
  uint32_t aad_len;
  uint32_t session;
  uint64_t max_out;    // bytes zero-filled on failure
};

// Streaming GCM state of one EVP_CIPHER context (GCM128_CONTEXT,
// crypto/modes/modes_lcl.h:79-95), in device memory; byte strings as
// big-endian words.  Operated on by gcm_stream.hip.
struct alignas(16) GcmStream {
  uint32_t Yi[4], EKi[4], EK0[4], Xi[4];
  uint64_t len_aad, len_data;
  uint32_t mres, ares;
  int32_t rc;       // result of the program's last step (gcm128.c return values;
                    // FINISH: 0 tag equal, 1 differs, -1 no tag)
  uint32_t reserved;
};
enum GcmOpKind : uint32_t {
  GCM_OP_SETIV = 0, GCM_OP_AAD = 1, GCM_OP_ENCRYPT = 2, GCM_OP_DECRYPT = 3, GCM_OP_FINISH = 4,
  GCM_OP_TAG = 5
};
struct GcmStreamOp {
  uint32_t kind;    // GcmOpKind
  uint32_t reserved;
  uint64_t len;
  uint64_t in, out; // device pointers
};

// Kernel launch parameters for the GCM / ChaCha batch kernels.
// Global-address-space views of generic pointers.  Record pointers reach the
// kernels through descriptors, structs and lane shuffles, where the compiler
// loses their address space and emits FLAT loads/stores; a FLAT op counts in
// lgkmcnt as well as vmcnt, so every LDS wait (s_waitcnt lgkmcnt) would also
// wait for the in-flight prefetch loads.  Going through an integer keeps them
// global_load / global_store.
template <class T>
__device__ __forceinline__ const __attribute__((address_space(1))) T* gld(const void* p) {
  return (const __attribute__((address_space(1))) T*)(uintptr_t)p;
}
template <class T>
__device__ __forceinline__ __attribute__((address_space(1))) T* gst(void* p) {
  return (__attribute__((address_space(1))) T*)(uintptr_t)p;
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
// 16 B through a global-address-space pointer (p 16-B aligned)
__device__ __forceinline__ uint4 gload16(const void* p) {
  const u32x4 v = *gld<u32x4>(p);
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void gstore16(void* p, uint4 v) {
  u32x4 w;
  w.x = v.x; w.y = v.y; w.z = v.z; w.w = v.w;
  *gst<u32x4>(p) = w;
}

// A full 16-B block at any byte address with dword loads: the dwords that hold
// its bytes (each contains at least one byte of the block, so none crosses the
// buffer's last page) funnel-shifted into place.  TLS wire fragments sit 5 B
// past their headers, so in-place opens of wire buffers take this path.
__device__ __forceinline__ void load16_any(const uint8_t* p, uint32_t v[4]) {
  const uintptr_t a = (uintptr_t)p;
  const uint32_t sh = (uint32_t)a & 3u;
  const auto q = gld<uint32_t>((const void*)(a & ~(uintptr_t)3));
  const uint32_t w0 = q[0], w1 = q[1], w2 = q[2], w3 = q[3];
  const uint32_t w4 = sh ? q[4] : 0u;
  v[0] = __builtin_amdgcn_alignbyte(w1, w0, sh);
  v[1] = __builtin_amdgcn_alignbyte(w2, w1, sh);
  v[2] = __builtin_amdgcn_alignbyte(w3, w2, sh);
  v[3] = __builtin_amdgcn_alignbyte(w4, w3, sh);
}

// The first nb (1..16) bytes of a block at any byte address, zero past them:
// dword loads only where a byte below nb lies (a record's last piece may end
// at its buffer's last page).
__device__ __forceinline__ void load16_upto(const uint8_t* p, uint32_t nb, uint32_t v[4]) {
  const uintptr_t a = (uintptr_t)p;
  const uint32_t sh = (uint32_t)a & 3u;
  const auto q = gld<uint32_t>((const void*)(a & ~(uintptr_t)3));
  const uint32_t nd = (sh + nb + 3) >> 2;  // dwords holding bytes [0, nb): 1..5
  const uint32_t w0 = q[0], w1 = nd > 1 ? q[1] : 0u, w2 = nd > 2 ? q[2] : 0u;
  const uint32_t w3 = nd > 3 ? q[3] : 0u, w4 = nd > 4 ? q[4] : 0u;
  v[0] = __builtin_amdgcn_alignbyte(w1, w0, sh);
  v[1] = __builtin_amdgcn_alignbyte(w2, w1, sh);
  v[2] = __builtin_amdgcn_alignbyte(w3, w2, sh);
  v[3] = __builtin_amdgcn_alignbyte(w4, w3, sh);
}

// The matching store: whole dwords inside the block, 1-2 byte/short stores at
// its two ends (never a read-modify-write of a neighbour's bytes).
__device__ __forceinline__ void store16_any(uint8_t* p, const uint32_t o[4]) {
  const uintptr_t a = (uintptr_t)p;
  const uint32_t sh = (uint32_t)a & 3u;
  if (sh == 0) {
    const auto q = gst<uint32_t>(p);
    q[0] = o[0]; q[1] = o[1]; q[2] = o[2]; q[3] = o[3];
    return;
  }
  const auto q = gst<uint32_t>((void*)(a - sh));  // q[1..3] lie inside the block
  const auto b = gst<uint8_t>(p);
  const auto h = gst<uint16_t>(p);  // used at even byte offsets only
  q[1] = __builtin_amdgcn_alignbyte(o[1], o[0], 4 - sh);
  q[2] = __builtin_amdgcn_alignbyte(o[2], o[1], 4 - sh);
  q[3] = __builtin_amdgcn_alignbyte(o[3], o[2], 4 - sh);
  if (sh == 1) {
    b[0] = (uint8_t)o[0];
    gst<uint16_t>(p + 1)[0] = (uint16_t)(o[0] >> 8);
    b[15] = (uint8_t)(o[3] >> 24);
  } else if (sh == 2) {
    h[0] = (uint16_t)o[0];
    h[7] = (uint16_t)(o[3] >> 16);
  } else {
    b[0] = (uint8_t)o[0];
    gst<uint16_t>(p + 13)[0] = (uint16_t)(o[3] >> 8);
    b[15] = (uint8_t)(o[3] >> 24);
  }
}

struct BatchArgs {
  const DevSession* sessions;
  const DevGcmTables* gcm_tables;   // indexed by session id
  const void* descs;                // tlsgpu_record[] or RawJob[]
  uint32_t n;
  uint32_t records_per_group;       // contiguous range per workgroup
  const uint8_t* in;
  uint8_t* out;
  int32_t* status;
  uint32_t n_sessions;              // descriptors naming a session >= this are invalid
  uint32_t bs_reserve;              // hybrid kernel: a bitsliced wave takes a record pair
                                    // only while >= this many records of the run are left
  uint32_t hy_flags;                // hybrid kernel experiments (env TLSGPU_HY_FLAGS):
                                    // 1 = no bitsliced pairs, 2 = T-table waves idle,
                                    // 4 = bitsliced waves idle
  unsigned long long* dbg;          // phase timing (PhaseClock), normally null
  uint32_t bs16_min;                // queue kernel: non-zero = the no-pack variant runs with
                                    // 4 packed bitsliced waves, which take records of n >= this
                                    // (<= 16384, 16-B aligned; gcm_queue_b16.hip); 0 = never
  uint32_t pack;                    // queue kernel: short records of one session share a
                                    // wave (gcm_pack); 0 = off
  uint32_t* sel;                    // queue impl: 4 selection words of this key size, filled
                                    // by the prep pass: [0] a record can be packed, [1] session
                                    // runs (records whose session differs from the previous
                                    // record's), [2] records.  The queue kernel's no-pack / pack
                                    // variants and the per-wave-session kernel all launch; the
                                    // ones the words do not select return (null: queue no-pack)
  uint32_t pws;                     // per-wave-session kernel: 0 auto (runs shorter than
                                    // kPwsRun records on average), 1 never, 2 always
  uint32_t* wg_next;                // per-wave-session kernel: one record counter per workgroup
  uint32_t fused;                   // queue no-pack kernel (round 5): the bounds check, the
                                    // initial statuses and the per-record constants of the
                                    // workgroup's records run in its own prologue (no
                                    // check_record_bounds / gcm_prep_kernel launches); descs
                                    // are the caller's, checked against in_bytes / out_bytes
  uint64_t in_bytes, out_bytes;     // fused: sizes of the caller's in / out buffers
  const unsigned long long* cut_work;  // fused, non-null: the work of each count range
                                       // (range_work_kernel); each workgroup takes the
                                       // records between its two work cuts instead
  uint32_t cut_snap;                // cut_work: snap a cut to a session-run boundary within
                                    // cut_snap / 1024 of a share of the work (0: exact cuts)
  const uint2* pieces;              // fused, non-null: whole pieces (a session run inside
  const uint32_t* n_pieces;         // one count range) sorted by work, largest first; workgroup
                                    // w takes pieces m*G + (m even ? w : G-1-w) (piece_sort_kernel;
                                    // *n_pieces == 0: the count ranges)
  unsigned long long* wg_times;     // diagnostic (TLSGPU_WG_TIMES=1), normally null: per
                                    // workgroup {start, end (s_memrealtime), rlo, rhi}
};

// Work-balanced ranges (round 5): a record's work for the cut — its payload
// bytes plus a per-record cost (parse, J0 / tag, the GHASH finish: about a
// quarter of a 1 KiB record's time in the queue kernel).  Any positive weight
// gives a correct partition (each cut is computed the same way by the two
// workgroups that share it); this one balances the Zipf-length workload.
constexpr uint32_t kCutRecordWork = 256;
__host__ __device__ __forceinline__ uint64_t cut_work_of(uint32_t len_type) {
  return (uint64_t)(len_type & 0xFFFFFFu) + kCutRecordWork;
}

// Average session-run length below which the per-wave-session kernel (gcm_pw.hip)
// replaces the queue kernel: a run shorter than the workgroup's wave count leaves
// waves idle at the run barrier.
constexpr uint32_t kPwsRun = 12;
// Selection words of the prep pass per key size: kSelSlots slots of kSelWords
// words (one 64-B line each) = {packable flag, session-run starts, records};
// a workgroup adds into slot blockIdx % kSelSlots, readers sum the slots.
constexpr int kSelSlots = 16;
constexpr int kSelWords = 16;
__host__ __device__ __forceinline__ bool pws_selected(uint32_t mode, uint32_t runs, uint32_t recs) {
  return mode == 2 || (mode == 0 && runs * kPwsRun > recs);
}

// Per-record constants of the hybrid kernel (gcm_prep_kernel, one per record,
// 48 B in a stream-ordered scratch buffer; read back with s_load).  All in the
// little-endian column form of the T-table path (gcm_device.h rec_consts).
struct alignas(16) RecPre {
  uint32_t ek0[4];    // E_K(J0), the tag mask
  uint32_t k1a, k1b;  // counter-independent parts of round-1 columns 0, 1 (incl. rk1)
  uint32_t k2[4];     // round-2 constants of the T-table fast path
  uint32_t sb2[2];    // SubBytes of round-1 output columns 2, 3 (bitsliced round 2)
};
static_assert(sizeof(RecPre) == 48, "RecPre layout");

}  // namespace tg

// Kernel launchers (defined in the .hip files).
namespace tg {
int launch_gcm(const BatchArgs& a, bool seal, bool raw, int rounds, int groups,
               hipStream_t s);
int launch_gcm_split(const BatchArgs& a, bool seal, int rounds, hipStream_t s);
int launch_gcm_prep(const BatchArgs& a, RecPre* pre, bool seal, int rounds, hipStream_t s);
int launch_range_work(const BatchArgs& a, int groups, unsigned long long* out, hipStream_t s);
// Whole-piece balance (round 5): the pieces of every count range, then all of
// them sorted by work (gcm_queue.hip).  scratch: kPieceScratchBytes(groups).
constexpr uint32_t kPiecesPerRange = 16;  // more in one count range: no plan (count ranges)
constexpr uint32_t kMaxPieces = 4096;     // the sort's LDS capacity
__host__ __device__ constexpr size_t kPieceScratchBytes(uint32_t groups) {
  return (size_t)groups * kPiecesPerRange * 16 + (size_t)((groups + 3) & ~3u) * 4 +
         (size_t)groups * kPiecesPerRange * 8 + 256;
}
int launch_piece_plan(const BatchArgs& a, int groups, uint8_t* scratch, const uint2** pieces,
                      const uint32_t** n_pieces, hipStream_t s);
int launch_gcm_queue(const BatchArgs& a, const RecPre* pre, bool seal, int rounds, int groups,
                     hipStream_t s);
int launch_gcm_queue_b16(const BatchArgs& a, const RecPre* pre, bool seal, int rounds, int groups,
                         hipStream_t s);
int launch_gcm_pw(const BatchArgs& a, const RecPre* pre, bool seal, int rounds, int groups,
                  hipStream_t s);
int launch_gcm_stream(const DevSession* sessions, const DevGcmTables* tables, uint32_t session,
                      GcmStream* st, const GcmStreamOp* ops, uint32_t nops, hipStream_t s);
int launch_gcm_hy10(const BatchArgs& a, const RecPre* pre, bool seal, int bs_waves, int groups,
                    hipStream_t s);
int launch_gcm_fused10(const BatchArgs& a, const RecPre* pre, bool seal, int groups, hipStream_t s);
int launch_gcm_fused14(const BatchArgs& a, const RecPre* pre, bool seal, int groups, hipStream_t s);
int launch_gcm_hy14(const BatchArgs& a, const RecPre* pre, bool seal, int bs_waves, int groups,
                    hipStream_t s);
int launch_bs_ecb(const DevSession* sessions, uint32_t session, int rounds, const void* d_in,
                  void* d_out, uint32_t nblocks, hipStream_t s);
int launch_chacha(const BatchArgs& a, bool seal, bool raw, bool rfc, bool old, hipStream_t s);

// Doorbell slot of the persistent EVP server (evp_server.hip, engine.cpp): one
// per calling thread, in pinned host memory, 256 B.  The thread fills the job
// (the RawJob itself and, when they fit, its nonce and AAD inline), then
// stores `post` (its next job number); a server workgroup that sees post != the
// number it last served copies the slot into LDS with one wave load, runs the
// job (its input read from and its output and status written to the thread's
// pinned staging buffer, zero-copy) and stores `done` = post after the output
// and status are visible to the host.
struct alignas(256) DoorbellSlot {
  uint32_t post;        // host: number of the posted job (written last)
  uint32_t done;        // device: number of the last job finished
  uint32_t op;          // bit 0: seal; bits 8-15: AES rounds (10 / 14); bit 16:
                        // nonce (then AAD) inline in `inl`
  uint32_t n_sessions;  // capacity of the context's session table
  uint32_t key_id;      // unique per installed key (process-wide): a server
                        // workgroup keeps the GCM tables of the last key it
                        // served in LDS and skips reloading them for the same id
  uint32_t reserved;
  uint64_t status;      // device address of the job's int32 status
  uint64_t sessions;    // const DevSession* of the context's table
  uint64_t gcm_tables;  // const DevGcmTables*
  RawJob job;           // 56 B; job.nonce / job.aad ignored when inline
  uint8_t inl[152];     // inline nonce || AAD
};
static_assert(sizeof(RawJob) == 56, "RawJob layout");
static_assert(sizeof(DoorbellSlot) == 256 && offsetof(DoorbellSlot, job) == 48,
              "DoorbellSlot layout");
constexpr uint32_t kDoorbellInline = 152;
// DoorbellSlot::op bits beyond the job (evp_server.hip): install the session
// image whose device address is in inl[0..7] before the job (deferred
// EVP_AEAD_CTX_init), with its GCM tables; op code (bits 8-15) 30: scrub the slot
constexpr uint32_t kDoorbellOpInstall = 1u << 17;
constexpr uint32_t kDoorbellOpInstallTables = 1u << 18;
constexpr uint32_t kDoorbellOpScrub = 30;
struct ServerArgs {
  DoorbellSlot* slots;        // device view of the pinned slot array
  uint32_t nslots;
  const uint32_t* stop;       // pinned word: non-zero = exit now
  unsigned long long lifetime;  // s_memrealtime ticks (100 MHz) a workgroup serves at most
  uint32_t* exited;             // pinned [gridDim.x]: a workgroup stores `seq` here as it
                                // leaves (the host's exit drain waits on it, no HIP call)
  uint32_t seq;                 // this instance's launch number (from 1)
  unsigned long long* trace;    // null, or pinned [nslots][kTraceWords]: realtime at pick,
                                // slot loaded, GCM job marks 0..6, job done, answer
                                // released (TLSGPU_EVP_DOORBELL_TRACE)
  unsigned long long* scrubs;   // HBM [1 + kScrubRing + 1]: scrub count, the ring of
                                // scrubbed key ids ((index + 1) << 32 | key), flushes done
};
constexpr uint32_t kScrubRing = 256;
constexpr int kTraceWords = 16;  // + the last working wave's marks 7, 8 at [11], [12]
int launch_evp_server(const ServerArgs& a, int groups, hipStream_t s);
int launch_session_install_arg(DevSession* sessions, DevGcmTables* tables,
                               const tlsgpu_session_params& p, uint32_t id, hipStream_t s);
int launch_session_install(DevSession* sessions, DevGcmTables* tables,
                           const tlsgpu_session_params* d_params, uint32_t first,
                           uint32_t n, hipStream_t s);
int launch_wire_frame(const tlsgpu_wire_stream* streams, uint32_t n_streams, const uint8_t* wire,
                      const DevSession* sessions, uint32_t n_sessions, uint32_t max_records,
                      tlsgpu_record* recs, tlsgpu_wire_result* results, uint32_t* total,
                      hipStream_t s);
int launch_wire_seal_frame(const tlsgpu_write_stream* streams, uint32_t n_streams,
                           const DevSession* sessions, uint32_t n_sessions, uint8_t* wire,
                           uint64_t wire_bytes, uint32_t max_records, tlsgpu_record* recs,
                           tlsgpu_write_result* results, uint32_t* total, hipStream_t s);
int launch_wire_finish(uint32_t n_streams, tlsgpu_wire_result* results, int32_t* status,
                       hipStream_t s);
int launch_fill_synthetic(uint8_t* d_out, uint64_t stride, uint32_t span_len,
                          uint32_t n, uint64_t seed, uint64_t index0, hipStream_t s);
int launch_upload_session(const void* img, DevSession* sess, DevGcmTables* tab,
                          uint32_t table_bytes, hipStream_t s);
int launch_scrub_session(DevSession* sess, DevGcmTables* tab, hipStream_t s);
// GCM table bytes the default kernels read (basis + Shoup tables; the
// bitsliced masks only in the experimental build)
#ifdef TG_EXPERIMENTAL
constexpr uint32_t kGcmTableUploadBytes = sizeof(DevGcmTables);
#else
constexpr uint32_t kGcmTableUploadBytes = offsetof(DevGcmTables, bsrk);
#endif
// session_host.cpp: the image install_body writes, built on the host (the
// bitsliced masks only when a kernel of this build reads them)
bool host_crypto_ok();  // AES-NI + PCLMUL present: the host image can be built
bool host_session_image(const tlsgpu_session_params& p, DevSession* s, DevGcmTables* t,
                        bool bitsliced_masks = kGcmTableUploadBytes > offsetof(DevGcmTables, bsrk),
                        bool compact = false);
void host_image_complete(DevGcmTables* t);  // a compact image's Shoup entries
int launch_check_bounds(const tlsgpu_record* recs, tlsgpu_record* safe, uint32_t n,
                        const DevSession* sessions, uint32_t n_sessions, uint64_t in_bytes,
                        uint64_t out_bytes, bool seal, int32_t* status, uint32_t* ctl,
                        uint32_t ctl_words, hipStream_t s);
int launch_fill_synthetic_spans(uint8_t* d_out, const uint64_t* d_offs, const uint32_t* d_lens,
                                uint32_t n, uint64_t seed, uint64_t index0, hipStream_t s);
// TaLoS TLS-processing hooks (talos_hooks.cpp): is a callback registered, and
// fire it (the callback may change *len) — used by the host-delivery paths.
bool talos_read_hooked();
bool talos_write_hooked();
void talos_read(const void* ssl, uint8_t* data, uint32_t* len);
void talos_write(const void* ssl, uint8_t* data, uint32_t* len);

}  // namespace tg
