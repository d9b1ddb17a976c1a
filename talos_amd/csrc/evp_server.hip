// evp_server.hip — persistent "doorbell" server for synchronous per-call
// EVP_AEAD_CTX_seal/open jobs on AES-GCM and RFC 7539 ChaCha20-Poly1305
// contexts.
//
// A per-call job (e_aes.c:1424-1510 through evp_aead.c:89-144) is one record,
// latency-bound: launching a kernel and waiting for it costs 11-12 µs on this
// box before any cipher work (tools/hip_latency.hip).  With TLSGPU_EVP_DOORBELL
// set, up to G workgroups of this kernel stay resident (one per CU and per
// calling thread, the T-tables loaded into LDS once), each polling the
// doorbell slots of its calling threads in pinned host memory (slot k belongs
// to workgroup k % gridDim.x).  A posted job is the same RawJob the launched
// path builds in the thread's pinned staging; the workgroup runs it with the
// launched path's own code (gcm_raw_job, gcm_raw.h; cc_wave_job,
// chacha_wave.h on wave 0), writes output and status straight to the staging
// buffer and answers in the slot: no launch per call.  Per installed key the
// workgroup keeps the GHASH tables and the DevSession in LDS; a short GCM
// job's input is staged into LDS by idle waves while the first waves parse.
//
// Coherence: the kernel outlives any one job, so nothing may be served from a
// cache that a launch would have invalidated.  Session data is read with
// vector loads (TG_VECTOR_SESSION_LOADS: no scalar-cache copies of a slot's
// round keys survive the slot's re-keying), and each job starts behind one
// system-scope acquire fence on wave 0 (vector L1 invalidated) and a barrier.
// The answer is published by a system-scope release after every wave's
// stores have completed.
//
// Termination: every workgroup exits when the stop word is set or after
// `lifetime` ticks of the 100 MHz realtime counter (checked before every poll,
// so a busy workgroup leaves on time too), whichever is first; the
// host relaunches (engine.cpp EvpServer) so that a job is only ever posted
// while an instance that will poll for at least half a lifetime is queued.
#define TG_VECTOR_SESSION_LOADS 1
// job phase marks (TLSGPU_EVP_DOORBELL_TRACE): thread t (0: wave 0, lane 0)
// stamps the realtime clock into LDS; the server copies them to the slot's
// trace row
#define TG_JOB_MARK_AT(i, t)                                                    \
  do {                                                                          \
    if (threadIdx.x == (t))                                                     \
      reinterpret_cast<unsigned long long*>(::tg::s_lds + ::tg::SRV_MARK_OFF)[i] = \
          __builtin_amdgcn_s_memrealtime();                                     \
  } while (0)
#define TG_JOB_MARK(i) TG_JOB_MARK_AT(i, 0)
#include "gcm_device.h"
namespace tg {
constexpr uint32_t SRV_MARK_OFF = PLAN_OFF + 5120;  // 9 job marks (after the ChaCha stage)
constexpr uint32_t SRV_STAGE_OFF = PLAN_OFF + 1024;  // 4 KiB: a ChaCha job's stage, a GCM job's input
constexpr uint32_t kSrvStageMax = 4096;
constexpr uint32_t kSrvStageWave = 12;  // waves 12..15 copy (idle: a 4 KiB job has <= 4 ranges)
}
#define TG_JOB_STAGE 1
// the server issues a GCM job's input staging itself, before the job's
// install (round 6): the two PCIe reads then overlap
#define TG_JOB_STAGE_EARLY 1
namespace tg {
__device__ __forceinline__ bool tg_stage_ok(const RawJob* J) {
  const uint32_t n = J->in_len;
  return n != 0 && n <= kSrvStageMax && (J->in & 15) == 0;
}
// waves 12..15: 256 lanes x 16 B; the staging buffer rounds the input up to
// 16 B (engine.cpp gpu_call_impl), so a whole 16 B read stays inside it
__device__ __forceinline__ void tg_stage_issue(const RawJob* J, uint32_t wave, uint32_t lane) {
  if (wave < kSrvStageWave) return;
  const uint32_t off = 16 * ((wave - kSrvStageWave) * kWave + lane);
  if (off < J->in_len)
    *reinterpret_cast<uint4*>(s_lds + SRV_STAGE_OFF + off) =
        *reinterpret_cast<const uint4*>(reinterpret_cast<const uint8_t*>(J->in) + off);
}
__device__ __forceinline__ const uint8_t* tg_stage_src() { return s_lds + SRV_STAGE_OFF; }
}  // namespace tg
#include "gcm_raw.h"
#include "chacha_wave.h"

namespace tg {

constexpr uint32_t kSrvExit = 0xFFFFFFFFu;
constexpr uint32_t kSrvFlush = 0xFFFFFFFEu;  // zero this workgroup's key copies (a scrub elsewhere)
// DoorbellSlot::op beyond bit 0 (seal), bits 8-15 (10 / 14 AES rounds, 20
// ChaCha) and bit 16 (inline nonce / AAD) — engine.cpp writes the same bits
constexpr uint32_t kOpInstall = kDoorbellOpInstall;            // the image at inl[0..7] first
constexpr uint32_t kOpInstallTables = kDoorbellOpInstallTables;  // ... with its GCM tables
constexpr uint32_t kOpScrub = kDoorbellOpScrub;                  // zero the slot (bits 8-15)
constexpr uint32_t SRV_SEL_OFF = PLAN_OFF + 16 * 16;  // after gcm_raw_job's part_y words
static_assert(SRV_SEL_OFF + 4 <= PLAN_OFF + 272, "gcm_raw_job's E_K(J0) word follows");
constexpr uint32_t SRV_SLOT_OFF = PLAN_OFF + 512;     // LDS copy of the picked slot (256 B)
static_assert(PLAN_OFF + 288 <= SRV_SLOT_OFF, "server LDS plan");
static_assert(SRV_SLOT_OFF + sizeof(DoorbellSlot) <= SRV_STAGE_OFF, "server LDS plan");
static_assert(SRV_STAGE_OFF + 4096 <= SRV_MARK_OFF, "server LDS plan");
static_assert(SRV_MARK_OFF + 88 <= SRV_MARK_OFF + 128, "11 job marks before the session copy");
// the GCM job's DevSession, copied into LDS once per installed key: the job's
// session reads (kind, rounds, tag_len, round keys) are then LDS reads, not
// one dependent HBM round trip each (round-4 trace: parse + setup ≈ 2.3 µs)
constexpr uint32_t SRV_SESS_OFF = SRV_MARK_OFF + 128;
static_assert(SRV_SESS_OFF % 16 == 0 && SRV_SESS_OFF + sizeof(DevSession) <= LDS_BYTES,
              "server LDS plan");
// slot words the copy needs (DoorbellSlot layout, tlsgpu_internal.h)
constexpr int kSlotWordNSess = 3, kSlotWordKey = 4, kSlotWordSessions = 8,
              kSlotWordSid = (int)(offsetof(DoorbellSlot, job) + offsetof(RawJob, session)) / 4;
static_assert(offsetof(DoorbellSlot, n_sessions) == 4 * kSlotWordNSess &&
              offsetof(DoorbellSlot, key_id) == 4 * kSlotWordKey &&
              offsetof(DoorbellSlot, sessions) == 4 * kSlotWordSessions, "slot layout");

// A ChaCha20-Poly1305 (RFC 7539) job on wave 0 (chacha_wave.h); the session's
// kind word by a vector load (lane-varying address), as everything else here.
template <bool SEAL>
__device__ __forceinline__ void srv_chacha_job(const BatchArgs& a, const RawJob& j) {
  if (threadIdx.x >= kWave) return;
  const uint32_t sid = j.session;
  if (sid >= a.n_sessions) {
    if (threadIdx.x == 0) a.status[0] = TLSGPU_REC_PUBLIC_INVALID;
    return;
  }
  const DevSession* S = a.sessions + sid;
  const uint32_t kw = reinterpret_cast<const uint32_t*>(S)[threadIdx.x & 7];
  if (__builtin_amdgcn_readlane(kw, 0) != TLSGPU_CHACHA20_POLY1305) {
    if (threadIdx.x == 0) a.status[0] = TLSGPU_REC_PUBLIC_INVALID;
    return;
  }
  cc_wave_job<SEAL>(j, S, a.status, s_lds + SRV_STAGE_OFF);
}

// A draft ("old") ChaCha20-Poly1305 job on wave 0 (round 5, chacha_wave.h
// cc_wave_job_old); inl: the AAD sits in the LDS copy of the slot.
template <bool SEAL>
__device__ __forceinline__ void srv_chacha_old_job(const BatchArgs& a, const RawJob& j, bool inl) {
  if (threadIdx.x >= kWave) return;
  const uint32_t sid = j.session;
  if (sid >= a.n_sessions) {
    if (threadIdx.x == 0) a.status[0] = TLSGPU_REC_PUBLIC_INVALID;
    return;
  }
  const DevSession* S = a.sessions + sid;
  const uint32_t kw = reinterpret_cast<const uint32_t*>(S)[threadIdx.x & 7];
  if (__builtin_amdgcn_readlane(kw, 0) != TLSGPU_CHACHA20_POLY1305_OLD) {
    if (threadIdx.x == 0) a.status[0] = TLSGPU_REC_PUBLIC_INVALID;
    return;
  }
  cc_wave_job_old<SEAL>(j, S, a.status, !inl, s_lds + SRV_STAGE_OFF);
}

__device__ __forceinline__ uint32_t sys_load(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Leaving: every earlier store of this workgroup completed (the done flags
// were released job by job), then the launch number into exited[blockIdx.x].
__device__ __forceinline__ void srv_leave(const ServerArgs& s) {
  if (threadIdx.x == 0) {
    __atomic_thread_fence(__ATOMIC_RELEASE);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(s.exited + blockIdx.x, s.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// The 64 KiB GHASH byte-position table (KT_OFF) from its one-bit entries,
// already in place: load_session_tables' arithmetic, with basis entry
// x^(8j + 7 - k) read as T[1 << k][j].  Wave j builds byte position j; the
// one-bit entries are rewritten with the values they hold.
__device__ void build_kt_in_place() {
  const uint32_t bl = threadIdx.x & 63;
  const uint32_t j = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // 16 waves, 16 positions
  auto one_bit = [&](int k) {
    return *reinterpret_cast<const uint4*>(s_lds + KT_OFF + (1u << k) * 256 + j * 16);
  };
  uint32_t lo[4] = {0, 0, 0, 0};
#pragma unroll
  for (int k = 0; k < 6; k++) {  // bit k of the byte <-> x^(8j + 7 - k)
    const uint32_t msk = 0u - ((bl >> k) & 1u);
    const uint4 b = one_bit(k);
    lo[0] ^= b.x & msk; lo[1] ^= b.y & msk; lo[2] ^= b.z & msk; lo[3] ^= b.w & msk;
  }
  const uint4 b6 = one_bit(6), b7 = one_bit(7);
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): every one-bit read before any write
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int q = 0; q < 4; q++) {
    const uint32_t m6 = (q & 1) ? 0xFFFFFFFFu : 0u, m7 = (q & 2) ? 0xFFFFFFFFu : 0u;
    const uint4 v = make_uint4(lo[0] ^ (b6.x & m6) ^ (b7.x & m7), lo[1] ^ (b6.y & m6) ^ (b7.y & m7),
                               lo[2] ^ (b6.z & m6) ^ (b7.z & m7), lo[3] ^ (b6.w & m6) ^ (b7.w & m7));
    *reinterpret_cast<uint4*>(s_lds + KT_OFF + (bl + 64u * q) * 256 + j * 16) = v;
  }
}
static_assert(kThreads == 16 * kWave, "one wave per byte position");

__global__ __launch_bounds__(kThreads, 1) void evp_server_kernel(ServerArgs s) {
  // an instance that only starts after the stop word was set (queued behind
  // the one the process was using at exit) leaves at once
  if (__hip_atomic_load(s.stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0) {
    srv_leave(s);
    return;
  }
  fill_aes_lds<kThreads>();
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint32_t* sel = reinterpret_cast<uint32_t*>(s_lds + SRV_SEL_OFF);
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  // lane l of wave 0 watches slot blockIdx.x + l * gridDim.x; `served` is the
  // number it last answered (from the slot itself: an earlier instance may
  // have served it)
  const uint32_t mine = blockIdx.x + lane * gridDim.x;
  uint32_t served = 0;
  if (wave == 0 && mine < s.nslots) served = sys_load(&s.slots[mine].done);
  uint32_t cached_key = 0;  // key id whose GCM tables are in LDS (0: none)
  uint32_t sess_key = 0;    // wave 0: key id whose DevSession is at SRV_SESS_OFF
  unsigned long long t_pick = 0, t_loaded = 0;  // trace (wave 0)
  // Scrubs served by other workgroups (round 6): each scrub job
  // appends its key id to a ring in HBM; wave 0 reads the new entries before
  // each pick and every 16 polls, and when one names a key whose tables or
  // DevSession this workgroup holds in LDS, the workgroup zeroes them
  // (kSrvFlush).  A ring lapped since the last look flushes whatever is held.
  unsigned long long scrub_seen =
      __hip_atomic_load(s.scrubs, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  auto scrubbed_here = [&]() -> bool {  // wave 0, wave-uniform
    const unsigned long long top =
        __hip_atomic_load(s.scrubs, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    bool hit = false;
    while (scrub_seen < top) {
      const unsigned long long e = __hip_atomic_load(s.scrubs + 1 + scrub_seen % kScrubRing,
                                                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned long long tag = e >> 32;
      if (tag == (scrub_seen + 1) % (1ull << 32)) {
        const uint32_t key = (uint32_t)e;
        hit = hit || (key != 0 && (key == cached_key || key == sess_key));
        scrub_seen++;
      } else if (tag > (scrub_seen + 1) % (1ull << 32)) {  // lapped: flush what is held
        hit = hit || cached_key != 0 || sess_key != 0;
        scrub_seen = top;
      } else {
        break;  // the entry is still being written: look again next time
      }
    }
    return hit;
  };
  for (;;) {
    if (wave == 0) {
      uint32_t pick = scrubbed_here() ? kSrvFlush : kSrvExit;
      for (uint32_t polls = 0; pick == kSrvExit; polls++) {
        // the lifetime first, busy or not: a workgroup that kept serving past
        // it would hold the next instance (queued on the same stream) off the
        // GPU, and with it the slots of workgroups that had already exited
        if (__builtin_amdgcn_s_memrealtime() - t0 > s.lifetime) break;
        const bool ready = mine < s.nslots && sys_load(&s.slots[mine].post) != served;
        const unsigned long long m = __ballot(ready);
        if (m) {
          pick = blockIdx.x + (uint32_t)(__ffsll((long long)m) - 1) * gridDim.x;
          t_pick = __builtin_amdgcn_s_memrealtime();
          break;
        }
        // the stop word every 16 polls (each poll is a PCIe read), and the
        // scrub ring (HBM)
        if ((polls & 15) == 15) {
          if (sys_load(s.stop) != 0) break;
          if (scrubbed_here()) {
            pick = kSrvFlush;
            break;
          }
        }
        __builtin_amdgcn_s_sleep(1);
      }
      if (lane == 0) *sel = pick;
      if (pick == kSrvFlush) sess_key = 0;  // zeroed below by every wave
      if (pick != kSrvExit && pick != kSrvFlush) {
        // the whole slot in one wave load (the job, its nonce and AAD: no
        // further PCIe round trip for them) into LDS; inline nonce / AAD are
        // then addressed in that copy
        DoorbellSlot* sl = s.slots + pick;
        const uint32_t w = sys_load(reinterpret_cast<const uint32_t*>(sl) + lane);
        DoorbellSlot* c = reinterpret_cast<DoorbellSlot*>(s_lds + SRV_SLOT_OFF);
        reinterpret_cast<uint32_t*>(c)[lane] = w;
        const uint32_t opw = __shfl(w, 2);  // DoorbellSlot::op
        if (lane == 0 && (opw & (1u << 16))) {
          c->job.nonce = (uint64_t)(uintptr_t)&c->inl[0];
          c->job.aad = (uint64_t)(uintptr_t)&c->inl[c->job.nonce_len];
        }
        // the job's input (pinned host memory) and its session (HBM, installed
        // by another kernel) are read fresh after this
        __atomic_thread_fence(__ATOMIC_ACQUIRE);
        const uint32_t kop = (opw >> 8) & 0xFFu;
        const uint32_t sid = __builtin_amdgcn_readlane(w, kSlotWordSid);
        const uint32_t key = __builtin_amdgcn_readlane(w, kSlotWordKey);
        if (opw & kOpInstall) {
          // the context's image is installed below by every wave, which also
          // fills the LDS DevSession copy (a ChaCha image too: the copy then
          // holds no GCM key's session)
          sess_key = (kop == 10 || kop == 14) ? key : 0u;
        } else if (kop == kOpScrub) {
          sess_key = 0;  // the scrub below zeroes the LDS copy
        } else if ((kop == 10 || kop == 14) &&
                   sid < (uint32_t)__builtin_amdgcn_readlane(w, kSlotWordNSess) && key != 0 &&
                   key != sess_key) {
          const uint64_t sp = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane(w, kSlotWordSessions + 1) << 32) |
                              (uint32_t)__builtin_amdgcn_readlane(w, kSlotWordSessions);
          const uint4* src = reinterpret_cast<const uint4*>(sp) + (size_t)sid * (sizeof(DevSession) / 16);
          reinterpret_cast<uint4*>(s_lds + SRV_SESS_OFF)[lane] = src[lane];  // 64 x 16 B = 1 KiB
          sess_key = key;
        }
      }
      if (lane < 11) reinterpret_cast<unsigned long long*>(s_lds + SRV_MARK_OFF)[lane] = 0;
      __builtin_amdgcn_s_waitcnt(0);
      t_loaded = __builtin_amdgcn_s_memrealtime();
    }
    __syncthreads();
    const uint32_t k = __builtin_amdgcn_readfirstlane(*sel);
    if (k == kSrvExit) break;
    if (k == kSrvFlush) {  // the key copies a scrub on another workgroup named
      const uint4 z = make_uint4(0, 0, 0, 0);
      for (uint32_t i = threadIdx.x; i < (R4_OFF - KT_OFF) / 16; i += kThreads)
        if (KT_OFF + 16 * i < AES_OFF || KT_OFF + 16 * i >= SH_OFF)
          reinterpret_cast<uint4*>(s_lds + KT_OFF)[i] = z;
      if (threadIdx.x < sizeof(DevSession) / 16)
        reinterpret_cast<uint4*>(s_lds + SRV_SESS_OFF)[threadIdx.x] = z;
      cached_key = 0;
      if (threadIdx.x == 0)
        __hip_atomic_fetch_add(s.scrubs + 1 + kScrubRing, 1ull, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
      __syncthreads();
      continue;
    }
    DoorbellSlot* sl = s.slots + k;
    const DoorbellSlot* c = reinterpret_cast<const DoorbellSlot*>(s_lds + SRV_SLOT_OFF);
    const uint32_t post = __builtin_amdgcn_readfirstlane(c->post);
    const uint32_t op = __builtin_amdgcn_readfirstlane(c->op) & 0xFFFFu;
    BatchArgs a = {};
    a.sessions = reinterpret_cast<const DevSession*>(c->sessions);
    a.gcm_tables = reinterpret_cast<const DevGcmTables*>(c->gcm_tables);
    a.descs = &c->job;  // LDS, through a generic pointer
    a.status = reinterpret_cast<int32_t*>(c->status);
    a.n = 1;
    a.n_sessions = __builtin_amdgcn_readfirstlane(c->n_sessions);
    const uint32_t key = __builtin_amdgcn_readfirstlane(c->key_id);
    const uint32_t sid = __builtin_amdgcn_readfirstlane(c->job.session);
    if (((op >> 8) == 10 || (op >> 8) == 14) && sid < a.n_sessions && key != 0)  // GCM: LDS copy
      a.sessions = reinterpret_cast<const DevSession*>(s_lds + SRV_SESS_OFF) - sid;
    // a GCM job's input into LDS by waves 12-15 now (gcm_raw_job's staging,
    // TG_JOB_STAGE_EARLY): its PCIe read overlaps the install's
    if (((op >> 8) == 10 || (op >> 8) == 14) && tg_stage_ok(&c->job))
      tg_stage_issue(&c->job, wave, threadIdx.x & 63);
    if (c->op & kOpInstall) {
      // EVP_AEAD_CTX_init's deferred install (round 5, engine.cpp): the image
      // the host built (session_host.cpp) goes from pinned memory into the
      // slot in HBM, and the DevSession also into the LDS copy, before the job
      // reads either; the GCM tables only when bit 18 says the image has them
      const uint4* img = reinterpret_cast<const uint4*>(
          *reinterpret_cast<const unsigned long long*>(&c->inl[0]));
      uint4* dsess = reinterpret_cast<uint4*>(const_cast<DevSession*>(
          reinterpret_cast<const DevSession*>(c->sessions) + sid));
      uint4* dtab = reinterpret_cast<uint4*>(const_cast<DevGcmTables*>(
          reinterpret_cast<const DevGcmTables*>(c->gcm_tables) + sid));
      constexpr uint32_t kS = sizeof(DevSession) / 16;
      constexpr uint32_t kB = sizeof(DevGcmTables::basis) / 16;  // 128 basis entries
      const bool tables = (c->op & kOpInstallTables) != 0;
      // round 6: only what the tables are made of crosses PCIe — the
      // DevSession, the basis H^64 * x^q and each power's Shoup entry m[8] =
      // H^e (257 words instead of the image's 1,225) — and the workgroup
      // builds its LDS tables and the slot's HBM copy from them: the byte
      // table from the basis, each power's 16 Shoup entries from H^e by three
      // multiplications by x (the linear span of gcm128.c's gcm_init_4bit
      // table, session_host.cpp shoup_table).  The connection's first call
      // paid ~16 us for the whole image through HBM (profiles/r06b_*).
      // no scratch: basis entry q = H^64 x^q IS the byte table's entry for
      // the one-bit byte 1 << (7 - q % 8) at position q / 8, and H^e IS its
      // Shoup table's entry m[8]: phase 1 puts them there, phase 2 derives
      // the rest of both tables from them (rewriting those entries with the
      // same values)
      const uint32_t nw = kS + (tables ? kB + kPowMax : 0u);
      if (sid < a.n_sessions && threadIdx.x < nw) {
        const uint32_t i = threadIdx.x;
        const uint32_t src = i < kS + kB ? i : kS + kB + 16u * (i - kS - kB) + 8u;
        const uint4 v = img[src];
        if (i < kS) {
          dsess[i] = v;
          reinterpret_cast<uint4*>(s_lds + SRV_SESS_OFF)[i] = v;
        } else if (i < kS + kB) {
          const uint32_t q = i - kS;
          dtab[q] = v;
          *reinterpret_cast<uint4*>(s_lds + KT_OFF + (1u << (7 - (q & 7))) * 256 + (q >> 3) * 16) = v;
        } else {
          *reinterpret_cast<uint4*>(s_lds + sh_base(1 + (i - kS - kB)) + 8u * 256u) = v;
        }
      }
      static_assert(kS + kB + kPowMax <= kThreads, "one image word per thread");
      __syncthreads();  // the one-bit byte entries and the powers in LDS
      TG_JOB_MARK(9);
      if (tables && sid < a.n_sessions) {
        build_kt_in_place();
        // Shoup entry v of power e: m[v] = [v&8] y ^ [v&4] y.x ^ [v&2] y.x^2 ^
        // [v&1] y.x^3, BE words (x = a right shift in gcm128.c's bit order)
        for (uint32_t t = threadIdx.x; t < kPowMax * 16; t += kThreads) {
          const uint32_t e = t >> 4, vsel = t & 15u;
          const uint4 y = *reinterpret_cast<const uint4*>(s_lds + sh_base(1 + e) + 8u * 256u);
          uint32_t w[4] = {y.x, y.y, y.z, y.w}, m[4] = {0, 0, 0, 0};
#pragma unroll
          for (int k = 3; k >= 0; k--) {  // bit k of v <-> y.x^(3 - k)
            const uint32_t msk = 0u - ((vsel >> k) & 1u);
            m[0] ^= w[0] & msk; m[1] ^= w[1] & msk; m[2] ^= w[2] & msk; m[3] ^= w[3] & msk;
            const uint32_t carry = 0u - (w[3] & 1u);
            w[3] = (w[3] >> 1) | (w[2] << 31);
            w[2] = (w[2] >> 1) | (w[1] << 31);
            w[1] = (w[1] >> 1) | (w[0] << 31);
            w[0] = (w[0] >> 1) ^ (carry & 0xE1000000u);
          }
          const uint4 mv = make_uint4(m[0], m[1], m[2], m[3]);
          *reinterpret_cast<uint4*>(s_lds + sh_base(1 + e) + vsel * 256u) = mv;
          dtab[kB + t] = mv;
        }
        cached_key = key;  // this job's tables are in LDS: gcm_raw_job skips the load
      }
      // the slot's HBM copy reaches other readers through the job's release
      // (every wave's stores complete before `done`, below): no fence here
      __syncthreads();
      TG_JOB_MARK(10);
    }
    if (op >> 8 == kOpScrub) {
      // EVP_AEAD_CTX_cleanup (e_aes.c:1415-1422 explicit_bzero analogue): the
      // slot's DevSession and GCM tables zeroed in HBM, and this workgroup's
      // LDS copies of them when they are this key's
      uint4* dsess = reinterpret_cast<uint4*>(const_cast<DevSession*>(
          reinterpret_cast<const DevSession*>(c->sessions) + sid));
      uint4* dtab = reinterpret_cast<uint4*>(const_cast<DevGcmTables*>(
          reinterpret_cast<const DevGcmTables*>(c->gcm_tables) + sid));
      constexpr uint32_t kS = sizeof(DevSession) / 16, kT = sizeof(DevGcmTables) / 16;
      const uint4 z = make_uint4(0, 0, 0, 0);
      if (sid < a.n_sessions)
        for (uint32_t i = threadIdx.x; i < kS + kT; i += kThreads) {
          if (i < kS) dsess[i] = z;
          else dtab[i - kS] = z;
        }
      if (key != 0 && key == cached_key) {  // the byte table (64 KiB at KT_OFF) and Shoup copy
        for (uint32_t i = threadIdx.x; i < (R4_OFF - KT_OFF) / 16; i += kThreads)
          if (KT_OFF + 16 * i < AES_OFF || KT_OFF + 16 * i >= SH_OFF)
            reinterpret_cast<uint4*>(s_lds + KT_OFF)[i] = z;
        cached_key = 0;
      }
      if (threadIdx.x < kS) reinterpret_cast<uint4*>(s_lds + SRV_SESS_OFF)[threadIdx.x] = z;
      __syncthreads();
      if (threadIdx.x == 0) {
        a.status[0] = 0;
        if (key != 0) {  // the other workgroups' copies: the scrub ring
          const unsigned long long idx = __hip_atomic_fetch_add(
              s.scrubs, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(s.scrubs + 1 + idx % kScrubRing,
                             (((idx + 1) % (1ull << 32)) << 32) | key, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
        }
      }
    }
    const bool hit = key != 0 && key == cached_key;
    // the table cache is keyed only on a job that really loaded (or kept)
    // its session's tables; a job rejected by the session check before the
    // load leaves LDS without valid tables; a ChaCha job leaves
    // the GCM tables alone
    switch (op) {
      case 10 << 8: cached_key = gcm_raw_job<false, 10>(a, 0, hit) ? key : 0; break;
      case (10 << 8) | 1: cached_key = gcm_raw_job<true, 10>(a, 0, hit) ? key : 0; break;
      case 14 << 8: cached_key = gcm_raw_job<false, 14>(a, 0, hit) ? key : 0; break;
      case (14 << 8) | 1: cached_key = gcm_raw_job<true, 14>(a, 0, hit) ? key : 0; break;
      case 20 << 8: srv_chacha_job<false>(a, c->job); break;
      case (20 << 8) | 1: srv_chacha_job<true>(a, c->job); break;
      case 21 << 8: srv_chacha_old_job<false>(a, c->job, (c->op & (1u << 16)) != 0); break;
      case (21 << 8) | 1: srv_chacha_old_job<true>(a, c->job, (c->op & (1u << 16)) != 0); break;
      case kOpScrub << 8: break;  // done above
      default:  // not a job this server runs (the host never posts one)
        if (threadIdx.x == 0) a.status[0] = TLSGPU_REC_PUBLIC_INVALID;
        cached_key = 0;
        break;
    }
    // every wave's output stores complete, then one release publishes them;
    // the asm wait keeps the flag behind the write-back (MI355X_MICROARCH.md,
    // compiler hazard: hipcc drops the vmcnt wait after buffer_wbl2 here)
    const unsigned long long t_job = __builtin_amdgcn_s_memrealtime();
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    if (threadIdx.x == 0) {
      if (s.trace) {  // diagnostic: ordered before `done` by the release below
        unsigned long long* tr = s.trace + kTraceWords * (size_t)k;
        const unsigned long long* mk =
            reinterpret_cast<const unsigned long long*>(s_lds + SRV_MARK_OFF);
        __hip_atomic_store(tr + 0, t_pick, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(tr + 1, t_loaded, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        for (int i = 0; i < 7; i++)
          __hip_atomic_store(tr + 2 + i, mk[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(tr + 9, t_job, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(tr + 10, (unsigned long long)__builtin_amdgcn_s_memrealtime(),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(tr + 11, mk[7], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(tr + 12, mk[8], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(tr + 13, mk[9], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(tr + 14, mk[10], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
      __atomic_thread_fence(__ATOMIC_RELEASE);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(&sl->done, post, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if (wave == 0 && mine == k) served = post;
  }
  srv_leave(s);
}

int launch_evp_server(const ServerArgs& a, int groups, hipStream_t s) {
  hipLaunchKernelGGL(evp_server_kernel, dim3(groups), dim3(kThreads), 0, s, a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace tg
