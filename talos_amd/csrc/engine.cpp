// engine.cpp — host side of libtlsgpu.so: the batch C ABI (include/tlsgpu.h)
// and the drop-in EVP_AEAD ABI (include/tlsgpu_evp.h).
//
// The EVP_AEAD functions keep LibreSSL 2.4.1's argument checks and error
// behaviour (crypto/evp/evp_aead.c:50-144, e_aes.c:1372-1510,
// e_chacha20poly1305.c:52-286): same return values, ERR queue entries when a
// LibreSSL libcrypto is present in the process (weak ERR_put_error), zero-fill
// of out[0..max_out_len) and *out_len = 0 on every failure.  The cipher work of
// each call runs on the GPU as a one-record "raw" batch; this library contains
// no CPU cipher path.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <unistd.h>
#include <climits>
#include <csignal>
#include <deque>
#include <execinfo.h>
#include <linux/futex.h>
#include <sched.h>
#include <sys/syscall.h>
#include <thread>
#include <vector>

#include "../../include/tlsgpu.h"
#include "../../include/tlsgpu_evp.h"
#include "tlsgpu_internal.h"

using namespace tg;

// ---------------------------------------------------------------------------
// error reporting
static thread_local char g_err[256] = "";

static int fail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}

#define HIPCHK(x)                                                              \
  do {                                                                         \
    hipError_t _e = (x);                                                       \
    if (_e != hipSuccess)                                                      \
      return fail(TLSGPU_EHIP, "%s: %s", #x, hipGetErrorString(_e));          \
  } while (0)

extern "C" const char* tlsgpu_last_error(void) { return g_err; }

// For group.cpp (same library, not exported): set the calling thread's
// tlsgpu_last_error, e.g. to a member worker's reason.
extern "C" int tg_internal_set_error(int code, const char* msg) {
  return fail(code, "%s", msg ? msg : "");
}

// ---------------------------------------------------------------------------
// engine / sessions
// Per-stream scratch for the per-record constants (RecPre) of the queue
// kernels: grow-only hipMalloc buffers, reused in stream order.  (The stream-
// ordered pool — hipMallocAsync — was measured to hand the queue kernel stale
// bytes on MI355X: ~20 % of seal batches in a loop of fresh batches read
// constants the prep kernel had not made visible; plain hipMalloc memory: 0 of
// 240.  See DESIGN.md §4.1.)
struct PreScratch {
  void* ptr = nullptr;
  size_t cap = 0;
};

// Host-resident pipeline state (tlsgpu_open_host): HBM mirrors of the host
// buffers (grow-only), a copy-in stream, `nstreams` compute streams and a
// copy-out stream, chained per chunk by events, so the host-to-device and
// device-to-host DMA engines each stream continuously.
struct HostPipe {
  std::mutex mu;
  unsigned nstreams = 2;
  size_t chunk_bytes = (size_t)32 << 20;
  std::vector<hipStream_t> streams;  // [0] copy in, [1] copy out, [2..] compute
  std::vector<hipEvent_t> events;    // 2 per chunk
  uint8_t *d_in = nullptr, *d_out = nullptr;
  tlsgpu_record* d_recs = nullptr;
  int32_t* d_status = nullptr;
  size_t cap_in = 0, cap_out = 0, cap_recs = 0, cap_status = 0;
};

struct tlsgpu_engine {
  int device;
  hipStream_t stream;
  int num_cus;
  std::mutex pre_mu;
  std::vector<std::pair<hipStream_t, PreScratch>> pre;  // few streams per engine
  HostPipe host;
};

// Scratch of at least `bytes` for stream s (enlarging waits for the stream's
// earlier work, which may still read the old buffer).
// TLSGPU_PRE_POOL=1 (diagnostic): take the scratch from the stream-ordered
// pool instead, as round 1 first did; tools/pool_probe.hip and DESIGN.md §4.1
// explain why that is wrong on MI355X.
static const bool g_pre_pool = [] {
  const char* v = getenv("TLSGPU_PRE_POOL");
  return v && *v == '1';
}();

static void* pre_scratch(tlsgpu_engine* e, hipStream_t s, size_t bytes) {
  std::lock_guard<std::mutex> g(e->pre_mu);
  PreScratch* ps = nullptr;
  for (auto& kv : e->pre)
    if (kv.first == s) ps = &kv.second;
  if (!ps) {
    e->pre.emplace_back(s, PreScratch{});
    ps = &e->pre.back().second;
  }
  if (ps->cap < bytes) {
    if (ps->ptr) {
      if (hipStreamSynchronize(s) != hipSuccess) return nullptr;
      (void)hipFree(ps->ptr);
      ps->ptr = nullptr;
      ps->cap = 0;
    }
    const size_t cap = std::max(bytes, (size_t)1 << 20);
    if (hipMalloc(&ps->ptr, cap) != hipSuccess) return nullptr;
    ps->cap = cap;
  }
  return ps->ptr;
}

struct tlsgpu_sessions {
  tlsgpu_engine* eng;
  uint32_t capacity;
  DevSession* d_sess;
  DevGcmTables* d_gcm;
  std::vector<int32_t> kinds;  // host mirror of installed kinds
  std::vector<uint8_t> tag_lens;  // and tag lengths (host pipeline output spans)
  std::vector<const void*> owners;  // SSL* per session for the TaLoS hooks (set_owner)
  bool have[5];                // any session of kind k installed
  std::atomic<unsigned> hints{0};  // TLSGPU_HINT_* (tlsgpu_sessions_hint)
  // EVP contexts: per-slot event of the slot's last install or scrub, so init
  // and cleanup need not wait on the device (created on a slot's first use)
  std::vector<hipEvent_t> slot_ev;
  std::mutex mu;               // host mirrors, when several threads install at once
};

extern "C" int tlsgpu_device_count(int* count) {
  if (!count) return fail(TLSGPU_EINVAL, "null out");
  *count = 0;
  HIPCHK(hipGetDeviceCount(count));
  return TLSGPU_OK;
}

extern "C" int tlsgpu_engine_create(int device, tlsgpu_engine** out) {
  if (!out) return fail(TLSGPU_EINVAL, "null out");
  *out = nullptr;
  int count = 0;
  HIPCHK(hipGetDeviceCount(&count));
  if (device < 0 || device >= count)
    return fail(TLSGPU_EINVAL, "device %d out of range (%d GPUs)", device, count);
  HIPCHK(hipSetDevice(device));
  auto* e = new (std::nothrow) tlsgpu_engine();
  if (!e) return fail(TLSGPU_ENOMEM, "engine alloc");
  e->device = device;
  HIPCHK(hipDeviceGetAttribute(&e->num_cus, hipDeviceAttributeMultiprocessorCount, device));
  HIPCHK(hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking));
  *out = e;
  return TLSGPU_OK;
}

extern "C" void tlsgpu_engine_destroy(tlsgpu_engine* e) {
  if (!e) return;
  (void)hipSetDevice(e->device);
  (void)hipStreamSynchronize(e->stream);
  (void)hipDeviceSynchronize();  // batches on user streams may still use the scratch
  for (auto& kv : e->pre) (void)hipFree(kv.second.ptr);
  for (hipStream_t hs : e->host.streams) (void)hipStreamDestroy(hs);  // host pipeline
  for (hipEvent_t ev : e->host.events) (void)hipEventDestroy(ev);
  (void)hipFree(e->host.d_in);
  (void)hipFree(e->host.d_out);
  (void)hipFree(e->host.d_recs);
  (void)hipFree(e->host.d_status);
  (void)hipStreamDestroy(e->stream);
  delete e;
}

extern "C" void* tlsgpu_engine_stream(tlsgpu_engine* e) { return e ? (void*)e->stream : nullptr; }

extern "C" int tlsgpu_engine_sync(tlsgpu_engine* e) {
  if (!e) return fail(TLSGPU_EINVAL, "null engine");
  HIPCHK(hipSetDevice(e->device));
  HIPCHK(hipStreamSynchronize(e->stream));
  return TLSGPU_OK;
}

extern "C" int tlsgpu_engine_num_cus(tlsgpu_engine* e) { return e ? e->num_cus : 0; }

extern "C" int tlsgpu_sessions_create(tlsgpu_engine* e, uint32_t capacity, tlsgpu_sessions** out) {
  if (!e || !out || capacity == 0) return fail(TLSGPU_EINVAL, "bad arguments");
  *out = nullptr;
  HIPCHK(hipSetDevice(e->device));
  auto* t = new (std::nothrow) tlsgpu_sessions();
  if (!t) return fail(TLSGPU_ENOMEM, "sessions alloc");
  t->eng = e;
  t->capacity = capacity;
  t->kinds.assign(capacity, 0);
  t->tag_lens.assign(capacity, 16);
  t->owners.assign(capacity, nullptr);
  memset(t->have, 0, sizeof(t->have));
  if (hipMalloc(&t->d_sess, sizeof(DevSession) * (size_t)capacity) != hipSuccess ||
      hipMalloc(&t->d_gcm, sizeof(DevGcmTables) * (size_t)capacity) != hipSuccess) {
    (void)hipFree(t->d_sess);
    delete t;
    return fail(TLSGPU_ENOMEM, "device session table (%u sessions)", capacity);
  }
  HIPCHK(hipMemsetAsync(t->d_sess, 0, sizeof(DevSession) * (size_t)capacity, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  *out = t;
  return TLSGPU_OK;
}

extern "C" void tlsgpu_sessions_destroy(tlsgpu_sessions* t) {
  if (!t) return;
  (void)hipSetDevice(t->eng->device);
  (void)hipStreamSynchronize(t->eng->stream);
  for (hipEvent_t ev : t->slot_ev)
    if (ev) {
      (void)hipEventSynchronize(ev);  // a scrub still running on a call stream
      (void)hipEventDestroy(ev);
    }
  (void)hipFree(t->d_sess);
  (void)hipFree(t->d_gcm);
  delete t;
}

static bool valid_params(const tlsgpu_session_params& p) {
  uint32_t tag = p.tag_len == 0 ? 16 : p.tag_len;
  if (tag > 16 || p.fixed_iv_len > 12) return false;
  switch (p.aead) {
    case TLSGPU_AES_128_GCM: return p.key_len == 16;
    case TLSGPU_AES_256_GCM:
    case TLSGPU_CHACHA20_POLY1305:
    case TLSGPU_CHACHA20_POLY1305_OLD: return p.key_len == 32;
  }
  return false;
}

extern "C" int tlsgpu_sessions_install(tlsgpu_sessions* t, uint32_t first, uint32_t n,
                                       const tlsgpu_session_params* params) {
  if (!t || (!params && n)) return fail(TLSGPU_EINVAL, "bad arguments");
  if ((uint64_t)first + n > t->capacity)
    return fail(TLSGPU_ERANGE, "sessions [%u, %u) exceed capacity %u", first, first + n,
                t->capacity);
  for (uint32_t i = 0; i < n; i++)
    if (!valid_params(params[i])) return fail(TLSGPU_EINVAL, "invalid session params at %u", i);
  if (n == 0) return TLSGPU_OK;
  HIPCHK(hipSetDevice(t->eng->device));
  tlsgpu_session_params* d_params = nullptr;
  HIPCHK(hipMalloc(&d_params, sizeof(tlsgpu_session_params) * n));
  hipError_t err = hipMemcpyAsync(d_params, params, sizeof(tlsgpu_session_params) * n,
                                  hipMemcpyHostToDevice, t->eng->stream);
  int rc = err == hipSuccess
               ? launch_session_install(t->d_sess, t->d_gcm, d_params, first, n, t->eng->stream)
               : -1;
  // the raw keys do not outlive the install in device memory
  (void)hipMemsetAsync(d_params, 0, sizeof(tlsgpu_session_params) * n, t->eng->stream);
  hipError_t serr = hipStreamSynchronize(t->eng->stream);
  (void)hipFree(d_params);
  if (err != hipSuccess || rc != 0 || serr != hipSuccess)
    return fail(TLSGPU_EHIP, "session install failed: %s",
                hipGetErrorString(err != hipSuccess ? err : serr));
  std::lock_guard<std::mutex> lk(t->mu);
  for (uint32_t i = 0; i < n; i++) {
    t->kinds[first + i] = params[i].aead;
    t->tag_lens[first + i] = (uint8_t)(params[i].tag_len ? params[i].tag_len : 16);
    t->have[params[i].aead] = true;
  }
  return TLSGPU_OK;
}

static int initial_gcm_impl() {
  const char* v = getenv("TLSGPU_GCM_IMPL");
  if (v && strcmp(v, "ttable") == 0) return TLSGPU_GCM_TTABLE;
  if (v && strcmp(v, "bitslice") == 0) return TLSGPU_GCM_BITSLICE;
  if (v && strcmp(v, "hybrid") == 0) return TLSGPU_GCM_HYBRID;
  if (v && strcmp(v, "fused") == 0) return TLSGPU_GCM_FUSED;
  if (v && strcmp(v, "queue") == 0) return TLSGPU_GCM_QUEUE;
  if (v && strcmp(v, "split") == 0) return TLSGPU_GCM_SPLIT;
  return TLSGPU_GCM_AUTO;
}
// The bitsliced / hybrid / fused GCM variants measured slower than the queue
// kernel; they are compiled only with `make EXPERIMENTAL=1`
// (-DTG_EXPERIMENTAL).  Without it, selecting them fails and the default stays.
#ifdef TG_EXPERIMENTAL
static constexpr bool kExperimental = true;
#else
static constexpr bool kExperimental = false;
#endif
static bool impl_built(int impl) {
  return impl == TLSGPU_GCM_QUEUE || impl == TLSGPU_GCM_TTABLE || impl == TLSGPU_GCM_SPLIT ||
         impl == TLSGPU_GCM_AUTO || kExperimental;
}
static std::atomic<int> g_gcm_impl{impl_built(initial_gcm_impl()) ? initial_gcm_impl()
                                                                 : (int)TLSGPU_GCM_AUTO};

extern "C" int tlsgpu_set_gcm_impl(int impl) {
  if (impl < TLSGPU_GCM_BITSLICE || impl > TLSGPU_GCM_AUTO)
    return fail(TLSGPU_EINVAL, "unknown gcm impl %d", impl);
  if (!impl_built(impl))
    return fail(TLSGPU_EINVAL, "gcm impl %d not built (make EXPERIMENTAL=1)", impl);
  g_gcm_impl.store(impl);
  return TLSGPU_OK;
}
extern "C" int tlsgpu_get_gcm_impl(void) { return g_gcm_impl.load(); }

extern "C" int tlsgpu_aes_ecb_bitsliced(tlsgpu_sessions* t, uint32_t session, const uint8_t* d_in,
                                        uint8_t* d_out, uint32_t nblocks, void* stream) {
  if (!t || (nblocks && (!d_in || !d_out))) return fail(TLSGPU_EINVAL, "bad arguments");
  if (session >= t->capacity ||
      (t->kinds[session] != TLSGPU_AES_128_GCM && t->kinds[session] != TLSGPU_AES_256_GCM))
    return fail(TLSGPU_EINVAL, "session %u is not an installed AES-GCM session", session);
#ifdef TG_EXPERIMENTAL
  HIPCHK(hipSetDevice(t->eng->device));
  int rounds = t->kinds[session] == TLSGPU_AES_128_GCM ? 10 : 14;
  if (launch_bs_ecb(t->d_sess, session, rounds, d_in, d_out, nblocks,
                    stream ? (hipStream_t)stream : t->eng->stream))
    return fail(TLSGPU_EHIP, "bs ecb launch: %s", hipGetErrorString(hipGetLastError()));
  return TLSGPU_OK;
#else
  (void)stream;
  return fail(TLSGPU_EINVAL, "bitsliced AES not built (make EXPERIMENTAL=1)");
#endif
}

// TLSGPU_WG_PER_CU (A/B): workgroups per CU.  Only one 16-wave workgroup fits
// a CU at a time (LDS), so k > 1 gives each CU k ranges in turn, handed out by
// the dispatcher as CUs free up: a CU that runs fast takes more of them.
static uint32_t wg_per_cu() {
  static const uint32_t v = [] {
    const char* e = getenv("TLSGPU_WG_PER_CU");
    const long k = e ? strtol(e, nullptr, 10) : 1;
    return (uint32_t)(k < 1 ? 1 : (k > 4 ? 4 : k));
  }();
  return v;
}
static int groups_for(const tlsgpu_engine* e, uint32_t n, uint32_t* per_group) {
  // one persistent 16-wave workgroup per CU, contiguous record ranges
  uint32_t groups = (uint32_t)e->num_cus * wg_per_cu();
  uint32_t min_per = 16;
  if ((uint64_t)groups * min_per > n) groups = (n + min_per - 1) / min_per;
  if (groups == 0) groups = 1;
  *per_group = (n + groups - 1) / groups;
  groups = (n + *per_group - 1) / *per_group;
  return (int)groups;
}

static uint32_t initial_bs_reserve() {
  const char* v = getenv("TLSGPU_BS_RESERVE");
  long r = v ? strtol(v, nullptr, 10) : 12;
  return (uint32_t)(r < 2 ? 2 : r);
}
static uint32_t g_bs_reserve = initial_bs_reserve();
// Diagnostic phase timing of the hybrid kernel (TLSGPU_PHASE_STATS=1): 32
// counters in device memory, read with tlsgpu_debug_phase_stats.
static unsigned long long* g_phase_stats = nullptr;
static int g_phase_stats_dev = -1;
extern "C" int tlsgpu_debug_phase_stats(tlsgpu_engine* e, unsigned long long* out32, int reset) {
  if (!e) return fail(TLSGPU_EINVAL, "null engine");
  HIPCHK(hipSetDevice(e->device));
  if (!g_phase_stats) {
    const char* v = getenv("TLSGPU_PHASE_STATS");
    if (!v || !*v || *v == '0') return fail(TLSGPU_EINVAL, "TLSGPU_PHASE_STATS not set");
    HIPCHK(hipMalloc((void**)&g_phase_stats, 64 * sizeof(unsigned long long)));
    HIPCHK(hipMemset(g_phase_stats, 0, 64 * sizeof(unsigned long long)));
    g_phase_stats_dev = e->device;
  }
  HIPCHK(hipDeviceSynchronize());
  if (out32) HIPCHK(hipMemcpy(out32, g_phase_stats, 32 * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  if (reset) HIPCHK(hipMemset(g_phase_stats, 0, 64 * sizeof(unsigned long long)));
  return TLSGPU_OK;
}

// Diagnostic per-workgroup timing of the queue kernel (TLSGPU_WG_TIMES=1):
// {start, end, rlo, rhi} of each workgroup of the last queue launch, read with
// tlsgpu_debug_wg_times (s_memrealtime ticks, 100 MHz).
static unsigned long long* g_wg_times = nullptr;
static int g_wg_times_dev = -1;  // the first engine's device only
static unsigned long long* wg_times_for(const tlsgpu_engine* e) {
  static const bool on = [] {
    const char* v = getenv("TLSGPU_WG_TIMES");
    return v && *v && *v != '0';
  }();
  if (!on) return nullptr;
  static std::mutex mu;
  std::lock_guard<std::mutex> lk(mu);
  if (!g_wg_times && hipMalloc((void**)&g_wg_times, 4 * 1024 * sizeof(unsigned long long)) == hipSuccess) {
    (void)hipMemset(g_wg_times, 0, 4 * 1024 * sizeof(unsigned long long));
    g_wg_times_dev = e->device;
  }
  return e->device == g_wg_times_dev ? g_wg_times : nullptr;
}
extern "C" int tlsgpu_debug_wg_times(tlsgpu_engine* e, unsigned long long* out, unsigned groups) {
  if (!e || !out || groups > 1024) return fail(TLSGPU_EINVAL, "bad arguments");
  if (!g_wg_times) return fail(TLSGPU_EINVAL, "TLSGPU_WG_TIMES not set");
  HIPCHK(hipSetDevice(e->device));
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(hipMemcpy(out, g_wg_times, 4 * (size_t)groups * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  return TLSGPU_OK;
}

// Hybrid-kernel experiment flags (TLSGPU_HY_FLAGS, tlsgpu_internal.h).  Bit 2
// parks the waves of gcm_hy_kernel that are not bitsliced-pair waves, bit 4 the
// bitsliced-pair waves.  A setting that parks every wave of the kernel that
// runs leaves every record of the batch unprocessed: round 2's
// gpurun_out/b16ab2 ("workload seal failed for 65536 records") ran the queue
// kernel, whose waves (T-table and packed-bitsliced role alike, BSW = 0) all
// obey bit 2.  Refused here: the park bits are dropped with a warning.
static uint32_t sane_hy_flags(uint32_t f, int impl) {
  const uint32_t parks = impl == TLSGPU_GCM_HYBRID ? 6u : impl == TLSGPU_GCM_BITSLICE ? 4u : 2u;
  if ((f & parks) == parks) {
    static std::once_flag warned;
    std::call_once(warned, [f] {
      fprintf(stderr, "libtlsgpu: TLSGPU_HY_FLAGS=%#x would park every wave; ignoring the "
                      "park bits\n", f);
    });
    return f & ~6u;
  }
  return f;
}
static uint32_t g_hy_flags = []() {
  const char* v = getenv("TLSGPU_HY_FLAGS");
  return v ? (uint32_t)strtoul(v, nullptr, 0) & 15u : 0u;
}();

// Queue kernel: records with n >= this take the packed bitsliced path
// (gcm_bs16.h); 0 = T-table only.  Env TLSGPU_BS16_MIN.
static uint32_t g_bs16_min = []() {
  const char* v = getenv("TLSGPU_BS16_MIN");
  return v ? (uint32_t)strtoul(v, nullptr, 0) : 0u;
}();

// Queue kernel: short-record packs (gcm_pack).  Env TLSGPU_PACK=0 turns them
// off, =1 keeps them on even when the caller hints NO_SHORT_RECORDS; unset
// (-1): on unless hinted off.
static int g_pack = []() {
  const char* v = getenv("TLSGPU_PACK");
  return v && *v ? (int)strtol(v, nullptr, 0) : -1;
}();

// Per-wave-session kernel (gcm_pw.hip): env TLSGPU_PWS=0 never, 1 always,
// unset = automatic (short session runs, tlsgpu_internal.h pws_selected).
static uint32_t g_pws = []() {
  const char* v = getenv("TLSGPU_PWS");
  if (!v || !*v) return 0u;
  return *v == '0' ? 1u : 2u;
}();

static const bool g_fused = [] {
  const char* v = getenv("TLSGPU_FUSED");
  return !(v && *v == '0');
}();
// Work-balanced ranges for the fused kernel (round 5, TLSGPU_BALANCE): 0 off
// (the default), 1 the pack variant (mixed record lengths), 2 always.  Equal
// record counts per workgroup leave the Zipf workload's slowest CU with 16 %
// more bytes than the mean, but a cut inside a session run costs both of its
// workgroups a table build, a plan and a run-end wait, and config D measured
// no faster with equal-work cuts.
static const uint32_t g_balance = [] {
  const char* v = getenv("TLSGPU_BALANCE");
  return v && *v ? (uint32_t)strtoul(v, nullptr, 10) : 0u;
}();
// Whole-piece balance (round 5, TLSGPU_PIECES): 0 off, 1 the pack variant
// (mixed record lengths; the default), 2 always — each workgroup takes whole
// pieces (a session run inside one count range) from a list sorted by work,
// in snake order (gcm_queue.hip piece_sort_kernel), instead of its count
// range: config D +1.4 % same-box, B (uniform records) −1 % (the two plan
// launches), DESIGN.md §4.1c.
static const uint32_t g_pieces = [] {
  const char* v = getenv("TLSGPU_PIECES");
  return v && *v ? (uint32_t)strtoul(v, nullptr, 10) : 1u;
}();
// ... and how near a session-run boundary a cut snaps to it, in 1/1024 of a
// workgroup's share of the work (TLSGPU_BALANCE_SNAP; 0: exact cuts)
static const uint32_t g_balance_snap = [] {
  const char* v = getenv("TLSGPU_BALANCE_SNAP");
  return v && *v ? (uint32_t)strtoul(v, nullptr, 10) : 0u;
}();

// bounds: {in_bytes, out_bytes} of a caller's TLS batch (checked by a pre-pass
// that hands the kernels a sanitized copy of the descriptors), or null for
// descriptors the engine built itself (raw EVP jobs, wire framing).
struct Bounds {
  uint64_t in_bytes, out_bytes;
};

// `kinds`: bit k set = the batch may hold records of AEAD kind k (a kernel is
// launched only for kinds that are installed AND in the mask; the EVP queue
// passes the kinds its jobs use).
static int run_batch(tlsgpu_sessions* t, const void* d_descs, uint32_t n, const uint8_t* d_in,
                     uint8_t* d_out, int32_t* d_status, hipStream_t s, bool seal, bool raw,
                     const Bounds* bounds = nullptr, unsigned kinds = ~0u,
                     unsigned hints = ~0u) {
  if (hints == ~0u) hints = t->hints.load(std::memory_order_relaxed);
  bool have[5];
  for (int k = 0; k < 5; k++) have[k] = t->have[k] && ((kinds >> k) & 1u);
  BatchArgs a = {};
  a.sessions = t->d_sess;
  a.gcm_tables = t->d_gcm;
  a.descs = d_descs;
  a.n = n;
  a.in = d_in;
  a.out = d_out;
  a.status = d_status;
  a.n_sessions = t->capacity;
  a.bs_reserve = g_bs_reserve;

  a.dbg = g_phase_stats;
  a.wg_times = wg_times_for(t->eng);
  a.bs16_min = g_bs16_min;
  // batch-shape hints rule out the kernels the device would not select
  // (tlsgpu_sessions_hint); the TLSGPU_PACK / TLSGPU_PWS overrides win
  a.pack = g_pack >= 0 ? (uint32_t)g_pack : (hints & TLSGPU_HINT_NO_SHORT_RECORDS) ? 0u : 1u;
  a.pws = (g_pws == 0 && (hints & TLSGPU_HINT_SESSION_RUNS)) ? 1u : g_pws;
  int groups = groups_for(t->eng, n, &a.records_per_group);
  const int sel_impl = g_gcm_impl.load();
  // small TLS batches (at most two records per CU): one record per workgroup,
  // its blocks split over the 16 waves, instead of one wave per record
  // (measured crossover, 16 KiB records: split 47 vs 77 us at 512 records,
  // 93 vs 81 us at 1,024)
  const bool split = !raw && (sel_impl == TLSGPU_GCM_SPLIT ||
                              (sel_impl == TLSGPU_GCM_AUTO && n <= 2u * (uint32_t)t->eng->num_cus));
  if (raw || split) {
    // raw EVP jobs: latency, not throughput — one workgroup per job, so a
    // batch of jobs on different contexts runs side by side instead of one
    // session run (table rebuild) after another inside one workgroup
    a.records_per_group = 1;
    groups = (int)n;
  }
  const int impl = raw ? TLSGPU_GCM_TTABLE
                       : split ? TLSGPU_GCM_SPLIT
                       : sel_impl == TLSGPU_GCM_AUTO ? TLSGPU_GCM_QUEUE : sel_impl;
  a.hy_flags = sane_hy_flags(g_hy_flags, impl);
  const bool gcm_pre = impl != TLSGPU_GCM_TTABLE && impl != TLSGPU_GCM_SPLIT &&
                       (have[TLSGPU_AES_128_GCM] || have[TLSGPU_AES_256_GCM]);
  // Fused (round 5): one queue kernel is the batch's only kernel — one AES key
  // size installed, no ChaCha, the hints rule out the per-wave-session kernel,
  // and they decide the variant (TLSGPU_HINT_NO_SHORT_RECORDS: no-pack, else
  // the pack variant, which also runs long records) — so it checks bounds,
  // writes the initial statuses and computes the per-record constants of its
  // own records in its prologue: no check_record_bounds, no gcm_prep_kernel, no
  // checked-descriptor copy, no variant that exits at once (TLSGPU_FUSED=0
  // keeps the launch sequence with the device-side selection).
  const bool fused_gcm = g_fused && bounds && impl == TLSGPU_GCM_QUEUE && a.pws == 1 &&
                         (have[TLSGPU_AES_128_GCM] != have[TLSGPU_AES_256_GCM]) &&
                         !have[TLSGPU_CHACHA20_POLY1305] && !have[TLSGPU_CHACHA20_POLY1305_OLD];
  // ... and the same for a batch of RFC 7539 ChaCha sessions only: the staged
  // ChaCha kernel checks bounds and writes the statuses of the records it does
  // not run itself (chacha_kernels.hip cc_tls_wave)
  const bool fused_cc = g_fused && bounds && !raw && have[TLSGPU_CHACHA20_POLY1305] &&
                        !have[TLSGPU_CHACHA20_POLY1305_OLD] && !have[TLSGPU_AES_128_GCM] &&
                        !have[TLSGPU_AES_256_GCM];
  const bool fused = fused_gcm || fused_cc;
  // per-stream scratch: [RecPre x n (queue kernels) | ctl_bytes control words |
  // checked descriptors x n].  Control words per key size k (0: AES-128, 1:
  // AES-256): selection words (kSelSlots x 64 B) at 1024 k, then one uint32
  // record counter per workgroup of the per-wave-session kernel at
  // 2048 + k * cnt_bytes, sized from the grid (any CU count).
  static_assert(kSelSlots * kSelWords * 4 <= 1024, "selection words exceed their slot");
  const size_t cnt_bytes = ((size_t)groups * 4 + 255) & ~(size_t)255;
  const size_t ctl_bytes = 2048 + 2 * cnt_bytes;
  const bool balance = fused_gcm && groups > 1 && groups <= 1024 &&
                       (g_balance >= 2 || (g_balance == 1 && a.pack != 0));
  const bool pieces = fused_gcm && !balance && groups > 1 && groups <= 1024 &&
                      (g_pieces >= 2 || (g_pieces == 1 && a.pack != 0));
  const size_t cut_bytes = balance  ? ((size_t)groups * 8 + 255) & ~(size_t)255
                           : pieces ? ((kPieceScratchBytes((uint32_t)groups) + 255) & ~(size_t)255) + 256
                                    : 0;
  const size_t pre_bytes =
      gcm_pre ? sizeof(RecPre) * (size_t)n + (fused ? cut_bytes : ctl_bytes) : 0;
  uint8_t* scratch = nullptr;
  uint8_t* pool_scratch = nullptr;
  if (pre_bytes || (bounds && !fused)) {
    const size_t sbytes = pre_bytes + (bounds && !fused ? sizeof(tlsgpu_record) * (size_t)n : 0);
    if (g_pre_pool) {  // diagnostic only (DESIGN.md §4.1 pool scratch): stream-ordered pool
      if (hipMallocAsync((void**)&scratch, sbytes, s) != hipSuccess) scratch = nullptr;
      pool_scratch = scratch;
    } else {
      scratch = (uint8_t*)pre_scratch(t->eng, s, sbytes);
    }
    if (!scratch) return fail(TLSGPU_ENOMEM, "batch scratch (%u records)", n);
  }
  RecPre* pre = nullptr;  // per-record constants of the queue kernels (per-stream scratch)
  uint8_t* ctl = nullptr;
  if (gcm_pre) {
    pre = reinterpret_cast<RecPre*>(scratch);
    ctl = fused ? nullptr : reinterpret_cast<uint8_t*>(pre + n);
  }
  uint8_t* const ctl_zero = impl == TLSGPU_GCM_QUEUE ? ctl : nullptr;
  if (fused) {
    a.fused = 1;
    a.in_bytes = bounds->in_bytes;
    a.out_bytes = bounds->out_bytes;
    if (balance) {  // each count range's work, then the kernel cuts at equal work
      auto* cw = reinterpret_cast<unsigned long long*>(pre + n);
      if (launch_range_work(a, groups, cw, s))
        return fail(TLSGPU_EHIP, "range work launch: %s", hipGetErrorString(hipGetLastError()));
      a.cut_work = cw;
      a.cut_snap = g_balance_snap;
    } else if (pieces) {  // whole pieces sorted by work
      uint8_t* ps = reinterpret_cast<uint8_t*>(pre + n);
      ps += (256 - ((uintptr_t)ps & 255)) & 255;
      if (launch_piece_plan(a, groups, ps, &a.pieces, &a.n_pieces, s))
        return fail(TLSGPU_EHIP, "piece plan launch: %s", hipGetErrorString(hipGetLastError()));
    }
  } else if (bounds) {
    // one setup launch: sanitized descriptors, every record's initial status
    // (records whose session is empty / invalid keep TLSGPU_REC_PUBLIC_INVALID)
    // and the zeroed control words
    auto* safe = reinterpret_cast<tlsgpu_record*>(scratch + pre_bytes);
    if (launch_check_bounds(reinterpret_cast<const tlsgpu_record*>(d_descs), safe, n, t->d_sess,
                            t->capacity, bounds->in_bytes, bounds->out_bytes, seal, d_status,
                            reinterpret_cast<uint32_t*>(ctl_zero),
                            ctl_zero ? (uint32_t)(ctl_bytes / 4) : 0u, s))
      return fail(TLSGPU_EHIP, "bounds launch: %s", hipGetErrorString(hipGetLastError()));
    a.descs = safe;
  } else {
    // records whose session is empty / invalid keep this status (raw EVP
    // jobs: the raw kernels write it themselves, so a queue batch launches no
    // fill kernel — round 2 measured ~18 K of them per queue run)
    if (!raw) HIPCHK(hipMemsetD32Async((hipDeviceptr_t)d_status, (int)TLSGPU_REC_PUBLIC_INVALID, n, s));
    if (ctl_zero) HIPCHK(hipMemsetAsync(ctl_zero, 0, ctl_bytes, s));
  }
  for (int rounds : {10, 14}) {
    if (!have[rounds == 10 ? TLSGPU_AES_128_GCM : TLSGPU_AES_256_GCM]) continue;
    // selection words and counters per key size: a short AES-128 record must
    // not send the AES-256 pass to the pack variant
    if (ctl && impl == TLSGPU_GCM_QUEUE) {
      const int k = rounds == 10 ? 0 : 1;
      a.sel = reinterpret_cast<uint32_t*>(ctl + 1024 * k);
      a.wg_next = reinterpret_cast<uint32_t*>(ctl + 2048 + cnt_bytes * k);
    }
    int rc;
    if (impl == TLSGPU_GCM_TTABLE) {
      rc = launch_gcm(a, seal, raw, rounds, groups, s);
    } else if (impl == TLSGPU_GCM_SPLIT) {
      rc = launch_gcm_split(a, seal, rounds, s);
    } else {
      rc = fused ? 0 : launch_gcm_prep(a, pre, seal, rounds, s);
      if (rc == 0) {
        if (impl == TLSGPU_GCM_QUEUE)
          rc = launch_gcm_queue(a, pre, seal, rounds, groups, s);
#ifdef TG_EXPERIMENTAL
        else if (impl == TLSGPU_GCM_FUSED)
          rc = (rounds == 10 ? launch_gcm_fused10 : launch_gcm_fused14)(a, pre, seal, groups, s);
        else
          rc = (rounds == 10 ? launch_gcm_hy10 : launch_gcm_hy14)(
              a, pre, seal, impl == TLSGPU_GCM_HYBRID ? 4 : 8, groups, s);
#else
        else
          rc = -1;
#endif
      }
    }
    if (rc) {
      return fail(TLSGPU_EHIP, "gcm-%d launch: %s", rounds == 10 ? 128 : 256,
                  hipGetErrorString(hipGetLastError()));
    }
  }
  if ((have[TLSGPU_CHACHA20_POLY1305] || have[TLSGPU_CHACHA20_POLY1305_OLD]) &&
      launch_chacha(a, seal, raw, have[TLSGPU_CHACHA20_POLY1305],
                    have[TLSGPU_CHACHA20_POLY1305_OLD], s))
    return fail(TLSGPU_EHIP, "chacha launch: %s", hipGetErrorString(hipGetLastError()));
  if (pool_scratch) HIPCHK(hipFreeAsync(pool_scratch, s));
  return TLSGPU_OK;
}

extern "C" int tlsgpu_sessions_hint(tlsgpu_sessions* t, unsigned hints) {
  if (!t || (hints & ~(TLSGPU_HINT_NO_SHORT_RECORDS | TLSGPU_HINT_SESSION_RUNS)))
    return fail(TLSGPU_EINVAL, "bad arguments");
  t->hints.store(hints, std::memory_order_relaxed);
  return TLSGPU_OK;
}

extern "C" int tlsgpu_open_batch(tlsgpu_sessions* t, const tlsgpu_record* d_recs, uint32_t n,
                                 const uint8_t* d_in, size_t in_bytes, uint8_t* d_out,
                                 size_t out_bytes, int32_t* d_status, void* stream) {
  if (!t || (n && (!d_recs || !d_in || !d_out || !d_status)))
    return fail(TLSGPU_EINVAL, "bad arguments");
  if (n == 0) return TLSGPU_OK;
  HIPCHK(hipSetDevice(t->eng->device));
  const Bounds b = {in_bytes, out_bytes};
  return run_batch(t, d_recs, n, d_in, d_out, d_status,
                   stream ? (hipStream_t)stream : t->eng->stream, false, false, &b);
}

extern "C" int tlsgpu_seal_batch(tlsgpu_sessions* t, const tlsgpu_record* d_recs, uint32_t n,
                                 const uint8_t* d_in, size_t in_bytes, uint8_t* d_out,
                                 size_t out_bytes, int32_t* d_status, void* stream) {
  if (!t || (n && (!d_recs || !d_in || !d_out || !d_status)))
    return fail(TLSGPU_EINVAL, "bad arguments");
  if (n == 0) return TLSGPU_OK;
  HIPCHK(hipSetDevice(t->eng->device));
  const Bounds b = {in_bytes, out_bytes};
  return run_batch(t, d_recs, n, d_in, d_out, d_status,
                   stream ? (hipStream_t)stream : t->eng->stream, true, false, &b);
}

// grow-only device buffer
static bool grow(void** p, size_t* cap, size_t want) {
  if (*cap >= want) return true;
  if (*p) (void)hipFree(*p);
  *p = nullptr;
  *cap = 0;
  if (hipMalloc(p, want ? want : 1) != hipSuccess) return false;
  *cap = want;
  return true;
}

extern "C" int tlsgpu_host_pipeline(tlsgpu_engine* e, unsigned streams, size_t chunk_bytes) {
  if (!e || streams > 8) return fail(TLSGPU_EINVAL, "bad arguments");
  std::lock_guard<std::mutex> lk(e->host.mu);
  if (streams) e->host.nstreams = streams;
  if (chunk_bytes) e->host.chunk_bytes = chunk_bytes;
  return TLSGPU_OK;
}

// Test hook (TLSGPU_TEST_HOST_FAIL_CHUNK=k): the host pipeline fails right
// after queueing chunk k's copy in, with earlier chunks still in flight.
static const long g_host_fail_chunk = [] {
  const char* v = getenv("TLSGPU_TEST_HOST_FAIL_CHUNK");
  return v && *v ? strtol(v, nullptr, 10) : -1L;
}();

// The host-resident pipeline for both directions (tlsgpu_open_host /
// tlsgpu_seal_host).  Open: in = record fragments, out = plaintext; seal: in =
// plaintext, out = fragments.  The TaLoS plaintext hooks run on the host
// plaintext: after the batch for reads, before its first copy for writes.
// The batch-shape hints of a host-resident slice (tlsgpu_sessions_hint): no
// record short enough for a pack (GCM n <= 992 B, the open length with the
// explicit nonce and the longest tag), and session runs long enough for the
// run-at-a-time queue kernel (pws_selected: runs * kPwsRun <= records).
static unsigned host_hints(const tlsgpu_record* r, uint32_t n, bool seal) {
  const uint32_t short_max = seal ? 992u : 992u + 8u + 16u;
  bool shorts = false;
  uint32_t runs = 0;
  for (uint32_t i = 0; i < n; i++) {
    shorts |= (r[i].len_type & 0xFFFFFFu) <= short_max;
    runs += (i == 0 || r[i].session != r[i - 1].session) ? 1u : 0u;
  }
  return (shorts ? 0u : TLSGPU_HINT_NO_SHORT_RECORDS) |
         ((uint64_t)runs * kPwsRun <= n ? TLSGPU_HINT_SESSION_RUNS : 0u);
}

static int host_batch(tlsgpu_sessions* t, bool seal, const tlsgpu_record* h_recs, uint32_t n,
                      const uint8_t* h_in, size_t in_bytes, uint8_t* h_out, size_t out_bytes,
                      int32_t* h_status) {
  if (!t || (n && (!h_recs || !h_in || !h_out || !h_status)))
    return fail(TLSGPU_EINVAL, "bad arguments");
  if (n == 0) return TLSGPU_OK;
  tlsgpu_engine* e = t->eng;
  HostPipe& hp = e->host;
  std::lock_guard<std::mutex> lk(hp.mu);
  HIPCHK(hipSetDevice(e->device));
  // TaLoS tls_processing_ssl_write (do_ssl3_write, s3_pkt.c.patch:19-33): on
  // each record's host plaintext before it goes to the device, in record
  // order; the module may rewrite the bytes and shorten the record (then a
  // private copy of the descriptors carries the new length)
  std::vector<tlsgpu_record> hooked;
  if (seal && talos_write_hooked()) {
    for (uint32_t i = 0; i < n; i++) {
      const uint32_t len = h_recs[i].len_type & 0xFFFFFFu;
      if (h_recs[i].session >= t->capacity || h_recs[i].in_off > in_bytes ||
          len > in_bytes - h_recs[i].in_off)
        continue;  // the bounds pass rejects it
      uint32_t hl = len;
      talos_write(t->owners[h_recs[i].session], const_cast<uint8_t*>(h_in) + h_recs[i].in_off,
                  &hl);
      if (hl < len) {
        if (hooked.empty()) hooked.assign(h_recs, h_recs + n);
        hooked[i].len_type = (hooked[i].len_type & 0xFF000000u) | hl;
      }
    }
    if (!hooked.empty()) h_recs = hooked.data();
  }
  const bool in_place = h_out == h_in;
  if (in_place) out_bytes = in_bytes;
  while (hp.streams.size() < 2 + hp.nstreams) {
    hipStream_t hs;
    HIPCHK(hipStreamCreateWithFlags(&hs, hipStreamNonBlocking));
    hp.streams.push_back(hs);
  }
  if (!grow((void**)&hp.d_in, &hp.cap_in, in_bytes) ||
      (!in_place && !grow((void**)&hp.d_out, &hp.cap_out, out_bytes)) ||
      !grow((void**)&hp.d_status, &hp.cap_status, sizeof(int32_t) * (size_t)n) ||
      !grow((void**)&hp.d_recs, &hp.cap_recs, sizeof(tlsgpu_record) * (size_t)n))
    return fail(TLSGPU_ENOMEM, "host pipeline buffers (%zu + %zu bytes)", in_bytes, out_bytes);
  uint8_t* d_in = hp.d_in;
  uint8_t* d_out = in_place ? hp.d_in : hp.d_out;
  // per-record spans (clamped to the buffers; the bounds pre-pass rejects the rest)
  auto span_in = [&](const tlsgpu_record& r, uint64_t* lo, uint64_t* hi) {
    *lo = std::min<uint64_t>(r.in_off, in_bytes);
    *hi = std::min<uint64_t>(r.in_off + (r.len_type & 0xFFFFFFu), in_bytes);
  };
  // the output span exactly (open: the plaintext, explicit nonce and tag
  // excluded; seal: the fragment): a neighbouring chunk's D2H on another stream
  // may own the next byte
  auto span_out = [&](const tlsgpu_record& r, uint64_t* lo, uint64_t* hi) {
    const uint64_t len = r.len_type & 0xFFFFFFu;
    uint64_t over = 0;
    if (r.session < t->capacity) {
      const int k = t->kinds[r.session];
      over = (k == TLSGPU_AES_128_GCM || k == TLSGPU_AES_256_GCM ? 8 : 0) + t->tag_lens[r.session];
    }
    *lo = std::min<uint64_t>(r.out_off, out_bytes);
    *hi = std::min<uint64_t>(r.out_off + (seal ? len + over : (len > over ? len - over : 0)),
                             out_bytes);
  };
  // chunks of ~chunk_bytes input when the layout ascends, else one chunk
  bool ascending = true;
  for (uint32_t i = 1; i < n && ascending; i++)
    ascending = h_recs[i].in_off >= h_recs[i - 1].in_off &&
                h_recs[i].out_off >= h_recs[i - 1].out_off;
  // chunk sizes ramp up from 1 MiB and back down at the end, so the pipeline
  // fills and drains on small transfers
  std::vector<uint32_t> cuts{0};
  if (ascending) {
    uint64_t total = 0;
    for (uint32_t i = 0; i < n; i++) total += h_recs[i].len_type & 0xFFFFFFu;
    uint64_t acc = 0, done = 0, target = std::min<uint64_t>(hp.chunk_bytes, 1u << 20);
    for (uint32_t i = 0; i < n; i++) {
      const uint64_t l = h_recs[i].len_type & 0xFFFFFFu;
      acc += l;
      done += l;
      if (acc >= target && i + 1 < n) {
        cuts.push_back(i + 1);
        acc = 0;
        const uint64_t left = total - done;
        target = std::min<uint64_t>({(uint64_t)hp.chunk_bytes, 2 * target,
                                     std::max<uint64_t>(left / 2, 1u << 20)});
      }
    }
  }
  cuts.push_back(n);
  const size_t nchunks = cuts.size() - 1;
  while (hp.events.size() < 2 * nchunks) {
    hipEvent_t ev;
    HIPCHK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    hp.events.push_back(ev);
  }
  hipStream_t s_in = hp.streams[0], s_out = hp.streams[1];
  const size_t ncomp = hp.streams.size() - 2;
  // Everything below is asynchronous on the pipeline streams; whatever fails,
  // the streams are drained before returning, so no copy into or out of the
  // caller's buffers is still running once the call has returned.
  auto issue = [&]() -> int {
    // all descriptors in one copy ahead of the first chunk, all statuses in one after the last
    HIPCHK(hipMemcpyAsync(hp.d_recs, h_recs, sizeof(tlsgpu_record) * (size_t)n,
                          hipMemcpyHostToDevice, s_in));
    for (size_t k = 0; k < nchunks; k++) {
      const uint32_t a = cuts[k], b = cuts[k + 1];
      hipStream_t hs = hp.streams[2 + k % ncomp];
      hipEvent_t ev_in = hp.events[2 * k], ev_done = hp.events[2 * k + 1];
      uint64_t ilo = UINT64_MAX, ihi = 0, olo = UINT64_MAX, ohi = 0;
      for (uint32_t i = a; i < b; i++) {
        uint64_t l, h;
        span_in(h_recs[i], &l, &h);
        ilo = std::min(ilo, l);
        ihi = std::max(ihi, h);
        span_out(h_recs[i], &l, &h);
        olo = std::min(olo, l);
        ohi = std::max(ohi, h);
      }
      if (!ascending) {  // one chunk: the whole buffers
        ilo = 0; ihi = in_bytes; olo = 0; ohi = out_bytes;
      }
      // copy in (DMA engine 1) -> kernels (compute stream) -> copy out (DMA engine 2)
      if (ihi > ilo)
        HIPCHK(hipMemcpyAsync(d_in + ilo, h_in + ilo, ihi - ilo, hipMemcpyHostToDevice, s_in));
      if ((long)k == g_host_fail_chunk)  // test hook: a failure with earlier chunks in flight
        return fail(TLSGPU_EHIP, "injected host pipeline failure at chunk %zu", k);
      HIPCHK(hipEventRecord(ev_in, s_in));
      HIPCHK(hipStreamWaitEvent(hs, ev_in, 0));
      // out of place, the HBM mirror is reused across calls: clear the range
      // copied back, so bytes between the records' output spans come back as
      // zeros, never as an earlier call's plaintext (in place, the whole range
      // was just copied in from h_in)
      if (!in_place && ohi > olo) HIPCHK(hipMemsetAsync(d_out + olo, 0, ohi - olo, hs));
      const Bounds bd = {in_bytes, out_bytes};
      const int rc = run_batch(t, hp.d_recs + a, b - a, d_in, d_out, hp.d_status + a, hs, seal,
                               false, &bd, ~0u, host_hints(h_recs + a, b - a, seal));
      if (rc != TLSGPU_OK) return rc;
      HIPCHK(hipEventRecord(ev_done, hs));
      HIPCHK(hipStreamWaitEvent(s_out, ev_done, 0));
      if (ohi > olo)
        HIPCHK(hipMemcpyAsync(h_out + olo, d_out + olo, ohi - olo, hipMemcpyDeviceToHost, s_out));
    }
    HIPCHK(hipMemcpyAsync(h_status, hp.d_status, sizeof(int32_t) * (size_t)n,
                          hipMemcpyDeviceToHost, s_out));
    return TLSGPU_OK;
  };
  int rc = issue();
  for (hipStream_t hs : hp.streams) {  // drain on success and on every failure
    const hipError_t e = hipStreamSynchronize(hs);
    if (e != hipSuccess && rc == TLSGPU_OK)
      rc = fail(TLSGPU_EHIP, "host pipeline sync: %s", hipGetErrorString(e));
  }
  if (rc != TLSGPU_OK) return rc;
  // TaLoS tls_processing_ssl_read (ssl3_read_bytes, s3_pkt.c.patch:39-52): on
  // each delivered record's plaintext in h_out, in record order; a module that
  // shortens it shortens what is delivered (h_status)
  if (!seal && talos_read_hooked()) {
    for (uint32_t i = 0; i < n; i++) {
      if (h_status[i] < 0) continue;
      uint32_t hl = (uint32_t)h_status[i];
      talos_read(t->owners[h_recs[i].session], h_out + h_recs[i].out_off, &hl);
      if (hl < (uint32_t)h_status[i]) h_status[i] = (int32_t)hl;
    }
  }
  return TLSGPU_OK;
}

extern "C" int tlsgpu_open_host(tlsgpu_sessions* t, const tlsgpu_record* h_recs, uint32_t n,
                                const uint8_t* h_in, size_t in_bytes, uint8_t* h_out,
                                size_t out_bytes, int32_t* h_status) {
  return host_batch(t, false, h_recs, n, h_in, in_bytes, h_out, out_bytes, h_status);
}

extern "C" int tlsgpu_seal_host(tlsgpu_sessions* t, const tlsgpu_record* h_recs, uint32_t n,
                                const uint8_t* h_in, size_t in_bytes, uint8_t* h_out,
                                size_t out_bytes, int32_t* h_status) {
  if (h_out == h_in && n) return fail(TLSGPU_EINVAL, "tlsgpu_seal_host cannot run in place");
  return host_batch(t, true, h_recs, n, h_in, in_bytes, h_out, out_bytes, h_status);
}

extern "C" int tlsgpu_sessions_set_owner(tlsgpu_sessions* t, uint32_t first, uint32_t n,
                                         const void* const* owners) {
  if (!t || (n && !owners)) return fail(TLSGPU_EINVAL, "bad arguments");
  if ((uint64_t)first + n > t->capacity)
    return fail(TLSGPU_ERANGE, "sessions [%u, %u) exceed capacity %u", first, first + n,
                t->capacity);
  for (uint32_t i = 0; i < n; i++) t->owners[first + i] = owners[i];
  return TLSGPU_OK;
}

// Host delivery of device-resident opens (tlsgpu_open_batch / tlsgpu_open_wire):
// descriptors and statuses back to the host, the delivered records' output
// range to h_out (same offsets as d_out), then the TaLoS read hook on each
// delivered record in record order.
extern "C" int tlsgpu_deliver_host(tlsgpu_sessions* t, const tlsgpu_record* d_recs,
                                   const int32_t* d_status, uint32_t n, const uint8_t* d_out,
                                   size_t out_bytes, uint8_t* h_out, int32_t* h_status,
                                   void* stream) {
  if (!t || (n && (!d_recs || !d_status || !d_out || !h_out || !h_status)))
    return fail(TLSGPU_EINVAL, "bad arguments");
  if (n == 0) return TLSGPU_OK;
  HIPCHK(hipSetDevice(t->eng->device));
  hipStream_t s = stream ? (hipStream_t)stream : t->eng->stream;
  std::vector<tlsgpu_record> recs(n);
  HIPCHK(hipMemcpyAsync(recs.data(), d_recs, sizeof(tlsgpu_record) * (size_t)n,
                        hipMemcpyDeviceToHost, s));
  HIPCHK(hipMemcpyAsync(h_status, d_status, sizeof(int32_t) * (size_t)n, hipMemcpyDeviceToHost,
                        s));
  HIPCHK(hipStreamSynchronize(s));
  uint64_t lo = UINT64_MAX, hi = 0;
  for (uint32_t i = 0; i < n; i++) {
    if (h_status[i] < 0) continue;
    const uint64_t o = recs[i].out_off, e = o + (uint64_t)h_status[i];
    if (o > out_bytes || e > out_bytes || recs[i].session >= t->capacity)
      return fail(TLSGPU_ERANGE, "record %u output [%llu, %llu) outside %zu bytes", i,
                  (unsigned long long)o, (unsigned long long)e, out_bytes);
    lo = std::min(lo, o);
    hi = std::max(hi, e);
  }
  if (hi > lo) {
    HIPCHK(hipMemcpyAsync(h_out + lo, d_out + lo, hi - lo, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
  }
  if (talos_read_hooked()) {
    for (uint32_t i = 0; i < n; i++) {
      if (h_status[i] < 0) continue;
      uint32_t hl = (uint32_t)h_status[i];
      talos_read(t->owners[recs[i].session], h_out + recs[i].out_off, &hl);
      if (hl < (uint32_t)h_status[i]) h_status[i] = (int32_t)hl;
    }
  }
  return TLSGPU_OK;
}

// The write side of tlsgpu_seal_wire for callers whose application data starts
// in host memory: the TaLoS write hook on every fragment do_ssl3_write would
// make of each stream (max_send_fragment split, s3_pkt.c:531-536), in place,
// before the caller copies h_data to the device.  Lengths stay.
extern "C" int tlsgpu_hook_write_streams(tlsgpu_sessions* t, const tlsgpu_write_stream* h_streams,
                                         uint32_t n_streams, uint8_t* h_data, size_t data_bytes) {
  if (!t || (n_streams && (!h_streams || !h_data))) return fail(TLSGPU_EINVAL, "bad arguments");
  if (!talos_write_hooked()) return TLSGPU_OK;
  for (uint32_t i = 0; i < n_streams; i++) {
    const tlsgpu_write_stream& st = h_streams[i];
    if (st.session >= t->capacity || st.data_off > data_bytes ||
        st.data_len > data_bytes - st.data_off)
      continue;
    const uint32_t frag = st.max_fragment == 0 || st.max_fragment > 16384 ? 16384 : st.max_fragment;
    for (uint64_t off = 0; off < st.data_len; off += frag) {
      uint32_t hl = (uint32_t)std::min<uint64_t>(frag, st.data_len - off);
      talos_write(t->owners[st.session], h_data + st.data_off + off, &hl);
    }
  }
  return TLSGPU_OK;
}

extern "C" int tlsgpu_open_wire(tlsgpu_sessions* t, const tlsgpu_wire_stream* d_streams,
                                uint32_t n_streams, uint8_t* d_wire, uint32_t max_records,
                                tlsgpu_record* d_recs, int32_t* d_status,
                                tlsgpu_wire_result* d_results, uint32_t* d_total, void* stream) {
  if (!t || !d_total || (n_streams && (!d_streams || !d_wire || !d_results)) ||
      (max_records && (!d_recs || !d_status)))
    return fail(TLSGPU_EINVAL, "bad arguments");
  HIPCHK(hipSetDevice(t->eng->device));
  hipStream_t s = stream ? (hipStream_t)stream : t->eng->stream;
  HIPCHK(hipMemsetAsync(d_total, 0, sizeof(uint32_t), s));
  if (n_streams == 0) return TLSGPU_OK;
  // unused record slots name no session (0xFFFFFFFF): the open kernels skip them
  if (max_records) HIPCHK(hipMemsetAsync(d_recs, 0xFF, sizeof(tlsgpu_record) * (size_t)max_records, s));
  if (launch_wire_frame(d_streams, n_streams, d_wire, t->d_sess, t->capacity, max_records, d_recs,
                        d_results, d_total, s))
    return fail(TLSGPU_EHIP, "wire frame launch: %s", hipGetErrorString(hipGetLastError()));
  if (max_records) {
    int rc = run_batch(t, d_recs, max_records, d_wire, d_wire, d_status, s, false, false);
    if (rc != TLSGPU_OK) return rc;
  }
  if (launch_wire_finish(n_streams, d_results, d_status, s))
    return fail(TLSGPU_EHIP, "wire finish launch: %s", hipGetErrorString(hipGetLastError()));
  return TLSGPU_OK;
}

extern "C" int tlsgpu_seal_wire(tlsgpu_sessions* t, const tlsgpu_write_stream* d_streams,
                                uint32_t n_streams, const uint8_t* d_data, size_t data_bytes,
                                uint8_t* d_wire, size_t wire_bytes, uint32_t max_records,
                                tlsgpu_record* d_recs, int32_t* d_status,
                                tlsgpu_write_result* d_results, uint32_t* d_total, void* stream) {
  if (!t || !d_total || (n_streams && (!d_streams || !d_data || !d_wire || !d_results)) ||
      (max_records && (!d_recs || !d_status)))
    return fail(TLSGPU_EINVAL, "bad arguments");
  HIPCHK(hipSetDevice(t->eng->device));
  hipStream_t s = stream ? (hipStream_t)stream : t->eng->stream;
  HIPCHK(hipMemsetAsync(d_total, 0, sizeof(uint32_t), s));
  if (n_streams == 0) return TLSGPU_OK;
  // unused record slots name no session (0xFFFFFFFF): the seal kernels skip them
  if (max_records) HIPCHK(hipMemsetAsync(d_recs, 0xFF, sizeof(tlsgpu_record) * (size_t)max_records, s));
  if (launch_wire_seal_frame(d_streams, n_streams, t->d_sess, t->capacity, d_wire, wire_bytes,
                             max_records, d_recs, d_results, d_total, s))
    return fail(TLSGPU_EHIP, "wire seal frame launch: %s", hipGetErrorString(hipGetLastError()));
  if (max_records) {
    const Bounds b = {data_bytes, wire_bytes};
    return run_batch(t, d_recs, max_records, d_data, d_wire, d_status, s, true, false, &b);
  }
  return TLSGPU_OK;
}

extern "C" uint64_t tlsgpu_seal_wire_size(int aead, uint32_t data_len, uint32_t max_fragment,
                                          uint32_t tag_len) {
  const uint32_t frag = max_fragment == 0 || max_fragment > 16384 ? 16384 : max_fragment;
  const uint64_t nrec = ((uint64_t)data_len + frag - 1) / frag;
  const uint64_t eiv = aead == TLSGPU_AES_128_GCM || aead == TLSGPU_AES_256_GCM ? 8 : 0;
  return data_len + nrec * (5 + eiv + (tag_len ? tag_len : 16));
}

extern "C" int tlsgpu_fill_synthetic(tlsgpu_engine* e, uint8_t* d_out, uint64_t stride,
                                     uint32_t span_len, uint32_t n, uint64_t seed,
                                     uint64_t index0, void* stream) {
  if (!e || (!d_out && n)) return fail(TLSGPU_EINVAL, "bad arguments");
  HIPCHK(hipSetDevice(e->device));
  if (launch_fill_synthetic(d_out, stride, span_len, n, seed, index0,
                            stream ? (hipStream_t)stream : e->stream))
    return fail(TLSGPU_EHIP, "fill launch: %s", hipGetErrorString(hipGetLastError()));
  return TLSGPU_OK;
}

extern "C" int tlsgpu_fill_synthetic_spans(tlsgpu_engine* e, uint8_t* d_out,
                                           const uint64_t* d_offsets, const uint32_t* d_lengths,
                                           uint32_t n, uint64_t seed, uint64_t index0,
                                           void* stream) {
  if (!e || (n && (!d_out || !d_offsets || !d_lengths))) return fail(TLSGPU_EINVAL, "bad arguments");
  HIPCHK(hipSetDevice(e->device));
  if (launch_fill_synthetic_spans(d_out, d_offsets, d_lengths, n, seed, index0,
                                  stream ? (hipStream_t)stream : e->stream))
    return fail(TLSGPU_EHIP, "fill launch: %s", hipGetErrorString(hipGetLastError()));
  return TLSGPU_OK;
}

// ---------------------------------------------------------------------------
// memory / streams / events
#define ENG_OR_FAIL(e) \
  if (!(e)) return fail(TLSGPU_EINVAL, "null engine"); \
  HIPCHK(hipSetDevice((e)->device))

static hipStream_t pick(tlsgpu_engine* e, void* s) { return s ? (hipStream_t)s : e->stream; }

extern "C" int tlsgpu_malloc(tlsgpu_engine* e, size_t bytes, void** d_ptr) {
  ENG_OR_FAIL(e);
  if (!d_ptr) return fail(TLSGPU_EINVAL, "null out");
  if (hipMalloc(d_ptr, bytes ? bytes : 1) != hipSuccess)
    return fail(TLSGPU_ENOMEM, "hipMalloc(%zu)", bytes);
  return TLSGPU_OK;
}
extern "C" int tlsgpu_free(tlsgpu_engine* e, void* d_ptr) {
  ENG_OR_FAIL(e);
  HIPCHK(hipFree(d_ptr));
  return TLSGPU_OK;
}
extern "C" int tlsgpu_host_alloc(tlsgpu_engine* e, size_t bytes, void** h_ptr) {
  ENG_OR_FAIL(e);
  if (!h_ptr) return fail(TLSGPU_EINVAL, "null out");
  if (hipHostMalloc(h_ptr, bytes ? bytes : 1, hipHostMallocDefault) != hipSuccess)
    return fail(TLSGPU_ENOMEM, "hipHostMalloc(%zu)", bytes);
  return TLSGPU_OK;
}
extern "C" int tlsgpu_host_free(tlsgpu_engine* e, void* h_ptr) {
  ENG_OR_FAIL(e);
  HIPCHK(hipHostFree(h_ptr));
  return TLSGPU_OK;
}
extern "C" int tlsgpu_memcpy(tlsgpu_engine* e, void* dst, const void* src, size_t bytes,
                             void* stream) {
  ENG_OR_FAIL(e);
  if (bytes) HIPCHK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDefault, pick(e, stream)));
  return TLSGPU_OK;
}
extern "C" int tlsgpu_memset(tlsgpu_engine* e, void* d_ptr, int value, size_t bytes,
                             void* stream) {
  ENG_OR_FAIL(e);
  if (bytes) HIPCHK(hipMemsetAsync(d_ptr, value, bytes, pick(e, stream)));
  return TLSGPU_OK;
}
extern "C" int tlsgpu_stream_create(tlsgpu_engine* e, void** stream) {
  ENG_OR_FAIL(e);
  hipStream_t s;
  HIPCHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  *stream = s;
  return TLSGPU_OK;
}
extern "C" int tlsgpu_stream_destroy(tlsgpu_engine* e, void* stream) {
  ENG_OR_FAIL(e);
  HIPCHK(hipStreamDestroy((hipStream_t)stream));
  return TLSGPU_OK;
}
extern "C" int tlsgpu_stream_sync(tlsgpu_engine* e, void* stream) {
  ENG_OR_FAIL(e);
  HIPCHK(hipStreamSynchronize(pick(e, stream)));
  return TLSGPU_OK;
}
extern "C" int tlsgpu_event_create(tlsgpu_engine* e, void** event) {
  ENG_OR_FAIL(e);
  hipEvent_t ev;
  HIPCHK(hipEventCreate(&ev));
  *event = ev;
  return TLSGPU_OK;
}
extern "C" int tlsgpu_event_destroy(tlsgpu_engine* e, void* event) {
  ENG_OR_FAIL(e);
  HIPCHK(hipEventDestroy((hipEvent_t)event));
  return TLSGPU_OK;
}
extern "C" int tlsgpu_event_record(tlsgpu_engine* e, void* event, void* stream) {
  ENG_OR_FAIL(e);
  HIPCHK(hipEventRecord((hipEvent_t)event, pick(e, stream)));
  return TLSGPU_OK;
}
extern "C" int tlsgpu_event_elapsed_ms(tlsgpu_engine* e, void* start, void* end, float* ms) {
  ENG_OR_FAIL(e);
  HIPCHK(hipEventSynchronize((hipEvent_t)end));
  HIPCHK(hipEventElapsedTime(ms, (hipEvent_t)start, (hipEvent_t)end));
  return TLSGPU_OK;
}

// ---------------------------------------------------------------------------
// EVP_AEAD drop-in (include/openssl/evp.h:1211-1315)

// ERR queue hook: resolved only when a LibreSSL libcrypto is in the process.
extern "C" void ERR_put_error(int lib, int func, int reason, const char* file, int line)
    __attribute__((weak));

// Values from LibreSSL include/openssl/evp.h:1327-1491 and err.h:163.
enum {
  ERR_LIB_EVP_ = 6,
  F_AEAD_AES_GCM_INIT = 187, F_AEAD_AES_GCM_OPEN = 188, F_AEAD_AES_GCM_SEAL = 189,
  F_AEAD_CHACHA20_POLY1305_INIT = 192, F_AEAD_CHACHA20_POLY1305_OPEN = 193,
  F_AEAD_CHACHA20_POLY1305_SEAL = 194, F_AEAD_CTX_OPEN = 185, F_AEAD_CTX_SEAL = 186,
  F_EVP_AEAD_CTX_INIT = 180,
  R_BAD_DECRYPT = 100, R_BAD_KEY_LENGTH = 137, R_BUFFER_TOO_SMALL = 155, R_IV_TOO_LARGE = 102,
  R_OUTPUT_ALIASES_INPUT = 172, R_TAG_TOO_LARGE = 171, R_TOO_LARGE = 164,
  R_UNSUPPORTED_KEY_SIZE = 108,
};

static void evp_err(int func, int reason) {
  if (ERR_put_error) ERR_put_error(ERR_LIB_EVP_, func, reason, __FILE__, __LINE__);
}

struct evp_aead_st {
  unsigned char key_len, nonce_len, overhead, max_tag_len;
  int kind;
};

static const evp_aead_st k_aes128 = {16, 12, 16, 16, TLSGPU_AES_128_GCM};
static const evp_aead_st k_aes256 = {32, 12, 16, 16, TLSGPU_AES_256_GCM};
static const evp_aead_st k_cc = {32, 12, 16, 16, TLSGPU_CHACHA20_POLY1305};
static const evp_aead_st k_cc_old = {32, 8, 16, 16, TLSGPU_CHACHA20_POLY1305_OLD};

extern "C" const EVP_AEAD* EVP_aead_aes_128_gcm(void) { return &k_aes128; }
extern "C" const EVP_AEAD* EVP_aead_aes_256_gcm(void) { return &k_aes256; }
extern "C" const EVP_AEAD* EVP_aead_chacha20_poly1305(void) { return &k_cc; }
extern "C" const EVP_AEAD* EVP_aead_chacha20_poly1305_old(void) { return &k_cc_old; }
extern "C" size_t EVP_AEAD_key_length(const EVP_AEAD* a) { return a->key_len; }
extern "C" size_t EVP_AEAD_nonce_length(const EVP_AEAD* a) { return a->nonce_len; }
extern "C" size_t EVP_AEAD_max_overhead(const EVP_AEAD* a) { return a->overhead; }
extern "C" size_t EVP_AEAD_max_tag_len(const EVP_AEAD* a) { return a->max_tag_len; }

// Process-wide engines of the per-call path, one per GPU the EVP surface uses:
// TLSGPU_DEVICE=d pins it to device d; otherwise every visible GPU takes new
// contexts in turn (EVP_AEAD_CTX_init round-robin), so an unchanged server's
// connections spread over the node's GPUs — one SSL per thread
// in the reference's worker model, one context per connection direction.
constexpr int kMaxEvpDevices = 16;
static std::mutex g_mu;
static std::vector<int> g_evp_devices;  // device ordinals, filled once
static tlsgpu_engine* g_engines[kMaxEvpDevices] = {};
static std::atomic<uint32_t> g_evp_rr{0};
static std::atomic<uint64_t> g_evp_dev_calls[kMaxEvpDevices];  // per EVP device
static std::atomic<uint64_t> g_evp_dev_ctx[kMaxEvpDevices];

static const std::vector<int>& evp_devices_locked() {
  if (g_evp_devices.empty()) {
    const char* d = getenv("TLSGPU_DEVICE");
    const char* list = getenv("TLSGPU_DEVICES");  // e.g. "0,1,2,3"; a device may repeat
    int count = 0;
    if (list && *list) {
      for (const char* c = list; *c && g_evp_devices.size() < (size_t)kMaxEvpDevices;) {
        char* end = nullptr;
        const long v = strtol(c, &end, 10);
        if (end == c) break;
        g_evp_devices.push_back((int)v);
        c = *end == ',' ? end + 1 : end;
      }
    }
    if (!g_evp_devices.empty()) {
    } else if (d && *d) {
      g_evp_devices.push_back(atoi(d));
    } else if (hipGetDeviceCount(&count) == hipSuccess && count > 0) {
      for (int i = 0; i < count && i < kMaxEvpDevices; i++) g_evp_devices.push_back(i);
    } else {
      g_evp_devices.push_back(0);
    }
  }
  return g_evp_devices;
}

// Engine of the k-th EVP device (created on first use), or nullptr.
static tlsgpu_engine* evp_engine(size_t k) {
  std::lock_guard<std::mutex> lk(g_mu);
  const auto& devs = evp_devices_locked();
  if (k >= devs.size()) return nullptr;
  if (!g_engines[k] && tlsgpu_engine_create(devs[k], &g_engines[k]) != TLSGPU_OK)
    g_engines[k] = nullptr;
  return g_engines[k];
}

static size_t evp_device_count() {
  std::lock_guard<std::mutex> lk(g_mu);
  return evp_devices_locked().size();
}

// The next device index for a new context (round-robin over the EVP devices).
static size_t evp_pick() { return g_evp_rr.fetch_add(1) % evp_device_count(); }

struct EvpBatcher;
constexpr int kImagePoisoned = 3;
struct AeadState {
  tlsgpu_sessions* sess;  // the device table holding the context's session
  uint32_t slot;          // session id in sess
  int kind;
  unsigned tag_len;
  EvpBatcher* batcher;    // the queue of the context's device (pooled contexts), or null
  uint32_t evp_dev;       // index of the context's device among the EVP devices
  hipEvent_t installed;   // the slot's event, recorded after the context's key install
  uint32_t key_id = 0;    // unique per install (doorbell server's LDS table cache)
  mutable std::atomic<bool> install_pending{true};  // no call has waited for it yet
  // Deferred install (round 5): the session image built on the host at init
  // (session_host.cpp) in a pinned image buffer, installed by the context's
  // first call — posted with the doorbell job, or one upload kernel ahead of a
  // launched job — so EVP_AEAD_CTX_init launches nothing.  0: on the device
  // (or no image), 1: image waiting, 2: a call is installing it,
  // kImagePoisoned: an install job went unanswered (image and slot leaked)
  mutable std::atomic<int> image{0};
  uint8_t* img_h = nullptr;  // pinned image (host / device views)
  uint8_t* img_d = nullptr;
  bool img_tables = false;   // the image has GCM tables
  bool img_compact = false;  // ... only m[8] = H^e of each Shoup table (round 6)
  hipEvent_t slot_ev = nullptr;  // the slot's event: its previous owner's scrub
};

// Pinned image buffers of deferred installs, per device, reused (zeroed on
// return: key material).
struct ImagePool {
  std::mutex mu;
  std::vector<std::pair<uint8_t*, uint8_t*>> free;  // (host, device view)
};
constexpr size_t kImageBytes = sizeof(DevSession) + sizeof(DevGcmTables);
constexpr size_t kImageSlab = 32;
static_assert(kImageBytes % 256 == 0, "session images stay 256-B aligned in a slab");
static ImagePool g_img_pool[64];
static bool image_take(int dev, uint8_t** h, uint8_t** d) {
  if (dev < 0 || dev >= 64) return false;
  {
    std::lock_guard<std::mutex> lk(g_img_pool[dev].mu);
    if (!g_img_pool[dev].free.empty()) {
      *h = g_img_pool[dev].free.back().first;
      *d = g_img_pool[dev].free.back().second;
      g_img_pool[dev].free.pop_back();
      return true;
    }
  }
  // none free: one pinned slab of kImageSlab images (one hipHostMalloc per 32
  // contexts instead of one per context; held for the process, like the pool)
  uint8_t *hs = nullptr, *ds = nullptr;
  if (hipSetDevice(dev) != hipSuccess ||
      hipHostMalloc((void**)&hs, kImageBytes * kImageSlab, hipHostMallocDefault) != hipSuccess)
    return false;
  if (hipHostGetDevicePointer((void**)&ds, hs, 0) != hipSuccess) {
    (void)hipHostFree(hs);
    return false;
  }
  memset(hs, 0, kImageBytes * kImageSlab);
  {
    std::lock_guard<std::mutex> lk(g_img_pool[dev].mu);
    for (size_t i = 1; i < kImageSlab; i++)
      g_img_pool[dev].free.emplace_back(hs + i * kImageBytes, ds + i * kImageBytes);
  }
  *h = hs;
  *d = ds;
  return true;
}
static void image_give(int dev, uint8_t* h, uint8_t* d) {
  explicit_bzero(h, kImageBytes);
  std::lock_guard<std::mutex> lk(g_img_pool[dev].mu);
  g_img_pool[dev].free.emplace_back(h, d);
}

// EVP context storage without a device allocation per context (connection
// churn): contexts outside the coalescing queue take a slot of
// per-device slab tables of kSlabSessions sessions, grown on demand; the slot
// is scrubbed on cleanup and reused.
constexpr uint32_t kSlabSessions = 1024;
struct EvpSlab {
  std::mutex mu;
  std::vector<tlsgpu_sessions*> chunks;
  std::vector<std::pair<tlsgpu_sessions*, uint32_t>> free;
};
static EvpSlab g_slabs[kMaxEvpDevices];

static bool slab_take(size_t dk, tlsgpu_engine* e, tlsgpu_sessions** t, uint32_t* slot) {
  EvpSlab& sl = g_slabs[dk];
  std::lock_guard<std::mutex> lk(sl.mu);
  if (sl.free.empty()) {
    tlsgpu_sessions* c = nullptr;
    if (tlsgpu_sessions_create(e, kSlabSessions, &c) != TLSGPU_OK) return false;
    sl.chunks.push_back(c);
    for (uint32_t i = kSlabSessions; i-- > 0;) sl.free.emplace_back(c, i);
  }
  *t = sl.free.back().first;
  *slot = sl.free.back().second;
  sl.free.pop_back();
  return true;
}

static void slab_give(size_t dk, tlsgpu_sessions* t, uint32_t slot) {
  EvpSlab& sl = g_slabs[dk];
  std::lock_guard<std::mutex> lk(sl.mu);
  sl.free.emplace_back(t, slot);
}

// ---------------------------------------------------------------------------
// EVP coalescing queue (TaLoS make_asynchronous_ecall,
// src/talos/enclaveshim/enclaveshim_ecalls.c:457-610, in GPU form).
//
// With batching on (tlsgpu_evp_set_batching or TLSGPU_EVP_BATCH_US > 0),
// EVP_AEAD_CTX_init installs the key into a slot of one shared device session
// pool, and every EVP_AEAD_CTX_seal/open joins the batch being built and
// blocks until it completes.  Batches live in a ring of kEvpSlots staging
// slots (pinned host + device, one HIP stream each):
//   caller      reserves a descriptor and byte ranges in the building slot
//               (under the lock), copies its nonce / AD / input into the
//               pinned slot itself (outside the lock, in parallel with the
//               other callers), then sleeps on the slot's futex word;
//   dispatcher  closes the building slot when the GPU is idle, the slot is
//               full, or the window since its first job has passed; waits for
//               the slot's writers, then issues one H2D, one raw batch per
//               direction, one D2H and an event on the slot's stream;
//   completer   waits on the events in order and wakes each slot's callers
//               with ONE futex wake; every caller copies its own output out,
//               and the last one returns the slot to the ring.
// So at most kEvpSlots-1 batches are in flight while the next one fills, no
// per-job work runs on the dispatcher, and results are the per-call path's,
// bit for bit (same raw kernels).
constexpr uint32_t kEvpSlots = 3;
constexpr uint32_t kEvpMaxJobs = 1024;
constexpr size_t kEvpDescBytes = sizeof(RawJob) * kEvpMaxJobs;
constexpr size_t kEvpInBytes = 8u << 20, kEvpOutBytes = 8u << 20;
constexpr size_t kEvpStatusOff = kEvpDescBytes + kEvpInBytes;   // int32 x kEvpMaxJobs
constexpr size_t kEvpOutOff = kEvpStatusOff + 4 * kEvpMaxJobs;
constexpr size_t kEvpSlotBytes = kEvpOutOff + kEvpOutBytes;

struct EvpSlot {
  uint8_t* h = nullptr;  // pinned: [RawJob x kEvpMaxJobs | inputs | status | outputs]
  uint8_t* d = nullptr;  // device, same layout (zero-copy: h as the device addresses it)
  bool zc = false;       // zero-copy: no device copy of the slot, no H2D / D2H
  hipStream_t stream = nullptr;
  hipEvent_t done = nullptr;
  // built under EvpBatcher::mu: seal descriptors from the front, open ones
  // from the back, so each direction is one contiguous raw batch
  uint32_t nseal = 0, nopen = 0;
  unsigned kinds_seal = 0, kinds_open = 0;  // AEAD kinds present (run_batch masks)
  size_t in_used = 0, out_used = 0;
  std::chrono::steady_clock::time_point first, submitted_at;
  std::atomic<uint32_t> writers{0};  // callers still copying in
  std::atomic<uint32_t> readers{0};  // callers still copying out
  std::atomic<uint32_t> gen{0};      // bumped on completion (futex word)
  bool ok = false;
  uint32_t jobs() const { return nseal + nopen; }
};

struct EvpBatcher {
  std::mutex mu;
  std::condition_variable cv_disp, cv_comp, cv_slot;
  EvpSlot slots[kEvpSlots];
  EvpSlot* building = nullptr;  // the slot callers join (nullptr: all busy)
  std::vector<EvpSlot*> free_ring;
  std::deque<EvpSlot*> submitted;
  uint32_t inflight = 0;
  bool full = false;  // a caller found the building slot full
  std::thread disp, comp;
  unsigned window_us = 0, max_jobs = kEvpMaxJobs;
  tlsgpu_sessions* pool = nullptr;
  std::vector<int> free_sessions;
  uint64_t batches = 0, jobs_done = 0;
  // TLSGPU_EVP_STATS=1: nanoseconds summed over batches (printed at exit)
  uint64_t ns_wait = 0, ns_writers = 0, ns_submit = 0, ns_gpu = 0;
  void dispatch_loop();
  void complete_loop();
  void submit(EvpSlot* s);
  bool submit_work(EvpSlot* s);
  void release(EvpSlot* s);
};
// one coalescing queue per EVP device (index as evp_engine); g_batcher_on once
// tlsgpu_evp_set_batching has created them
static EvpBatcher* g_batchers[kMaxEvpDevices] = {};
static std::mutex g_batcher_mu;

// Give a context's session slot back to its queue pool or slab.
static void release_slot(AeadState* st) {
  if (st->batcher) {
    std::lock_guard<std::mutex> lk(g_batcher_mu);
    st->batcher->free_sessions.push_back((int)st->slot);
  } else {
    slab_give(st->evp_dev, st->sess, st->slot);
  }
}
static bool g_batcher_on = false;

static inline void futex_wait(std::atomic<uint32_t>* w, uint32_t v) {
  syscall(SYS_futex, reinterpret_cast<uint32_t*>(w), FUTEX_WAIT_PRIVATE, v, nullptr, nullptr, 0);
}
static inline void futex_wake_all(std::atomic<uint32_t>* w) {
  syscall(SYS_futex, reinterpret_cast<uint32_t*>(w), FUTEX_WAKE_PRIVATE, INT_MAX, nullptr, nullptr,
          0);
}

// Per-thread staging for one call: pinned host + device buffer and a stream
// (calls on one ctx may run concurrently from several threads,
// evp.h:1273-1274).  Layout [RawJob | nonce | ad | in | status | out], so one
// H2D covers the job up to its preset status and one D2H status and output.
// Threads share kCallStreams streams per process (more streams than the
// hardware queues, GPU_MAX_HW_QUEUES = 4, cost 3x in call rate at 64 threads:
// tools/hip_latency); each thread waits on its own event, i.e. on its own
// work and what was queued before it on that stream.
constexpr int kCallStreams = 4;
constexpr int kMaxDev = 64;  // device ordinals a thread may stage for
static hipStream_t g_call_streams[kMaxDev][kCallStreams];
static std::once_flag g_call_streams_once[kMaxDev];
static bool g_call_streams_ok[kMaxDev];
static std::atomic<uint32_t> g_call_thread_seq{0};

// Pinned staging chunks (round 6): a thread's
// per-call staging is one kStageChunk of pinned host memory carved from
// kStageSlab-byte slabs (one hipHostMalloc per 32 threads), enough for any TLS
// record job ([RawJob | nonce | ad | 16 KiB + 2 KiB in | status | out] <=
// 40 KiB); a thread that makes a larger EVP call grows to its own allocation.
// Chunks go back to the free list without a HIP call (a thread's exit makes
// none), so the pinned bytes are bounded by the peak number
// of calling threads x 64 KiB.  No device buffer unless a path needs one (the
// zero-copy per-call path, the default, reads and writes the pinned chunk).
constexpr size_t kStageChunk = 64u << 10;
constexpr size_t kStageSlab = 2u << 20;
struct StageChunks {
  std::mutex mu;
  std::vector<std::pair<uint8_t*, uint8_t*>> free;  // (host, device view)
  std::atomic<uint64_t> slabs{0};
};
static StageChunks g_stage_chunks[kMaxDev];
static bool stage_chunk_take(int dev, uint8_t** h, uint8_t** d) {
  StageChunks& c = g_stage_chunks[dev];
  {
    std::lock_guard<std::mutex> lk(c.mu);
    if (!c.free.empty()) {
      *h = c.free.back().first;
      *d = c.free.back().second;
      c.free.pop_back();
      return true;
    }
  }
  uint8_t *hs = nullptr, *ds = nullptr;
  if (hipHostMalloc((void**)&hs, kStageSlab, hipHostMallocDefault) != hipSuccess) return false;
  if (hipHostGetDevicePointer((void**)&ds, hs, 0) != hipSuccess) ds = nullptr;
  c.slabs.fetch_add(1, std::memory_order_relaxed);
  {
    std::lock_guard<std::mutex> lk(c.mu);
    for (size_t i = 1; i < kStageSlab / kStageChunk; i++)
      c.free.emplace_back(hs + i * kStageChunk, ds ? ds + i * kStageChunk : nullptr);
  }
  *h = hs;
  *d = ds;
  return true;
}
static void stage_chunk_give(int dev, uint8_t* h, uint8_t* d) {
  std::lock_guard<std::mutex> lk(g_stage_chunks[dev].mu);
  g_stage_chunks[dev].free.emplace_back(h, d);
}

// One per (thread, device): buffers, stream and event belong to that device.
struct Staging {
  int device = -1;
  hipStream_t stream = nullptr;
  hipEvent_t done = nullptr;
  uint8_t* d_buf = nullptr;  // device buffer (only the staged, non-zero-copy paths)
  uint8_t* h_buf = nullptr;
  uint8_t* h_dev = nullptr;  // h_buf as the device addresses it (zero-copy calls)
  size_t cap = 0;            // bytes of h_buf (kStageChunk: a pooled chunk)
  size_t dcap = 0;           // bytes of d_buf
  // key areas (round 5; round 6: buffers from the shared pinned image pool,
  // not per thread): install_one builds the slot's image here
  // (session_host.cpp) and one kernel copies it into the slot; `dirty` until
  // the copy is known done (its event), then zeroed and given back to the pool
  // (explicit_bzero analogue, image_give)
  struct KeyArea {
    uint8_t* h = nullptr;
    uint8_t* dev = nullptr;
    hipEvent_t ev = nullptr;
    bool dirty = false;
  };
  static constexpr int kKeyAreas = 4;
  static constexpr size_t kKeyAreaBytes = sizeof(DevSession) + sizeof(DevGcmTables);
  KeyArea keys[kKeyAreas];
  uint32_t key_next = 0;
  void give_key_area(KeyArea& k) {
    image_give(device, k.h, k.dev);  // zeroes it
    k.h = k.dev = nullptr;
    k.dirty = false;
  }
  // the next key area (waiting for and zeroing its previous image if needed)
  KeyArea* take_key_area() {
    KeyArea& k = keys[key_next++ % kKeyAreas];
    if (!k.ev && hipEventCreateWithFlags(&k.ev, hipEventDisableTiming) != hipSuccess) {
      k.ev = nullptr;
      return nullptr;
    }
    if (k.dirty) {
      if (hipEventSynchronize(k.ev) != hipSuccess) return nullptr;
      give_key_area(k);
    }
    if (!image_take(device, &k.h, &k.dev)) return nullptr;
    return &k;
  }
  // zero and give back every key area whose copy has finished (no wait)
  void sweep_key_areas() {
    for (KeyArea& k : keys)
      if (k.dirty && hipEventQuery(k.ev) == hipSuccess) give_key_area(k);
  }
  bool any_dirty_key_area() const {
    for (const KeyArea& k : keys)
      if (k.dirty) return true;
    return false;
  }
  ~Staging() {
    if (device >= 0) (void)hipSetDevice(device);  // the buffers' and the event's device
    if (d_buf) (void)hipFree(d_buf);
    release_host();
    if (done) (void)hipEventDestroy(done);
  }
  void release_host() {
    if (h_buf && cap == kStageChunk) stage_chunk_give(device, h_buf, h_dev);
    else if (h_buf) (void)hipHostFree(h_buf);
    h_buf = h_dev = nullptr;
    cap = 0;
  }
  // A job that may still run on the device owns the buffers (a doorbell post
  // nobody answered): forget them without freeing, the next ensure allocates.
  void abandon() {
    d_buf = h_buf = h_dev = nullptr;
    cap = dcap = 0;
  }
  // `bytes` of pinned staging (and of device staging when `dev_buf`) on `dev`
  bool ensure(int dev, size_t bytes, bool dev_buf = false) {
    if (dev < 0 || dev >= kMaxDev || hipSetDevice(dev) != hipSuccess) return false;
    if (!stream) {
      std::call_once(g_call_streams_once[dev], [dev] {
        bool ok = true;
        for (hipStream_t& cs : g_call_streams[dev])
          ok &= hipStreamCreateWithFlags(&cs, hipStreamNonBlocking) == hipSuccess;
        g_call_streams_ok[dev] = ok;
      });
      if (!g_call_streams_ok[dev] ||
          hipEventCreateWithFlags(&done, hipEventDisableTiming) != hipSuccess)
        return false;
      stream = g_call_streams[dev][g_call_thread_seq.fetch_add(1) % kCallStreams];
    }
    device = dev;
    if (cap < bytes) {
      release_host();  // this thread's calls are synchronous: nothing in flight
      if (bytes <= kStageChunk) {
        if (!stage_chunk_take(dev, &h_buf, &h_dev)) return false;
        cap = kStageChunk;
      } else {
        const size_t want = (bytes + kStageChunk - 1) & ~(kStageChunk - 1);
        if (hipHostMalloc((void**)&h_buf, want, hipHostMallocDefault) != hipSuccess) {
          h_buf = nullptr;
          return false;
        }
        if (hipHostGetDevicePointer((void**)&h_dev, h_buf, 0) != hipSuccess) h_dev = nullptr;
        cap = want;
      }
    }
    if (dev_buf && dcap < bytes) {
      if (d_buf) (void)hipFree(d_buf);
      d_buf = nullptr;
      dcap = 0;
      const size_t want = (bytes + kStageChunk - 1) & ~(kStageChunk - 1);
      if (hipMalloc(&d_buf, want) != hipSuccess) {
        d_buf = nullptr;
        return false;
      }
      dcap = want;
    }
    return true;
  }
};
// Staging of exited threads, per device, for the next thread (round 5): a
// thread's exit makes no HIP call — hipFree / hipHostFree would synchronise
// the device, i.e. wait behind doorbell server instances that other threads
// keep relaunching, and at process exit they ran before the servers were
// stopped.  The buffers live until the runtime's teardown.
static std::mutex g_stage_pool_mu;
static std::vector<Staging*> g_stage_pool[kMaxDev];
static void evp_shutdown_main_thread_exit();
struct StagingSet {
  Staging* by_dev[kMaxDev] = {};
  ~StagingSet() {
    // the main thread's staging goes at exit(): stop and drain the doorbell
    // servers first (shutdown contract)
    evp_shutdown_main_thread_exit();
    std::lock_guard<std::mutex> lk(g_stage_pool_mu);
    for (int d = 0; d < kMaxDev; d++)
      if (by_dev[d]) g_stage_pool[d].push_back(by_dev[d]);
  }
};
static thread_local StagingSet t_stages;

// This thread's staging for device `dev` (nullptr on a bad ordinal / no memory).
static Staging* stage_for(int dev) {
  if (dev < 0 || dev >= kMaxDev) return nullptr;
  Staging*& st = t_stages.by_dev[dev];
  if (!st) {
    std::lock_guard<std::mutex> lk(g_stage_pool_mu);
    if (!g_stage_pool[dev].empty()) {
      st = g_stage_pool[dev].back();
      g_stage_pool[dev].pop_back();
    }
  }
  // an exited thread's installs may have left images in its key areas
  // (ADVICE r05): zero the ones whose copies are done before reuse
  if (st && st->any_dirty_key_area()) st->sweep_key_areas();
  if (!st) st = new (std::nothrow) Staging();
  return st;
}

// The event of a slot (created on first use).
static hipEvent_t slot_event(tlsgpu_sessions* t, uint32_t slot) {
  std::lock_guard<std::mutex> lk(t->mu);
  if (t->slot_ev.size() < t->capacity) t->slot_ev.resize(t->capacity, nullptr);
  hipEvent_t& ev = t->slot_ev[slot];
  if (!ev && hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) ev = nullptr;
  return ev;
}

// One session install for an EVP context on the calling thread's call stream,
// asynchronous (round 3): the parameters travel as a kernel argument (no
// staging copy to wait for), the install is ordered after the slot's previous
// scrub by the slot's event and records it again when done; the context's
// first call waits for that event on the device (gpu_call_impl).  A
// connection's key install at ChangeCipherSpec (t1_enc.c:444-495) then costs
// no device round trip of its own.
// Round 5 (hygiene): the image is built on the
// calling thread (session_host.cpp: key schedule, H, the GHASH power tables —
// the ~25 µs of one wave install_session_arg spent) into a pinned key area,
// and one short kernel copies it into the slot: no key material in kernel
// arguments, and the area is zeroed once its copy has finished
// (sweep_key_areas after the thread's next synchronised call, or when the
// area is reused).  TLSGPU_EVP_DEVICE_INSTALL=1 keeps the device install.
// A host without AES-NI or PCLMUL builds no host image (session_host.cpp: no
// table-driven key schedule on the CPU) and takes the device install too.
static const bool g_device_install = [] {
  const char* v = getenv("TLSGPU_EVP_DEVICE_INSTALL");
  return (v && *v && *v != '0') || !host_crypto_ok();
}();

static int install_one(tlsgpu_sessions* t, uint32_t slot, const tlsgpu_session_params& p,
                       hipEvent_t* installed) {
  if (!valid_params(p) || slot >= t->capacity) return fail(TLSGPU_EINVAL, "bad session");
  Staging* stg = stage_for(t->eng->device);
  if (!stg || !stg->ensure(t->eng->device, 16)) return fail(TLSGPU_ENOMEM, "staging");
  const hipEvent_t ev = slot_event(t, slot);  // on the slot's device (ensure set it)
  if (!ev) return fail(TLSGPU_EHIP, "slot event");
  bool ok;
  if (g_device_install) {
    ok = hipStreamWaitEvent(stg->stream, ev, 0) == hipSuccess &&
         launch_session_install_arg(t->d_sess, t->d_gcm, p, slot, stg->stream) == 0 &&
         hipEventRecord(ev, stg->stream) == hipSuccess;
  } else {
    Staging::KeyArea* ka = stg->take_key_area();
    if (!ka) return fail(TLSGPU_ENOMEM, "key area");
    auto* img_s = reinterpret_cast<DevSession*>(ka->h);
    auto* img_t = reinterpret_cast<DevGcmTables*>(ka->h + sizeof(DevSession));
    const bool tables = host_session_image(p, img_s, img_t);
    ka->dirty = true;
    ok = hipStreamWaitEvent(stg->stream, ev, 0) == hipSuccess &&
         launch_upload_session(ka->dev, t->d_sess + slot, t->d_gcm + slot,
                               tables ? kGcmTableUploadBytes : 0u, stg->stream) == 0 &&
         hipEventRecord(ka->ev, stg->stream) == hipSuccess &&
         hipEventRecord(ev, stg->stream) == hipSuccess;
  }
  if (!ok) return fail(TLSGPU_EHIP, "session install: %s", hipGetErrorString(hipGetLastError()));
  *installed = ev;
  std::lock_guard<std::mutex> lk(t->mu);
  t->kinds[slot] = p.aead;
  t->tag_lens[slot] = (uint8_t)(p.tag_len ? p.tag_len : 16);
  t->have[p.aead] = true;
  return TLSGPU_OK;
}

// Zero a session slot's key material on the calling thread's stream without
// waiting: ordered after the slot's install by the slot's event, which then
// orders the slot's next install after the scrub.
static void scrub_slot(tlsgpu_sessions* t, uint32_t slot) {
  Staging* stg = stage_for(t->eng->device);
  const bool staged = stg && stg->ensure(t->eng->device, 16);
  const hipEvent_t ev = staged ? slot_event(t, slot) : nullptr;
  // after the slot's install (a context cleaned up before any call, from
  // another thread, may still have its install queued on another stream)
  if (ev && hipStreamWaitEvent(stg->stream, ev, 0) == hipSuccess &&
      launch_scrub_session(t->d_sess + slot, t->d_gcm + slot, stg->stream) == 0 &&
      hipEventRecord(ev, stg->stream) == hipSuccess) {
    stg->sweep_key_areas();
    return;
  }
  (void)hipSetDevice(t->eng->device);  // fall back to the synchronous form
  (void)hipDeviceSynchronize();
  (void)hipMemset(t->d_sess + slot, 0, sizeof(DevSession));
  (void)hipMemset(t->d_gcm + slot, 0, sizeof(DevGcmTables));
}

static bool doorbell_enabled();
// A context whose calls can take the doorbell defers its install to its first
// call (TLSGPU_EVP_DEFERRED_INSTALL=0: never).
static const bool g_deferred_install = [] {
  const char* v = getenv("TLSGPU_EVP_DEFERRED_INSTALL");
  return !(v && *v == '0');
}();
static bool deferred_install_ok(int kind);

static int defer_install(AeadState* st, const tlsgpu_session_params& p) {
  tlsgpu_sessions* t = st->sess;
  if (!valid_params(p) || st->slot >= t->capacity) return fail(TLSGPU_EINVAL, "bad session");
  if (hipSetDevice(t->eng->device) != hipSuccess) return fail(TLSGPU_EHIP, "set device");
  st->slot_ev = slot_event(t, st->slot);  // its previous owner's scrub, if launched
  if (!st->slot_ev) return fail(TLSGPU_EHIP, "slot event");
  if (!image_take(t->eng->device, &st->img_h, &st->img_d)) return fail(TLSGPU_ENOMEM, "session image");
  // compact (round 6): the doorbell install reads m[8] = H^e of each Shoup
  // table and expands the rest on the device; a launched first call
  // completes the image on the host before its upload
  st->img_tables = host_session_image(p, reinterpret_cast<DevSession*>(st->img_h),
                                      reinterpret_cast<DevGcmTables*>(st->img_h + sizeof(DevSession)),
                                      kGcmTableUploadBytes > offsetof(DevGcmTables, bsrk), true);
  st->img_compact = st->img_tables;
  st->installed = st->slot_ev;
  st->install_pending.store(false, std::memory_order_release);  // nothing queued
  st->image.store(1, std::memory_order_release);
  std::lock_guard<std::mutex> lk(t->mu);
  t->kinds[st->slot] = p.aead;
  t->tag_lens[st->slot] = (uint8_t)(p.tag_len ? p.tag_len : 16);
  t->have[p.aead] = true;
  return TLSGPU_OK;
}

static void evp_sweep_scrubs_for(size_t dk);
extern "C" int EVP_AEAD_CTX_init(EVP_AEAD_CTX* ctx, const EVP_AEAD* aead, const unsigned char* key,
                                 size_t key_len, size_t tag_len, ENGINE* impl) {
  (void)impl;
  ctx->aead = aead;
  ctx->aead_state = nullptr;
  if (key_len != aead->key_len) {  // evp_aead.c:55-58
    evp_err(F_EVP_AEAD_CTX_INIT, R_UNSUPPORTED_KEY_SIZE);
    return 0;
  }
  bool gcm = aead->kind == TLSGPU_AES_128_GCM || aead->kind == TLSGPU_AES_256_GCM;
  if (tag_len == EVP_AEAD_DEFAULT_TAG_LENGTH) tag_len = 16;
  if (tag_len > 16) {  // e_aes.c:1388-1391, e_chacha20poly1305.c:62-65
    evp_err(gcm ? F_AEAD_AES_GCM_INIT : F_AEAD_CHACHA20_POLY1305_INIT,
            gcm ? R_TAG_TOO_LARGE : R_TOO_LARGE);
    return 0;
  }
  const size_t dk = evp_pick();  // this context's GPU (round-robin over the EVP devices)
  tlsgpu_engine* e = evp_engine(dk);
  if (!e) return 0;
  auto* st = new (std::nothrow) AeadState();
  if (!st) return 0;
  st->kind = aead->kind;
  static std::atomic<uint32_t> g_key_ids{0};
  do st->key_id = g_key_ids.fetch_add(1, std::memory_order_relaxed) + 1;
  while (st->key_id == 0);  // 0 means "no key" to the server's table cache
  st->tag_len = (unsigned)tag_len;
  st->batcher = nullptr;
  st->evp_dev = (uint32_t)dk;
  {
    std::lock_guard<std::mutex> lk(g_batcher_mu);
    // a queue counts only once tlsgpu_evp_set_batching has published every
    // device's (a partial setup that failed leaves g_batcher_on false)
    EvpBatcher* b = g_batcher_on ? g_batchers[dk] : nullptr;
    if (b && !b->free_sessions.empty()) {
      st->slot = (uint32_t)b->free_sessions.back();
      b->free_sessions.pop_back();
      st->sess = b->pool;
      st->batcher = b;
    }
  }
  if (!st->batcher) evp_sweep_scrubs_for(dk);  // answered cleanup scrubs: slots back first
  if (!st->batcher && !slab_take(dk, e, &st->sess, &st->slot)) {
    delete st;
    return 0;
  }
  tlsgpu_session_params p;
  memset(&p, 0, sizeof(p));
  p.aead = aead->kind;
  p.key_len = (uint32_t)key_len;
  memcpy(p.key, key, key_len);
  p.tag_len = (uint32_t)tag_len;
  p.version = 0x0303;
  // deferred (round 5) where the first call can take the doorbell: nothing is
  // launched here, the first call installs the host-built image; otherwise on
  // this thread's call stream, not waited for: installs of concurrent threads
  // overlap, and the context's first call is ordered after it
  const int rc = (!st->batcher && deferred_install_ok(aead->kind)) ? defer_install(st, p)
                                                                   : install_one(st->sess, st->slot, p, &st->installed);
  memset(&p, 0, sizeof(p));
  if (rc != TLSGPU_OK) {
    if (st->img_h) image_give(st->sess->eng->device, st->img_h, st->img_d);
    release_slot(st);
    delete st;
    return 0;
  }
  g_evp_dev_ctx[dk].fetch_add(1, std::memory_order_relaxed);
  ctx->aead_state = st;
  return 1;
}

static bool doorbell_scrub(const AeadState* st);
static bool doorbell_scrub_async(const AeadState* st);
static void evp_wait_scrub_of(const tlsgpu_sessions* t, uint32_t slot);
static const bool g_async_scrub = [] {
  const char* v = getenv("TLSGPU_EVP_ASYNC_SCRUB");
  return !(v && *v == '0');
}();
extern "C" void EVP_AEAD_CTX_cleanup(EVP_AEAD_CTX* ctx) {
  if (ctx->aead == nullptr) return;
  auto* st = (AeadState*)ctx->aead_state;
  if (st) {
    const int img = st->image.load(std::memory_order_acquire);
    if (img == kImagePoisoned) {
      // an install job that never answered may still copy the image into the
      // slot: leak both (never reused, as stg->abandon() leaks staging) —
      // no scrub either, its synchronous fallback would wait on that device
      delete st;
      ctx->aead_state = nullptr;
      ctx->aead = nullptr;
      return;
    }
    if (img == 1) {
      // deferred and never called: no key material reached the device
      image_give(st->sess->eng->device, st->img_h, st->img_d);
    } else if (g_async_scrub && doorbell_scrub_async(st)) {
      // posted: the slot goes back once the server has answered (sweep_scrubs)
      delete st;
      ctx->aead_state = nullptr;
      ctx->aead = nullptr;
      return;
    } else if (!doorbell_scrub(st)) {
      // scrub the device key material before the slot is reused
      // (explicit_bzero analogue, e_aes.c:1415-1422), on this thread's stream
      scrub_slot(st->sess, st->slot);
    }
    release_slot(st);
    delete st;
  }
  ctx->aead_state = nullptr;
  ctx->aead = nullptr;
}

// Test support (include/tlsgpu.h): where a live EVP context's key material
// sits, and the bytes of a session slot once every queued install / scrub of
// that slot has finished — so a test can check that EVP_AEAD_CTX_cleanup's
// asynchronous scrub really zeroes the device copy (e_aes.c:1415-1422).
extern "C" int tlsgpu_evp_context_slot(const EVP_AEAD_CTX* ctx, tlsgpu_sessions** sessions,
                                       uint32_t* slot) {
  const auto* st = ctx ? (const AeadState*)ctx->aead_state : nullptr;
  if (!st || !sessions || !slot) return fail(TLSGPU_EINVAL, "no live EVP context");
  *sessions = st->sess;
  *slot = st->slot;
  return TLSGPU_OK;
}

extern "C" int tlsgpu_sessions_debug_read(tlsgpu_sessions* t, uint32_t slot, uint8_t* out,
                                          size_t n) {
  if (!t || !out || slot >= t->capacity || n > sizeof(DevSession) + sizeof(DevGcmTables))
    return fail(TLSGPU_EINVAL, "bad slot read");
  evp_wait_scrub_of(t, slot);  // an asynchronous cleanup scrub of this slot (round 6)
  HIPCHK(hipSetDevice(t->eng->device));
  if (const hipEvent_t ev = slot_event(t, slot)) HIPCHK(hipEventSynchronize(ev));
  const size_t a = std::min(n, sizeof(DevSession));
  HIPCHK(hipMemcpy(out, t->d_sess + slot, a, hipMemcpyDeviceToHost));
  if (n > a) HIPCHK(hipMemcpy(out + a, t->d_gcm + slot, n - a, hipMemcpyDeviceToHost));
  return TLSGPU_OK;
}

static int check_alias(const unsigned char* in, size_t in_len, const unsigned char* out) {
  if (out <= in) return 1;
  if (in + in_len <= out) return 1;
  return 0;
}

// EVP calls whose cipher work ran on the GPU (tlsgpu_evp_call_stats), and per
// EVP device (tlsgpu_evp_device_stats).
static std::atomic<uint64_t> g_evp_calls[2];  // [0] open, [1] seal


extern "C" int tlsgpu_evp_call_stats(uint64_t* seal_calls, uint64_t* open_calls) {
  if (seal_calls) *seal_calls = g_evp_calls[1].load();
  if (open_calls) *open_calls = g_evp_calls[0].load();
  return TLSGPU_OK;
}

extern "C" int tlsgpu_evp_device_stats(uint32_t k, int* device, uint64_t* contexts,
                                       uint64_t* calls) {
  if (k >= evp_device_count()) return fail(TLSGPU_ERANGE, "EVP device %u of %zu", k,
                                           evp_device_count());
  if (device) {
    std::lock_guard<std::mutex> lk(g_mu);
    *device = evp_devices_locked()[k];
  }
  if (contexts) *contexts = g_evp_dev_ctx[k].load();
  if (calls) *calls = g_evp_dev_calls[k].load();
  return TLSGPU_OK;
}

extern "C" uint32_t tlsgpu_evp_device_count(void) { return (uint32_t)evp_device_count(); }

static int gpu_call_impl(const AeadState* st, bool seal, unsigned char* out, size_t* out_len,
                         size_t max_out_len, const unsigned char* nonce, size_t nonce_len,
                         const unsigned char* in, size_t in_len, const unsigned char* ad,
                         size_t ad_len);

static const bool g_evp_zerocopy = [] {
  const char* v = getenv("TLSGPU_EVP_ZEROCOPY");
  return !(v && *v == '0');
}();

// ---------------------------------------------------------------------------
// Doorbell server (round 4, evp_server.hip): per-call AES-GCM and RFC 7539
// ChaCha20-Poly1305 jobs without a kernel launch.  TLSGPU_EVP_DOORBELL=<G> (or tlsgpu_evp_set_doorbell) keeps G
// server workgroups resident per EVP device while calls arrive; a calling
// thread owns one slot of kSlotsPerGroup * G (slot k -> workgroup k % G), posts
// its job number there and spins on the answer.  An instance lives `lifetime`
// (TLSGPU_EVP_DOORBELL_MS, default 5 ms) and is relaunched by the first post
// after half of that has passed, on the same stream: a job is only posted
// while an instance that still polls for at least half a lifetime is queued or
// running, so every posted job is served, and a process that stops calling
// leaves nothing spinning.  AES-GCM, RFC 7539 and (round 5) draft ChaCha20-
// Poly1305 jobs; pooled (queued) contexts keep the launched path; a context's first call carries its
// deferred install (the host-built image, defer_install) and its cleanup posts
// a scrub job; a short GCM job's input is staged into LDS by the server's idle
// waves.  On by default (round 5, kDoorbellDefaultGroups).
// The lifetime is short on purpose: this box runs at most GPU_MAX_HW_QUEUES = 4
// hardware queues per process, so with more streams than that (engine + 4 call
// streams + server) the server's queue is shared, and a kernel launched on a
// stream that shares it waits until the running instance exits
// (tools/doorbell_probe.hip: 2.7 s behind a 3 s instance with 8 other streams).
// 5 ms bounds that wait; relaunching every 2.5 ms under load costs one launch.
constexpr uint32_t kSlotsPerGroup = 8;
struct EvpServer {
  int device = -1;
  uint32_t groups = 0, nslots = 0;
  uint64_t lifetime_ns = 0;
  DoorbellSlot* slots = nullptr;  // pinned host
  DoorbellSlot* d_slots = nullptr;
  uint32_t* stop = nullptr;       // pinned host word
  uint32_t* d_stop = nullptr;
  hipStream_t stream = nullptr;
  std::mutex mu;
  std::atomic<uint64_t> deadline_ns{0};  // post only before this (host clock), else relaunch
  uint64_t end_ns = 0;                   // when the last queued instance stops polling, at the
                                         // earliest (host clock; under mu)
  std::vector<uint32_t> free_slots;
  std::atomic<uint64_t> jobs{0}, launches{0};
  // threads holding a slot, and 1 + the highest slot ever handed out: an
  // instance is launched with as many workgroups as there are calling
  // threads (at most `groups`), and enough that its 64 polling lanes per
  // workgroup cover every slot in use
  std::atomic<uint32_t> active{0}, hi_slot{0};
  std::atomic<uint32_t> covered{0};  // slots the last launched instance polls (64 per workgroup)
  std::atomic<uint32_t> last_launched_g{0};  // workgroups of the last launched instance
  uint32_t launch_seq = 0, last_g = 0;  // the last launched instance (under mu)
  // every launched instance whose workgroups have not all been seen leaving:
  // (launch number, workgroups), oldest first (under mu; pruned at each launch)
  std::vector<std::pair<uint32_t, uint32_t>> outstanding;
  // TLSGPU_EVP_DOORBELL_TRACE=1: per-slot device timestamps (pinned) and their
  // sums, printed at exit: pick -> slot loaded -> job done -> released (ticks
  // of 10 ns), and the caller's post -> done-seen wall time (ns)
  uint64_t* d_scrubs = nullptr;  // HBM: the scrub ring (ServerArgs::scrubs)
  // asynchronous cleanup scrubs (round 6): a status word per doorbell slot
  // (pinned) and the scrubs posted but not yet seen done, whose session slots
  // go back to their slab only then
  int32_t* scrub_status = nullptr;
  int32_t* d_scrub_status = nullptr;
  struct PendingScrub {
    tlsgpu_sessions* sess;
    uint32_t slot;
    size_t evp_dev;
    DoorbellSlot* ds;
    uint32_t post;
    uint64_t t0;
  };
  std::mutex pend_mu;
  std::vector<PendingScrub> pending;
  std::atomic<uint32_t> npending{0};  // pending.size(), read without the lock
  uint64_t* trace = nullptr;
  uint64_t* d_trace = nullptr;
  std::atomic<uint64_t> tr_n{0}, tr_load{0}, tr_job{0}, tr_rel{0}, tr_host_ns{0};
  std::atomic<uint64_t> tr_marks_n{0}, tr_phase[8] = {};  // GCM jobs: loaded -> mark 0 .. 6 -> done
  std::atomic<uint64_t> tr_last[4] = {};  // since loaded: wave 0 blocks / shoup, last wave blocks / shoup
  std::atomic<uint64_t> tr_inst_n{0}, tr_inst[2] = {};  // install jobs: loaded -> image read -> tables built
};
static EvpServer* g_servers[kMaxEvpDevices] = {};
// the servers whose setup succeeded, read without the lock on every call (a
// process-wide mutex per call cost 16 calling threads more than the call)
static std::atomic<EvpServer*> g_ready_servers[kMaxEvpDevices] = {};
constexpr uint32_t kExitedWord = 32;  // exit marks after the stop word (256 workgroups max)
static std::mutex g_server_mu;
// On by default (round 5), G = 64: TLSGPU_EVP_DOORBELL=0 or
// tlsgpu_evp_set_doorbell(0, 0) turns it off.  The round-4 exit SIGSEGV is
// explained and removed (thread-exit destructors made HIP
// calls; the shutdown contract below drains every instance).  Design grounds:
// the EVP surface's users are per-call callers (an unchanged libssl under
// LD_PRELOAD), for whom the doorbell is 1.5-6x the launched path and makes
// init / cleanup launch-free; a process that never calls EVP never creates a
// server; an instance holds only as many CUs as calling threads (<= G), and
// only while calls arrive plus one lifetime (5 ms).
constexpr unsigned kDoorbellDefaultGroups = 64;
static unsigned g_doorbell_groups = [] {
  const char* v = getenv("TLSGPU_EVP_DOORBELL");
  return v && *v ? (unsigned)strtoul(v, nullptr, 10) : kDoorbellDefaultGroups;
}();
static unsigned g_doorbell_ms = [] {
  const char* v = getenv("TLSGPU_EVP_DOORBELL_MS");
  const unsigned ms = v && *v ? (unsigned)strtoul(v, nullptr, 10) : 5u;
  return ms ? ms : 5u;
}();

static uint64_t mono_ns() {
  return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

// stop every server at exit: one host store each (no HIP call: the runtime
// may already be going away); an instance exits within one poll
// A waiting caller spins this long before it starts yielding the core
// (TLSGPU_EVP_DOORBELL_YIELD_US, default 100): with more calling threads than
// cores, spinners keep the threads that would post from running.
static const uint64_t g_doorbell_yield_ns = [] {
  const char* v = getenv("TLSGPU_EVP_DOORBELL_YIELD_US");
  return (v && *v ? (uint64_t)strtoull(v, nullptr, 10) : 100ull) * 1000ull;
}();

// Test hook (tests/test_evp_doorbell.py): sleep this long between a call's
// server_ensure and its post, as a caller descheduled there would.
// Test hook (TLSGPU_TEST_FAIL_INSTALLS=k): the first k calls that claim a
// deferred install fail before posting it (waiters must re-claim).
static std::atomic<int> g_test_fail_installs{[] {
  const char* v = getenv("TLSGPU_TEST_FAIL_INSTALLS");
  return v ? atoi(v) : 0;
}()};
static const unsigned g_test_post_delay_us = [] {
  const char* v = getenv("TLSGPU_TEST_DOORBELL_POST_DELAY_US");
  return v && *v ? (unsigned)strtoul(v, nullptr, 10) : 0u;
}();

static const bool g_doorbell_trace = [] {
  const char* v = getenv("TLSGPU_EVP_DOORBELL_TRACE");
  return v && *v && *v != '0';
}();

// ---------------------------------------------------------------------------
// Shutdown contract (round 5).
// A server instance reads and writes pinned host memory (its slots, the stop
// page, the callers' staging) for as long as it runs, and instances queue on
// the server's stream (and on whatever shares its hardware queue).  Before
// the HIP runtime tears down — it frees every pinned allocation — every
// instance ever launched must have left.  tlsgpu_evp_shutdown():
//   1. no new instance and no new post from here on (g_evp_shutdown);
//   2. the stop word of every server: a running instance leaves within 16
//      polls or after the job it is on, a queued one at its first instruction;
//   3. waits for EVERY outstanding instance's exit marks (not only the last
//      one's), reading pinned memory only — no HIP call — with no silent cap:
//      a note on stderr after 1 s, TLSGPU_ETIMEOUT after TLSGPU_EVP_SHUTDOWN_MS
//      (default 60,000);
//   4. callers still spinning on a post see the drain and take the launched
//      path for that call if no instance served it.
// It runs at the earliest point of process exit (a thread-local guard of the
// main thread: thread-local destructors of the exiting thread run before any
// atexit or static destructor, so before the runtime's), again from an atexit
// handler (exit from another thread) and from the library destructor
// (dlclose); it is idempotent.  At exit a drain that timed out ends the
// process with _exit(70) before the runtime's teardown can free memory a
// still-running instance uses.
static std::atomic<int> g_evp_shutdown{0};  // 0 running, 1 stopping, 2 drained
static std::mutex g_shutdown_mu;
static const uint64_t g_shutdown_cap_ns = [] {
  const char* v = getenv("TLSGPU_EVP_SHUTDOWN_MS");
  const uint64_t ms = v && *v ? strtoull(v, nullptr, 10) : 60000ull;
  return (ms ? ms : 60000ull) * 1000000ull;
}();
static const bool g_shutdown_verbose = [] {
  const char* v = getenv("TLSGPU_EVP_SHUTDOWN_VERBOSE");
  return v && *v && *v != '0';
}();

// Every workgroup of instance `seq` (g workgroups) has left.  A workgroup
// stores its instance's launch number into exited[b] as its last act;
// instances of one server run one after another on its stream, so a mark
// >= seq (wrapping compare) means workgroup b of this instance or of a later
// one — which only started after this one ended — has left.
static bool instance_left(const EvpServer* sv, uint32_t seq, uint32_t g) {
  for (uint32_t b = 0; b < g; b++)
    if ((int32_t)(__atomic_load_n(sv->stop + kExitedWord + b, __ATOMIC_ACQUIRE) - seq) < 0)
      return false;
  return true;
}

static void print_doorbell_trace();

// Which exit hook is running (TLSGPU_CRASH_TRACE names it in a fault report):
// 0 running, 1 the main thread's exit guard, 2 atexit, 3 library destructor.
static volatile sig_atomic_t g_exit_phase = 0;
static void sweep_scrubs(EvpServer* sv, uint64_t wait_ns, const tlsgpu_sessions* only_t = nullptr,
                         uint32_t only_slot = 0);

extern "C" int tlsgpu_evp_shutdown(void) {
  std::lock_guard<std::mutex> lk(g_shutdown_mu);
  if (g_evp_shutdown.load(std::memory_order_acquire) == 2) return TLSGPU_OK;
  // cleanup scrubs still in flight are answered before the servers stop (up
  // to 2 s each server; they take microseconds)
  if (g_evp_shutdown.load(std::memory_order_acquire) == 0)
    for (EvpServer* sv : g_servers)
      if (sv && sv->slots && sv->npending.load(std::memory_order_relaxed) != 0)
        sweep_scrubs(sv, 2000000000ull);
  g_evp_shutdown.store(1, std::memory_order_seq_cst);
  for (EvpServer* sv : g_servers)
    if (sv && sv->stop) __atomic_store_n(sv->stop, 1u, __ATOMIC_SEQ_CST);
  const uint64_t t0 = mono_ns();
  bool noted = false;
  uint32_t waited = 0;
  for (EvpServer* sv : g_servers) {
    if (!sv || !sv->stop) continue;
    std::vector<std::pair<uint32_t, uint32_t>> pend;
    {
      // server_ensure checks g_evp_shutdown under this lock: no instance is
      // launched after this copy
      std::lock_guard<std::mutex> lk2(sv->mu);
      pend = sv->outstanding;
    }
    for (const auto& inst : pend) {
      waited++;
      while (!instance_left(sv, inst.first, inst.second)) {
        __builtin_ia32_pause();
        const uint64_t t = mono_ns() - t0;
        if (!noted && t > 1000000000ull) {
          fprintf(stderr,
                  "tlsgpu: waiting for doorbell server instance %u (%u workgroups) on device %d "
                  "to leave\n",
                  inst.first, inst.second, sv->device);
          noted = true;
        }
        if (t > g_shutdown_cap_ns)
          return fail(TLSGPU_ETIMEOUT,
                      "doorbell server instance %u on device %d still running after %llu ms",
                      inst.first, sv->device, (unsigned long long)(g_shutdown_cap_ns / 1000000));
      }
    }
    std::lock_guard<std::mutex> lk2(sv->mu);
    sv->outstanding.clear();
  }
  g_evp_shutdown.store(2, std::memory_order_release);
  if (g_shutdown_verbose)
    fprintf(stderr, "{\"evp_shutdown\": {\"instances_waited\": %u, \"ms\": %.3f}}\n", waited,
            (mono_ns() - t0) * 1e-6);
  print_doorbell_trace();
  return TLSGPU_OK;
}


// TLSGPU_CRASH_TRACE=1: a fatal signal prints the exit phase and a native
// backtrace before the default action (Python's faulthandler, when enabled
// after the library loaded, chains to this handler after its own dump).
// Async-signal-safe: fixed strings and a hand-rolled integer
// formatter through write(2); backtrace() was called once at install, so the
// unwinder (libgcc) is loaded before any fault and the handler does not
// dlopen or malloc.
static void write_str(const char* p) { (void)!write(2, p, strlen(p)); }
static void write_int(long v) {
  char d[24];
  int i = (int)sizeof d;
  const bool neg = v < 0;
  unsigned long u = neg ? 0ul - (unsigned long)v : (unsigned long)v;
  do {
    d[--i] = (char)('0' + u % 10);
    u /= 10;
  } while (u && i > 1);
  if (neg) d[--i] = '-';
  (void)!write(2, d + i, sizeof d - (size_t)i);
}
static void crash_report(int sig) {
  write_str("tlsgpu: fatal signal ");
  write_int(sig);
  write_str(" in exit phase ");
  write_int((long)g_exit_phase);
  write_str(" (0 running, 1 main-thread exit guard, 2 atexit, 3 library destructor)\n");
  void* fr[64];
  backtrace_symbols_fd(fr, backtrace(fr, 64), 2);
  signal(sig, SIG_DFL);
  raise(sig);
}
__attribute__((constructor)) static void install_crash_report() {
  const char* v = getenv("TLSGPU_CRASH_TRACE");
  if (!v || !*v || *v == '0') return;
  void* warm[2];
  (void)backtrace(warm, 2);  // loads the unwinder now, not inside the handler
  struct sigaction sa;
  memset(&sa, 0, sizeof sa);
  sa.sa_handler = crash_report;
  sa.sa_flags = SA_RESETHAND;
  for (int sig : {SIGSEGV, SIGBUS, SIGABRT, SIGILL, SIGFPE}) sigaction(sig, &sa, nullptr);
}

static void evp_shutdown_at_exit() {
  bool any = false;
  for (EvpServer* sv : g_servers) any = any || (sv && sv->stop);
  if (!any || tlsgpu_evp_shutdown() == TLSGPU_OK) return;
  fprintf(stderr, "tlsgpu: %s; leaving before the runtime's teardown (exit status 70)\n",
          tlsgpu_last_error());
  fflush(stderr);
  _exit(70);
}

// The main thread's exit guard: armed by the library constructor when it runs
// on the main thread (LD_PRELOAD, or a dlopen from the main thread), so its
// destructor runs among the main thread's thread-local destructors, first
// thing in exit().
namespace {
struct MainExitGuard {
  ~MainExitGuard() {
    g_exit_phase = 1;
    evp_shutdown_at_exit();
  }
};
}  // namespace
// The main thread's own staging set is destroyed among its thread-local
// destructors at exit(), before the guard (constructed at load, so destroyed
// later): drain there first.
static void evp_shutdown_main_thread_exit() {
  if ((pid_t)syscall(SYS_gettid) != getpid()) return;
  g_exit_phase = 1;
  evp_shutdown_at_exit();
}
__attribute__((constructor)) static void arm_main_exit_guard() {
  if ((pid_t)syscall(SYS_gettid) != getpid()) return;
  static thread_local MainExitGuard guard;
  (void)&guard;
}
__attribute__((destructor)) static void evp_shutdown_at_unload() {
  g_exit_phase = 3;
  evp_shutdown_at_exit();
}
static void evp_shutdown_atexit() {
  g_exit_phase = 2;
  evp_shutdown_at_exit();
}

static void print_doorbell_trace() {
  for (EvpServer* sv : g_servers) {
    const uint64_t n = sv ? sv->tr_n.load() : 0;
    if (!n) continue;
    fprintf(stderr,
            "{\"doorbell_trace\": {\"jobs\": %llu, \"us_slot_load\": %.2f, \"us_job\": %.2f, "
            "\"us_release\": %.2f, \"us_host_round_trip\": %.2f}}\n",
            (unsigned long long)n, sv->tr_load.load() * 0.01 / n, sv->tr_job.load() * 0.01 / n,
            sv->tr_rel.load() * 0.01 / n, sv->tr_host_ns.load() * 1e-3 / n);
    const uint64_t m = sv->tr_marks_n.load();
    if (m) {  // gcm_raw.h TG_JOB_MARK phases
      static const char* names[8] = {"tables+barrier", "parse", "ctr_setup", "blocks",
                                     "close+shoup", "reduce+barrier", "ek0_aes", "tag"};
      fprintf(stderr, "{\"doorbell_gcm_phases_us\": {\"jobs\": %llu", (unsigned long long)m);
      for (int i = 0; i < 8; i++) fprintf(stderr, ", \"%s\": %.2f", names[i], sv->tr_phase[i].load() * 0.01 / m);
      fprintf(stderr, ", \"since_loaded_us\": {\"wave0_blocks\": %.2f, \"wave0_shoup\": %.2f, "
                      "\"last_wave_blocks\": %.2f, \"last_wave_shoup\": %.2f}}}\n",
              sv->tr_last[0].load() * 0.01 / m, sv->tr_last[1].load() * 0.01 / m,
              sv->tr_last[2].load() * 0.01 / m, sv->tr_last[3].load() * 0.01 / m);
      if (const uint64_t ni = sv->tr_inst_n.load())
        fprintf(stderr, "{\"doorbell_install_us\": {\"jobs\": %llu, \"image_read\": %.2f, "
                        "\"tables_built\": %.2f}}\n", (unsigned long long)ni,
                sv->tr_inst[0].load() * 0.01 / ni, sv->tr_inst[1].load() * 0.01 / ni);
    }
  }
}

// The server of EVP device k (created on first use when the doorbell is on).
static EvpServer* evp_server(size_t k, tlsgpu_engine* e) {
  if (!g_doorbell_groups || k >= (size_t)kMaxEvpDevices ||
      g_evp_shutdown.load(std::memory_order_acquire) != 0)
    return nullptr;
  if (EvpServer* ready = g_ready_servers[k].load(std::memory_order_acquire)) return ready;
  std::lock_guard<std::mutex> lk(g_server_mu);
  if (g_servers[k]) return g_servers[k]->slots ? g_servers[k] : nullptr;
  auto* sv = new (std::nothrow) EvpServer();
  if (!sv) return nullptr;
  g_servers[k] = sv;  // a failed setup stays registered (slots == nullptr): not retried
  sv->device = e->device;
  sv->groups = std::min(g_doorbell_groups, 256u);
  sv->nslots = sv->groups * kSlotsPerGroup;
  sv->lifetime_ns = (uint64_t)g_doorbell_ms * 1000000ull;
  DoorbellSlot* h = nullptr;
  uint32_t* stop = nullptr;
  if (hipSetDevice(e->device) != hipSuccess ||
      hipHostMalloc((void**)&h, sizeof(DoorbellSlot) * sv->nslots, hipHostMallocDefault) !=
          hipSuccess)
    return nullptr;
  memset(h, 0, sizeof(DoorbellSlot) * sv->nslots);
  // one pinned page: [0] the stop word, [kExitedWord + b] workgroup b's exit mark
  if (hipHostMalloc((void**)&stop, 4096, hipHostMallocDefault) != hipSuccess ||
      hipHostGetDevicePointer((void**)&sv->d_slots, h, 0) != hipSuccess ||
      hipHostGetDevicePointer((void**)&sv->d_stop, stop, 0) != hipSuccess ||
      hipStreamCreateWithFlags(&sv->stream, hipStreamNonBlocking) != hipSuccess ||
      hipMalloc((void**)&sv->d_scrubs, 8 * (kScrubRing + 2)) != hipSuccess ||
      hipMemset(sv->d_scrubs, 0, 8 * (kScrubRing + 2)) != hipSuccess) {
    (void)hipHostFree(h);
    if (stop) (void)hipHostFree(stop);
    return nullptr;
  }
  if (hipHostMalloc((void**)&sv->scrub_status, 4 * sv->nslots, hipHostMallocDefault) != hipSuccess ||
      hipHostGetDevicePointer((void**)&sv->d_scrub_status, sv->scrub_status, 0) != hipSuccess)
    sv->scrub_status = sv->d_scrub_status = nullptr;  // cleanup scrubs stay synchronous
  if (g_doorbell_trace &&
      (hipHostMalloc((void**)&sv->trace, 8 * kTraceWords * sv->nslots, hipHostMallocDefault) !=
           hipSuccess ||
       hipHostGetDevicePointer((void**)&sv->d_trace, sv->trace, 0) != hipSuccess))
    sv->trace = sv->d_trace = nullptr;
  memset(stop, 0, 4096);
  sv->stop = stop;
  for (uint32_t i = sv->nslots; i-- > 0;) sv->free_slots.push_back(i);
  sv->slots = h;
  static std::once_flag once;
  std::call_once(once, [] { atexit(evp_shutdown_atexit); });
  g_ready_servers[k].store(sv, std::memory_order_release);
  return sv;
}

// Launch an instance if the one queued last may stop polling within half a
// lifetime.  Returns false if the launch failed.
static bool server_ensure(EvpServer* sv) {
  const uint64_t now = mono_ns();
  if (now < sv->deadline_ns.load(std::memory_order_acquire)) return true;  // no lock per call
  std::lock_guard<std::mutex> lk(sv->mu);
  if (now < sv->deadline_ns.load(std::memory_order_relaxed)) return true;
  // the shutdown contract copies `outstanding` under this lock: nothing is
  // launched after it
  if (g_evp_shutdown.load(std::memory_order_acquire) != 0) return false;
  if (hipSetDevice(sv->device) != hipSuccess) return false;
  // forget instances that have left (the list stays a few entries long)
  sv->outstanding.erase(std::remove_if(sv->outstanding.begin(), sv->outstanding.end(),
                                       [sv](const std::pair<uint32_t, uint32_t>& i) {
                                         return instance_left(sv, i.first, i.second);
                                       }),
                        sv->outstanding.end());
  ServerArgs a;
  a.slots = sv->d_slots;
  // poll the slots handed out so far, rounded up to 16 (so that a burst of new
  // threads forces few relaunches): every poll is a PCIe read, and at 64
  // threads polling all 8 G slots was 8x the reads the calls needed
  const uint32_t hi = std::max(1u, sv->hi_slot.load(std::memory_order_acquire));
  a.nslots = std::min(sv->nslots, (hi + 15) & ~15u);
  a.stop = sv->d_stop;
  a.lifetime = sv->lifetime_ns / 10;  // 100 MHz realtime ticks
  a.trace = reinterpret_cast<unsigned long long*>(sv->d_trace);
  a.scrubs = reinterpret_cast<unsigned long long*>(sv->d_scrubs);
  a.exited = sv->d_stop + kExitedWord;
  a.seq = sv->launch_seq + 1;
  const uint32_t cover = (hi + kWave - 1) / kWave;
  const uint32_t g = std::min(sv->groups, std::max({1u, sv->active.load(std::memory_order_acquire), cover}));
  if (launch_evp_server(a, (int)g, sv->stream) != 0) return false;
  sv->launch_seq = a.seq;
  sv->last_g = g;
  sv->outstanding.emplace_back(a.seq, g);
  sv->covered.store(std::min(g * (uint32_t)kWave, a.nslots), std::memory_order_release);
  sv->last_launched_g.store(g, std::memory_order_release);
  // instances on one stream run one after another: this one starts when the
  // one queued before it ends (never before now) and polls for a lifetime
  // from then; post to it until half of that is left.  (Counting from the
  // launch instead queued a new instance every half lifetime behind ones
  // that each ran a whole lifetime: the queue grew without bound.)
  sv->end_ns = std::max(now, sv->end_ns) + sv->lifetime_ns;
  sv->deadline_ns.store(sv->end_ns - sv->lifetime_ns / 2, std::memory_order_release);
  sv->launches.fetch_add(1, std::memory_order_relaxed);
  return true;
}

// The calling thread's slot on a server (assigned on first use, given back
// when the thread exits); -1 when all are taken.
struct ThreadSlots {
  int slot[kMaxEvpDevices];
  uint32_t seq[kMaxEvpDevices];
  // a second slot for the thread's asynchronous cleanup scrubs (round 6): the
  // scrub runs while the thread's next call uses its own slot
  int scrub[kMaxEvpDevices];
  uint32_t scrub_seq[kMaxEvpDevices];
  ThreadSlots() {
    for (int& x : slot) x = -2;  // not asked yet
    for (int& x : scrub) x = -2;
  }
  ~ThreadSlots() {
    for (int k = 0; k < kMaxEvpDevices; k++) {
      if (!g_servers[k]) continue;
      std::lock_guard<std::mutex> lk(g_servers[k]->mu);
      if (slot[k] >= 0) {
        g_servers[k]->free_slots.push_back((uint32_t)slot[k]);
        g_servers[k]->active.fetch_sub(1, std::memory_order_release);
      }
      // a scrub slot with its last post still unanswered is not handed on
      // (its next owner would number from `done`): kept out of use
      if (scrub[k] >= 0) {
        g_servers[k]->active.fetch_sub(1, std::memory_order_release);
        if (__atomic_load_n(&g_servers[k]->slots[scrub[k]].done, __ATOMIC_ACQUIRE) == scrub_seq[k])
          g_servers[k]->free_slots.push_back((uint32_t)scrub[k]);
      }
    }
  }
};
static thread_local ThreadSlots t_slots;

static DoorbellSlot* thread_slot(EvpServer* sv, size_t k, uint32_t** seq) {
  int& s = t_slots.slot[k];
  if (s == -2) {
    std::lock_guard<std::mutex> lk(sv->mu);
    if (sv->free_slots.empty()) {
      s = -1;
    } else {
      s = (int)sv->free_slots.back();
      sv->free_slots.pop_back();
      sv->active.fetch_add(1, std::memory_order_release);
      if ((uint32_t)s + 1 > sv->hi_slot.load(std::memory_order_relaxed))
        sv->hi_slot.store((uint32_t)s + 1, std::memory_order_release);
      // a slot the queued instance does not poll: relaunch wider before the
      // first post (the caller's server_ensure follows)
      if ((uint32_t)s >= sv->covered.load(std::memory_order_acquire))
        sv->deadline_ns.store(0, std::memory_order_release);
      // continue the slot's numbering (an earlier thread may have used it)
      t_slots.seq[k] = __atomic_load_n(&sv->slots[s].done, __ATOMIC_ACQUIRE);
    }
  }
  if (s < 0) return nullptr;
  *seq = &t_slots.seq[k];
  return &sv->slots[s];
}

// The calling thread's scrub slot on a server (round 6; nullptr when none is
// free).  Its numbering continues from the slot's `done`, which equals its
// `post`: a slot is only ever handed on with no post outstanding.
static DoorbellSlot* thread_scrub_slot(EvpServer* sv, size_t k, uint32_t** seq) {
  int& s = t_slots.scrub[k];
  if (s == -2) {
    std::lock_guard<std::mutex> lk(sv->mu);
    if (sv->free_slots.empty()) {
      s = -1;
    } else {
      s = (int)sv->free_slots.back();
      sv->free_slots.pop_back();
      // counted as a caller: an instance then has a workgroup for it beside
      // the thread's own slot's (slot m is served by workgroup m mod G), so
      // the scrub runs while the thread's next call is served
      sv->active.fetch_add(1, std::memory_order_release);
      if ((uint32_t)s + 1 > sv->hi_slot.load(std::memory_order_relaxed))
        sv->hi_slot.store((uint32_t)s + 1, std::memory_order_release);
      if ((uint32_t)s >= sv->covered.load(std::memory_order_acquire) ||
          sv->active.load(std::memory_order_relaxed) > sv->last_launched_g.load(std::memory_order_relaxed))
        sv->deadline_ns.store(0, std::memory_order_release);
      t_slots.scrub_seq[k] = __atomic_load_n(&sv->slots[s].done, __ATOMIC_ACQUIRE);
    }
  }
  if (s < 0) return nullptr;
  *seq = &t_slots.scrub_seq[k];
  return &sv->slots[s];
}

static void slab_give(size_t dk, tlsgpu_sessions* t, uint32_t slot);
constexpr uint32_t kScrubSweepBatch = 32;  // pending scrubs before an init sweeps
// Give back the session slots whose cleanup scrub has been answered; wait up to
// `wait_ns` for the others (relaunching the server when an instance left before
// picking a post up).  With `only`, just the entries of that (table, slot).
static void sweep_scrubs(EvpServer* sv, uint64_t wait_ns, const tlsgpu_sessions* only_t,
                         uint32_t only_slot) {
  const uint64_t t0 = mono_ns();
  for (;;) {
    bool left = false, overdue = false;
    {
      // no wait asked: another thread's sweep does the work (init and cleanup
      // of many threads must not queue on this lock)
      std::unique_lock<std::mutex> lk(sv->pend_mu, std::defer_lock);
      if (wait_ns == 0) {
        if (!lk.try_lock()) return;
      } else {
        lk.lock();
      }
      auto& v = sv->pending;
      for (size_t i = 0; i < v.size();) {
        const auto& e = v[i];
        if ((int32_t)(__atomic_load_n(&e.ds->done, __ATOMIC_ACQUIRE) - e.post) >= 0) {
          slab_give(e.evp_dev, e.sess, e.slot);
          v[i] = v.back();
          v.pop_back();
          sv->npending.fetch_sub(1, std::memory_order_relaxed);
          continue;
        }
        if (!only_t || (e.sess == only_t && e.slot == only_slot)) left = true;
        if (mono_ns() - e.t0 > 2000000ull) overdue = true;  // 2 ms: look at the server
        i++;
      }
    }
    // (no launch from an exit hook: HIP calls there race the runtime's teardown)
    if (overdue && g_evp_shutdown.load(std::memory_order_acquire) == 0 && g_exit_phase == 0)
      (void)server_ensure(sv);
    if (!left || mono_ns() - t0 >= wait_ns) return;
    __builtin_ia32_pause();
    sched_yield();
  }
}

// EVP_AEAD_CTX_cleanup's scrub posted without waiting (round 6, VERDICT r05
// next-round 6: one-thread connection setup): the job goes to the thread's
// scrub slot and the session slot stays out of the free list until the server
// has answered, so no new context can install into it first.  false: not
// posted (no server / scrub slot, or the previous scrub on it still running
// after 10 s) — the caller scrubs synchronously.
static bool doorbell_scrub_async(const AeadState* st) {
  if (st->batcher || !g_evp_zerocopy || !doorbell_enabled() ||
      st->install_pending.load(std::memory_order_acquire))
    return false;
  tlsgpu_engine* e = st->sess->eng;
  EvpServer* sv = evp_server(st->evp_dev, e);
  if (!sv || !sv->scrub_status) return false;
  uint32_t* seq = nullptr;
  DoorbellSlot* ds = thread_scrub_slot(sv, st->evp_dev, &seq);
  if (!ds) return false;
  const uint64_t t0 = mono_ns();
  for (uint64_t spins = 1; __atomic_load_n(&ds->done, __ATOMIC_ACQUIRE) != *seq; spins++) {
    // the previous scrub on this slot (normally answered long ago)
    if (mono_ns() - t0 > 10000000000ull) return false;
    __builtin_ia32_pause();
    if ((spins & 255) == 0) {
      sweep_scrubs(sv, 0);  // relaunches the server if an instance left before picking it up
      sched_yield();
    }
  }
  if (!server_ensure(sv)) return false;
  const uint32_t idx = (uint32_t)(ds - sv->slots);
  sv->scrub_status[idx] = -1;
  ds->op = kDoorbellOpScrub << 8;
  ds->n_sessions = st->sess->capacity;
  memset(&ds->job, 0, sizeof(RawJob));
  ds->job.session = st->slot;
  ds->status = (uint64_t)(sv->d_scrub_status + idx);
  ds->sessions = (uint64_t)st->sess->d_sess;
  ds->gcm_tables = (uint64_t)st->sess->d_gcm;
  ds->key_id = st->key_id;
  const uint32_t n = ++*seq;
  {
    std::lock_guard<std::mutex> lk(sv->pend_mu);
    sv->pending.push_back({st->sess, st->slot, st->evp_dev, ds, n, mono_ns()});
    sv->npending.fetch_add(1, std::memory_order_relaxed);
  }
  __atomic_store_n(&ds->post, n, __ATOMIC_RELEASE);
  sv->jobs.fetch_add(1, std::memory_order_relaxed);
  return true;
}

// EVP_AEAD_CTX_init's look at device dk's answered scrubs (their slots back to
// the slab before it takes one); tlsgpu_sessions_debug_read's wait for a slot.
static void evp_sweep_scrubs_for(size_t dk) {
  if (dk >= (size_t)kMaxEvpDevices) return;
  EvpServer* sv = g_ready_servers[dk].load(std::memory_order_acquire);
  // answered scrubs' slots go back in batches: a sweep per init cost 16
  // calling threads ~10 us of lock hand-offs each (profiles/r06f_evp_churn)
  if (sv && sv->npending.load(std::memory_order_relaxed) >= kScrubSweepBatch) sweep_scrubs(sv, 0);
}
static void evp_wait_scrub_of(const tlsgpu_sessions* t, uint32_t slot) {
  for (size_t k = 0; k < (size_t)kMaxEvpDevices; k++) {
    EvpServer* sv = g_ready_servers[k].load(std::memory_order_acquire);
    if (sv && sv->npending.load(std::memory_order_relaxed) != 0)
      sweep_scrubs(sv, 10000000000ull, t, slot);
  }
}

extern "C" int tlsgpu_evp_set_doorbell(unsigned groups, unsigned lifetime_ms) {
  std::lock_guard<std::mutex> lk(g_server_mu);
  for (EvpServer* sv : g_servers)
    if (sv) return fail(TLSGPU_EINVAL, "the doorbell server is already set up");
  g_doorbell_groups = groups;
  if (lifetime_ms) g_doorbell_ms = lifetime_ms;
  return TLSGPU_OK;
}

extern "C" int tlsgpu_evp_doorbell_warm(void) {
  if (!g_doorbell_groups || g_evp_shutdown.load(std::memory_order_acquire) != 0) return TLSGPU_OK;
  for (size_t k = 0; k < evp_device_count() && k < (size_t)kMaxEvpDevices; k++) {
    tlsgpu_engine* e = evp_engine(k);
    EvpServer* sv = e ? evp_server(k, e) : nullptr;
    if (sv && !server_ensure(sv) && g_evp_shutdown.load() == 0)
      return fail(TLSGPU_EHIP, "doorbell server launch on EVP device %zu", k);
  }
  return TLSGPU_OK;
}

extern "C" int tlsgpu_evp_doorbell_stats(uint64_t* jobs, uint64_t* launches) {
  uint64_t j = 0, l = 0;
  for (EvpServer* sv : g_servers)
    if (sv) {
      j += sv->jobs.load();
      l += sv->launches.load();
    }
  if (jobs) *jobs = j;
  if (launches) *launches = l;
  return TLSGPU_OK;
}

extern "C" int tlsgpu_evp_doorbell_scrub_stats(uint64_t* scrubs, uint64_t* flushes) {
  uint64_t n = 0, f = 0;
  for (EvpServer* sv : g_servers)
    if (sv && sv->d_scrubs) {
      uint64_t w[2] = {0, 0};
      if (hipSetDevice(sv->device) != hipSuccess ||
          hipMemcpy(&w[0], sv->d_scrubs, 8, hipMemcpyDeviceToHost) != hipSuccess ||
          hipMemcpy(&w[1], sv->d_scrubs + 1 + kScrubRing, 8, hipMemcpyDeviceToHost) != hipSuccess)
        return fail(TLSGPU_EHIP, "scrub stats");
      n += w[0];
      f += w[1];
    }
  if (scrubs) *scrubs = n;
  if (flushes) *flushes = f;
  return TLSGPU_OK;
}

// One EVP call on the GPU: 1 = success, 0 = authentication failure / rejected
// by the kernel (output zero-filled), -1 = runtime failure.
static int gpu_call(const AeadState* st, bool seal, unsigned char* out, size_t* out_len,
                    size_t max_out_len, const unsigned char* nonce, size_t nonce_len,
                    const unsigned char* in, size_t in_len, const unsigned char* ad,
                    size_t ad_len) {
  int r = gpu_call_impl(st, seal, out, out_len, max_out_len, nonce, nonce_len, in, in_len, ad,
                        ad_len);
  if (r >= 0) {
    g_evp_calls[seal ? 1 : 0].fetch_add(1, std::memory_order_relaxed);
    g_evp_dev_calls[st->evp_dev].fetch_add(1, std::memory_order_relaxed);
  }
  return r;
}

static int evp_queue_call(EvpBatcher* b, const AeadState* st, bool seal, unsigned char* out,
                          size_t* out_len, size_t max_out_len, const unsigned char* nonce,
                          size_t nonce_len, const unsigned char* in, size_t in_len,
                          const unsigned char* ad, size_t ad_len);

// Wait for a per-call event: blocking (hipEventSynchronize), or with
// TLSGPU_EVP_SPIN=1 by polling hipEventQuery.  The probe had a host spin on
// the kernel's own completion word 5-6 µs faster than the blocking wait
// (tools/doorbell_probe.hip: 9.6 vs 15.4 µs for a 1,400-B job), but polling
// the event measured no better in the library (profiles/r04h_doorbell_bench:
// 36.1 vs 37.6 K calls/s at 1 thread, 42.0 vs 45.2 K at 64) and burns a core
// per waiting thread, so the blocking wait stays the default.
static const bool g_evp_spin = [] {
  const char* v = getenv("TLSGPU_EVP_SPIN");
  return v && *v && *v != '0';
}();
static bool event_spin(hipEvent_t ev) {
  if (!g_evp_spin) return hipEventSynchronize(ev) == hipSuccess;
  for (uint64_t spins = 1;; spins++) {
    const hipError_t q = hipEventQuery(ev);
    if (q == hipSuccess) return true;
    if (q != hipErrorNotReady) return false;
    __builtin_ia32_pause();
    if ((spins & 255) == 0 && spins > 4096) sched_yield();  // a long job: let others run
  }
}

// Post the job written into `slot` (the caller's doorbell slot on server sv,
// EVP device k) and wait for its answer.  1: served; 0: not served and never
// will be (shutdown) — take the launched path; -1: failure, nothing posted
// (launch failed); -2: posted but no answer in 10 s (the job may still run:
// the slot is retired and the staging abandoned).
static int doorbell_post_wait(EvpServer* sv, DoorbellSlot* slot, uint32_t* seq, size_t k,
                              Staging* stg, uint64_t* t0_out) {
  if (!server_ensure(sv)) {
    if (g_evp_shutdown.load(std::memory_order_acquire) == 0) return -1;  // launch failed
    return 0;  // shutting down: nothing was posted
  }
  const uint32_t n = ++*seq;
  const uint64_t t0 = mono_ns();
  *t0_out = t0;
  if (g_test_post_delay_us) usleep(g_test_post_delay_us);  // test hook: a descheduled caller
  __atomic_store_n(&slot->post, n, __ATOMIC_RELEASE);
  for (uint64_t spins = 1; __atomic_load_n(&slot->done, __ATOMIC_ACQUIRE) != n; spins++) {
    __builtin_ia32_pause();
    if ((spins & 127) == 0) {
      // the instance the post was meant for may have left before the post
      // landed (this thread descheduled between server_ensure and the store
      // for more than half a lifetime): past the deadline, relaunch — the new
      // instance picks the post up
      const int sd = g_evp_shutdown.load(std::memory_order_acquire);
      if (sd == 0 && !server_ensure(sv) && g_evp_shutdown.load() == 0) return -1;
      if (sd == 2) {  // drained: no instance will ever serve it
        if (__atomic_load_n(&slot->done, __ATOMIC_ACQUIRE) == n) return 1;
        t_slots.slot[k] = -1;  // this thread posts no more
        return 0;
      }
      const uint64_t waited = mono_ns() - t0;
      if (waited > 10000000000ull) {  // 10 s: the device is gone
        // the post stays outstanding: retire the slot (never handed out
        // again) and leave the staging buffer to the job that may still run
        // (never freed, never reused)
        t_slots.slot[k] = -1;
        stg->abandon();
        return -2;
      }
      if (waited > g_doorbell_yield_ns) sched_yield();  // let other callers post
    }
  }
  return 1;
}

static bool doorbell_enabled() {
  return g_doorbell_groups != 0 && g_evp_shutdown.load(std::memory_order_acquire) == 0;
}
static bool deferred_install_ok(int kind) {
  return g_deferred_install && !g_device_install && g_evp_zerocopy && doorbell_enabled() &&
         (kind == TLSGPU_AES_128_GCM || kind == TLSGPU_AES_256_GCM ||
          kind == TLSGPU_CHACHA20_POLY1305 || kind == TLSGPU_CHACHA20_POLY1305_OLD);
}

// EVP_AEAD_CTX_cleanup through the doorbell (round 5): a scrub job zeroes the
// slot on the device and the serving workgroup's LDS copies of this key,
// synchronously — no launch; the other server workgroups zero theirs when
// they next look at the scrub ring (round 6, evp_server.hip: before their
// next job, or within 16 idle polls).  false: no server / slot for this thread (the caller scrubs on a
// stream instead).
static bool doorbell_scrub(const AeadState* st) {
  if (st->batcher || !g_evp_zerocopy || !doorbell_enabled() ||
      st->install_pending.load(std::memory_order_acquire))
    return false;
  tlsgpu_engine* e = st->sess->eng;
  EvpServer* sv = evp_server(st->evp_dev, e);
  uint32_t* seq = nullptr;
  DoorbellSlot* slot = sv ? thread_slot(sv, st->evp_dev, &seq) : nullptr;
  Staging* stg = slot ? stage_for(e->device) : nullptr;
  if (!stg || !stg->ensure(e->device, 64) || !stg->h_dev) return false;
  int32_t* status = reinterpret_cast<int32_t*>(stg->h_buf);
  *status = -1;
  slot->op = kDoorbellOpScrub << 8;
  slot->n_sessions = st->sess->capacity;
  memset(&slot->job, 0, sizeof(RawJob));
  slot->job.session = st->slot;
  slot->status = (uint64_t)stg->h_dev;
  slot->sessions = (uint64_t)st->sess->d_sess;
  slot->gcm_tables = (uint64_t)st->sess->d_gcm;
  slot->key_id = st->key_id;
  uint64_t t0 = 0;
  return doorbell_post_wait(sv, slot, seq, st->evp_dev, stg, &t0) == 1 &&
         __atomic_load_n(status, __ATOMIC_ACQUIRE) == 0;
}

static int gpu_call_impl(const AeadState* st, bool seal, unsigned char* out, size_t* out_len,
                         size_t max_out_len, const unsigned char* nonce, size_t nonce_len,
                         const unsigned char* in, size_t in_len, const unsigned char* ad,
                         size_t ad_len) {
  // the context's key install (EVP_AEAD_CTX_init does not wait for it)
  const bool wait_install = st->install_pending.load(std::memory_order_acquire);
  if (st->batcher) {  // pooled context: join the coalescing queue (large jobs run alone)
    if (wait_install) {
      if (hipEventSynchronize(st->installed) != hipSuccess) return -1;
      st->install_pending.store(false, std::memory_order_release);
    }
    int r = evp_queue_call(st->batcher, st, seal, out, out_len, max_out_len, nonce, nonce_len,
                           in, in_len, ad, ad_len);
    if (r != -2) return r;
  }
  // a deferred install (EVP_AEAD_CTX_init, round 5): one caller installs the
  // image with its call, concurrent first callers wait for it; a failed call
  // leaves the image waiting (1) for the next caller — a waiter that sees it
  // back at 1 claims it itself.  Once the image's address has
  // reached the device (a posted doorbell job, a queued upload) a failure
  // poisons the context instead (3, kImagePoisoned): the job may still run, so
  // the image buffer and the slot are never handed to anyone else, and every
  // later call fails (a doorbell timeout).
  struct InstallClaim {
    const AeadState* st;
    bool active = false;
    bool posted = false;  // the device may read the image from now on
    ~InstallClaim() {
      if (active) st->image.store(posted ? kImagePoisoned : 1, std::memory_order_release);
    }
    void done() {  // on the device: the image buffer goes back, zeroed
      active = false;
      st->image.store(0, std::memory_order_release);
      image_give(st->sess->eng->device, st->img_h, st->img_d);
    }
  } claim{st};
  if (st->image.load(std::memory_order_acquire) != 0) {
    for (uint64_t spins = 1;; spins++) {
      int expect = 1;
      if (st->image.compare_exchange_strong(expect, 2, std::memory_order_acq_rel)) {
        claim.active = true;
        // the slot's previous owner's scrub, if it went through a stream
        if (hipEventQuery(st->slot_ev) != hipSuccess &&
            hipEventSynchronize(st->slot_ev) != hipSuccess)
          return -1;
        if (g_test_fail_installs.load(std::memory_order_relaxed) > 0 &&
            g_test_fail_installs.fetch_sub(1) > 0) {  // test hook: the claimer fails
          usleep(20000);  // with the other first callers waiting on it
          return -1;
        }
        break;
      }
      if (expect == 0) break;               // installed by the caller that claimed it
      if (expect == kImagePoisoned) return -1;
      // 2: another caller is installing right now
      __builtin_ia32_pause();
      if ((spins & 255) == 0) sched_yield();
      if (spins > (1ull << 34)) return -1;
    }
  }
  auto al = [](size_t v) { return (v + 15) & ~(size_t)15; };
  const size_t out_bytes = seal ? in_len + st->tag_len : std::max(max_out_len, in_len);
  const size_t o_nonce = al(sizeof(RawJob)), o_ad = o_nonce + al(nonce_len);
  const size_t o_in = o_ad + al(ad_len), o_status = o_in + al(in_len);
  const size_t o_out = o_status + 16, total = o_out + al(out_bytes + 1);
  tlsgpu_engine* e = st->sess->eng;
  Staging* stg = stage_for(e->device);
  if (!stg || !stg->ensure(e->device, total)) return -1;
  // zero-copy (round 3, default): the kernel reads the job from and writes its
  // status and output to the pinned staging buffer itself — no H2D / D2H
  // launches around a one-record batch; TLSGPU_EVP_ZEROCOPY=0 stages through HBM
  const bool zc = g_evp_zerocopy && stg->h_dev;
  if (!zc && !stg->ensure(e->device, total, true)) return -1;
  uint8_t* d = zc ? stg->h_dev : stg->d_buf;
  uint8_t* h = stg->h_buf;
  hipStream_t s = stg->stream;
  if (st->install_pending.load(std::memory_order_acquire) &&
      hipStreamWaitEvent(s, st->installed, 0) != hipSuccess)
    return -1;
  RawJob* j = reinterpret_cast<RawJob*>(h);
  j->in = (uint64_t)(d + o_in);
  j->out = (uint64_t)(d + o_out);
  j->nonce = (uint64_t)(d + o_nonce);
  j->aad = (uint64_t)(d + o_ad);
  j->in_len = (uint32_t)in_len;
  j->nonce_len = (uint32_t)nonce_len;
  j->aad_len = (uint32_t)ad_len;
  j->session = st->slot;
  j->max_out = max_out_len;
  if (nonce_len) memcpy(h + o_nonce, nonce, nonce_len);
  if (ad_len) memcpy(h + o_ad, ad, ad_len);
  if (in_len) memcpy(h + o_in, in, in_len);
  // a job the kernel rejects keeps this status (never a stale one)
  *reinterpret_cast<int32_t*>(h + o_status) = TLSGPU_REC_PUBLIC_INVALID;
  if (!zc && hipMemcpyAsync(d, h, o_status + 4, hipMemcpyHostToDevice, s) != hipSuccess) return -1;
  const bool gcm = st->kind == TLSGPU_AES_128_GCM || st->kind == TLSGPU_AES_256_GCM;
  // doorbell (zero-copy AES-GCM and RFC 7539 ChaCha20-Poly1305 calls): post
  // the job to a resident server workgroup instead of launching; the staging
  // buffer is the job's memory
  if (zc && (gcm || st->kind == TLSGPU_CHACHA20_POLY1305 ||
             st->kind == TLSGPU_CHACHA20_POLY1305_OLD)) {
    EvpServer* sv = evp_server(st->evp_dev, e);
    uint32_t* seq = nullptr;
    DoorbellSlot* slot = sv ? thread_slot(sv, st->evp_dev, &seq) : nullptr;
    // a context's first call, its key install still queued, takes the
    // launched path below (ordered after the install on the device, no host
    // wait): waiting for the install here halved connection churn at 16
    // threads (profiles/r04l_doorbell_bench.jsonl: 17.7 vs 43.7 K/s)
    if (slot && !st->install_pending.load(std::memory_order_acquire)) {
      // the job travels in the slot (one wave load brings it to the server),
      // nonce and AAD inline when they fit
      // (an installing call carries the image's address in `inl` instead)
      const bool inl = !claim.active && nonce_len + ad_len <= kDoorbellInline;
      const uint32_t kop = st->kind == TLSGPU_AES_128_GCM   ? 10u
                           : st->kind == TLSGPU_AES_256_GCM ? 14u
                           : st->kind == TLSGPU_CHACHA20_POLY1305 ? 20u
                                                                  : 21u;  // draft ChaCha
      slot->op = (uint32_t)(seal ? 1 : 0) | (kop << 8) | (inl ? 1u << 16 : 0u) |
                 (claim.active ? kDoorbellOpInstall : 0u) |
                 (claim.active && st->img_tables ? kDoorbellOpInstallTables : 0u);
      slot->n_sessions = st->sess->capacity;
      memcpy(&slot->job, j, sizeof(RawJob));
      if (inl) {
        if (nonce_len) memcpy(slot->inl, nonce, nonce_len);
        if (ad_len) memcpy(slot->inl + nonce_len, ad, ad_len);
      } else if (claim.active) {
        const uint64_t img = (uint64_t)st->img_d;
        memcpy(slot->inl, &img, sizeof(img));
      }
      slot->status = (uint64_t)(d + o_status);
      slot->sessions = (uint64_t)st->sess->d_sess;
      slot->gcm_tables = (uint64_t)st->sess->d_gcm;
      slot->key_id = st->key_id;
      uint64_t t0 = 0;
      const int pr = doorbell_post_wait(sv, slot, seq, st->evp_dev, stg, &t0);
      if (pr == -2) claim.posted = true;  // unanswered: the job may still copy the image
      if (pr < 0) return -1;
      if (pr == 0) goto launched;
      if (claim.active) claim.done();
      sv->jobs.fetch_add(1, std::memory_order_relaxed);
      if (sv->trace) {
        const uint64_t* tr = sv->trace + kTraceWords * (size_t)(slot - sv->slots);
        sv->tr_n.fetch_add(1, std::memory_order_relaxed);
        sv->tr_load.fetch_add(tr[1] - tr[0], std::memory_order_relaxed);
        sv->tr_job.fetch_add(tr[9] - tr[1], std::memory_order_relaxed);
        sv->tr_rel.fetch_add(tr[10] - tr[9], std::memory_order_relaxed);
        sv->tr_host_ns.fetch_add(mono_ns() - t0, std::memory_order_relaxed);
        bool all = true;
        for (int i = 2; i < 9; i++) all = all && tr[i] >= tr[i - 1];
        if (all && tr[9] >= tr[8]) {
          sv->tr_marks_n.fetch_add(1, std::memory_order_relaxed);
          for (int i = 0; i < 8; i++)
            sv->tr_phase[i].fetch_add(tr[i + 2] - tr[i + 1], std::memory_order_relaxed);
          const uint64_t lw_b = tr[11] >= tr[1] ? tr[11] - tr[1] : 0, lw_s = tr[12] >= tr[1] ? tr[12] - tr[1] : 0;
          sv->tr_last[0].fetch_add(tr[5] - tr[1], std::memory_order_relaxed);
          sv->tr_last[1].fetch_add(tr[6] - tr[1], std::memory_order_relaxed);
          sv->tr_last[2].fetch_add(lw_b, std::memory_order_relaxed);
          sv->tr_last[3].fetch_add(lw_s, std::memory_order_relaxed);
          if (tr[13] >= tr[1] && tr[14] >= tr[13] && tr[13] != 0) {  // an install job (round 6)
            sv->tr_inst_n.fetch_add(1, std::memory_order_relaxed);
            sv->tr_inst[0].fetch_add(tr[13] - tr[1], std::memory_order_relaxed);
            sv->tr_inst[1].fetch_add(tr[14] - tr[13], std::memory_order_relaxed);
          }
        }
      }
      const int32_t status = *reinterpret_cast<const int32_t*>(h + o_status);
      if (status < 0) {  // the kernel's zero-fill of max_out_len bytes (evp_aead.c:137-143)
        if (max_out_len) memset(out, 0, max_out_len);
        return 0;
      }
      if (status) memcpy(out, h + o_out, (size_t)status);
      *out_len = (size_t)status;
      return 1;
    }
  }
launched:
  BatchArgs a = {};
  a.sessions = st->sess->d_sess;
  a.gcm_tables = st->sess->d_gcm;
  a.descs = d;
  a.n = 1;
  a.records_per_group = 1;
  a.status = reinterpret_cast<int32_t*>(d + o_status);
  a.n_sessions = st->sess->capacity;
  // a deferred install on the launched path: one upload kernel ahead of the job
  if (claim.active) {
    if (hipStreamWaitEvent(s, st->slot_ev, 0) != hipSuccess) return -1;
    if (st->img_compact)  // the upload copies whole Shoup tables
      host_image_complete(reinterpret_cast<DevGcmTables*>(st->img_h + sizeof(DevSession)));
    claim.posted = true;  // queued from here on, whatever fails after it
    if (launch_upload_session(st->img_d, st->sess->d_sess + st->slot, st->sess->d_gcm + st->slot,
                              st->img_tables ? kGcmTableUploadBytes : 0u, s) != 0)
      return -1;
  }
  int rc = gcm ? launch_gcm(a, seal, true, st->kind == TLSGPU_AES_128_GCM ? 10 : 14, 1, s)
               : launch_chacha(a, seal, true, true, true, s);
  if (rc) return -1;
  // success writes at most in_len + tag (seal) / in_len - tag (open) bytes
  const size_t back = seal ? in_len + st->tag_len : std::min(max_out_len, in_len);
  if ((!zc && hipMemcpyAsync(h + o_status, d + o_status, o_out - o_status + back,
                             hipMemcpyDeviceToHost, s) != hipSuccess) ||
      hipEventRecord(stg->done, s) != hipSuccess || !event_spin(stg->done))
    return -1;
  st->install_pending.store(false, std::memory_order_release);  // done before this call's work
  if (claim.active) claim.done();
  if (stg->any_dirty_key_area()) stg->sweep_key_areas();  // this context's image, copied by now
  const int32_t status = *reinterpret_cast<const int32_t*>(h + o_status);
  if (status < 0) {  // the kernel's zero-fill of max_out_len bytes (evp_aead.c:137-143)
    if (max_out_len) memset(out, 0, max_out_len);
    return 0;
  }
  if (status) memcpy(out, h + o_out, (size_t)status);
  *out_len = (size_t)status;
  return 1;
}

extern "C" int EVP_AEAD_CTX_seal(const EVP_AEAD_CTX* ctx, unsigned char* out, size_t* out_len,
                                 size_t max_out_len, const unsigned char* nonce, size_t nonce_len,
                                 const unsigned char* in, size_t in_len, const unsigned char* ad,
                                 size_t ad_len) {
  const AeadState* st = (const AeadState*)ctx->aead_state;
  size_t possible_out_len = in_len + ctx->aead->overhead;
  bool gcm = ctx->aead->kind == TLSGPU_AES_128_GCM || ctx->aead->kind == TLSGPU_AES_256_GCM;
  int r;
  if (possible_out_len < in_len) {  // evp_aead.c:96-100
    evp_err(F_AEAD_CTX_SEAL, R_TOO_LARGE);
    goto error;
  }
  if (!check_alias(in, in_len, out)) {
    evp_err(F_AEAD_CTX_SEAL, R_OUTPUT_ALIASES_INPUT);
    goto error;
  }
  if (!st) goto error;
  if (gcm) {
    if (max_out_len < in_len + st->tag_len) {  // e_aes.c:1434-1437
      evp_err(F_AEAD_AES_GCM_SEAL, R_BUFFER_TOO_SMALL);
      goto error;
    }
    if (in_len > TLSGPU_MAX_RECORD * 64ull || ad_len > TLSGPU_MAX_RECORD * 64ull) goto error;
  } else {
    if ((uint64_t)in_len >= (1ull << 32) * 64 - 64) {  // e_chacha20poly1305.c:144-147
      evp_err(F_AEAD_CHACHA20_POLY1305_SEAL, R_TOO_LARGE);
      goto error;
    }
    if (max_out_len < in_len + st->tag_len) {
      evp_err(F_AEAD_CHACHA20_POLY1305_SEAL, R_BUFFER_TOO_SMALL);
      goto error;
    }
    if (nonce_len != ctx->aead->nonce_len) {
      evp_err(F_AEAD_CHACHA20_POLY1305_SEAL, R_IV_TOO_LARGE);
      goto error;
    }
  }
  r = gpu_call(st, true, out, out_len, max_out_len, nonce, nonce_len, in, in_len, ad, ad_len);
  if (r == 1) return 1;
error:
  memset(out, 0, max_out_len);  // evp_aead.c:113-118
  *out_len = 0;
  return 0;
}

extern "C" int EVP_AEAD_CTX_open(const EVP_AEAD_CTX* ctx, unsigned char* out, size_t* out_len,
                                 size_t max_out_len, const unsigned char* nonce, size_t nonce_len,
                                 const unsigned char* in, size_t in_len, const unsigned char* ad,
                                 size_t ad_len) {
  const AeadState* st = (const AeadState*)ctx->aead_state;
  bool gcm = ctx->aead->kind == TLSGPU_AES_128_GCM || ctx->aead->kind == TLSGPU_AES_256_GCM;
  int r;
  if (!check_alias(in, in_len, out)) {
    evp_err(F_AEAD_CTX_OPEN, R_OUTPUT_ALIASES_INPUT);
    goto error;
  }
  if (!st) goto error;
  if (gcm) {
    if (in_len < st->tag_len) {  // e_aes.c:1473-1476
      evp_err(F_AEAD_AES_GCM_OPEN, R_BAD_DECRYPT);
      goto error;
    }
    if (max_out_len < in_len - st->tag_len) {
      evp_err(F_AEAD_AES_GCM_OPEN, R_BUFFER_TOO_SMALL);
      goto error;
    }
    if (in_len > TLSGPU_MAX_RECORD * 64ull || ad_len > TLSGPU_MAX_RECORD * 64ull) goto error;
  } else {
    if (in_len < st->tag_len) {  // e_chacha20poly1305.c:223-226
      evp_err(F_AEAD_CHACHA20_POLY1305_OPEN, R_BAD_DECRYPT);
      goto error;
    }
    if ((uint64_t)in_len >= (1ull << 32) * 64 - 64) {
      evp_err(F_AEAD_CHACHA20_POLY1305_OPEN, R_TOO_LARGE);
      goto error;
    }
    if (nonce_len != ctx->aead->nonce_len) {
      evp_err(F_AEAD_CHACHA20_POLY1305_OPEN, R_IV_TOO_LARGE);
      goto error;
    }
    if (max_out_len < in_len - st->tag_len) {
      evp_err(F_AEAD_CHACHA20_POLY1305_OPEN, R_BUFFER_TOO_SMALL);
      goto error;
    }
  }
  r = gpu_call(st, false, out, out_len, max_out_len, nonce, nonce_len, in, in_len, ad, ad_len);
  if (r == 1) return 1;
  evp_err(gcm ? F_AEAD_AES_GCM_OPEN : F_AEAD_CHACHA20_POLY1305_OPEN, R_BAD_DECRYPT);
error:
  memset(out, 0, max_out_len);  // evp_aead.c:137-143
  *out_len = 0;
  return 0;
}

// ---------------------------------------------------------------------------
// Legacy EVP_CIPHER GCM surface (crypto/evp/e_aes.c:687-1059).
// The object's function pointers are called by the generic EVP_Cipher* code of
// whatever libcrypto the application links; the cipher work runs as programs
// of GCM128 steps on the gcm_stream kernel (one launch per call).
namespace {
enum {
  kCtrlInit = 0x0, kCtrlCopy = 0x8, kGcmSetIvlen = 0x9, kGcmGetTag = 0x10, kGcmSetTag = 0x11,
  kGcmSetIvFixed = 0x12, kGcmIvGen = 0x13, kAeadTls1Aad = 0x16, kGcmSetIvInv = 0x18,
  kTlsExplicitIv = 8, kTlsTag = 16,  // EVP_GCM_TLS_EXPLICIT_IV_LEN / _TAG_LEN (evp.h:394-398)
};
// EVP_CIPH_GCM_MODE | CUSTOM_IV | ALWAYS_CALL_INIT | CTRL_INIT | CUSTOM_COPY |
// FLAG_DEFAULT_ASN1 | FLAG_FIPS | FLAG_CUSTOM_CIPHER | FLAG_AEAD_CIPHER (e_aes.c:1049-1059)
constexpr unsigned long kGcmCipherFlags =
    0x6 | 0x10 | 0x20 | 0x40 | 0x400 | 0x1000 | 0x4000 | 0x100000 | 0x200000;

// EVP_AES_GCM_CTX (e_aes.c:74-85) with the GCM128 state on the device
struct GpuGcm {
  tlsgpu_sessions* sess;  // one-session table: key schedule, H tables
  GcmStream* d_st;        // GCM128_CONTEXT
  unsigned char key[32];
  int key_set, iv_set;
  unsigned char* iv;      // ctx->iv, or heap for IVs longer than 16 bytes
  int ivlen, taglen, iv_gen, tls_aad_len;
};

std::atomic<uint64_t> g_cipher_programs{0};

// One program of GCM128 steps.  Step i reads in[i] (host, len[i] bytes) and
// writes out[i] (host, len[i] bytes; TAG: len bytes of tag).  Returns the rc
// of the last step run (gcm128.c conventions), or -100 on a runtime failure.
struct Step {
  uint32_t kind;
  const unsigned char* in;
  unsigned char* out;
  size_t len;
};
int run_program(GpuGcm* g, const Step* steps, int nsteps) {
  tlsgpu_engine* e = g->sess->eng;
  auto al = [](size_t v) { return (v + 255) & ~(size_t)255; };
  size_t total = al(sizeof(GcmStreamOp) * (size_t)nsteps);
  std::vector<size_t> o_in(nsteps), o_out(nsteps);
  for (int i = 0; i < nsteps; i++) {
    o_in[i] = total;
    total += al(steps[i].in ? steps[i].len : 0);
    o_out[i] = total;
    total += al(steps[i].out ? steps[i].len : 0);
  }
  Staging* stg = stage_for(e->device);
  if (!stg || !stg->ensure(e->device, total, true)) return -100;
  uint8_t* b = stg->d_buf;
  hipStream_t s = stg->stream;
  std::vector<GcmStreamOp> ops(nsteps);
  for (int i = 0; i < nsteps; i++) {
    ops[i].kind = steps[i].kind;
    ops[i].reserved = 0;
    ops[i].len = steps[i].len;
    ops[i].in = steps[i].in ? (uint64_t)(b + o_in[i]) : 0;
    ops[i].out = steps[i].out ? (uint64_t)(b + o_out[i]) : 0;
    if (steps[i].in && steps[i].len &&
        hipMemcpyAsync(b + o_in[i], steps[i].in, steps[i].len, hipMemcpyHostToDevice, s))
      return -100;
  }
  if (hipMemcpyAsync(b, ops.data(), sizeof(GcmStreamOp) * nsteps, hipMemcpyHostToDevice, s) ||
      launch_gcm_stream(g->sess->d_sess, g->sess->d_gcm, 0, g->d_st,
                        reinterpret_cast<const GcmStreamOp*>(b), (uint32_t)nsteps, s))
    return -100;
  int32_t rc = -100;
  if (hipMemcpyAsync(&rc, &g->d_st->rc, sizeof(rc), hipMemcpyDeviceToHost, s) ||
      hipStreamSynchronize(s))
    return -100;
  for (int i = 0; i < nsteps; i++)
    if (steps[i].out && steps[i].len &&
        hipMemcpy(steps[i].out, b + o_out[i], steps[i].len, hipMemcpyDeviceToHost))
      return -100;
  g_cipher_programs.fetch_add(1, std::memory_order_relaxed);
  return rc;
}

bool gcm_set_key(GpuGcm* g, const unsigned char* key, int key_len) {
  // a cipher context keeps the GPU of its first key (its session table lives there)
  tlsgpu_engine* e = g->sess ? g->sess->eng : evp_engine(evp_pick());
  if (!e) return false;
  if (!g->sess && tlsgpu_sessions_create(e, 1, &g->sess) != TLSGPU_OK) return false;
  if (!g->d_st) {
    if (hipSetDevice(e->device) != hipSuccess ||
        hipMalloc((void**)&g->d_st, sizeof(GcmStream)) != hipSuccess) {
      g->d_st = nullptr;
      return false;
    }
  }
  if (hipMemset(g->d_st, 0, sizeof(GcmStream)) != hipSuccess) return false;
  tlsgpu_session_params p;
  memset(&p, 0, sizeof(p));
  p.aead = key_len == 16 ? TLSGPU_AES_128_GCM : TLSGPU_AES_256_GCM;
  p.key_len = (uint32_t)key_len;
  memcpy(p.key, key, key_len);
  p.version = 0x0303;
  memcpy(g->key, key, key_len);
  const bool ok = tlsgpu_sessions_install(g->sess, 0, 1, &p) == TLSGPU_OK;
  memset(&p, 0, sizeof(p));
  return ok;
}

int gcm_setiv(GpuGcm* g, const unsigned char* iv, int ivlen) {
  const Step st = {GCM_OP_SETIV, iv, nullptr, (size_t)ivlen};
  return run_program(g, &st, 1);
}

// ctr64_inc (e_aes.c:697-712)
void ctr64_inc(unsigned char* counter) {
  for (int n = 7; n >= 0; n--)
    if (++counter[n]) return;
}

int gcm_ctrl(EVP_CIPHER_CTX* c, int type, int arg, void* ptr);

int gcm_init_key(EVP_CIPHER_CTX* ctx, const unsigned char* key, const unsigned char* iv, int enc) {
  (void)enc;
  auto* g = (GpuGcm*)ctx->cipher_data;
  if (!iv && !key) return 1;
  if (key) {
    if (ctx->key_len != 16 && ctx->key_len != 32) return 0;
    if (!gcm_set_key(g, key, ctx->key_len)) return 0;
    if (iv == nullptr && g->iv_set) iv = g->iv;
    if (iv) {
      if (gcm_setiv(g, iv, g->ivlen) != 0) return 0;
      g->iv_set = 1;
    }
    g->key_set = 1;
  } else {
    if (g->key_set) {
      if (gcm_setiv(g, iv, g->ivlen) != 0) return 0;
    } else {
      memcpy(g->iv, iv, g->ivlen);
    }
    g->iv_set = 1;
    g->iv_gen = 0;
  }
  return 1;
}

int gcm_ctrl(EVP_CIPHER_CTX* c, int type, int arg, void* ptr) {
  auto* g = (GpuGcm*)c->cipher_data;
  switch (type) {
    case kCtrlInit:
      memset(g, 0, sizeof(*g));
      g->ivlen = c->cipher->iv_len;
      g->iv = c->iv;
      g->taglen = -1;
      g->tls_aad_len = -1;
      return 1;
    case kGcmSetIvlen:
      if (arg <= 0) return 0;
      if (arg > EVP_MAX_IV_LENGTH && arg > g->ivlen) {
        if (g->iv != c->iv) free(g->iv);
        g->iv = (unsigned char*)malloc(arg);
        if (!g->iv) return 0;
      }
      g->ivlen = arg;
      return 1;
    case kGcmSetTag:
      if (arg <= 0 || arg > 16 || c->encrypt) return 0;
      memcpy(c->buf, ptr, arg);
      g->taglen = arg;
      return 1;
    case kGcmGetTag:
      if (arg <= 0 || arg > 16 || !c->encrypt || g->taglen < 0) return 0;
      memcpy(ptr, c->buf, arg);
      return 1;
    case kGcmSetIvFixed:
      if (arg == -1) {
        memcpy(g->iv, ptr, g->ivlen);
        g->iv_gen = 1;
        return 1;
      }
      if (arg < 4 || (g->ivlen - arg) < 8) return 0;
      if (arg) memcpy(g->iv, ptr, arg);
      if (c->encrypt && getentropy(g->iv + arg, g->ivlen - arg) != 0) return 0;
      g->iv_gen = 1;
      return 1;
    case kGcmIvGen:
      if (g->iv_gen == 0 || g->key_set == 0) return 0;
      if (gcm_setiv(g, g->iv, g->ivlen) != 0) return 0;
      if (arg <= 0 || arg > g->ivlen) arg = g->ivlen;
      memcpy(ptr, g->iv + g->ivlen - arg, arg);
      ctr64_inc(g->iv + g->ivlen - 8);
      g->iv_set = 1;
      return 1;
    case kGcmSetIvInv:
      if (g->iv_gen == 0 || g->key_set == 0 || c->encrypt) return 0;
      memcpy(g->iv + g->ivlen - arg, ptr, arg);
      if (gcm_setiv(g, g->iv, g->ivlen) != 0) return 0;
      g->iv_set = 1;
      return 1;
    case kAeadTls1Aad: {
      if (arg != 13) return 0;
      memcpy(c->buf, ptr, arg);
      g->tls_aad_len = arg;
      unsigned int len = c->buf[arg - 2] << 8 | c->buf[arg - 1];
      len -= kTlsExplicitIv;            // correct length for the explicit IV
      if (!c->encrypt) len -= kTlsTag;  // and the tag when decrypting
      c->buf[arg - 2] = len >> 8;
      c->buf[arg - 1] = len & 0xff;
      return kTlsTag;  // extra padding: the tag appended to the record
    }
    case kCtrlCopy: {  // the GCM state and the key schedule get their own device copies
      auto* out = (EVP_CIPHER_CTX*)ptr;
      auto* go = (GpuGcm*)out->cipher_data;
      go->sess = nullptr;
      go->d_st = nullptr;
      if (g->key_set) {
        if (!gcm_set_key(go, g->key, c->key_len)) return 0;
        if (hipMemcpy(go->d_st, g->d_st, sizeof(GcmStream), hipMemcpyDeviceToDevice) != hipSuccess)
          return 0;
      }
      if (g->iv == c->iv) {
        go->iv = out->iv;
      } else {
        go->iv = (unsigned char*)malloc(g->ivlen);
        if (!go->iv) return 0;
        memcpy(go->iv, g->iv, g->ivlen);
      }
      return 1;
    }
    default:
      return -1;
  }
}

// aes_gcm_tls_cipher (e_aes.c:917-985): one TLS record in place
int gcm_tls_cipher(EVP_CIPHER_CTX* ctx, unsigned char* out, const unsigned char* in, size_t len) {
  auto* g = (GpuGcm*)ctx->cipher_data;
  int rv = -1;
  if (out != in || len < (size_t)(kTlsExplicitIv + kTlsTag)) return -1;
  // IV from the record (decrypt) or generated and written to it (encrypt);
  // the setiv of IV_GEN / SET_IV_INV runs as the program's first step
  if (ctx->encrypt) {
    if (g->iv_gen == 0 || g->key_set == 0) goto err;
    memcpy(out, g->iv + g->ivlen - kTlsExplicitIv, kTlsExplicitIv);
  } else {
    if (g->iv_gen == 0 || g->key_set == 0) goto err;
    memcpy(g->iv + g->ivlen - kTlsExplicitIv, out, kTlsExplicitIv);
  }
  {
    unsigned char iv[64];
    if (g->ivlen > (int)sizeof(iv)) goto err;
    memcpy(iv, g->iv, g->ivlen);
    if (ctx->encrypt) ctr64_inc(g->iv + g->ivlen - 8);
    g->iv_set = 1;
    const size_t plen = len - kTlsExplicitIv - kTlsTag;
    unsigned char* p = out + kTlsExplicitIv;
    unsigned char tag[16];
    const Step prog[4] = {{GCM_OP_SETIV, iv, nullptr, (size_t)g->ivlen},
                          {GCM_OP_AAD, ctx->buf, nullptr, (size_t)g->tls_aad_len},
                          {ctx->encrypt ? (uint32_t)GCM_OP_ENCRYPT : (uint32_t)GCM_OP_DECRYPT,
                           in + kTlsExplicitIv, p, plen},
                          {GCM_OP_TAG, nullptr, ctx->encrypt ? p + plen : tag, (size_t)kTlsTag}};
    if (run_program(g, prog, 4) != 0) goto err;
    if (ctx->encrypt) {
      rv = (int)(plen + kTlsExplicitIv + kTlsTag);
    } else {
      memcpy(ctx->buf, tag, kTlsTag);
      if (memcmp(ctx->buf, in + kTlsExplicitIv + plen, kTlsTag)) {  // wipe on mismatch
        memset(p, 0, plen);
        goto err;
      }
      rv = (int)plen;
    }
  }
err:
  g->iv_set = 0;
  g->tls_aad_len = -1;
  return rv;
}

// aes_gcm_cipher (e_aes.c:987-1047)
int gcm_cipher(EVP_CIPHER_CTX* ctx, unsigned char* out, const unsigned char* in, size_t len) {
  auto* g = (GpuGcm*)ctx->cipher_data;
  if (!g->key_set) return -1;
  if (g->tls_aad_len >= 0) return gcm_tls_cipher(ctx, out, in, len);
  if (!g->iv_set) return -1;
  if (in) {
    Step st;
    if (out == nullptr) {
      st = {GCM_OP_AAD, in, nullptr, len};
    } else {
      st = {ctx->encrypt ? (uint32_t)GCM_OP_ENCRYPT : (uint32_t)GCM_OP_DECRYPT, in, out, len};
    }
    if (run_program(g, &st, 1) != 0) return -1;
    return (int)len;
  }
  if (!ctx->encrypt) {
    if (g->taglen < 0) return -1;
    const Step st = {GCM_OP_FINISH, ctx->buf, nullptr, (size_t)g->taglen};
    if (run_program(g, &st, 1) != 0) return -1;
    g->iv_set = 0;
    return 0;
  }
  const Step st = {GCM_OP_TAG, nullptr, ctx->buf, 16};
  if (run_program(g, &st, 1) != 0) return -1;
  g->taglen = 16;
  g->iv_set = 0;  // don't reuse the IV
  return 0;
}

// aes_gcm_cleanup (e_aes.c:686-695)
int gcm_cleanup(EVP_CIPHER_CTX* c) {
  auto* g = (GpuGcm*)c->cipher_data;
  if (!g) return 1;
  if (g->iv != c->iv) free(g->iv);
  if (g->d_st) {
    (void)hipMemset(g->d_st, 0, sizeof(GcmStream));
    (void)hipFree(g->d_st);
  }
  if (g->sess) tlsgpu_sessions_destroy(g->sess);
  memset(g, 0, sizeof(*g));
  return 1;
}

const EVP_CIPHER k_aes_128_gcm = {895, 1, 16, 12, kGcmCipherFlags, gcm_init_key, gcm_cipher,
                                  gcm_cleanup, (int)sizeof(GpuGcm), nullptr, nullptr, gcm_ctrl,
                                  nullptr};
const EVP_CIPHER k_aes_256_gcm = {901, 1, 32, 12, kGcmCipherFlags, gcm_init_key, gcm_cipher,
                                  gcm_cleanup, (int)sizeof(GpuGcm), nullptr, nullptr, gcm_ctrl,
                                  nullptr};
}  // namespace

extern "C" const EVP_CIPHER* EVP_aes_128_gcm(void) { return &k_aes_128_gcm; }
extern "C" const EVP_CIPHER* EVP_aes_256_gcm(void) { return &k_aes_256_gcm; }
extern "C" int tlsgpu_evp_cipher_stats(uint64_t* programs) {
  if (programs) *programs = g_cipher_programs.load();
  return TLSGPU_OK;
}

// ---------------------------------------------------------------------------
// EVP coalescing queue: callers, dispatcher, completer

// 1 / 0 / -1 as gpu_call; -2: the job is too large for a staging slot (the
// caller runs it on its own staging instead).
static int evp_queue_call(EvpBatcher* b, const AeadState* st, bool seal, unsigned char* out,
                          size_t* out_len, size_t max_out_len, const unsigned char* nonce,
                          size_t nonce_len, const unsigned char* in, size_t in_len,
                          const unsigned char* ad, size_t ad_len) {
  auto al = [](size_t v) { return (v + 15) & ~(size_t)15; };
  const size_t need_in = al(nonce_len) + al(ad_len) + al(in_len);
  const size_t out_bytes = seal ? in_len + st->tag_len : std::max(max_out_len, in_len);
  const size_t need_out = al(out_bytes + 1);
  if (need_in > kEvpInBytes / 4 || need_out > kEvpOutBytes / 4) return -2;
  std::unique_lock<std::mutex> lk(b->mu);
  EvpSlot* s;
  for (;;) {
    s = b->building;
    if (s && s->jobs() < b->max_jobs && s->in_used + need_in <= kEvpInBytes &&
        s->out_used + need_out <= kEvpOutBytes)
      break;
    if (s && !b->full) {  // no room: have it dispatched now
      b->full = true;
      b->cv_disp.notify_one();
    }
    b->cv_slot.wait(lk);
  }
  const bool first = s->jobs() == 0;
  const uint32_t idx = seal ? s->nseal++ : kEvpMaxJobs - 1 - s->nopen++;
  (seal ? s->kinds_seal : s->kinds_open) |= 1u << st->kind;
  const size_t io = kEvpDescBytes + s->in_used, oo = kEvpOutOff + s->out_used;
  s->in_used += need_in;
  s->out_used += need_out;
  s->writers.fetch_add(1, std::memory_order_relaxed);
  const uint32_t gen = s->gen.load(std::memory_order_relaxed);
  if (first) {
    s->first = std::chrono::steady_clock::now();
    b->cv_disp.notify_one();
  }
  lk.unlock();
  RawJob* rj = reinterpret_cast<RawJob*>(s->h) + idx;
  size_t o = io;
  rj->nonce = (uint64_t)(s->d + o);
  if (nonce_len) memcpy(s->h + o, nonce, nonce_len);
  o += al(nonce_len);
  rj->aad = (uint64_t)(s->d + o);
  if (ad_len) memcpy(s->h + o, ad, ad_len);
  o += al(ad_len);
  rj->in = (uint64_t)(s->d + o);
  if (in_len) memcpy(s->h + o, in, in_len);
  rj->out = (uint64_t)(s->d + oo);
  rj->in_len = (uint32_t)in_len;
  rj->nonce_len = (uint32_t)nonce_len;
  rj->aad_len = (uint32_t)ad_len;
  rj->session = st->slot;
  rj->max_out = max_out_len;
  s->writers.fetch_sub(1, std::memory_order_release);
  while (s->gen.load(std::memory_order_acquire) == gen) futex_wait(&s->gen, gen);
  int r;
  if (!s->ok) {
    r = -1;
  } else {
    const int32_t status = reinterpret_cast<const int32_t*>(s->h + kEvpStatusOff)[idx];
    if (status < 0) {  // the kernel's zero-fill (evp_aead.c:137-143)
      if (max_out_len) memset(out, 0, max_out_len);
      r = 0;
    } else {
      if (status) memcpy(out, s->h + oo, (size_t)status);
      *out_len = (size_t)status;
      r = 1;
    }
  }
  if (s->readers.fetch_sub(1, std::memory_order_acq_rel) == 1) b->release(s);
  return r;
}

// The last reader hands the slot back: it becomes the building slot if there
// is none, else waits in the ring.
void EvpBatcher::release(EvpSlot* s) {
  std::lock_guard<std::mutex> lk(mu);
  s->nseal = s->nopen = 0;
  s->kinds_seal = s->kinds_open = 0;
  s->in_used = s->out_used = 0;
  if (!building) {
    building = s;
    full = false;
    cv_slot.notify_all();
  } else {
    free_ring.push_back(s);
  }
}

void EvpBatcher::dispatch_loop() {
  std::unique_lock<std::mutex> lk(mu);
  for (;;) {
    cv_disp.wait(lk, [&] { return building && building->jobs() > 0; });
    // batching policy: go now when the GPU is idle or the slot is full,
    // else when the window since the slot's first job has passed
    const auto deadline = building->first + std::chrono::microseconds(window_us);
    cv_disp.wait_until(lk, deadline, [&] { return inflight == 0 || full; });
    EvpSlot* s = building;
    full = false;
    const auto t_close = std::chrono::steady_clock::now();
    ns_wait += std::chrono::duration_cast<std::chrono::nanoseconds>(t_close - s->first).count();
    if (free_ring.empty()) {
      building = nullptr;
    } else {
      building = free_ring.back();
      free_ring.pop_back();
      cv_slot.notify_all();
    }
    inflight++;
    s->readers.store(s->jobs(), std::memory_order_relaxed);
    lk.unlock();
    while (s->writers.load(std::memory_order_acquire)) std::this_thread::yield();
    const auto t_sub = std::chrono::steady_clock::now();
    submit(s);
    s->submitted_at = std::chrono::steady_clock::now();
    lk.lock();
    ns_writers += std::chrono::duration_cast<std::chrono::nanoseconds>(t_sub - t_close).count();
    ns_submit +=
        std::chrono::duration_cast<std::chrono::nanoseconds>(s->submitted_at - t_sub).count();
    submitted.push_back(s);
    cv_comp.notify_one();
  }
}

void EvpBatcher::submit(EvpSlot* s) {
  s->ok = false;
  if (hipSetDevice(pool->eng->device) != hipSuccess) return;
  if (!submit_work(s)) {
    // part of the batch may already be queued: let it drain before the slot's
    // pinned and device buffers go back to the ring for the next batch
    (void)hipStreamSynchronize(s->stream);
    return;
  }
  s->ok = true;
}

bool EvpBatcher::submit_work(EvpSlot* s) {
  const uint32_t ns = s->nseal, no = s->nopen;
  int32_t* d_status = reinterpret_cast<int32_t*>(s->d + kEvpStatusOff);
  const RawJob* d_desc = reinterpret_cast<const RawJob*>(s->d);
  if (!s->zc && hipMemcpyAsync(s->d, s->h, kEvpDescBytes + s->in_used, hipMemcpyHostToDevice,
                               s->stream) != hipSuccess)
    return false;
  if (ns && run_batch(pool, d_desc, ns, nullptr, nullptr, d_status, s->stream, true, true,
                     nullptr, s->kinds_seal) != TLSGPU_OK)
    return false;
  if (no && run_batch(pool, d_desc + (kEvpMaxJobs - no), no, nullptr, nullptr,
                      d_status + (kEvpMaxJobs - no), s->stream, false, true, nullptr,
                      s->kinds_open) != TLSGPU_OK)
    return false;
  return (s->zc || hipMemcpyAsync(s->h + kEvpStatusOff, s->d + kEvpStatusOff,
                                  kEvpOutOff - kEvpStatusOff + s->out_used,
                                  hipMemcpyDeviceToHost, s->stream) == hipSuccess) &&
         hipEventRecord(s->done, s->stream) == hipSuccess;
}

void EvpBatcher::complete_loop() {
  std::unique_lock<std::mutex> lk(mu);
  for (;;) {
    cv_comp.wait(lk, [&] { return !submitted.empty(); });
    EvpSlot* s = submitted.front();
    submitted.pop_front();
    lk.unlock();
    if (s->ok && hipEventSynchronize(s->done) != hipSuccess) {
      s->ok = false;
      (void)hipStreamSynchronize(s->stream);  // nothing of the slot may still run
    }
    const uint64_t gpu_ns = std::chrono::duration_cast<std::chrono::nanoseconds>(
                                std::chrono::steady_clock::now() - s->submitted_at)
                                .count();
    const uint32_t n = s->jobs();
    s->gen.fetch_add(1, std::memory_order_release);
    futex_wake_all(&s->gen);
    lk.lock();
    batches++;
    jobs_done += n;
    ns_gpu += gpu_ns;
    inflight--;
    cv_disp.notify_one();
  }
}

// One device's queue: pool table, kEvpSlots staging slots, dispatcher and
// completer threads (they live as long as the process).  nullptr on failure.
static EvpBatcher* make_batcher(tlsgpu_engine* e, unsigned window_us, unsigned max_jobs,
                                uint32_t cap) {
  auto* b = new (std::nothrow) EvpBatcher();
  if (!b) {
    fail(TLSGPU_ENOMEM, "batcher");
    return nullptr;
  }
  b->window_us = window_us;
  b->max_jobs = max_jobs ? std::min(max_jobs, kEvpMaxJobs) : kEvpMaxJobs;
  if (tlsgpu_sessions_create(e, cap, &b->pool) != TLSGPU_OK) {
    delete b;
    return nullptr;
  }
  bool ok = hipSetDevice(e->device) == hipSuccess;
  for (EvpSlot& s : b->slots) {
    ok = ok && hipHostMalloc((void**)&s.h, kEvpSlotBytes, hipHostMallocDefault) == hipSuccess;
    // zero-copy (TLSGPU_EVP_ZEROCOPY, default on): the batch kernels read the
    // jobs from and write statuses and outputs to the pinned slot directly
    s.zc = ok && g_evp_zerocopy && hipHostGetDevicePointer((void**)&s.d, s.h, 0) == hipSuccess;
    if (!s.zc) s.d = nullptr;
    ok = ok && (s.zc || hipMalloc((void**)&s.d, kEvpSlotBytes) == hipSuccess) &&
         hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking) == hipSuccess &&
         hipEventCreateWithFlags(&s.done, hipEventDisableTiming) == hipSuccess;
  }
  if (!ok) {  // never started: nothing queued on its streams
    fail(TLSGPU_EHIP, "EVP queue staging on device %d", e->device);
    for (EvpSlot& s : b->slots) {
      if (s.h) (void)hipHostFree(s.h);
      if (s.d && !s.zc) (void)hipFree(s.d);
    }
    tlsgpu_sessions_destroy(b->pool);
    delete b;
    return nullptr;
  }
  b->building = &b->slots[0];
  for (uint32_t i = kEvpSlots - 1; i >= 1; i--) b->free_ring.push_back(&b->slots[i]);
  for (int i = (int)cap - 1; i >= 0; i--) b->free_sessions.push_back(i);
  b->disp = std::thread([b] { b->dispatch_loop(); });
  b->comp = std::thread([b] { b->complete_loop(); });
  return b;
}

extern "C" int tlsgpu_evp_set_batching(unsigned window_us, unsigned max_jobs,
                                       unsigned pool_sessions) {
  std::lock_guard<std::mutex> lk(g_batcher_mu);
  if (g_batcher_on) {  // already running: adjust the window / batch size only
    for (EvpBatcher* b : g_batchers) {
      if (!b) continue;
      std::lock_guard<std::mutex> lk2(b->mu);
      b->window_us = window_us;
      if (max_jobs) b->max_jobs = std::min(max_jobs, kEvpMaxJobs);
    }
    return TLSGPU_OK;
  }
  if (window_us == 0 && max_jobs == 0) return TLSGPU_OK;  // stays off
  // one queue per EVP device: contexts initialised afterwards take a pool slot
  // on the device evp_pick gives them
  const uint32_t cap = pool_sessions ? pool_sessions : 1024;
  const size_t ndev = evp_device_count();
  // All devices or none: a queue built before a later device failed stays in
  // g_batchers unused (g_batcher_on stays false, so no context takes its pool
  // slots) and a retry reuses it instead of building a second one over it —
  // its dispatcher and completer threads never outlive their queue's pointer.
  for (size_t k = 0; k < ndev; k++) {
    if (g_batchers[k]) {
      std::lock_guard<std::mutex> lk2(g_batchers[k]->mu);
      g_batchers[k]->window_us = window_us;
      if (max_jobs) g_batchers[k]->max_jobs = std::min(max_jobs, kEvpMaxJobs);
      continue;
    }
    tlsgpu_engine* e = evp_engine(k);
    if (!e) return fail(TLSGPU_EHIP, "no GPU engine for EVP device %zu", k);
    EvpBatcher* b = make_batcher(e, window_us, max_jobs, cap);
    if (!b) return TLSGPU_EHIP;
    g_batchers[k] = b;
  }
  g_batcher_on = true;
  if (getenv("TLSGPU_EVP_STATS")) {
    atexit([] {
      uint64_t nb = 0, nj = 0, w = 0, wr = 0, sb = 0, gp = 0;
      for (EvpBatcher* q : g_batchers) {
        if (!q) continue;
        std::lock_guard<std::mutex> lk3(q->mu);
        nb += q->batches;
        nj += q->jobs_done;
        w += q->ns_wait;
        wr += q->ns_writers;
        sb += q->ns_submit;
        gp += q->ns_gpu;
      }
      const double d = nb ? (double)nb : 1.0;
      fprintf(stderr,
              "{\"evp_queue\": {\"devices\": %zu, \"batches\": %llu, \"jobs\": %llu, "
              "\"jobs_per_batch\": %.2f, \"us_first_to_close\": %.1f, \"us_writers\": %.1f, "
              "\"us_submit\": %.1f, \"us_submit_to_done\": %.1f}}\n",
              evp_device_count(), (unsigned long long)nb, (unsigned long long)nj, nj / d,
              w / d / 1e3, wr / d / 1e3, sb / d / 1e3, gp / d / 1e3);
    });
  }
  return TLSGPU_OK;
}

extern "C" int tlsgpu_evp_batch_stats(uint64_t* batches, uint64_t* jobs) {
  std::lock_guard<std::mutex> lk(g_batcher_mu);
  uint64_t nb = 0, nj = 0;
  for (EvpBatcher* b : g_batchers) {
    if (!b) continue;
    std::lock_guard<std::mutex> lk2(b->mu);
    nb += b->batches;
    nj += b->jobs_done;
  }
  if (batches) *batches = nb;
  if (jobs) *jobs = nj;
  return TLSGPU_OK;
}

// TLSGPU_EVP_BATCH_US=<window> turns the queue on at load time for unchanged
// applications (LD_PRELOAD); TLSGPU_EVP_POOL sets the pooled context count.
__attribute__((constructor)) static void evp_batching_from_env() {
  const char* w = getenv("TLSGPU_EVP_BATCH_US");
  if (!w || !*w) return;
  const char* p = getenv("TLSGPU_EVP_POOL");
  tlsgpu_evp_set_batching((unsigned)strtoul(w, nullptr, 10), 0,
                          p ? (unsigned)strtoul(p, nullptr, 10) : 0);
}
