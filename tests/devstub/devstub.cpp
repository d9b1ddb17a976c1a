// devstub.cpp — a recording stand-in for the HIP runtime and the kernel
// launchers, for the multi-GPU device-affinity audit (VERDICT r04 next-round 5,
// tests/test_device_affinity.py).
//
// libtlsgpu_devstub.so links the engine's unmodified host objects
// (engine.cpp, group.cpp, talos_hooks.cpp, compiled by talos_amd/Makefile) with
// this file instead of libamdhip64 and the kernel objects, so the C ABI runs on
// a CPU box with TLSGPU_STUB_DEVICES fake GPUs.  Every allocation, stream and
// event remembers the device that was current on the calling thread when it
// was made; every stream-ordered call (kernel launch, async copy / memset,
// event record) must be issued with its stream's device current and may only
// touch device memory of that device (HIP launches on the stream's device but
// allocates on the current one, so a missing hipSetDevice on a worker or
// calling thread shows up here as a cross-device pointer or stream).  Memory is
// host memory, copies and memsets are performed, kernels do nothing: the audit
// is about which device each call reaches, not about results.
//
// Test-only; never shipped or loaded by the product.
#include <hip/hip_runtime_api.h>

#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "../../talos_amd/csrc/tlsgpu_internal.h"

namespace {

std::mutex g_mu;
int g_ndev = [] {
  const char* v = getenv("TLSGPU_STUB_DEVICES");
  const int n = v && *v ? atoi(v) : 4;
  return n > 0 ? n : 4;
}();
thread_local int t_dev = 0;

// The runtime's own per-thread state (libamdhip64 registers a thread-local
// destructor at a thread's first HIP call; tools/exit_order_probe.hip): here a
// sentinel created at the thread's first stub call.  A HIP call after it was
// destroyed — from a thread-local destructor of ours that runs later — is the
// hazard of the round-4 exit SIGSEGV and a violation.
struct RuntimeTls {
  bool alive = true;
  ~RuntimeTls() { alive = false; }
};
thread_local RuntimeTls t_rt;
thread_local bool t_rt_seen = false;
void rt_enter(const char* what);

struct Alloc {
  size_t size;
  int dev;
  bool pinned;
};
std::map<uintptr_t, Alloc> g_allocs;        // base -> allocation
std::map<const void*, int> g_streams;       // stream -> device
std::map<const void*, int> g_events;        // event -> device
std::vector<std::string> g_violations;
uint64_t g_checked = 0;                     // stream-ordered calls checked
uint64_t g_pinned_cross = 0;                // pinned memory of one device used by another's work

void violation(const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_violations.emplace_back(buf);
}

// the allocation holding p (nullptr: not ours, e.g. pageable host memory)
const Alloc* find(const void* p) {
  const uintptr_t a = (uintptr_t)p;
  auto it = g_allocs.upper_bound(a);
  if (it == g_allocs.begin()) return nullptr;
  --it;
  return a < it->first + (it->second.size ? it->second.size : 1) ? &it->second : nullptr;
}

// the device a stream-ordered call runs on; checks it is the current one
int stream_dev(const char* what, hipStream_t s) {
  g_checked++;
  int d = t_dev;  // null stream: the current device's
  if (s) {
    auto it = g_streams.find(s);
    if (it == g_streams.end()) {
      violation("%s: unknown stream %p", what, (void*)s);
      return t_dev;
    }
    d = it->second;
  }
  if (d != t_dev)
    violation("%s: stream of device %d issued with device %d current", what, d, t_dev);
  return d;
}

// device memory touched by work on device `dev`: must be that device's (pinned
// host memory is mapped for every device)
void mem_on(const char* what, const char* arg, const void* p, int dev) {
  if (!p) return;
  const Alloc* a = find(p);
  if (!a) return;
  if (a->pinned) {  // mapped for every device (hipHostMalloc): counted, not a violation
    if (a->dev != dev) g_pinned_cross++;
    return;
  }
  if (a->dev != dev)
    violation("%s: %s is memory of device %d, used by work on device %d", what, arg, a->dev, dev);
}

void* alloc(size_t n, bool pinned) {
  void* p = aligned_alloc(256, ((n ? n : 1) + 255) & ~(size_t)255);
  if (p) {
    memset(p, 0, n ? n : 1);
    g_allocs[(uintptr_t)p] = Alloc{n, t_dev, pinned};
  }
  return p;
}

hipError_t release(void* p, bool pinned, const char* what) {
  if (!p) return hipSuccess;
  auto it = g_allocs.find((uintptr_t)p);
  if (it == g_allocs.end() || it->second.pinned != pinned) {
    violation("%s: %p is not a live allocation of that kind", what, p);
    return hipErrorInvalidValue;
  }
  if (!pinned && it->second.dev != t_dev)
    violation("%s: memory of device %d freed with device %d current", what, it->second.dev, t_dev);
  g_allocs.erase(it);
  free(p);
  return hipSuccess;
}

void rt_enter(const char* what) {
  if (!t_rt_seen) {
    t_rt_seen = true;
    (void)&t_rt;  // constructed now: its destructor is registered at this point
  } else if (!t_rt.alive) {
    std::lock_guard<std::mutex> lk(g_mu);
    violation("%s: HIP call from a thread-exit destructor after the runtime's thread state "
              "was destroyed", what);
  }
}

}  // namespace

// ---------------------------------------------------------------------------
// the runtime subset the engine's host code calls
extern "C" {

hipError_t hipSetDevice(int d) {
  rt_enter("hipSetDevice");
  if (d < 0 || d >= g_ndev) return hipErrorInvalidDevice;
  t_dev = d;
  return hipSuccess;
}
hipError_t hipGetDeviceCount(int* c) {
  rt_enter("hipGetDeviceCount");
  *c = g_ndev;
  return hipSuccess;
}
hipError_t hipDeviceGetAttribute(int* v, hipDeviceAttribute_t, int d) {
  rt_enter("hipDeviceGetAttribute");
  if (d < 0 || d >= g_ndev) return hipErrorInvalidDevice;
  *v = 256;
  return hipSuccess;
}
hipError_t hipDeviceSynchronize(void) {
  rt_enter("hipDeviceSynchronize"); return hipSuccess; }
hipError_t hipGetLastError(void) {
  rt_enter("hipGetLastError"); return hipSuccess; }
const char* hipGetErrorString(hipError_t) {
  rt_enter("hipGetErrorString"); return "devstub"; }

hipError_t hipMalloc(void** p, size_t n) {
  rt_enter("hipMalloc");
  std::lock_guard<std::mutex> lk(g_mu);
  *p = alloc(n, false);
  return *p ? hipSuccess : hipErrorOutOfMemory;
}
hipError_t hipMallocAsync(void** p, size_t n, hipStream_t s) {
  rt_enter("hipMallocAsync");
  std::lock_guard<std::mutex> lk(g_mu);
  stream_dev("hipMallocAsync", s);
  *p = alloc(n, false);
  return *p ? hipSuccess : hipErrorOutOfMemory;
}
hipError_t hipFree(void* p) {
  rt_enter("hipFree");
  std::lock_guard<std::mutex> lk(g_mu);
  return release(p, false, "hipFree");
}
hipError_t hipFreeAsync(void* p, hipStream_t s) {
  rt_enter("hipFreeAsync");
  std::lock_guard<std::mutex> lk(g_mu);
  stream_dev("hipFreeAsync", s);
  return release(p, false, "hipFreeAsync");
}
hipError_t hipHostMalloc(void** p, size_t n, unsigned int) {
  rt_enter("hipHostMalloc");
  std::lock_guard<std::mutex> lk(g_mu);
  *p = alloc(n, true);
  return *p ? hipSuccess : hipErrorOutOfMemory;
}
hipError_t hipHostFree(void* p) {
  rt_enter("hipHostFree");
  std::lock_guard<std::mutex> lk(g_mu);
  return release(p, true, "hipHostFree");
}
hipError_t hipHostGetDevicePointer(void** d, void* h, unsigned int) {
  rt_enter("hipHostGetDevicePointer");
  *d = h;
  return hipSuccess;
}

hipError_t hipStreamCreateWithFlags(hipStream_t* s, unsigned int) {
  rt_enter("hipStreamCreateWithFlags");
  std::lock_guard<std::mutex> lk(g_mu);
  *s = reinterpret_cast<hipStream_t>(new char);
  g_streams[*s] = t_dev;
  return hipSuccess;
}
hipError_t hipStreamDestroy(hipStream_t s) {
  rt_enter("hipStreamDestroy");
  std::lock_guard<std::mutex> lk(g_mu);
  auto it = g_streams.find(s);
  if (it == g_streams.end()) return hipErrorInvalidHandle;
  g_streams.erase(it);
  delete reinterpret_cast<char*>(s);
  return hipSuccess;
}
hipError_t hipStreamSynchronize(hipStream_t) {
  rt_enter("hipStreamSynchronize"); return hipSuccess; }
hipError_t hipStreamWaitEvent(hipStream_t s, hipEvent_t e, unsigned int) {
  rt_enter("hipStreamWaitEvent");
  std::lock_guard<std::mutex> lk(g_mu);
  stream_dev("hipStreamWaitEvent", s);
  if (!g_events.count(e)) violation("hipStreamWaitEvent: unknown event");
  return hipSuccess;
}

hipError_t hipEventCreateWithFlags(hipEvent_t* e, unsigned int) {
  rt_enter("hipEventCreateWithFlags");
  std::lock_guard<std::mutex> lk(g_mu);
  *e = reinterpret_cast<hipEvent_t>(new char);
  g_events[*e] = t_dev;
  return hipSuccess;
}
hipError_t hipEventCreate(hipEvent_t* e) {
  rt_enter("hipEventCreate"); return hipEventCreateWithFlags(e, 0); }
hipError_t hipEventDestroy(hipEvent_t e) {
  rt_enter("hipEventDestroy");
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_events.erase(e)) return hipErrorInvalidHandle;
  delete reinterpret_cast<char*>(e);
  return hipSuccess;
}
hipError_t hipEventRecord(hipEvent_t e, hipStream_t s) {
  rt_enter("hipEventRecord");
  std::lock_guard<std::mutex> lk(g_mu);
  const int d = stream_dev("hipEventRecord", s);
  auto it = g_events.find(e);
  if (it == g_events.end()) violation("hipEventRecord: unknown event");
  else if (it->second != d)
    violation("hipEventRecord: event of device %d recorded on a stream of device %d", it->second, d);
  return hipSuccess;
}
hipError_t hipEventSynchronize(hipEvent_t) {
  rt_enter("hipEventSynchronize"); return hipSuccess; }
hipError_t hipEventQuery(hipEvent_t) {
  rt_enter("hipEventQuery"); return hipSuccess; }
hipError_t hipEventElapsedTime(float* ms, hipEvent_t, hipEvent_t) {
  rt_enter("hipEventElapsedTime");
  *ms = 1.0f;
  return hipSuccess;
}

hipError_t hipMemcpy(void* d, const void* s, size_t n, hipMemcpyKind) {
  rt_enter("hipMemcpy");
  if (n) memmove(d, s, n);
  return hipSuccess;
}
hipError_t hipMemcpyAsync(void* d, const void* s, size_t n, hipMemcpyKind, hipStream_t st) {
  rt_enter("hipMemcpyAsync");
  {
    std::lock_guard<std::mutex> lk(g_mu);
    const int dev = stream_dev("hipMemcpyAsync", st);
    mem_on("hipMemcpyAsync", "dst", d, dev);
    mem_on("hipMemcpyAsync", "src", s, dev);
  }
  if (n) memmove(d, s, n);
  return hipSuccess;
}
hipError_t hipMemset(void* p, int v, size_t n) {
  rt_enter("hipMemset");
  {
    std::lock_guard<std::mutex> lk(g_mu);
    mem_on("hipMemset", "dst", p, t_dev);
  }
  if (n) memset(p, v, n);
  return hipSuccess;
}
hipError_t hipMemsetAsync(void* p, int v, size_t n, hipStream_t s) {
  rt_enter("hipMemsetAsync");
  {
    std::lock_guard<std::mutex> lk(g_mu);
    mem_on("hipMemsetAsync", "dst", p, stream_dev("hipMemsetAsync", s));
  }
  if (n) memset(p, v, n);
  return hipSuccess;
}
hipError_t hipMemsetD32Async(hipDeviceptr_t p, int v, size_t n, hipStream_t s) {
  rt_enter("hipMemsetD32Async");
  {
    std::lock_guard<std::mutex> lk(g_mu);
    mem_on("hipMemsetD32Async", "dst", p, stream_dev("hipMemsetD32Async", s));
  }
  for (size_t i = 0; i < n; i++) reinterpret_cast<int32_t*>(p)[i] = v;
  return hipSuccess;
}

// the audit's own entry points (tests/test_device_affinity.py)
// live bytes of pinned host memory and of device memory (all devices), and
// the number of live pinned allocations
void devstub_mem(uint64_t* pinned, uint64_t* device, uint64_t* pinned_allocs) {
  std::lock_guard<std::mutex> lk(g_mu);
  uint64_t p = 0, d = 0, np = 0;
  for (const auto& kv : g_allocs) {
    if (kv.second.pinned) {
      p += kv.second.size;
      np++;
    } else {
      d += kv.second.size;
    }
  }
  if (pinned) *pinned = p;
  if (device) *device = d;
  if (pinned_allocs) *pinned_allocs = np;
}

int devstub_report(char* buf, size_t n, uint64_t* checked, uint64_t* pinned_cross) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (pinned_cross) *pinned_cross = g_pinned_cross;
  std::string all;
  for (const std::string& v : g_violations) all += v + "\n";
  if (buf && n) snprintf(buf, n, "%s", all.c_str());
  if (checked) *checked = g_checked;
  return (int)g_violations.size();
}

}  // extern "C"

// ---------------------------------------------------------------------------
// kernel launchers: check the stream and the device memory each kernel reads
// or writes; run nothing
namespace tg {
namespace {
int launch(const char* what, hipStream_t s, std::initializer_list<std::pair<const char*, const void*>> mem) {
  std::lock_guard<std::mutex> lk(g_mu);
  const int d = stream_dev(what, s);
  for (const auto& m : mem) mem_on(what, m.first, m.second, d);
  return 0;
}
int launch_batch(const char* what, const BatchArgs& a, hipStream_t s,
                 std::initializer_list<std::pair<const char*, const void*>> more = {}) {
  std::lock_guard<std::mutex> lk(g_mu);
  const int d = stream_dev(what, s);
  const std::pair<const char*, const void*> mem[] = {
      {"sessions", a.sessions}, {"gcm_tables", a.gcm_tables}, {"descs", a.descs}, {"in", a.in},
      {"out", a.out}, {"status", a.status}, {"sel", a.sel}, {"wg_next", a.wg_next}, {"dbg", a.dbg},
      {"cut_work", a.cut_work}, {"pieces", a.pieces}};
  for (const auto& m : mem) mem_on(what, m.first, m.second, d);
  for (const auto& m : more) mem_on(what, m.first, m.second, d);
  return 0;
}
}  // namespace

int launch_gcm(const BatchArgs& a, bool, bool, int, int, hipStream_t s) {
  return launch_batch("launch_gcm", a, s);
}
int launch_gcm_split(const BatchArgs& a, bool, int, hipStream_t s) {
  return launch_batch("launch_gcm_split", a, s);
}
int launch_gcm_prep(const BatchArgs& a, RecPre* pre, bool, int, hipStream_t s) {
  return launch_batch("launch_gcm_prep", a, s, {{"pre", pre}});
}
int launch_piece_plan(const BatchArgs& a, int, uint8_t* scratch, const uint2** pieces,
                      const uint32_t** n_pieces, hipStream_t s) {
  *pieces = reinterpret_cast<const uint2*>(scratch);
  *n_pieces = reinterpret_cast<const uint32_t*>(scratch);
  return launch_batch("launch_piece_plan", a, s, {{"scratch", scratch}});
}
int launch_range_work(const BatchArgs& a, int, unsigned long long* out, hipStream_t s) {
  return launch_batch("launch_range_work", a, s, {{"out", out}});
}
int launch_gcm_queue(const BatchArgs& a, const RecPre* pre, bool, int, int, hipStream_t s) {
  return launch_batch("launch_gcm_queue", a, s, {{"pre", pre}});
}
int launch_gcm_stream(const DevSession* sessions, const DevGcmTables* tables, uint32_t, GcmStream* st,
                      const GcmStreamOp* ops, uint32_t, hipStream_t s) {
  return launch("launch_gcm_stream", s, {{"sessions", sessions}, {"tables", tables}, {"state", st}, {"ops", ops}});
}
int launch_chacha(const BatchArgs& a, bool, bool, bool, bool, hipStream_t s) {
  return launch_batch("launch_chacha", a, s);
}
int launch_evp_server(const ServerArgs& a, int, hipStream_t s) {
  return launch("launch_evp_server", s, {{"slots", a.slots}, {"stop", a.stop}, {"exited", a.exited}});
}
int launch_session_install_arg(DevSession* sessions, DevGcmTables* tables, const tlsgpu_session_params&,
                               uint32_t, hipStream_t s) {
  return launch("launch_session_install_arg", s, {{"sessions", sessions}, {"tables", tables}});
}
int launch_session_install(DevSession* sessions, DevGcmTables* tables, const tlsgpu_session_params* p,
                           uint32_t, uint32_t, hipStream_t s) {
  return launch("launch_session_install", s, {{"sessions", sessions}, {"tables", tables}, {"params", p}});
}
int launch_upload_session(const void* img, DevSession* sess, DevGcmTables* tab, uint32_t table_bytes,
                          hipStream_t s) {
  launch("launch_upload_session", s, {{"img", img}, {"sessions", sess}, {"tables", tab}});
  memcpy(sess, img, sizeof(DevSession));
  if (table_bytes) memcpy(tab, reinterpret_cast<const uint8_t*>(img) + sizeof(DevSession), table_bytes);
  return 0;
}
int launch_scrub_session(DevSession* sess, DevGcmTables* tab, hipStream_t s) {
  return launch("launch_scrub_session", s, {{"sessions", sess}, {"tables", tab}});
}
int launch_wire_frame(const tlsgpu_wire_stream* streams, uint32_t, const uint8_t* wire,
                      const DevSession* sessions, uint32_t, uint32_t, tlsgpu_record* recs,
                      tlsgpu_wire_result* results, uint32_t* total, hipStream_t s) {
  return launch("launch_wire_frame", s, {{"streams", streams}, {"wire", wire}, {"sessions", sessions},
                                         {"recs", recs}, {"results", results}, {"total", total}});
}
int launch_wire_seal_frame(const tlsgpu_write_stream* streams, uint32_t, const DevSession* sessions,
                           uint32_t, uint8_t* wire, uint64_t, uint32_t, tlsgpu_record* recs,
                           tlsgpu_write_result* results, uint32_t* total, hipStream_t s) {
  return launch("launch_wire_seal_frame", s, {{"streams", streams}, {"sessions", sessions}, {"wire", wire},
                                              {"recs", recs}, {"results", results}, {"total", total}});
}
int launch_wire_finish(uint32_t, tlsgpu_wire_result* results, int32_t* status, hipStream_t s) {
  return launch("launch_wire_finish", s, {{"results", results}, {"status", status}});
}
int launch_fill_synthetic(uint8_t* d_out, uint64_t, uint32_t, uint32_t, uint64_t, uint64_t, hipStream_t s) {
  return launch("launch_fill_synthetic", s, {{"out", d_out}});
}
int launch_fill_synthetic_spans(uint8_t* d_out, const uint64_t* offs, const uint32_t* lens, uint32_t,
                                uint64_t, uint64_t, hipStream_t s) {
  return launch("launch_fill_synthetic_spans", s, {{"out", d_out}, {"offs", offs}, {"lens", lens}});
}
int launch_check_bounds(const tlsgpu_record* recs, tlsgpu_record* safe, uint32_t n, const DevSession* sessions,
                        uint32_t, uint64_t, uint64_t, bool, int32_t* status, uint32_t* ctl, uint32_t,
                        hipStream_t s) {
  launch("launch_check_bounds", s, {{"recs", recs}, {"safe", safe}, {"sessions", sessions},
                                    {"status", status}, {"ctl", ctl}});
  // the engine's later kernels read the sanitized copy: give them the input's
  if (n && safe && recs) memmove(safe, recs, sizeof(tlsgpu_record) * (size_t)n);
  return 0;
}

}  // namespace tg
