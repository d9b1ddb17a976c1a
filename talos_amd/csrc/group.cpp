// group.cpp — multi-GPU batch split in the C ABI (include/tlsgpu.h,
// tlsgpu_group_*; SURVEY.md §8e, BASELINE configs[4]).
//
// Records are independent and the session state is read-only, so a batch of
// many connections splits into contiguous slices of about equal bytes, one per
// GPU of the node, with no collective: each member runs the single-GPU path
// (tlsgpu_open_host / tlsgpu_open_batch ...) on its own slice.  One engine per
// member (its own device, HIP stream, scratch and host pipeline) and one host
// worker thread per member, so the members' PCIe copies and kernels run at the
// same time.  Written purely against the public ABI: a member is exactly a
// single-GPU engine.
#include <hip/hip_runtime.h>

#include <condition_variable>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <functional>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include "../../include/tlsgpu.h"

// engine.cpp: sets the calling thread's tlsgpu_last_error (not exported)
extern "C" int tg_internal_set_error(int code, const char* msg);

namespace {

// A worker thread that runs one job at a time for its member.
struct Worker {
  std::thread th;
  std::mutex mu;
  std::condition_variable cv;
  std::function<int()> job;
  bool has_job = false, done = false, quit = false;
  int rc = TLSGPU_OK;
  char err[256] = "";  // the job's tlsgpu_last_error (thread-local to this worker)

  void loop() {
    std::unique_lock<std::mutex> lk(mu);
    for (;;) {
      cv.wait(lk, [&] { return has_job || quit; });
      if (quit) return;
      auto f = std::move(job);
      has_job = false;
      lk.unlock();
      const int r = f();
      if (r != TLSGPU_OK) snprintf(err, sizeof(err), "%s", tlsgpu_last_error());
      lk.lock();
      rc = r;
      done = true;
      cv.notify_all();
    }
  }
  void post(std::function<int()> f) {
    std::lock_guard<std::mutex> lk(mu);
    job = std::move(f);
    has_job = true;
    done = false;
    cv.notify_all();
  }
  int wait() {
    std::unique_lock<std::mutex> lk(mu);
    cv.wait(lk, [&] { return done; });
    return rc;
  }
};

}  // namespace

struct tlsgpu_group {
  std::vector<tlsgpu_engine*> engines;
  std::vector<Worker*> workers;
  std::mutex mu;  // one group call at a time
};

struct tlsgpu_group_sessions {
  tlsgpu_group* g;
  std::vector<tlsgpu_sessions*> members;
};

// A group-level failure: the reason goes to the caller's tlsgpu_last_error.
static int gfail(int code, const char* what) { return tg_internal_set_error(code, what); }

extern "C" int tlsgpu_group_create(const int* devices, uint32_t n, tlsgpu_group** out) {
  if (!out) return TLSGPU_EINVAL;
  *out = nullptr;
  std::vector<int> devs;
  if (devices && n) {
    devs.assign(devices, devices + n);
  } else {
    int count = 0;
    if (tlsgpu_device_count(&count) != TLSGPU_OK || count <= 0) return TLSGPU_EHIP;
    for (int d = 0; d < count; d++) devs.push_back(d);
  }
  auto* g = new (std::nothrow) tlsgpu_group();
  if (!g) return TLSGPU_ENOMEM;
  for (int d : devs) {
    tlsgpu_engine* e = nullptr;
    const int rc = tlsgpu_engine_create(d, &e);
    if (rc != TLSGPU_OK) {
      tlsgpu_group_destroy(g);
      return rc;
    }
    g->engines.push_back(e);
    auto* w = new Worker();
    w->th = std::thread([w] { w->loop(); });
    g->workers.push_back(w);
  }
  *out = g;
  return TLSGPU_OK;
}

extern "C" void tlsgpu_group_destroy(tlsgpu_group* g) {
  if (!g) return;
  for (Worker* w : g->workers) {
    {
      std::lock_guard<std::mutex> lk(w->mu);
      w->quit = true;
      w->cv.notify_all();
    }
    w->th.join();
    delete w;
  }
  for (tlsgpu_engine* e : g->engines) tlsgpu_engine_destroy(e);
  delete g;
}

extern "C" uint32_t tlsgpu_group_size(const tlsgpu_group* g) {
  return g ? (uint32_t)g->engines.size() : 0;
}

extern "C" tlsgpu_engine* tlsgpu_group_engine(tlsgpu_group* g, uint32_t member) {
  return g && member < g->engines.size() ? g->engines[member] : nullptr;
}

extern "C" int tlsgpu_group_sessions_create(tlsgpu_group* g, uint32_t capacity,
                                            tlsgpu_group_sessions** out) {
  if (!g || !out || capacity == 0) return gfail(TLSGPU_EINVAL, "group sessions: bad arguments");
  *out = nullptr;
  auto* gs = new (std::nothrow) tlsgpu_group_sessions();
  if (!gs) return TLSGPU_ENOMEM;
  gs->g = g;
  for (tlsgpu_engine* e : g->engines) {
    tlsgpu_sessions* t = nullptr;
    const int rc = tlsgpu_sessions_create(e, capacity, &t);
    if (rc != TLSGPU_OK) {
      tlsgpu_group_sessions_destroy(gs);
      return rc;
    }
    gs->members.push_back(t);
  }
  *out = gs;
  return TLSGPU_OK;
}

extern "C" void tlsgpu_group_sessions_destroy(tlsgpu_group_sessions* gs) {
  if (!gs) return;
  for (tlsgpu_sessions* t : gs->members) tlsgpu_sessions_destroy(t);
  delete gs;
}

extern "C" tlsgpu_sessions* tlsgpu_group_sessions_member(tlsgpu_group_sessions* gs,
                                                         uint32_t member) {
  return gs && member < gs->members.size() ? gs->members[member] : nullptr;
}

// Runs f(k) for every member k on the members' worker threads, waits for all,
// returns the first non-OK code in member order.
static int run_members(tlsgpu_group* g, const std::function<int(uint32_t)>& f) {
  const uint32_t m = (uint32_t)g->workers.size();
  for (uint32_t k = 0; k < m; k++) g->workers[k]->post([&f, k] { return f(k); });
  int rc = TLSGPU_OK;
  for (uint32_t k = 0; k < m; k++) {
    const int r = g->workers[k]->wait();
    if (rc == TLSGPU_OK && r != TLSGPU_OK) {
      // the member worker's reason, carried to the caller's thread
      char msg[300];
      snprintf(msg, sizeof(msg), "group member %u: %s", k, g->workers[k]->err);
      rc = tg_internal_set_error(r, msg);
    }
  }
  return rc;
}

extern "C" int tlsgpu_group_sessions_install(tlsgpu_group_sessions* gs, uint32_t first, uint32_t n,
                                             const tlsgpu_session_params* params) {
  if (!gs || (!params && n)) return gfail(TLSGPU_EINVAL, "group install: bad arguments");
  std::lock_guard<std::mutex> lk(gs->g->mu);
  return run_members(gs->g, [&](uint32_t k) {
    return tlsgpu_sessions_install(gs->members[k], first, n, params);
  });
}

extern "C" int tlsgpu_split_by_bytes(const tlsgpu_record* recs, uint32_t n, uint32_t parts,
                                     uint32_t* cuts) {
  if (!cuts || parts == 0 || (n && !recs)) return gfail(TLSGPU_EINVAL, "split_by_bytes: bad arguments");
  // prefix sums in 64 bits; cut k = first i with prefix[i] * parts >= total * k
  // (unsigned __int128 keeps the products exact for any byte total)
  unsigned __int128 total = 0;
  for (uint32_t i = 0; i < n; i++) total += recs[i].len_type & 0xFFFFFFu;
  cuts[0] = 0;
  uint64_t prefix = 0;
  uint32_t i = 0;
  for (uint32_t k = 1; k < parts; k++) {
    const unsigned __int128 want = total * k;
    while (i < n && (unsigned __int128)prefix * parts < want) {
      prefix += recs[i].len_type & 0xFFFFFFu;
      i++;
    }
    cuts[k] = i;
  }
  cuts[parts] = n;
  return TLSGPU_OK;
}

// Host-resident: slice k's descriptors keep their offsets into the caller's
// whole h_in / h_out, so each member's tlsgpu_*_host reads and writes exactly
// its records' spans (the pipeline mirrors only the ranges a slice touches).
static int group_host(tlsgpu_group_sessions* gs, bool seal, const tlsgpu_record* h_recs,
                      uint32_t n, const uint8_t* h_in, size_t in_bytes, uint8_t* h_out,
                      size_t out_bytes, int32_t* h_status) {
  if (!gs || (n && (!h_recs || !h_in || !h_out || !h_status)))
    return gfail(TLSGPU_EINVAL, "group host batch: null buffer");
  if (n == 0) return TLSGPU_OK;
  tlsgpu_group* g = gs->g;
  const uint32_t m = (uint32_t)g->engines.size();
  // slices own disjoint byte ranges only when the layout ascends; otherwise a
  // member's pipeline copies whole buffers back, so one member takes it all
  bool ascending = true;
  for (uint32_t i = 1; i < n && ascending; i++)
    ascending = h_recs[i].in_off >= h_recs[i - 1].in_off &&
                h_recs[i].out_off >= h_recs[i - 1].out_off;
  std::vector<uint32_t> cuts(m + 1);
  int rc = tlsgpu_split_by_bytes(h_recs, n, ascending ? m : 1, cuts.data());
  if (rc != TLSGPU_OK) return rc;
  if (!ascending)
    for (uint32_t k = 2; k <= m; k++) cuts[k] = n;
  std::lock_guard<std::mutex> lk(g->mu);
  return run_members(g, [&](uint32_t k) -> int {
    const uint32_t a = cuts[k], b = cuts[k + 1];
    if (a == b) return TLSGPU_OK;
    return seal ? tlsgpu_seal_host(gs->members[k], h_recs + a, b - a, h_in, in_bytes, h_out,
                                   out_bytes, h_status + a)
                : tlsgpu_open_host(gs->members[k], h_recs + a, b - a, h_in, in_bytes, h_out,
                                   out_bytes, h_status + a);
  });
}

extern "C" int tlsgpu_group_open_host(tlsgpu_group_sessions* gs, const tlsgpu_record* h_recs,
                                      uint32_t n, const uint8_t* h_in, size_t in_bytes,
                                      uint8_t* h_out, size_t out_bytes, int32_t* h_status) {
  return group_host(gs, false, h_recs, n, h_in, in_bytes, h_out, out_bytes, h_status);
}

extern "C" int tlsgpu_group_seal_host(tlsgpu_group_sessions* gs, const tlsgpu_record* h_recs,
                                      uint32_t n, const uint8_t* h_in, size_t in_bytes,
                                      uint8_t* h_out, size_t out_bytes, int32_t* h_status) {
  if (n && h_out == h_in) return gfail(TLSGPU_EINVAL, "seal cannot run in place");
  return group_host(gs, true, h_recs, n, h_in, in_bytes, h_out, out_bytes, h_status);
}

// Device-resident: launches are asynchronous, so the caller's thread issues
// every member's batch on that member's engine stream back to back.
static int group_batch(tlsgpu_group_sessions* gs, bool seal, const tlsgpu_shard* shards) {
  if (!gs || !shards) return gfail(TLSGPU_EINVAL, "group batch: null sessions or shards");
  tlsgpu_group* g = gs->g;
  std::lock_guard<std::mutex> lk(g->mu);
  int rc = TLSGPU_OK;
  for (uint32_t k = 0; k < g->engines.size() && rc == TLSGPU_OK; k++) {
    const tlsgpu_shard& s = shards[k];
    rc = seal ? tlsgpu_seal_batch(gs->members[k], s.d_recs, s.n, s.d_in, s.in_bytes, s.d_out,
                                  s.out_bytes, s.d_status, nullptr)
              : tlsgpu_open_batch(gs->members[k], s.d_recs, s.n, s.d_in, s.in_bytes, s.d_out,
                                  s.out_bytes, s.d_status, nullptr);
  }
  return rc;
}

extern "C" int tlsgpu_group_open_batch(tlsgpu_group_sessions* gs, const tlsgpu_shard* shards) {
  return group_batch(gs, false, shards);
}

extern "C" int tlsgpu_group_seal_batch(tlsgpu_group_sessions* gs, const tlsgpu_shard* shards) {
  return group_batch(gs, true, shards);
}

extern "C" int tlsgpu_group_sync(tlsgpu_group* g) {
  if (!g) return TLSGPU_EINVAL;
  int rc = TLSGPU_OK;
  for (tlsgpu_engine* e : g->engines) {
    const int r = tlsgpu_engine_sync(e);
    if (rc == TLSGPU_OK) rc = r;
  }
  return rc;
}
