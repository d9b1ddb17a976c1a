// doorbell_probe.hip — the floor of a persistent-kernel ("doorbell") EVP call
// path on this box, before building it into the
// engine:
//   * ping-pong: one host thread bumps a word in pinned host memory, one wave of
//     a persistent kernel polling that word answers in another word; host-side
//     round trip per call, for 1 and T threads (T slots, T polling waves);
//   * zero-copy job: the same, with the wave reading 1,400 B of "input" from
//     pinned memory and writing 1,400 B back before it answers;
//   * side traffic: while the server kernel runs, an empty kernel launched on
//     each of S other streams must still complete (the box has
//     GPU_MAX_HW_QUEUES = 4: a stream that shared the server's hardware queue
//     would wait for the server to exit) — latency per launch reported.
// The server kernel exits on a stop word or after its lifetime (s_memrealtime),
// whichever comes first: no run can leave it spinning.
// usage: doorbell_probe
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));  \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

struct alignas(128) Slot {
  uint32_t post;  // host: sequence number of the posted call
  uint32_t done;  // device: sequence number answered
  uint32_t bytes;
  uint32_t pad[29];
};

__device__ __forceinline__ uint32_t sys_load(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void sys_store(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// one wave per slot; lane 0 polls.  data: per slot 2 x 4 KiB (in, out)
__global__ void __launch_bounds__(64) server(Slot* slots, const uint32_t* stop, uint8_t* data,
                                             unsigned long long lifetime) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  Slot* s = slots + blockIdx.x;
  uint32_t seen = 0;
  const uint32_t lane = threadIdx.x;
  for (;;) {
    uint32_t p = 0, quit = 0;
    if (lane == 0) {
      p = sys_load(&s->post);
      quit = sys_load(stop) | (__builtin_amdgcn_s_memrealtime() - t0 > lifetime);
    }
    p = __shfl(p, 0);
    quit = __shfl(quit, 0);
    if (p != seen) {
      const uint32_t n = sys_load(&s->bytes);
      const uint4* in = reinterpret_cast<const uint4*>(data + blockIdx.x * 8192);
      uint4* out = reinterpret_cast<uint4*>(data + blockIdx.x * 8192 + 4096);
      for (uint32_t i = lane; i < (n + 15) / 16; i += 64) {
        uint4 v = in[i];
        v.x ^= p;
        out[i] = v;
      }
      __builtin_amdgcn_s_waitcnt(0);
      __atomic_thread_fence(__ATOMIC_RELEASE);  // system scope: host sees out before done
      if (lane == 0) sys_store(&s->done, p);
      seen = p;
      continue;
    }
    if (quit) break;
    __builtin_amdgcn_s_sleep(1);
  }
}

__global__ void empty_kernel() {}

// a launched one-job kernel that signals completion in pinned memory: the host
// spins on the word instead of waiting for the stream / event
__global__ void __launch_bounds__(64) signal_kernel(uint32_t* flag, uint32_t v, const uint8_t* in,
                                                    uint8_t* out, uint32_t n) {
  const uint4* i4 = reinterpret_cast<const uint4*>(in);
  uint4* o4 = reinterpret_cast<uint4*>(out);
  for (uint32_t i = threadIdx.x; i < (n + 15) / 16; i += 64) o4[i] = i4[i];
  __builtin_amdgcn_s_waitcnt(0);
  __atomic_thread_fence(__ATOMIC_RELEASE);
  if (threadIdx.x == 0) sys_store(flag, v);
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

int main() {
  const int kSlots = 64;
  Slot* slots;
  uint32_t* stop;
  uint8_t* data;
  CK(hipHostMalloc((void**)&slots, sizeof(Slot) * kSlots, hipHostMallocDefault));
  CK(hipHostMalloc((void**)&stop, 64, hipHostMallocDefault));
  CK(hipHostMalloc((void**)&data, 8192 * kSlots, hipHostMallocDefault));
  memset(slots, 0, sizeof(Slot) * kSlots);
  memset(data, 7, 8192 * kSlots);
  *stop = 0;
  Slot* d_slots;
  uint32_t* d_stop;
  uint8_t* d_data;
  CK(hipHostGetDevicePointer((void**)&d_slots, slots, 0));
  CK(hipHostGetDevicePointer((void**)&d_stop, stop, 0));
  CK(hipHostGetDevicePointer((void**)&d_data, data, 0));
  hipStream_t srv;
  CK(hipStreamCreateWithFlags(&srv, hipStreamNonBlocking));
  // lifetime 3 s of the 100 MHz realtime counter: the probe ends well before
  server<<<kSlots, 64, 0, srv>>>(d_slots, d_stop, d_data, 300000000ull);
  CK(hipGetLastError());
  printf("{\"bench\": \"doorbell\"");
  // ping-pong and zero-copy job, T threads each on its own slot
  for (uint32_t bytes : {0u, 1400u}) {
    for (int T : {1, 4, 16, 32}) {
      const int iters = 2000;
      std::vector<std::thread> th;
      std::atomic<int> bad{0};
      const double t0 = now_us();
      for (int t = 0; t < T; t++)
        th.emplace_back([&, t] {
          Slot* s = slots + t;
          uint32_t seq = __atomic_load_n(&s->done, __ATOMIC_ACQUIRE);
          for (int i = 0; i < iters; i++) {
            __atomic_store_n(&s->bytes, bytes, __ATOMIC_RELAXED);
            __atomic_store_n(&s->post, ++seq, __ATOMIC_RELEASE);
            long spins = 0;
            while (__atomic_load_n(&s->done, __ATOMIC_ACQUIRE) != seq) {
              __builtin_ia32_pause();
              if (++spins > 200000000L) {  // ~seconds: the server is gone
                bad++;
                return;
              }
            }
            if (bytes && data[t * 8192 + 4096] != (uint8_t)(7 ^ (seq & 0xFF))) bad++;
          }
        });
      for (auto& x : th) x.join();
      const double dt = now_us() - t0;
      printf(", \"rt_%uB_T%d_us\": %.2f, \"calls_%uB_T%d_per_s\": %.0f", bytes, T,
             dt / iters, bytes, T, (double)iters * T / (dt * 1e-6));
      if (bad) printf(", \"errors_%uB_T%d\": %d", bytes, T, bad.load());
    }
  }
  // launch per call: event sync vs host spin on a pinned flag (1400 B job)
  {
    hipStream_t ls;
    hipEvent_t ev;
    CK(hipStreamCreateWithFlags(&ls, hipStreamNonBlocking));
    CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    uint32_t* flag = reinterpret_cast<uint32_t*>(data + 8192 * (kSlots - 1));
    uint32_t* d_flag = reinterpret_cast<uint32_t*>(d_data + 8192 * (kSlots - 1));
    const uint8_t* d_in = d_data + 8192 * (kSlots - 2);
    uint8_t* d_out = d_data + 8192 * (kSlots - 2) + 4096;
    const int iters = 2000;
    for (int mode = 0; mode < 2; mode++) {
      const double t0 = now_us();
      for (int i = 1; i <= iters; i++) {
        signal_kernel<<<1, 64, 0, ls>>>(d_flag, (uint32_t)i + mode * iters, d_in, d_out, 1400);
        if (mode == 0) {
          CK(hipEventRecord(ev, ls));
          CK(hipEventSynchronize(ev));
        } else {
          long spins = 0;
          while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != (uint32_t)i + iters)
            if (++spins > 2000000000L) break;
        }
      }
      printf(", \"launch_%s_1400B_us\": %.2f", mode ? "spin" : "eventsync", (now_us() - t0) / iters);
    }
    CK(hipStreamSynchronize(ls));
  }
  // side traffic on other streams while the server runs
  for (int S : {1, 4, 8}) {
    std::vector<hipStream_t> ss(S);
    for (auto& x : ss) CK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
    double worst = 0;
    for (int rep = 0; rep < 20; rep++)
      for (auto& x : ss) {
        const double t0 = now_us();
        empty_kernel<<<1, 64, 0, x>>>();
        CK(hipStreamSynchronize(x));
        worst = std::max(worst, now_us() - t0);
      }
    printf(", \"side_launch_streams%d_worst_us\": %.1f", S, worst);
    for (auto& x : ss) CK(hipStreamDestroy(x));
  }
  __atomic_store_n(stop, 1u, __ATOMIC_RELEASE);
  const double t0 = now_us();
  CK(hipStreamSynchronize(srv));
  printf(", \"stop_to_exit_us\": %.1f}\n", now_us() - t0);
  return 0;
}
