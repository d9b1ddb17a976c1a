// hip_latency.hip — HIP runtime round-trip latencies on this box, the budget
// of one synchronous EVP call (engine.cpp gpu_call_impl / the EVP queue):
// empty kernel, small pinned H2D / D2H, event vs stream sync, zero-copy kernel
// access to pinned host memory, and the same from T concurrent threads.
// usage: hip_latency [spin]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));      \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

__global__ void empty_kernel(int* p) {
  if (p && threadIdx.x == 0 && blockIdx.x == 0) p[0] += 1;
}

// reads n uint4 from src (host or device) and writes them to dst
__global__ void copy_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x)
    dst[i] = src[i];
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

struct Ctx {
  hipStream_t s;
  hipEvent_t ev;
  uint8_t *h, *d, *h2;
  int* dflag;
};

static Ctx make_ctx() {
  Ctx c;
  CK(hipStreamCreateWithFlags(&c.s, hipStreamNonBlocking));
  CK(hipEventCreateWithFlags(&c.ev, hipEventDisableTiming));
  CK(hipHostMalloc((void**)&c.h, 1 << 20, hipHostMallocDefault));
  CK(hipHostMalloc((void**)&c.h2, 1 << 20, hipHostMallocDefault));
  CK(hipMalloc((void**)&c.d, 1 << 20));
  CK(hipMalloc((void**)&c.dflag, 64));
  memset(c.h, 1, 1 << 20);
  return c;
}

// one "call" shape; returns µs per iteration
static double run(Ctx& c, int what, int iters) {
  for (int w = 0; w < 2; w++) {
    double t0 = now_us();
    for (int i = 0; i < iters; i++) {
      switch (what) {
        case 0:  // empty kernel + stream sync
          hipLaunchKernelGGL(empty_kernel, 1, 64, 0, c.s, c.dflag);
          CK(hipStreamSynchronize(c.s));
          break;
        case 1:  // empty kernel + event sync
          hipLaunchKernelGGL(empty_kernel, 1, 64, 0, c.s, c.dflag);
          CK(hipEventRecord(c.ev, c.s));
          CK(hipEventSynchronize(c.ev));
          break;
        case 2:  // 4 KiB H2D + sync
          CK(hipMemcpyAsync(c.d, c.h, 4096, hipMemcpyHostToDevice, c.s));
          CK(hipStreamSynchronize(c.s));
          break;
        case 3:  // 4 KiB D2H + sync
          CK(hipMemcpyAsync(c.h, c.d, 4096, hipMemcpyDeviceToHost, c.s));
          CK(hipStreamSynchronize(c.s));
          break;
        case 4:  // EVP call shape: H2D 4 KiB, kernel, D2H 4 KiB, sync
          CK(hipMemcpyAsync(c.d, c.h, 4096, hipMemcpyHostToDevice, c.s));
          hipLaunchKernelGGL(empty_kernel, 1, 64, 0, c.s, c.dflag);
          CK(hipMemcpyAsync(c.h, c.d, 4096, hipMemcpyDeviceToHost, c.s));
          CK(hipStreamSynchronize(c.s));
          break;
        case 5:  // zero-copy: kernel reads 4 KiB pinned host, writes 4 KiB pinned host
          hipLaunchKernelGGL(copy_kernel, 1, 256, 0, c.s, (const uint4*)c.h, (uint4*)c.h2,
                             (size_t)256);
          CK(hipStreamSynchronize(c.s));
          break;
        case 6:  // same as 4 with 64 KiB each way
          CK(hipMemcpyAsync(c.d, c.h, 65536, hipMemcpyHostToDevice, c.s));
          hipLaunchKernelGGL(empty_kernel, 1, 64, 0, c.s, c.dflag);
          CK(hipMemcpyAsync(c.h, c.d, 65536, hipMemcpyDeviceToHost, c.s));
          CK(hipStreamSynchronize(c.s));
          break;
        case 7:  // zero-copy 64 KiB each way
          hipLaunchKernelGGL(copy_kernel, 16, 256, 0, c.s, (const uint4*)c.h, (uint4*)c.h2,
                             (size_t)4096);
          CK(hipStreamSynchronize(c.s));
          break;
        case 8:  // zero-copy 1 MiB each way
          hipLaunchKernelGGL(copy_kernel, 256, 256, 0, c.s, (const uint4*)c.h, (uint4*)c.h2,
                             (size_t)65536);
          CK(hipStreamSynchronize(c.s));
          break;
        case 9:  // copies 1 MiB each way
          CK(hipMemcpyAsync(c.d, c.h, 1 << 20, hipMemcpyHostToDevice, c.s));
          hipLaunchKernelGGL(empty_kernel, 1, 64, 0, c.s, c.dflag);
          CK(hipMemcpyAsync(c.h, c.d, 1 << 20, hipMemcpyDeviceToHost, c.s));
          CK(hipStreamSynchronize(c.s));
          break;
      }
    }
    double t = (now_us() - t0) / iters;
    if (w == 1) return t;
  }
  return 0;
}

int main(int argc, char** argv) {
  if (argc > 1 && !strcmp(argv[1], "spin")) CK(hipSetDeviceFlags(hipDeviceScheduleSpin));
  if (argc > 1 && !strcmp(argv[1], "yield")) CK(hipSetDeviceFlags(hipDeviceScheduleYield));
  if (argc > 1 && !strcmp(argv[1], "block")) CK(hipSetDeviceFlags(hipDeviceScheduleBlockingSync));
  CK(hipSetDevice(0));
  const char* names[] = {"kernel+streamsync", "kernel+eventsync", "h2d4k", "d2h4k",
                         "evp_shape_4k",      "zerocopy4k",       "evp_shape_64k",
                         "zerocopy64k",       "zerocopy1m",       "evp_shape_1m"};
  printf("{\"mode\": \"%s\"", argc > 1 ? argv[1] : "default");
  Ctx c = make_ctx();
  for (int w = 0; w < 10; w++) printf(", \"%s_us\": %.2f", names[w], run(c, w, 300));
  // concurrency: T threads each doing the EVP shape on their own stream
  for (int T : {4, 16, 64}) {
    std::vector<Ctx> cs;
    for (int i = 0; i < T; i++) cs.push_back(make_ctx());
    std::vector<std::thread> th;
    double t0 = now_us();
    const int iters = 200;
    for (int i = 0; i < T; i++) th.emplace_back([&, i] { run(cs[i], 4, iters); });
    for (auto& t : th) t.join();
    double dt = now_us() - t0;
    printf(", \"evp_shape_4k_T%d_calls_per_s\": %.0f", T, 2.0 * iters * T / (dt * 1e-6));
    th.clear();
    t0 = now_us();
    for (int i = 0; i < T; i++) th.emplace_back([&, i] { run(cs[i], 5, iters); });
    for (auto& t : th) t.join();
    dt = now_us() - t0;
    printf(", \"zerocopy4k_T%d_calls_per_s\": %.0f", T, 2.0 * iters * T / (dt * 1e-6));
  }
  printf("}\n");
  return 0;
}
