// pcie_probe.hip — host<->device bandwidth on this box by copy engine (SDMA,
// hipMemcpyAsync) and by shader zero-copy (a kernel loading / storing pinned
// host memory directly), each direction alone and both at once.  Sizing for
// the host-resident record path (tlsgpu_open_host).
// usage: pcie_probe [MiB] [coherent|noncoherent]
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

__global__ void copy16(const uint4* __restrict__ src, uint4* __restrict__ dst, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x)
    dst[i] = src[i];
}

// two copies in one launch: first half of the grid copies a->b, second half c->d
__global__ void copy16x2(const uint4* __restrict__ a, uint4* __restrict__ b,
                         const uint4* __restrict__ c, uint4* __restrict__ d, size_t n) {
  const uint32_t half = gridDim.x / 2;
  const bool second = blockIdx.x >= half;
  const uint4* src = second ? c : a;
  uint4* dst = second ? d : b;
  const size_t g = (second ? blockIdx.x - half : blockIdx.x);
  for (size_t i = g * blockDim.x + threadIdx.x; i < n; i += (size_t)half * blockDim.x)
    dst[i] = src[i];
}

static double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  const size_t mib = argc > 1 ? (size_t)atoi(argv[1]) : 1024;
  const bool nc = argc > 2 && !strcmp(argv[2], "noncoherent");
  const size_t bytes = mib << 20, n16 = bytes / 16;
  CK(hipSetDevice(0));
  uint8_t *h_in, *h_out, *d_a, *d_b;
  const unsigned fl = nc ? hipHostMallocNonCoherent : hipHostMallocDefault;
  CK(hipHostMalloc((void**)&h_in, bytes, fl));
  CK(hipHostMalloc((void**)&h_out, bytes, fl));
  CK(hipMalloc((void**)&d_a, bytes));
  CK(hipMalloc((void**)&d_b, bytes));
  memset(h_in, 1, bytes);
  memset(h_out, 2, bytes);
  hipStream_t s0, s1;
  CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int grid = cus * 8;
  auto timeit = [&](auto&& f) {
    f();
    CK(hipDeviceSynchronize());
    double best = 1e30;
    for (int r = 0; r < 3; r++) {
      const double t0 = now_s();
      f();
      CK(hipDeviceSynchronize());
      best = std::min(best, now_s() - t0);
    }
    return best;
  };
  const double gb = bytes / 1e9;
  printf("{\"mib\": %zu, \"host_mem\": \"%s\"", mib, nc ? "noncoherent" : "coherent");
  double t;
  t = timeit([&] { CK(hipMemcpyAsync(d_a, h_in, bytes, hipMemcpyHostToDevice, s0)); });
  printf(", \"sdma_h2d_GBs\": %.1f", gb / t);
  t = timeit([&] { CK(hipMemcpyAsync(h_out, d_b, bytes, hipMemcpyDeviceToHost, s0)); });
  printf(", \"sdma_d2h_GBs\": %.1f", gb / t);
  t = timeit([&] {
    CK(hipMemcpyAsync(d_a, h_in, bytes, hipMemcpyHostToDevice, s0));
    CK(hipMemcpyAsync(h_out, d_b, bytes, hipMemcpyDeviceToHost, s1));
  });
  printf(", \"sdma_both_GBs_total\": %.1f", 2 * gb / t);
  t = timeit([&] { hipLaunchKernelGGL(copy16, dim3(grid), dim3(256), 0, s0, (const uint4*)h_in, (uint4*)d_a, n16); });
  printf(", \"zc_h2d_GBs\": %.1f", gb / t);
  t = timeit([&] { hipLaunchKernelGGL(copy16, dim3(grid), dim3(256), 0, s0, (const uint4*)d_b, (uint4*)h_out, n16); });
  printf(", \"zc_d2h_GBs\": %.1f", gb / t);
  t = timeit([&] {
    hipLaunchKernelGGL(copy16x2, dim3(2 * grid), dim3(256), 0, s0, (const uint4*)h_in, (uint4*)d_a,
                       (const uint4*)d_b, (uint4*)h_out, n16);
  });
  printf(", \"zc_both_GBs_total\": %.1f", 2 * gb / t);
  t = timeit([&] { hipLaunchKernelGGL(copy16, dim3(grid), dim3(256), 0, s0, (const uint4*)h_in, (uint4*)h_out, n16); });
  printf(", \"zc_host_to_host_GBs_each_way\": %.1f", gb / t);
  t = timeit([&] {
    hipLaunchKernelGGL(copy16, dim3(grid), dim3(256), 0, s0, (const uint4*)h_in, (uint4*)d_a, n16);
    CK(hipMemcpyAsync(h_out, d_b, bytes, hipMemcpyDeviceToHost, s1));
  });
  printf(", \"zc_h2d_plus_sdma_d2h_GBs_total\": %.1f", 2 * gb / t);
  t = timeit([&] {
    CK(hipMemcpyAsync(d_a, h_in, bytes, hipMemcpyHostToDevice, s1));
    hipLaunchKernelGGL(copy16, dim3(grid), dim3(256), 0, s0, (const uint4*)d_b, (uint4*)h_out, n16);
  });
  printf(", \"sdma_h2d_plus_zc_d2h_GBs_total\": %.1f}\n", 2 * gb / t);
  return 0;
}
