// pool_probe.hip — does a kernel see the previous kernel's stores to
// stream-ordered pool memory (hipMallocAsync) on MI355X?  Root-cause probe for
// the RecPre stale reads of DESIGN.md §4.1 ("pool scratch").
//
// Per iteration: allocate `bytes` of scratch (pool: hipMallocAsync/hipFreeAsync
// on the stream; plain: one hipMalloc buffer reused), kernel W writes a
// pattern that depends on the iteration into it, kernel R reads it back from a
// DIFFERENT workgroup than the writer (workgroup w reads what w + shift wrote,
// so with 8 XCDs and round-robin workgroup placement the reader normally sits
// on another XCD, i.e. behind another L2) with vector loads and with scalar
// (s_load, address space 4) loads, and counts words that differ: stale from an
// earlier iteration, zero, or other.
// churn = 1: every iteration also hipMalloc's, fills (H2D) and, after the
// readback, hipFree's five ordinary buffers (1 KiB .. 1 MiB), the pattern of a
// loop of fresh batches (tests/test_gpu_parity.py::test_batch_repeated_fresh_batches).
// sync_alloc = 1: hipStreamSynchronize right after each hipMallocAsync.
// With sync = 1 the scratch is also copied back once the stream has drained
// and its zero words counted (end_zero_words): stores lost vs reads stale.
// fence = 1: the writer ends with a system-scope release fence and the reader
// starts with a system-scope acquire fence.
// usage: pool_probe MODE ITERS [shift] [sync] [churn] [fixed] [sync_alloc] [fence]
//        MODE = pool | plain | pool_keep
#include <hip/hip_runtime.h>

#include <algorithm>
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

typedef __attribute__((address_space(4))) const uint32_t cu32;

constexpr int kWG = 256;         // threads per workgroup
constexpr int kWords = 12;       // words per record (a RecPre is 48 B)
__device__ __forceinline__ uint32_t pat(uint32_t rec, uint32_t w, uint32_t it) {
  return (rec * 2654435761u) ^ (w * 40503u) ^ (it * 0x9E3779B9u) ^ 0x80000000u;  // never 0
}

// one record per thread; records [wg * kWG, (wg + 1) * kWG) written by wg
template <bool FENCE>
__global__ void writer(uint32_t* p, uint32_t n, uint32_t it) {
  const uint32_t r = blockIdx.x * kWG + threadIdx.x;
  if (r < n)
    for (int w = 0; w < kWords; w++) p[r * kWords + w] = pat(r, w, it);
  if (FENCE) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // system-scope release
}

// counts[0] vector mismatches, [1] of them zero, [2] of them equal to iteration it-1's value
// counts[3] scalar mismatches, [4] zero, [5] previous iteration
template <bool FENCE>
__global__ void reader(const uint32_t* p, uint32_t n, uint32_t it, uint32_t shift,
                       unsigned long long* counts) {
  if (FENCE) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // system-scope acquire
  const uint32_t g = (blockIdx.x + shift) % gridDim.x;  // read another workgroup's records
  const uint32_t r = g * kWG + threadIdx.x;
  uint32_t bad = 0, zero = 0, prev = 0;
  if (r < n) {
    for (int w = 0; w < kWords; w++) {
      const uint32_t v = p[r * kWords + w];
      if (v != pat(r, w, it)) {
        bad++;
        zero += v == 0;
        prev += it > 0 && v == pat(r, w, it - 1);
      }
    }
  }
  // scalar: each wave reads the first record of its 64 through s_load
  const uint32_t r0 = __builtin_amdgcn_readfirstlane(g * kWG + (threadIdx.x & ~63u));
  uint32_t sbad = 0, szero = 0, sprev = 0;
  if (r0 < n && (threadIdx.x & 63) == 0) {
    cu32* q = (cu32*)(p + r0 * kWords);
    for (int w = 0; w < kWords; w++) {
      const uint32_t v = q[w];
      if (v != pat(r0, w, it)) {
        sbad++;
        szero += v == 0;
        sprev += it > 0 && v == pat(r0, w, it - 1);
      }
    }
  }
  if (bad) { atomicAdd(counts + 0, bad); atomicAdd(counts + 1, zero); atomicAdd(counts + 2, prev); }
  if (sbad) { atomicAdd(counts + 3, sbad); atomicAdd(counts + 4, szero); atomicAdd(counts + 5, sprev); }
}

int main(int argc, char** argv) {
  if (argc < 3) {
    fprintf(stderr, "usage: %s pool|plain|pool_keep ITERS [shift] [sync]\n", argv[0]);
    return 2;
  }
  const char* mode = argv[1];
  const int iters = atoi(argv[2]);
  const uint32_t shift = argc > 3 ? (uint32_t)atoi(argv[3]) : 1;
  const int sync = argc > 4 ? atoi(argv[4]) : 1;
  const int churn = argc > 5 ? atoi(argv[5]) : 0;
  const int fixed = argc > 6 ? atoi(argv[6]) : 0;  // 1: every iteration the same size
  const int sync_alloc = argc > 7 ? atoi(argv[7]) : 0;  // 1: host sync right after hipMallocAsync
  const int fence = argc > 8 ? atoi(argv[8]) : 0;  // 1: system-scope release/acquire in the kernels
  static uint32_t back[(1u << 20) * kWords];
  unsigned long long end_zero = 0;  // zero words in the scratch after the iteration (host copy)
  static char hbuf[1 << 20];
  memset(hbuf, 0x5A, sizeof(hbuf));
  CK(hipSetDevice(0));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipMemPool_t pool;
  CK(hipDeviceGetDefaultMemPool(&pool, 0));
  if (!strcmp(mode, "pool_keep")) {  // keep freed pool memory mapped (release threshold max)
    uint64_t thr = ~0ull;
    CK(hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &thr));
  }
  const uint32_t sizes[4] = {65536, 1u << 20, 3 * 65536, 200000};  // records
  unsigned long long* d_counts;
  CK(hipMalloc(&d_counts, 6 * sizeof(unsigned long long)));
  CK(hipMemset(d_counts, 0, 6 * sizeof(unsigned long long)));
  uint32_t* plain = nullptr;
  if (!strcmp(mode, "plain")) CK(hipMalloc(&plain, (size_t)(1u << 20) * kWords * 4));
  unsigned long long tot[6] = {0, 0, 0, 0, 0, 0};
  int bad_iters = 0;
  uint32_t* last = nullptr;
  int same_va = 0;
  for (int it = 0; it < iters; it++) {
    const uint32_t n = fixed ? sizes[1] : sizes[it % 4];
    void* extra[5] = {};
    if (churn) {
      for (int k = 0; k < 5; k++) {
        const size_t b = (size_t)1024 << (2 * k);
        CK(hipMalloc(&extra[k], b));
        CK(hipMemcpy(extra[k], hbuf, b, hipMemcpyHostToDevice));
      }
    }
    uint32_t* p = plain;
    if (!plain) CK(hipMallocAsync((void**)&p, (size_t)n * kWords * 4, s));
    if (sync_alloc) CK(hipStreamSynchronize(s));
    same_va += p == last;
    last = p;
    const uint32_t groups = (n + kWG - 1) / kWG;
    if (fence) {
      hipLaunchKernelGGL(writer<true>, dim3(groups), dim3(kWG), 0, s, p, n, (uint32_t)it);
      hipLaunchKernelGGL(reader<true>, dim3(groups), dim3(kWG), 0, s, p, n, (uint32_t)it, shift,
                         d_counts);
    } else {
      hipLaunchKernelGGL(writer<false>, dim3(groups), dim3(kWG), 0, s, p, n, (uint32_t)it);
      hipLaunchKernelGGL(reader<false>, dim3(groups), dim3(kWG), 0, s, p, n, (uint32_t)it, shift,
                         d_counts);
    }
    if (sync) {  // what the scratch holds once the stream has drained (before the free)
      CK(hipMemcpyAsync(back, p, (size_t)n * kWords * 4, hipMemcpyDeviceToHost, s));
      CK(hipStreamSynchronize(s));
      unsigned long long z = 0;
      for (size_t k = 0; k < (size_t)n * kWords; k++) z += back[k] == 0;
      if (z) {
        // which 2 MiB pages (from the allocation base) hold the zeros, and how fully
        const size_t words = (size_t)n * kWords, per = (2u << 20) / 4;
        fprintf(stderr, "iter %d: %llu zero words in the scratch after the stream drained; base %p; "
                "2MiB pages (index:zero%%):", it, z, (void*)p);
        for (size_t pg = 0; pg * per < words; pg++) {
          size_t zz = 0, m = std::min(words, (pg + 1) * per);
          for (size_t k = pg * per; k < m; k++) zz += back[k] == 0;
          if (zz) fprintf(stderr, " %zu:%.0f", pg, 100.0 * zz / (m - pg * per));
        }
        fprintf(stderr, "\n");
      }
      end_zero += z;
    }
    if (!plain) CK(hipFreeAsync(p, s));
    if (sync) {
      unsigned long long c[6];
      CK(hipMemcpyAsync(c, d_counts, sizeof(c), hipMemcpyDeviceToHost, s));
      CK(hipStreamSynchronize(s));
      CK(hipMemsetAsync(d_counts, 0, sizeof(c), s));
      bool any = false;
      for (int k = 0; k < 6; k++) { tot[k] += c[k]; any |= c[k] != 0; }
      if (any)
        fprintf(stderr, "bad iter %d records %u prev records %u vec_bad %llu s_bad %llu\n", it, n,
                it ? (fixed ? sizes[1] : sizes[(it - 1) % 4]) : 0, c[0], c[3]);
      bad_iters += any;
    }
    for (void* e : extra)
      if (e) CK(hipFree(e));
  }
  if (!sync) {
    CK(hipMemcpy(tot, d_counts, sizeof(tot), hipMemcpyDeviceToHost));
  }
  CK(hipStreamSynchronize(s));
  hipPointerAttribute_t at;
  memset(&at, 0, sizeof(at));
  const hipError_t ae = hipPointerGetAttributes(&at, last);
  printf("{\"mode\": \"%s\", \"fence\": %d, \"sync_alloc\": %d, \"end_zero_words\": %llu, \"fixed\": %d, \"churn\": %d, \"iters\": %d, \"shift\": %u, \"sync\": %d, \"same_va_iters\": %d, "
         "\"bad_iters\": %d, \"vec_bad\": %llu, \"vec_zero\": %llu, \"vec_prev\": %llu, "
         "\"s_bad\": %llu, \"s_zero\": %llu, \"s_prev\": %llu, \"attr_ok\": %d, \"mem_type\": %d}\n",
         mode, fence, sync_alloc, end_zero, fixed, churn, iters, shift, sync, same_va, bad_iters, tot[0], tot[1], tot[2], tot[3], tot[4],
         tot[5], ae == hipSuccess, (int)at.type);
  return 0;
}
