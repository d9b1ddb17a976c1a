// gcm_queue.hip — the per-record prep pass and the T-table queue kernel
// (gcm_hy_kernel<1024 threads, no bitsliced waves, 2 blocks per lane>), the
// default AES-GCM TLS batch path.
#include "gcm_hybrid.h"

namespace tg {

#ifndef TG_QUEUE_NB
#define TG_QUEUE_NB 2
#endif

int launch_gcm_prep(const BatchArgs& a, RecPre* pre, bool seal, int rounds, hipStream_t s) {
  if (a.n == 0) return 0;
  const dim3 g((a.n + kPrepThreads - 1) / kPrepThreads), b(kPrepThreads);
  if (rounds == 10) {
    if (seal) hipLaunchKernelGGL((gcm_prep_kernel<true, 10>), g, b, 0, s, a, pre);
    else hipLaunchKernelGGL((gcm_prep_kernel<false, 10>), g, b, 0, s, a, pre);
  } else {
    if (seal) hipLaunchKernelGGL((gcm_prep_kernel<true, 14>), g, b, 0, s, a, pre);
    else hipLaunchKernelGGL((gcm_prep_kernel<false, 14>), g, b, 0, s, a, pre);
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// Work-balanced ranges (round 5, engine.cpp run_batch): the work
// (cut_work_of) of each count range [g * rpg, (g + 1) * rpg), one workgroup
// per range; the queue kernel's prologue cuts the batch at equal work from
// these sums (work_cut, gcm_hybrid.h).  Reads 4 bytes of each 32-byte
// descriptor: ~8 MiB of lines for 256 Ki records, a few microseconds.
__global__ __launch_bounds__(256) void range_work_kernel(const tlsgpu_record* __restrict__ D,
                                                         uint32_t n, uint32_t rpg,
                                                         unsigned long long* __restrict__ out) {
  __shared__ unsigned long long part[4];
  const uint32_t lo = blockIdx.x * rpg, hi = min(n, lo + rpg);
  unsigned long long s = 0;
  for (uint32_t i = lo + threadIdx.x; i < hi; i += 256) s += cut_work_of(D[i].len_type);
  for (int d = 32; d > 0; d >>= 1) s += __shfl_down(s, d);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) out[blockIdx.x] = part[0] + part[1] + part[2] + part[3];
}

int launch_range_work(const BatchArgs& a, int groups, unsigned long long* out, hipStream_t s) {
  if (a.n == 0 || groups <= 0) return 0;
  hipLaunchKernelGGL(range_work_kernel, dim3(groups), dim3(256), 0, s,
                     reinterpret_cast<const tlsgpu_record*>(a.descs), a.n, a.records_per_group, out);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_gcm_queue(const BatchArgs& a, const RecPre* pre, bool seal, int rounds, int groups,
                     hipStream_t s) {
  if (a.n == 0) return 0;
  const dim3 g(groups), b(1024);
#ifdef TG_EXPERIMENTAL
  if (a.bs16_min != 0 && a.sel) {  // no-pack variant with bitsliced waves (gcm_queue_b16.hip)
    if (launch_gcm_queue_b16(a, pre, seal, rounds, groups, s)) return -1;
  } else
#endif
  if (a.fused && a.pack) {
    // fused (engine.cpp run_batch): only the pack variant runs, with its own prologue
  } else if (rounds == 10) {
    if (seal) hipLaunchKernelGGL((gcm_hy_kernel<true, 10, 1024, 0, TG_QUEUE_NB>), g, b, 0, s, a, pre);
    else hipLaunchKernelGGL((gcm_hy_kernel<false, 10, 1024, 0, TG_QUEUE_NB>), g, b, 0, s, a, pre);
  } else {
    if (seal) hipLaunchKernelGGL((gcm_hy_kernel<true, 14, 1024, 0, TG_QUEUE_NB>), g, b, 0, s, a, pre);
    else hipLaunchKernelGGL((gcm_hy_kernel<false, 14, 1024, 0, TG_QUEUE_NB>), g, b, 0, s, a, pre);
  }
  if ((a.sel || a.fused) && a.pack) {  // the pack variant: runs instead when the prep pass saw a short record
    if (rounds == 10) {
      if (seal) hipLaunchKernelGGL((gcm_hy_kernel<true, 10, 1024, 0, TG_QUEUE_NB, true>), g, b, 0, s, a, pre);
      else hipLaunchKernelGGL((gcm_hy_kernel<false, 10, 1024, 0, TG_QUEUE_NB, true>), g, b, 0, s, a, pre);
    } else {
      if (seal) hipLaunchKernelGGL((gcm_hy_kernel<true, 14, 1024, 0, TG_QUEUE_NB, true>), g, b, 0, s, a, pre);
      else hipLaunchKernelGGL((gcm_hy_kernel<false, 14, 1024, 0, TG_QUEUE_NB, true>), g, b, 0, s, a, pre);
    }
  }
  if (a.sel && a.pws != 1 && hipGetLastError() == hipSuccess)  // per-wave sessions (gcm_pw.hip)
    return launch_gcm_pw(a, pre, seal, rounds, groups, s);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace tg
