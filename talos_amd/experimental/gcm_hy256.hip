// gcm_hy256.hip — AES-256-GCM instantiations of gcm_hy_kernel with
// bitsliced waves: 4 of 8 (TLSGPU_GCM_HYBRID) or all 8 (TLSGPU_GCM_BITSLICE).
#include "../csrc/gcm_hybrid.h"

namespace tg {

int launch_gcm_hy14(const BatchArgs& a, const RecPre* pre, bool seal, int bs_waves, int groups,
                     hipStream_t s) {
  if (a.n == 0) return 0;
#ifdef TG_DEV_QUEUE_ONLY
  return launch_gcm_queue(a, pre, seal, 14, groups, s);
#else
  const dim3 g(groups), b(kHyThreads);
#ifdef TG_DEV_OPEN128
  if (seal || 14 != 10 || bs_waves != kHyBsWaves) return launch_gcm_queue(a, pre, seal, 14, groups, s);
  hipLaunchKernelGGL((gcm_hy_kernel<false, 14, kHyThreads, kHyBsWaves, 4>), g, b, 0, s, a, pre);
#else
  if (bs_waves == kHyBsWaves) {
    if (seal) hipLaunchKernelGGL((gcm_hy_kernel<true, 14, kHyThreads, kHyBsWaves, 4>), g, b, 0, s, a, pre);
    else hipLaunchKernelGGL((gcm_hy_kernel<false, 14, kHyThreads, kHyBsWaves, 4>), g, b, 0, s, a, pre);
  } else {
    if (seal) hipLaunchKernelGGL((gcm_hy_kernel<true, 14, kHyThreads, 8, 4>), g, b, 0, s, a, pre);
    else hipLaunchKernelGGL((gcm_hy_kernel<false, 14, kHyThreads, 8, 4>), g, b, 0, s, a, pre);
  }
#endif
  return hipGetLastError() == hipSuccess ? 0 : -1;
#endif
}

}  // namespace tg
