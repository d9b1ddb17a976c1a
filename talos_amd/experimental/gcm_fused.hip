// gcm_fused.hip — instantiations of the fused kernel (gcm_fused.h),
// TLSGPU_GCM_FUSED.  AES-128 and AES-256 build in their own translation units
// (gcm_fused.hip / gcm_fused256.hip) so they compile in parallel.
#include "gcm_fused.h"

namespace tg {

#ifndef TG_FUSED_ROUNDS
#define TG_FUSED_ROUNDS 10
#endif

#if TG_FUSED_ROUNDS == 10
int launch_gcm_fused10(const BatchArgs& a, const RecPre* pre, bool seal, int groups, hipStream_t s) {
#else
int launch_gcm_fused14(const BatchArgs& a, const RecPre* pre, bool seal, int groups, hipStream_t s) {
#endif
  if (a.n == 0) return 0;
#ifdef TG_DEV_QUEUE_ONLY
  return launch_gcm_queue(a, pre, seal, TG_FUSED_ROUNDS, groups, s);
#else
  const dim3 g(groups), b(kFuThreads);
#ifdef TG_DEV_OPEN128
  if (seal || TG_FUSED_ROUNDS != 10) return launch_gcm_queue(a, pre, seal, TG_FUSED_ROUNDS, groups, s);
  hipLaunchKernelGGL((gcm_fused_kernel<false, TG_FUSED_ROUNDS>), g, b, 0, s, a, pre);
#else
  if (seal) hipLaunchKernelGGL((gcm_fused_kernel<true, TG_FUSED_ROUNDS>), g, b, 0, s, a, pre);
  else hipLaunchKernelGGL((gcm_fused_kernel<false, TG_FUSED_ROUNDS>), g, b, 0, s, a, pre);
#endif
  return hipGetLastError() == hipSuccess ? 0 : -1;
#endif
}

}  // namespace tg
