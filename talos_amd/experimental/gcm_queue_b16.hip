// gcm_queue_b16.hip — the no-pack queue kernel with 4 packed bitsliced waves
// (gcm_hy_kernel<…, B16W = 4>): T-table waves keep the LDS
// pipe busy while the bitsliced waves run AES on the VALU.  Selected by
// BatchArgs::bs16_min != 0 (env TLSGPU_BS16_MIN); its own translation unit so
// the bitsliced code compiles in parallel with gcm_queue.hip.
#include "../csrc/gcm_hybrid.h"

namespace tg {

#ifndef TG_QUEUE_NB
#define TG_QUEUE_NB 2
#endif

int launch_gcm_queue_b16(const BatchArgs& a, const RecPre* pre, bool seal, int rounds, int groups,
                         hipStream_t s) {
  const dim3 g(groups), b(1024);
  if (rounds == 10) {
    if (seal) hipLaunchKernelGGL((gcm_hy_kernel<true, 10, 1024, 0, TG_QUEUE_NB, false, 4>), g, b, 0, s, a, pre);
    else hipLaunchKernelGGL((gcm_hy_kernel<false, 10, 1024, 0, TG_QUEUE_NB, false, 4>), g, b, 0, s, a, pre);
  } else {
    if (seal) hipLaunchKernelGGL((gcm_hy_kernel<true, 14, 1024, 0, TG_QUEUE_NB, false, 4>), g, b, 0, s, a, pre);
    else hipLaunchKernelGGL((gcm_hy_kernel<false, 14, 1024, 0, TG_QUEUE_NB, false, 4>), g, b, 0, s, a, pre);
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace tg
