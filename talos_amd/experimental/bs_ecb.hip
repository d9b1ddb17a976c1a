// bs_ecb.hip — diagnostic self-test of the bitsliced AES core (bs_aes.h):
// ECB encryption under a session's key, checked bit-exact against the oracle
// by tests/test_gpu_parity.py (tlsgpu_aes_ecb_bitsliced).
#include "../csrc/gcm_device.h"

namespace tg {

// Self-test of the bitsliced core: ECB encryption of nblocks blocks, 32 per lane.
template <int ROUNDS>
__global__ __launch_bounds__(256) void bs_ecb_kernel(const DevSession* __restrict__ sessions,
                                                     uint32_t sid, const uint4* __restrict__ in,
                                                     uint4* __restrict__ out, uint32_t nblocks) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t st[128];
#pragma unroll
  for (int j = 0; j < 32; j++) {
    const uint32_t blk = g * 32 + j;
    const uint4 v = blk < nblocks ? in[blk] : make_uint4(0, 0, 0, 0);
    st[j] = v.x; st[32 + j] = v.y; st[64 + j] = v.z; st[96 + j] = v.w;
  }
  transpose_all(st);
  bs_encrypt<ROUNDS, false>(st, SgprMasks{as_const(sessions[sid].rk)});
  transpose_all(st);
#pragma unroll
  for (int j = 0; j < 32; j++) {
    const uint32_t blk = g * 32 + j;
    if (blk < nblocks) out[blk] = make_uint4(st[j], st[32 + j], st[64 + j], st[96 + j]);
  }
}

int launch_bs_ecb(const DevSession* sessions, uint32_t session, int rounds, const void* d_in,
                  void* d_out, uint32_t nblocks, hipStream_t s) {
  if (nblocks == 0) return 0;
  const uint32_t lanes = (nblocks + 31) / 32, groups = (lanes + 255) / 256;
  if (rounds == 10)
    hipLaunchKernelGGL((bs_ecb_kernel<10>), dim3(groups), dim3(256), 0, s, sessions, session,
                       (const uint4*)d_in, (uint4*)d_out, nblocks);
  else
    hipLaunchKernelGGL((bs_ecb_kernel<14>), dim3(groups), dim3(256), 0, s, sessions, session,
                       (const uint4*)d_in, (uint4*)d_out, nblocks);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace tg
