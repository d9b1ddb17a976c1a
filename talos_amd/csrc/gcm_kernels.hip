// gcm_kernels.hip — AES-GCM TLS record open/seal for gfx950 (MI355X).
//
// Replaces, per record, aead_aes_gcm_open/seal (crypto/evp/e_aes.c:1424-1510)
// driven by tls1_enc (ssl/t1_enc.c:832-975), i.e. CRYPTO_gcm128_setiv
// (gcm128.c:749-824), _aad (:826-881), _decrypt_ctr32/_encrypt_ctr32
// (:1242-1475, inc32 counter), _finish/_tag (:1477-1521) and the
// constant-time tag check (e_aes.c:1502) with zero-fill on failure
// (evp_aead.c:137-143).
//
// Layout and mapping:
//   * persistent workgroups of 16 waves, one per CU, each owning a contiguous
//     range of records; a record is processed by one wave, block i of the
//     record by lane i % 64 at step i / 64 (coalesced 16-B lane accesses);
//   * LDS (one array, 147,520 B):
//       AES  [0, 64K):      row x = 32 bank-replicated copies of Te0[x] then of
//                           Te1[x]; address = v_perm(state byte, lane bank) so a
//                           lookup is 1 VALU + 1 conflict-free ds_read_b32;
//       KTAB [64K, 128K):   T[j][b] = (byte b at position j) * H^64, row b,
//                           slot j; lane m = lane%16 reads position (k+m)%16
//                           at step k (its state pre-rotated by m bytes) so the
//                           16 lanes of every ds_read_b128 group hit 16
//                           different slots: conflict-free GHASH lookups;
//       SHOUP [128K, +20K): 4-bit tables of H^1..H^65 (column = power) for the per-lane final
//                           multiply; REM4: 16-entry reduction table;
//   * GHASH: lane l runs a Horner chain x <- x*H^64 ^ E_j over the extended
//     block sequence E = [AAD', C_0..C_{nb-1}, lengths] (j = l mod 64), then
//     y_l = x_l * H^(nb+1-jlast_l) and an XOR butterfly across the wave.
#include "gcm_device.h"
#include "gcm_raw.h"

namespace tg {

template <bool SEAL, bool RAW, int ROUNDS>
__global__ __launch_bounds__(kThreads, 1) void gcm_batch_kernel(BatchArgs a) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t laneoff = aes_laneoff(lane);
  const GhLane gl = gh_lane(lane);

  fill_aes_lds<kThreads>();

  const uint32_t rlo = blockIdx.x * a.records_per_group;
  const uint32_t rhi = min(a.n, rlo + a.records_per_group);
  uint32_t cur = 0xFFFFFFFFu;
  uint32_t pos = rlo;
  while (pos < rhi) {
    // session id of this run (wave-uniform; every wave computes the same run)
    const uint32_t sid = __builtin_amdgcn_readfirstlane(
        RAW ? reinterpret_cast<const RawJob*>(a.descs)[pos].session
            : reinterpret_cast<const tlsgpu_record*>(a.descs)[pos].session);
    uint32_t run_end = pos + 1;
    while (run_end < rhi) {
      uint32_t p = run_end + lane;
      uint32_t s = p < rhi ? (RAW ? reinterpret_cast<const RawJob*>(a.descs)[p].session
                                  : reinterpret_cast<const tlsgpu_record*>(a.descs)[p].session)
                           : sid;
      uint64_t diff = __ballot(p < rhi && s != sid);
      if (diff) { run_end += __builtin_amdgcn_readfirstlane((uint32_t)__builtin_ctzll(diff)); break; }
      run_end = min(rhi, run_end + 64);
    }
    const bool in_range = sid < a.n_sessions;
    const DevSession* __restrict__ S = a.sessions + (in_range ? sid : 0);
    const uint32_t kind = as_const(&S->kind)[0];
    const bool usable = in_range && is_gcm(kind) && (int)as_const(&S->rounds)[0] == ROUNDS;
    if (usable && sid != cur) {
      __syncthreads();
      load_session_tables<kThreads>(a.gcm_tables + sid);
      __syncthreads();
      cur = sid;
    }
    if (usable && RAW) {
      const RecConsts none = {};
      for (uint32_t r = pos + wave; r < run_end; r += kWaves) {
        RecCtx rc;
        parse_raw<SEAL>(reinterpret_cast<const RawJob*>(a.descs)[r], S, rc);
        gcm_record<SEAL, ROUNDS, false>(rc, S, none, a.status + r, lane, laneoff, gl);
      }
    } else if (usable) {
      cu32* rk = as_const(S->rk);
      cu32* rkr = as_const(S->rk_rot);
      const tlsgpu_record* D = reinterpret_cast<const tlsgpu_record*>(a.descs);
      // this wave's records are pos + wave + 16 j; constants for 64 of them at once
      for (uint32_t chunk = pos + wave; chunk < run_end; chunk += kWaves * kWave) {
        uint32_t j0[4];
        lane_j0<SEAL>(D, chunk + kWaves * lane, run_end, S, a.in, j0);
        const RecConsts mine = rec_consts<ROUNDS>(j0, rk, rkr, laneoff);
        for (uint32_t j = 0; j < (uint32_t)kWave; j++) {
          const uint32_t r = chunk + kWaves * j;
          if (r >= run_end) break;
          RecCtx rc;
          int32_t* slot = a.status + r;
          if (!parse_tls<SEAL>(load_desc(D + r), S, a.in, a.out, slot, lane, rc)) continue;
          // parse_tls guarantees n <= TLSGPU_MAX_RECORD, so the counters
          // 2..nb+1 stay below 2^16 and the FAST form applies
          RecConsts rcc;
#pragma unroll
          for (int w = 0; w < 4; w++) rcc.ek0[w] = __builtin_amdgcn_readlane(mine.ek0[w], j);
          rcc.k1a = __builtin_amdgcn_readlane(mine.k1a, j);
          rcc.k1b = __builtin_amdgcn_readlane(mine.k1b, j);
#pragma unroll
          for (int w = 0; w < 4; w++) rcc.k2[w] = __builtin_amdgcn_readlane(mine.k2[w], j);
          gcm_record<SEAL, ROUNDS, true>(rc, S, rcc, slot, lane, laneoff, gl);
        }
      }
    }
    pos = run_end;
  }
}

// Raw EVP jobs and small TLS batches: one job per workgroup (gcm_raw.h).
template <bool SEAL, int ROUNDS, bool TLS = false>
__global__ __launch_bounds__(kThreads, 1) void gcm_raw_kernel(BatchArgs a) {
  fill_aes_lds<kThreads>();  // the job's barrier after its table load covers this
  gcm_raw_job<SEAL, ROUNDS, TLS>(a, blockIdx.x);
}

template <bool SEAL, int ROUNDS, bool TLS = false>
static int launch_raw(const BatchArgs& a, hipStream_t s) {
  hipLaunchKernelGGL((gcm_raw_kernel<SEAL, ROUNDS, TLS>), dim3(a.n), dim3(kThreads), 0, s, a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_gcm_split(const BatchArgs& a, bool seal, int rounds, hipStream_t s) {
  if (a.n == 0) return 0;
  if (rounds == 10) return seal ? launch_raw<true, 10, true>(a, s) : launch_raw<false, 10, true>(a, s);
  return seal ? launch_raw<true, 14, true>(a, s) : launch_raw<false, 14, true>(a, s);
}

template <bool SEAL, bool RAW, int ROUNDS>
static int launch_one(const BatchArgs& a, int groups, hipStream_t s) {
  hipLaunchKernelGGL((gcm_batch_kernel<SEAL, RAW, ROUNDS>), dim3(groups), dim3(kThreads), 0, s, a);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_gcm(const BatchArgs& a, bool seal, bool raw, int rounds, int groups, hipStream_t s) {
  if (a.n == 0) return 0;
  if (raw) {  // one workgroup per job (a.n jobs), blocks split over its waves
    if (rounds == 10) return seal ? launch_raw<true, 10>(a, s) : launch_raw<false, 10>(a, s);
    return seal ? launch_raw<true, 14>(a, s) : launch_raw<false, 14>(a, s);
  }
  if (rounds == 10)
    return seal ? launch_one<true, false, 10>(a, groups, s) : launch_one<false, false, 10>(a, groups, s);
  return seal ? launch_one<true, false, 14>(a, groups, s) : launch_one<false, false, 14>(a, groups, s);
}

}  // namespace tg

