// gcm_raw.h — one EVP_AEAD job (or one record of a small TLS batch) on one
// 1024-thread workgroup: the body of gcm_raw_kernel (gcm_kernels.hip), shared
// with the persistent EVP server kernel (evp_server.hip).
#pragma once
#include "gcm_device.h"

// Phase marks of one job (diagnostic): the doorbell server defines this to
// stamp the realtime clock into LDS from wave 0 (TLSGPU_EVP_DOORBELL_TRACE);
// elsewhere it compiles to nothing.
#ifndef TG_JOB_MARK
#define TG_JOB_MARK(i)
#define TG_JOB_MARK_AT(i, t)
#endif

// Input staging (the doorbell server): idle waves copy a short job's input
// into LDS while the first waves parse, so the block loop reads LDS instead
// of pinned host memory across PCIe.  Elsewhere: nothing.
#ifndef TG_JOB_STAGE
#define TG_JOB_STAGE 0
__device__ __forceinline__ bool tg_stage_ok(const void*) { return false; }
__device__ __forceinline__ void tg_stage_issue(const void*, uint32_t, uint32_t) {}
__device__ __forceinline__ const uint8_t* tg_stage_src() { return nullptr; }
#endif

namespace tg {

// Raw EVP jobs (EVP_AEAD_CTX_seal/open, any nonce / AAD length; TLS = false)
// or the records of a small TLS batch (TLS = true: tlsgpu_record descriptors,
// parse_tls): one job per workgroup and the job's blocks split over the 16
// waves, for latency — a synchronous EVP call waits for its one job, a small
// batch leaves most CUs idle with one wave per record, and a coalesced batch
// runs its jobs side by side on as many CUs.  Wave w takes the 64-aligned block range
// [64 * spw * w, 64 * spw * (w + 1)); its lane chains are the record's chains
// restricted to that range, so their weights are H^(nb + 1 - jlast) as in the
// one-wave form: the last range closes with the lengths block as usual, the
// others raise their chains by (H^64)^q with q extra Horner steps and finish
// with one Shoup multiply.  The 16 partial GHASH values meet in LDS and wave 0
// forms / checks the tag (and zero-fills on failure) after the barrier.
//
// gcm_raw_job runs job r of `a` on the calling 1024-thread workgroup, the
// T-tables already in LDS (fill_aes_lds); it loads the session's GCM tables
// into LDS behind a barrier and returns with nothing of the job left in
// flight except the tag / status of wave 0, so the persistent EVP server
// (evp_server.hip) can start its next job after one more barrier.
// tables_loaded: the session's GCM tables are already in LDS (the server's
// previous job had the same installed key).  Returns whether the LDS holds
// the job's session tables afterwards (false: the session check failed before
// any table was loaded, so the server must not key its table cache on it).
template <bool SEAL, int ROUNDS, bool TLS = false>
__device__ __forceinline__ bool gcm_raw_job(const BatchArgs& a, uint32_t r,
                                            bool tables_loaded = false) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t laneoff = aes_laneoff(lane);
  const GhLane gl = gh_lane(lane);
  const RawJob* J = reinterpret_cast<const RawJob*>(a.descs) + r;
  const tlsgpu_record* D = reinterpret_cast<const tlsgpu_record*>(a.descs) + r;
  const uint32_t sid = __builtin_amdgcn_readfirstlane(TLS ? as_const(D)[6] : J->session);
  const bool in_range = sid < a.n_sessions;
  const DevSession* __restrict__ S = a.sessions + (in_range ? sid : 0);
  const uint32_t kind = as_const(&S->kind)[0];
  if (!(in_range && is_gcm(kind) && (int)as_const(&S->rounds)[0] == ROUNDS)) {
    // raw jobs: no per-batch status memset (run_batch); a job no kernel of
    // this launch set takes (bad or empty session) is publicly invalid here
    if (!TLS && threadIdx.x == 0 && !(in_range && kind >= TLSGPU_AES_128_GCM &&
                                       kind <= TLSGPU_CHACHA20_POLY1305_OLD))
      a.status[r] = TLSGPU_REC_PUBLIC_INVALID;
    return false;
  }
  if (!tables_loaded) load_session_tables<kThreads>(a.gcm_tables + sid);
  __syncthreads();
  TG_JOB_MARK(0);
  const bool staged = !TLS && TG_JOB_STAGE && tg_stage_ok(J);
#ifndef TG_JOB_STAGE_EARLY
  if (staged) tg_stage_issue(J, wave, lane);
#endif
  RecCtx rc;
  if (TLS) {
    // every wave parses (same descriptor): a publicly invalid record returns
    // from all of them before the barrier below
    if (!parse_tls<SEAL>(load_desc(D), S, a.in, a.out, a.status + r, lane, rc)) return true;
  } else {
    parse_raw<SEAL>(*J, S, rc);
  }
  TG_JOB_MARK(1);
  if (staged) {  // the staging waves' LDS writes, before any block is read
    __syncthreads();
    rc.src = tg_stage_src();  // the tag (open) was read from the job's own input by parse_raw
  }
  cu32* rk = as_const(S->rk);
  const uint32_t nb = (rc.n + 15) >> 4;
  const uint32_t nsteps = (nb + kWave - 1) / kWave;
  const uint32_t spw = nsteps == 0 ? 1 : (nsteps + kWaves - 1) / kWaves;  // steps per wave
  const uint32_t nwork = nsteps == 0 ? 1 : (nsteps + spw - 1) / spw;
  uint32_t y[4] = {0, 0, 0, 0};
  uint4* part_y = reinterpret_cast<uint4*>(s_lds + PLAN_OFF);
  // E_K(J0) for the tag, off wave 0's path to the barrier: on the last wave
  // when it has no block range (jobs below 15 steps), beside the blocks; else
  // on the last working wave after its chain (the wave with the fewest
  // Horner steps to raise its range by, so it has the slack).  Into LDS
  // after the 16 partial sums (and the server's selection word).
  uint4* ek_lds = reinterpret_cast<uint4*>(s_lds + PLAN_OFF + 272);
  const bool ek_early = nwork < (uint32_t)kWaves;
  const uint32_t ek_wave = ek_early ? (uint32_t)kWaves - 1 : nwork - 1;
  auto form_ek0 = [&]() {
    uint32_t ek[4] = {rc.j0[0], rc.j0[1], rc.j0[2], rc.j0[3]};
    aes_block<ROUNDS>(ek, rk, as_const(S->rk_rot), laneoff);
    if (lane == 0) *ek_lds = make_uint4(ek[0], ek[1], ek[2], ek[3]);
  };
  if (ek_early && wave == ek_wave) form_ek0();
  if (wave < nwork) {
    const CtrConst cc = ctr_setup(rc.j0, rk, laneoff);
    TG_JOB_MARK(2);
    const RecConsts none = {};
    const uint32_t s0 = wave * spw * kWave;
    uint32_t x[4] = {0, 0, 0, 0};
    if (wave == 0 && rc.aad_len != 0 && lane == 63) {
      x[0] = bswap32(rc.aad_be[0]); x[1] = bswap32(rc.aad_be[1]);
      x[2] = bswap32(rc.aad_be[2]); x[3] = bswap32(rc.aad_be[3]);
    }
    uint32_t xb[4];
    uint32_t e;
    if (wave == nwork - 1) {  // the last range: partial tail, lengths block
      gcm_blocks<SEAL, ROUNDS, false>(rc, S, none, cc, x, s0, lane, laneoff, gl);
      TG_JOB_MARK(3);
      TG_JOB_MARK_AT(7, 64 * (nwork - 1));
      e = gcm_close_chain(rc, x, xb, lane, gl);
    } else {
      RecCtx part = rc;
      const uint32_t e1 = s0 + spw * kWave;  // full blocks only
      part.n = 16u * e1;
      gcm_blocks<SEAL, ROUNDS, false>(part, S, none, cc, x, s0, lane, laneoff, gl);
      TG_JOB_MARK(3);
      e = nb + 1 - (e1 - kWave + lane);
      while (e > (uint32_t)kPowMax) {  // weight (H^64)^q: q more Horner steps
        uint32_t xk[4];
        gl.mul64(x, xk);
        x[0] = xk[0]; x[1] = xk[1]; x[2] = xk[2]; x[3] = xk[3];
        e -= kWave;
      }
      be_from_le(x, xb);
    }
    if (e != 0) gl.shoup(xb, e, y);
    TG_JOB_MARK(4);
    TG_JOB_MARK_AT(8, 64 * (nwork - 1));
    y[0] = wave_xor_total(y[0]);
    y[1] = wave_xor_total(y[1]);
    y[2] = wave_xor_total(y[2]);
    y[3] = wave_xor_total(y[3]);
    if (!ek_early && wave == ek_wave) form_ek0();
  }
  if (lane == 0 && wave < nwork) part_y[wave] = make_uint4(y[0], y[1], y[2], y[3]);
  __syncthreads();
  if (wave != 0) return true;
  TG_JOB_MARK(5);
  uint32_t t[4] = {0, 0, 0, 0};
  if (lane == 0) {
    for (uint32_t w = 0; w < nwork; w++) {
      const uint4 v = part_y[w];
      t[0] ^= v.x; t[1] ^= v.y; t[2] ^= v.z; t[3] ^= v.w;
    }
  }
  const uint4 ekv = *ek_lds;
  const uint32_t ek0[4] = {ekv.x, ekv.y, ekv.z, ekv.w};
  TG_JOB_MARK(6);
  gcm_tag<SEAL>(rc, t, ek0, S, a.status + r, lane);
  return true;
}

}  // namespace tg
