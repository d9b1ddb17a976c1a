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

// Whole-piece balance (round 5, engine.cpp run_batch `pieces`).  A piece is
// a session run inside one count range [g * rpg, (g + 1) * rpg): the unit the
// queue kernel already processes without splitting anything.  piece_scan
// finds each range's pieces and their work (cut_work_of); piece_sort sorts all
// of them by work, largest first, and the queue kernel's workgroup w takes
// pieces m G + (m even ? w : G - 1 - w), m = 0, 1, ... (a snake over the sorted
// list: longest-processing-time order without a heap).  More than
// kPiecesPerRange pieces in a range, or more than kMaxPieces in all, and the
// plan says 0 pieces: the count ranges.
__global__ __launch_bounds__(1024) void piece_scan_kernel(const tlsgpu_record* __restrict__ D,
                                                          uint32_t n, uint32_t rpg,
                                                          uint4* __restrict__ out,
                                                          uint32_t* __restrict__ counts) {
  __shared__ uint64_t tmp[16];
  __shared__ uint32_t s_start[kPiecesPerRange];
  __shared__ uint64_t s_wb[kPiecesPerRange];
  const uint32_t g = blockIdx.x, lo = g * rpg, hi = min(n, lo + rpg);
  uint64_t base = 0;   // work of the range's records before this chunk
  uint32_t pbase = 0;  // pieces that start before this chunk
  for (uint32_t c = lo; c < hi; c += 1024) {  // workgroup-uniform trip count
    const uint32_t i = c + threadIdx.x;
    const bool in = i < hi;
    const uint32_t sess = in ? D[i].session : 0u;
    const bool start = in && (i == lo || D[i - 1].session != sess);
    const uint64_t w = in ? cut_work_of(D[i].len_type) : 0u;
    uint64_t tot, ftot;
    const uint64_t incl = block_scan_incl<1024>(w, tmp, &tot);
    const uint64_t fincl = block_scan_incl<1024>(start ? 1u : 0u, tmp, &ftot);
    if (start) {
      const uint32_t k = pbase + (uint32_t)fincl - 1u;
      if (k < kPiecesPerRange) {
        s_start[k] = i;
        s_wb[k] = base + incl - w;
      }
    }
    base += tot;
    pbase += (uint32_t)ftot;
  }
  __syncthreads();
  if (pbase > kPiecesPerRange) {
    if (threadIdx.x == 0) counts[g] = 0xFFFFFFFFu;
    return;
  }
  const uint32_t k = threadIdx.x;
  if (k < pbase) {
    const uint32_t end = k + 1 < pbase ? s_start[k + 1] : hi;
    const uint64_t wk = (k + 1 < pbase ? s_wb[k + 1] : base) - s_wb[k];
    out[(size_t)g * kPiecesPerRange + k] = make_uint4(s_start[k], end, (uint32_t)wk, (uint32_t)(wk >> 32));
  }
  if (threadIdx.x == 0) counts[g] = pbase;
}

__global__ __launch_bounds__(1024) void piece_sort_kernel(const uint4* __restrict__ in,
                                                          const uint32_t* __restrict__ counts,
                                                          uint32_t G, uint2* __restrict__ sorted,
                                                          uint32_t* __restrict__ n_out) {
  __shared__ uint64_t key[kMaxPieces];
  __shared__ uint32_t val[kMaxPieces];
  __shared__ uint64_t tmp[16];
  __shared__ uint32_t s_bad;
  const uint32_t t = threadIdx.x;
  const uint32_t c = t < G ? counts[t] : 0u;
  if (t == 0) s_bad = G > 1024u ? 1u : 0u;
  __syncthreads();
  if (c == 0xFFFFFFFFu) atomicOr(&s_bad, 1u);
  __syncthreads();
  if (s_bad) {
    if (t == 0) *n_out = 0;
    return;
  }
  uint64_t total;
  const uint32_t off = (uint32_t)(block_scan_incl<1024>(c, tmp, &total) - c);
  const uint32_t P = (uint32_t)total;
  if (P > kMaxPieces || P == 0) {
    if (t == 0) *n_out = 0;
    return;
  }
  for (uint32_t k = 0; k < c; k++) {
    const uint4 v = in[(size_t)t * kPiecesPerRange + k];
    key[off + k] = ((uint64_t)v.w << 32) | v.z;
    val[off + k] = t * kPiecesPerRange + k;
  }
  uint32_t np = 1;
  while (np < P) np <<= 1;
  for (uint32_t i = P + t; i < np; i += 1024) {  // padding sorts last (a piece's work is > 0)
    key[i] = 0;
    val[i] = 0xFFFFFFFFu;
  }
  __syncthreads();
  // bitonic sort, descending
  for (uint32_t size = 2; size <= np; size <<= 1) {
    for (uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
      for (uint32_t i = t; i < np / 2; i += 1024) {
        const uint32_t j = 2 * stride * (i / stride) + (i % stride), q = j + stride;
        const bool desc = (j & size) == 0;
        const uint64_t kj = key[j], kq = key[q];
        if (desc ? kj < kq : kj > kq) {
          key[j] = kq; key[q] = kj;
          const uint32_t vj = val[j];
          val[j] = val[q]; val[q] = vj;
        }
      }
      __syncthreads();
    }
  }
  for (uint32_t i = t; i < P; i += 1024) {
    const uint4 v = in[val[i]];
    sorted[i] = make_uint2(v.x, v.y);
  }
  if (t == 0) *n_out = P;
}

int launch_piece_plan(const BatchArgs& a, int groups, uint8_t* scratch, const uint2** pieces,
                      const uint32_t** n_pieces, hipStream_t s) {
  if (a.n == 0 || groups <= 0) return 0;
  uint4* raw = reinterpret_cast<uint4*>(scratch);
  uint32_t* counts = reinterpret_cast<uint32_t*>(raw + (size_t)groups * kPiecesPerRange);
  uint2* sorted = reinterpret_cast<uint2*>(counts + ((groups + 3) & ~3));
  uint32_t* np = reinterpret_cast<uint32_t*>(sorted + (size_t)groups * kPiecesPerRange);
  hipLaunchKernelGGL(piece_scan_kernel, dim3(groups), dim3(1024), 0, s,
                     reinterpret_cast<const tlsgpu_record*>(a.descs), a.n, a.records_per_group, raw,
                     counts);
  hipLaunchKernelGGL(piece_sort_kernel, dim3(1), dim3(1024), 0, s, raw, counts, (uint32_t)groups,
                     sorted, np);
  *pieces = sorted;
  *n_pieces = np;
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
