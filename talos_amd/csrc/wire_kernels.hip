// wire_kernels.hip — device framing of raw TLS wire records,
// the record-layer half of ssl3_get_record (ssl/s3_pkt.c:279-495) for the AEAD
// suites; the cipher half is the batch open kernels (tls1_enc(s, 0)).
//
//   wire_frame_kernel   one wave per stream: walks the 5-byte headers
//                       (s3_pkt.c:304-341), applies the version / length checks
//                       (:319-341, :376), reserves a contiguous range of record
//                       slots (one atomic per workgroup) and writes the in-place
//                       open descriptors (t1_enc.c:951-955);
//   wire_finish_kernel  one wave per stream: maps the open statuses to the
//                       reference's alerts in record order (:385-390 decryption
//                       failed, :450-462 bad_record_mac, :465-469 record
//                       overflow) and marks the records after the first failure
//                       as not delivered.
// Header walks are a dependent chain of small reads per stream: the parallelism
// is across streams (connections), as a server's batch has it, and each round
// trip covers many headers (wire_walk).
#include "tlsgpu_internal.h"

namespace tg {

constexpr uint32_t kHdr = 5;                         // SSL3_RT_HEADER_LENGTH
constexpr uint32_t kMaxEncrypted = 256 + 64 + 16384;  // SSL3_RT_MAX_ENCRYPTED_LENGTH
constexpr uint32_t kMaxPlain = 16384;                 // SSL3_RT_MAX_PLAIN_LENGTH
constexpr uint32_t kDefaultRbuf = 16384 + 320 + 5 + 3;  // ssl3_setup_read_buffer (s3_both.c:667-675)
constexpr int32_t kAlertBadRecordMac = 20, kAlertDecryptionFailed = 21, kAlertRecordOverflow = 22,
                  kAlertProtocolVersion = 70;

struct WireWalk {
  uint32_t records;   // complete records that pass the header checks
  uint32_t consumed;  // their bytes
  int32_t alert;      // header-level failure after them (0: none / incomplete)
};

struct Hdr {
  uint32_t type, ver, len;
};
// The 5 header bytes from the two dwords that hold them (each holds a header
// byte, so neither reaches past the buffer's last page): 2 loads, not 5.
__device__ __forceinline__ Hdr read_hdr(const uint8_t* h) {
  const uintptr_t a = (uintptr_t)h;
  const uint32_t* q = reinterpret_cast<const uint32_t*>(a & ~(uintptr_t)3);
  const uint32_t sh = (uint32_t)a & 3u;
  const uint32_t q0 = q[0], q1 = q[1];
  const uint32_t lo = __builtin_amdgcn_alignbyte(q1, q0, sh);  // header bytes 0..3
  const uint32_t b4 = (q1 >> (8 * sh)) & 0xFFu;                // header byte 4
  return {lo & 0xFFu, (((lo >> 8) & 0xFFu) << 8) | ((lo >> 16) & 0xFFu), ((lo >> 24) << 8) | b4};
}

// The header walk is a chain of dependent reads (each header gives the next
// one's offset), so one wave walks one stream and covers many headers per
// memory round trip in two ways at once:
//   * a 16 KiB window of the stream at the walk position, loaded by the whole
//     wave (16 coalesced 1 KiB loads) into LDS: the headers of short, varying
//     records (Zipf mixes: ~10 per window) are then LDS reads;
//   * 64 speculative headers, lane k at pos + k * (last record's size): a bulk
//     sender's runs of equal-size records (16 KiB fragments) need one round
//     trip per 64 records.
// A header neither covers starts the next round trip at the walk position.
constexpr uint32_t kWin = 16384;   // LDS window per wave (bytes)
constexpr int kFrameWaves = 4;     // streams (waves) per 256-thread workgroup

// Stream bytes [lo, lo + kWin) into `win`, lo = p rounded down to the
// 16-B-aligned address; bytes outside [0, len) read as zero (never used: the
// walk only reads headers inside the stream).
__device__ __forceinline__ int32_t win_load(const uint8_t* w, uint32_t len, uint32_t p, uint8_t* win,
                                            uint32_t lane) {
  const uint32_t sh = (uint32_t)((uintptr_t)(w + p) & 15u);
  const int32_t lo = (int32_t)p - (int32_t)sh;
  const uint8_t* A = w + p - sh;
  uint4 v[kWin / 1024];
#pragma unroll
  for (int j = 0; j < (int)(kWin / 1024); j++) {
    const int32_t o = lo + (int32_t)(1024 * j + 16 * lane);
    const uint8_t* src = A + 1024 * j + 16 * lane;
    v[j] = make_uint4(0, 0, 0, 0);
    if (o >= 0 && o + 16 <= (int32_t)len) {
      v[j] = gload16(src);
    } else if (o < (int32_t)len && o + 16 > 0) {  // the stream's first / last piece
      uint32_t q[4] = {0, 0, 0, 0};
      for (int b = 0; b < 16; b++)
        if (o + b >= 0 && o + b < (int32_t)len) q[b >> 2] |= (uint32_t)gld<uint8_t>(src)[b] << (8 * (b & 3));
      v[j] = make_uint4(q[0], q[1], q[2], q[3]);
    }
  }
#pragma unroll
  for (int j = 0; j < (int)(kWin / 1024); j++) *reinterpret_cast<uint4*>(win + 1024 * j + 16 * lane) = v[j];
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  return lo;
}

__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

// Visits the complete records of stream `st` that pass the header checks, in
// order, at most `limit`: visit(index, offset, header) for one record at a time
// (wave-uniform arguments), bulk(index, k0, m, base, stride, header) for m
// records accepted at once from the speculative headers — lane k in
// [k0, k0 + m) holds record index + k - k0 at base + k * stride.  Whole wave,
// `win` = the wave's kWin LDS bytes.
template <class Visit, class Bulk>
__device__ __forceinline__ WireWalk wire_walk(const tlsgpu_wire_stream& st, const uint8_t* w,
                                              uint32_t limit, uint8_t* win, uint32_t lane,
                                              Visit&& visit, Bulk&& bulk) {
  WireWalk r = {0, 0, 0};
  const uint32_t rbuf = st.rbuf_len ? st.rbuf_len : kDefaultRbuf;
  const uint32_t len = st.wire_len;
  uint32_t pos = 0, stride = 0;
  int32_t lo = 0;
  bool have_win = false;
  uint32_t cbase = 0, cstride = 0, cnext = 64;  // speculative headers: cnext = next usable lane
  Hdr cand = {0, 0, 0};
  while (r.records < limit && pos + kHdr <= len) {
    Hdr h;
    if (cnext < 64 && pos == cbase + cnext * cstride) {
      // lanes k >= cnext whose header passes every check below and repeats the
      // stride: records k = cnext .. cnext + m - 1 are accepted together
      const uint32_t ck = cbase + lane * cstride;
      const bool ok = lane >= cnext && ck + kHdr <= len &&
                      ((st.flags & TLSGPU_WIRE_FIRST_PACKET) || cand.ver == st.version) &&
                      (cand.ver >> 8) == 3 && cand.len <= rbuf - kHdr &&
                      ck + kHdr + cand.len <= len && cand.len <= kMaxEncrypted &&
                      cand.len + kHdr == cstride && r.records + (lane - cnext) < limit;
      const uint64_t run = ~__ballot(ok) >> cnext;  // bit j: lane cnext + j fails
      const uint32_t m = run ? (uint32_t)__builtin_ctzll(run) : 64u - cnext;
      if (m != 0) {
        bulk(r.records, cnext, m, cbase, cstride, cand);
        r.records += m;
        pos += m * cstride;
        r.consumed = pos;
        stride = cstride;
        cnext += m;
        continue;
      }
      h.type = uni(__builtin_amdgcn_readlane(cand.type, cnext));
      h.ver = uni(__builtin_amdgcn_readlane(cand.ver, cnext));
      h.len = uni(__builtin_amdgcn_readlane(cand.len, cnext));
      cnext++;
    } else if (have_win && (int32_t)pos >= lo && (int32_t)(pos + kHdr) <= lo + (int32_t)kWin) {
      const uint8_t* q = win + ((int32_t)pos - lo);
      h.type = q[0];
      h.ver = ((uint32_t)q[1] << 8) | q[2];
      h.len = ((uint32_t)q[3] << 8) | q[4];
      h.type = uni(h.type); h.ver = uni(h.ver); h.len = uni(h.len);
      cnext = 64;
    } else {  // one round trip: the window at pos and 64 headers at pos + k * stride
      cbase = pos;
      cstride = stride;
      cnext = stride ? 0u : 64u;
      if (stride) cand = read_hdr(w + min(pos + lane * stride, len - kHdr));
      lo = win_load(w, len, pos, win, lane);
      have_win = true;
      continue;
    }
    if (!(st.flags & TLSGPU_WIRE_FIRST_PACKET) && h.ver != st.version) {
      r.alert = kAlertProtocolVersion;  // s3_pkt.c:319-329
      break;
    }
    if ((h.ver >> 8) != 3) {  // SSL3_VERSION_MAJOR, :331-335 (goto err: no alert)
      r.alert = -1;
      break;
    }
    if (h.len > rbuf - kHdr) {  // :337-341
      r.alert = kAlertRecordOverflow;
      break;
    }
    if (pos + kHdr + h.len > len) break;  // fragment not complete yet
    if (h.len > kMaxEncrypted) {  // :376-380
      r.alert = kAlertRecordOverflow;
      break;
    }
    visit(r.records, pos, h);
    r.records++;
    pos += kHdr + h.len;
    r.consumed = pos;
    stride = kHdr + h.len;
  }
  return r;
}

// One wave per stream (kFrameWaves streams per workgroup): walk, reserve the
// stream's descriptor range (one atomic per workgroup), then write the in-place
// open descriptors from the walk's LDS list of (offset, type|length) — or, for
// a stream of more than kList records, walk again (the window loads now hit
// the cache) writing them.
constexpr uint32_t kList = 1024;  // records per stream remembered by the first walk
__global__ __launch_bounds__(64 * kFrameWaves) void wire_frame_kernel(
    const tlsgpu_wire_stream* __restrict__ streams, uint32_t n_streams, const uint8_t* wire,
    const DevSession* __restrict__ sessions, uint32_t n_sessions, uint32_t max_records,
    tlsgpu_record* __restrict__ recs, tlsgpu_wire_result* __restrict__ results, uint32_t* total) {
  __shared__ __attribute__((aligned(16))) uint8_t wins[kFrameWaves][kWin];
  __shared__ uint2 lists[kFrameWaves][kList];  // {offset, type << 24 | length}
  __shared__ uint32_t cnt[kFrameWaves], base_slot;
  const uint32_t lane = threadIdx.x & 63, wave = uni(threadIdx.x >> 6);
  const uint32_t s = blockIdx.x * kFrameWaves + wave;
  const bool active = s < n_streams;
  uint2* list = lists[wave];
  tlsgpu_wire_stream st = {};
  WireWalk walk = {};
  if (active) {
    st = streams[s];
    walk = wire_walk(st, wire + st.wire_off, 0xFFFFFFFFu, wins[wave], lane,
                     [&](uint32_t i, uint32_t pos, const Hdr& h) {
                       if (lane == 0 && i < kList) list[i] = make_uint2(pos, (h.type << 24) | h.len);
                     },
                     [&](uint32_t i, uint32_t k0, uint32_t m, uint32_t base, uint32_t stride,
                         const Hdr& h) {
                       const uint32_t j = i + lane - k0;
                       if (lane >= k0 && lane < k0 + m && j < kList)
                         list[j] = make_uint2(base + lane * stride, (h.type << 24) | h.len);
                     });
  }
  if (lane == 0) cnt[wave] = active ? walk.records : 0u;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t sum = 0;
    for (int k = 0; k < kFrameWaves; k++) sum += cnt[k];
    base_slot = sum ? atomicAdd(total, sum) : 0u;
  }
  __syncthreads();
  if (!active) return;
  uint32_t slot0 = base_slot;
  for (uint32_t k = 0; k < wave; k++) slot0 += cnt[k];
  slot0 = uni(slot0);
  const uint32_t first = walk.records ? slot0 : 0u;
  const uint8_t* w = wire + st.wire_off;
  uint32_t n = walk.records;
  if (first >= max_records) {
    n = 0;
  } else if (first + n > max_records) {
    n = max_records - first;
  }
  // explicit nonce length of the session's AEAD (GCM 8, ChaCha 0); an unknown
  // session still gets descriptors, which the open kernels leave PUBLIC_INVALID
  uint32_t eiv = 0;
  if (st.session < n_sessions) {
    const uint32_t kind = sessions[st.session].kind;
    eiv = (kind == TLSGPU_AES_128_GCM || kind == TLSGPU_AES_256_GCM) ? 8u : 0u;
  }
  if (walk.records <= kList) {  // descriptors from the list, 64 per wave store
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    for (uint32_t i0 = 0; i0 < n; i0 += 64) {
      const uint32_t i = i0 + lane;
      if (i < n) {
        const uint2 e = list[i];
        tlsgpu_record d;
        d.in_off = st.wire_off + e.x + kHdr;
        d.out_off = d.in_off + eiv;
        d.seq = st.seq + i;
        d.session = st.session;
        d.len_type = e.y;
        recs[first + i] = d;
      }
    }
    if (n != walk.records) {  // truncated at a record boundary: no alert reached
      const uint2 e = n ? list[n - 1] : make_uint2(0, 0);
      walk.records = n;
      walk.consumed = n ? e.x + kHdr + (e.y & 0xFFFFFFu) : 0u;
      walk.alert = 0;
    }
  } else {
    // descriptors gathered 64 at a time in the lanes, stored by the whole wave
    tlsgpu_record d = {};
    uint32_t held = 0;
    auto flush = [&](uint32_t upto) {
      if (lane < held) recs[first + upto - held + lane] = d;
      held = 0;
    };
    const WireWalk w2 = wire_walk(st, w, n, wins[wave], lane, [&](uint32_t i, uint32_t pos, const Hdr& h) {
      if (lane == held) {
        d.in_off = st.wire_off + pos + kHdr;
        d.out_off = d.in_off + eiv;
        d.seq = st.seq + i;
        d.session = st.session;
        d.len_type = (h.type << 24) | h.len;
      }
      if (++held == 64) flush(i + 1);
    }, [&](uint32_t i, uint32_t k0, uint32_t m, uint32_t base, uint32_t stride, const Hdr& h) {
      flush(i);  // the held records end at index i
      if (lane >= k0 && lane < k0 + m) {
        tlsgpu_record e;
        e.in_off = st.wire_off + base + lane * stride + kHdr;
        e.out_off = e.in_off + eiv;
        e.seq = st.seq + i + (lane - k0);
        e.session = st.session;
        e.len_type = (h.type << 24) | h.len;
        recs[first + i + (lane - k0)] = e;
      }
    });
    flush(w2.records);
    if (n != walk.records) {  // truncated at a record boundary: no alert reached
      walk = w2;
      walk.alert = 0;
    }
  }
  if (lane == 0) {
    tlsgpu_wire_result r;
    r.first = n ? first : 0u;
    r.records = n;
    r.delivered = n;
    r.consumed = walk.consumed;
    r.alert = walk.alert;
    r.alert_record = n;
    r.reserved[0] = r.reserved[1] = 0;
    results[s] = r;
  }
}

// One wave per stream: the statuses of 64 records per load, the first failing
// record found with a ballot (s3_pkt.c alert order: the first failure wins,
// later records are not delivered).
__global__ __launch_bounds__(256) void wire_finish_kernel(uint32_t n_streams,
                                                          tlsgpu_wire_result* __restrict__ results,
                                                          int32_t* __restrict__ status) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t s = blockIdx.x * 4 + uni(threadIdx.x >> 6);
  if (s >= n_streams) return;
  tlsgpu_wire_result r = results[s];
  bool dead = false;
  for (uint32_t i0 = 0; i0 < r.records; i0 += 64) {
    const uint32_t i = i0 + lane;
    const bool in = i < r.records;
    int32_t* sp = status + r.first + i;
    if (dead) {
      if (in) *sp = TLSGPU_REC_SKIPPED;
      continue;
    }
    const int32_t st = in ? *sp : 0;
    const int32_t alert = !in ? 0
                          : st == TLSGPU_REC_BAD_MAC        ? kAlertBadRecordMac
                          : st == TLSGPU_REC_PUBLIC_INVALID ? kAlertDecryptionFailed
                          : st > (int32_t)kMaxPlain         ? kAlertRecordOverflow
                                                            : 0;
    const uint64_t bad = __ballot(alert != 0);
    if (!bad) continue;
    const uint32_t fl = (uint32_t)__builtin_ctzll(bad);  // first failing lane
    if (lane == fl && alert == kAlertRecordOverflow) *sp = TLSGPU_REC_OVERFLOW;
    if (in && lane > fl) *sp = TLSGPU_REC_SKIPPED;
    dead = true;
    r.alert = __shfl(alert, (int)fl);
    r.alert_record = i0 + fl;
    r.delivered = i0 + fl;
  }
  if (lane == 0) results[s] = r;
}

// Reserve k consecutive descriptor slots per lane with ONE atomic per wave on
// `total` (an inclusive scan over the wave, lane 63 adds the wave's sum):
// same-address atomics from every lane serialise at one L2 channel.  All 64
// lanes must be active (inactive streams pass k = 0).
__device__ __forceinline__ uint32_t wave_reserve(uint32_t* total, uint32_t k) {
  const uint32_t lane = threadIdx.x & 63;
  uint32_t incl = k;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(incl, d);
    if (lane >= (uint32_t)d) incl += y;
  }
  const uint32_t sum = __shfl(incl, 63);
  uint32_t base = 0;
  if (lane == 63 && sum) base = atomicAdd(total, sum);
  base = __shfl(base, 63);
  return base + incl - k;
}

// Write-side framing (ssl3_write_bytes / do_ssl3_write, s3_pkt.c:501-762), one
// lane per stream: reserves the stream's record slots, writes each record's
// 5-byte header and its seal descriptor (fragment at header + 5; the seal
// kernels write explicit nonce || ciphertext || tag there).
__global__ __launch_bounds__(256) void wire_seal_frame_kernel(
    const tlsgpu_write_stream* __restrict__ streams, uint32_t n_streams,
    const DevSession* __restrict__ sessions, uint32_t n_sessions, uint8_t* __restrict__ wire,
    uint64_t wire_bytes, uint32_t max_records, tlsgpu_record* __restrict__ recs,
    tlsgpu_write_result* __restrict__ results, uint32_t* __restrict__ total) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const bool active = i < n_streams;
  tlsgpu_write_stream st = {};
  if (active) st = streams[i];
  tlsgpu_write_result res = {};
  res.next_seq = st.seq;
  const bool ok = active && st.session < n_sessions && sessions[st.session].kind != 0;
  const uint32_t frag = st.max_fragment == 0 || st.max_fragment > kMaxPlain ? kMaxPlain
                                                                           : st.max_fragment;
  // record count in 64 bits (data_len near 2^32 must not wrap; same arithmetic
  // as tlsgpu_seal_wire_size), then at most max_records slots per stream
  const uint64_t nrec64 = ok ? ((uint64_t)st.data_len + frag - 1) / frag : 0;  // len 0: nothing (:593-594)
  uint32_t nrec = (uint32_t)min(nrec64, (uint64_t)max_records);
  const uint32_t slot0 = wave_reserve(total, nrec);
  if (!active) return;
  const uint32_t first = nrec ? slot0 : 0u;
  if (first >= max_records) nrec = 0;
  else if ((uint64_t)first + nrec > max_records) nrec = max_records - first;
  res.first = first;
  if (nrec) {
    const DevSession& S = sessions[st.session];
    const uint32_t over = (S.nonce_in_record ? 8u : 0u) + S.tag_len;  // eivlen + tag
    uint64_t pos = st.wire_off;
    for (uint32_t k = 0; k < nrec; k++) {
      const uint32_t len = min(frag, st.data_len - k * frag);
      const uint32_t L = len + over;  // the length field (s3_pkt.c:733)
      if (pos <= wire_bytes && (uint64_t)kHdr + L <= wire_bytes - pos) {  // no wrap
        uint8_t* h = wire + pos;
        h[0] = st.type;
        h[1] = (uint8_t)(st.version >> 8);
        h[2] = (uint8_t)st.version;
        h[3] = (uint8_t)(L >> 8);
        h[4] = (uint8_t)L;
      }
      tlsgpu_record d;
      d.in_off = st.data_off + (uint64_t)k * frag;
      d.out_off = pos + kHdr;
      d.seq = st.seq + k;
      d.session = st.session;
      d.len_type = TLSGPU_LEN_TYPE(len, st.type);
      recs[first + k] = d;
      pos += kHdr + L;
    }
    res.records = nrec;
    res.wire_len = pos - st.wire_off;
    res.next_seq = st.seq + nrec;
  }
  results[i] = res;
}

int launch_wire_seal_frame(const tlsgpu_write_stream* streams, uint32_t n_streams,
                           const DevSession* sessions, uint32_t n_sessions, uint8_t* wire,
                           uint64_t wire_bytes, uint32_t max_records, tlsgpu_record* recs,
                           tlsgpu_write_result* results, uint32_t* total, hipStream_t s) {
  if (n_streams == 0) return 0;
  hipLaunchKernelGGL(wire_seal_frame_kernel, dim3((n_streams + 255) / 256), dim3(256), 0, s, streams,
                     n_streams, sessions, n_sessions, wire, wire_bytes, max_records, recs, results,
                     total);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_wire_frame(const tlsgpu_wire_stream* streams, uint32_t n_streams, const uint8_t* wire,
                      const DevSession* sessions, uint32_t n_sessions, uint32_t max_records,
                      tlsgpu_record* recs, tlsgpu_wire_result* results, uint32_t* total,
                      hipStream_t s) {
  if (n_streams == 0) return 0;
  hipLaunchKernelGGL(wire_frame_kernel, dim3((n_streams + kFrameWaves - 1) / kFrameWaves),
                     dim3(64 * kFrameWaves), 0, s, streams,
                     n_streams, wire, sessions, n_sessions, max_records, recs, results, total);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_wire_finish(uint32_t n_streams, tlsgpu_wire_result* results, int32_t* status,
                       hipStream_t s) {
  if (n_streams == 0) return 0;
  hipLaunchKernelGGL(wire_finish_kernel, dim3((n_streams + 3) / 4), dim3(256), 0, s, n_streams,
                     results, status);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace tg
