// wire_kernels.hip — device framing of raw TLS wire records,
// the record-layer half of ssl3_get_record (ssl/s3_pkt.c:279-495) for the AEAD
// suites; the cipher half is the batch open kernels (tls1_enc(s, 0)).
//
//   wire_frame_kernel   one lane per stream: walks the 5-byte headers
//                       (s3_pkt.c:304-341), applies the version / length checks
//                       (:319-341, :376), reserves a contiguous range of record
//                       slots (one atomic per stream) and writes the in-place
//                       open descriptors (t1_enc.c:951-955);
//   wire_finish_kernel  one lane per stream: maps the open statuses to the
//                       reference's alerts in record order (:385-390 decryption
//                       failed, :450-462 bad_record_mac, :465-469 record
//                       overflow) and marks the records after the first failure
//                       as not delivered.
// Header walks are a dependent chain of small reads per stream, so the
// parallelism is across streams (connections), as a server's batch has it.
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
// one's offset): one memory round trip per record.  It covers up to kSpec
// headers per round trip by speculating that the next records have the last
// record's length (a bulk sender's stream is runs of equal-size records): the
// speculative headers are loaded together, and header k is used only if the
// real walk lands exactly on it; a misprediction restarts from the real offset.
constexpr int kSpec = 8;

// Visits the complete records of stream `st` that pass the header checks, in
// order, at most `limit`, calling visit(index, offset, header) for each.
template <class Visit>
__device__ __forceinline__ WireWalk wire_walk(const tlsgpu_wire_stream& st, const uint8_t* w,
                                              uint32_t limit, Visit&& visit) {
  WireWalk r = {0, 0, 0};
  const uint32_t rbuf = st.rbuf_len ? st.rbuf_len : kDefaultRbuf;
  uint32_t pos = 0, stride = 0;
  bool stop = false;
  while (!stop && r.records < limit && pos + kHdr <= st.wire_len) {
    const uint32_t base = pos, sb = stride;
    Hdr hs[kSpec];
#pragma unroll
    for (int k = 0; k < kSpec; k++) {  // unconditional loads (clamped into the stream):
      // a header past the stream end is never used (the walk stops first)
      const uint32_t p = min(base + (uint32_t)k * sb, st.wire_len - kHdr);
      hs[k] = read_hdr(w + p);
    }
#pragma unroll
    for (int k = 0; k < kSpec; k++) {
      if (k > 0 && (sb == 0 || pos != base + (uint32_t)k * sb)) break;  // mispredicted
      if (r.records >= limit || pos + kHdr > st.wire_len) {
        stop = true;
        break;
      }
      const Hdr h = hs[k];
      if (!(st.flags & TLSGPU_WIRE_FIRST_PACKET) && h.ver != st.version) {
        r.alert = kAlertProtocolVersion;  // s3_pkt.c:319-329
        stop = true;
        break;
      }
      if ((h.ver >> 8) != 3) {  // SSL3_VERSION_MAJOR, :331-335 (goto err: no alert)
        r.alert = -1;
        stop = true;
        break;
      }
      if (h.len > rbuf - kHdr) {  // :337-341
        r.alert = kAlertRecordOverflow;
        stop = true;
        break;
      }
      if (pos + kHdr + h.len > st.wire_len) {  // fragment not complete yet
        stop = true;
        break;
      }
      if (h.len > kMaxEncrypted) {  // :376-380
        r.alert = kAlertRecordOverflow;
        stop = true;
        break;
      }
      visit(r.records, pos, h);
      r.records++;
      pos += kHdr + h.len;
      r.consumed = pos;
      stride = kHdr + h.len;
    }
  }
  return r;
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

__global__ __launch_bounds__(256) void wire_frame_kernel(const tlsgpu_wire_stream* __restrict__ streams,
                                                         uint32_t n_streams, const uint8_t* wire,
                                                         const DevSession* __restrict__ sessions,
                                                         uint32_t n_sessions, uint32_t max_records,
                                                         tlsgpu_record* __restrict__ recs,
                                                         tlsgpu_wire_result* __restrict__ results,
                                                         uint32_t* total) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  const bool active = s < n_streams;
  tlsgpu_wire_stream st = {};
  WireWalk walk = {};
  if (active) {
    st = streams[s];
    walk = wire_walk(st, wire + st.wire_off, 0xFFFFFFFFu, [](uint32_t, uint32_t, const Hdr&) {});
  }
  const uint32_t slot0 = wave_reserve(total, active ? walk.records : 0u);
  if (!active) return;
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
  // second walk (headers now cache-resident) writes the in-place descriptors
  const WireWalk w2 = wire_walk(st, w, n, [&](uint32_t i, uint32_t pos, const Hdr& h) {
    tlsgpu_record d;
    d.in_off = st.wire_off + pos + kHdr;
    d.out_off = d.in_off + eiv;
    d.seq = st.seq + i;
    d.session = st.session;
    d.len_type = (h.type << 24) | h.len;
    recs[first + i] = d;
  });
  if (n != walk.records) {  // truncated at a record boundary: no alert reached
    walk = w2;
    walk.alert = 0;
  }
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

__global__ __launch_bounds__(256) void wire_finish_kernel(uint32_t n_streams,
                                                          tlsgpu_wire_result* __restrict__ results,
                                                          int32_t* __restrict__ status) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n_streams) return;
  tlsgpu_wire_result r = results[s];
  bool dead = false;
  // statuses in groups of 8 loaded together (independent loads, one round trip)
  for (uint32_t i0 = 0; i0 < r.records; i0 += 8) {
    int32_t sv[8];
#pragma unroll
    for (int k = 0; k < 8; k++) sv[k] = i0 + k < r.records ? status[r.first + i0 + k] : 0;
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const uint32_t i = i0 + k;
      if (i >= r.records) break;
      int32_t* sp = status + r.first + i;
      if (dead) {
        *sp = TLSGPU_REC_SKIPPED;
        continue;
      }
      const int32_t st = sv[k];
      int32_t alert = 0;
      if (st == TLSGPU_REC_BAD_MAC) {
        alert = kAlertBadRecordMac;
      } else if (st == TLSGPU_REC_PUBLIC_INVALID) {
        alert = kAlertDecryptionFailed;
      } else if (st > (int32_t)kMaxPlain) {
        alert = kAlertRecordOverflow;
        *sp = TLSGPU_REC_OVERFLOW;
      }
      if (alert) {
        dead = true;
        r.alert = alert;
        r.alert_record = i;
        r.delivered = i;
      }
    }
  }
  results[s] = r;
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
  uint32_t nrec = ok ? (st.data_len + frag - 1) / frag : 0;  // len 0: nothing (:593-594)
  const uint32_t slot0 = wave_reserve(total, nrec);
  if (!active) return;
  const uint32_t first = nrec ? slot0 : 0u;
  if (first >= max_records) nrec = 0;
  else if (first + nrec > max_records) nrec = max_records - first;
  res.first = first;
  if (nrec) {
    const DevSession& S = sessions[st.session];
    const uint32_t over = (S.nonce_in_record ? 8u : 0u) + S.tag_len;  // eivlen + tag
    uint64_t pos = st.wire_off;
    for (uint32_t k = 0; k < nrec; k++) {
      const uint32_t len = min(frag, st.data_len - k * frag);
      const uint32_t L = len + over;  // the length field (s3_pkt.c:733)
      if (pos + kHdr + L <= wire_bytes) {
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
  // 64-lane groups: the scattered header loads of one wave per CU, not four
  hipLaunchKernelGGL(wire_frame_kernel, dim3((n_streams + 63) / 64), dim3(64), 0, s, streams,
                     n_streams, wire, sessions, n_sessions, max_records, recs, results, total);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_wire_finish(uint32_t n_streams, tlsgpu_wire_result* results, int32_t* status,
                       hipStream_t s) {
  if (n_streams == 0) return 0;
  hipLaunchKernelGGL(wire_finish_kernel, dim3((n_streams + 63) / 64), dim3(64), 0, s, n_streams,
                     results, status);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace tg
