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

__device__ __forceinline__ WireWalk wire_walk(const tlsgpu_wire_stream& st, const uint8_t* w,
                                              uint32_t limit) {
  WireWalk r = {0, 0, 0};
  const uint32_t rbuf = st.rbuf_len ? st.rbuf_len : kDefaultRbuf;
  uint32_t pos = 0;
  while (r.records < limit && pos + kHdr <= st.wire_len) {
    const uint8_t* h = w + pos;
    const uint32_t ver = ((uint32_t)h[1] << 8) | h[2];
    const uint32_t len = ((uint32_t)h[3] << 8) | h[4];
    if (!(st.flags & TLSGPU_WIRE_FIRST_PACKET) && ver != st.version) {
      r.alert = kAlertProtocolVersion;  // s3_pkt.c:319-329
      break;
    }
    if ((ver >> 8) != 3) {  // SSL3_VERSION_MAJOR, :331-335 (goto err: no alert)
      r.alert = -1;
      break;
    }
    if (len > rbuf - kHdr) {  // :337-341
      r.alert = kAlertRecordOverflow;
      break;
    }
    if (pos + kHdr + len > st.wire_len) break;  // fragment not complete yet
    if (len > kMaxEncrypted) {  // :376-380
      r.alert = kAlertRecordOverflow;
      break;
    }
    r.records++;
    pos += kHdr + len;
    r.consumed = pos;
  }
  return r;
}

__global__ __launch_bounds__(256) void wire_frame_kernel(const tlsgpu_wire_stream* __restrict__ streams,
                                                         uint32_t n_streams, const uint8_t* wire,
                                                         const DevSession* __restrict__ sessions,
                                                         uint32_t n_sessions, uint32_t max_records,
                                                         tlsgpu_record* __restrict__ recs,
                                                         tlsgpu_wire_result* __restrict__ results,
                                                         uint32_t* total) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n_streams) return;
  const tlsgpu_wire_stream st = streams[s];
  const uint8_t* w = wire + st.wire_off;
  WireWalk walk = wire_walk(st, w, 0xFFFFFFFFu);
  uint32_t first = walk.records ? atomicAdd(total, walk.records) : 0u;
  uint32_t n = walk.records;
  if (first >= max_records) {
    n = 0;
  } else if (first + n > max_records) {
    n = max_records - first;
  }
  if (n != walk.records) {  // truncated at a record boundary: no alert reached
    walk = wire_walk(st, w, n);
    walk.alert = 0;
  }
  // explicit nonce length of the session's AEAD (GCM 8, ChaCha 0); an unknown
  // session still gets descriptors, which the open kernels leave PUBLIC_INVALID
  uint32_t eiv = 0;
  if (st.session < n_sessions) {
    const uint32_t kind = sessions[st.session].kind;
    eiv = (kind == TLSGPU_AES_128_GCM || kind == TLSGPU_AES_256_GCM) ? 8u : 0u;
  }
  uint32_t pos = 0;
  for (uint32_t i = 0; i < n; i++) {
    const uint8_t* h = w + pos;
    const uint32_t len = ((uint32_t)h[3] << 8) | h[4];
    tlsgpu_record d;
    d.in_off = st.wire_off + pos + kHdr;
    d.out_off = d.in_off + eiv;
    d.seq = st.seq + i;
    d.session = st.session;
    d.len_type = ((uint32_t)h[0] << 24) | len;
    recs[first + i] = d;
    pos += kHdr + len;
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
  for (uint32_t i = 0; i < r.records; i++) {
    int32_t* sp = status + r.first + i;
    if (dead) {
      *sp = TLSGPU_REC_SKIPPED;
      continue;
    }
    const int32_t st = *sp;
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
  results[s] = r;
}

int launch_wire_frame(const tlsgpu_wire_stream* streams, uint32_t n_streams, const uint8_t* wire,
                      const DevSession* sessions, uint32_t n_sessions, uint32_t max_records,
                      tlsgpu_record* recs, tlsgpu_wire_result* results, uint32_t* total,
                      hipStream_t s) {
  if (n_streams == 0) return 0;
  hipLaunchKernelGGL(wire_frame_kernel, dim3((n_streams + 255) / 256), dim3(256), 0, s, streams,
                     n_streams, wire, sessions, n_sessions, max_records, recs, results, total);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_wire_finish(uint32_t n_streams, tlsgpu_wire_result* results, int32_t* status,
                       hipStream_t s) {
  if (n_streams == 0) return 0;
  hipLaunchKernelGGL(wire_finish_kernel, dim3((n_streams + 255) / 256), dim3(256), 0, s, n_streams,
                     results, status);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace tg
