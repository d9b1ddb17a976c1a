/*
 * tlsgpu.h — MI355X-native TLS 1.2 record bulk-cipher engine: batch C ABI.
 *
 * This is the GPU extension that sits beside the drop-in EVP_AEAD ABI
 * (include/tlsgpu_evp.h).  It has no reference counterpart; it batches the
 * per-record work that LibreSSL 2.4.1 does one record at a time in
 *   tls1_enc() AEAD branch            ssl/t1_enc.c:832-975
 *     -> EVP_AEAD_CTX_seal / _open    crypto/evp/evp_aead.c:89-144
 *       -> aead_aes_gcm_seal / _open  crypto/evp/e_aes.c:1424-1510
 *       -> aead_chacha20_poly1305_*   crypto/evp/e_chacha20poly1305.c:124-286
 * and moves the per-direction key install of
 *   tls1_change_cipher_state_aead()   ssl/t1_enc.c:444-495
 * into a device session table.
 *
 * All pointers named d_* are device (HBM) pointers; the API never touches
 * torch or any framework type.  Streams are hipStream_t passed as void*.
 * Every function returns TLSGPU_OK (0) or a negative TLSGPU_E* code.
 */
#ifndef TLSGPU_H
#define TLSGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TLSGPU_ABI_VERSION 2	/* 2: batch calls take buffer sizes */

/* AEAD kinds (crypto/evp/e_aes.c:1512-1546, e_chacha20poly1305.c:288-322). */
enum tlsgpu_aead {
	TLSGPU_AES_128_GCM = 1,
	TLSGPU_AES_256_GCM = 2,
	TLSGPU_CHACHA20_POLY1305 = 3,	/* RFC 7539/7905, 12-byte nonce */
	TLSGPU_CHACHA20_POLY1305_OLD = 4	/* draft-agl, 8-byte nonce */
};

/* Return codes. */
#define TLSGPU_OK 0
#define TLSGPU_EINVAL (-1)
#define TLSGPU_ENOMEM (-2)
#define TLSGPU_EHIP (-3)	/* HIP runtime error (no GPU, launch failure) */
#define TLSGPU_ERANGE (-4)	/* session id / size out of range */
#define TLSGPU_ETIMEOUT (-5)	/* a bounded wait expired (tlsgpu_evp_shutdown) */

/* Per-record status written by the batch calls (int32 per record).
 *   >= 0  success: plaintext length (open) or record body length (seal)
 *   TLSGPU_REC_BAD_MAC         tls1_enc returns -1 -> bad_record_mac alert
 *                              (s3_pkt.c:450-462); the plaintext region
 *                              [out, out+len) is zero-filled as
 *                              EVP_AEAD_CTX_open does (evp_aead.c:137-143)
 *   TLSGPU_REC_PUBLIC_INVALID  tls1_enc returns 0: record shorter than the
 *                              explicit nonce or the tag (t1_enc.c:930,958)
 */
#define TLSGPU_REC_BAD_MAC (-1)
#define TLSGPU_REC_PUBLIC_INVALID (-2)
/* tlsgpu_open_wire only: an earlier record of the same stream failed, so
 * ssl3_get_record would never have returned this one (not delivered). */
#define TLSGPU_REC_SKIPPED (-3)
/* tlsgpu_open_wire only: plaintext longer than SSL3_RT_MAX_PLAIN_LENGTH
 * (s3_pkt.c:465-469) -> record_overflow alert, not delivered. */
#define TLSGPU_REC_OVERFLOW (-4)
/* tlsgpu_open_batch / _seal_batch: the record's input span (in_off, length) or
 * output span (out_off, plaintext / fragment length) leaves d_in / d_out as
 * sized by the caller; nothing of the record was read or written. */
#define TLSGPU_REC_OUT_OF_BOUNDS (-5)

/* Largest plaintext per record the batch kernels accept: 65534 AES blocks, so
 * GCM counters 2..nb+1 stay below 2^16 (TLS records are <= 16 KiB + 2 KiB,
 * ssl3.h:259-280).  Longer records get TLSGPU_REC_PUBLIC_INVALID. */
#define TLSGPU_MAX_RECORD (65534u * 16u)

/* One TLS record, 32 bytes, device-resident array.
 * open: in_off -> record fragment after the 5-byte header
 *       (GCM: explicit nonce(8) || ct || tag(16); ChaCha: ct || tag(16)),
 *       length = fragment length; plaintext written at out_off
 *       (the TLS layer passes out = fragment + 8 for GCM, t1_enc.c:951-955).
 * seal: in_off -> plaintext, length = plaintext length; the fragment
 *       (explicit nonce || ct || tag) is written at out_off (t1_enc.c:898-914).
 * seq is the record's 64-bit sequence number (read_sequence/write_sequence
 * before tls1_record_sequence_increment, t1_enc.c:258-266,841-847). */
typedef struct tlsgpu_record {
	uint64_t in_off;
	uint64_t out_off;
	uint64_t seq;
	uint32_t session;
	uint32_t len_type;	/* bits 0-23: length; bits 24-31: content type */
} tlsgpu_record;

#define TLSGPU_LEN_TYPE(len, type) (((uint32_t)(type) << 24) | ((uint32_t)(len) & 0xFFFFFFu))

/* Session parameters as installed at ChangeCipherSpec
 * (t1_enc.c:444-495; nonce lengths from s3_lib.c cipher table). */
typedef struct tlsgpu_session_params {
	int32_t aead;			/* enum tlsgpu_aead */
	uint32_t key_len;		/* 16 or 32 */
	uint8_t key[32];
	uint32_t fixed_iv_len;		/* 4 (GCM), 12 (ChaCha), 0 (ChaCha old) */
	uint8_t fixed_iv[12];
	uint32_t tag_len;		/* 0 = default 16 (EVP_AEAD_DEFAULT_TAG_LENGTH) */
	uint16_t version;		/* s->version, e.g. 0x0303 */
	uint16_t reserved;
} tlsgpu_session_params;

typedef struct tlsgpu_engine tlsgpu_engine;
typedef struct tlsgpu_sessions tlsgpu_sessions;

/* Number of visible GPUs (0 when no device / no driver). */
int tlsgpu_device_count(int *count);

/* Engine = one GPU + one HIP stream + scratch pools. */
int tlsgpu_engine_create(int device, tlsgpu_engine **out);
void tlsgpu_engine_destroy(tlsgpu_engine *e);
/* The engine's stream (hipStream_t) for callers that order their own work. */
void *tlsgpu_engine_stream(tlsgpu_engine *e);
int tlsgpu_engine_sync(tlsgpu_engine *e);
/* Compute units of the engine's device (256 on MI355X). */
int tlsgpu_engine_num_cus(tlsgpu_engine *e);

/* Device session table with room for `capacity` sessions. */
int tlsgpu_sessions_create(tlsgpu_engine *e, uint32_t capacity, tlsgpu_sessions **out);
void tlsgpu_sessions_destroy(tlsgpu_sessions *t);
/* Install n sessions (host params) at ids first..first+n-1.  Key schedule,
 * H = E_K(0^128) and the GHASH power tables are derived on the device. */
int tlsgpu_sessions_install(tlsgpu_sessions *t, uint32_t first, uint32_t n,
    const tlsgpu_session_params *params);

/* Batch record decrypt / encrypt (device-resident).  Any record order is
 * correct; grouping each session's records together is fastest.  in_bytes /
 * out_bytes are the sizes of d_in / d_out: records whose spans leave them get
 * TLSGPU_REC_OUT_OF_BOUNDS and are not touched.  d_status: int32 per record.
 * d_in == d_out is allowed (in-place open at out_off = in_off + 8 for GCM,
 * t1_enc.c:951-955).  Asynchronous on `stream` (NULL = engine stream). */
int tlsgpu_open_batch(tlsgpu_sessions *t, const tlsgpu_record *d_recs, uint32_t n,
    const uint8_t *d_in, size_t in_bytes, uint8_t *d_out, size_t out_bytes, int32_t *d_status,
    void *stream);
int tlsgpu_seal_batch(tlsgpu_sessions *t, const tlsgpu_record *d_recs, uint32_t n,
    const uint8_t *d_in, size_t in_bytes, uint8_t *d_out, size_t out_bytes, int32_t *d_status,
    void *stream);

/* Batch-shape hints for the AES-GCM batch calls of this session table
 * (performance only: results never depend on them, any batch stays correct).
 * The default kernel selection happens on the device, so every GCM batch
 * dispatches the long-record kernel, its short-record-pack variant and the
 * per-wave-session kernel, and the two not selected exit at once (~5 us each).
 * A caller that knows its batches rules them out:
 *   TLSGPU_HINT_NO_SHORT_RECORDS  no GCM record of <= 62 blocks (open: length
 *                                 <= 1,016 B with the 8-B explicit nonce and a
 *                                 16-B tag): the pack variant is not launched;
 *   TLSGPU_HINT_SESSION_RUNS      records come in session runs of >= 12
 *                                 records on average: the per-wave-session
 *                                 kernel is not launched.
 * A wrong hint costs speed only (short records then take the long-record
 * path, short runs the run-at-a-time queue).  tlsgpu_open_host /
 * tlsgpu_seal_host derive the hints from the host descriptors themselves. */
#define TLSGPU_HINT_NO_SHORT_RECORDS 1u
#define TLSGPU_HINT_SESSION_RUNS 2u
int tlsgpu_sessions_hint(tlsgpu_sessions *t, unsigned hints);

/* ---------------------------------------------------------------------------
 * Host-resident batch open: records that start and end in
 * host memory, as socket buffers do.  Replaces, for a batch of connections,
 * ssl3_read_n's BIO_read into rbuf (ssl/s3_pkt.c:134-267), tls1_enc(s, 0)
 * and the copy of the plaintext to the application buffer (s3_pkt.c:957).
 *
 * h_recs / h_in / h_out / h_status are HOST pointers (pinned memory from
 * tlsgpu_host_alloc for full PCIe rate; pageable memory works, slower).
 * Descriptor offsets are relative to h_in / h_out exactly as for
 * tlsgpu_open_batch; h_out == h_in opens in place.  The engine mirrors the
 * buffers in HBM and pipelines the batch in chunks (H2D of chunk k+1 and D2H
 * of chunk k-1 on their own streams overlap the kernels of chunk k) when
 * the records' in_off and out_off ascend with the record index; otherwise it
 * runs the batch as one chunk.  Synchronous: returns when h_out and h_status
 * are final, and also on every error — no copy into or out of the caller's
 * buffers is still running once it has returned.  Bytes of h_out between the
 * records' plaintext spans (from the first span to the last, or all of
 * out_bytes when the layout does not ascend) come back as zeros out of place;
 * in place, the headers, explicit nonces and tags are written back unchanged.
 * Bytes outside that range are not touched. */
int tlsgpu_open_host(tlsgpu_sessions *t, const tlsgpu_record *h_recs, uint32_t n,
    const uint8_t *h_in, size_t in_bytes, uint8_t *h_out, size_t out_bytes, int32_t *h_status);
/* The write direction: plaintext records in host memory (h_in) sealed into
 * host fragments (h_out, explicit nonce || ciphertext || tag at out_off;
 * headers are the caller's, or use tlsgpu_seal_wire).  Not in place. */
int tlsgpu_seal_host(tlsgpu_sessions *t, const tlsgpu_record *h_recs, uint32_t n,
    const uint8_t *h_in, size_t in_bytes, uint8_t *h_out, size_t out_bytes, int32_t *h_status);

/* TaLoS plaintext-processing hooks.  libtlsgpu implements TaLoS's own
 * interface (include/tlsgpu_talos.h: tls_processing_register_*_cb with the
 * reference signatures, tls_processing_interface.h:23-27), so a TaLoS module
 * registers against the engine unchanged.  The registered read / write
 * callbacks run on host plaintext, with the SSL* the caller associated with
 * the record's session (NULL if none):
 *   write  tlsgpu_seal_host: each record before the batch is copied to the
 *          device, in record order (do_ssl3_write's call, s3_pkt.c.patch:19-33);
 *          the module may rewrite the bytes in place and shorten the record;
 *          tlsgpu_hook_write_streams: each fragment of host application data
 *          that tlsgpu_seal_wire will seal;
 *   read   tlsgpu_open_host and tlsgpu_deliver_host (the batch and wire paths'
 *          host delivery): each delivered record's plaintext once it is in
 *          host memory, in record order (ssl3_read_bytes' call,
 *          s3_pkt.c.patch:39-52); a module that shortens *len shortens the
 *          delivered status.
 * tlsgpu_group_* calls run them per member, in record order within each
 * member's slice. */
int tlsgpu_sessions_set_owner(tlsgpu_sessions *t, uint32_t first, uint32_t n,
    const void *const *owners);
/* Host delivery of a device-resident open (tlsgpu_open_batch, or
 * tlsgpu_open_wire with d_out = d_wire): copies the n descriptors' statuses to
 * h_status and the delivered records' output range [first out_off, last
 * out_off + status) of d_out to the same offsets of h_out (out_bytes = size of
 * d_out / h_out), then runs the read hook on each delivered record.
 * Synchronous on `stream` (NULL = engine stream; order it after the open). */
int tlsgpu_deliver_host(tlsgpu_sessions *t, const tlsgpu_record *d_recs, const int32_t *d_status,
    uint32_t n, const uint8_t *d_out, size_t out_bytes, uint8_t *h_out, int32_t *h_status,
    void *stream);
/* Write hook over host application data before the caller uploads it for
 * tlsgpu_seal_wire: every fragment of every stream (h_streams: host copy of
 * the write streams, offsets into h_data), in place, lengths unchanged. */
struct tlsgpu_write_stream; /* defined below, with tlsgpu_seal_wire */
int tlsgpu_hook_write_streams(tlsgpu_sessions *t, const struct tlsgpu_write_stream *h_streams,
    uint32_t n_streams, uint8_t *h_data, size_t data_bytes);
/* read / write hook invocations since load (from the patched record layer
 * and the engine's paths alike). */
int tlsgpu_talos_hook_stats(uint64_t *read_calls, uint64_t *write_calls);
/* Pipeline shape of tlsgpu_open_host: `streams` compute streams (1..8, default
 * 2; copies in and out have a stream each), chunks of about `chunk_bytes`
 * input bytes (default 32 MiB). */
int tlsgpu_host_pipeline(tlsgpu_engine *e, unsigned streams, size_t chunk_bytes);

/* ---------------------------------------------------------------------------
 * Multi-GPU batch split (BASELINE configs[4]).  Records are
 * independent, so a batch splits into contiguous slices of about equal bytes,
 * one per GPU, with no collective and no xGMI traffic.  A group is one engine
 * per listed device (the same device may be listed twice: two engines, two
 * streams) and one host worker thread per engine; session tables are
 * replicated on every member.  This is what a caller of the per-record
 * tls1_enc (ssl/t1_enc.c:911,964) that batches — a record layer with
 * read-ahead over many connections — binds to use every GPU of the node. */
typedef struct tlsgpu_group tlsgpu_group;
typedef struct tlsgpu_group_sessions tlsgpu_group_sessions;

/* devices == NULL or n == 0: every visible GPU. */
int tlsgpu_group_create(const int *devices, uint32_t n, tlsgpu_group **out);
void tlsgpu_group_destroy(tlsgpu_group *g);
uint32_t tlsgpu_group_size(const tlsgpu_group *g);
tlsgpu_engine *tlsgpu_group_engine(tlsgpu_group *g, uint32_t member);
/* One session table per member, same capacity; install writes every member. */
int tlsgpu_group_sessions_create(tlsgpu_group *g, uint32_t capacity, tlsgpu_group_sessions **out);
void tlsgpu_group_sessions_destroy(tlsgpu_group_sessions *gs);
tlsgpu_sessions *tlsgpu_group_sessions_member(tlsgpu_group_sessions *gs, uint32_t member);
int tlsgpu_group_sessions_install(tlsgpu_group_sessions *gs, uint32_t first, uint32_t n,
    const tlsgpu_session_params *params);

/* Byte-balanced contiguous split of n records into `parts` slices: cuts[0] = 0
 * <= cuts[1] <= ... <= cuts[parts] = n, slice k = records [cuts[k], cuts[k+1]).
 * Cut k is the first record boundary whose prefix of record lengths (len_type
 * bits 0-23) reaches k/parts of the total (integer arithmetic; equal lengths
 * give equal counts).  Host only, no GPU call. */
int tlsgpu_split_by_bytes(const tlsgpu_record *recs, uint32_t n, uint32_t parts, uint32_t *cuts);

/* Host-resident batch over the group: slice k (tlsgpu_split_by_bytes) runs as
 * tlsgpu_open_host / tlsgpu_seal_host on member k, all members at once, each
 * from its own worker thread (its own PCIe link and HBM).  Same buffers,
 * offsets, statuses and synchronous contract as the single-GPU calls; the
 * first member error is returned after every member has finished. */
int tlsgpu_group_open_host(tlsgpu_group_sessions *gs, const tlsgpu_record *h_recs, uint32_t n,
    const uint8_t *h_in, size_t in_bytes, uint8_t *h_out, size_t out_bytes, int32_t *h_status);
int tlsgpu_group_seal_host(tlsgpu_group_sessions *gs, const tlsgpu_record *h_recs, uint32_t n,
    const uint8_t *h_in, size_t in_bytes, uint8_t *h_out, size_t out_bytes, int32_t *h_status);

/* Device-resident batch over the group (per-GPU pools): shards[k] is member
 * k's slice, already in that member's HBM.  Launched on every member's engine
 * stream; asynchronous — tlsgpu_group_sync waits for all members. */
typedef struct tlsgpu_shard {
	const tlsgpu_record *d_recs;
	uint32_t n;
	uint32_t reserved;
	const uint8_t *d_in;
	size_t in_bytes;
	uint8_t *d_out;
	size_t out_bytes;
	int32_t *d_status;
} tlsgpu_shard;
int tlsgpu_group_open_batch(tlsgpu_group_sessions *gs, const tlsgpu_shard *shards);
int tlsgpu_group_seal_batch(tlsgpu_group_sessions *gs, const tlsgpu_shard *shards);
int tlsgpu_group_sync(tlsgpu_group *g);

/* ---------------------------------------------------------------------------
 * Wire-record framing: ssl3_get_record (ssl/s3_pkt.c:279-495)
 * for the AEAD suites over raw read-ahead bytes, many connections at once.
 *
 * Each stream is one connection's read direction: wire_len bytes of TLS
 * records (5-byte header + fragment) at d_wire + wire_off, as ssl3_read_n
 * leaves them in rbuf with read_ahead (s3_pkt.c:134-267).  Per stream, records
 * are framed in order with the header checks of s3_pkt.c:304-341,376:
 *   version != stream version (unless TLSGPU_WIRE_FIRST_PACKET) -> alert
 *   protocol_version (70); major != 3 -> error without alert (alert = -1);
 *   length > rbuf_len - 5 (rbuf_len 0 = the reference's 16712) or
 *   length > SSL3_RT_MAX_ENCRYPTED_LENGTH (16704) -> record_overflow (22);
 *   a record whose fragment is not complete ends the stream's batch (the
 *   caller keeps the bytes from `consumed` on for the next call).
 * Framed records get descriptors (written to d_recs, grouped by stream, seq =
 * stream seq + index) and are opened IN PLACE like tls1_enc(s, 0)
 * (t1_enc.c:951-955: plaintext at fragment + explicit nonce length).  Then,
 * in order, the first record with an AEAD failure or a plaintext longer than
 * 16384 B ends the stream: bad_record_mac (20) for TLSGPU_REC_BAD_MAC,
 * decryption_failed (21) for TLSGPU_REC_PUBLIC_INVALID, record_overflow (22)
 * for TLSGPU_REC_OVERFLOW; later records of that stream get
 * TLSGPU_REC_SKIPPED.  Zero-length plaintexts are delivered with status 0 (the
 * reference reads on, s3_pkt.c:486-488).
 *
 * max_records bounds d_recs / d_status; streams whose records do not fit are
 * truncated at a record boundary (their `records`/`consumed` say how far).
 * d_total receives the number of descriptors written.  Asynchronous. */
#define TLSGPU_WIRE_FIRST_PACKET 1u	/* s->first_packet: accept any version */
typedef struct tlsgpu_wire_stream {
	uint64_t wire_off;	/* first byte of the stream in d_wire */
	uint32_t wire_len;	/* bytes available */
	uint32_t session;	/* read-direction session id */
	uint64_t seq;		/* read sequence number of the first record */
	uint16_t version;	/* s->version, e.g. 0x0303 */
	uint16_t flags;		/* TLSGPU_WIRE_* */
	uint32_t rbuf_len;	/* read buffer size for the overflow check; 0 = 16712 */
} tlsgpu_wire_stream;

typedef struct tlsgpu_wire_result {
	uint32_t first;		/* index of the stream's first record in d_recs / d_status */
	uint32_t records;	/* records framed (descriptors written) */
	uint32_t delivered;	/* records before the first failure */
	uint32_t consumed;	/* bytes of the framed records (header + fragment) */
	int32_t alert;		/* 0, a fatal TLS AlertDescription, or -1 (error, no alert) */
	uint32_t alert_record;	/* index within the stream of the record that failed */
	uint32_t reserved[2];
} tlsgpu_wire_result;

int tlsgpu_open_wire(tlsgpu_sessions *t, const tlsgpu_wire_stream *d_streams,
    uint32_t n_streams, uint8_t *d_wire, uint32_t max_records, tlsgpu_record *d_recs,
    int32_t *d_status, tlsgpu_wire_result *d_results, uint32_t *d_total, void *stream);

/* ---------------------------------------------------------------------------
 * Write-side framing: ssl3_write_bytes + do_ssl3_write
 * (ssl/s3_pkt.c:501-557, 560-762) for the AEAD suites, many connections at
 * once.  Each stream is one connection's SSL_write: data_len bytes of
 * application data at d_data + data_off, split into records of at most
 * max_fragment bytes (max_send_fragment, s3_pkt.c:531-536; a zero-length
 * write sends nothing, :593-594), each written to d_wire as the 5-byte header
 * (type, version, length = explicit nonce + ciphertext + tag, :662-677, :733)
 * followed by tls1_enc(s, 1)'s fragment (explicit nonce = sequence number for
 * GCM, t1_enc.c:887-914), back to back from d_wire + wire_off.  Sequence
 * numbers run seq, seq + 1, ... (t1_enc.c:258-266).  The sealed records also
 * get descriptors in d_recs (slots reserved per stream, like tlsgpu_open_wire;
 * streams that do not fit max_records are cut at a record boundary) and a
 * status each.  data_bytes / wire_bytes bound the buffers
 * (TLSGPU_REC_OUT_OF_BOUNDS).  tlsgpu_seal_wire_size gives a stream's wire
 * bytes.  Asynchronous. */
typedef struct tlsgpu_write_stream {
	uint64_t data_off;	/* application data at d_data + data_off */
	uint64_t wire_off;	/* the stream's records go to d_wire + wire_off */
	uint64_t seq;		/* write sequence number of the first record */
	uint32_t data_len;	/* bytes to send (ssl3_write_bytes' len) */
	uint32_t session;	/* write-direction session id */
	uint16_t version;	/* s->version, e.g. 0x0303 */
	uint8_t type;		/* content type, 23 = application data */
	uint8_t reserved;
	uint32_t max_fragment;	/* s->max_send_fragment; 0 = 16384 */
} tlsgpu_write_stream;

typedef struct tlsgpu_write_result {
	uint32_t first;		/* index of the stream's first record in d_recs / d_status */
	uint32_t records;	/* records written */
	uint64_t wire_len;	/* bytes written from wire_off (headers + fragments) */
	uint64_t next_seq;	/* the write sequence number after the last record */
	uint64_t reserved;
} tlsgpu_write_result;

int tlsgpu_seal_wire(tlsgpu_sessions *t, const tlsgpu_write_stream *d_streams,
    uint32_t n_streams, const uint8_t *d_data, size_t data_bytes, uint8_t *d_wire,
    size_t wire_bytes, uint32_t max_records, tlsgpu_record *d_recs, int32_t *d_status,
    tlsgpu_write_result *d_results, uint32_t *d_total, void *stream);
/* Wire bytes of one stream: ceil(len / frag) records of 5 + explicit nonce
 * (8 for GCM, 0 for ChaCha) + fragment + tag_len bytes (0 when len == 0). */
uint64_t tlsgpu_seal_wire_size(int aead, uint32_t data_len, uint32_t max_fragment,
    uint32_t tag_len);

/* GCM TLS batch kernel selection (process-wide; results are identical).
 * TLSGPU_GCM_AUTO (default): TLSGPU_GCM_SPLIT for batches of at most two
 * records per CU of the device, TLSGPU_GCM_QUEUE for larger ones.
 * TLSGPU_GCM_SPLIT: one record per 16-wave workgroup, the record's blocks split
 * over the waves (latency: a 16 KiB record in ~20 us instead of one wave's
 * serial pass).
 * TLSGPU_GCM_QUEUE: a prep pass computes every record's E_K(J0) and
 * round-1/2 constants, then 16 T-table waves per CU (AES rounds as LDS
 * lookups) pull records from a per-session-run queue.  Records of <= 62
 * blocks share a wave in packs (environment TLSGPU_PACK=0 turns packs off).
 * TLSGPU_GCM_TTABLE: T-table waves with in-kernel constants, static split.
 * TLSGPU_GCM_HYBRID: 4 bitsliced waves (AES-CTR on the VALU, pairs of
 * 16-byte-aligned records of >= 16 KiB) beside 4 T-table waves per CU.
 * TLSGPU_GCM_BITSLICE: 8 bitsliced waves per CU.
 * TLSGPU_GCM_FUSED: 8 waves per CU, each running a bitsliced record pair with
 * a T-table record interleaved into its AES rounds.
 * The environment variable TLSGPU_GCM_IMPL=auto|split|queue|ttable|hybrid|bitslice|fused
 * sets the initial value.  The per-call EVP path always uses the split kernel
 * on its raw jobs. */
enum tlsgpu_gcm_impl {
  TLSGPU_GCM_BITSLICE = 0, TLSGPU_GCM_TTABLE = 1, TLSGPU_GCM_HYBRID = 2, TLSGPU_GCM_QUEUE = 3,
  TLSGPU_GCM_FUSED = 4, TLSGPU_GCM_SPLIT = 5, TLSGPU_GCM_AUTO = 6
};
int tlsgpu_set_gcm_impl(int impl);
int tlsgpu_get_gcm_impl(void);

/* EVP coalescing queue.  Turns on batching for the per-call
 * EVP_AEAD_* drop-in: contexts initialised afterwards take a slot of one shared
 * device session pool (pool_sessions, default 1024; contexts beyond it keep a
 * private table and the per-call path), and their seal/open calls are queued;
 * a dispatcher thread runs everything that arrives within window_us (or
 * max_jobs, default 4096) as one raw batch per direction and wakes the callers.
 * Outputs, return values and zero-fill are those of the per-call path.  Calling
 * it again adjusts window_us / max_jobs.  The environment variables
 * TLSGPU_EVP_BATCH_US / TLSGPU_EVP_POOL do the same at library load.
 * tlsgpu_evp_batch_stats: batches run and jobs served so far. */
int tlsgpu_evp_set_batching(unsigned window_us, unsigned max_jobs, unsigned pool_sessions);
int tlsgpu_evp_batch_stats(uint64_t *batches, uint64_t *jobs);
/* EVP_AEAD_CTX_seal / _open calls whose cipher work ran on the GPU (per-call
 * or queued; authentication failures included, argument-check rejections
 * not), process-wide since load.  Lets a caller that interposed the library
 * under an unchanged libssl check that every TLS record went through it. */
int tlsgpu_evp_call_stats(uint64_t *seal_calls, uint64_t *open_calls);
/* Doorbell server for per-call EVP calls (round 4).  groups > 0 keeps up to
 * that many 1024-thread server workgroups (one CU each, one per calling thread)
 * resident on every EVP device while calls arrive: a calling thread posts its
 * job (the same zero-copy RawJob the launched path builds) in a slot of pinned
 * host memory and spins on the answer, so a synchronous EVP_AEAD_CTX_seal /
 * _open on an AES-GCM, RFC 7539 or draft ChaCha20-Poly1305 context costs one
 * PCIe round trip instead of a kernel launch + stream sync.  Each server
 * instance exits after lifetime_ms (0 = 5 ms) and is relaunched by the next
 * call, so an idle process leaves nothing running.  Threads beyond
 * 8 * groups per device and pooled (queued) contexts use the other paths.
 * Same as
 * TLSGPU_EVP_DOORBELL=<groups> (TLSGPU_EVP_DOORBELL_MS=<lifetime>) at load;
 * on by default with 64 groups (round 5; 0 turns it off); must be called
 * before the first EVP call.  With it on, EVP_AEAD_CTX_init launches nothing
 * (the session image is built on the host and installed by the context's
 * first call) and EVP_AEAD_CTX_cleanup scrubs the slot through the server.
 * tlsgpu_evp_doorbell_stats: jobs served and instances launched so far.
 * tlsgpu_evp_doorbell_scrub_stats (round 6): scrub jobs served, and times a
 * server workgroup other than the scrubbing one zeroed its LDS copy of a
 * scrubbed key (the scrub ring). */
int tlsgpu_evp_set_doorbell(unsigned groups, unsigned lifetime_ms);
int tlsgpu_evp_doorbell_stats(uint64_t *jobs, uint64_t *launches);
int tlsgpu_evp_doorbell_scrub_stats(uint64_t *scrubs, uint64_t *flushes);
/* tlsgpu_evp_doorbell_warm: launch a server instance now on every EVP device
 * whose queued instance would stop polling within half a lifetime (what the
 * next call would do), e.g. before a burst of calls.  No-op with the doorbell
 * off or after shutdown.
 * tlsgpu_evp_shutdown: the doorbell's shutdown contract.  Stops every server,
 * then waits until every instance ever launched — running or still queued
 * behind other work — has left, reading pinned memory only (no HIP call);
 * later EVP calls take the launched path.  TLSGPU_ETIMEOUT if an instance is
 * still running after TLSGPU_EVP_SHUTDOWN_MS (default 60 s).  Idempotent.
 * The library runs it itself first thing at process exit (the main thread's
 * thread-local destructors run before the HIP runtime's exit-time teardown),
 * from an atexit handler and from its destructor; an application that tears
 * the runtime down itself (hipDeviceReset) calls it before. */
int tlsgpu_evp_doorbell_warm(void);
/* Test support: the device image of one session as EVP_AEAD_CTX_init builds it
 * on the host (DevSession, 1 KiB, then the GCM tables: basis, Shoup tables of
 * H^1..H^65, bitsliced masks; zero for ChaCha) into out[0..n), n >= 27,392.
 * tests/test_session_image.py checks it against the device install kernel. */
int tlsgpu_session_image(const tlsgpu_session_params *p, uint8_t *out, size_t n);
int tlsgpu_evp_shutdown(void);
/* Test support.  tlsgpu_evp_context_slot: the session table and slot that hold
 * a live EVP context's device key material.  tlsgpu_sessions_debug_read: after
 * every queued install / scrub of `slot` has finished, copy its first n bytes
 * (DevSession, then the GCM tables) to host memory — EVP_AEAD_CTX_cleanup
 * scrubs the slot asynchronously, and this shows the scrub happened.  (The key
 * also travels to the install kernel as a kernel argument, in the HIP
 * runtime's argument buffer, which later launches overwrite but nothing
 * zeroes: DESIGN.md §4.7.) */
struct evp_aead_ctx_st; /* EVP_AEAD_CTX, include/tlsgpu_evp.h */
int tlsgpu_evp_context_slot(const struct evp_aead_ctx_st *ctx, tlsgpu_sessions **sessions,
    uint32_t *slot);
int tlsgpu_sessions_debug_read(tlsgpu_sessions *t, uint32_t slot, uint8_t *out, size_t n);
/* The EVP surface's GPUs.  TLSGPU_DEVICES=a,b,... (a device may repeat: two
 * engines on one GPU) or TLSGPU_DEVICE=d pin them; by default every visible
 * GPU.  EVP_AEAD_CTX_init gives new contexts (and EVP_CIPHER contexts their
 * first key) to these devices in turn; each device has its own engine, call
 * streams and, with batching on, its own coalescing queue and session pool
 * (pool_sessions each).  tlsgpu_evp_device_stats(k, ...): device ordinal,
 * contexts created and EVP calls run on the k-th of them. */
uint32_t tlsgpu_evp_device_count(void);
int tlsgpu_evp_device_stats(uint32_t k, int *device, uint64_t *contexts, uint64_t *calls);
/* GPU programs run by the EVP_aes_{128,256}_gcm EVP_CIPHER objects
 * (include/tlsgpu_evp.h), process-wide since load. */
int tlsgpu_evp_cipher_stats(uint64_t *programs);

/* Diagnostic: hybrid-kernel phase timing.  With TLSGPU_PHASE_STATS=1 in the
 * environment, the first call allocates 32 device counters (shader cycles and
 * event counts per phase, summed over waves) that later hybrid launches fill;
 * each call synchronizes the device, copies them to out32 (may be NULL) and
 * optionally resets them.  Fails when the variable is not set. */
int tlsgpu_debug_phase_stats(tlsgpu_engine *e, unsigned long long *out32, int reset);

/* Diagnostic: per-workgroup timing of the queue kernel.  With
 * TLSGPU_WG_TIMES=1 in the environment every queue launch writes, per
 * workgroup g, out[4g..4g+3] = {start, end (100 MHz s_memrealtime ticks),
 * records, work (payload bytes + 256 per record)} of the records it ran; this
 * call synchronizes the device and copies the first `groups` (<= 1024)
 * entries of the last launch.  Fails when the
 * variable is not set or before the first launch. */
int tlsgpu_debug_wg_times(tlsgpu_engine *e, unsigned long long *out, unsigned groups);

/* Diagnostic: ECB-encrypt nblocks 16-byte blocks (device memory) under the
 * AES key of GCM session `session` with the bitsliced AES core. */
int tlsgpu_aes_ecb_bitsliced(tlsgpu_sessions *t, uint32_t session, const uint8_t *d_in,
    uint8_t *d_out, uint32_t nblocks, void *stream);

/* Deterministic synthetic bytes, counter-based SplitMix64 keyed by
 * (seed, index0 + i) for each of n spans of span_len bytes at d_out + i*stride
 * (same stream as the oracle's oracle_fill_bytes; used by bench/tests). */
int tlsgpu_fill_synthetic(tlsgpu_engine *e, uint8_t *d_out, uint64_t stride,
    uint32_t span_len, uint32_t n, uint64_t seed, uint64_t index0, void *stream);
/* The same stream for n variable-length spans in one launch: span i covers
 * d_lengths[i] bytes at d_out + d_offsets[i] (device arrays) and is keyed
 * (seed, index0 + i). */
int tlsgpu_fill_synthetic_spans(tlsgpu_engine *e, uint8_t *d_out, const uint64_t *d_offsets,
    const uint32_t *d_lengths, uint32_t n, uint64_t seed, uint64_t index0, void *stream);

/* Device / pinned-host memory, copies and events on the engine's device, so
 * callers need no other GPU runtime (the bench and tests use only these). */
int tlsgpu_malloc(tlsgpu_engine *e, size_t bytes, void **d_ptr);
int tlsgpu_free(tlsgpu_engine *e, void *d_ptr);
int tlsgpu_host_alloc(tlsgpu_engine *e, size_t bytes, void **h_ptr);	/* pinned */
int tlsgpu_host_free(tlsgpu_engine *e, void *h_ptr);
/* Async copy in any direction (hipMemcpyDefault) on `stream` (NULL = engine). */
int tlsgpu_memcpy(tlsgpu_engine *e, void *dst, const void *src, size_t bytes, void *stream);
int tlsgpu_memset(tlsgpu_engine *e, void *d_ptr, int value, size_t bytes, void *stream);
int tlsgpu_stream_create(tlsgpu_engine *e, void **stream);
int tlsgpu_stream_destroy(tlsgpu_engine *e, void *stream);
int tlsgpu_stream_sync(tlsgpu_engine *e, void *stream);
int tlsgpu_event_create(tlsgpu_engine *e, void **event);
int tlsgpu_event_destroy(tlsgpu_engine *e, void *event);
int tlsgpu_event_record(tlsgpu_engine *e, void *event, void *stream);
/* Milliseconds between two recorded events (waits for `end`). */
int tlsgpu_event_elapsed_ms(tlsgpu_engine *e, void *start, void *end, float *ms);

/* Human-readable last error of this thread. */
const char *tlsgpu_last_error(void);

#ifdef __cplusplus
}
#endif
#endif
