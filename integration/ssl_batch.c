/*
 * ssl_batch.c — batching TLS record-layer consumer (see ssl_batch.h).
 *
 * Per call:
 *   1. gather   per connection: the partial record kept from the last call,
 *               then BIO_read of the connection's read BIO into the pinned
 *               wire buffer (ssl3_read_n's job, s3_pkt.c:134-267, for all
 *               connections into one buffer instead of one rbuf each);
 *   2. frame    walk the 5-byte headers with ssl3_get_record's rules
 *               (s3_pkt.c:305-380: version == s->version, major 3, length <=
 *               SSL3_RT_MAX_ENCRYPTED_LENGTH) and build one tlsgpu_record per
 *               complete application-data record: the fragment, its sequence
 *               number (s3->read_sequence + k), the connection's session;
 *   3. open     one tlsgpu_open_host over all of them, in place (plaintext at
 *               fragment + 8 for GCM, t1_enc.c:951-955);
 *   4. deliver  per connection, in record order, until its first failure;
 *               read_sequence += records opened (tls1_record_sequence_increment,
 *               t1_enc.c:258-266, once per record as tls1_enc does).
 */
#include "ssl_batch.h"

#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "ssl_locl.h" /* SSL_AEAD_CTX, SSL3_STATE (the reference tree's own header) */

struct conn {
	SSL *s;
	int attached;
	uint32_t eiv;             /* explicit nonce bytes in the fragment (8 for GCM) */
	uint8_t *pend;            /* partial record kept between calls */
	size_t pend_len;
};

struct tlsgpu_ssl_batch {
	tlsgpu_engine *e;
	tlsgpu_sessions *t;
	uint32_t cap;
	struct conn *c;
	uint8_t *wire;            /* pinned */
	size_t wire_cap;
	tlsgpu_record *recs;      /* pinned */
	int32_t *status;          /* pinned */
	uint32_t rec_cap;
	uint32_t *first, *count;  /* per position in conns[]: its descriptors */
	double t_gather, t_open, t_deliver;  /* the last call's phases, seconds */
};

static double
now_s(void)
{
	struct timespec ts;
	clock_gettime(CLOCK_MONOTONIC, &ts);
	return ts.tv_sec + ts.tv_nsec * 1e-9;
}

void
tlsgpu_ssl_batch_times(const tlsgpu_ssl_batch *b, double *gather_s, double *open_s,
    double *deliver_s)
{
	*gather_s = b->t_gather;
	*open_s = b->t_open;
	*deliver_s = b->t_deliver;
}

int
tlsgpu_ssl_batch_create(int device, uint32_t max_conns, size_t wire_bytes, tlsgpu_ssl_batch **out)
{
	tlsgpu_ssl_batch *b = calloc(1, sizeof(*b));
	int rc;
	if (!b || !max_conns || wire_bytes < SSL3_RT_MAX_PACKET_SIZE)
		return free(b), TLSGPU_EINVAL;
	b->cap = max_conns;
	/* at most one record per 5 + 1 header + fragment bytes: size the
	 * descriptor arrays for the smallest legal AEAD record (tag only) */
	b->rec_cap = (uint32_t)(wire_bytes / (SSL3_RT_HEADER_LENGTH + 16) + 1);
	if ((rc = tlsgpu_engine_create(device, &b->e)) != TLSGPU_OK ||
	    (rc = tlsgpu_sessions_create(b->e, max_conns, &b->t)) != TLSGPU_OK ||
	    (rc = tlsgpu_host_alloc(b->e, wire_bytes, (void **)&b->wire)) != TLSGPU_OK ||
	    (rc = tlsgpu_host_alloc(b->e, sizeof(tlsgpu_record) * (size_t)b->rec_cap,
	        (void **)&b->recs)) != TLSGPU_OK ||
	    (rc = tlsgpu_host_alloc(b->e, 4 * (size_t)b->rec_cap, (void **)&b->status)) != TLSGPU_OK) {
		tlsgpu_ssl_batch_destroy(b);
		return rc;
	}
	b->wire_cap = wire_bytes;
	b->c = calloc(max_conns, sizeof(*b->c));
	b->first = calloc(max_conns, sizeof(uint32_t));
	b->count = calloc(max_conns, sizeof(uint32_t));
	if (!b->c || !b->first || !b->count) {
		tlsgpu_ssl_batch_destroy(b);
		return TLSGPU_ENOMEM;
	}
	*out = b;
	return TLSGPU_OK;
}

void
tlsgpu_ssl_batch_destroy(tlsgpu_ssl_batch *b)
{
	if (!b)
		return;
	if (b->c)
		for (uint32_t i = 0; i < b->cap; i++)
			free(b->c[i].pend);
	if (b->e) {
		if (b->wire)
			tlsgpu_host_free(b->e, b->wire);
		if (b->recs)
			tlsgpu_host_free(b->e, b->recs);
		if (b->status)
			tlsgpu_host_free(b->e, b->status);
	}
	if (b->t)
		tlsgpu_sessions_destroy(b->t);
	if (b->e)
		tlsgpu_engine_destroy(b->e);
	free(b->c);
	free(b->first);
	free(b->count);
	free(b);
}

int
tlsgpu_ssl_batch_attach(tlsgpu_ssl_batch *b, uint32_t conn, SSL *s, const uint8_t *key,
    size_t key_len)
{
	const SSL_AEAD_CTX *a;
	tlsgpu_session_params p;
	int rc;
	if (!b || conn >= b->cap || !s || !(a = s->aead_read_ctx) || !key ||
	    (key_len != 16 && key_len != 32) || a->fixed_nonce_len > 12)
		return TLSGPU_EINVAL;
	memset(&p, 0, sizeof(p));
	/* the suite from the record layer's nonce layout (t1_enc.c:444-495:
	 * GCM carries an 8-byte explicit nonce after a 4-byte fixed one; RFC 7539
	 * ChaCha XORs a 12-byte fixed nonce; the draft suite has neither) */
	if (a->variable_nonce_in_record)
		p.aead = key_len == 16 ? TLSGPU_AES_128_GCM : TLSGPU_AES_256_GCM;
	else if (a->xor_fixed_nonce)
		p.aead = TLSGPU_CHACHA20_POLY1305;
	else
		p.aead = TLSGPU_CHACHA20_POLY1305_OLD;
	p.key_len = (uint32_t)key_len;
	memcpy(p.key, key, key_len);
	p.fixed_iv_len = a->fixed_nonce_len;
	memcpy(p.fixed_iv, a->fixed_nonce, a->fixed_nonce_len);
	p.tag_len = a->tag_len;
	p.version = (uint16_t)s->version;
	rc = tlsgpu_sessions_install(b->t, conn, 1, &p);
	explicit_bzero(&p, sizeof(p));
	if (rc != TLSGPU_OK)
		return rc;
	{
		const void *owner = s;  /* TaLoS read hook: the record's SSL* */
		if ((rc = tlsgpu_sessions_set_owner(b->t, conn, 1, &owner)) != TLSGPU_OK)
			return rc;
	}
	if (!b->c[conn].pend && !(b->c[conn].pend = malloc(SSL3_RT_MAX_PACKET_SIZE)))
		return TLSGPU_ENOMEM;
	b->c[conn].s = s;
	b->c[conn].attached = 1;
	b->c[conn].eiv = a->variable_nonce_in_record ? 8u : 0u;
	b->c[conn].pend_len = 0;
	return TLSGPU_OK;
}

static uint64_t
seq_load(const unsigned char *q)
{
	uint64_t v = 0;
	for (int i = 0; i < 8; i++)
		v = (v << 8) | q[i];
	return v;
}

static void
seq_store(unsigned char *q, uint64_t v)
{
	for (int i = 7; i >= 0; i--, v >>= 8)
		q[i] = (unsigned char)v;
}

int
tlsgpu_ssl_batch_read(tlsgpu_ssl_batch *b, const uint32_t *conns, uint32_t n,
    tlsgpu_ssl_deliver_fn deliver, void *arg, int *conn_status)
{
	size_t used = 0;
	uint32_t nrec = 0;
	int delivered = 0, rc;
	if (!b || (n && (!conns || !conn_status)))
		return TLSGPU_EINVAL;
	const double t0 = now_s();
	b->t_gather = b->t_open = b->t_deliver = 0;
	for (uint32_t i = 0; i < n; i++) {
		const uint32_t id = conns[i];
		struct conn *c = id < b->cap ? &b->c[id] : NULL;
		b->first[i] = nrec;
		b->count[i] = 0;
		conn_status[i] = TLSGPU_SSL_OK;
		if (!c || !c->attached) {
			conn_status[i] = TLSGPU_SSL_NOT_ATTACHED;
			continue;
		}
		/* 1. gather: the kept partial record, then the BIO's bytes */
		const size_t start = used;
		if (c->pend_len > b->wire_cap - used)
			continue;  /* no room this call: the connection waits for the next */
		memcpy(b->wire + used, c->pend, c->pend_len);
		used += c->pend_len;
		c->pend_len = 0;
		BIO *rb = SSL_get_rbio(c->s);
		for (int k; used < b->wire_cap &&
		    (k = BIO_read(rb, b->wire + used, (int)(b->wire_cap - used > 1u << 30 ?
		    1u << 30 : b->wire_cap - used))) > 0;)
			used += (size_t)k;
		/* 2. frame (ssl3_get_record's header checks) */
		const uint64_t seq0 = seq_load(c->s->s3->read_sequence);
		size_t p = start;
		while (used - p >= SSL3_RT_HEADER_LENGTH) {
			const uint8_t *h = b->wire + p;
			const unsigned type = h[0], version = (unsigned)h[1] << 8 | h[2];
			const size_t len = (size_t)h[3] << 8 | h[4];
			if (version != (unsigned)c->s->version) {
				conn_status[i] = TLSGPU_SSL_WRONG_VERSION;
				break;
			}
			if (len > SSL3_RT_MAX_ENCRYPTED_LENGTH) {
				conn_status[i] = TLSGPU_SSL_RECORD_OVERFLOW;
				break;
			}
			if (used - p - SSL3_RT_HEADER_LENGTH < len)
				break;  /* partial: kept for the next call */
			if (type != SSL3_RT_APPLICATION_DATA) {
				conn_status[i] = TLSGPU_SSL_NOT_APP_DATA;
				break;
			}
			if (nrec == b->rec_cap)
				break;
			tlsgpu_record *r = &b->recs[nrec++];
			r->in_off = p + SSL3_RT_HEADER_LENGTH;
			r->out_off = r->in_off + c->eiv;
			r->seq = seq0 + b->count[i];
			r->session = id;
			r->len_type = TLSGPU_LEN_TYPE(len, type);
			b->count[i]++;
			p += SSL3_RT_HEADER_LENGTH + len;
		}
		/* what is not framed stays with the connection (at most one
		 * partial record, or the bytes after a failure / non-data record) */
		const size_t rest = used - p;
		if (rest) {
			if (rest > SSL3_RT_MAX_PACKET_SIZE) {
				uint8_t *q = realloc(c->pend, rest);
				if (!q)
					return TLSGPU_ENOMEM;
				c->pend = q;
			}
			memcpy(c->pend, b->wire + p, rest);
			c->pend_len = rest;
		}
		used = p;
	}
	const double t1 = now_s();
	b->t_gather = t1 - t0;
	if (nrec == 0)
		return 0;
	/* 3. one batch for every connection's records, in place */
	if ((rc = tlsgpu_open_host(b->t, b->recs, nrec, b->wire, used, b->wire, used,
	    b->status)) != TLSGPU_OK)
		return rc;
	const double t2 = now_s();
	b->t_open = t2 - t1;
	/* 4. deliver in record order per connection; the read sequence advances
	 *    over every record opened (a failed one ends the connection's batch) */
	for (uint32_t i = 0; i < n; i++) {
		if (conn_status[i] == TLSGPU_SSL_NOT_ATTACHED)
			continue;
		struct conn *c = &b->c[conns[i]];
		uint32_t k = 0;
		for (; k < b->count[i]; k++) {
			const tlsgpu_record *r = &b->recs[b->first[i] + k];
			const int32_t st = b->status[b->first[i] + k];
			if (st < 0) {
				conn_status[i] = TLSGPU_SSL_BAD_RECORD_MAC;
				break;
			}
			if (deliver)
				deliver(arg, conns[i], c->s, b->wire + r->out_off, (size_t)st);
			delivered++;
		}
		seq_store(c->s->s3->read_sequence, seq_load(c->s->s3->read_sequence) + k);
	}
	b->t_deliver = now_s() - t2;
	return delivered;
}
