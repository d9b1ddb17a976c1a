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
 *
 * Pipelined: the connections are taken in groups of about kGroupBytes of wire,
 * alternating between two halves of the pinned buffer.  A worker thread runs
 * group k's tlsgpu_open_host while the calling thread delivers group k-1 and
 * gathers group k+1, so the GPU batch (PCIe in, kernels, PCIe out) overlaps
 * the host copies.  BIO reads, delivery callbacks and SSL state stay on the
 * calling thread.
 */
#include "ssl_batch.h"

#include <pthread.h>
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
	int wattached;            /* write key installed (session cap + id) */
	uint32_t weiv, wtag;      /* write side: explicit nonce and tag bytes */
};

/* wire bytes per group: the pipeline's unit (16 MiB: ~0.4 ms of PCIe each way) */
static const size_t kGroupBytes = (size_t)16 << 20;

struct group {
	uint32_t i0, i1;          /* positions in conns[] */
	size_t used;              /* wire bytes */
	uint32_t nrec;
};

struct tlsgpu_ssl_batch {
	tlsgpu_engine *e;
	tlsgpu_sessions *t;
	uint32_t cap;
	struct conn *c;
	uint8_t *wire;            /* pinned, nslot slots of slot_cap bytes */
	size_t wire_cap, slot_cap;
	tlsgpu_record *recs;      /* pinned, rec_cap per slot */
	int32_t *status;          /* pinned, rec_cap per slot */
	uint32_t rec_cap, nslot;
	uint32_t *first, *count;  /* per position in conns[]: its descriptors in its slot */
	/* write side (allocated at the first tlsgpu_ssl_batch_attach_write):
	 * nslot slots of w_cap plaintext in and w_cap wire out, w_rec_cap records */
	uint8_t *w_in, *w_out;    /* pinned */
	tlsgpu_record *w_recs;    /* pinned */
	int32_t *w_status;        /* pinned */
	uint32_t *w_pos;          /* position in conns[] of each write descriptor */
	size_t w_cap;
	uint32_t w_rec_cap;
	struct wgroup {
		uint32_t nrec;
		size_t in_used, out_used;
	} wg[2];
	struct group g[2];
	double t_gather, t_open, t_deliver;  /* the last call's phases, seconds (overlapped) */
	/* the GPU worker: runs tlsgpu_open_host on one posted slot at a time */
	pthread_t worker;
	/* jobs: 0 / 1 = open read slot 0 / 1, 2 / 3 = seal write slot 0 / 1 */
	int have_worker, quit, posted, done[4], rc[4];
	pthread_mutex_t mu;
	pthread_cond_t cv;
};

static double now_s(void);

static void *
gpu_worker(void *p)
{
	tlsgpu_ssl_batch *b = p;
	pthread_mutex_lock(&b->mu);
	for (;;) {
		while (!b->quit && b->posted < 0)
			pthread_cond_wait(&b->cv, &b->mu);
		if (b->quit)
			break;
		const int j = b->posted;
		b->posted = -1;
		const struct group g = b->g[j & 1];
		const struct wgroup wgj = b->wg[j & 1];
		pthread_mutex_unlock(&b->mu);
		const size_t s = (size_t)(j & 1);
		const double t0 = now_s();
		int rc;
		if (j < 2) {
			uint8_t *w = b->wire + s * b->slot_cap;
			rc = tlsgpu_open_host(b->t, b->recs + s * b->rec_cap, g.nrec, w, g.used, w, g.used,
			    b->status + s * b->rec_cap);
		} else {
			rc = tlsgpu_seal_host(b->t, b->w_recs + s * b->w_rec_cap, wgj.nrec,
			    b->w_in + s * b->w_cap, wgj.in_used, b->w_out + s * b->w_cap, wgj.out_used,
			    b->w_status + s * b->w_rec_cap);
		}
		const double dt = now_s() - t0;
		pthread_mutex_lock(&b->mu);
		b->t_open += dt;
		b->rc[j] = rc;
		b->done[j] = 1;
		pthread_cond_broadcast(&b->cv);
	}
	pthread_mutex_unlock(&b->mu);
	return NULL;
}

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
	/* two slots (pipelined) when each still holds two records of the largest size */
	b->nslot = wire_bytes >= 4 * (size_t)SSL3_RT_MAX_PACKET_SIZE ? 2u : 1u;
	b->slot_cap = wire_bytes / b->nslot;
	/* at most one record per 5 + 1 header + fragment bytes: size the
	 * descriptor arrays for the smallest legal AEAD record (tag only) */
	b->rec_cap = (uint32_t)(b->slot_cap / (SSL3_RT_HEADER_LENGTH + 16) + 1);
	b->posted = -1;
	if (pthread_mutex_init(&b->mu, NULL) != 0)
		return free(b), TLSGPU_ENOMEM;
	if (pthread_cond_init(&b->cv, NULL) != 0) {
		pthread_mutex_destroy(&b->mu);
		return free(b), TLSGPU_ENOMEM;
	}
	if ((rc = tlsgpu_engine_create(device, &b->e)) != TLSGPU_OK ||
	    (rc = tlsgpu_sessions_create(b->e, 2 * max_conns, &b->t)) != TLSGPU_OK ||
	    (rc = tlsgpu_host_alloc(b->e, wire_bytes, (void **)&b->wire)) != TLSGPU_OK ||
	    (rc = tlsgpu_host_alloc(b->e, sizeof(tlsgpu_record) * b->nslot * (size_t)b->rec_cap,
	        (void **)&b->recs)) != TLSGPU_OK ||
	    (rc = tlsgpu_host_alloc(b->e, 4 * (size_t)b->nslot * b->rec_cap,
	        (void **)&b->status)) != TLSGPU_OK) {
		tlsgpu_ssl_batch_destroy(b);
		return rc;
	}
	b->wire_cap = wire_bytes;
	if (pthread_create(&b->worker, NULL, gpu_worker, b) != 0) {
		tlsgpu_ssl_batch_destroy(b);
		return TLSGPU_ENOMEM;
	}
	b->have_worker = 1;
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
	if (b->have_worker) {
		pthread_mutex_lock(&b->mu);
		b->quit = 1;
		pthread_cond_broadcast(&b->cv);
		pthread_mutex_unlock(&b->mu);
		pthread_join(b->worker, NULL);
	}
	pthread_cond_destroy(&b->cv);
	pthread_mutex_destroy(&b->mu);
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
		if (b->w_in)
			tlsgpu_host_free(b->e, b->w_in);
		if (b->w_out)
			tlsgpu_host_free(b->e, b->w_out);
		if (b->w_recs)
			tlsgpu_host_free(b->e, b->w_recs);
		if (b->w_status)
			tlsgpu_host_free(b->e, b->w_status);
	}
	free(b->w_pos);
	if (b->t)
		tlsgpu_sessions_destroy(b->t);
	if (b->e)
		tlsgpu_engine_destroy(b->e);
	free(b->c);
	free(b->first);
	free(b->count);
	free(b);
}

/* Install one direction's key in session `slot` from that direction's record
 * state (the SSL_AEAD_CTX tls1_change_cipher_state_aead filled). */
static int
install_direction(tlsgpu_ssl_batch *b, uint32_t slot, SSL *s, const SSL_AEAD_CTX *a,
    const uint8_t *key, size_t key_len)
{
	tlsgpu_session_params p;
	int rc;
	if (!a || !key || (key_len != 16 && key_len != 32) || a->fixed_nonce_len > 12)
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
	rc = tlsgpu_sessions_install(b->t, slot, 1, &p);
	explicit_bzero(&p, sizeof(p));
	if (rc != TLSGPU_OK)
		return rc;
	const void *owner = s;  /* TaLoS read / write hooks: the record's SSL* */
	return tlsgpu_sessions_set_owner(b->t, slot, 1, &owner);
}

int
tlsgpu_ssl_batch_attach(tlsgpu_ssl_batch *b, uint32_t conn, SSL *s, const uint8_t *key,
    size_t key_len)
{
	int rc;
	if (!b || conn >= b->cap || !s)
		return TLSGPU_EINVAL;
	const SSL_AEAD_CTX *a = s->aead_read_ctx;
	if ((rc = install_direction(b, conn, s, a, key, key_len)) != TLSGPU_OK)
		return rc;
	if (!b->c[conn].pend && !(b->c[conn].pend = malloc(SSL3_RT_MAX_PACKET_SIZE)))
		return TLSGPU_ENOMEM;
	b->c[conn].s = s;
	b->c[conn].attached = 1;
	b->c[conn].eiv = a->variable_nonce_in_record ? 8u : 0u;
	b->c[conn].pend_len = 0;
	return TLSGPU_OK;
}

int
tlsgpu_ssl_batch_attach_write(tlsgpu_ssl_batch *b, uint32_t conn, SSL *s, const uint8_t *key,
    size_t key_len)
{
	int rc;
	if (!b || conn >= b->cap || !s)
		return TLSGPU_EINVAL;
	const SSL_AEAD_CTX *a = s->aead_write_ctx;
	if (!b->w_in) {  /* the write side's buffers, once: nslot slots of up to 2 groups */
		b->w_cap = b->slot_cap < 2 * kGroupBytes ? b->slot_cap : 2 * kGroupBytes;
		b->w_rec_cap = (uint32_t)(b->w_cap / (SSL3_RT_HEADER_LENGTH + 16) + 1);
		const size_t ns = b->nslot;
		if ((rc = tlsgpu_host_alloc(b->e, ns * b->w_cap, (void **)&b->w_in)) != TLSGPU_OK ||
		    (rc = tlsgpu_host_alloc(b->e, ns * b->w_cap, (void **)&b->w_out)) != TLSGPU_OK ||
		    (rc = tlsgpu_host_alloc(b->e, ns * sizeof(tlsgpu_record) * b->w_rec_cap,
		        (void **)&b->w_recs)) != TLSGPU_OK ||
		    (rc = tlsgpu_host_alloc(b->e, ns * 4 * (size_t)b->w_rec_cap,
		        (void **)&b->w_status)) != TLSGPU_OK)
			return rc;
		if (!(b->w_pos = malloc(ns * sizeof(uint32_t) * b->w_rec_cap)))
			return TLSGPU_ENOMEM;
	}
	if ((rc = install_direction(b, b->cap + conn, s, a, key, key_len)) != TLSGPU_OK)
		return rc;
	b->c[conn].s = s;
	b->c[conn].wattached = 1;
	b->c[conn].weiv = a->variable_nonce_in_record ? 8u : 0u;
	b->c[conn].wtag = a->tag_len;
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

/* Deliver group slot s (its open is done): per connection, in record order,
 * until its first failure; the read sequence advances over every record
 * opened (a failed one ends the connection's batch). */
/* What a finished slot needs: the call's connections and statuses, and the
 * read side's delivery callback. */
struct finish_ctx {
	const uint32_t *conns;
	int *conn_status;
	tlsgpu_ssl_deliver_fn deliver;
	void *arg;
	int total;   /* records delivered / written */
	int err;     /* the first GPU job error */
};
typedef int (*finish_fn)(tlsgpu_ssl_batch *b, uint32_t s, struct finish_ctx *f);

static int
deliver_group(tlsgpu_ssl_batch *b, uint32_t s, struct finish_ctx *f)
{
	const uint32_t *conns = f->conns;
	int *conn_status = f->conn_status;
	const double t0 = now_s();
	const struct group *g = &b->g[s];
	const tlsgpu_record *recs = b->recs + (size_t)s * b->rec_cap;
	const int32_t *status = b->status + (size_t)s * b->rec_cap;
	const uint8_t *w = b->wire + (size_t)s * b->slot_cap;
	int delivered = 0;
	for (uint32_t i = g->i0; i < g->i1; i++) {
		if (conn_status[i] == TLSGPU_SSL_NOT_ATTACHED)
			continue;
		struct conn *c = &b->c[conns[i]];
		uint32_t k = 0;
		for (; k < b->count[i]; k++) {
			const tlsgpu_record *r = &recs[b->first[i] + k];
			const int32_t st = status[b->first[i] + k];
			if (st < 0) {
				conn_status[i] = TLSGPU_SSL_BAD_RECORD_MAC;
				break;
			}
			if (f->deliver)
				f->deliver(f->arg, conns[i], c->s, w + r->out_off, (size_t)st);
			delivered++;
		}
		seq_store(c->s->s3->read_sequence, seq_load(c->s->s3->read_sequence) + k);
	}
	b->t_deliver += now_s() - t0;
	return delivered;
}

/* Wait for slot s's open; its status, or TLSGPU_OK when nothing was posted. */
static int
wait_slot(tlsgpu_ssl_batch *b, uint32_t s)
{
	pthread_mutex_lock(&b->mu);
	while (!b->done[s])
		pthread_cond_wait(&b->cv, &b->mu);
	const int rc = b->rc[s];
	pthread_mutex_unlock(&b->mu);
	return rc;
}

/* The two-slot pipeline, shared by reads (worker jobs 0 / 1) and writes
 * (jobs 2 / 3): slot `s` is being filled on the calling thread while slot
 * `inflight` is on the GPU. */
struct pipe {
	uint32_t s;
	int inflight;
};

static void
post_job(tlsgpu_ssl_batch *b, int j)
{
	pthread_mutex_lock(&b->mu);
	b->done[j] = 0;
	b->posted = j;
	pthread_cond_broadcast(&b->cv);
	pthread_mutex_unlock(&b->mu);
}

static void
pipe_finish(tlsgpu_ssl_batch *b, uint32_t slot, int rc, finish_fn fin, struct finish_ctx *f)
{
	if (rc != TLSGPU_OK) {
		if (f->err == TLSGPU_OK)
			f->err = rc;
	} else
		f->total += fin(b, slot, f);
}

/* Hand the filled slot to the worker, finish the previous one while it runs,
 * and move to the other slot (one slot: run it and finish it in turn). */
static void
pipe_close(tlsgpu_ssl_batch *b, struct pipe *p, int base, finish_fn fin, struct finish_ctx *f)
{
	int prc = TLSGPU_OK;
	if (p->inflight >= 0)
		prc = wait_slot(b, (uint32_t)(base + p->inflight));
	post_job(b, base + (int)p->s);
	if (p->inflight >= 0)
		pipe_finish(b, (uint32_t)p->inflight, prc, fin, f);
	p->inflight = (int)p->s;
	if (b->nslot == 2) {
		p->s ^= 1u;
	} else {
		const int rc = wait_slot(b, (uint32_t)base + p->s);
		p->inflight = -1;
		pipe_finish(b, p->s, rc, fin, f);
	}
}

static void
pipe_drain(tlsgpu_ssl_batch *b, struct pipe *p, int base, finish_fn fin, struct finish_ctx *f)
{
	if (p->inflight >= 0) {
		const int rc = wait_slot(b, (uint32_t)(base + p->inflight));
		pipe_finish(b, (uint32_t)p->inflight, rc, fin, f);
		p->inflight = -1;
	}
}

int
tlsgpu_ssl_batch_read(tlsgpu_ssl_batch *b, const uint32_t *conns, uint32_t n,
    tlsgpu_ssl_deliver_fn deliver, void *arg, int *conn_status)
{
	if (!b || (n && (!conns || !conn_status)))
		return TLSGPU_EINVAL;
	b->t_gather = b->t_open = b->t_deliver = 0;
	struct finish_ctx f = {conns, conn_status, deliver, arg, 0, TLSGPU_OK};
	struct pipe pp = {0, -1};
	uint32_t s = 0;  /* pp.s: the slot being gathered */
	b->g[0] = (struct group){0, 0, 0, 0};
	double tg = now_s();
	for (uint32_t i = 0; i < n; i++) {
		const uint32_t id = conns[i];
		struct conn *c = id < b->cap ? &b->c[id] : NULL;
		b->first[i] = b->g[s].nrec;
		b->count[i] = 0;
		conn_status[i] = TLSGPU_SSL_OK;
		if (!c || !c->attached) {
			conn_status[i] = TLSGPU_SSL_NOT_ATTACHED;
			continue;
		}
		/* the group is full, or cannot take this connection's kept bytes and
		 * what its BIO holds (at least one more record): hand it to the GPU
		 * and gather into the other slot */
		BIO *rb = SSL_get_rbio(c->s);
		const size_t pending = (size_t)BIO_ctrl_pending(rb);
		const size_t want = c->pend_len + (pending > SSL3_RT_MAX_PACKET_SIZE ? pending :
		    SSL3_RT_MAX_PACKET_SIZE);
		if (b->g[s].nrec != 0 && (b->g[s].used >= kGroupBytes ||
		    b->slot_cap - b->g[s].used < want)) {
			b->t_gather += now_s() - tg;
			b->g[s].i1 = i;
			pipe_close(b, &pp, 0, deliver_group, &f);
			s = pp.s;
			b->g[s] = (struct group){i, i, 0, 0};
			tg = now_s();
			b->first[i] = 0;
		}
		uint8_t *w = b->wire + (size_t)s * b->slot_cap;
		tlsgpu_record *recs = b->recs + (size_t)s * b->rec_cap;
		size_t used = b->g[s].used;
		uint32_t nrec = b->g[s].nrec;
		/* 1. gather: the kept partial record, then the BIO's bytes */
		const size_t start = used;
		if (c->pend_len > b->slot_cap - used)
			continue;  /* no room this call: the connection waits for the next */
		memcpy(w + used, c->pend, c->pend_len);
		used += c->pend_len;
		c->pend_len = 0;
		for (int k; used < b->slot_cap &&
		    (k = BIO_read(rb, w + used, (int)(b->slot_cap - used > 1u << 30 ?
		    1u << 30 : b->slot_cap - used))) > 0;)
			used += (size_t)k;
		/* 2. frame (ssl3_get_record's header checks) */
		const uint64_t seq0 = seq_load(c->s->s3->read_sequence);
		size_t p = start;
		while (used - p >= SSL3_RT_HEADER_LENGTH) {
			const uint8_t *h = w + p;
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
			tlsgpu_record *r = &recs[nrec++];
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
				if (!q) {
					f.err = TLSGPU_ENOMEM;
					b->g[s].used = p;
					b->g[s].nrec = nrec;
					n = i + 1;  /* stop gathering: drain what is posted */
					break;
				}
				c->pend = q;
			}
			memcpy(c->pend, w + p, rest);
			c->pend_len = rest;
		}
		b->g[s].used = p;
		b->g[s].nrec = nrec;
	}
	b->t_gather += now_s() - tg;
	b->g[s].i1 = n;  /* a last group without records has nothing to open */
	if (b->g[s].nrec != 0)
		pipe_close(b, &pp, 0, deliver_group, &f);
	pipe_drain(b, &pp, 0, deliver_group, &f);
	return f.err != TLSGPU_OK ? f.err : f.total;
}

/* Hand write slot s's sealed records to their connections' write BIOs with
 * do_ssl3_write's header (s3_pkt.c:662-677, 733).  Returns the records
 * written. */
static int
emit_write_slot(tlsgpu_ssl_batch *b, uint32_t s, struct finish_ctx *f)
{
	const uint32_t *conns = f->conns;
	int *conn_status = f->conn_status;
	const tlsgpu_record *recs = b->w_recs + (size_t)s * b->w_rec_cap;
	const int32_t *status = b->w_status + (size_t)s * b->w_rec_cap;
	const uint32_t *pos = b->w_pos + (size_t)s * b->w_rec_cap;
	uint8_t *out = b->w_out + (size_t)s * b->w_cap;
	int written = 0;
	for (uint32_t r = 0; r < b->wg[s].nrec; r++) {
		const uint32_t i = pos[r];
		if (conn_status[i] != TLSGPU_SSL_OK)
			continue;  /* an earlier record of this connection failed */
		const struct conn *c = &b->c[conns[i]];
		const int32_t st = status[r];
		uint8_t *h = out + recs[r].out_off - SSL3_RT_HEADER_LENGTH;
		const int len = SSL3_RT_HEADER_LENGTH + st;
		if (st < 0) {
			conn_status[i] = TLSGPU_SSL_WRITE_FAILED;
			continue;
		}
		h[0] = SSL3_RT_APPLICATION_DATA;
		h[1] = (uint8_t)(c->s->version >> 8);
		h[2] = (uint8_t)c->s->version;
		h[3] = (uint8_t)(st >> 8);
		h[4] = (uint8_t)st;
		if (BIO_write(SSL_get_wbio(c->s), h, len) != len) {
			conn_status[i] = TLSGPU_SSL_WRITE_FAILED;
			continue;
		}
		written++;
	}
	return written;
}

int
tlsgpu_ssl_batch_write(tlsgpu_ssl_batch *b, const uint32_t *conns, uint32_t n,
    const uint8_t *const *data, const size_t *len, int *conn_status)
{
	if (!b || (n && (!conns || !data || !len || !conn_status)))
		return TLSGPU_EINVAL;
	for (uint32_t i = 0; i < n; i++) {
		const uint32_t id = conns[i];
		conn_status[i] = id < b->cap && b->c[id].wattached ? TLSGPU_SSL_OK :
		    TLSGPU_SSL_NOT_ATTACHED;
	}
	struct finish_ctx f = {conns, conn_status, NULL, NULL, 0, TLSGPU_OK};
	struct pipe pp = {0, -1};
	uint32_t i = 0;
	size_t off = 0;  /* bytes of conns[i]'s data already framed */
	while (i < n) {
		const uint32_t s = pp.s;
		/* frame records (do_ssl3_write: fragments of at most
		 * SSL3_RT_MAX_PLAIN_LENGTH, s3_pkt.c:531-536) into slot s until it is
		 * a group's worth or full; each record takes the connection's next
		 * write sequence number (advanced here, once per record, as
		 * tls1_enc(s, 1) does: t1_enc.c:258-266) */
		uint8_t *in = b->w_in + (size_t)s * b->w_cap;
		tlsgpu_record *recs = b->w_recs + (size_t)s * b->w_rec_cap;
		uint32_t *pos = b->w_pos + (size_t)s * b->w_rec_cap;
		size_t in_used = 0, out_used = 0;
		uint32_t nrec = 0;
		while (i < n && in_used < kGroupBytes) {
			if (conn_status[i] != TLSGPU_SSL_OK || off == len[i]) {
				i++, off = 0;  /* not attached, or done (a zero-length write sends nothing) */
				continue;
			}
			const struct conn *c = &b->c[conns[i]];
			const size_t frag = len[i] - off > SSL3_RT_MAX_PLAIN_LENGTH ?
			    SSL3_RT_MAX_PLAIN_LENGTH : len[i] - off;
			const size_t need = SSL3_RT_HEADER_LENGTH + c->weiv + frag + c->wtag;
			if (in_used + frag > b->w_cap || out_used + need > b->w_cap ||
			    nrec == b->w_rec_cap)
				break;
			memcpy(in + in_used, data[i] + off, frag);
			tlsgpu_record *r = &recs[nrec];
			const uint64_t seq = seq_load(c->s->s3->write_sequence);
			seq_store(c->s->s3->write_sequence, seq + 1);
			r->in_off = in_used;
			r->out_off = out_used + SSL3_RT_HEADER_LENGTH;
			r->seq = seq;
			r->session = b->cap + conns[i];
			r->len_type = TLSGPU_LEN_TYPE(frag, SSL3_RT_APPLICATION_DATA);
			pos[nrec++] = i;
			in_used += frag;
			out_used += need;
			off += frag;
		}
		if (nrec == 0)
			break;  /* nothing framed: every remaining connection is done */
		b->wg[s] = (struct wgroup){nrec, in_used, out_used};
		/* sealed on the worker while the previous group is written out */
		pipe_close(b, &pp, 2, emit_write_slot, &f);
	}
	pipe_drain(b, &pp, 2, emit_write_slot, &f);
	return f.err != TLSGPU_OK ? f.err : f.total;
}
