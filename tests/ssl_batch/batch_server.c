/*
 * batch_server.c — TEST HARNESS for integration/ssl_batch.c: N real TLS 1.2
 * connections of the reference's unmodified libssl (oracle/_ref/libssl_ref.so,
 * LibreSSL 2.4.1 compiled from /root/reference), handshaken over memory BIOs,
 * whose server-side reads go through ONE GPU batch per round instead of one
 * SSL_read per record (VERDICT r05 missing 2).
 *
 *   phase 1  every client SSL_write()s a list of writes (SplitMix64 payloads);
 *            the server reads all connections with tlsgpu_ssl_batch_read and
 *            every connection's delivered bytes must equal what its client
 *            wrote, in order;
 *   phase 2  the clients write again, and the server reads with plain SSL_read
 *            (the reference's CPU record layer): the SSL objects are still
 *            consistent after the batch (read_sequence advanced as tls1_enc
 *            would have);
 *   phase 4  the server writes every connection in one
 *            tlsgpu_ssl_batch_write (records cut, GPU-sealed, framed into the
 *            write BIOs) and every client reads it with SSL_read; phase 5:
 *            the server's own SSL_write after it, read by the clients;
 *   phase 6  every connection's wire cut at an arbitrary byte and fed in
 *            two parts, one batch read after each (partial records kept
 *            across calls);
 *   phase 3  (-t K, after 4-6) one bit of connection K's next record is flipped on the
 *            wire: the batch reports K as bad_record_mac, every other
 *            connection is delivered;
 *   -b       bench: after the checks, R records of L bytes per connection,
 *            timed through the batch (gather + H2D + open + D2H + delivery)
 *            and, on fresh copies of the same wire, through SSL_read on one
 *            CPU thread (the reference path), both as payload GiB/s.
 *
 * The read key of each connection is taken where the record layer hands it
 * to EVP_AEAD_CTX_init (tls1_change_cipher_state_aead, t1_enc.c:444-495),
 * by interposing that one call (the real one runs): a patched record layer
 * would call tlsgpu_ssl_batch_attach there instead.
 *
 * usage: batch_server -p server.pem -c CIPHER -n CONNS [-t K] [-b -r R -l L] [-w BYTES]
 * prints one JSON line; exit status 0 only if every check passed.
 */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include <openssl/bio.h>
#include <openssl/ec.h>
#include <openssl/err.h>
#include <openssl/evp.h>
#include <openssl/ssl.h>

#include "ssl_locl.h"
#include "../../integration/ssl_batch.h"

/* ---- the interposed key hand-off (the real EVP_AEAD_CTX_init runs) ---- */
struct keyrec {
	const void *ctx;
	unsigned char key[32];
	size_t len;
};
static struct keyrec *keys;
static int nkeys, capkeys;

int
EVP_AEAD_CTX_init(EVP_AEAD_CTX *ctx, const EVP_AEAD *aead, const unsigned char *key,
    size_t key_len, size_t tag_len, ENGINE *impl)
{
	static int (*real)(EVP_AEAD_CTX *, const EVP_AEAD *, const unsigned char *, size_t,
	    size_t, ENGINE *);
	if (!real)
		real = (int (*)(EVP_AEAD_CTX *, const EVP_AEAD *, const unsigned char *, size_t,
		    size_t, ENGINE *))dlsym(RTLD_NEXT, "EVP_AEAD_CTX_init");
	if (!real)
		abort();
	int slot = -1;
	for (int i = nkeys - 1; i >= 0 && slot < 0; i--)
		if (keys[i].ctx == ctx)
			slot = i;
	if (slot < 0) {
		if (nkeys == capkeys) {
			capkeys = capkeys ? 2 * capkeys : 256;
			keys = realloc(keys, sizeof(*keys) * capkeys);
		}
		slot = nkeys++;
	}
	keys[slot].ctx = ctx;
	keys[slot].len = key_len <= 32 ? key_len : 0;
	memcpy(keys[slot].key, key, keys[slot].len);
	return real(ctx, aead, key, key_len, tag_len, impl);
}

static const struct keyrec *
key_of(const void *ctx)
{
	for (int i = nkeys - 1; i >= 0; i--)
		if (keys[i].ctx == ctx)
			return &keys[i];
	return NULL;
}

static void
fill(unsigned char *p, long n, uint64_t key)
{
	uint64_t x = key * 0x9E3779B97F4A7C15ull;
	for (long i = 0; i < n; i += 8) {
		uint64_t z = (x += 0x9E3779B97F4A7C15ull);
		z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
		z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
		z ^= z >> 31;
		for (int b = 0; b < 8 && i + b < n; b++)
			p[i + b] = (unsigned char)(z >> (8 * b));
	}
}

static long
pump(BIO *from, BIO *to)
{
	unsigned char buf[16384];
	long moved = 0;
	int n;
	while ((n = BIO_read(from, buf, sizeof(buf))) > 0) {
		if (BIO_write(to, buf, n) != n)
			return -1;
		moved += n;
	}
	return moved;
}

static double
now(void)
{
	struct timespec ts;
	clock_gettime(CLOCK_MONOTONIC, &ts);
	return ts.tv_sec + ts.tv_nsec * 1e-9;
}

struct pair {
	SSL *c, *s;
	BIO *c_in, *c_out, *s_in, *s_out;
	unsigned char *got;   /* bytes the server delivered this phase */
	long got_len, got_cap;
};

static void
on_deliver(void *arg, uint32_t conn, SSL *s, const uint8_t *data, size_t len)
{
	struct pair *P = &((struct pair *)arg)[conn];
	(void)s;
	if (P->got_len + (long)len > P->got_cap) {
		P->got_cap = 2 * (P->got_cap + (long)len);
		P->got = realloc(P->got, P->got_cap);
	}
	memcpy(P->got + P->got_len, data, len);
	P->got_len += (long)len;
}

static int
want_io(SSL *s, int rc)
{
	int e = SSL_get_error(s, rc);
	return e == SSL_ERROR_WANT_READ || e == SSL_ERROR_WANT_WRITE;
}

static int
handshake(struct pair *P)
{
	int c_done = 0, s_done = 0;
	for (int it = 0; it < 1000 && !(c_done && s_done); it++) {
		if (!c_done) {
			int rc = SSL_do_handshake(P->c);
			if (rc == 1)
				c_done = 1;
			else if (!want_io(P->c, rc))
				return 0;
		}
		if (pump(P->c_out, P->s_in) < 0)
			return 0;
		if (!s_done) {
			int rc = SSL_do_handshake(P->s);
			if (rc == 1)
				s_done = 1;
			else if (!want_io(P->s, rc))
				return 0;
		}
		if (pump(P->s_out, P->c_in) < 0)
			return 0;
	}
	pump(P->c_out, P->s_in);
	pump(P->s_out, P->c_in);
	return c_done && s_done;
}

/* the writes of connection i in phase ph: lengths over the record edges */
static const long lens[] = {1, 17, 1400, 16384, 16385, 40000, 5, 4096};
#define NLENS ((int)(sizeof(lens) / sizeof(lens[0])))

static long client_writes_to(struct pair *P, int i, int ph, unsigned char **exp, int pump_it);

static long
client_writes(struct pair *P, int i, int ph, unsigned char **exp)
{
	return client_writes_to(P, i, ph, exp, 1);
}

/* the client's writes; pump_it = 0 leaves the wire in the client's out BIO */
static long
client_writes_to(struct pair *P, int i, int ph, unsigned char **exp, int pump_it)
{
	long total = 0, off = 0;
	for (int k = 0; k < NLENS; k++)
		total += lens[(k + i) % NLENS];
	*exp = malloc(total);
	for (int k = 0; k < NLENS; k++) {
		const long n = lens[(k + i) % NLENS];
		fill(*exp + off, n, ((uint64_t)ph << 48) | ((uint64_t)i << 16) | (uint64_t)k);
		if (SSL_write(P->c, *exp + off, (int)n) != n)
			return -1;
		off += n;
	}
	if (pump_it && pump(P->c_out, P->s_in) < 0)
		return -1;
	return total;
}

int
main(int argc, char **argv)
{
	const char *pem = NULL, *cipher = "ECDHE-RSA-AES128-GCM-SHA256";
	int nconn = 8, tamper = -1, bench = 0, brec = 8, blen = 16384, o;
	size_t wire_opt = 0;
	while ((o = getopt(argc, argv, "p:c:n:t:br:l:w:")) != -1) {
		switch (o) {
		case 'p': pem = optarg; break;
		case 'c': cipher = optarg; break;
		case 'n': nconn = atoi(optarg); break;
		case 't': tamper = atoi(optarg); break;
		case 'b': bench = 1; break;
		case 'r': brec = atoi(optarg); break;
		case 'l': blen = atoi(optarg); break;
		case 'w': wire_opt = (size_t)atol(optarg); break;
		default: return 2;
		}
	}
	if (!pem || nconn < 1) {
		fprintf(stderr, "usage: %s -p server.pem -c cipher -n conns [-t K] [-b -r R -l L] "
		    "[-w WIRE_BYTES]\n",
		    argv[0]);
		return 2;
	}
	SSL_library_init();
	SSL_load_error_strings();
	SSL_CTX *s_ctx = SSL_CTX_new(TLSv1_2_server_method());
	SSL_CTX *c_ctx = SSL_CTX_new(TLSv1_2_client_method());
	EC_KEY *ecdh = EC_KEY_new_by_curve_name(NID_X9_62_prime256v1);
	if (!s_ctx || !c_ctx || !ecdh || !SSL_CTX_set_tmp_ecdh(s_ctx, ecdh) ||
	    SSL_CTX_use_certificate_file(s_ctx, pem, SSL_FILETYPE_PEM) != 1 ||
	    SSL_CTX_use_PrivateKey_file(s_ctx, pem, SSL_FILETYPE_PEM) != 1 ||
	    !SSL_CTX_set_cipher_list(c_ctx, cipher) || !SSL_CTX_set_cipher_list(s_ctx, cipher)) {
		ERR_print_errors_fp(stderr);
		return 1;
	}
	EC_KEY_free(ecdh);
	SSL_CTX_set_verify(c_ctx, SSL_VERIFY_NONE, NULL);
	/* session resumption keeps N handshakes cheap (one full handshake) */
	SSL_CTX_set_session_cache_mode(s_ctx, SSL_SESS_CACHE_SERVER);
	SSL_CTX_set_session_id_context(s_ctx, (const unsigned char *)"tg", 2);
	struct pair *P = calloc(nconn, sizeof(*P));
	SSL_SESSION *sess = NULL;
	for (int i = 0; i < nconn; i++) {
		P[i].c = SSL_new(c_ctx);
		P[i].s = SSL_new(s_ctx);
		P[i].c_in = BIO_new(BIO_s_mem());
		P[i].c_out = BIO_new(BIO_s_mem());
		P[i].s_in = BIO_new(BIO_s_mem());
		P[i].s_out = BIO_new(BIO_s_mem());
		BIO_set_mem_eof_return(P[i].c_in, -1);
		BIO_set_mem_eof_return(P[i].s_in, -1);
		SSL_set_bio(P[i].c, P[i].c_in, P[i].c_out);
		SSL_set_bio(P[i].s, P[i].s_in, P[i].s_out);
		SSL_set_connect_state(P[i].c);
		SSL_set_accept_state(P[i].s);
		if (sess)
			SSL_set_session(P[i].c, sess);
		if (!handshake(&P[i])) {
			fprintf(stderr, "handshake %d failed\n", i);
			ERR_print_errors_fp(stderr);
			return 1;
		}
		if (!sess)
			sess = SSL_get1_session(P[i].c);
	}
	/* attach every server connection's read key (the consumer's one hook) */
	tlsgpu_ssl_batch *B = NULL;
	size_t wire = (size_t)nconn * 128 * 1024 + (bench ? (size_t)nconn * brec * (blen + 64) : 0);
	if (wire < (4u << 20))
		wire = 4u << 20;
	if (wire_opt)  /* -w: a small pinned buffer, so one read runs many pipeline groups */
		wire = wire_opt;
	if (tlsgpu_ssl_batch_create(0, (uint32_t)nconn, wire, &B) != TLSGPU_OK) {
		fprintf(stderr, "tlsgpu_ssl_batch_create failed\n");
		return 1;
	}
	for (int i = 0; i < nconn; i++) {
		const struct keyrec *k = key_of(&P[i].s->aead_read_ctx->ctx);
		if (!k || tlsgpu_ssl_batch_attach(B, (uint32_t)i, P[i].s, k->key, k->len) != TLSGPU_OK) {
			fprintf(stderr, "attach %d failed\n", i);
			return 1;
		}
	}
	uint32_t *ids = malloc(sizeof(uint32_t) * nconn);
	int *st = malloc(sizeof(int) * nconn);
	for (int i = 0; i < nconn; i++)
		ids[i] = (uint32_t)i;
	int ok = 1;
	long records1 = 0;
	/* phase 1: one batch read over every connection */
	unsigned char **exp = calloc(nconn, sizeof(*exp));
	long *explen = calloc(nconn, sizeof(long));
	for (int i = 0; i < nconn; i++)
		if ((explen[i] = client_writes(&P[i], i, 1, &exp[i])) < 0)
			return 1;
	int r = tlsgpu_ssl_batch_read(B, ids, (uint32_t)nconn, on_deliver, P, st);
	records1 = r;
	for (int i = 0; i < nconn && ok; i++) {
		if (r < 0 || st[i] != TLSGPU_SSL_OK || P[i].got_len != explen[i] ||
		    memcmp(P[i].got, exp[i], explen[i]) != 0) {
			fprintf(stderr, "phase 1: connection %d: rc %d status %d got %ld of %ld\n", i, r,
			    st[i], P[i].got_len, explen[i]);
			ok = 0;
		}
		P[i].got_len = 0;
		free(exp[i]);
	}
	/* phase 2: the same SSL objects through the reference's SSL_read */
	long records2 = 0;
	for (int i = 0; i < nconn && ok; i++) {
		if ((explen[i] = client_writes(&P[i], i, 2, &exp[i])) < 0)
			return 1;
		unsigned char *buf = malloc(explen[i]);
		long got = 0;
		while (got < explen[i]) {
			int rc = SSL_read(P[i].s, buf + got, (int)(explen[i] - got));
			if (rc <= 0) {
				fprintf(stderr, "phase 2: SSL_read on connection %d returned %d\n", i, rc);
				ERR_print_errors_fp(stderr);
				ok = 0;
				break;
			}
			got += rc;
			records2++;
		}
		if (ok && memcmp(buf, exp[i], explen[i]) != 0) {
			fprintf(stderr, "phase 2: connection %d payload mismatch\n", i);
			ok = 0;
		}
		free(buf);
		free(exp[i]);
	}
	/* phase 4: the server writes every connection in one call
	 * (tlsgpu_ssl_batch_write: records cut, sealed on the GPU, framed into
	 * each write BIO); every client reads with the reference's SSL_read.
	 * Phase 5: the server's own SSL_write on the same SSL objects, read by
	 * the clients (write_sequence stayed consistent). */
	long records4 = -1;
	int write_ok = -1;
	if (ok) {
		write_ok = 1;
		for (int i = 0; i < nconn; i++) {
			const struct keyrec *k = key_of(&P[i].s->aead_write_ctx->ctx);
			if (!k || tlsgpu_ssl_batch_attach_write(B, (uint32_t)i, P[i].s, k->key,
			    k->len) != TLSGPU_OK) {
				fprintf(stderr, "attach_write %d failed\n", i);
				return 1;
			}
		}
		const uint8_t **wd = calloc(nconn, sizeof(*wd));
		size_t *wl = calloc(nconn, sizeof(size_t));
		int *wst = calloc(nconn, sizeof(int));
		for (int i = 0; i < nconn; i++) {
			/* 0 B, single records, the 16 KiB edges, multi-record writes */
			wl[i] = i % 9 == 4 ? 0 : (size_t)lens[i % NLENS] * (1 + i % 3) + (size_t)(i % 5);
			unsigned char *d = malloc(wl[i] + 1);
			fill(d, (long)wl[i], ((uint64_t)4 << 48) | (uint64_t)i);
			wd[i] = d;
		}
		records4 = tlsgpu_ssl_batch_write(B, ids, (uint32_t)nconn, wd, wl, wst);
		for (int i = 0; i < nconn && write_ok; i++) {
			if (records4 < 0 || wst[i] != TLSGPU_SSL_OK || pump(P[i].s_out, P[i].c_in) < 0) {
				fprintf(stderr, "phase 4: connection %d: rc %ld status %d\n", i, records4, wst[i]);
				write_ok = 0;
				break;
			}
			unsigned char *buf = malloc(wl[i] + 1);
			size_t got = 0;
			while (got < wl[i]) {
				int rc = SSL_read(P[i].c, buf + got, (int)(wl[i] - got));
				if (rc <= 0) {
					fprintf(stderr, "phase 4: client %d SSL_read returned %d after %zu of %zu\n",
					    i, rc, got, wl[i]);
					ERR_print_errors_fp(stderr);
					write_ok = 0;
					break;
				}
				got += (size_t)rc;
			}
			if (write_ok && memcmp(buf, wd[i], wl[i]) != 0) {
				fprintf(stderr, "phase 4: client %d payload mismatch\n", i);
				write_ok = 0;
			}
			free(buf);
		}
		for (int i = 0; i < nconn && write_ok; i++) {  /* phase 5 */
			unsigned char msg[1400], back[1400];
			fill(msg, sizeof(msg), ((uint64_t)5 << 48) | (uint64_t)i);
			int got = 0, rc = 0;
			if (SSL_write(P[i].s, msg, sizeof(msg)) != (int)sizeof(msg) ||
			    pump(P[i].s_out, P[i].c_in) < 0)
				write_ok = 0;
			while (write_ok && got < (int)sizeof(msg) &&
			    (rc = SSL_read(P[i].c, back + got, (int)sizeof(msg) - got)) > 0)
				got += rc;
			if (!write_ok || got != (int)sizeof(msg) || memcmp(back, msg, sizeof(msg)) != 0) {
				fprintf(stderr, "phase 5: connection %d: SSL_write / client SSL_read got %d (rc %d)\n",
				    i, got, rc);
				ERR_print_errors_fp(stderr);
				write_ok = 0;
			}
		}
		for (int i = 0; i < nconn; i++)
			free((void *)wd[i]);
		free(wd);
		free(wl);
		free(wst);
		ok = ok && write_ok;
	}
	/* phase 6: every connection's wire cut at an arbitrary byte (inside a
	 * header, a fragment or a tag) and fed in two parts, one batch read
	 * after each: the partial record kept by the first read completes in
	 * the second, and the bytes delivered over both equal the writes */
	int split_ok = -1;
	if (ok) {
		split_ok = 1;
		unsigned char **rest = calloc(nconn, sizeof(*rest));
		long *rest_len = calloc(nconn, sizeof(long));
		for (int i = 0; i < nconn; i++) {
			if ((explen[i] = client_writes_to(&P[i], i, 6, &exp[i], 0)) < 0)
				return 1;
			long wl = (long)BIO_ctrl_pending(P[i].c_out);
			unsigned char *w = malloc(wl + 1);
			if (BIO_read(P[i].c_out, w, (int)wl) != wl)
				return 1;
			const long cut = (long)(((uint64_t)i * 7919u + 13u) % (uint64_t)(wl + 1));
			BIO_write(P[i].s_in, w, (int)cut);
			rest_len[i] = wl - cut;
			rest[i] = malloc(rest_len[i] + 1);
			memcpy(rest[i], w + cut, rest_len[i]);
			free(w);
		}
		int r1 = tlsgpu_ssl_batch_read(B, ids, (uint32_t)nconn, on_deliver, P, st);
		for (int i = 0; i < nconn && r1 >= 0; i++) {
			if (st[i] != TLSGPU_SSL_OK)
				r1 = -1000 - i;
			BIO_write(P[i].s_in, rest[i], (int)rest_len[i]);
		}
		int r2 = r1 < 0 ? -1 : tlsgpu_ssl_batch_read(B, ids, (uint32_t)nconn, on_deliver, P, st);
		for (int i = 0; i < nconn; i++) {
			if (r1 < 0 || r2 < 0 || st[i] != TLSGPU_SSL_OK || P[i].got_len != explen[i] ||
			    memcmp(P[i].got, exp[i], explen[i]) != 0) {
				if (split_ok)
					fprintf(stderr, "phase 6: connection %d: rc %d / %d status %d got %ld of %ld\n",
					    i, r1, r2, st[i], P[i].got_len, explen[i]);
				split_ok = 0;
			}
			P[i].got_len = 0;
			free(exp[i]);
			free(rest[i]);
		}
		free(rest);
		free(rest_len);
		ok = ok && split_ok;
	}
	/* phase 3: a flipped bit on connection `tamper` */
	int tamper_ok = -1;
	if (ok && tamper >= 0 && tamper < nconn) {
		for (int i = 0; i < nconn; i++) {
			if (i != tamper) {
				if ((explen[i] = client_writes(&P[i], i, 3, &exp[i])) < 0)
					return 1;
				continue;
			}
			unsigned char msg[1400];
			fill(msg, sizeof(msg), 3);
			if (SSL_write(P[i].c, msg, sizeof(msg)) != (int)sizeof(msg))
				return 1;
			unsigned char w[2048];
			int n = BIO_read(P[i].c_out, w, sizeof(w));
			w[n - 20] ^= 0x10;  /* inside the ciphertext */
			BIO_write(P[i].s_in, w, n);
			explen[i] = 0;
			exp[i] = NULL;
		}
		r = tlsgpu_ssl_batch_read(B, ids, (uint32_t)nconn, on_deliver, P, st);
		tamper_ok = r >= 0;
		for (int i = 0; i < nconn; i++) {
			const int want = i == tamper ? TLSGPU_SSL_BAD_RECORD_MAC : TLSGPU_SSL_OK;
			if (st[i] != want || P[i].got_len != explen[i] ||
			    (explen[i] && memcmp(P[i].got, exp[i], explen[i]) != 0)) {
				fprintf(stderr, "phase 3: connection %d status %d (want %d) got %ld of %ld\n",
				    i, st[i], want, P[i].got_len, explen[i]);
				tamper_ok = 0;
			}
			P[i].got_len = 0;
			free(exp[i]);
		}
		ok = ok && tamper_ok;
	}
	printf("{\"cipher\": \"%s\", \"conns\": %d, \"batch_records\": %ld, "
	    "\"ssl_read_records_after\": %ld, \"batch_write_records\": %ld, \"write_checked\": %d, "
	    "\"split_checked\": %d, \"tamper_checked\": %d", SSL_get_cipher_name(P[0].c),
	    nconn, records1, records2, records4, write_ok, split_ok, tamper_ok);
	/* bench: R records of L bytes per connection (fresh connections' state is
	 * not needed: the server reads the same wire twice, from two copies) */
	if (ok && bench) {
		long bytes = 0;
		unsigned char *msg = malloc(blen);
		BIO **copy = calloc(nconn, sizeof(BIO *));
		for (int i = 0; i < nconn; i++) {
			if (i == tamper)
				continue;
			for (int k = 0; k < brec; k++) {
				fill(msg, blen, ((uint64_t)9 << 48) | ((uint64_t)i << 16) | (uint64_t)k);
				if (SSL_write(P[i].c, msg, blen) != blen)
					return 1;
				bytes += blen;
			}
			/* the wire twice: into the server BIO and a spare copy */
			copy[i] = BIO_new(BIO_s_mem());
			unsigned char buf[16384];
			int n;
			while ((n = BIO_read(P[i].c_out, buf, sizeof(buf))) > 0) {
				BIO_write(P[i].s_in, buf, n);
				BIO_write(copy[i], buf, n);
			}
		}
		/* snapshot each server's read sequence, to replay the CPU pass */
		unsigned char (*seq)[8] = calloc(nconn, 8);
		for (int i = 0; i < nconn; i++)
			memcpy(seq[i], P[i].s->s3->read_sequence, 8);
		/* delivery buffers sized and touched before the clock starts (the
		 * SSL_read pass reads into one reused buffer: no first-touch faults
		 * on either side) */
		for (int i = 0; i < nconn; i++) {
			const long want = (long)brec * blen;
			if (P[i].got_cap < want) {
				P[i].got = realloc(P[i].got, want);
				P[i].got_cap = want;
			}
			memset(P[i].got, 0, want);
			P[i].got_len = 0;
		}
		uint32_t *bids = malloc(sizeof(uint32_t) * nconn);
		int nb = 0;
		for (int i = 0; i < nconn; i++)
			if (i != tamper)
				bids[nb++] = (uint32_t)i;
		double t0 = now();
		r = tlsgpu_ssl_batch_read(B, bids, (uint32_t)nb, on_deliver, P, st);
		double t1 = now();
		double tg, to, td;
		tlsgpu_ssl_batch_times(B, &tg, &to, &td);
		long gbytes = 0;
		for (int i = 0; i < nb; i++) {
			if (st[i] != TLSGPU_SSL_OK)
				ok = 0;
			gbytes += P[bids[i]].got_len;
			P[bids[i]].got_len = 0;
		}
		/* the same wire through SSL_read (reference CPU path, one thread) */
		for (int i = 0; i < nconn; i++) {
			if (i == tamper)
				continue;
			memcpy(P[i].s->s3->read_sequence, seq[i], 8);
			SSL_set_bio(P[i].s, copy[i], SSL_get_wbio(P[i].s));
		}
		long cbytes = 0;
		double t2 = now();
		for (int i = 0; i < nconn; i++) {
			if (i == tamper)
				continue;
			int rc;
			while ((rc = SSL_read(P[i].s, msg, blen)) > 0)
				cbytes += rc;
		}
		double t3 = now();
		if (gbytes != bytes || cbytes != bytes)
			ok = 0;
		printf(", \"bench\": {\"records_per_conn\": %d, \"record_len\": %d, \"payload_bytes\": %ld, "
		    "\"batch_records\": %d, \"batch_s\": %.6f, \"batch_GiBps\": %.3f, "
		    "\"batch_phases_s\": {\"gather\": %.6f, \"gpu_open_host\": %.6f, \"deliver\": %.6f}, "
		    "\"gpu_open_host_GiBps\": %.3f, "
		    "\"ssl_read_cpu1_s\": %.6f, \"ssl_read_cpu1_GiBps\": %.3f, "
		    "\"timing\": \"wall clock: tlsgpu_ssl_batch_read (BIO gather + pinned H2D + open + "
		    "D2H + delivery copy) vs SSL_read over the same wire on one thread\"}",
		    brec, blen, bytes, r, t1 - t0, bytes / (t1 - t0) / 1073741824.0, tg, to, td,
		    bytes / to / 1073741824.0, t3 - t2,
		    cbytes / (t3 - t2) / 1073741824.0);
		/* write bench: R x L bytes to every connection in one
		 * tlsgpu_ssl_batch_write, against R SSL_write calls per connection on
		 * one thread (the reference path); the write BIOs are emptied first
		 * and in between, so both sides append to empty memory BIOs */
		const size_t wlen = (size_t)brec * blen;
		unsigned char *big = malloc(wlen);
		fill(big, (long)wlen, 6);
		const uint8_t **wd = malloc(sizeof(*wd) * nconn);
		size_t *wl = malloc(sizeof(size_t) * nconn);
		int *wst = malloc(sizeof(int) * nconn);
		for (int i = 0; i < nconn; i++) {
			wd[i] = big;
			wl[i] = wlen;
			/* grow and touch each write BIO's buffer to the wire size first,
			 * so neither pass pays the memory BIO's growth */
			const size_t grow = wlen + (size_t)brec * 64;
			for (size_t w = 0; w < grow; w += (size_t)blen)
				BIO_write(P[i].s_out, big, (int)(grow - w < (size_t)blen ? grow - w : (size_t)blen));
			(void)BIO_reset(P[i].s_out);
		}
		double w0 = now();
		const int wr = tlsgpu_ssl_batch_write(B, bids, (uint32_t)nb, wd, wl, wst);
		double w1 = now();
		long wbytes = 0;
		for (int i = 0; i < nb; i++) {
			if (wst[i] != TLSGPU_SSL_OK)
				ok = 0;
			wbytes += (long)BIO_ctrl_pending(P[bids[i]].s_out);
			(void)BIO_reset(P[bids[i]].s_out);
		}
		double w2 = now();
		long cw = 0;
		for (int i = 0; i < nb; i++)
			for (int k = 0; k < brec; k++)
				cw += SSL_write(P[bids[i]].s, big + (size_t)k * blen, blen) == blen ? blen : 0;
		double w3 = now();
		if (wr != nb * brec || cw != bytes)
			ok = 0;
		printf(", \"write_bench\": {\"batch_records\": %d, \"wire_bytes\": %ld, \"batch_s\": %.6f, "
		    "\"batch_GiBps\": %.3f, \"ssl_write_cpu1_s\": %.6f, \"ssl_write_cpu1_GiBps\": %.3f, "
		    "\"timing\": \"wall clock: tlsgpu_ssl_batch_write (copy in + pinned H2D + seal + D2H + "
		    "header + BIO_write) vs SSL_write on one thread, payload GiB/s\"}",
		    wr, wbytes, w1 - w0, bytes / (w1 - w0) / 1073741824.0, w3 - w2,
		    bytes / (w3 - w2) / 1073741824.0);
		free(big);
		free(wd);
		free(wl);
		free(wst);
		free(msg);
	}
	printf(", \"ok\": %d}\n", ok);
	tlsgpu_ssl_batch_destroy(B);
	return ok ? 0 : 1;
}
