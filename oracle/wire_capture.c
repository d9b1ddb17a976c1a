/*
 * wire_capture.c — TEST INFRASTRUCTURE ONLY (fixture generator).
 *
 * Records what the reference's own, unmodified TLS 1.2 record layer puts on
 * the wire, so the device framing (tlsgpu_open_wire / tlsgpu_seal_wire and the
 * in-kernel nonce/AAD of the batch path) is pinned to bytes made by
 * ssl/s3_pkt.c:560-762 (do_ssl3_write) and ssl/t1_enc.c:832-975 (tls1_enc),
 * not to a restatement of them.
 *
 * A client and a server SSL object of oracle/_ref/libssl_ref.so (LibreSSL
 * 2.4.1 compiled from /root/reference) handshake through memory BIOs.  After
 * the handshake the harness reads, per direction, the record layer's own AEAD
 * state — the write side's SSL_AEAD_CTX (ssl/ssl_locl.h:527-543: fixed_nonce,
 * fixed_nonce_len, xor_fixed_nonce, variable_nonce_in_record, tag_len) and
 * s3->write_sequence (ssl3.h:368) — plus the raw AEAD key, which the record
 * layer hands to EVP_AEAD_CTX_init (tls1_change_cipher_state_aead,
 * t1_enc.c:444-495) and which this program records by interposing that one
 * call (the real one runs, from libssl_ref.so).  Then the writer SSL_write()s a
 * list of application writes (deterministic SplitMix64 payloads, seed
 * (dir << 32) | k), every byte do_ssl3_write emits is captured from the memory
 * BIO, and the peer SSL_read()s it back (so the reference itself accepted every
 * captured record).
 *
 * usage: wire_capture -p server.pem -c CIPHER -o PREFIX
 * writes PREFIX.c2s.bin / PREFIX.s2c.bin (the raw wire of each direction) and
 * prints one JSON line of metadata; exit status 0 only if everything
 * round-tripped.
 */
#define _GNU_SOURCE	/* RTLD_NEXT */
#include <dlfcn.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <openssl/bio.h>
#include <openssl/ec.h>
#include <openssl/err.h>
#include <openssl/evp.h>
#include <openssl/ssl.h>

#include "ssl_locl.h"	/* struct ssl_aead_ctx_st, read from the reference tree */

/* ---- the one interposed call: remember each AEAD context's raw key ---- */
struct keyrec {
	const void *ctx;
	unsigned char key[64];
	size_t len;
};
static struct keyrec keys[64];
static int nkeys;

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
	for (int i = 0; i < nkeys; i++)
		if (keys[i].ctx == ctx)
			slot = i;
	if (slot < 0 && nkeys < 64)
		slot = nkeys++;
	if (slot >= 0 && key_len <= sizeof(keys[0].key)) {
		keys[slot].ctx = ctx;
		memcpy(keys[slot].key, key, key_len);
		keys[slot].len = key_len;
	}
	return real(ctx, aead, key, key_len, tag_len, impl);
}

static const struct keyrec *
key_of(const void *ctx)
{
	for (int i = 0; i < nkeys; i++)
		if (keys[i].ctx == ctx)
			return &keys[i];
	return NULL;
}

/* deterministic payload: SplitMix64, the generator of ssl_loopback.c */
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

/* move everything pending in `from` into `to`; optionally append it to cap */
static long
pump(BIO *from, BIO *to, unsigned char **cap, long *caplen, long *capcap)
{
	unsigned char buf[8192];
	long moved = 0;
	int n;
	while ((n = BIO_read(from, buf, sizeof(buf))) > 0) {
		if (BIO_write(to, buf, n) != n)
			return -1;
		if (cap) {
			if (*caplen + n > *capcap) {
				*capcap = 2 * (*capcap + n);
				*cap = realloc(*cap, *capcap);
			}
			memcpy(*cap + *caplen, buf, n);
			*caplen += n;
		}
		moved += n;
	}
	return moved;
}

static void
hex(FILE *f, const unsigned char *p, size_t n)
{
	for (size_t i = 0; i < n; i++)
		fprintf(f, "%02x", p[i]);
}

static int
want_io(SSL *s, int rc)
{
	int e = SSL_get_error(s, rc);
	return e == SSL_ERROR_WANT_READ || e == SSL_ERROR_WANT_WRITE;
}

/* application writes of the client (c2s) and of the server (s2c) */
static const long c2s_lens[] = {1, 2, 15, 16, 17, 63, 64, 255, 256, 1000, 1023, 1024, 1400,
    4096, 16383, 16384, 16385, 40000};
static const long s2c_lens[] = {5, 1400, 16384, 20000};

/* One direction: writer -> reader.  Prints the direction's JSON object. */
static int
direction(const char *name, int dir, SSL *w, BIO *w_out, SSL *r, BIO *r_in, const long *lens,
    int nlens, const char *path, int first)
{
	SSL_AEAD_CTX *a = w->aead_write_ctx;
	SSL_AEAD_CTX *ra = r->aead_read_ctx;
	if (!a || !ra) {
		fprintf(stderr, "%s: no AEAD record state (not an AEAD suite?)\n", name);
		return 0;
	}
	const struct keyrec *k = key_of(&a->ctx), *rk = key_of(&ra->ctx);
	if (!k || !rk || k->len != rk->len || memcmp(k->key, rk->key, k->len) != 0) {
		fprintf(stderr, "%s: writer and reader keys not found or different\n", name);
		return 0;
	}
	unsigned char seq[SSL3_SEQUENCE_SIZE];
	memcpy(seq, w->s3->write_sequence, sizeof(seq));
	if (memcmp(seq, r->s3->read_sequence, sizeof(seq)) != 0) {
		fprintf(stderr, "%s: writer and reader sequence numbers differ\n", name);
		return 0;
	}
	unsigned char *cap = NULL, *buf = NULL, *rbuf = NULL;
	long caplen = 0, capcap = 0;
	printf("%s{\"dir\": \"%s\", \"key\": \"", first ? "" : ", ", name);
	hex(stdout, k->key, k->len);
	printf("\", \"fixed_nonce\": \"");
	hex(stdout, a->fixed_nonce, a->fixed_nonce_len);
	printf("\", \"variable_nonce_len\": %u, \"xor_fixed_nonce\": %u, "
	    "\"variable_nonce_in_record\": %d, \"tag_len\": %u, \"version\": %d, \"start_seq\": \"",
	    a->variable_nonce_len, a->xor_fixed_nonce, a->variable_nonce_in_record, a->tag_len,
	    w->version);
	hex(stdout, seq, sizeof(seq));
	printf("\", \"writes\": [");
	for (int i = 0; i < nlens; i++) {
		const long n = lens[i];
		const uint64_t seed = ((uint64_t)dir << 32) | (uint64_t)i;
		buf = realloc(buf, n);
		rbuf = realloc(rbuf, n);
		fill(buf, n, seed);
		const long off = caplen;
		int rc = SSL_write(w, buf, (int)n);
		if (rc != n) {
			fprintf(stderr, "%s: SSL_write(%ld) returned %d\n", name, n, rc);
			return 0;
		}
		if (pump(w_out, r_in, &cap, &caplen, &capcap) < 0)
			return 0;
		long got = 0;
		while (got < n) {
			rc = SSL_read(r, rbuf + got, (int)(n - got));
			if (rc <= 0) {
				fprintf(stderr, "%s: SSL_read returned %d\n", name, rc);
				return 0;
			}
			got += rc;
		}
		if (memcmp(buf, rbuf, n) != 0) {
			fprintf(stderr, "%s: payload mismatch on write %d\n", name, i);
			return 0;
		}
		printf("%s{\"len\": %ld, \"seed\": %llu, \"wire_off\": %ld, \"wire_len\": %ld}",
		    i ? ", " : "", n, (unsigned long long)seed, off, caplen - off);
	}
	printf("], \"wire_bytes\": %ld, \"end_seq\": \"", caplen);
	hex(stdout, w->s3->write_sequence, SSL3_SEQUENCE_SIZE);
	printf("\"}");
	FILE *f = fopen(path, "wb");
	if (!f || fwrite(cap, 1, caplen, f) != (size_t)caplen || fclose(f) != 0) {
		fprintf(stderr, "cannot write %s\n", path);
		return 0;
	}
	free(cap);
	free(buf);
	free(rbuf);
	return 1;
}

int
main(int argc, char **argv)
{
	const char *pem = NULL, *cipher = "ECDHE-RSA-AES128-GCM-SHA256", *prefix = NULL;
	int o;
	while ((o = getopt(argc, argv, "p:c:o:")) != -1) {
		switch (o) {
		case 'p': pem = optarg; break;
		case 'c': cipher = optarg; break;
		case 'o': prefix = optarg; break;
		default:
			fprintf(stderr, "usage: %s -p server.pem -c cipher -o prefix\n", argv[0]);
			return 2;
		}
	}
	if (!pem || !prefix) {
		fprintf(stderr, "usage: %s -p server.pem -c cipher -o prefix\n", argv[0]);
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
		fprintf(stderr, "context setup failed\n");
		ERR_print_errors_fp(stderr);
		return 1;
	}
	EC_KEY_free(ecdh);
	SSL_CTX_set_verify(c_ctx, SSL_VERIFY_NONE, NULL);
	SSL *c = SSL_new(c_ctx), *s = SSL_new(s_ctx);
	BIO *c_in = BIO_new(BIO_s_mem()), *c_out = BIO_new(BIO_s_mem());
	BIO *s_in = BIO_new(BIO_s_mem()), *s_out = BIO_new(BIO_s_mem());
	if (!c || !s || !c_in || !c_out || !s_in || !s_out)
		return 1;
	BIO_set_mem_eof_return(c_in, -1);	/* empty = retry, not EOF */
	BIO_set_mem_eof_return(s_in, -1);
	SSL_set_bio(c, c_in, c_out);
	SSL_set_bio(s, s_in, s_out);
	SSL_set_connect_state(c);
	SSL_set_accept_state(s);
	int c_done = 0, s_done = 0;
	for (int it = 0; it < 1000 && !(c_done && s_done); it++) {
		if (!c_done) {
			int rc = SSL_do_handshake(c);
			if (rc == 1)
				c_done = 1;
			else if (!want_io(c, rc))
				break;
		}
		if (pump(c_out, s_in, NULL, NULL, NULL) < 0)
			break;
		if (!s_done) {
			int rc = SSL_do_handshake(s);
			if (rc == 1)
				s_done = 1;
			else if (!want_io(s, rc))
				break;
		}
		if (pump(s_out, c_in, NULL, NULL, NULL) < 0)
			break;
	}
	if (!(c_done && s_done)) {
		fprintf(stderr, "handshake did not finish\n");
		ERR_print_errors_fp(stderr);
		return 1;
	}
	/* drain anything the last handshake step left in flight */
	pump(c_out, s_in, NULL, NULL, NULL);
	pump(s_out, c_in, NULL, NULL, NULL);
	char p1[4096], p2[4096];
	snprintf(p1, sizeof(p1), "%s.c2s.bin", prefix);
	snprintf(p2, sizeof(p2), "%s.s2c.bin", prefix);
	printf("{\"cipher\": \"%s\", \"directions\": [", SSL_get_cipher_name(c));
	int ok = direction("c2s", 1, c, c_out, s, s_in, c2s_lens,
	    (int)(sizeof(c2s_lens) / sizeof(c2s_lens[0])), p1, 1);
	ok = ok && direction("s2c", 2, s, s_out, c, c_in, s2c_lens,
	    (int)(sizeof(s2c_lens) / sizeof(s2c_lens[0])), p2, 0);
	printf("]}\n");
	SSL_free(c);
	SSL_free(s);
	SSL_CTX_free(s_ctx);
	SSL_CTX_free(c_ctx);
	return ok ? 0 : 1;
}
