/*
 * ssl_loopback.c — TEST / MEASUREMENT INFRASTRUCTURE ONLY.
 *
 * In-process TLS 1.2 loopback over the reference's own, unmodified LibreSSL
 * 2.4.1 libssl + libcrypto (oracle/_ref/libssl_ref.so, compiled from
 * /root/reference by oracle/Makefile): BASELINE configs[0], the memory-BIO
 * loopback of tests/ssltest.c:1324 (doit) / :959 (doit_biopair), written for
 * this repository.  A client and a server SSL object per thread talk through a
 * BIO pair; after the handshake the client SSL_write()s records of -r bytes
 * (do_ssl3_write -> tls1_enc(s,1) -> EVP_AEAD_CTX_seal, ssl/s3_pkt.c:560-762,
 * ssl/t1_enc.c:911), the server SSL_read()s and checks them
 * (ssl3_get_record -> tls1_enc(s,0) -> EVP_AEAD_CTX_open, s3_pkt.c:279-495,
 * t1_enc.c:964) and echoes them back the same way.
 *
 * Run as is, every record cipher call is the reference's CPU path.  Run with
 * LD_PRELOAD=talos_amd/libtlsgpu.so, the record layer's EVP_AEAD_* PLT calls
 * bind to libtlsgpu.so instead (no change to libssl or to this program); the
 * harness then reads libtlsgpu's call counters (tlsgpu_evp_call_stats, looked
 * up with dlsym) and reports them next to the number of records the TLS
 * exchange must have sealed and opened, so a test can check that every record
 * ran on the GPU.
 *
 * -m (TaLoS module check, for the TaLoS-patched build _ref/ssl_loopback_talos):
 * before any SSL object exists the harness calls ecall_tls_processing_module_init
 * (src/talos/enclaveshim/tls_processing_interface.c:60, what TaLoS's
 * initialize_library does, enclaveshim_ecalls.c:440), so the linked module
 * (oracle/talos_module.c) registers its callbacks; afterwards it checks that the
 * module saw, per SSL object and direction, the plaintext of every application
 * record in order (hooks of s3_pkt.c.patch:19-33 and :39-52) and one
 * new/free connection call per SSL object (ssl_lib.c.patch).
 *
 * usage: ssl_loopback -p server.pem [-c cipher] [-r record_bytes]
 *                     [-n records_per_direction] [-t threads] [-m]
 * prints one JSON line; exit status 0 only if every byte round-tripped (and,
 * with -m, the module check passed).
 */
#define _GNU_SOURCE	/* RTLD_DEFAULT */
#include <dlfcn.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include <openssl/bio.h>
#include <openssl/crypto.h>
#include <openssl/ec.h>
#include <openssl/err.h>
#include <openssl/ssl.h>

#define MAX_PLAIN 16384	/* SSL3_RT_MAX_PLAIN_LENGTH, ssl3.h:259 */

static const char *pem = NULL;
static const char *cipher = "ECDHE-RSA-AES128-GCM-SHA256";
static long rec_bytes = 1024;
static long nrec = 4096;
static int nthreads = 1;
static int module_check = 0;

/* LibreSSL 2.4.1 takes OpenSSL-1.0-style locking callbacks from the app. */
static pthread_mutex_t *locks;

static void
lock_cb(int mode, int type, const char *file, int line)
{
	(void)file;
	(void)line;
	if (mode & CRYPTO_LOCK)
		pthread_mutex_lock(&locks[type]);
	else
		pthread_mutex_unlock(&locks[type]);
}

static unsigned long
id_cb(void)
{
	return (unsigned long)pthread_self();
}

static double
now(void)
{
	struct timespec ts;
	clock_gettime(CLOCK_MONOTONIC, &ts);
	return ts.tv_sec + ts.tv_nsec * 1e-9;
}

/* deterministic payload: SplitMix64 keyed by (thread, direction, record) */
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

struct targ {
	int id;
	int ok;
	SSL *c, *s;	/* freed by main after the module check (no address reuse) */
	char err[200];
	char negotiated[64];
	double t_data;
	long long bytes;
};

static SSL_CTX *s_ctx, *c_ctx;

/* ---- TaLoS module check (-m) ---- */
struct talos_log_entry {
	const void *ssl;
	uint32_t dir, len;
	uint64_t fnv;
};

static uint64_t
fnv1a(const unsigned char *p, long n)
{
	uint64_t h = 0xcbf29ce484222325ull;
	for (long i = 0; i < n; i++)
		h = (h ^ p[i]) * 0x100000001b3ull;
	return h;
}

/* The last nrec chunks the module logged for (ssl, dir) must be the nrec
 * payloads of that direction, in order (earlier chunks are handshake records). */
static int
check_stream(const struct talos_log_entry *e, uint64_t n, const void *ssl, uint32_t dir,
    int id, int echo, unsigned char *buf, long *seen)
{
	long cnt = 0;
	for (uint64_t i = 0; i < n; i++)
		cnt += e[i].ssl == ssl && e[i].dir == dir;
	*seen += cnt;
	if (cnt < nrec)
		return 0;
	long skip = cnt - nrec, k = 0;
	for (uint64_t i = 0; i < n; i++) {
		if (e[i].ssl != ssl || e[i].dir != dir || skip-- > 0)
			continue;
		fill(buf, rec_bytes, ((uint64_t)id << 40) ^ ((uint64_t)k << 1) ^ (uint64_t)echo);
		if (e[i].len != (uint32_t)rec_bytes || e[i].fnv != fnv1a(buf, rec_bytes))
			return 0;
		k++;
	}
	return k == nrec;
}

static int
check_module(struct targ *ta, char *out, size_t outlen)
{
	const struct talos_log_entry *(*get)(uint64_t *, uint64_t *, uint64_t *) =
	    (const struct talos_log_entry *(*)(uint64_t *, uint64_t *, uint64_t *))dlsym(
	    RTLD_DEFAULT, "talos_module_log");
	int (*hooks)(uint64_t *, uint64_t *) =
	    (int (*)(uint64_t *, uint64_t *))dlsym(RTLD_DEFAULT, "tlsgpu_talos_hook_stats");
	uint64_t hr = 0, hw = 0;
	if (hooks)
		hooks(&hr, &hw);
	if (!get || rec_bytes > MAX_PLAIN) {
		snprintf(out, outlen, "{\"ok\": false, \"why\": \"%s\"}",
		    get ? "record_bytes > 16384" : "no module linked");
		return 0;
	}
	uint64_t n, nnew, nfree;
	const struct talos_log_entry *e = get(&n, &nnew, &nfree);
	unsigned char *buf = malloc(rec_bytes);
	long seen = 0, streams_ok = 0;
	for (int t = 0; t < nthreads; t++) {
		/* client writes k, server reads it; server echoes k ^ 1, client reads it */
		streams_ok += check_stream(e, n, ta[t].c, 1, t, 0, buf, &seen);
		streams_ok += check_stream(e, n, ta[t].s, 0, t, 0, buf, &seen);
		streams_ok += check_stream(e, n, ta[t].s, 1, t, 1, buf, &seen);
		streams_ok += check_stream(e, n, ta[t].c, 0, t, 1, buf, &seen);
	}
	free(buf);
	const int ok = streams_ok == 4L * nthreads && nnew == 2ull * nthreads;
	snprintf(out, outlen,
	    "{\"ok\": %s, \"chunks_logged\": %llu, \"streams_ok\": %ld, \"streams\": %d, "
	    "\"app_records_checked\": %ld, \"new_connections\": %llu, \"freed_before_check\": %llu, "
	    "\"tlsgpu_hook_read_calls\": %llu, \"tlsgpu_hook_write_calls\": %llu, "
	    "\"tlsgpu_hooks\": %s}",
	    ok ? "true" : "false", (unsigned long long)n, streams_ok, 4 * nthreads,
	    4L * nthreads * nrec, (unsigned long long)nnew, (unsigned long long)nfree,
	    (unsigned long long)hr, (unsigned long long)hw, hooks ? "true" : "false");
	(void)seen;
	return ok;
}

static int
want_io(SSL *s, int rc)
{
	int e = SSL_get_error(s, rc);
	return e == SSL_ERROR_WANT_READ || e == SSL_ERROR_WANT_WRITE;
}

/* move `len` bytes from `from` to `to` with SSL_write/SSL_read; the BIO pair
 * buffers hold a whole write, so the writer never blocks on the reader. */
static int
transfer(SSL *from, SSL *to, const unsigned char *buf, unsigned char *rbuf, long len,
    struct targ *t)
{
	int w = SSL_write(from, buf, (int)len);
	if (w != len) {
		snprintf(t->err, sizeof(t->err), "SSL_write returned %d (err %d)", w,
		    SSL_get_error(from, w));
		return 0;
	}
	long got = 0;
	while (got < len) {
		int r = SSL_read(to, rbuf + got, (int)(len - got));
		if (r <= 0) {
			snprintf(t->err, sizeof(t->err), "SSL_read returned %d (err %d) after %ld of %ld",
			    r, SSL_get_error(to, r), got, len);
			return 0;
		}
		got += r;
	}
	if (memcmp(buf, rbuf, len) != 0) {
		snprintf(t->err, sizeof(t->err), "payload mismatch");
		return 0;
	}
	return 1;
}

static void *
run(void *arg)
{
	struct targ *t = arg;
	SSL *c = SSL_new(c_ctx), *s = SSL_new(s_ctx);
	BIO *cb = NULL, *sb = NULL;
	unsigned char *buf = malloc(rec_bytes), *rbuf = malloc(rec_bytes);
	t->ok = 0;
	if (!c || !s || !buf || !rbuf ||
	    !BIO_new_bio_pair(&cb, 4 * (rec_bytes + 4096), &sb, 4 * (rec_bytes + 4096))) {
		snprintf(t->err, sizeof(t->err), "setup failed");
		goto out;
	}
	SSL_set_bio(c, cb, cb);
	SSL_set_bio(s, sb, sb);
	SSL_set_connect_state(c);
	SSL_set_accept_state(s);
	/* handshake, both ends stepped in turn (ssltest.c:1372-1470 loop) */
	int c_done = 0, s_done = 0;
	for (int it = 0; it < 1000 && !(c_done && s_done); it++) {
		if (!c_done) {
			int rc = SSL_do_handshake(c);
			if (rc == 1)
				c_done = 1;
			else if (!want_io(c, rc)) {
				snprintf(t->err, sizeof(t->err), "client handshake error %d",
				    SSL_get_error(c, rc));
				goto out;
			}
		}
		if (!s_done) {
			int rc = SSL_do_handshake(s);
			if (rc == 1)
				s_done = 1;
			else if (!want_io(s, rc)) {
				snprintf(t->err, sizeof(t->err), "server handshake error %d",
				    SSL_get_error(s, rc));
				goto out;
			}
		}
	}
	if (!(c_done && s_done)) {
		snprintf(t->err, sizeof(t->err), "handshake did not finish");
		goto out;
	}
	snprintf(t->negotiated, sizeof(t->negotiated), "%s", SSL_get_cipher_name(c));
	double t0 = now();
	for (long k = 0; k < nrec; k++) {
		fill(buf, rec_bytes, ((uint64_t)t->id << 40) ^ ((uint64_t)k << 1));
		if (!transfer(c, s, buf, rbuf, rec_bytes, t))
			goto out;
		fill(buf, rec_bytes, ((uint64_t)t->id << 40) ^ ((uint64_t)k << 1) ^ 1);
		if (!transfer(s, c, buf, rbuf, rec_bytes, t))
			goto out;
	}
	t->t_data = now() - t0;
	t->bytes = 2LL * nrec * rec_bytes;
	t->ok = 1;
out:
	t->c = c;
	t->s = s;
	free(buf);
	free(rbuf);
	return NULL;
}

int
main(int argc, char **argv)
{
	int o;
	while ((o = getopt(argc, argv, "p:c:r:n:t:m")) != -1) {
		switch (o) {
		case 'm': module_check = 1; break;
		case 'p': pem = optarg; break;
		case 'c': cipher = optarg; break;
		case 'r': rec_bytes = atol(optarg); break;
		case 'n': nrec = atol(optarg); break;
		case 't': nthreads = atoi(optarg); break;
		default:
			fprintf(stderr, "usage: %s -p server.pem [-c cipher] [-r bytes] [-n records] "
			    "[-t threads]\n", argv[0]);
			return 2;
		}
	}
	if (!pem || rec_bytes < 1 || rec_bytes > 4 * MAX_PLAIN || nrec < 0 || nthreads < 1 ||
	    nthreads > 256) {
		fprintf(stderr, "bad arguments\n");
		return 2;
	}
	SSL_library_init();
	SSL_load_error_strings();
	locks = calloc(CRYPTO_num_locks(), sizeof(*locks));
	for (int i = 0; i < CRYPTO_num_locks(); i++)
		pthread_mutex_init(&locks[i], NULL);
	CRYPTO_set_id_callback(id_cb);
	CRYPTO_set_locking_callback(lock_cb);

	s_ctx = SSL_CTX_new(TLSv1_2_server_method());
	c_ctx = SSL_CTX_new(TLSv1_2_client_method());
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

	if (module_check) {	/* TaLoS initialize_library -> module init */
		void (*init)(void) = (void (*)(void))dlsym(RTLD_DEFAULT,
		    "ecall_tls_processing_module_init");
		if (!init) {
			fprintf(stderr, "no TaLoS tls_processing interface in this process\n");
			return 1;
		}
		init();
	}
	/* libtlsgpu's EVP call counters, present only when it is interposed */
	int (*stats)(uint64_t *, uint64_t *) =
	    (int (*)(uint64_t *, uint64_t *))dlsym(RTLD_DEFAULT, "tlsgpu_evp_call_stats");
	uint64_t seal0 = 0, open0 = 0, seal1 = 0, open1 = 0;
	if (stats)
		stats(&seal0, &open0);

	struct targ *ta = calloc(nthreads, sizeof(*ta));
	pthread_t *th = calloc(nthreads, sizeof(*th));
	double t0 = now();
	for (int i = 0; i < nthreads; i++) {
		ta[i].id = i;
		pthread_create(&th[i], NULL, run, &ta[i]);
	}
	for (int i = 0; i < nthreads; i++)
		pthread_join(th[i], NULL);
	double wall = now() - t0;
	if (stats)
		stats(&seal1, &open1);

	int ok = 1;
	long long bytes = 0;
	double tmax = 0;
	for (int i = 0; i < nthreads; i++) {
		if (!ta[i].ok) {
			ok = 0;
			fprintf(stderr, "thread %d: %s\n", i, ta[i].err);
		}
		bytes += ta[i].bytes;
		if (ta[i].t_data > tmax)
			tmax = ta[i].t_data;
	}
	if (!ok)
		ERR_print_errors_fp(stderr);
	char mod[400] = "null";
	if (module_check)
		ok &= check_module(ta, mod, sizeof(mod));
	for (int i = 0; i < nthreads; i++) {
		if (ta[i].c)
			SSL_free(ta[i].c);
		if (ta[i].s)
			SSL_free(ta[i].s);
	}
	/* records each side must seal (and the peer open): its Finished plus
	 * nrec writes of ceil(rec_bytes / max_send_fragment) records each
	 * (ssl3_write_bytes splits at 16 KiB, s3_pkt.c:531-536) */
	long long per_write = (rec_bytes + MAX_PLAIN - 1) / MAX_PLAIN;
	long long expect = (long long)nthreads * 2 * (1 + nrec * per_write);
	printf("{\"ok\": %s, \"cipher\": \"%s\", \"threads\": %d, \"record_bytes\": %ld, "
	    "\"writes_per_direction\": %ld, \"payload_bytes\": %lld, \"data_seconds_max\": %.6f, "
	    "\"wall_seconds\": %.6f, \"gib_per_s\": %.4f, \"records_sealed_expected\": %lld, "
	    "\"records_opened_expected\": %lld, \"tlsgpu_interposed\": %s, "
	    "\"tlsgpu_seal_calls\": %llu, \"tlsgpu_open_calls\": %llu, \"talos_module\": %s}\n",
	    ok ? "true" : "false", ta[0].negotiated, nthreads, rec_bytes, nrec, bytes, tmax, wall,
	    tmax > 0 ? bytes / tmax / (1024.0 * 1024 * 1024) : 0.0, expect, expect,
	    stats ? "true" : "false", (unsigned long long)(seal1 - seal0),
	    (unsigned long long)(open1 - open0), mod);
	SSL_CTX_free(s_ctx);
	SSL_CTX_free(c_ctx);
	return ok ? 0 : 1;
}
