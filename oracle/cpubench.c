/*
 * cpubench.c — CPU baseline driver (TEST / MEASUREMENT INFRASTRUCTURE ONLY).
 *
 * dlopen()s a library that exports the LibreSSL EVP_AEAD ABI (normally
 * oracle/_ref/libref.so, the reference compiled from its own sources) and
 * times EVP_AEAD_CTX_open or _seal the way tls1_enc calls them per record
 * (ssl/t1_enc.c:911-914 seal, :964-967 open): 12-byte nonce = 4-byte fixed
 * IV || 8-byte explicit nonce (GCM) or fixed IV XOR seq (ChaCha), 13-byte AAD.
 * One pthread per requested core over contiguous record slices, session setup
 * (EVP_AEAD_CTX_init) and ciphertext preparation excluded from timing
 * (SURVEY.md §8d "CPU baseline").
 *
 * usage: cpubench LIB AEAD OP REC_LEN|@lengths.u32 NREC THREADS SECONDS
 *   @file: NREC little-endian uint32 record lengths (the config-D Zipf mix)
 *   AEAD: aes-128-gcm | aes-256-gcm | chacha20-poly1305 | chacha20-poly1305-old (8-byte nonce)
 *   OP:   open | seal | both  (both = seal then open per record, config C)
 *         init  connection churn: every thread loops EVP_AEAD_CTX_init with a
 *               fresh key + one seal of a REC_LEN record + EVP_AEAD_CTX_cleanup
 *               (a connection direction's key install at ChangeCipherSpec,
 *               t1_enc.c:444-495 -> e_aes.c:1372-1413, its first record, and
 *               ssl_clear_cipher_ctx); reports contexts/s
 * prints one JSON object.
 */
#include <dlfcn.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

typedef struct { const void *aead; void *state; } EVP_AEAD_CTX;
typedef const void *(*aead_fn)(void);
typedef int (*init_fn)(EVP_AEAD_CTX *, const void *, const unsigned char *,
    size_t, size_t, void *);
typedef int (*crypt_fn)(const EVP_AEAD_CTX *, unsigned char *, size_t *, size_t,
    const unsigned char *, size_t, const unsigned char *, size_t,
    const unsigned char *, size_t);

static size_t g_nonce_len = 12;	/* 8 for the draft ChaCha AEAD */
static init_fn p_init;
static crypt_fn p_seal, p_open;
static void (*p_cleanup)(EVP_AEAD_CTX *);

#define NSESS 64

struct rec {
	unsigned char nonce[12], ad[13];
	unsigned char *ct;	/* ct || tag */
	unsigned char *pt;
	size_t len;
	int sess;
};

static EVP_AEAD_CTX ctxs[NSESS];
static struct rec *recs;
static size_t rec_len, max_len, nrec;
static int op;	/* 0 open, 1 seal, 2 both */
static double budget;

struct targ {
	size_t lo, hi;
	unsigned long long bytes, records, failures;
	double secs;
	double ph[3];	/* churn: seconds in init, first seal, cleanup */
};

static double
now(void)
{
	struct timespec ts;
	clock_gettime(CLOCK_MONOTONIC, &ts);
	return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static uint64_t
sm64(uint64_t *s)
{
	uint64_t z = (*s += 0x9E3779B97F4A7C15ULL);
	z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
	z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
	return z ^ (z >> 31);
}

static void
fill(uint64_t seed, unsigned char *p, size_t n)
{
	size_t i;
	for (i = 0; i < n; i++) {
		if (i % 8 == 0)
			seed = sm64(&seed) ^ i;
		p[i] = (unsigned char)(seed >> (8 * (i % 8)));
	}
}

static const void *g_aead;
static size_t g_key_len;

/* OP init: contexts per second (key install + first record + cleanup) */
static void *
churn_worker(void *arg)
{
	struct targ *t = arg;
	unsigned char *pt = calloc(1, rec_len + 1), *out = malloc(rec_len + 16);
	unsigned char key[32], nonce[12] = {0}, ad[13] = {0};
	size_t out_len;
	uint64_t seed = 0xC4A2ULL + t->lo;
	double t0 = now();
	for (;;) {
		EVP_AEAD_CTX c;
		fill(sm64(&seed), key, g_key_len);
		double a = now();
		if (!p_init(&c, g_aead, key, g_key_len, 0, NULL)) {
			t->failures++;
			break;
		}
		double b = now();
		if (!p_seal(&c, out, &out_len, rec_len + 16, nonce, g_nonce_len, pt, rec_len, ad, 13))
			t->failures++;
		double d = now();
		p_cleanup(&c);
		double e = now();
		t->ph[0] += b - a;	/* phases of one connection (round 6) */
		t->ph[1] += d - b;
		t->ph[2] += e - d;
		t->records++;
		t->bytes += rec_len;
		if (now() - t0 >= budget)
			break;
	}
	t->secs = now() - t0;
	free(pt);
	free(out);
	return NULL;
}

static void *
worker(void *arg)
{
	struct targ *t = arg;
	unsigned char *out = malloc(max_len + 16);
	size_t i = t->lo, out_len;
	double t0 = now(), t1;

	for (;;) {
		struct rec *r = &recs[i];
		const EVP_AEAD_CTX *c = &ctxs[r->sess];
		int ok = 1;
		if (op == 0 || op == 2) {
			if (op == 2)
				ok &= p_seal(c, out, &out_len, r->len + 16, r->nonce, g_nonce_len,
				    r->pt, r->len, r->ad, 13);
			ok &= p_open(c, out, &out_len, r->len, r->nonce, g_nonce_len, r->ct,
			    r->len + 16, r->ad, 13);
		} else {
			ok &= p_seal(c, out, &out_len, r->len + 16, r->nonce, g_nonce_len, r->pt,
			    r->len, r->ad, 13);
		}
		t->failures += !ok;
		t->bytes += r->len;
		t->records++;
		if (++i == t->hi)
			i = t->lo;
		if ((t->records & 7) == 0 && (t1 = now()) - t0 >= budget)
			break;
	}
	t->secs = now() - t0;
	free(out);
	return NULL;
}

int
main(int argc, char **argv)
{
	void *h;
	aead_fn which;
	const void *aead;
	int threads, i;
	size_t key_len, k;
	pthread_t *tid;
	struct targ *ta;
	unsigned long long bytes = 0, records = 0, failures = 0;
	double secs = 0;

	if (argc != 8) {
		fprintf(stderr, "usage: %s LIB AEAD OP REC_LEN NREC THREADS SECONDS\n",
		    argv[0]);
		return 2;
	}
	h = dlopen(argv[1], RTLD_NOW | RTLD_LOCAL);
	if (!h) {
		fprintf(stderr, "dlopen: %s\n", dlerror());
		return 1;
	}
	p_init = (init_fn)dlsym(h, "EVP_AEAD_CTX_init");
	p_seal = (crypt_fn)dlsym(h, "EVP_AEAD_CTX_seal");
	p_open = (crypt_fn)dlsym(h, "EVP_AEAD_CTX_open");
	p_cleanup = (void (*)(EVP_AEAD_CTX *))dlsym(h, "EVP_AEAD_CTX_cleanup");
	if (!strcmp(argv[2], "aes-128-gcm")) {
		which = (aead_fn)dlsym(h, "EVP_aead_aes_128_gcm");
		key_len = 16;
	} else if (!strcmp(argv[2], "aes-256-gcm")) {
		which = (aead_fn)dlsym(h, "EVP_aead_aes_256_gcm");
		key_len = 32;
	} else if (!strcmp(argv[2], "chacha20-poly1305-old")) {
		which = (aead_fn)dlsym(h, "EVP_aead_chacha20_poly1305_old");
		key_len = 32;
		g_nonce_len = 8;
	} else {
		which = (aead_fn)dlsym(h, "EVP_aead_chacha20_poly1305");
		key_len = 32;
	}
	if (!p_init || !p_seal || !p_open || !which) {
		fprintf(stderr, "missing EVP_AEAD symbols\n");
		return 1;
	}
	aead = which();
	op = !strcmp(argv[3], "open") ? 0 : !strcmp(argv[3], "seal") ? 1 :
	    !strcmp(argv[3], "init") ? 3 : 2;
	nrec = strtoul(argv[5], NULL, 0);
	uint32_t *lens = NULL;
	if (argv[4][0] == '@') {
		FILE *f = fopen(argv[4] + 1, "rb");
		lens = malloc(4 * (nrec ? nrec : 1));
		if (!f || fread(lens, 4, nrec, f) != nrec) {
			fprintf(stderr, "cannot read %zu lengths from %s\n", nrec, argv[4] + 1);
			return 2;
		}
		fclose(f);
		rec_len = 0;
	} else {
		rec_len = strtoul(argv[4], NULL, 0);
	}
	threads = atoi(argv[6]);
	budget = atof(argv[7]);
	if (threads < 1 || nrec < (size_t)threads) {
		fprintf(stderr, "need NREC >= THREADS >= 1\n");
		return 2;
	}

	if (op == 3) {	/* connection churn */
		if (!p_cleanup || argv[4][0] == '@') {
			fprintf(stderr, "init needs EVP_AEAD_CTX_cleanup and a fixed REC_LEN\n");
			return 2;
		}
		g_aead = aead;
		g_key_len = key_len;
		tid = calloc(threads, sizeof(*tid));
		ta = calloc(threads, sizeof(*ta));
		for (i = 0; i < threads; i++) {
			ta[i].lo = (size_t)i;
			pthread_create(&tid[i], NULL, churn_worker, &ta[i]);
		}
		double ph[3] = {0, 0, 0};
		for (i = 0; i < threads; i++) {
			pthread_join(tid[i], NULL);
			records += ta[i].records;
			failures += ta[i].failures;
			if (ta[i].secs > secs)
				secs = ta[i].secs;
			for (k = 0; k < 3; k++)
				ph[k] += ta[i].ph[k];
		}
		double rn = records ? (double)records : 1.0;
		printf("{\"aead\": \"%s\", \"op\": \"init\", \"rec_len\": %zu, \"threads\": %d, "
		    "\"contexts\": %llu, \"seconds\": %.4f, \"contexts_per_s\": %.1f, "
		    "\"us_per_context_per_thread\": %.2f, \"us_init\": %.2f, \"us_first_seal\": %.2f, "
		    "\"us_cleanup\": %.2f, \"failures\": %llu}\n", argv[2], rec_len,
		    threads, records, secs, records / secs, secs * 1e6 * threads / rn,
		    ph[0] * 1e6 / rn, ph[1] * 1e6 / rn, ph[2] * 1e6 / rn, failures);
		return failures ? 1 : 0;
	}
	for (i = 0; i < NSESS; i++) {
		unsigned char key[32];
		fill(0x5EED0001ULL + 977 * i, key, key_len);
		if (!p_init(&ctxs[i], aead, key, key_len, 0, NULL)) {
			fprintf(stderr, "EVP_AEAD_CTX_init failed\n");
			return 1;
		}
	}
	recs = calloc(nrec, sizeof(*recs));
	for (k = 0; k < nrec; k++) {
		struct rec *r = &recs[k];
		size_t ol;
		r->sess = (int)(k % NSESS);
		r->len = lens ? lens[k] : rec_len;
		if (r->len > max_len)
			max_len = r->len;
		r->pt = malloc(r->len ? r->len : 1);
		r->ct = malloc(r->len + 16);
		fill(0xC0FFEEULL + k, r->pt, r->len);
		fill(0xABCDULL + k, r->nonce, 12);
		fill(0x1234ULL + k, r->ad, 13);
		r->ad[11] = (unsigned char)(r->len >> 8);
		r->ad[12] = (unsigned char)r->len;
		if (!p_seal(&ctxs[r->sess], r->ct, &ol, r->len + 16, r->nonce, g_nonce_len,
		    r->pt, r->len, r->ad, 13)) {
			fprintf(stderr, "seal failed\n");
			return 1;
		}
	}
	tid = calloc(threads, sizeof(*tid));
	ta = calloc(threads, sizeof(*ta));
	for (i = 0; i < threads; i++) {
		ta[i].lo = nrec * i / threads;
		ta[i].hi = nrec * (i + 1) / threads;
		pthread_create(&tid[i], NULL, worker, &ta[i]);
	}
	for (i = 0; i < threads; i++) {
		pthread_join(tid[i], NULL);
		bytes += ta[i].bytes;
		records += ta[i].records;
		failures += ta[i].failures;
		if (ta[i].secs > secs)
			secs = ta[i].secs;
	}
	int (*bstats)(uint64_t *, uint64_t *) =
	    (int (*)(uint64_t *, uint64_t *))dlsym(h, "tlsgpu_evp_batch_stats");
	uint64_t nb = 0, nj = 0;
	if (bstats)
		bstats(&nb, &nj);
	if (nb)
		fprintf(stderr, "{\"evp_batches\": %llu, \"evp_jobs\": %llu}\n", (unsigned long long)nb,
		    (unsigned long long)nj);
	printf("{\"aead\": \"%s\", \"op\": \"%s\", \"rec_len\": %zu, \"threads\": %d, "
	    "\"records\": %llu, \"bytes\": %llu, \"seconds\": %.4f, "
	    "\"gib_per_s\": %.4f, \"failures\": %llu}\n",
	    argv[2], argv[3], rec_len, threads, records, bytes, secs,
	    bytes / secs / (1024.0 * 1024 * 1024), failures);
	return failures ? 1 : 0;
}
