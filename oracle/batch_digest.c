/*
 * batch_digest.c — TEST INFRASTRUCTURE ONLY (fixture generator, run in the
 * build container by tests/golden/make_golden.py).
 *
 * Seals a full-size synthetic TLS record batch (BASELINE configs B/C/D,
 * SURVEY.md §8d) with the reference's own EVP_AEAD (oracle/_ref/libssl_ref.so,
 * compiled from /root/reference) using tls1_enc's framing
 * (ssl/t1_enc.c:832-975: 13-byte AAD seq||type||version||len; GCM nonce =
 * fixed IV || seq as explicit nonce, ChaCha nonce = fixed IV XOR (0^4||seq),
 * old ChaCha nonce = seq), flips one bit in every `tamper_every`-th record, opens
 * every record again with EVP_AEAD_CTX_open (zero-fill on failure,
 * evp_aead.c:137-143) and prints SHA-256 digests of
 *   sealed: the record bodies in record order, before tampering;
 *   opened: the opened plaintexts (tampered ones zero-filled) in record order.
 * The workload definition is talos_amd/workload.py's (sessions, sequence
 * numbers with near-carry starts, counter-SplitMix64 plaintexts, tamper rule),
 * so the GPU test regenerates the same batch on the device and compares.
 *
 * usage: batch_digest AEAD N_RECORDS N_SESSIONS SEED TAMPER_EVERY LEN|@lengths.u32
 *                     [interleave] [range=LO:HI]
 *   AEAD: aes-128-gcm | aes-256-gcm | chacha20-poly1305 | chacha20-poly1305-old
 *   interleave: records dealt to sessions round-robin (workload.py session_plan)
 *   range=LO:HI: digest only records [LO, HI) of the N-record batch — one GPU's
 *     shard of a batch split across GPUs (config E).  Sessions,
 *     sequence numbers, plaintexts and the tamper rule stay those of the whole
 *     batch (global record index), as talos_amd.workload.Workload(shard=) builds
 *     them on each GPU.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <openssl/evp.h>
#include <openssl/sha.h>

#define KEY_TAG 0x4B45590000000000ull
#define IV_TAG 0x4956000000000000ull
#define SEQ_TAG 0x5345510000000000ull

/* counter SplitMix64, identical to talos_amd.workload.fill_bytes */
static void
fill(uint64_t seed, uint64_t index, unsigned char *out, size_t n)
{
	uint64_t st = seed ^ (index * 0xD1B54A32D192ED03ull);
	for (size_t i = 0, w = 1; i < n; i += 8, w++) {
		uint64_t z = st + w * 0x9E3779B97F4A7C15ull;
		z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
		z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
		z ^= z >> 31;
		for (size_t b = 0; b < 8 && i + b < n; b++)
			out[i + b] = (unsigned char)(z >> (8 * b));
	}
}

static void
be64(unsigned char *p, uint64_t v)
{
	for (int i = 7; i >= 0; i--, v >>= 8)
		p[i] = (unsigned char)v;
}

static void
hex(const unsigned char *d, char *out)
{
	for (int i = 0; i < 32; i++)
		sprintf(out + 2 * i, "%02x", d[i]);
}

int
main(int argc, char **argv)
{
	if (argc < 7 || argc > 9) {
		fprintf(stderr, "usage: %s AEAD N S SEED TAMPER_EVERY LEN|@file [interleave] [range=LO:HI]\n",
		    argv[0]);
		return 2;
	}
	int interleave = 0;
	long lo = 0, hi = -1;
	for (int a = 7; a < argc; a++) {
		if (!strcmp(argv[a], "interleave"))
			interleave = 1;
		else if (sscanf(argv[a], "range=%ld:%ld", &lo, &hi) != 2) {
			fprintf(stderr, "bad argument %s\n", argv[a]);
			return 2;
		}
	}
	const char *name = argv[1];
	long n = atol(argv[2]), S = atol(argv[3]);
	if (hi < 0)
		hi = n;
	if (lo < 0 || lo > hi || hi > n) {
		fprintf(stderr, "range %ld:%ld outside [0, %ld]\n", lo, hi, n);
		return 2;
	}
	uint64_t seed = strtoull(argv[4], NULL, 0);
	long tamper = atol(argv[5]);
	const EVP_AEAD *aead;
	int gcm = 0, fiv_len;
	if (!strcmp(name, "aes-128-gcm")) {
		aead = EVP_aead_aes_128_gcm(); gcm = 1; fiv_len = 4;
	} else if (!strcmp(name, "aes-256-gcm")) {
		aead = EVP_aead_aes_256_gcm(); gcm = 1; fiv_len = 4;
	} else if (!strcmp(name, "chacha20-poly1305")) {
		aead = EVP_aead_chacha20_poly1305(); fiv_len = 12;
	} else if (!strcmp(name, "chacha20-poly1305-old")) {
		aead = EVP_aead_chacha20_poly1305_old(); fiv_len = 0;
	} else {
		fprintf(stderr, "unknown AEAD %s\n", name);
		return 2;
	}
	uint32_t *lens = malloc(sizeof(uint32_t) * n);
	if (argv[6][0] == '@') {
		FILE *f = fopen(argv[6] + 1, "rb");
		if (!f || fread(lens, 4, n, f) != (size_t)n) {
			fprintf(stderr, "cannot read %s\n", argv[6] + 1);
			return 2;
		}
		fclose(f);
	} else {
		for (long i = 0; i < n; i++)
			lens[i] = (uint32_t)atol(argv[6]);
	}
	size_t keylen = EVP_AEAD_key_length(aead);
	EVP_AEAD_CTX *ctx = calloc(S, sizeof(*ctx));
	unsigned char (*fiv)[12] = calloc(S, 12);
	uint64_t *seq0 = calloc(S, 8);
	for (long s = 0; s < S; s++) {
		unsigned char key[32], sq[8];
		fill(seed ^ KEY_TAG, s, key, keylen);
		fill(seed ^ IV_TAG, s, fiv[s], fiv_len);
		fill(seed ^ SEQ_TAG, s, sq, 8);
		uint64_t q = 0;
		for (int b = 7; b >= 0; b--)
			q = (q << 8) | sq[b];	/* little endian */
		if (s % 7 == 1)
			q = (q | 0xFF) - 3;
		else if (s % 7 == 2)
			q = (q | 0xFFFFFFFFull) - 5;
		seq0[s] = q;
		if (!EVP_AEAD_CTX_init(&ctx[s], aead, key, keylen, EVP_AEAD_DEFAULT_TAG_LENGTH, NULL)) {
			fprintf(stderr, "init failed\n");
			return 1;
		}
	}
	long per = n / S > 0 ? n / S : 1;
	const int eiv = gcm ? 8 : 0;
	size_t maxlen = 0;
	for (long i = lo; i < hi; i++)
		if (lens[i] > maxlen)
			maxlen = lens[i];
	unsigned char *pt = malloc(maxlen + 1), *body = malloc(maxlen + 64), *back = malloc(maxlen + 1);
	SHA256_CTX hs, ho;
	SHA256_Init(&hs);
	SHA256_Init(&ho);
	long bad = 0;
	for (long r = lo; r < hi; r++) {
		long s = interleave ? r % S : (r / per < S - 1 ? r / per : S - 1);
		uint64_t seq = seq0[s] + (uint64_t)(interleave ? r / S : r % per);
		size_t len = lens[r];
		fill(seed, r, pt, len);
		unsigned char ad[13], nonce[12];
		be64(ad, seq);
		ad[8] = 23;
		ad[9] = 3;
		ad[10] = 3;
		ad[11] = (unsigned char)(len >> 8);
		ad[12] = (unsigned char)len;
		size_t nonce_len = 12;
		if (gcm) {	/* t1_enc.c:887-892, explicit nonce = seq (:902-906) */
			memcpy(nonce, fiv[s], 4);
			be64(nonce + 4, seq);
			be64(body, seq);
		} else if (fiv_len == 12) {	/* t1_enc.c:870-881 */
			memcpy(nonce, fiv[s], 12);
			unsigned char q[8];
			be64(q, seq);
			for (int b = 0; b < 8; b++)
				nonce[4 + b] ^= q[b];
		} else {	/* old ChaCha: 8-byte nonce = seq */
			be64(nonce, seq);
			nonce_len = 8;
		}
		size_t out_len = 0;
		if (!EVP_AEAD_CTX_seal(&ctx[s], body + eiv, &out_len, len + 16, nonce, nonce_len, pt, len,
		    ad, 13)) {
			fprintf(stderr, "seal failed at %ld\n", r);
			return 1;
		}
		size_t blen = eiv + out_len;
		SHA256_Update(&hs, body, blen);
		if (tamper && r % tamper == tamper / 2) {	/* workload.py apply_tamper */
			size_t pos = eiv + (size_t)(((uint64_t)r * 7919) % (len + 16));
			body[pos] ^= (unsigned char)(1u << (r % 8));
		}
		/* open as tls1_enc(s, 0): nonce from the explicit part (t1_enc.c:941-948) */
		if (gcm)
			memcpy(nonce + 4, body, 8);
		size_t ol = 0;
		if (!EVP_AEAD_CTX_open(&ctx[s], back, &ol, len, nonce, nonce_len, body + eiv, len + 16,
		    ad, 13))
			bad++;	/* back[0..len) zero-filled by the reference */
		SHA256_Update(&ho, back, len);
	}
	unsigned char d1[32], d2[32];
	char h1[65], h2[65];
	SHA256_Final(d1, &hs);
	SHA256_Final(d2, &ho);
	hex(d1, h1);
	hex(d2, h2);
	long long payload = 0;
	for (long i = lo; i < hi; i++)
		payload += lens[i];
	printf("{\"aead\": \"%s\", \"records\": %ld, \"sessions\": %ld, \"seed\": %llu, "
	    "\"tamper_every\": %ld, \"interleave\": %s, \"range\": [%ld, %ld], \"payload_bytes\": %lld, "
	    "\"bad_record_mac\": %ld, \"sealed_sha256\": \"%s\", \"opened_sha256\": \"%s\"}\n", name, n,
	    S, (unsigned long long)seed, tamper, interleave ? "true" : "false", lo, hi, payload, bad, h1, h2);
	return 0;
}
