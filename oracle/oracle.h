/*
 * oracle.h — CPU restatement of the TaLoS/LibreSSL 2.4.1 TLS record bulk-cipher
 * path.  TEST INFRASTRUCTURE ONLY: this library is the parity checker for the
 * HIP engine in talos_amd/.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it.  The product path never links or calls it.
 *
 * Every function cites the reference file:line it restates (paths relative to
 * /root/reference/src/libressl-2.4.1).  Parity of this restatement is pinned by
 * the reference's own known-answer vectors (tests/aeadtests.txt, the
 * tests/gcm128test.c, chachatest.c and poly1305test.c vectors re-encoded under
 * tests/golden/) and by record-level vectors produced by the reference itself
 * (oracle/_ref/libref.so, built from the reference sources by oracle/Makefile).
 */
#ifndef TLSGPU_ORACLE_H
#define TLSGPU_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- primitives ------------------------------------------------------- */

/* AES key schedule (crypto/aes/aes_core.c:628-723) and block encryption
 * (aes_core.c:789-972).  rk holds 4*(rounds+1) big-endian words. */
typedef struct {
	uint32_t rk[60];
	int rounds;
} oracle_aes_key;

int oracle_aes_set_encrypt_key(const uint8_t *key, int bits, oracle_aes_key *k);
void oracle_aes_encrypt(const uint8_t in[16], uint8_t out[16],
    const oracle_aes_key *k);

/* GCM mode (crypto/modes/gcm128.c).  Mirrors GCM128_CONTEXT semantics
 * (modes_lcl.h:79-95): setiv resets state, aad must precede data, tag via
 * finish.  GHASH uses the 4-bit Shoup tables of gcm128.c:255-393. */
typedef struct {
	uint8_t Yi[16], EKi[16], EK0[16], Xi[16], H[16];
	uint64_t Htable[16][2];
	uint64_t aad_len, msg_len;
	unsigned ares, mres;
	oracle_aes_key key;
} oracle_gcm_ctx;

void oracle_gcm_init(oracle_gcm_ctx *c, const oracle_aes_key *k);
void oracle_gcm_setiv(oracle_gcm_ctx *c, const uint8_t *iv, size_t len);
int oracle_gcm_aad(oracle_gcm_ctx *c, const uint8_t *aad, size_t len);
int oracle_gcm_encrypt(oracle_gcm_ctx *c, const uint8_t *in, uint8_t *out,
    size_t len);
int oracle_gcm_decrypt(oracle_gcm_ctx *c, const uint8_t *in, uint8_t *out,
    size_t len);
void oracle_gcm_tag(oracle_gcm_ctx *c, uint8_t *tag, size_t len);
/* GF(2^128) product in GCM bit order (x^0 = MSB of byte 0). */
void oracle_gf128_mul(const uint8_t a[16], const uint8_t b[16], uint8_t out[16]);

/* ChaCha20 with a 64-bit block counter (crypto/chacha/chacha.c:59-77,
 * chacha-merged.c:78-270). */
void oracle_chacha20(uint8_t *out, const uint8_t *in, size_t len,
    const uint8_t key[32], const uint8_t iv[8], uint64_t counter);

/* Poly1305 one-shot (crypto/poly1305/poly1305-donna.c:54-321). */
typedef struct {
	uint32_t r[5], h[5], pad[4];
	size_t leftover;
	uint8_t buffer[16];
} oracle_poly1305_ctx;
void oracle_poly1305_init(oracle_poly1305_ctx *c, const uint8_t key[32]);
void oracle_poly1305_update(oracle_poly1305_ctx *c, const uint8_t *m, size_t n);
void oracle_poly1305_finish(oracle_poly1305_ctx *c, uint8_t mac[16]);

/* ---- EVP_AEAD restatement (crypto/evp/evp_aead.c, e_aes.c:1360-1548,
 * e_chacha20poly1305.c:40-322) ------------------------------------------- */

enum oracle_aead_kind {
	ORACLE_AES_128_GCM = 1,
	ORACLE_AES_256_GCM = 2,
	ORACLE_CHACHA20_POLY1305 = 3,
	ORACLE_CHACHA20_POLY1305_OLD = 4,
};

typedef struct {
	int kind;
	size_t key_len, nonce_len, tag_len;
	uint8_t key[32];
	oracle_aes_key aes;
	oracle_gcm_ctx gcm;	/* H / Htable precomputed at init */
} oracle_aead_ctx;

/* Return 1 on success, 0 on failure; failure code in *err (EVP_R_* value). */
int oracle_aead_init(oracle_aead_ctx *c, int kind, const uint8_t *key,
    size_t key_len, size_t tag_len);
int oracle_aead_seal(const oracle_aead_ctx *c, uint8_t *out, size_t *out_len,
    size_t max_out_len, const uint8_t *nonce, size_t nonce_len,
    const uint8_t *in, size_t in_len, const uint8_t *ad, size_t ad_len);
int oracle_aead_open(const oracle_aead_ctx *c, uint8_t *out, size_t *out_len,
    size_t max_out_len, const uint8_t *nonce, size_t nonce_len,
    const uint8_t *in, size_t in_len, const uint8_t *ad, size_t ad_len);

/* ---- TLS 1.2 AEAD record framing (ssl/t1_enc.c:832-975) ---------------- */

typedef struct {
	oracle_aead_ctx aead;
	uint8_t fixed_nonce[12];
	size_t fixed_nonce_len;
	size_t variable_nonce_len;	/* 8 */
	int xor_fixed_nonce;		/* ChaCha (RFC 7905) */
	int variable_nonce_in_record;	/* GCM */
	uint16_t version;		/* s->version, e.g. 0x0303 */
} oracle_tls_session;

/* Install per-direction AEAD state as tls1_change_cipher_state_aead does
 * (t1_enc.c:444-495; nonce parameters from ssl_ciph.c / s3_lib.c). */
int oracle_tls_session_init(oracle_tls_session *s, int kind,
    const uint8_t *key, size_t key_len, const uint8_t *fixed_iv,
    size_t fixed_iv_len, uint16_t version);

/* Decrypt one record body in place semantics of tls1_enc(s, 0).
 * body: record fragment after the 5-byte header, body_len bytes.
 * Plaintext is written to out (out == body + variable_nonce_len for GCM in
 * the TLS layer, == body for ChaCha).  Returns 1 ok (*pt_len set),
 * 0 publicly invalid, -1 bad_record_mac (out zeroed for *pt_len bytes as
 * EVP_AEAD_CTX_open does with max_out_len). */
int oracle_tls_open(const oracle_tls_session *s, uint64_t seq, uint8_t type,
    const uint8_t *body, size_t body_len, uint8_t *out, size_t *pt_len);
/* Encrypt one record as tls1_enc(s, 1): writes the record body
 * (explicit nonce || ct || tag for GCM, ct || tag for ChaCha) into out and
 * returns its length through *body_len.  Returns 1 ok, -1 error. */
int oracle_tls_seal(const oracle_tls_session *s, uint64_t seq, uint8_t type,
    const uint8_t *pt, size_t pt_len, uint8_t *out, size_t *body_len);

/* ---- synthetic workload -------------------------------- */
uint64_t oracle_splitmix64(uint64_t *state);
/* Deterministic bytes keyed by (seed, index): used by tests and the CPU
 * baseline to regenerate any record of a batch independently. */
void oracle_fill_bytes(uint64_t seed, uint64_t index, uint8_t *out, size_t n);

#ifdef __cplusplus
}
#endif
#endif
