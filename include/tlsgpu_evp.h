/*
 * tlsgpu_evp.h — drop-in EVP_AEAD ABI exported by libtlsgpu.so.
 *
 * Same names, signatures, struct layout and error behaviour as LibreSSL
 * 2.4.1 include/openssl/evp.h:1211-1315 (implemented there by
 * crypto/evp/evp_aead.c, e_aes.c:1360-1548, e_chacha20poly1305.c).  The
 * callers this replaces are tls1_enc (ssl/t1_enc.c:911,964),
 * tls1_change_cipher_state_aead (t1_enc.c:460-487), ssl_cipher_get_evp_aead
 * (ssl/ssl_ciph.c:726-737), ssl_clear_cipher_ctx (ssl/ssl_lib.c:2699-2708),
 * apps/openssl/speed.c:1242-1300 and tests/aeadtest.c.  Because tls1_enc calls
 * EVP_AEAD_CTX_seal/open through the PLT, link order or LD_PRELOAD routes every
 * record of an unmodified LibreSSL/TaLoS application through the GPU engine
 * (INTEGRATION.md).
 *
 * Each seal/open runs on the GPU (a one-record batch on the calling thread's
 * engine stream); there is no CPU cipher path in this library.
 */
#ifndef TLSGPU_EVP_H
#define TLSGPU_EVP_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#ifndef HEADER_EVP_H	/* when included next to LibreSSL's own evp.h */
struct evp_aead_st;
typedef struct evp_aead_st EVP_AEAD;
typedef struct engine_st ENGINE;

/* evp.h:1244-1248 — public, embedded by value in SSL_AEAD_CTX. */
typedef struct evp_aead_ctx_st {
	const EVP_AEAD *aead;
	void *aead_state;
} EVP_AEAD_CTX;

#define EVP_AEAD_MAX_TAG_LENGTH 16	/* evp.h:1252 */
#define EVP_AEAD_DEFAULT_TAG_LENGTH 0	/* evp.h:1257 */

/* Legacy EVP_CIPHER GCM surface.  Layouts of LibreSSL
 * 2.4.1's public structs (evp.h:297-313, 405-423): libcrypto's generic
 * EVP_CipherInit_ex / EVP_CipherUpdate / EVP_CIPHER_CTX_ctrl / _copy /
 * _cleanup (crypto/evp/evp_enc.c) call the function pointers of the object
 * EVP_aes_*_gcm() returns, so exporting these two getters is the whole
 * interposition. */
typedef struct evp_cipher_st EVP_CIPHER;
typedef struct evp_cipher_ctx_st EVP_CIPHER_CTX;
typedef struct asn1_type_st ASN1_TYPE;
#define EVP_MAX_IV_LENGTH 16		/* evp.h:79 */
#define EVP_MAX_BLOCK_LENGTH 32		/* evp.h:80 */
struct evp_cipher_st {
	int nid;
	int block_size;
	int key_len;
	int iv_len;
	unsigned long flags;
	int (*init)(EVP_CIPHER_CTX *ctx, const unsigned char *key, const unsigned char *iv,
	    int enc);
	int (*do_cipher)(EVP_CIPHER_CTX *ctx, unsigned char *out, const unsigned char *in,
	    size_t inl);
	int (*cleanup)(EVP_CIPHER_CTX *);
	int ctx_size;
	int (*set_asn1_parameters)(EVP_CIPHER_CTX *, ASN1_TYPE *);
	int (*get_asn1_parameters)(EVP_CIPHER_CTX *, ASN1_TYPE *);
	int (*ctrl)(EVP_CIPHER_CTX *, int type, int arg, void *ptr);
	void *app_data;
};
struct evp_cipher_ctx_st {
	const EVP_CIPHER *cipher;
	ENGINE *engine;
	int encrypt;
	int buf_len;
	unsigned char oiv[EVP_MAX_IV_LENGTH];
	unsigned char iv[EVP_MAX_IV_LENGTH];
	unsigned char buf[EVP_MAX_BLOCK_LENGTH];
	int num;
	void *app_data;
	int key_len;
	unsigned long flags;
	void *cipher_data;
	int final_used;
	int block_mask;
	unsigned char final[EVP_MAX_BLOCK_LENGTH];
};
#endif

/* e_aes.c:1054-1059: AES-128/256 GCM as EVP_CIPHERs (the init / do_cipher /
 * ctrl / cleanup of e_aes.c:687-1047, cipher work on the GPU).  AES-192-GCM
 * is not provided by this engine. */
const EVP_CIPHER *EVP_aes_128_gcm(void);
const EVP_CIPHER *EVP_aes_256_gcm(void);

/* evp.h:1211-1223 */
const EVP_AEAD *EVP_aead_aes_128_gcm(void);
const EVP_AEAD *EVP_aead_aes_256_gcm(void);
const EVP_AEAD *EVP_aead_chacha20_poly1305(void);
const EVP_AEAD *EVP_aead_chacha20_poly1305_old(void);

/* evp.h:1225-1240 */
size_t EVP_AEAD_key_length(const EVP_AEAD *aead);
size_t EVP_AEAD_nonce_length(const EVP_AEAD *aead);
size_t EVP_AEAD_max_overhead(const EVP_AEAD *aead);
size_t EVP_AEAD_max_tag_len(const EVP_AEAD *aead);

/* evp.h:1259-1315 */
int EVP_AEAD_CTX_init(EVP_AEAD_CTX *ctx, const EVP_AEAD *aead,
    const unsigned char *key, size_t key_len, size_t tag_len, ENGINE *impl);
void EVP_AEAD_CTX_cleanup(EVP_AEAD_CTX *ctx);
int EVP_AEAD_CTX_seal(const EVP_AEAD_CTX *ctx, unsigned char *out,
    size_t *out_len, size_t max_out_len, const unsigned char *nonce,
    size_t nonce_len, const unsigned char *in, size_t in_len,
    const unsigned char *ad, size_t ad_len);
int EVP_AEAD_CTX_open(const EVP_AEAD_CTX *ctx, unsigned char *out,
    size_t *out_len, size_t max_out_len, const unsigned char *nonce,
    size_t nonce_len, const unsigned char *in, size_t in_len,
    const unsigned char *ad, size_t ad_len);

#ifdef __cplusplus
}
#endif
#endif
