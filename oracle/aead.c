/*
 * EVP_AEAD and TLS-record restatements for the oracle (TEST INFRASTRUCTURE
 * ONLY — see oracle.h).
 *
 * AEAD layer:  crypto/evp/evp_aead.c:50-144 (key-length check, overflow and
 * alias checks, zero-fill of max_out_len and *out_len = 0 on any failure),
 * crypto/evp/e_aes.c:1372-1510 (AES-GCM: tag_len default/limit, buffer
 * checks, setiv/aad/crypt/tag, constant-time tag compare :1502) and
 * crypto/evp/e_chacha20poly1305.c:52-286 (draft "old" 8-byte nonce and RFC
 * 7539 12-byte nonce constructions, MAC-before-decrypt on open :276-283).
 *
 * Record layer: ssl/t1_enc.c:832-975 (tls1_enc AEAD branch: 13-byte AAD
 * seq||type||version||len, GCM nonce fixed||explicit, ChaCha nonce
 * fixed XOR (0^4||seq), explicit nonce carried in the record for GCM),
 * parameters as tls1_change_cipher_state_aead (t1_enc.c:444-495).
 */
#include <string.h>
#include "oracle.h"

#define R_BAD_DECRYPT 100
#define R_BUFFER_TOO_SMALL 155
#define R_TOO_LARGE 164

static int
ct_memcmp(const uint8_t *a, const uint8_t *b, size_t n)
{
	/* timingsafe_memcmp: only equality matters to callers here */
	uint8_t d = 0;
	size_t i;
	for (i = 0; i < n; i++)
		d |= a[i] ^ b[i];
	return d != 0;
}

static size_t
aead_key_len(int kind)
{
	switch (kind) {
	case ORACLE_AES_128_GCM: return 16;
	case ORACLE_AES_256_GCM: return 32;
	case ORACLE_CHACHA20_POLY1305: return 32;
	case ORACLE_CHACHA20_POLY1305_OLD: return 32;
	}
	return 0;
}

int
oracle_aead_init(oracle_aead_ctx *c, int kind, const uint8_t *key,
    size_t key_len, size_t tag_len)
{
	memset(c, 0, sizeof(*c));
	c->kind = kind;
	if (aead_key_len(kind) == 0 || key_len != aead_key_len(kind))
		return 0;	/* EVP_R_UNSUPPORTED_KEY_SIZE, evp_aead.c:55-58 */
	if (tag_len == 0)
		tag_len = 16;
	if (tag_len > 16)
		return 0;
	c->key_len = key_len;
	c->tag_len = tag_len;
	c->nonce_len = (kind == ORACLE_CHACHA20_POLY1305_OLD) ? 8 : 12;
	memcpy(c->key, key, key_len);
	if (kind == ORACLE_AES_128_GCM || kind == ORACLE_AES_256_GCM) {
		oracle_aes_set_encrypt_key(key, (int)key_len * 8, &c->aes);
		oracle_gcm_init(&c->gcm, &c->aes);
	}
	return 1;
}

static void
poly_pad16(oracle_poly1305_ctx *p, const uint8_t *d, size_t n)
{
	static const uint8_t zero[16];
	oracle_poly1305_update(p, d, n);
	if (n % 16)
		oracle_poly1305_update(p, zero, 16 - n % 16);
}

static void
poly_len(oracle_poly1305_ctx *p, const uint8_t *d, size_t n)
{
	uint8_t lb[8];
	uint64_t j = n;
	int i;
	for (i = 0; i < 8; i++) {
		lb[i] = (uint8_t)j;
		j >>= 8;
	}
	if (d != NULL)
		oracle_poly1305_update(p, d, n);
	oracle_poly1305_update(p, lb, 8);
}

/* MAC over (ad, ct) for either ChaCha construction; polykey derived here. */
static void
chacha_mac(const oracle_aead_ctx *c, const uint8_t *nonce, const uint8_t *ad,
    size_t ad_len, const uint8_t *ct, size_t ct_len, uint8_t mac[16],
    const uint8_t **iv_out, uint64_t *ctr_out)
{
	uint8_t pk[32];
	oracle_poly1305_ctx p;
	const uint8_t *iv;
	uint64_t ctr;

	memset(pk, 0, sizeof(pk));
	if (c->nonce_len == 8) {
		iv = nonce;
		ctr = 0;
		oracle_chacha20(pk, pk, 32, c->key, iv, 0);
		oracle_poly1305_init(&p, pk);
		poly_len(&p, ad, ad_len);
		poly_len(&p, ct, ct_len);
	} else {
		ctr = (uint64_t)((uint32_t)nonce[0] | (uint32_t)nonce[1] << 8 |
		    (uint32_t)nonce[2] << 16 | (uint32_t)nonce[3] << 24) << 32;
		iv = nonce + 4;
		oracle_chacha20(pk, pk, 32, c->key, iv, ctr);
		oracle_poly1305_init(&p, pk);
		poly_pad16(&p, ad, ad_len);
		poly_pad16(&p, ct, ct_len);
		poly_len(&p, NULL, ad_len);
		poly_len(&p, NULL, ct_len);
	}
	oracle_poly1305_finish(&p, mac);
	*iv_out = iv;
	*ctr_out = ctr;
}

static int
do_seal(const oracle_aead_ctx *c, uint8_t *out, size_t *out_len,
    size_t max_out_len, const uint8_t *nonce, size_t nonce_len,
    const uint8_t *in, size_t in_len, const uint8_t *ad, size_t ad_len)
{
	if (c->kind == ORACLE_AES_128_GCM || c->kind == ORACLE_AES_256_GCM) {
		oracle_gcm_ctx g;
		if (max_out_len < in_len + c->tag_len)
			return 0;
		g = c->gcm;
		oracle_gcm_setiv(&g, nonce, nonce_len);
		if (ad_len > 0 && oracle_gcm_aad(&g, ad, ad_len))
			return 0;
		if (oracle_gcm_encrypt(&g, in, out, in_len))
			return 0;
		oracle_gcm_tag(&g, out + in_len, c->tag_len);
		*out_len = in_len + c->tag_len;
		return 1;
	} else {
		uint8_t mac[16];
		const uint8_t *iv;
		uint64_t ctr, pk_ctr;
		if ((uint64_t)in_len >= (1ULL << 32) * 64 - 64)
			return 0;
		if (max_out_len < in_len + c->tag_len)
			return 0;
		if (nonce_len != c->nonce_len)
			return 0;
		/* encrypt first (ct feeds the MAC) */
		if (c->nonce_len == 8) {
			iv = nonce;
			ctr = 1;
		} else {
			pk_ctr = (uint64_t)((uint32_t)nonce[0] | (uint32_t)nonce[1] << 8 |
			    (uint32_t)nonce[2] << 16 | (uint32_t)nonce[3] << 24) << 32;
			iv = nonce + 4;
			ctr = pk_ctr + 1;
		}
		oracle_chacha20(out, in, in_len, c->key, iv, ctr);
		chacha_mac(c, nonce, ad, ad_len, out, in_len, mac, &iv, &pk_ctr);
		memcpy(out + in_len, mac, c->tag_len);
		*out_len = in_len + c->tag_len;
		return 1;
	}
}

static int
do_open(const oracle_aead_ctx *c, uint8_t *out, size_t *out_len,
    size_t max_out_len, const uint8_t *nonce, size_t nonce_len,
    const uint8_t *in, size_t in_len, const uint8_t *ad, size_t ad_len)
{
	size_t pt_len;
	if (c->kind == ORACLE_AES_128_GCM || c->kind == ORACLE_AES_256_GCM) {
		oracle_gcm_ctx g;
		uint8_t tag[16];
		if (in_len < c->tag_len)
			return 0;
		pt_len = in_len - c->tag_len;
		if (max_out_len < pt_len)
			return 0;
		g = c->gcm;
		oracle_gcm_setiv(&g, nonce, nonce_len);
		if (oracle_gcm_aad(&g, ad, ad_len))
			return 0;
		if (oracle_gcm_decrypt(&g, in, out, pt_len))
			return 0;
		oracle_gcm_tag(&g, tag, c->tag_len);
		if (ct_memcmp(tag, in + pt_len, c->tag_len))
			return 0;
		*out_len = pt_len;
		return 1;
	} else {
		uint8_t mac[16];
		const uint8_t *iv;
		uint64_t ctr;
		if (in_len < c->tag_len)
			return 0;
		if ((uint64_t)in_len >= (1ULL << 32) * 64 - 64)
			return 0;
		if (nonce_len != c->nonce_len)
			return 0;
		pt_len = in_len - c->tag_len;
		if (max_out_len < pt_len)
			return 0;
		chacha_mac(c, nonce, ad, ad_len, in, pt_len, mac, &iv, &ctr);
		if (ct_memcmp(mac, in + pt_len, c->tag_len))
			return 0;
		oracle_chacha20(out, in, pt_len, c->key, iv, ctr + 1);
		*out_len = pt_len;
		return 1;
	}
}

static int
check_alias(const uint8_t *in, size_t in_len, const uint8_t *out)
{
	if (out <= in)
		return 1;
	if (in + in_len <= out)
		return 1;
	return 0;
}

int
oracle_aead_seal(const oracle_aead_ctx *c, uint8_t *out, size_t *out_len,
    size_t max_out_len, const uint8_t *nonce, size_t nonce_len,
    const uint8_t *in, size_t in_len, const uint8_t *ad, size_t ad_len)
{
	size_t possible = in_len + 16;
	if (possible < in_len || !check_alias(in, in_len, out) ||
	    !do_seal(c, out, out_len, max_out_len, nonce, nonce_len, in, in_len,
	    ad, ad_len)) {
		memset(out, 0, max_out_len);
		*out_len = 0;
		return 0;
	}
	return 1;
}

int
oracle_aead_open(const oracle_aead_ctx *c, uint8_t *out, size_t *out_len,
    size_t max_out_len, const uint8_t *nonce, size_t nonce_len,
    const uint8_t *in, size_t in_len, const uint8_t *ad, size_t ad_len)
{
	if (!check_alias(in, in_len, out) ||
	    !do_open(c, out, out_len, max_out_len, nonce, nonce_len, in, in_len,
	    ad, ad_len)) {
		memset(out, 0, max_out_len);
		*out_len = 0;
		return 0;
	}
	return 1;
}

/* ---- TLS record framing ---------------------------------------------- */

int
oracle_tls_session_init(oracle_tls_session *s, int kind, const uint8_t *key,
    size_t key_len, const uint8_t *fixed_iv, size_t fixed_iv_len,
    uint16_t version)
{
	memset(s, 0, sizeof(*s));
	if (!oracle_aead_init(&s->aead, kind, key, key_len, 0))
		return 0;
	if (fixed_iv_len > sizeof(s->fixed_nonce))
		return 0;
	memcpy(s->fixed_nonce, fixed_iv, fixed_iv_len);
	s->fixed_nonce_len = fixed_iv_len;
	s->variable_nonce_len = 8;
	s->variable_nonce_in_record =
	    (kind == ORACLE_AES_128_GCM || kind == ORACLE_AES_256_GCM);
	s->xor_fixed_nonce = (kind == ORACLE_CHACHA20_POLY1305);
	s->version = version;
	if (s->xor_fixed_nonce) {
		if (s->fixed_nonce_len != s->aead.nonce_len)
			return 0;
	} else if (s->fixed_nonce_len + s->variable_nonce_len != s->aead.nonce_len) {
		return 0;
	}
	return 1;
}

static void
build_nonce(const oracle_tls_session *s, const uint8_t seq8[8],
    const uint8_t *explicit8, uint8_t nonce[16], size_t *nonce_used)
{
	size_t i;
	if (s->xor_fixed_nonce) {
		size_t pad = s->fixed_nonce_len - s->variable_nonce_len;
		memset(nonce, 0, pad);
		memcpy(nonce + pad, seq8, s->variable_nonce_len);
		for (i = 0; i < s->fixed_nonce_len; i++)
			nonce[i] ^= s->fixed_nonce[i];
		*nonce_used = s->fixed_nonce_len;
	} else {
		memcpy(nonce, s->fixed_nonce, s->fixed_nonce_len);
		memcpy(nonce + s->fixed_nonce_len, explicit8, s->variable_nonce_len);
		*nonce_used = s->fixed_nonce_len + s->variable_nonce_len;
	}
}

static void
seq_bytes(uint64_t seq, uint8_t out[8])
{
	int i;
	for (i = 7; i >= 0; i--) {
		out[i] = (uint8_t)seq;
		seq >>= 8;
	}
}

int
oracle_tls_open(const oracle_tls_session *s, uint64_t seq, uint8_t type,
    const uint8_t *body, size_t body_len, uint8_t *out, size_t *pt_len)
{
	uint8_t ad[13], nonce[16];
	size_t nonce_used, len = body_len, out_len = 0;
	const uint8_t *in = body;

	seq_bytes(seq, ad);
	ad[8] = type;
	ad[9] = (uint8_t)(s->version >> 8);
	ad[10] = (uint8_t)s->version;
	if (len < s->variable_nonce_len)
		return 0;
	build_nonce(s, ad, s->variable_nonce_in_record ? in : ad, nonce,
	    &nonce_used);
	if (s->variable_nonce_in_record) {
		in += s->variable_nonce_len;
		len -= s->variable_nonce_len;
	}
	if (len < s->aead.tag_len)
		return 0;
	len -= s->aead.tag_len;
	ad[11] = (uint8_t)(len >> 8);
	ad[12] = (uint8_t)len;
	*pt_len = len;
	if (!oracle_aead_open(&s->aead, out, &out_len, len, nonce, nonce_used,
	    in, len + s->aead.tag_len, ad, sizeof(ad)))
		return -1;
	*pt_len = out_len;
	return 1;
}

int
oracle_tls_seal(const oracle_tls_session *s, uint64_t seq, uint8_t type,
    const uint8_t *pt, size_t pt_len, uint8_t *out, size_t *body_len)
{
	uint8_t ad[13], nonce[16];
	size_t nonce_used, out_len = 0, eivlen = 0;

	seq_bytes(seq, ad);
	ad[8] = type;
	ad[9] = (uint8_t)(s->version >> 8);
	ad[10] = (uint8_t)s->version;
	build_nonce(s, ad, ad, nonce, &nonce_used);
	if (s->variable_nonce_in_record) {
		memcpy(out, ad, s->variable_nonce_len);
		eivlen = s->variable_nonce_len;
	}
	ad[11] = (uint8_t)(pt_len >> 8);
	ad[12] = (uint8_t)pt_len;
	if (!oracle_aead_seal(&s->aead, out + eivlen, &out_len,
	    pt_len + s->aead.tag_len, nonce, nonce_used, pt, pt_len, ad,
	    sizeof(ad)))
		return -1;
	*body_len = out_len + eivlen;
	return 1;
}

/* ---- synthetic workload ---------------------------------------------- */

uint64_t
oracle_splitmix64(uint64_t *state)
{
	uint64_t z = (*state += 0x9E3779B97F4A7C15ULL);
	z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
	z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
	return z ^ (z >> 31);
}

void
oracle_fill_bytes(uint64_t seed, uint64_t index, uint8_t *out, size_t n)
{
	uint64_t st = seed ^ (index * 0xD1B54A32D192ED03ULL);
	size_t i;
	for (i = 0; i < n; i += 8) {
		uint64_t v = oracle_splitmix64(&st);
		size_t k;
		for (k = 0; k < 8 && i + k < n; k++)
			out[i + k] = (uint8_t)(v >> (8 * k));
	}
}
