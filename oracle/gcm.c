/*
 * GCM restatement for the oracle (TEST INFRASTRUCTURE ONLY — see oracle.h).
 *
 * Follows crypto/modes/gcm128.c of LibreSSL 2.4.1:
 *   CRYPTO_gcm128_init      :681-747  (H = E_K(0^128), 4-bit Htable)
 *   gcm_init_4bit           :255-324  (Htable[8]=H, halving chain, XOR fill)
 *   gcm_gmult_4bit          :333-393  (Shoup 4-bit, rem_4bit reduction)
 *   CRYPTO_gcm128_setiv     :749-824  (12-byte IV fast path, else GHASH(IV))
 *   CRYPTO_gcm128_aad       :826-881  (partial-block carry in ares)
 *   CRYPTO_gcm128_encrypt   :883-1057 / _decrypt :1059-1240 (byte-exact
 *                                      semantics of the ctr32 variants
 *                                      :1242-1475: inc32 on Yi[12..15])
 *   CRYPTO_gcm128_finish    :1477-1515, _tag :1517-1521
 * Elements are (hi, lo) 64-bit halves of the big-endian 16-byte string, as
 * in the reference's u128 after byte swapping.
 */
#include <string.h>
#include "oracle.h"

static uint64_t
load_be64(const uint8_t *p)
{
	uint64_t v = 0;
	int i;
	for (i = 0; i < 8; i++)
		v = (v << 8) | p[i];
	return v;
}

static void
store_be64(uint8_t *p, uint64_t v)
{
	int i;
	for (i = 7; i >= 0; i--) {
		p[i] = (uint8_t)v;
		v >>= 8;
	}
}

static uint32_t
load_be32(const uint8_t *p)
{
	return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}

static void
store_be32(uint8_t *p, uint32_t v)
{
	p[0] = (uint8_t)(v >> 24);
	p[1] = (uint8_t)(v >> 16);
	p[2] = (uint8_t)(v >> 8);
	p[3] = (uint8_t)v;
}

/* Multiply (hi,lo) by x: one right shift in GCM bit order, reduce with
 * 0xE1 || 0^120 (gcm128.c:72-83, REDUCE1BIT). */
static void
mulx(uint64_t *hi, uint64_t *lo)
{
	uint64_t carry = *lo & 1;
	*lo = (*lo >> 1) | (*hi << 63);
	*hi = (*hi >> 1) ^ (carry ? 0xE100000000000000ULL : 0);
}

/* rem_4bit (gcm128.c:327-331): reduction term for the four bits that leave
 * the low end when Z is shifted right by 4; derived by four mulx steps. */
static uint64_t rem4[16];
static int rem4_ready;

static void
build_rem4(void)
{
	int i, k;
	if (rem4_ready)
		return;
	for (i = 0; i < 16; i++) {
		uint64_t hi = 0, lo = (uint64_t)i;
		for (k = 0; k < 4; k++)
			mulx(&hi, &lo);
		rem4[i] = hi;
	}
	rem4_ready = 1;
}

static void
init_4bit(uint64_t Htable[16][2], const uint8_t H[16])
{
	uint64_t hi = load_be64(H), lo = load_be64(H + 8);
	int i, j;

	build_rem4();
	Htable[0][0] = Htable[0][1] = 0;
	Htable[8][0] = hi;
	Htable[8][1] = lo;
	for (i = 4; i > 0; i >>= 1) {
		mulx(&hi, &lo);
		Htable[i][0] = hi;
		Htable[i][1] = lo;
	}
	for (i = 2; i < 16; i <<= 1)
		for (j = 1; j < i; j++) {
			Htable[i + j][0] = Htable[i][0] ^ Htable[j][0];
			Htable[i + j][1] = Htable[i][1] ^ Htable[j][1];
		}
}

/* Xi <- Xi * H  (gcm_gmult_4bit, gcm128.c:333-393). */
static void
gmult_4bit(uint8_t Xi[16], const uint64_t Htable[16][2])
{
	uint64_t zh, zl;
	int cnt = 15;
	unsigned nlo, nhi, rem;

	nlo = Xi[15];
	nhi = nlo >> 4;
	nlo &= 0xf;
	zh = Htable[nlo][0];
	zl = Htable[nlo][1];
	for (;;) {
		rem = (unsigned)zl & 0xf;
		zl = (zh << 60) | (zl >> 4);
		zh = (zh >> 4) ^ rem4[rem];
		zh ^= Htable[nhi][0];
		zl ^= Htable[nhi][1];
		if (--cnt < 0)
			break;
		nlo = Xi[cnt];
		nhi = nlo >> 4;
		nlo &= 0xf;
		rem = (unsigned)zl & 0xf;
		zl = (zh << 60) | (zl >> 4);
		zh = (zh >> 4) ^ rem4[rem];
		zh ^= Htable[nlo][0];
		zl ^= Htable[nlo][1];
	}
	store_be64(Xi, zh);
	store_be64(Xi + 8, zl);
}

/* Bit-serial product (NIST SP 800-38D Algorithm 1); independent of the
 * table path above, used to build and cross-check device tables. */
void
oracle_gf128_mul(const uint8_t a[16], const uint8_t b[16], uint8_t out[16])
{
	uint64_t zh = 0, zl = 0, vh = load_be64(b), vl = load_be64(b + 8);
	int i;
	for (i = 0; i < 128; i++) {
		if ((a[i / 8] >> (7 - i % 8)) & 1) {
			zh ^= vh;
			zl ^= vl;
		}
		mulx(&vh, &vl);
	}
	store_be64(out, zh);
	store_be64(out + 8, zl);
}

void
oracle_gcm_init(oracle_gcm_ctx *c, const oracle_aes_key *k)
{
	memset(c, 0, sizeof(*c));
	c->key = *k;
	oracle_aes_encrypt(c->H, c->H, k);	/* H = E_K(0) */
	init_4bit(c->Htable, c->H);
}

void
oracle_gcm_setiv(oracle_gcm_ctx *c, const uint8_t *iv, size_t len)
{
	uint32_t ctr;
	size_t i;

	memset(c->Yi, 0, 16);
	memset(c->Xi, 0, 16);
	c->aad_len = c->msg_len = 0;
	c->ares = c->mres = 0;
	if (len == 12) {
		memcpy(c->Yi, iv, 12);
		c->Yi[15] = 1;
		ctr = 1;
	} else {
		uint64_t len0 = (uint64_t)len;
		while (len >= 16) {
			for (i = 0; i < 16; i++)
				c->Yi[i] ^= iv[i];
			gmult_4bit(c->Yi, c->Htable);
			iv += 16;
			len -= 16;
		}
		if (len) {
			for (i = 0; i < len; i++)
				c->Yi[i] ^= iv[i];
			gmult_4bit(c->Yi, c->Htable);
		}
		len0 <<= 3;
		for (i = 0; i < 8; i++)
			c->Yi[8 + i] ^= (uint8_t)(len0 >> (56 - 8 * i));
		gmult_4bit(c->Yi, c->Htable);
		ctr = load_be32(c->Yi + 12);
	}
	oracle_aes_encrypt(c->Yi, c->EK0, &c->key);
	++ctr;
	store_be32(c->Yi + 12, ctr);
}

int
oracle_gcm_aad(oracle_gcm_ctx *c, const uint8_t *aad, size_t len)
{
	uint64_t alen = c->aad_len;
	unsigned n;
	size_t i;

	if (c->msg_len)
		return -2;
	alen += len;
	if (alen > (1ULL << 61) || alen < len)
		return -1;
	c->aad_len = alen;
	n = c->ares;
	if (n) {
		while (n && len) {
			c->Xi[n] ^= *aad++;
			--len;
			n = (n + 1) % 16;
		}
		if (n == 0) {
			gmult_4bit(c->Xi, c->Htable);
		} else {
			c->ares = n;
			return 0;
		}
	}
	while (len >= 16) {
		for (i = 0; i < 16; i++)
			c->Xi[i] ^= aad[i];
		gmult_4bit(c->Xi, c->Htable);
		aad += 16;
		len -= 16;
	}
	n = 0;
	if (len) {
		n = (unsigned)len;
		for (i = 0; i < len; i++)
			c->Xi[i] ^= aad[i];
	}
	c->ares = n;
	return 0;
}

static int
gcm_crypt(oracle_gcm_ctx *c, const uint8_t *in, uint8_t *out, size_t len,
    int decrypt)
{
	uint64_t mlen = c->msg_len + len;
	uint32_t ctr;
	unsigned n;

	if (mlen > ((1ULL << 36) - 32) || mlen < len)
		return -1;
	c->msg_len = mlen;
	if (c->ares) {
		/* first data call finalises GHASH(AAD) */
		gmult_4bit(c->Xi, c->Htable);
		c->ares = 0;
	}
	ctr = load_be32(c->Yi + 12);
	n = c->mres;
	while (len--) {
		uint8_t ci;
		if (n == 0) {
			oracle_aes_encrypt(c->Yi, c->EKi, &c->key);
			++ctr;	/* inc32: only the low 32 bits move */
			store_be32(c->Yi + 12, ctr);
		}
		ci = *in++;
		*out = ci ^ c->EKi[n];
		c->Xi[n] ^= decrypt ? ci : *out;
		out++;
		n = (n + 1) % 16;
		if (n == 0)
			gmult_4bit(c->Xi, c->Htable);
	}
	c->mres = n;
	return 0;
}

int
oracle_gcm_encrypt(oracle_gcm_ctx *c, const uint8_t *in, uint8_t *out, size_t len)
{
	return gcm_crypt(c, in, out, len, 0);
}

int
oracle_gcm_decrypt(oracle_gcm_ctx *c, const uint8_t *in, uint8_t *out, size_t len)
{
	return gcm_crypt(c, in, out, len, 1);
}

void
oracle_gcm_tag(oracle_gcm_ctx *c, uint8_t *tag, size_t len)
{
	uint8_t lens[16];
	int i;

	if (c->mres || c->ares)
		gmult_4bit(c->Xi, c->Htable);
	store_be64(lens, c->aad_len << 3);
	store_be64(lens + 8, c->msg_len << 3);
	for (i = 0; i < 16; i++)
		c->Xi[i] ^= lens[i];
	gmult_4bit(c->Xi, c->Htable);
	for (i = 0; i < 16; i++)
		c->Xi[i] ^= c->EK0[i];
	memcpy(tag, c->Xi, len <= 16 ? len : 16);
}
