/*
 * ChaCha20 and Poly1305 restatements for the oracle (TEST INFRASTRUCTURE
 * ONLY — see oracle.h).
 *
 * ChaCha20 follows crypto/chacha/chacha.c:59-77 (CRYPTO_chacha_20: key setup,
 * iv in words 14-15, 64-bit block counter in words 12-13 set from `counter`)
 * and chacha-merged.c:113-270 (20 rounds = 10 double rounds of the quarter
 * round at :69-73, counter carry word 12 -> 13 at :230-236, partial last
 * block through a temporary at :144-150).
 *
 * Poly1305 follows crypto/poly1305/poly1305-donna.c: r clamping (:59-64),
 * 26-bit limbs with the 2^128 bit added per full block (:86), the final
 * padded block with hibit cleared (:214-230), full carry, conditional
 * subtraction of p = 2^130-5 and addition of the pad mod 2^128 (:231-321).
 */
#include <string.h>
#include "oracle.h"

static uint32_t
le32(const uint8_t *p)
{
	return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) |
	    ((uint32_t)p[3] << 24);
}

static void
put_le32(uint8_t *p, uint32_t v)
{
	p[0] = (uint8_t)v;
	p[1] = (uint8_t)(v >> 8);
	p[2] = (uint8_t)(v >> 16);
	p[3] = (uint8_t)(v >> 24);
}

#define ROTL32(v, n) (((v) << (n)) | ((v) >> (32 - (n))))
#define QR(a, b, c, d) do {                                  \
	a += b; d ^= a; d = ROTL32(d, 16);                   \
	c += d; b ^= c; b = ROTL32(b, 12);                   \
	a += b; d ^= a; d = ROTL32(d, 8);                    \
	c += d; b ^= c; b = ROTL32(b, 7);                    \
} while (0)

static void
chacha_block(const uint32_t in[16], uint8_t out[64])
{
	uint32_t x[16];
	int i;
	memcpy(x, in, sizeof(x));
	for (i = 0; i < 10; i++) {
		QR(x[0], x[4], x[8], x[12]);
		QR(x[1], x[5], x[9], x[13]);
		QR(x[2], x[6], x[10], x[14]);
		QR(x[3], x[7], x[11], x[15]);
		QR(x[0], x[5], x[10], x[15]);
		QR(x[1], x[6], x[11], x[12]);
		QR(x[2], x[7], x[8], x[13]);
		QR(x[3], x[4], x[9], x[14]);
	}
	for (i = 0; i < 16; i++)
		put_le32(out + 4 * i, x[i] + in[i]);
}

void
oracle_chacha20(uint8_t *out, const uint8_t *in, size_t len,
    const uint8_t key[32], const uint8_t iv[8], uint64_t counter)
{
	static const uint8_t sigma[16] = "expand 32-byte k";
	uint32_t st[16];
	uint8_t ks[64];
	size_t i, n;

	for (i = 0; i < 4; i++)
		st[i] = le32(sigma + 4 * i);
	for (i = 0; i < 8; i++)
		st[4 + i] = le32(key + 4 * i);
	st[12] = (uint32_t)counter;
	st[13] = (uint32_t)(counter >> 32);
	st[14] = le32(iv);
	st[15] = le32(iv + 4);
	while (len) {
		chacha_block(st, ks);
		n = len < 64 ? len : 64;
		for (i = 0; i < n; i++)
			out[i] = in[i] ^ ks[i];
		out += n;
		in += n;
		len -= n;
		if (++st[12] == 0)
			++st[13];
	}
}

static void
poly_blocks(oracle_poly1305_ctx *c, const uint8_t *m, size_t bytes, uint32_t hibit)
{
	const uint32_t r0 = c->r[0], r1 = c->r[1], r2 = c->r[2], r3 = c->r[3],
	    r4 = c->r[4];
	const uint32_t s1 = r1 * 5, s2 = r2 * 5, s3 = r3 * 5, s4 = r4 * 5;
	uint32_t h0 = c->h[0], h1 = c->h[1], h2 = c->h[2], h3 = c->h[3],
	    h4 = c->h[4];

	while (bytes >= 16) {
		uint64_t d0, d1, d2, d3, d4;
		uint32_t cr;
		h0 += le32(m + 0) & 0x3ffffff;
		h1 += (le32(m + 3) >> 2) & 0x3ffffff;
		h2 += (le32(m + 6) >> 4) & 0x3ffffff;
		h3 += (le32(m + 9) >> 6) & 0x3ffffff;
		h4 += (le32(m + 12) >> 8) | hibit;
		d0 = (uint64_t)h0 * r0 + (uint64_t)h1 * s4 + (uint64_t)h2 * s3 +
		    (uint64_t)h3 * s2 + (uint64_t)h4 * s1;
		d1 = (uint64_t)h0 * r1 + (uint64_t)h1 * r0 + (uint64_t)h2 * s4 +
		    (uint64_t)h3 * s3 + (uint64_t)h4 * s2;
		d2 = (uint64_t)h0 * r2 + (uint64_t)h1 * r1 + (uint64_t)h2 * r0 +
		    (uint64_t)h3 * s4 + (uint64_t)h4 * s3;
		d3 = (uint64_t)h0 * r3 + (uint64_t)h1 * r2 + (uint64_t)h2 * r1 +
		    (uint64_t)h3 * r0 + (uint64_t)h4 * s4;
		d4 = (uint64_t)h0 * r4 + (uint64_t)h1 * r3 + (uint64_t)h2 * r2 +
		    (uint64_t)h3 * r1 + (uint64_t)h4 * r0;
		cr = (uint32_t)(d0 >> 26); h0 = (uint32_t)d0 & 0x3ffffff;
		d1 += cr; cr = (uint32_t)(d1 >> 26); h1 = (uint32_t)d1 & 0x3ffffff;
		d2 += cr; cr = (uint32_t)(d2 >> 26); h2 = (uint32_t)d2 & 0x3ffffff;
		d3 += cr; cr = (uint32_t)(d3 >> 26); h3 = (uint32_t)d3 & 0x3ffffff;
		d4 += cr; cr = (uint32_t)(d4 >> 26); h4 = (uint32_t)d4 & 0x3ffffff;
		h0 += cr * 5; cr = h0 >> 26; h0 &= 0x3ffffff;
		h1 += cr;
		m += 16;
		bytes -= 16;
	}
	c->h[0] = h0; c->h[1] = h1; c->h[2] = h2; c->h[3] = h3; c->h[4] = h4;
}

void
oracle_poly1305_init(oracle_poly1305_ctx *c, const uint8_t key[32])
{
	c->r[0] = le32(key + 0) & 0x3ffffff;
	c->r[1] = (le32(key + 3) >> 2) & 0x3ffff03;
	c->r[2] = (le32(key + 6) >> 4) & 0x3ffc0ff;
	c->r[3] = (le32(key + 9) >> 6) & 0x3f03fff;
	c->r[4] = (le32(key + 12) >> 8) & 0x00fffff;
	memset(c->h, 0, sizeof(c->h));
	c->pad[0] = le32(key + 16);
	c->pad[1] = le32(key + 20);
	c->pad[2] = le32(key + 24);
	c->pad[3] = le32(key + 28);
	c->leftover = 0;
}

void
oracle_poly1305_update(oracle_poly1305_ctx *c, const uint8_t *m, size_t n)
{
	size_t i, want;
	if (c->leftover) {
		want = 16 - c->leftover;
		if (want > n)
			want = n;
		for (i = 0; i < want; i++)
			c->buffer[c->leftover + i] = m[i];
		n -= want;
		m += want;
		c->leftover += want;
		if (c->leftover < 16)
			return;
		poly_blocks(c, c->buffer, 16, 1u << 24);
		c->leftover = 0;
	}
	if (n >= 16) {
		want = n & ~(size_t)15;
		poly_blocks(c, m, want, 1u << 24);
		m += want;
		n -= want;
	}
	for (i = 0; i < n; i++)
		c->buffer[c->leftover + i] = m[i];
	c->leftover += n;
}

void
oracle_poly1305_finish(oracle_poly1305_ctx *c, uint8_t mac[16])
{
	uint32_t h0, h1, h2, h3, h4, cr, g0, g1, g2, g3, g4, mask;
	uint64_t f;

	if (c->leftover) {
		size_t i = c->leftover;
		c->buffer[i++] = 1;
		for (; i < 16; i++)
			c->buffer[i] = 0;
		poly_blocks(c, c->buffer, 16, 0);
	}
	h0 = c->h[0]; h1 = c->h[1]; h2 = c->h[2]; h3 = c->h[3]; h4 = c->h[4];
	cr = h1 >> 26; h1 &= 0x3ffffff;
	h2 += cr; cr = h2 >> 26; h2 &= 0x3ffffff;
	h3 += cr; cr = h3 >> 26; h3 &= 0x3ffffff;
	h4 += cr; cr = h4 >> 26; h4 &= 0x3ffffff;
	h0 += cr * 5; cr = h0 >> 26; h0 &= 0x3ffffff;
	h1 += cr;
	/* g = h + 5 - 2^130; select g if no borrow */
	g0 = h0 + 5; cr = g0 >> 26; g0 &= 0x3ffffff;
	g1 = h1 + cr; cr = g1 >> 26; g1 &= 0x3ffffff;
	g2 = h2 + cr; cr = g2 >> 26; g2 &= 0x3ffffff;
	g3 = h3 + cr; cr = g3 >> 26; g3 &= 0x3ffffff;
	g4 = h4 + cr - (1u << 26);
	mask = (g4 >> 31) - 1;	/* all ones when h >= p */
	h0 = (h0 & ~mask) | (g0 & mask);
	h1 = (h1 & ~mask) | (g1 & mask);
	h2 = (h2 & ~mask) | (g2 & mask);
	h3 = (h3 & ~mask) | (g3 & mask);
	h4 = (h4 & ~mask) | (g4 & mask);
	/* pack to 4 x 32 bits and add the pad mod 2^128 */
	h0 = (h0) | (h1 << 26);
	h1 = (h1 >> 6) | (h2 << 20);
	h2 = (h2 >> 12) | (h3 << 14);
	h3 = (h3 >> 18) | (h4 << 8);
	f = (uint64_t)h0 + c->pad[0]; h0 = (uint32_t)f;
	f = (uint64_t)h1 + c->pad[1] + (f >> 32); h1 = (uint32_t)f;
	f = (uint64_t)h2 + c->pad[2] + (f >> 32); h2 = (uint32_t)f;
	f = (uint64_t)h3 + c->pad[3] + (f >> 32); h3 = (uint32_t)f;
	put_le32(mac + 0, h0);
	put_le32(mac + 4, h1);
	put_le32(mac + 8, h2);
	put_le32(mac + 12, h3);
}
