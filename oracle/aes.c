/*
 * AES restatement for the oracle (TEST INFRASTRUCTURE ONLY — see oracle.h).
 *
 * Follows the behaviour of crypto/aes/aes_core.c: AES_set_encrypt_key
 * (:628-723, 10/12/14 rounds, big-endian round-key words) and AES_encrypt
 * (:789-972).  Written byte-wise from FIPS-197 rather than with the
 * reference's T-tables; the S-box is derived at first use from the GF(2^8)
 * inverse plus the affine map, so no table is copied.
 */
#include <string.h>
#include "oracle.h"

static uint8_t sbox[256];
static int sbox_ready;

static uint8_t
xtime(uint8_t x)
{
	return (uint8_t)((x << 1) ^ ((x & 0x80) ? 0x1b : 0));
}

static uint8_t
gmul(uint8_t a, uint8_t b)
{
	uint8_t p = 0;
	while (b) {
		if (b & 1)
			p ^= a;
		a = xtime(a);
		b >>= 1;
	}
	return p;
}

static void
build_sbox(void)
{
	int x;
	if (sbox_ready)
		return;
	for (x = 0; x < 256; x++) {
		uint8_t inv = 0, s;
		int y;
		if (x) {
			for (y = 1; y < 256; y++)
				if (gmul((uint8_t)x, (uint8_t)y) == 1) {
					inv = (uint8_t)y;
					break;
				}
		}
		/* affine: s = inv ^ rotl1 ^ rotl2 ^ rotl3 ^ rotl4 ^ 0x63 */
		s = inv;
		for (y = 1; y <= 4; y++)
			s ^= (uint8_t)((inv << y) | (inv >> (8 - y)));
		sbox[x] = s ^ 0x63;
	}
	sbox_ready = 1;
}

static uint32_t
sub_word(uint32_t w)
{
	return ((uint32_t)sbox[w >> 24] << 24) | ((uint32_t)sbox[(w >> 16) & 0xff] << 16) |
	    ((uint32_t)sbox[(w >> 8) & 0xff] << 8) | sbox[w & 0xff];
}

/* aes_core.c:628-723 — returns 0 on success, -2 on bad bit length. */
int
oracle_aes_set_encrypt_key(const uint8_t *key, int bits, oracle_aes_key *k)
{
	int nk, i, total;
	uint32_t rcon = 1;

	build_sbox();
	if (bits != 128 && bits != 192 && bits != 256)
		return -2;
	nk = bits / 32;
	k->rounds = nk + 6;
	total = 4 * (k->rounds + 1);
	for (i = 0; i < nk; i++)
		k->rk[i] = ((uint32_t)key[4 * i] << 24) | ((uint32_t)key[4 * i + 1] << 16) |
		    ((uint32_t)key[4 * i + 2] << 8) | key[4 * i + 3];
	for (i = nk; i < total; i++) {
		uint32_t t = k->rk[i - 1];
		if (i % nk == 0) {
			t = sub_word((t << 8) | (t >> 24)) ^ (rcon << 24);
			rcon = xtime((uint8_t)rcon);
		} else if (nk > 6 && i % nk == 4) {
			t = sub_word(t);
		}
		k->rk[i] = k->rk[i - nk] ^ t;
	}
	return 0;
}

/* aes_core.c:789-972 — state as s[col*4+row]. */
void
oracle_aes_encrypt(const uint8_t in[16], uint8_t out[16], const oracle_aes_key *k)
{
	uint8_t s[16], t[16];
	int r, c, i;

	for (i = 0; i < 16; i++)
		s[i] = in[i] ^ (uint8_t)(k->rk[i / 4] >> (24 - 8 * (i % 4)));
	for (r = 1; r <= k->rounds; r++) {
		/* SubBytes + ShiftRows: row j of column c comes from column c+j */
		for (c = 0; c < 4; c++)
			for (i = 0; i < 4; i++)
				t[c * 4 + i] = sbox[s[((c + i) % 4) * 4 + i]];
		if (r != k->rounds) {
			for (c = 0; c < 4; c++) {
				uint8_t a0 = t[c * 4], a1 = t[c * 4 + 1], a2 = t[c * 4 + 2],
				    a3 = t[c * 4 + 3];
				uint8_t all = a0 ^ a1 ^ a2 ^ a3;
				s[c * 4 + 0] = a0 ^ all ^ xtime(a0 ^ a1);
				s[c * 4 + 1] = a1 ^ all ^ xtime(a1 ^ a2);
				s[c * 4 + 2] = a2 ^ all ^ xtime(a2 ^ a3);
				s[c * 4 + 3] = a3 ^ all ^ xtime(a3 ^ a0);
			}
		} else {
			memcpy(s, t, 16);
		}
		for (i = 0; i < 16; i++)
			s[i] ^= (uint8_t)(k->rk[4 * r + i / 4] >> (24 - 8 * (i % 4)));
	}
	memcpy(out, s, 16);
}
