"""The device Poly1305's two-level parallel carry (talos_amd/csrc/chacha_kernels.hip
poly_block, round 4) restated limb for limb on the CPU: against Poly1305 as a
big-integer computation (RFC 7539 §2.5, the function poly1305-donna.c:54-321
implements), with the limb and product bounds its comment states checked on
every block — including all-0xFF keys and messages, the worst case for every
bound.  The GPU tests (full-size config C digest, aeadtests vectors) check the
kernel itself; this pins the arithmetic argument that it never overflows."""
import random

M = 0x3FFFFFF
P = (1 << 130) - 5
U32 = (1 << 32) - 1


def clamp_limbs(k: bytes):
    t0, t1, t2, t3 = (int.from_bytes(k[i:i + 4], "little") for i in (0, 4, 8, 12))
    return [t0 & 0x3FFFFFF, ((t0 >> 26) | (t1 << 6)) & 0x3FFFF03,
            ((t1 >> 20) | (t2 << 12)) & 0x3FFC0FF, ((t2 >> 14) | (t3 << 18)) & 0x3F03FFF,
            (t3 >> 8) & 0x00FFFFF]


def block(h, r, m, hibit=1 << 24):
    """poly_block with the parallel carry; asserts the stated bounds."""
    m0, m1, m2, m3 = m
    r0, r1, r2, r3, r4 = r
    s1, s2, s3, s4 = r1 * 5, r2 * 5, r3 * 5, r4 * 5
    h0 = h[0] + (m0 & M)
    h1 = h[1] + (((m0 >> 26) | (m1 << 6)) & M)
    h2 = h[2] + (((m1 >> 20) | (m2 << 12)) & M)
    h3 = h[3] + (((m2 >> 14) | (m3 << 18)) & M)
    h4 = h[4] + ((m3 >> 8) | hibit)
    assert max(h0, h1, h2, h3, h4) < 1 << 32
    d = [h0 * r0 + h1 * s4 + h2 * s3 + h3 * s2 + h4 * s1,
         h0 * r1 + h1 * r0 + h2 * s4 + h3 * s3 + h4 * s2,
         h0 * r2 + h1 * r1 + h2 * r0 + h3 * s4 + h4 * s3,
         h0 * r3 + h1 * r2 + h2 * r1 + h3 * r0 + h4 * s4,
         h0 * r4 + h1 * r3 + h2 * r2 + h3 * r1 + h4 * r0]
    assert all(x < 1 << 58 for x in d)            # c_i = d_i >> 26 exact in 32 bits
    c = [x >> 26 for x in d]
    assert c[4] * 5 < 1 << 32
    e = [(d[0] & M) + c[4] * 5, (d[1] & M) + c[0], (d[2] & M) + c[1], (d[3] & M) + c[2],
         (d[4] & M) + c[3]]
    assert all(x <= U32 for x in e)
    n = [(e[0] & M) + (e[4] >> 26) * 5, (e[1] & M) + (e[0] >> 26), (e[2] & M) + (e[1] >> 26),
         (e[3] & M) + (e[2] >> 26), (e[4] & M) + (e[3] >> 26)]
    assert all(x < (1 << 26) + 45 for x in n)      # the invariant on entry to the next block
    return n


def finish(h, pad):
    """poly_finish (poly1305-donna.c:231-321), 32-bit limb arithmetic."""
    h0, h1, h2, h3, h4 = h
    c = h1 >> 26; h1 &= M; h2 += c; c = h2 >> 26; h2 &= M; h3 += c; c = h3 >> 26; h3 &= M
    h4 += c; c = h4 >> 26; h4 &= M; h0 += c * 5; c = h0 >> 26; h0 &= M; h1 += c
    g0 = h0 + 5; c = g0 >> 26; g0 &= M; g1 = h1 + c; c = g1 >> 26; g1 &= M
    g2 = h2 + c; c = g2 >> 26; g2 &= M; g3 = h3 + c; c = g3 >> 26; g3 &= M
    g4 = (h4 + c - (1 << 26)) & U32
    mask = ((g4 >> 31) - 1) & U32
    nm = ~mask & U32
    h0, h1, h2, h3, h4 = ((a & nm) | (b & mask) for a, b in
                          zip((h0, h1, h2, h3, h4), (g0, g1, g2, g3, g4)))
    w = [(h0 | (h1 << 26)) & U32, ((h1 >> 6) | (h2 << 20)) & U32,
         ((h2 >> 12) | (h3 << 14)) & U32, ((h3 >> 18) | (h4 << 8)) & U32]
    out, f = [], 0
    for i in range(4):
        f = w[i] + pad[i] + (f >> 32)
        out.append(f & U32)
    return b"".join(x.to_bytes(4, "little") for x in out)


def poly1305_bigint(key: bytes, msg: bytes) -> bytes:
    r = int.from_bytes(key[:16], "little") & 0x0FFFFFFC0FFFFFFC0FFFFFFC0FFFFFFF
    a = 0
    for i in range(0, len(msg), 16):
        a = (a + int.from_bytes(msg[i:i + 16] + b"\x01", "little")) * r % P
    return ((a + int.from_bytes(key[16:], "little")) % (1 << 128)).to_bytes(16, "little")


def test_parallel_carry_poly1305_matches_bigint():
    rnd = random.Random(5)
    for trial in range(600):
        kind = trial % 4
        key = bytes([0xFF] * 32) if kind == 0 else bytes(rnd.randrange(256) for _ in range(32))
        nb = rnd.choice([1, 2, 5, 17, 64, 88])
        msg = (bytes([0xFF] * 16 * nb) if kind in (0, 1)
               else bytes(rnd.randrange(256) for _ in range(16 * nb)))
        r = clamp_limbs(key)
        pad = [int.from_bytes(key[16 + 4 * i:20 + 4 * i], "little") for i in range(4)]
        h = [0] * 5
        for i in range(nb):
            h = block(h, r, [int.from_bytes(msg[16 * i + 4 * j:16 * i + 4 * j + 4], "little")
                             for j in range(4)])
        assert finish(h, pad) == poly1305_bigint(key, msg), trial
