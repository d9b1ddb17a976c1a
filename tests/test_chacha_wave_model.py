"""Model of the one-wave ChaCha20-Poly1305 job (talos_amd/csrc/chacha_wave.h),
checked on the CPU: the lane / pass / LDS-stage indexing and the 26-bit-limb
arithmetic of cc_wave_job, restated limb for limb with every intermediate
checked against the 32-/64-bit register widths the kernel uses, must give the
serial Poly1305 sum (poly1305-donna.c:54-321 over the RFC 7539 layout,
e_chacha20poly1305.c:182-190) for adversarial blocks (all ones) and keys.
The GPU parity of the kernel itself is tests/test_gpu_parity.py::
test_evp_chacha_wave_jobs; this test pins the bounds argument in its header."""
import random

import pytest

M26 = (1 << 26) - 1
P1305 = (1 << 130) - 5


def chk32(x):
    assert 0 <= x < 1 << 32, hex(x)
    return x


def chk64(x):
    assert 0 <= x < 1 << 64, hex(x)
    return x


def p5_block(m, hibit):
    """p5_block: a 16-byte block (little-endian int) as five 26-bit limbs."""
    w = [(m >> (32 * i)) & 0xFFFFFFFF for i in range(4)]
    return [w[0] & M26, ((w[0] >> 26) | (w[1] << 6)) & M26, ((w[1] >> 20) | (w[2] << 12)) & M26,
            ((w[2] >> 14) | (w[3] << 18)) & M26, (w[3] >> 8) | hibit]


def p5_add(a, b):
    return [chk32(x + y) for x, y in zip(a, b)]


def p5_carry(a):
    a = list(a)
    c = a[0] >> 26
    a[0] &= M26
    for i in range(1, 5):
        a[i] = chk32(a[i] + c)
        c = a[i] >> 26
        a[i] &= M26
    a[0] = chk32(a[0] + chk32(c * 5))
    c = a[0] >> 26
    a[0] &= M26
    a[1] = chk32(a[1] + c)
    return a


def p5_mul(a, b):
    """p5_mul: column sums in 64 bits, every carry in 32 bits."""
    s = [chk32(x * 5) for x in b]
    d = [0] * 5
    for i in range(5):
        for k in range(5):
            if i + k < 5:
                d[i + k] += a[i] * b[k]
            else:
                d[i + k - 5] += a[i] * s[k]
    for x in d:
        chk64(x)
    h = [0] * 5
    c = chk32(d[0] >> 26)
    h[0] = d[0] & M26
    for i in range(1, 5):
        d[i] = chk64(d[i] + c)
        c = chk32(d[i] >> 26)
        h[i] = d[i] & M26
    h[0] = chk32(h[0] + chk32(c * 5))
    c = h[0] >> 26
    h[0] &= M26
    h[1] = chk32(h[1] + c)
    return h


def value(a):
    return sum(x << (26 * i) for i, x in enumerate(a)) % P1305


def clamp(r):
    return r & 0x0FFFFFFC0FFFFFFC0FFFFFFC0FFFFFFF


def limbs(r):
    return [(r >> (26 * i)) & M26 for i in range(5)]


def serial(r, blocks):
    """poly1305-donna's chain: h = (h + c) * r for every block, in order."""
    h = 0
    for c in blocks:
        h = (h + c + (1 << 128)) * r % P1305
    return h


def wave(r, ad_blocks, data_blocks, len_block):
    """cc_wave_job's Poly1305 for one job, lane by lane."""
    na, nc = len(ad_blocks), len(data_blocks)
    N = na + nc + 1
    pw = [limbs(r) for _ in range(64)]          # lane l: r^(l+1), by doubling
    for lev in range(6):
        step = 1 << lev
        base = pw[step - 1]
        prod = [p5_mul(pw[(l - step) % 64], base) for l in range(64)]
        pw = [prod[l] if step <= l < 2 * step else pw[l] for l in range(64)]
    for l in range(64):
        assert value(pw[l]) == pow(r, l + 1, P1305)
    r64 = pw[63]
    acc = [[0] * 5 for _ in range(64)]
    for l in range(64):                          # AD blocks b = l, l + 64, ...
        for b in range(l, na, 64):
            acc[l] = p5_add(p5_mul(acc[l], r64), p5_block(ad_blocks[b], 1 << 24))
    nkb = (nc + 3) // 4                          # 64-B keystream blocks of data
    for t in range((nkb + 1 + 63) // 64):        # passes: counters 64t .. 64t+63
        lo, hi = (0 if t == 0 else 256 * t - 4), min(nc, 256 * t + 252)
        for l in range(64):
            i0 = lo + ((l - na - lo) & 63)
            for s in range(4):
                i = i0 + 64 * s
                if i < hi:
                    off = 16 * (i - 256 * t + 4)     # LDS stage offset
                    assert 0 <= off < 4096
                    writer = off // 64               # lane that staged it: counter 64t + writer
                    assert 4 * (64 * t + writer - 1) + (off % 64) // 16 == i
                    acc[l] = p5_add(p5_mul(acc[l], r64), p5_block(data_blocks[i], 1 << 24))
    last = (N - 1) & 63
    acc[last] = p5_add(p5_mul(acc[last], r64), p5_block(len_block, 1 << 24))
    for l in range(64):
        w = N - (l + 64 * ((N - 1 - l) >> 6)) if l < N else 1
        assert 1 <= w <= 64
        acc[l] = p5_mul(acc[l], pw[w - 1])
    return value(wave_sum(acc))


def wave_sum(v):
    """p5_wave_sum: the DPP row-shift / row-broadcast reduction, lane 63."""
    zero = [0] * 5

    def shr(a, n, banks):  # row_shr:n on the lanes of the enabled banks (4 lanes each)
        return [a[l - n] if (l % 16) >= n and ((banks >> ((l % 16) // 4)) & 1) else zero
                for l in range(64)]

    def bcast(a, src, rows):  # row_bcast: lane src's value into the enabled rows
        return [a[src if src == 31 else (l // 16) * 16 - 1] if (rows >> (l // 16)) & 1 else zero
                for l in range(64)]

    s1, s2, s3 = shr(v, 1, 0xF), shr(v, 2, 0xF), shr(v, 3, 0xF)
    a = [p5_carry(p5_add(p5_add(v[l], s1[l]), p5_add(s2[l], s3[l]))) for l in range(64)]
    t = shr(a, 4, 0xE)
    a = [p5_carry(p5_add(a[l], t[l])) for l in range(64)]
    t = shr(a, 8, 0xC)
    a = [p5_carry(p5_add(a[l], t[l])) for l in range(64)]
    t = bcast(a, 15, 0xA)
    a = [p5_carry(p5_add(a[l], t[l])) for l in range(64)]
    t = bcast(a, 31, 0xC)
    a = [p5_carry(p5_add(a[l], t[l])) for l in range(64)]
    return a[63]


CASES = [(0, 0), (13, 0), (0, 1), (13, 1400), (13, 4031), (13, 4032), (13, 4033), (0, 4096),
         (17, 8128), (1024, 8129), (1029, 16384), (2049, 16400), (13, 20000)]


@pytest.mark.parametrize("ad_len,n", CASES)
def test_wave_poly1305_model_matches_serial(ad_len, n):
    rnd = random.Random(ad_len * 100003 + n)
    for trial in range(3):
        allones = trial == 0
        r = clamp((1 << 128) - 1 if allones else rnd.getrandbits(128))
        def rb():
            return (1 << 128) - 1 if allones else rnd.getrandbits(128)
        na, nc = (ad_len + 15) // 16, (n + 15) // 16
        adb = [rb() for _ in range(na)]
        db = [rb() for _ in range(nc)]
        if ad_len % 16:
            adb[-1] &= (1 << (8 * (ad_len % 16))) - 1
        if n % 16:
            db[-1] &= (1 << (8 * (n % 16))) - 1
        lb = ad_len | (n << 64)
        assert wave(r, adb, db, lb) == serial(r, adb + db + [lb]), (ad_len, n, trial)
