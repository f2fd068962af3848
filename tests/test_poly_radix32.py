"""The device Poly1305 block step (cz_device.h poly_block, radix 2^32) restated with Python
integers: every intermediate is checked against the bound its VALU instruction assumes
(u64 product columns, single-bit carries, 32-bit top word, h4 <= 4) and the running value
against the big-integer definition (h + m) * r mod 2^130 - 5, over adversarial inputs
(all-ones r and message words) and random ones.

Two reductions are restated: the shipped one-chain form (the 2^130 == 5 fold and the column
carries in one v_addc_co_u32 chain) and the round-1/2 two-chain form it replaced (column
carries, then the fold in a second chain).  The GPU parity tests pin the compiled kernels
against the oracle.
"""
import random

import pytest

M32 = (1 << 32) - 1
P = (1 << 130) - 5


def poly_block(h, r, m, hibit, one_chain=True):
    h0, h1, h2, h3, h4 = h
    r0, r1, r2, r3 = r
    s1, s2, s3 = r1 + (r1 >> 2), r2 + (r2 >> 2), r3 + (r3 >> 2)
    a, c = [], 0
    for hv, mv in zip((h0, h1, h2, h3), m):
        t = hv + mv + c
        a.append(t & M32)
        c = t >> 32
    a0, a1, a2, a3 = a
    a4 = h4 + c + hibit
    assert a4 <= 6
    d0 = a0 * r0 + a1 * s3 + a2 * s2 + a3 * s1
    d1 = a0 * r1 + a1 * r0 + a2 * s3 + a3 * s2 + a4 * s1
    d2 = a0 * r2 + a1 * r1 + a2 * r0 + a3 * s3 + a4 * s2
    d3 = a0 * r3 + a1 * r2 + a2 * r1 + a3 * r0 + a4 * s3
    assert all(d < 1 << 64 for d in (d0, d1, d2, d3))  # v_mad_u64_u32 columns
    h4r = a4 * r0
    assert h4r <= M32  # v_mul_lo_u32 is exact
    if one_chain:
        x = (d3 >> 32) + h4r
        assert x <= M32  # v_add_u32, no carry out
        q = x >> 2
        k = 5 * q
        assert k <= M32  # v_lshl_add_u32
        pairs = (((d0 & M32), k), ((d1 & M32), d0 >> 32), ((d2 & M32), d1 >> 32), ((d3 & M32), d2 >> 32))
        out, c = [], 0
        for lo, hi in pairs:
            t = lo + hi + c
            out.append(t & M32)
            c = t >> 32
            assert c <= 1  # one v_addc_co_u32 per limb
        n4 = (x & 3) + c
        assert n4 <= 4
        return (*out, n4)
    # two-chain form: e = column carries, then fold e4's bits above 2^130 as 5q into limb 0
    e, c = [d0 & M32], 0
    for lo, hi in (((d1 & M32), d0 >> 32), ((d2 & M32), d1 >> 32), ((d3 & M32), d2 >> 32)):
        t = lo + hi + c
        e.append(t & M32)
        c = t >> 32
        assert c <= 1
    e4 = (d3 >> 32) + h4r + c
    assert e4 <= M32  # no carry out of the top word (all-ones inputs reach 2^31.02)
    q = e4 >> 2
    k = 5 * q
    assert k <= M32  # v_lshl_add_u32
    out, c = [], 0
    for j in range(4):
        t = e[j] + (k if j == 0 else 0) + c
        out.append(t & M32)
        c = t >> 32
        assert c <= 1
    n4 = (e4 & 3) + c
    assert n4 <= 4
    return (*out, n4)


def value(h):
    return h[0] | h[1] << 32 | h[2] << 64 | h[3] << 96 | h[4] << 128


def _run(r_words, msgs, one_chain):
    r = (r_words[0] & 0x0FFFFFFF, r_words[1] & 0x0FFFFFFC, r_words[2] & 0x0FFFFFFC, r_words[3] & 0x0FFFFFFC)
    rv = r[0] | r[1] << 32 | r[2] << 64 | r[3] << 96
    h, ref = (0, 0, 0, 0, 0), 0
    for m in msgs:
        h = poly_block(h, r, m, 1, one_chain)
        ref = (ref + (m[0] | m[1] << 32 | m[2] << 64 | m[3] << 96 | 1 << 128)) * rv % P
        assert value(h) % P == ref
    return h


@pytest.mark.parametrize("one_chain", [False, True])
def test_poly_radix32_extremes(one_chain):
    ones = [M32] * 4
    _run(ones, [ones] * 64, one_chain)
    _run(ones, [[0] * 4] * 64, one_chain)
    _run([0, 0, 0, 0], [ones] * 8, one_chain)


@pytest.mark.parametrize("one_chain", [False, True])
def test_poly_radix32_random(one_chain):
    rng = random.Random(20261017)
    for trial in range(300):
        rw = [rng.getrandbits(32) for _ in range(4)]
        msgs = [[M32] * 4 if (trial + b) % 5 == 0 else [rng.getrandbits(32) for _ in range(4)] for b in range(20)]
        _run(rw, msgs, one_chain)
