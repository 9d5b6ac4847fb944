"""Address decoding / set-index hashing."""
import pytest


def _ipoly16_equations(a, b):
    # hand-written GF(2) rows of IPOLY(5): x^4 + x + 1 (the reference lists
    # the same rows in hashing.cc); bit j of `a` contributes x^(4+j) mod P.
    bit = lambda v, i: (v >> i) & 1
    n0 = bit(a, 11) ^ bit(a, 10) ^ bit(a, 9) ^ bit(a, 8) ^ bit(a, 6) ^ bit(a, 4) ^ bit(a, 3) ^ bit(a, 0) ^ bit(b, 0)
    n1 = bit(a, 12) ^ bit(a, 8) ^ bit(a, 7) ^ bit(a, 6) ^ bit(a, 5) ^ bit(a, 3) ^ bit(a, 1) ^ bit(a, 0) ^ bit(b, 1)
    n2 = bit(a, 9) ^ bit(a, 8) ^ bit(a, 7) ^ bit(a, 6) ^ bit(a, 4) ^ bit(a, 2) ^ bit(a, 1) ^ bit(b, 2)
    n3 = bit(a, 10) ^ bit(a, 9) ^ bit(a, 8) ^ bit(a, 7) ^ bit(a, 5) ^ bit(a, 3) ^ bit(a, 2) ^ bit(b, 3)
    return n0 | n1 << 1 | n2 << 2 | n3 << 3


def test_ipoly16_matches_gf2_rows(native):
    import random
    rnd = random.Random(1)
    for _ in range(2000):
        a = rnd.getrandbits(40)
        b = rnd.getrandbits(4)
        assert native.ipoly_hash(a, b, 16) == _ipoly16_equations(a, b)


@pytest.mark.parametrize("nb", [16, 32, 64])
def test_ipoly_conflict_free_power_of_two_strides(native, nb):
    # IPOLY's defining property: nb consecutive multiples of any 2^k stride
    # land in nb distinct banks
    for k in range(0, 10):
        banks = set()
        for i in range(nb):
            addr_line = (i << k)
            idx = addr_line & (nb - 1)
            hi = addr_line >> (nb.bit_length() - 1)
            banks.add(native.ipoly_hash(hi, idx, nb))
        assert len(banks) == nb, (nb, k)


def test_qv100_subpartition_spread(native, qv100_args):
    # consecutive 256B chunks spread over all 64 sub-partitions
    subs = [native.addr_decode(qv100_args, 0x7000_0000_0000 + i * 256)["sub"] for i in range(4096)]
    assert set(subs) == set(range(64))
    counts = [subs.count(s) for s in range(64)]
    assert max(counts) - min(counts) <= 8


def test_linear_set_index(native):
    g = "N:64:128:16,L:R:f:N:L,S:2:48,4"
    for a in (0, 128, 64 * 128, 12345 * 128):
        assert native.cache_set_index(g, a) == (a >> 7) & 63
