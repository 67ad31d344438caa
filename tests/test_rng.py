"""Pins include/gs_rng.h (the canonical replacement for math/rand) against the
Random123 Philox4x32-10 known-answer vectors (kat_vectors, philox4x32_10)."""
import ctypes as C


def _philox(olib, ctr, key):
    c = (C.c_uint32 * 4)(*ctr)
    k = (C.c_uint32 * 2)(*key)
    o = (C.c_uint32 * 4)()
    olib.orng_philox(c, k, o)
    return list(o)


def test_philox_kat_zero(olib):
    assert _philox(olib, [0, 0, 0, 0], [0, 0]) == [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]


def test_philox_kat_ones(olib):
    f = 0xFFFFFFFF
    assert _philox(olib, [f, f, f, f], [f, f]) == [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]


def test_philox_kat_pi(olib):
    out = _philox(olib, [0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344], [0xA4093822, 0x299F31D0])
    assert out == [0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]


def test_key64_layout(olib):
    o = _philox(olib, [1, 2, 3, 4], [7, 12])
    assert olib.orng_key64(7, 12, 1, 2, 3, 4) == (o[0] << 32) | o[1]


def test_key64_mid_pairs(olib):
    """The message-id sites take both halves of a block: ids 2j and 2j + 1 share
    the block of counter word j (gs_rng.h gs_key64_mid)."""
    for j in (0, 1, 2500, 0x7FFFFFFF):
        o = _philox(olib, [5, 9, j, 33], [7, 11])
        assert olib.orng_key64_mid(7, 11, 5, 9, 2 * j, 33) == (o[0] << 32) | o[1]
        assert olib.orng_key64_mid(7, 11, 5, 9, 2 * j + 1, 33) == (o[2] << 32) | o[3]
