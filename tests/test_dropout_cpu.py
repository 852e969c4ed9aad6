"""Dropout mask definition (oracle/dropout.py) on CPU: Philox4x32-10 against the Random123
known-answer vectors, keep rate / scale, and independence of sites, rows and offsets."""
import numpy as np

from oracle.dropout import dropout_mult, philox4x32_10


def test_philox_known_answers():
    # Random123 kat_vectors, philox4x32 10 rounds
    kat = [((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
           ((0xFFFFFFFF,) * 4, (0xFFFFFFFF,) * 2, (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
           ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
            (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1))]
    for ctr, key, want in kat:
        got = tuple(int(x) for x in philox4x32_10(*ctr, *key))
        assert got == want, [hex(v) for v in got]


def test_mask_rate_scale_and_independence():
    p = 0.1
    m = dropout_mult(p, 7, 0x0123456789ABCDEF, 11, 1024, 768)
    keep = m > 0
    assert abs(keep.mean() - (1 - p)) < 3e-3
    assert np.allclose(m[keep], 1 / (1 - p))
    # different site / offset / rows give (nearly) independent masks
    for other in (dropout_mult(p, 8, 0x0123456789ABCDEF, 11, 1024, 768),
                  dropout_mult(p, 7, 0x0123456789ABCDEF, 12, 1024, 768),
                  dropout_mult(p, 7, 0x0123456789ABCDEF, 11, 1024, 768, row0=1024)):
        agree = ((other > 0) == keep).mean()
        assert abs(agree - ((1 - p) ** 2 + p ** 2)) < 5e-3
    # a sub-block with row0 / row_stride is the same as slicing the full mask
    full = dropout_mult(p, 3, 99, 5, 64, 40)
    assert np.array_equal(dropout_mult(p, 3, 99, 5, 16, 40, row0=8), full[8:24])
    assert np.array_equal(dropout_mult(p, 3, 99, 5, 8, 40, row_stride=8), full[::8])
    assert np.array_equal(dropout_mult(0.0, 3, 99, 5, 4, 4), np.ones((4, 4), np.float32))
