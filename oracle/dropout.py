"""Dropout masks of the HIP path, restated on the CPU (test infrastructure only).

The reference applies torch's nn.Dropout (src/model.py:19-20, 46-49, 124-125), whose RNG stream
cannot be reproduced outside torch. The MI355X path instead draws a counter-based mask (see
`vit_dropout` in include/vit_hip.h): element (row, col) of a dropout site is kept iff the 16-bit
half (col % 8) of Philox4x32-10(counter = {col // 8, row, site, offset_lo},
key = {seed_lo, seed_hi ^ offset_hi}) is >= round(p * 65536), and kept values are scaled by
1 / (1 - p). This module restates that definition in numpy so the tests can (1) pin the Philox
implementation against the Random123 known-answer vectors, (2) check the GPU masks bit-exactly,
and (3) run the oracle forward (vit_oracle.forward(..., drop=...)) with the very same masks.
Distributional parity with nn.Dropout (keep rate 1 - p, scale 1/(1 - p)) is what the reference
contract fixes; the individual masks are necessarily implementation-defined.
"""
import numpy as np

_M32 = np.uint64(0xFFFFFFFF)


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    """Random123 Philox4x32-10 on numpy uint64 arrays holding 32-bit values (broadcasting)."""
    c = [np.asarray(x, dtype=np.uint64) & _M32 for x in (c0, c1, c2, c3)]
    k0 = np.uint64(int(k0) & 0xFFFFFFFF)
    k1 = np.uint64(int(k1) & 0xFFFFFFFF)
    for _ in range(10):
        p0 = np.uint64(0xD2511F53) * c[0]
        p1 = np.uint64(0xCD9E8D57) * c[2]
        c = [(p1 >> np.uint64(32)) ^ c[1] ^ k0, p1 & _M32, (p0 >> np.uint64(32)) ^ c[3] ^ k1, p0 & _M32]
        k0 = (k0 + np.uint64(0x9E3779B9)) & _M32
        k1 = (k1 + np.uint64(0xBB67AE85)) & _M32
    return c


def dropout_mult(p, site, seed, offset, rows, cols, row0=0, row_stride=1):
    """[rows, cols] float32 multipliers (0 or 1/(1-p)) of rows row0.., as the HIP kernels use them."""
    thr = min(int(p * 65536.0 + 0.5), 65536)
    if p <= 0 or thr == 0:
        return np.ones((rows, cols), np.float32)
    r = (np.arange(rows, dtype=np.uint64) * np.uint64(max(1, row_stride)) + np.uint64(row0))[:, None]
    col = np.arange(cols, dtype=np.uint64)[None, :]
    out = philox4x32_10(col >> np.uint64(3), r, np.uint64(site), np.uint64(offset & 0xFFFFFFFF), seed & 0xFFFFFFFF,
                        ((seed >> 32) ^ (offset >> 32)) & 0xFFFFFFFF)
    k = (col & np.uint64(7)).astype(np.int64)
    word = np.choose(np.broadcast_to(k >> 1, (rows, cols)), [np.broadcast_to(w, (rows, cols)) for w in out])
    half = (word >> (np.uint64(16) * (np.broadcast_to(k, (rows, cols)) & 1).astype(np.uint64))) & np.uint64(0xFFFF)
    scale = np.float32(1.0 / (1.0 - p))
    return np.where(half >= np.uint64(thr), scale, np.float32(0.0)).astype(np.float32)
