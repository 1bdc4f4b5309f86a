"""The fused single-pair matcher's fp16 -> int8 code conversion
(another-cuda-sift_amd/csrc/match.hip, codes16), restated in numpy over every
fp16 bit pattern: v + 1024 puts an integer 0..255 in the low mantissa byte,
the low byte ^ 0x80 is the int8 code v - 128, and a value is accepted only if
the high byte is 0x64 and (v + 1024) - 1024 gives v back bit for bit.  Exactly
the integers 0..255 are accepted (-0 is rejected: the workgroup then takes the
fp16 path, which is exact on it too), with the codes k_match_prep writes."""
import numpy as np


def test_codes16_accepts_exactly_integers_0_255():
    bits = np.arange(65536, dtype=np.uint16)
    x = bits.view(np.float16)
    with np.errstate(all="ignore"):
        y = (x + np.float16(1024)).astype(np.float16)
        back = (y - np.float16(1024)).astype(np.float16)
    yb, bb = y.view(np.uint16), back.view(np.uint16)
    good = ((yb & 0xFF00) == 0x6400) & (bb == bits)
    xf = x.astype(np.float64)
    with np.errstate(invalid="ignore"):
        expect = np.isfinite(xf) & (xf >= 0) & (xf <= 255) & (xf == np.floor(xf)) & (bits != 0x8000)
    assert np.array_equal(good, expect) and good.sum() == 256
    code = ((yb & 0xFF) ^ 0x80).astype(np.uint8).view(np.int8).astype(np.int32)
    assert np.array_equal(code[good], xf[good].astype(np.int32) - 128)
    # the squared norm by 4-byte dot products equals the plain sum
    rng = np.random.default_rng(0)
    v = rng.integers(0, 256, 128)
    c = (v - 128).astype(np.int8).astype(np.int32)
    assert sum(int(np.dot(c[k:k + 4], c[k:k + 4])) for k in range(0, 128, 4)) == int(((v - 128) ** 2).sum())
