"""The numpy MXFP8 restatement (tests/mx_ref.py) pinned on known e4m3 values
(OCP e4m3fn table: max 448, min subnormal 2^-9, RNE) before it checks the GPU."""
import numpy as np

from mx_ref import E4M3, e4m3_encode, mx_dequantize, mx_quantize


def test_e4m3_known_codes():
    assert E4M3[0x7E] == 448.0 and np.isnan(E4M3[0x7F]) and E4M3[0x01] == 2.0 ** -9
    assert E4M3[0x38] == 1.0 and E4M3[0x08] == 2.0 ** -6
    x = np.array([1.0, 1.0625, 1.1875, 448.0, 464.0, 1e6, 2.0 ** -10, 3 * 2.0 ** -11, 0.3, -2.5])
    want = [0x38, 0x38, 0x3A, 0x7E, 0x7E, 0x7E, 0x00, 0x01, 0x2A, 0xC2]
    # the first four and 0.3 / 2^-10 / 3*2^-11 were measured on the MI355X's
    # v_cvt_pk_fp8_f32 (scripts/probe_mx.py); 464 rounds to 448 there too
    np.testing.assert_array_equal(e4m3_encode(x), np.array(want, np.uint8))


def test_roundtrip_error_bound():
    rng = np.random.default_rng(0)
    x = rng.standard_normal((7, 256)) * np.exp(rng.uniform(-8, 8, (7, 1)))
    q, s = mx_quantize(x)
    y = mx_dequantize(q, s)
    xa = np.abs(x.reshape(7, 8, 32))
    err = np.abs((y - x).reshape(7, 8, 32))
    scale = 2.0 ** (s.astype(np.int64) - 127)[:, :, None]
    # e4m3 has 3 mantissa bits: |err| <= 2^-4 |x| for normals, plus the subnormal
    # spacing 2^-9 scale; values above 448 scale saturate (OCP MX clamps)
    sat = np.maximum(xa - 448 * scale, 0)
    assert np.all(err <= xa * 2.0 ** -4 + scale * 2.0 ** -10 + sat + 1e-300)
    assert np.all(s >= 1) and np.all(s <= 253)
    z, zs = mx_quantize(np.zeros((1, 32)))
    assert not z.any() and zs[0, 0] == 127


def test_oracle_mx_qdq_matches_numpy():
    """the C oracle's MXFP8 quantise-dequantise (its fp8 network emulation) equals
    the numpy restatement bit for bit"""
    import oracle
    rng = np.random.default_rng(3)
    x = (rng.standard_normal((40, 256)) * np.exp(rng.uniform(-10, 10, (40, 1)))).astype(np.float32)
    x[0, :32] = 0
    x[1, 5] = 448.0 * 2 ** 7
    q, s = mx_quantize(x)
    np.testing.assert_array_equal(oracle.mx_qdq_rows(x), mx_dequantize(q, s).astype(np.float32))
