"""numpy restatement of the OCP MX (MXFP8, e4m3 + E8M0) quantisation rule of
kf_quant_mxfp8 / the GEMM epilogue's out8 (include/kf_ops.h), for the tests.

Block of 32 values along a row: amax = max|v|; e = floor(log2 amax) - 8 clamped to
[-126, 126] (0 when amax == 0); q = e4m3_rne(clamp(v / 2^e, -448, 448)); scale
byte e + 127. e4m3 is OCP e4m3fn: bias 7, no infinities, 0x7F / 0xFF NaN.
"""
import numpy as np


def e4m3_table():
    v = np.empty(256)
    for code in range(256):
        s = -1.0 if code & 0x80 else 1.0
        e, m = (code >> 3) & 0xF, code & 7
        if e == 15 and m == 7:
            v[code] = np.nan
        elif e == 0:
            v[code] = s * m / 8 * 2.0 ** -6
        else:
            v[code] = s * (1 + m / 8) * 2.0 ** (e - 7)
    return v


E4M3 = e4m3_table()
_POS = E4M3[:127]  # codes 0..126: 0 .. 448 ascending


def e4m3_encode(x):
    """round-to-nearest-even onto e4m3fn codes; |x| <= 448 expected (clamped)"""
    x = np.asarray(x, np.float64)
    a = np.minimum(np.abs(x), 448.0)
    hi = np.clip(np.searchsorted(_POS, a), 0, 126)
    lo = np.clip(hi - 1, 0, 126)
    dlo, dhi = a - _POS[lo], _POS[hi] - a
    pick_hi = (dhi < dlo) | ((dhi == dlo) & (hi % 2 == 0))
    code = np.where(pick_hi, hi, lo).astype(np.uint8)
    code = np.where(np.signbit(x) & (code != 0), code | 0x80, code)
    code = np.where(np.signbit(x) & (code == 0), 0x80, code)  # -0 keeps its sign
    return code.astype(np.uint8)


def mx_quantize(x):
    """x [rows, cols] (cols % 32 == 0) -> (codes uint8 [rows, cols], scale bytes [rows, cols/32])"""
    x = np.asarray(x, np.float32).astype(np.float64)
    rows, cols = x.shape
    xb = x.reshape(rows, cols // 32, 32)
    amax = np.abs(xb).max(2)
    _, e2 = np.frexp(amax)  # amax = m 2^e2, m in [0.5, 1): floor(log2 amax) = e2 - 1
    ex = np.where(amax > 0, e2 - 1 - 8, 0)
    ex = np.clip(ex, -126, 126).astype(np.int64)
    q = e4m3_encode(xb / (2.0 ** ex)[:, :, None]).reshape(rows, cols)
    return q, (ex + 127).astype(np.uint8)


def mx_dequantize(codes, scales):
    rows, cols = codes.shape
    v = E4M3[codes].reshape(rows, cols // 32, 32) * (2.0 ** (scales.astype(np.int64) - 127))[:, :, None]
    return v.reshape(rows, cols)
