"""Halo-resident convolution (conv_halo_kernel, taken by kf_gemm_fused for conv
im2col / col2im operands with 64-channel parts) against a float64 im2col GEMM.

Covers every CNN-TDNN conv shape class: 1, 2 and 4 channel chunks (single and
double halo images), height stride 2 (parity-de-interleaved halo), the
residue-split input gradient of a strided conv (network.cpp), partial last tiles
(T not a multiple of the tile's frames) and the fused bias/ReLU/mask epilogue."""
import ctypes as C

import numpy as np
import pytest

from test_gpu_kernels import _check, _h, im2col

pytestmark = pytest.mark.gpu

OFFS = [(a, b) for a in (-1, 0, 1) for b in (-1, 0, 1)]


def _col2im_ref(dP, T, hin, hout, sub, fin):
    ref = np.zeros((T, hin, fin))
    for o, (dt, dh) in enumerate(OFFS):
        for t in range(T):
            ts = t + dt
            if not 0 <= ts < T:
                continue
            for h in range(hout):
                hs = h * sub + dh
                if 0 <= hs < hin:
                    ref[ts, hs] += dP[t * hout + h, o * fin:(o + 1) * fin]
    return ref.reshape(T * hin, fin)


# (hin, fin, hout, sub, fout, T): cnn2..cnn6 shape classes at small T
SHAPES = [(40, 64, 40, 1, 64, 37), (40, 64, 20, 2, 128, 23), (20, 128, 20, 1, 128, 29),
          (20, 128, 10, 2, 256, 19), (10, 256, 10, 1, 256, 41), (10, 256, 10, 1, 256, 3)]
# stride 2 with an odd output height: no halo row pitch = hout (mod 8) exists, so the
# pad search must give up (it looped forever before r5) and keep the unpadded pitch
ODD = [(10, 64, 5, 2, 64, 13), (18, 128, 9, 2, 128, 7)]


@pytest.mark.parametrize("hin,fin,hout,sub,fout,T", SHAPES + ODD)
def test_conv_halo_forward(gpu, hin, fin, hout, sub, fout, T):
    kf = gpu
    rng = np.random.default_rng(hin * fin + T)
    x = _h(rng.standard_normal((T, hin * fin)))
    W = _h(rng.standard_normal((9 * fin, fout)) / 16)
    bias = _h(rng.uniform(-0.5, 0.5, fout))
    dx, dW, db = kf.upload_fp16(x), kf.upload_fp16(W), kf.upload_fp16(bias)
    M, K = T * hout, 9 * fin
    out = kf.DeviceBuffer(M * fout * 2)
    mask = kf.DeviceBuffer(M * fout // 8 + 64)
    a = kf.operand(dx.ptr, hin * fin, M, K, 1, nparts=9, part_width=fin, T=T, hout=hout, hsrc=hin,
                   hmul=sub, hdiv=1, tpolicy=0, dt=[o[0] for o in OFFS], dh=[o[1] for o in OFFS])
    b = kf.operand(dW.ptr, fout, K, fout, 0)
    e = kf.KfEpilogue(out=out.ptr, ldo=fout, alpha=1.0, bias=db.ptr, relu=1, mask_out=mask.ptr)
    kf.check(kf.core.kf_gemm_fused(M, fout, K, C.byref(a), C.byref(b), C.byref(e)))
    pre = im2col(x.astype(np.float64), T, hin, fin, hout, sub, OFFS) @ W.astype(np.float64)
    pre += bias.astype(np.float64)
    got = kf.read_fp16(out.ptr, (M, fout)).astype(np.float64)
    _check(got, np.maximum(pre, 0), K)
    bits = np.unpackbits(np.frombuffer(kf.read_fp16(mask.ptr, (M * fout // 16,)).tobytes(), np.uint8),
                         bitorder="little").reshape(M, fout)
    decided = np.abs(pre) > 1e-2 * np.abs(pre).max()
    assert np.array_equal(bits[decided], (pre[decided] > 0).astype(np.uint8))


@pytest.mark.parametrize("hin,fin,hout,sub,fout,T", SHAPES + ODD)
def test_conv_halo_input_grad(gpu, hin, fin, hout, sub, fout, T):
    """dx = col2im(dz . W^T): one transposed conv (stride 1) or one GEMM per input
    height residue (stride 2), built exactly as host/network.cpp builds them"""
    kf = gpu
    rng = np.random.default_rng(7 + hin * fout + T)
    W = _h(rng.standard_normal((9 * fin, fout)) / 16)
    M = T * hout
    dz = _h(rng.standard_normal((M, fout)))
    dW, ddz = kf.upload_fp16(W), kf.upload_fp16(dz)
    gx = kf.DeviceBuffer(T * hin * fin * 2)
    if sub == 1:
        a2 = kf.operand(ddz.ptr, hout * fout, T * hin, 9 * fout, 1, nparts=9, part_width=fout, T=T,
                        hout=hin, hsrc=hout, hmul=1, hdiv=1, tpolicy=0,
                        dt=[-o[0] for o in OFFS], dh=[-o[1] for o in OFFS])
        b2 = kf.operand(dW.ptr, fout, fin, 9 * fout, 1, nparts=9, part_width=fout, T=9 * fin,
                        dt=[p * fin for p in range(9)])
        e2 = kf.KfEpilogue(out=gx.ptr, ldo=fin, alpha=1.0)
        kf.check(kf.core.kf_gemm_fused(T * hin, fin, 9 * fout, C.byref(a2), C.byref(b2), C.byref(e2)))
    else:
        for pi in range(sub):
            taps = [(o, dt, (pi - dh) // sub) for o, (dt, dh) in enumerate(OFFS) if (pi - dh) % sub == 0]
            np_ = len(taps)
            a2 = kf.operand(ddz.ptr, hout * fout, T * (hin // sub), np_ * fout, 1, nparts=np_,
                            part_width=fout, T=T, hout=hin // sub, hsrc=hout, hmul=1, hdiv=1, tpolicy=0,
                            dt=[-t[1] for t in taps], dh=[t[2] for t in taps])
            b2 = kf.operand(dW.ptr, fout, fin, np_ * fout, 1, nparts=np_, part_width=fout, T=9 * fin,
                            dt=[t[0] * fin for t in taps])
            e2 = kf.KfEpilogue(out=gx.ptr + pi * fin * 2, ldo=sub * fin, alpha=1.0)
            kf.check(kf.core.kf_gemm_fused(T * (hin // sub), fin, np_ * fout, C.byref(a2), C.byref(b2),
                                           C.byref(e2)))
    ref = _col2im_ref(dz.astype(np.float64) @ W.astype(np.float64).T, T, hin, hout, sub, fin)
    _check(kf.read_fp16(gx.ptr, (T * hin, fin)).astype(np.float64), ref, 9 * fout)


# weight gradient (conv_wgrad_halo_kernel, taken by kf_gemm_wgrad for 9-tap im2col
# operands with 64-channel parts): small T (one split, partial last K-step) and
# larger T (many splits over the reduction, K-steps straddling frames)
WSHAPES = SHAPES + [(40, 64, 40, 1, 64, 203), (40, 64, 20, 2, 128, 171), (20, 128, 20, 1, 128, 150),
                    (20, 128, 10, 2, 256, 333), (10, 256, 10, 1, 256, 257)]


@pytest.mark.parametrize("hin,fin,hout,sub,fout,T", WSHAPES)
def test_conv_halo_wgrad(gpu, hin, fin, hout, sub, fout, T):
    kf = gpu
    rng = np.random.default_rng(11 + hin * fout + T)
    x = _h(rng.standard_normal((T, hin * fin)))
    M, K = T * hout, 9 * fin
    dz = _h(rng.standard_normal((M, fout)))
    dx, ddz = kf.upload_fp16(x), kf.upload_fp16(dz)
    gW = kf.DeviceBuffer(K * fout * 4)
    gb = kf.DeviceBuffer(fout * 4)
    a = kf.operand(dx.ptr, hin * fin, M, K, 0, nparts=9, part_width=fin, T=T, hout=hout, hsrc=hin,
                   hmul=sub, hdiv=1, tpolicy=0, dt=[o[0] for o in OFFS], dh=[o[1] for o in OFFS])
    b = kf.operand(ddz.ptr, fout, M, fout, 0)
    kf.check(kf.core.kf_gemm_wgrad(K, fout, M, C.byref(a), C.byref(b), gW.ptr, fout, gb.ptr, 0))
    P = im2col(x.astype(np.float64), T, hin, fin, hout, sub, OFFS)
    _check(kf.read_f32(gW.ptr, (K, fout)), P.T @ dz.astype(np.float64), M)
    _check(kf.read_f32(gb.ptr, (fout,)), dz.astype(np.float64).sum(0), M)
    # accumulate = 1 adds onto the existing gradient
    kf.check(kf.core.kf_gemm_wgrad(K, fout, M, C.byref(a), C.byref(b), gW.ptr, fout, gb.ptr, 1))
    _check(kf.read_f32(gW.ptr, (K, fout)), 2 * (P.T @ dz.astype(np.float64)), M)


@pytest.mark.parametrize("hin,fin,hout,sub,fout,T", [SHAPES[0], SHAPES[3], SHAPES[4]])
def test_conv_halo_out8_bit_exact(gpu, hin, fin, hout, sub, fout, T):
    """The MXFP8 copy of a conv output (the [(t, h) x fout] rows the TDNN-F above reads as
    [t x hout * fout], network.cpp) written by the halo kernel's epilogue: small-integer
    inputs and weights keep every output exact in fp16 and fp32, so the codes and scales
    must equal the numpy quantisation of the fp16 output (tests/mx_ref.py)."""
    from mx_ref import mx_quantize
    kf = gpu
    rng = np.random.default_rng(3 * hin + fout + T)
    x = _h(rng.integers(-1, 2, (T, hin * fin)))
    W = _h(rng.integers(-1, 2, (9 * fin, fout)) * (rng.random((9 * fin, fout)) < 0.3))
    dx, dW = kf.upload_fp16(x), kf.upload_fp16(W)
    M, K = T * hout, 9 * fin
    out = kf.DeviceBuffer(M * fout * 2)
    q8, s8 = kf.DeviceBuffer(M * fout), kf.DeviceBuffer(M * fout // 32)
    kf.core.bridge_gpu_memset(q8.ptr, 0, M * fout)
    kf.core.bridge_gpu_memset(s8.ptr, 0, M * fout // 32)
    a = kf.operand(dx.ptr, hin * fin, M, K, 1, nparts=9, part_width=fin, T=T, hout=hout, hsrc=hin,
                   hmul=sub, hdiv=1, tpolicy=0, dt=[o[0] for o in OFFS], dh=[o[1] for o in OFFS])
    b = kf.operand(dW.ptr, fout, K, fout, 0)
    e = kf.KfEpilogue(out=out.ptr, ldo=fout, alpha=1.0, relu=1, out8=q8.ptr, ldo8=fout, scale8=s8.ptr)
    kf.check(kf.core.kf_gemm_fused(M, fout, K, C.byref(a), C.byref(b), C.byref(e)))
    kf.sync()
    ref = np.maximum(im2col(x.astype(np.float64), T, hin, fin, hout, sub, OFFS) @ W.astype(np.float64), 0)
    got = kf.read_fp16(out.ptr, (M, fout)).astype(np.float32)
    np.testing.assert_array_equal(got, ref.astype(np.float32))
    codes = np.frombuffer(kf.read_fp16(q8.ptr, (M * fout // 2,)).tobytes(), np.uint8).reshape(M, fout)
    scales = np.frombuffer(kf.read_fp16(s8.ptr, (M * fout // 64,)).tobytes(), np.uint8).reshape(M, fout // 32)
    rq, rs = mx_quantize(got)
    np.testing.assert_array_equal(codes, rq)
    np.testing.assert_array_equal(scales, rs)

