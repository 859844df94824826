"""Row-panel fused GEMM (csrc/rowpanel.hip, taken by kf_gemm_fused for K = 160 / 256 / 320
with N % 64 == 0 and k-contiguous weights) against a float64 numpy restatement of the
operand addressing (kf_ops.h) and the fused epilogue (gemm_common.h epilogue8).

Cases follow host/network.cpp's uses: the TDNN-F affine forward (clamped [0, +s] splice
of the bottleneck, bias / ReLU + mask / BN / bypass residual), the linear layer's input
gradient (zero-padded [+s, 0] splice with an edge row, op_wrows weights, residual,
second output masked by the input ReLU bits and scaled), the prefinal big affine (K = 256)
and the stride-0 layer (K = 160), with row counts that leave a partial last block."""
import ctypes as C

import numpy as np
import pytest

from test_gpu_kernels import _h, splice

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def rowpanel_on(gpu):
    """the kernel is off by default (measured slower): force it on here"""
    gpu.core.kf_gemm_debug_rowpanel.argtypes = [C.c_int]
    gpu.core.kf_gemm_debug_rowpanel(1)
    yield
    gpu.core.kf_gemm_debug_rowpanel(-1)


def _rel(a, b):
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


def _bits(kf, ptr, M, N, ld):
    raw = np.frombuffer(kf.read_fp16(ptr, (M * ld // 16 + 1,)).tobytes(), np.uint8)[: M * ld // 8]
    return np.unpackbits(raw, bitorder="little").reshape(M, ld)[:, :N]


@pytest.mark.parametrize("T,bn,N,s", [(1000, 160, 1536, 3), (333, 160, 256, 1), (128, 160, 512, 3),
                                      (77, 160, 64, 3)])
def test_rowpanel_affine_forward(gpu, T, bn, N, s):
    kf = gpu
    rng = np.random.default_rng(T + N)
    x = _h(rng.standard_normal((T, bn)))
    Wt = _h(rng.standard_normal((N, 2 * bn)) / 16)  # k-contiguous weights [N x K]
    bias = _h(rng.uniform(-0.3, 0.3, N))
    scale = rng.uniform(0.5, 1.5, N).astype(np.float32)
    shift = rng.uniform(-0.2, 0.2, N).astype(np.float32)
    res = _h(rng.standard_normal((T, N)))
    dx, dW, db, dr = kf.upload_fp16(x), kf.upload_fp16(Wt), kf.upload_fp16(bias), kf.upload_fp16(res)
    dsc, dsh = kf.upload_f32(scale), kf.upload_f32(shift)
    out = kf.DeviceBuffer(T * N * 2)
    mask = kf.DeviceBuffer(T * N // 8 + 64)
    a = kf.operand(dx.ptr, bn, T, 2 * bn, 1, nparts=2, part_width=bn, tpolicy=1, dt=(0, s))
    b = kf.operand(dW.ptr, 2 * bn, N, 2 * bn, 1)
    e = kf.KfEpilogue(out=out.ptr, ldo=N, alpha=1.0, bias=db.ptr, relu=1, mask_out=mask.ptr, scale=dsc.ptr,
                      shift=dsh.ptr, resid=dr.ptr, ldr=N, resid_alpha=0.66)
    kf.check(kf.core.kf_gemm_fused(T, N, 2 * bn, C.byref(a), C.byref(b), C.byref(e)))
    pre = splice(x.astype(np.float64), (0, s), 1) @ Wt.astype(np.float64).T + bias.astype(np.float64)
    ref = np.maximum(pre, 0) * scale + shift + 0.66 * res.astype(np.float64)
    got = kf.read_fp16(out.ptr, (T, N)).astype(np.float64)
    assert _rel(got, ref) < 2e-3
    decided = np.abs(pre) > 1e-2 * np.abs(pre).max()
    bits = _bits(kf, mask.ptr, T, N, N)
    assert np.array_equal(bits[decided], (pre[decided] > 0).astype(np.uint8))


@pytest.mark.parametrize("T,din,bn,s", [(1000, 1536, 160, 3), (259, 256, 160, 1), (64, 512, 160, 3)])
def test_rowpanel_linear_input_grad(gpu, T, din, bn, s):
    """dx = splice^T(dbott) . W^T as network.cpp builds it: A = dbott spliced [+s, 0] with
    zero padding and the edge row T (the clamped-splice transpose's sum), B = op_wrows"""
    kf = gpu
    rng = np.random.default_rng(T + din)
    dbott = _h(rng.standard_normal((T + 1, bn)))  # row T: the edge sum row
    W = _h(rng.standard_normal((2 * din, bn)) / 16)  # the linear weight [2 din x bn]
    gcur = _h(rng.standard_normal((T, din)))
    scale2 = rng.uniform(0.5, 1.5, din).astype(np.float32)
    mbits = rng.integers(0, 2, (T, din)).astype(np.uint8)
    mpack = np.packbits(mbits, axis=1, bitorder="little")
    dd, dW, dg = kf.upload_fp16(dbott), kf.upload_fp16(W), kf.upload_fp16(gcur)
    ds2 = kf.upload_f32(scale2)
    dm = kf.DeviceBuffer(mpack.nbytes + 64)
    mwords = np.ascontiguousarray(np.pad(mpack.reshape(-1), (0, (-mpack.size) % 4))).view(np.int32)
    kf.check(kf.core.bridge_transfer_int32(dm.ptr, mwords.ctypes.data, mwords.size))
    gout = kf.DeviceBuffer(T * din * 2)
    dzout = kf.DeviceBuffer(T * din * 2)
    a = kf.operand(dd.ptr, bn, T, 2 * bn, 1, nparts=2, part_width=bn, tpolicy=0, dt=(s, 0), edges=[(0, 0, T)])
    b = kf.operand(dW.ptr, bn, din, 2 * bn, 1, nparts=2, part_width=bn, T=2 * din, dt=(0, din))
    e = kf.KfEpilogue(out=gout.ptr, ldo=din, alpha=1.0, resid=dg.ptr, ldr=din, resid_alpha=0.66, out2=dzout.ptr,
                      ldo2=din, scale2=ds2.ptr, mask_in=dm.ptr)
    kf.check(kf.core.kf_gemm_fused(T, din, 2 * bn, C.byref(a), C.byref(b), C.byref(e)))
    d64 = dbott.astype(np.float64)
    p0 = np.where((np.arange(T) + s < T)[:, None], d64[np.clip(np.arange(T) + s, 0, T)], 0.0)
    p0[0] = d64[T]  # edge row of part 0 at t = 0
    A = np.concatenate([p0, d64[:T]], 1)
    Bm = np.concatenate([W[:din], W[din:]], 1).astype(np.float64)  # B'[j][(p, n)] = W[p*din + j][n]
    v = A @ Bm.T + 0.66 * gcur.astype(np.float64)
    assert _rel(kf.read_fp16(gout.ptr, (T, din)).astype(np.float64), v) < 2e-3
    ref2 = v * scale2 * mbits
    assert _rel(kf.read_fp16(dzout.ptr, (T, din)).astype(np.float64), ref2) < 2e-3


@pytest.mark.parametrize("T,K,N", [(1000, 256, 1536), (515, 160, 1536), (300, 320, 64)])
def test_rowpanel_plain(gpu, T, K, N):
    kf = gpu
    rng = np.random.default_rng(T + K + N)
    A = _h(rng.standard_normal((T, K)))
    Wt = _h(rng.standard_normal((N, K)) / 16)
    dA, dW = kf.upload_fp16(A), kf.upload_fp16(Wt)
    out = kf.DeviceBuffer(T * N * 2)
    a = kf.operand(dA.ptr, K, T, K, 1)
    b = kf.operand(dW.ptr, K, N, K, 1)
    e = kf.KfEpilogue(out=out.ptr, ldo=N, alpha=1.0)
    kf.check(kf.core.kf_gemm_fused(T, N, K, C.byref(a), C.byref(b), C.byref(e)))
    ref = A.astype(np.float64) @ Wt.astype(np.float64).T
    assert _rel(kf.read_fp16(out.ptr, (T, N)).astype(np.float64), ref) < 2e-3
