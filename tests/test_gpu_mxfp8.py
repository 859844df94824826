"""MXFP8 (OCP e4m3 + E8M0 per-32 block scales) path of kf_ops.h on the GPU:
kf_quant_mxfp8 bit-exact against the numpy restatement (tests/mx_ref.py), the
MXFP8 GEMM (v_mfma_scale_f32_16x16x128_f8f6f4) against a float64 product of the
dequantised operands, and the GEMM epilogue's out8 copy bit-exact on values the
fp16 output represents exactly.

GEMM tolerance: the products of dequantised operands are exact in fp32, so only
the fp32 accumulation and the final fp16 store round:
|d| <= 2 ulp_fp16(|c|) + K 2^-23 sum|a b|.
"""
import ctypes as C

import numpy as np
import pytest

from mx_ref import mx_dequantize, mx_quantize

pytestmark = pytest.mark.gpu


def h(a):
    return np.asarray(a, np.float32).astype(np.float16)


def ulp16(x):
    return np.spacing(np.abs(np.asarray(x, np.float32)).astype(np.float16)).astype(np.float64)


def quant_gpu(kf, x, transpose=False):
    """x fp16 [R, Cc] (transpose: quantise columns) -> (codes, scales) via kf_quant_mxfp8"""
    x = h(x)
    rows, cols = (x.shape[1], x.shape[0]) if transpose else x.shape
    cpad = (cols + 127) // 128 * 128
    src = kf.upload_fp16(x)
    q = kf.DeviceBuffer(rows * cpad)
    sc = kf.DeviceBuffer(rows * cpad // 32)
    kf.check(kf.core.kf_quant_mxfp8(src.ptr, x.shape[1], rows, cols, int(transpose), q.ptr, cpad, sc.ptr,
                                    cpad // 32), "quant")
    kf.sync()
    codes = np.frombuffer(kf.read_fp16(q.ptr, (rows * cpad // 2,)).tobytes(), np.uint8).reshape(rows, cpad)
    scales = np.frombuffer(kf.read_fp16(sc.ptr, (rows * cpad // 64,)).tobytes(), np.uint8).reshape(rows, cpad // 32)
    return codes, scales, (q, sc, cpad)


@pytest.mark.parametrize("transpose", [False, True])
def test_quantiser_bit_exact(gpu, transpose):
    kf = gpu
    rng = np.random.default_rng(1 + transpose)
    x = rng.standard_normal((96, 200)) * np.exp(rng.uniform(-6, 6, (96, 1)))
    x[3, :40] = 0.0                     # an all-zero block
    x[5, 7] = 60000.0                   # a block whose amax is near the fp16 top
    x[6, :32] = 2.0 ** -20              # fp16 subnormals
    xh = h(x)
    codes, scales, _ = quant_gpu(kf, xh.T.copy() if transpose else xh, transpose)
    src = xh.astype(np.float32)
    pad = np.zeros((96, 256), np.float32)
    pad[:, :200] = src
    rq, rs = mx_quantize(pad)
    np.testing.assert_array_equal(codes, rq)
    np.testing.assert_array_equal(scales, rs)
    assert not codes[:, 200:].any()


def mx_operand(kf, x, *, splice=None):
    """quantise x [rows, K] on the GPU; returns (KfOperand builder args, dequantised float64)"""
    codes, scales, (q, sc, cpad) = quant_gpu(kf, x)
    deq = mx_dequantize(codes, scales)
    return q, sc, cpad, deq


def gemm_check(got, a, b, bias=None, relu=False):
    ref = a @ b
    if bias is not None:
        ref = ref + bias
    bound = 2 * ulp16(ref) + a.shape[1] * 2.0 ** -23 * (np.abs(a) @ np.abs(b)) + 1e-6
    if relu:
        ref = np.maximum(ref, 0)
    err = np.abs(got.astype(np.float64) - ref)
    assert np.all(err <= bound), float(np.max(err - bound))


@pytest.mark.parametrize("M,N,K", [(300, 320, 256), (513, 512, 384), (64, 3080, 256), (260, 128, 640)])
def test_mxfp8_gemm_plain(gpu, M, N, K):
    kf = gpu
    rng = np.random.default_rng(M + N + K)
    x = rng.standard_normal((M, K)) * 2
    w = rng.standard_normal((N, K)) * 0.05            # B stored [N][K] (k-contiguous)
    qa, sa, lda, a = mx_operand(kf, x)
    qb, sb, ldb, b = mx_operand(kf, w)
    A = kf.operand(qa.ptr, lda, M, K, 1, scales=sa.ptr, lds=lda // 32)
    B = kf.operand(qb.ptr, ldb, N, K, 1, scales=sb.ptr, lds=ldb // 32)
    y = kf.DeviceBuffer(M * N * 2)
    bias = h(rng.standard_normal(N) * 0.1)
    db = kf.upload_fp16(bias)
    E = kf.KfEpilogue(out=y.ptr, ldo=N, alpha=1.0, bias=db.ptr, relu=1)
    kf.check(kf.core.kf_gemm_fused(M, N, K, C.byref(A), C.byref(B), C.byref(E)), "mxfp8 gemm")
    kf.sync()
    gemm_check(kf.read_fp16(y.ptr, (M, N)), a, b.T, bias.astype(np.float64), relu=True)


def test_mxfp8_gemm_time_splice(gpu):
    """TDNN-F linear shape: A = [x(t-3) | x(t)] with clamped edges (forward.go:745-790)"""
    kf = gpu
    rng = np.random.default_rng(7)
    T, d, N = 333, 256, 320
    x = rng.standard_normal((T, d))
    w = rng.standard_normal((N, 2 * d)) * 0.05
    qx, sx, ldx, xd = mx_operand(kf, x)
    qb, sb, ldb, b = mx_operand(kf, w)
    A = kf.operand(qx.ptr, ldx, T, 2 * d, 1, nparts=2, part_width=d, tpolicy=1, dt=(-3, 0),
                   scales=sx.ptr, lds=ldx // 32)
    B = kf.operand(qb.ptr, ldb, N, 2 * d, 1, scales=sb.ptr, lds=ldb // 32)
    y = kf.DeviceBuffer(T * N * 2)
    E = kf.KfEpilogue(out=y.ptr, ldo=N, alpha=1.0)
    kf.check(kf.core.kf_gemm_fused(T, N, 2 * d, C.byref(A), C.byref(B), C.byref(E)), "mxfp8 splice")
    kf.sync()
    a = np.concatenate([xd[np.clip(np.arange(T) - 3, 0, T - 1)], xd], 1)
    gemm_check(kf.read_fp16(y.ptr, (T, N)), a, b.T)


def test_mxfp8_rejects_mixed_formats(gpu):
    kf = gpu
    qa, sa, lda, _ = mx_operand(kf, np.ones((16, 128)))
    A = kf.operand(qa.ptr, lda, 16, 128, 1, scales=sa.ptr, lds=lda // 32)
    wb = kf.upload_fp16(np.ones((128, 64), np.float16))
    B = kf.operand(wb.ptr, 64, 128, 64, 0)
    y = kf.DeviceBuffer(16 * 64 * 2)
    E = kf.KfEpilogue(out=y.ptr, ldo=64, alpha=1.0)
    assert kf.core.kf_gemm_fused(16, 64, 128, C.byref(A), C.byref(B), C.byref(E)) != 0
    assert b"MXFP8" in kf.core.kf_last_error()
    kf.core.kf_clear_error()


@pytest.mark.parametrize("N", [256, 320, 96])
def test_epilogue_out8_bit_exact(gpu, N):
    """an fp16 GEMM whose outputs are small integers (exact in fp16 and fp32) also
    writes the MXFP8 copy; it must equal the numpy quantisation of the fp16 output"""
    kf = gpu
    rng = np.random.default_rng(N)
    M, K = 200, 64
    x = h(rng.integers(-3, 4, (M, K)))
    w = h(rng.integers(-2, 3, (K, N)))
    x[7] = 0  # an all-zero output row -> zero blocks
    dx, dw = kf.upload_fp16(x), kf.upload_fp16(w)
    A = kf.operand(dx.ptr, K, M, K, 1)
    B = kf.operand(dw.ptr, N, K, N, 0)
    y = kf.DeviceBuffer(M * N * 2)
    ld8 = (N + 127) // 128 * 128
    q8 = kf.DeviceBuffer(M * ld8)
    s8 = kf.DeviceBuffer(M * ld8 // 32)
    kf.core.bridge_gpu_memset(q8.ptr, 0, M * ld8)
    kf.core.bridge_gpu_memset(s8.ptr, 0, M * ld8 // 32)
    E = kf.KfEpilogue(out=y.ptr, ldo=N, alpha=1.0, relu=1, out8=q8.ptr, ldo8=ld8, scale8=s8.ptr)
    kf.check(kf.core.kf_gemm_fused(M, N, K, C.byref(A), C.byref(B), C.byref(E)), "out8 gemm")
    kf.sync()
    out = kf.read_fp16(y.ptr, (M, N)).astype(np.float32)
    np.testing.assert_array_equal(out, np.maximum(x.astype(np.float32) @ w.astype(np.float32), 0))
    codes = np.frombuffer(kf.read_fp16(q8.ptr, (M * ld8 // 2,)).tobytes(), np.uint8).reshape(M, ld8)
    scales = np.frombuffer(kf.read_fp16(s8.ptr, (M * ld8 // 64,)).tobytes(), np.uint8).reshape(M, ld8 // 32)
    rq, rs = mx_quantize(out)
    np.testing.assert_array_equal(codes[:, :N], rq)
    np.testing.assert_array_equal(scales[:, :N // 32], rs)
    assert not codes[:, N:].any() and not scales[:, N // 32:].any()  # padding untouched


class _QuantJob(C.Structure):
    _fields_ = [("src", C.c_void_p), ("ld_src", C.c_longlong), ("rows", C.c_int), ("cols", C.c_int),
                ("transpose", C.c_int), ("q", C.c_void_p), ("ldq", C.c_longlong), ("scales", C.c_void_p),
                ("lds", C.c_longlong)]


def test_quantiser_batch_matches_single_calls(gpu):
    """kf_quant_mxfp8_batch (the weight copies after each update, several matrices per
    launch) writes exactly what one kf_quant_mxfp8 call per job writes, for transposed
    (weights) and row (activations) jobs of ragged sizes."""
    kf = gpu
    rng = np.random.default_rng(11)
    shapes = [(96, 200, 1), (320, 256, 1), (37, 130, 0), (1, 8, 0), (160, 64, 1), (50, 264, 0), (9, 3072, 0)]
    jobs, refs, keep = [], [], []
    for rows, cols, tr in shapes:
        x = h(rng.standard_normal((rows, cols)) * np.exp(rng.uniform(-4, 4, (rows, 1))))
        src = x.T.copy() if tr else x
        codes, scales, _ = quant_gpu(kf, src, bool(tr))
        refs.append((codes, scales))
        cpad = (cols + 127) // 128 * 128
        dsrc = kf.upload_fp16(src)
        q, sc = kf.DeviceBuffer(rows * cpad), kf.DeviceBuffer(rows * cpad // 32)
        kf.core.bridge_gpu_memset(q.ptr, 0x5A, rows * cpad)
        keep += [dsrc, q, sc]
        jobs.append(_QuantJob(dsrc.ptr, src.shape[1], rows, cols, tr, q.ptr, cpad, sc.ptr, cpad // 32))
    arr = (_QuantJob * len(jobs))(*jobs)
    kf.core.kf_quant_mxfp8_batch.argtypes = [C.c_int, C.c_void_p]
    kf.check(kf.core.kf_quant_mxfp8_batch(len(jobs), C.cast(arr, C.c_void_p)), "quant batch")
    kf.sync()
    for j, ((rows, cols, tr), (rc, rs)) in enumerate(zip(shapes, refs)):
        cpad = (cols + 127) // 128 * 128
        q, sc = keep[3 * j + 1], keep[3 * j + 2]
        codes = np.frombuffer(kf.read_fp16(q.ptr, (rows * cpad // 2,)).tobytes(), np.uint8).reshape(rows, cpad)
        scales = np.frombuffer(kf.read_fp16(sc.ptr, (rows * cpad // 64,)).tobytes(), np.uint8).reshape(rows, cpad // 32)
        np.testing.assert_array_equal(codes, rc)
        np.testing.assert_array_equal(scales, rs)


@pytest.mark.parametrize("M,N,K,cols", [(767, 320, 512, 1536), (384, 160, 256, 3072)])
def test_mxfp8_gemm_with_edge_row(gpu, M, N, K, cols):
    """kf_gemm_fused_edge: the MXFP8 product's rows 0 .. M-1 equal kf_gemm_fused's bit for bit,
    and row M (written by the last row tile's workgroups) is the fp16 two-part dot product of
    kf_dot2_rows (the TDNN-F affine input gradient's clamped-edge row, network.cpp)."""
    kf = gpu
    rng = np.random.default_rng(M + cols)
    x = rng.standard_normal((M, K)) * 2
    w = rng.standard_normal((N, K)) * 0.05
    qa, sa, lda, a = mx_operand(kf, x)
    qb, sb, ldb, b = mx_operand(kf, w)
    A = kf.operand(qa.ptr, lda, M, K, 1, scales=sa.ptr, lds=lda // 32)
    B = kf.operand(qb.ptr, ldb, N, K, 1, scales=sb.ptr, lds=ldb // 32)
    x0, x1 = h(rng.standard_normal(cols)), h(rng.standard_normal(cols))
    W = h(rng.standard_normal((2 * N, cols)) / np.sqrt(cols))
    dx0, dx1, dW = kf.upload_fp16(x0), kf.upload_fp16(x1), kf.upload_fp16(W)
    y1, y2 = kf.DeviceBuffer((M + 1) * N * 2), kf.DeviceBuffer((M + 1) * N * 2)
    E1, E2 = kf.KfEpilogue(out=y1.ptr, ldo=N, alpha=1.0), kf.KfEpilogue(out=y2.ptr, ldo=N, alpha=1.0)
    kf.check(kf.core.kf_gemm_fused(M, N, K, C.byref(A), C.byref(B), C.byref(E1)), "mxfp8 gemm")
    kf.check(kf.core.kf_dot2_rows(y1.ptr + M * N * 2, dx0.ptr, dx1.ptr, dW.ptr, N, cols), "dot2")
    kf.check(kf.core.kf_gemm_fused_edge(M, N, K, C.byref(A), C.byref(B), C.byref(E2), y2.ptr + M * N * 2,
                                        dx0.ptr, dx1.ptr, dW.ptr, cols), "mxfp8 gemm + edge row")
    kf.sync()
    g1, g2 = kf.read_fp16(y1.ptr, (M + 1, N)), kf.read_fp16(y2.ptr, (M + 1, N))
    assert np.array_equal(g1[:M].view(np.uint16), g2[:M].view(np.uint16))
    W64 = W.astype(np.float64)
    ref = W64[:N] @ x0.astype(np.float64) + W64[N:] @ x1.astype(np.float64)
    mag = np.abs(W64[:N]) @ np.abs(x0.astype(np.float64)) + np.abs(W64[N:]) @ np.abs(x1.astype(np.float64))
    tol = 2 * cols * 2.0 ** -23 * mag + np.abs(ref) * 2.0 ** -10 + 2.0 ** -24
    for g in (g1[M], g2[M]):
        assert np.all(np.abs(g.astype(np.float64) - ref) <= tol)
