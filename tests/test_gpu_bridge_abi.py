"""The go/kaldibridge ABI (kaldi_*, libkaldi_fp16_cgo.so) and the CNN launch
wrappers (launch_*, cnn_fp16.h) against numpy restatements of
cpp/src/cgo_interface.cu and cpp/cuda/cnn_kernels.cu.

Tolerances: fp16 storage, fp32 accumulation. GEMM elements obey the SURVEY §8c
bound |d| <= 2 ulp_fp16(|c|) + K 2^-23 sum|a b|; element-wise ops are checked at
1 fp16 ulp of the fp32-computed value (one RNE store); reductions at 2 ulps.
"""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def kb(gpu):
    from kfp16 import bridge_abi
    return bridge_abi


def h(a):
    return np.asarray(a, np.float32).astype(np.float16).astype(np.float32)


def ulp16(x):
    x = np.abs(np.asarray(x, np.float32)).astype(np.float16)
    return (np.spacing(x).astype(np.float32))


def assert_ulps(got, ref, n=1.0, floor=0.0):
    got = np.asarray(got, np.float32)
    ref = np.asarray(ref, np.float64)
    tol = n * ulp16(ref) + floor
    bad = np.abs(got - ref) > tol
    assert not bad.any(), (np.argwhere(bad)[:5], got[bad][:5], ref[bad][:5])


# ---------------------------------------------------------------- kaldi_*
def test_tensor_roundtrip_rne(kb):
    rng = np.random.default_rng(0)
    x = (rng.standard_normal((37, 19)) * 10).astype(np.float32)
    x[0, :4] = [60000.0, -1e-8, 65519.0, 2.0 ** -25]
    t = kb.Tensor.from_numpy(x)
    assert (t.rows, t.cols) == (37, 19)
    assert kb.cgo.kaldi_tensor_size(t.h) == 37 * 19
    np.testing.assert_array_equal(t.numpy(), x.astype(np.float16).astype(np.float32))
    z = kb.Tensor(5, 3, "zeros").numpy()
    o = kb.Tensor(5, 3, "ones").numpy()
    assert not z.any() and (o == 1).all()
    # count is clamped to the tensor size (cgo_interface.cu:162-165)
    big = np.arange(100, dtype=np.float32)
    t2 = kb.Tensor(3, 3)
    kb.cgo.kaldi_tensor_copy_from_host_fp32(t2.h, big.ctypes.data_as(C.POINTER(C.c_float)), 100)
    np.testing.assert_array_equal(t2.numpy().ravel(), big[:9])


@pytest.mark.parametrize("ta,tb", [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize("M,N,K", [(64, 512, 40), (1500, 512, 40), (37, 29, 13), (128, 96, 256)])
def test_gemm(kb, ta, tb, M, N, K):
    rng = np.random.default_rng(M + N + K + 2 * ta + tb)
    A = h(rng.standard_normal((K, M) if ta else (M, K)))
    B = h(rng.standard_normal((N, K) if tb else (K, N)))
    C0 = h(rng.standard_normal((M, N)))
    alpha, beta = 0.7, 0.3
    ctx = kb.cgo.kaldi_cublas_create()
    kb.cgo.kaldi_cublas_enable_tensor_cores(ctx)
    tA, tB, tC = kb.Tensor.from_numpy(A), kb.Tensor.from_numpy(B), kb.Tensor.from_numpy(C0)
    kb.cgo.kaldi_gemm(ctx, tA.h, tB.h, tC.h, alpha, beta, ta, tb)
    assert kb.last_error() is None
    got = tC.numpy()
    kb.cgo.kaldi_cublas_destroy(ctx)
    a = (A.T if ta else A).astype(np.float64)
    b = (B.T if tb else B).astype(np.float64)
    ah, bh = float(np.float16(alpha)), float(np.float16(beta))  # half alpha/beta
    ref = ah * (a @ b) + bh * C0
    bound = 2 * ulp16(ref) + K * 2.0 ** -23 * (np.abs(a) @ np.abs(b)) * ah + 1e-7
    assert np.all(np.abs(got - ref) <= bound), float(np.max(np.abs(got - ref) - bound))


def test_gemm_shape_mismatch_sets_error(kb):
    ctx = kb.cgo.kaldi_cublas_create()
    a, b, c = kb.Tensor(4, 8), kb.Tensor(9, 8), kb.Tensor(4, 8)
    kb.cgo.kaldi_clear_error()
    kb.cgo.kaldi_gemm(ctx, a.h, b.h, c.h, 1.0, 0.0, 0, 0)
    assert "mismatch" in kb.last_error()
    kb.cgo.kaldi_clear_error()
    kb.cgo.kaldi_gemm(None, a.h, b.h, c.h, 1.0, 0.0, 0, 0)
    assert kb.last_error() == "null pointer in GEMM"
    kb.cgo.kaldi_clear_error()
    assert kb.last_error() is None
    kb.cgo.kaldi_cublas_destroy(ctx)


def test_activations_add_scale(kb):
    rng = np.random.default_rng(3)
    x = h(rng.standard_normal((33, 65)) * 3)
    y = h(rng.standard_normal((33, 65)))
    for fn, ref in [("kaldi_relu", np.maximum(x, 0)), ("kaldi_sigmoid", 1 / (1 + np.exp(-x.astype(np.float64)))),
                    ("kaldi_tanh", np.tanh(x.astype(np.float64)))]:
        t = kb.Tensor.from_numpy(x)
        getattr(kb.cgo, fn)(t.h)
        assert_ulps(t.numpy(), ref, 1.0, 1e-7)
    t = kb.Tensor.from_numpy(x)
    kb.cgo.kaldi_scale(t.h, 0.37)
    assert_ulps(t.numpy(), x.astype(np.float64) * np.float32(0.37), 1.0, 1e-8)
    t, u = kb.Tensor.from_numpy(x), kb.Tensor.from_numpy(y)
    kb.cgo.kaldi_add(t.h, u.h)
    np.testing.assert_array_equal(t.numpy(), h(x + y))
    kb.cgo.kaldi_clear_error()
    kb.cgo.kaldi_add(t.h, kb.Tensor(2, 2).h)  # b smaller than a: refused
    assert "add" in kb.last_error()
    kb.cgo.kaldi_clear_error()


@pytest.mark.parametrize("cols", [7, 3080, 300])
def test_softmax_two_roundings(kb, cols):
    rng = np.random.default_rng(cols)
    x = h(rng.standard_normal((17, cols)) * 4)
    t = kb.Tensor.from_numpy(x)
    kb.cgo.kaldi_softmax(t.h)
    e = np.exp(x.astype(np.float64) - x.max(1, keepdims=True))
    ref = h(e) / e.sum(1, keepdims=True)  # fp16(exp) / fp32 sum of unrounded exps
    assert_ulps(t.numpy(), ref, 1.0, 1e-7)


# ---------------------------------------------------------------- launch_*
def dev(kf, a):
    return kf.upload_fp16(np.asarray(a, np.float16))


def out_buf(kf, n, nbytes=2):
    b = kf.DeviceBuffer(n * nbytes)
    kf.core.bridge_gpu_memset(b.ptr, 0, n * nbytes)
    return b


def conv1d_ref(x, w, b, stride, pad, dil):
    B, Ti, Ci = x.shape
    Co, _, K = w.shape
    To = (Ti + 2 * pad - dil * (K - 1) - 1) // stride + 1
    out = np.zeros((B, To, Co))
    for k in range(K):
        ti = np.arange(To) * stride - pad + k * dil
        ok = (ti >= 0) & (ti < Ti)
        xs = np.zeros((B, To, Ci))
        xs[:, ok] = x[:, ti[ok]]
        out += xs @ w[:, :, k].T.astype(np.float64)
    if b is not None:
        out += b
    return out


@pytest.mark.parametrize("stride,pad,dil", [(1, 1, 1), (2, 0, 1), (1, 2, 2)])
def test_conv1d_forward_backward(gpu, kb, stride, pad, dil):
    kf = gpu
    rng = np.random.default_rng(stride * 10 + pad + dil)
    B, Ti, Ci, Co, K = 3, 23, 12, 10, 3
    x = h(rng.standard_normal((B, Ti, Ci)))
    w = h(rng.standard_normal((Co, Ci, K)) * 0.3)
    bias = h(rng.standard_normal(Co) * 0.1)
    To = (Ti + 2 * pad - dil * (K - 1) - 1) // stride + 1
    dx, dw, db = dev(kf, x), dev(kf, w), dev(kf, bias)
    y = out_buf(kf, B * To * Co)
    kb.core.launch_conv1d_forward_fp16(dx.ptr, dw.ptr, db.ptr, y.ptr, B, Ti, Ci, Co, K, stride, pad, dil, None)
    kf.sync()
    ref = conv1d_ref(x, w, bias, stride, pad, dil)
    got = kf.read_fp16(y.ptr, (B, To, Co))
    assert_ulps(got, ref, 2.0, 1e-3)
    # backward: exact gradients of the forward (float64 via the adjoint)
    g = h(rng.standard_normal((B, To, Co)))
    dg = dev(kf, g)
    gi, gw, gb = out_buf(kf, B * Ti * Ci), out_buf(kf, Co * Ci * K), out_buf(kf, Co)
    kb.core.launch_conv1d_backward_fp16(dx.ptr, dg.ptr, dw.ptr, gi.ptr, gw.ptr, gb.ptr, B, Ti, Ci, Co, K,
                                        stride, pad, dil, None)
    kf.sync()
    ref_gi = np.zeros((B, Ti, Ci))
    ref_gw = np.zeros((Co, Ci, K))
    for k in range(K):
        ti = np.arange(To) * stride - pad + k * dil
        ok = (ti >= 0) & (ti < Ti)
        np.add.at(ref_gi, (slice(None), ti[ok]), g[:, ok] @ w[:, :, k].astype(np.float64))
        ref_gw[:, :, k] = np.einsum("bto,bti->oi", g[:, ok].astype(np.float64), x[:, ti[ok]])
    assert_ulps(kf.read_fp16(gi.ptr, (B, Ti, Ci)), ref_gi, 2.0, 1e-3)
    assert_ulps(kf.read_fp16(gw.ptr, (Co, Ci, K)), ref_gw, 2.0, 1e-3)
    assert_ulps(kf.read_fp16(gb.ptr, (Co,)), g.sum((0, 1)), 2.0, 1e-3)


def test_maxpool_forward_backward(gpu, kb):
    kf = gpu
    rng = np.random.default_rng(5)
    B, Ti, Cc, K, S = 2, 17, 9, 3, 2
    x = h(rng.standard_normal((B, Ti, Cc)))
    x[0, 0:3, 0] = 1.0  # ties: the first maximum wins
    To = (Ti - K) // S + 1
    dx = dev(kf, x)
    y, idx = out_buf(kf, B * To * Cc), out_buf(kf, B * To * Cc, 4)
    kb.core.launch_maxpool1d_forward_fp16(dx.ptr, y.ptr, idx.ptr, B, Ti, Cc, K, S, None)
    kf.sync()
    win = np.stack([x[:, np.arange(To) * S + k] for k in range(K)], 0)
    ref_idx = np.argmax(win, 0) + (np.arange(To) * S)[None, :, None]
    np.testing.assert_array_equal(kf.read_fp16(y.ptr, (B, To, Cc)), win.max(0))
    got_idx = np.frombuffer(kf.read_f32(idx.ptr, (B * To * Cc,)).tobytes(), np.int32).reshape(B, To, Cc)
    np.testing.assert_array_equal(got_idx, ref_idx)
    assert got_idx[0, 0, 0] == 0
    g = h(rng.standard_normal((B, To, Cc)))
    dg = dev(kf, g)
    gi = out_buf(kf, B * Ti * Cc)
    kb.core.launch_maxpool1d_backward_fp16(dg.ptr, idx.ptr, gi.ptr, B, Ti, To, Cc, None)
    kf.sync()
    ref = np.zeros((B, Ti, Cc), np.float32)
    for b in range(B):  # fp16 accumulation in time order
        for t in range(To):
            for c in range(Cc):
                ref[b, ref_idx[b, t, c], c] = h(ref[b, ref_idx[b, t, c], c] + g[b, t, c])
    np.testing.assert_array_equal(kf.read_fp16(gi.ptr, (B, Ti, Cc)), ref)


def test_stats_pooling_and_norms(gpu, kb):
    kf = gpu
    rng = np.random.default_rng(6)
    B, T, Cc = 3, 41, 24
    x = h(rng.standard_normal((B, T, Cc)) * 2 + 0.5)
    dx = dev(kf, x)
    y = out_buf(kf, B * 2 * Cc)
    kb.core.launch_stats_pooling_fp16(dx.ptr, y.ptr, B, T, Cc, None)
    kf.sync()
    xd = x.astype(np.float64)
    ref = np.concatenate([xd.mean(1), np.sqrt(xd.var(1) + 1e-10)], 1)
    assert_ulps(kf.read_fp16(y.ptr, (B, 2 * Cc)), ref, 2.0, 1e-6)
    # batchnorm1d, training then inference (cnn_kernels.cu:236-312)
    gamma, beta = h(rng.uniform(0.5, 1.5, Cc)), h(rng.standard_normal(Cc) * 0.1)
    rm, rv = h(rng.standard_normal(Cc) * 0.1), h(rng.uniform(0.5, 2, Cc))
    dgm, dbt, drm, drv = dev(kf, gamma), dev(kf, beta), dev(kf, rm), dev(kf, rv)
    out, sm, si = out_buf(kf, B * T * Cc), out_buf(kf, Cc), out_buf(kf, Cc)
    kb.core.launch_batchnorm1d_forward_fp16(dx.ptr, dgm.ptr, dbt.ptr, drm.ptr, drv.ptr, out.ptr, sm.ptr,
                                            si.ptr, B, T, Cc, 0.1, 1e-5, True, None)
    kf.sync()
    mean, var = xd.reshape(-1, Cc).mean(0), xd.reshape(-1, Cc).var(0)
    inv = 1 / np.sqrt(var + 1e-5)
    assert_ulps(kf.read_fp16(out.ptr, (B, T, Cc)), (xd - mean) * inv * gamma + beta, 2.0, 1e-5)
    assert_ulps(kf.read_fp16(sm.ptr, (Cc,)), mean, 1.0, 1e-6)
    assert_ulps(kf.read_fp16(si.ptr, (Cc,)), inv, 1.0, 1e-6)
    assert_ulps(kf.read_fp16(drm.ptr, (Cc,)), rm * 0.9 + mean * 0.1, 1.0, 1e-6)
    assert_ulps(kf.read_fp16(drv.ptr, (Cc,)), rv * 0.9 + var * 0.1, 1.0, 1e-6)
    rm2, rv2 = kf.read_fp16(drm.ptr, (Cc,)), kf.read_fp16(drv.ptr, (Cc,))
    kb.core.launch_batchnorm1d_forward_fp16(dx.ptr, dgm.ptr, dbt.ptr, drm.ptr, drv.ptr, out.ptr, None,
                                            None, B, T, Cc, 0.1, 1e-5, False, None)
    kf.sync()
    ref = (xd - rm2) / np.sqrt(rv2.astype(np.float64) + 1e-5) * gamma + beta
    assert_ulps(kf.read_fp16(out.ptr, (B, T, Cc)), ref, 2.0, 1e-5)
    np.testing.assert_array_equal(kf.read_fp16(drm.ptr, (Cc,)), rm2)  # inference leaves stats
    # layernorm over channels
    kb.core.launch_layernorm_forward_fp16(dx.ptr, dgm.ptr, dbt.ptr, out.ptr, B, T, Cc, 1e-5, None)
    kf.sync()
    mu = xd.mean(2, keepdims=True)
    ref = (xd - mu) / np.sqrt(xd.var(2, keepdims=True) + 1e-5) * gamma + beta
    assert_ulps(kf.read_fp16(out.ptr, (B, T, Cc)), ref, 2.0, 1e-4)


def test_depthwise_pointwise(gpu, kb):
    kf = gpu
    rng = np.random.default_rng(7)
    B, Ti, Cc, K, S, P, Co = 2, 19, 16, 5, 2, 2, 24
    x = h(rng.standard_normal((B, Ti, Cc)))
    w = h(rng.standard_normal((Cc, K)) * 0.5)
    bias = h(rng.standard_normal(Cc) * 0.1)
    To = (Ti + 2 * P - K) // S + 1
    dx, dw, db = dev(kf, x), dev(kf, w), dev(kf, bias)
    y = out_buf(kf, B * To * Cc)
    kb.core.launch_depthwise_conv1d_fp16(dx.ptr, dw.ptr, db.ptr, y.ptr, B, Ti, Cc, K, S, P, None)
    kf.sync()
    ref = np.zeros((B, To, Cc)) + bias
    for k in range(K):
        ti = np.arange(To) * S - P + k
        ok = (ti >= 0) & (ti < Ti)
        ref[:, ok] += x[:, ti[ok]] * w[:, k]
    assert_ulps(kf.read_fp16(y.ptr, (B, To, Cc)), ref, 2.0, 1e-4)
    wp = h(rng.standard_normal((Co, Cc)) * 0.3)
    bp = h(rng.standard_normal(Co) * 0.1)
    dwp, dbp = dev(kf, wp), dev(kf, bp)
    y2 = out_buf(kf, B * Ti * Co)
    kb.core.launch_pointwise_conv1d_fp16(dx.ptr, dwp.ptr, dbp.ptr, y2.ptr, B, Ti, Cc, Co, None)
    kf.sync()
    ref2 = x.astype(np.float64) @ wp.T.astype(np.float64) + bp
    assert_ulps(kf.read_fp16(y2.ptr, (B, Ti, Co)), ref2, 2.0, 1e-4)
