"""The reference's per-op C-ABI (what the Go internal/gpu package calls on every op),
called through ctypes exactly as internal/gpu/ops.go:21-366 and backward_ops.go bind
it, against numpy restatements of the reference kernels' rounding points:

- ops_*            cpp/cuda/ops.cu:26-320, :439-643
- ops_*_backward, ops_transpose, ops_fp16_to_fp32, ops_sgd_update
                   cpp/cuda/backward_wrappers.cu:41-291
- ops_gemm_strided cpp/cuda/ops.cu:402-430
- bridge_batch_*, bridge_host_*   cpp/cuda/bridge.cu:75-113, :177-267
- chain_*_det, chain_workspace_bytes   cpp/cuda/chain_det.cu:24-477, chain.cu:361-366

Counts are ragged (not multiples of 8) and pointers are offset by one fp16 element
so that both the 16-byte vector path and the scalar path of each kernel run; guard
elements around every destination must come back untouched.

Tolerances: data movement (copy, fill, concat/slice, combine, subsample, transpose,
relu, relu-backward, fp16->fp32) and the fp16-arithmetic backward chains
(sigmoid/tanh backward, whose products of two fp16 values are exact in fp32) are
bit-exact. Element-wise math that calls expf/tanhf/sqrtf or may be fma-contracted
by either compiler is held to 1 fp16 ulp of the float64 value. The analytic pins of
cmd/sgdtest/main.go:38-193 and cmd/backtest/main.go:51-213 keep their own
thresholds.
"""
import ctypes as C
import zlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

COUNTS = [1, 7, 8, 9, 1000, 4099]


@pytest.fixture(scope="module")
def ab(gpu):
    from kfp16 import ops_abi
    return ops_abi


def f16(a):
    return np.asarray(a, np.float32).astype(np.float16)


def bits(a):
    return np.asarray(a, np.float16).view(np.uint16)


def ulp_dist(got, ref):
    """distance in fp16 ulps between got (fp16) and ref (float64, rounded to fp16 grid)"""
    g = np.asarray(got, np.float16).astype(np.float64)
    r = np.asarray(ref, np.float64)
    sp = np.spacing(np.abs(r).astype(np.float16)).astype(np.float64)
    return np.abs(g - r) / sp


class Slot:
    """fp16 device array placed `off` elements into a buffer with 8 guard elements of
    sentinel on each side (so unaligned pointers and overruns are both exercised)."""
    SENT = np.float16(-777.0)

    def __init__(self, gpu, data, off=0):
        data = np.ascontiguousarray(data, np.float16).ravel()
        self.n, self.off = data.size, off
        host = np.full(self.n + 16 + off, self.SENT, np.float16)
        host[8 + off:8 + off + self.n] = data
        self.buf = gpu.upload_fp16(host)
        self.gpu = gpu
        self.ptr = self.buf.ptr + 2 * (8 + off)

    def read(self):
        host = self.gpu.read_fp16(self.buf.ptr, (self.n + 16 + self.off,))
        guard = np.concatenate([host[:8 + self.off], host[8 + self.off + self.n:]])
        assert np.all(bits(guard) == bits(np.full(guard.size, self.SENT, np.float16))), "overrun"
        return host[8 + self.off:8 + self.off + self.n]


def rng_for(*k):
    return np.random.default_rng(zlib.crc32(repr(k).encode()))


# ----------------------------------------------------------------- activations
@pytest.mark.parametrize("count", COUNTS)
@pytest.mark.parametrize("off", [0, 1])
def test_relu_clipped_exact(gpu, ab, count, off):
    """kernel_relu / kernel_clipped_relu (ops.cu:26-67): pure selects, bit-exact."""
    x = f16(rng_for("relu", count, off).standard_normal(count) * 3)
    x[:min(count, 2)] = [-0.0, 0.0][:min(count, 2)]
    s = Slot(gpu, x, off)
    assert gpu.core.ops_relu(s.ptr, count) == 0
    ref = np.where(x < 0, np.float16(0), x)
    np.testing.assert_array_equal(bits(s.read()), bits(ref))
    s = Slot(gpu, x, off)
    assert gpu.core.ops_clipped_relu(s.ptr, count, 1.5) == 0
    ref = f16(np.maximum(0.0, np.minimum(x.astype(np.float32), 1.5)))
    np.testing.assert_array_equal(s.read().astype(np.float32), ref.astype(np.float32))


@pytest.mark.parametrize("count", COUNTS)
@pytest.mark.parametrize("off", [0, 1])
def test_sigmoid_tanh(gpu, ab, count, off):
    """kernel_sigmoid / kernel_tanh (ops.cu:36-54): fp32 math, one RNE store."""
    x = f16(rng_for("sig", count, off).standard_normal(count) * 4)
    xd = x.astype(np.float64)
    for fn, ref in ((gpu.core.ops_sigmoid, 1 / (1 + np.exp(-xd))), (gpu.core.ops_tanh_act, np.tanh(xd))):
        s = Slot(gpu, x, off)
        assert fn(s.ptr, count) == 0
        assert ulp_dist(s.read(), ref).max() <= 1.0


def test_negative_count_is_an_error(gpu, ab):
    s = Slot(gpu, np.zeros(4))
    gpu.core.ops_clear_error()
    assert gpu.core.ops_relu(s.ptr, -1) == -1
    assert b"negative" in gpu.core.ops_last_error()
    assert gpu.core.ops_relu(s.ptr, 0) == 0


# ----------------------------------------------------------------- softmax
def _softmax_ref(x):
    """ops.cu:70-118: e = expf(x - max) stored as fp16, sum over the fp32 e,
    out = fp16(fp16(e) * (1/sum))"""
    xf = x.astype(np.float32)
    e = np.exp((xf - xf.max(1, keepdims=True)).astype(np.float64)).astype(np.float32)
    s = e.sum(1, dtype=np.float64).astype(np.float32)
    inv = (np.float32(1) / s)[:, None]
    return f16(e).astype(np.float64) * inv.astype(np.float64)


@pytest.mark.parametrize("rows,cols", [(1, 1), (3, 7), (17, 40), (5, 3080), (2, 5000)])
def test_softmax_reference_rounding(gpu, ab, rows, cols):
    rng = rng_for("sm", rows, cols)
    x = f16(rng.standard_normal((rows, cols)) * 3)
    x[:, 0] = np.abs(x[:, 0]) + np.float16(0.5)  # a positive max: the reference's int atomicMax is right
    s = Slot(gpu, x)
    assert gpu.core.ops_softmax(s.ptr, rows, cols) == 0
    got = s.read().reshape(rows, cols)
    assert ulp_dist(got, _softmax_ref(x)).max() <= 1.0
    assert np.all(np.abs(got.astype(np.float64).sum(1) - 1) < 2e-3 * np.sqrt(cols) + 1e-3)


@pytest.mark.parametrize("rows,cols", [(3, 7), (9, 40), (4, 3080), (2, 4097)])
def test_log_softmax(gpu, ab, rows, cols):
    """ops.cu:120-166: fp16(x - (max + logf(sum exp(x - max))))."""
    x = f16(rng_for("lsm", rows, cols).standard_normal((rows, cols)) * 3)
    x[:, 0] = np.abs(x[:, 0]) + np.float16(0.5)
    s = Slot(gpu, x)
    assert gpu.core.ops_log_softmax(s.ptr, rows, cols) == 0
    xd = x.astype(np.float64)
    m = xd.max(1, keepdims=True)
    ref = xd - (m + np.log(np.exp(xd - m).sum(1, keepdims=True)))
    assert ulp_dist(s.read().reshape(rows, cols), ref).max() <= 1.0


def test_softmax_all_negative_row_is_finite(gpu, ab):
    """Documented fix (include/ops.h): the reference's int atomicMax on float bits keeps
    its -1e30 seed for an all-negative row and returns NaN; this build returns the
    true softmax."""
    x = f16(-np.arange(1, 9, dtype=np.float32))[None, :]
    s = Slot(gpu, x)
    assert gpu.core.ops_softmax(s.ptr, 1, 8) == 0
    got = s.read().astype(np.float64)
    assert np.all(np.isfinite(got)) and abs(got.sum() - 1) < 4e-3
    assert ulp_dist(got[None], _softmax_ref(x)).max() <= 1.0


# ----------------------------------------------------------------- batchnorm
def _bn_params(rng, D):
    mean = rng.standard_normal(D).astype(np.float32)
    var = (rng.random(D) * 1.5 + 0.5).astype(np.float32)
    gamma = (rng.random(D) + 0.5).astype(np.float32)
    beta = rng.standard_normal(D).astype(np.float32)
    return mean, var, gamma, beta


@pytest.mark.parametrize("T,D", [(1, 1), (13, 37), (64, 128), (7, 1536), (1001, 160), (3, 8)])
def test_batchnorm_forward_and_rms(gpu, ab, T, D):
    """ops.cu:171-204 (inference BN with frozen statistics): one fp16 ulp of the float64
    value, plus the fp32 evaluation's own error where gamma * norm and beta cancel (the
    subtraction, sqrtf, division and fma each round once: <= 2^-21 (|gamma norm| + |beta|))."""
    rng = rng_for("bn", T, D)
    x = f16(rng.standard_normal((T, D)) * 2)
    mean, var, gamma, beta = _bn_params(rng, D)
    dm, dv, dg, db = (gpu.upload_f32(a) for a in (mean, var, gamma, beta))
    eps = 1e-3
    norm = (x.astype(np.float64) - mean) / np.sqrt(var.astype(np.float64) + np.float32(eps))

    def within(got, ref, terms):
        sp = np.spacing(np.abs(ref).astype(np.float16)).astype(np.float64)
        err = np.abs(np.asarray(got, np.float64) - ref)
        assert np.all(err <= sp + 2.0 ** -21 * terms), float(np.max((err - 2.0 ** -21 * terms) / sp))
    s = Slot(gpu, x)
    assert gpu.core.ops_batchnorm_forward(s.ptr, T, D, dm.ptr, dv.ptr, dg.ptr, db.ptr, eps) == 0
    within(s.read().reshape(T, D), gamma * norm + beta, np.abs(gamma * norm) + np.abs(beta))
    s = Slot(gpu, x)
    assert gpu.core.ops_batchnorm_forward_rms(s.ptr, T, D, dm.ptr, dv.ptr, 0.5, eps) == 0
    within(s.read().reshape(T, D), norm * 0.5, np.abs(norm * 0.5))


def test_batchnorm_backward_backtest_pin(gpu, ab):
    """cmd/backtest/main.go:176-213: rows 64, cols 128, gamma U[0.5,1.5), var U[0.5,2),
    eps 1e-5; max rel err <= 0.02 against grad * gamma / sqrt(var + eps). Also 1 ulp of
    the float64 value (backward_wrappers.cu:105-115)."""
    rng = np.random.default_rng(176)
    rows, cols = 64, 128
    g = f16(rng.random((rows, cols)) * 2 - 1)
    gamma = (rng.random(cols) + 0.5).astype(np.float32)
    var = (rng.random(cols) * 1.5 + 0.5).astype(np.float32)
    dgm, dv = gpu.upload_f32(gamma), gpu.upload_f32(var)
    go, gi = Slot(gpu, g), Slot(gpu, np.zeros_like(g))
    assert gpu.core.ops_batchnorm_backward(go.ptr, gi.ptr, dgm.ptr, dv.ptr, 1e-5, rows, cols) == 0
    got = gi.read().reshape(rows, cols).astype(np.float64)
    scale = gamma / np.sqrt(var.astype(np.float64) + np.float32(1e-5))
    ref = g.astype(np.float64) * scale
    rel = np.abs(got - ref) / np.maximum(np.abs(ref), 1e-6)
    assert rel.max() <= 0.02
    assert ulp_dist(got, ref).max() <= 1.0


@pytest.mark.parametrize("rows,cols,off", [(13, 37, 0), (1001, 160, 0), (9, 64, 1)])
def test_batchnorm_backward_shapes(gpu, ab, rows, cols, off):
    """backward_wrappers.cu:105-115 on the scalar kernel (ragged cols, misaligned) and the
    8-column vector kernel (16-byte-granular rows): 1 ulp of grad * gamma / sqrt(var + eps)."""
    rng = rng_for("bnb", rows, cols, off)
    g = f16(rng.standard_normal((rows, cols)))
    gamma = (rng.random(cols) + 0.5).astype(np.float32)
    var = (rng.random(cols) * 1.5 + 0.5).astype(np.float32)
    dgm, dv = gpu.upload_f32(gamma), gpu.upload_f32(var)
    go, gi = Slot(gpu, g, off), Slot(gpu, np.zeros_like(g), off)
    assert gpu.core.ops_batchnorm_backward(go.ptr, gi.ptr, dgm.ptr, dv.ptr, 1e-3, rows, cols) == 0
    ref = g.astype(np.float64) * (gamma / np.sqrt(var.astype(np.float64) + np.float32(1e-3)))
    assert ulp_dist(gi.read().reshape(rows, cols), ref).max() <= 1.0


# ----------------------------------------------------------------- element-wise
@pytest.mark.parametrize("count", COUNTS)
@pytest.mark.parametrize("off", [0, 1])
def test_add_add_scaled(gpu, ab, count, off):
    """ops.cu:207-229: fp32 math on fp16 inputs, one RNE store."""
    rng = rng_for("add", count, off)
    d0, s0 = f16(rng.standard_normal(count)), f16(rng.standard_normal(count))
    src = Slot(gpu, s0, off)
    dst = Slot(gpu, d0, off)
    assert gpu.core.ops_add(dst.ptr, src.ptr, count) == 0
    np.testing.assert_array_equal(bits(dst.read()), bits(f16(d0.astype(np.float32) + s0.astype(np.float32))))
    dst = Slot(gpu, d0, 1 - off)  # mixed alignment: scalar path
    assert gpu.core.ops_add_scaled(dst.ptr, src.ptr, count, 0.7, -1.3) == 0
    ref = np.float32(0.7) * s0.astype(np.float64) + np.float32(-1.3) * d0.astype(np.float64)
    assert ulp_dist(dst.read(), ref).max() <= 1.0


@pytest.mark.parametrize("count", COUNTS)
def test_copy_fill_fp16_to_fp32(gpu, ab, count):
    rng = rng_for("copy", count)
    x = f16(rng.standard_normal(count))
    src, dst = Slot(gpu, x, 1), Slot(gpu, np.zeros(count), 0)
    assert gpu.core.ops_copy(dst.ptr, src.ptr, count) == 0
    np.testing.assert_array_equal(bits(dst.read()), bits(x))
    assert gpu.core.ops_fill(dst.ptr, count, 0.1) == 0
    np.testing.assert_array_equal(bits(dst.read()), bits(np.full(count, np.float16(0.1))))
    out = gpu.DeviceBuffer(4 * count + 4)
    assert gpu.core.ops_fp16_to_fp32(src.ptr, out.ptr + 4, count) == 0
    gpu.sync()
    np.testing.assert_array_equal(gpu.read_f32(out.ptr + 4, (count,)), x.astype(np.float32))


@pytest.mark.parametrize("count", [8, 1000, 4099, 8 * 1024 * 256 * 4 + 8 * 37])
def test_copy_aligned_vector_path(gpu, count):
    """16-byte aligned, count % 8 == 0: k_copy_v8 (four vectors per thread, then the tail
    of whole vectors); otherwise the blit. Guards on both sides stay untouched."""
    rng = rng_for("copyv", count)
    x = f16(rng.standard_normal(count))
    src, dst = Slot(gpu, x, 0), Slot(gpu, np.zeros(count), 0)
    assert gpu.core.ops_copy(dst.ptr, src.ptr, count) == 0
    np.testing.assert_array_equal(bits(dst.read()), bits(x))


# ----------------------------------------------------------------- layout ops
@pytest.mark.parametrize("T,src_cols,dst_cols,off,soff", [(1, 1, 3, 2, 1), (11, 40, 72, 32, 1), (37, 129, 300, 7, 1),
                                                           (11, 40, 72, 32, 0), (301, 160, 320, 160, 0),
                                                           (5, 1536, 3072, 0, 0), (9, 24, 64, 8, 0)])
def test_concat_slice_cols(gpu, ab, T, src_cols, dst_cols, off, soff):
    """ops.cu:241-254 and :308-320: column placement / extraction, bit-exact. soff = 1
    misaligns the source (scalar kernel); 16-byte-granular shapes with soff = 0 run the
    8-column vector kernel."""
    rng = rng_for("cat", T, src_cols)
    src = f16(rng.standard_normal((T, src_cols)))
    base = f16(rng.standard_normal((T, dst_cols)))
    d = Slot(gpu, base)
    s = Slot(gpu, src, soff)
    assert gpu.core.ops_concat_cols(d.ptr, T, dst_cols, s.ptr, src_cols, off) == 0
    ref = base.copy()
    ref[:, off:off + src_cols] = src
    got = d.read().reshape(T, dst_cols)
    np.testing.assert_array_equal(bits(got), bits(ref))
    out = Slot(gpu, np.zeros((T, src_cols)))
    assert gpu.core.ops_slice_cols(d.ptr, T, dst_cols, out.ptr, src_cols, off) == 0
    np.testing.assert_array_equal(bits(out.read().reshape(T, src_cols)), bits(src))


def test_concat_slice_bad_offset(gpu, ab):
    a, b = Slot(gpu, np.zeros(40)), Slot(gpu, np.zeros(40))
    gpu.core.ops_clear_error()
    assert gpu.core.ops_concat_cols(a.ptr, 2, 20, b.ptr, 8, 13) == -1
    assert b"concat_cols" in gpu.core.ops_last_error()
    assert gpu.core.ops_slice_cols(a.ptr, 2, 20, b.ptr, 8, -1) == -1


@pytest.mark.parametrize("T,H,f1,f2", [(1, 1, 1, 1), (9, 40, 1, 5), (31, 13, 3, 7)])
def test_combine_feature_maps(gpu, ab, T, H, f1, f2):
    """ops.cu:258-287: [T x (H*F1 | H*F2)] -> [T x H*(F1+F2)] in place."""
    D = H * (f1 + f2)
    x = f16(rng_for("cfm", T, H).standard_normal((T, D)))
    s = Slot(gpu, x)
    assert gpu.core.ops_combine_feature_maps(s.ptr, T, D, H, f1, f2) == 0
    a = x[:, :H * f1].reshape(T, H, f1)
    b = x[:, H * f1:].reshape(T, H, f2)
    ref = np.concatenate([a, b], 2).reshape(T, D)
    np.testing.assert_array_equal(bits(s.read().reshape(T, D)), bits(ref))
    gpu.core.ops_clear_error()
    assert gpu.core.ops_combine_feature_maps(s.ptr, T, D + 1, H, f1, f2) == -1


@pytest.mark.parametrize("in_rows,cols,stride,off", [(10, 3, 3, 1), (1500, 40, 3, 0), (7, 9, 2, 6),
                                                     (5, 4, 3, 7)])
def test_subsample_rows(gpu, ab, in_rows, cols, stride, off):
    """ops.cu:632-643: void and silent; (in_rows-off+stride-1)/stride rows."""
    x = f16(rng_for("sub", in_rows, cols).standard_normal((in_rows, cols)))
    out_rows = max(0, (in_rows - off + stride - 1) // stride)
    s = Slot(gpu, x)
    d = Slot(gpu, np.zeros((max(out_rows, 1), cols)))
    assert gpu.core.ops_subsample_rows(d.ptr, s.ptr, in_rows, cols, stride, off) is None
    if out_rows:
        np.testing.assert_array_equal(bits(d.read().reshape(-1, cols)), bits(x[off::stride]))
    else:
        np.testing.assert_array_equal(bits(d.read()), bits(np.zeros(cols, np.float16)))
    gpu.core.ops_subsample_rows(d.ptr, s.ptr, in_rows, cols, 0, 0)  # stride 0: silent no-op


@pytest.mark.parametrize("M,N", [(32, 64), (1, 1), (65, 130), (1500, 40)])
def test_transpose(gpu, ab, M, N):
    """backward_wrappers.cu:75-86 and the round trip of cmd/backtest/main.go:51-65."""
    x = f16(rng_for("tr", M, N).random((M, N)) * 2 - 1)
    s, t, back = Slot(gpu, x), Slot(gpu, np.zeros((N, M))), Slot(gpu, np.zeros((M, N)))
    assert gpu.core.ops_transpose(s.ptr, t.ptr, M, N) == 0
    np.testing.assert_array_equal(bits(t.read().reshape(N, M)), bits(x.T))
    assert gpu.core.ops_transpose(t.ptr, back.ptr, N, M) == 0
    np.testing.assert_array_equal(bits(back.read().reshape(M, N)), bits(x))


def test_transpose_batch(gpu):
    """kf_transpose_batch (kf_ops.h): several ragged transposes in one launch, each equal to
    ops_transpose's; more jobs than the limit is an error"""
    shapes = [(320, 1536), (1, 1), (65, 130), (1500, 40), (160, 3072)]
    xs = [f16(rng_for("trb", M, N).random((M, N)) * 2 - 1) for M, N in shapes]
    src = [Slot(gpu, x) for x in xs]
    dst = [Slot(gpu, np.zeros((N, M))) for M, N in shapes]
    n = len(shapes)
    arr = lambda t, v: (t * n)(*v)
    gpu.core.kf_transpose_batch.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
    rc = gpu.core.kf_transpose_batch(n, arr(C.c_void_p, [s.ptr for s in src]), arr(C.c_void_p, [d.ptr for d in dst]),
                                     arr(C.c_int, [M for M, _ in shapes]), arr(C.c_int, [N for _, N in shapes]))
    assert rc == 0
    for x, d, (M, N) in zip(xs, dst, shapes):
        np.testing.assert_array_equal(bits(d.read().reshape(N, M)), bits(x.T))
    big = 49
    assert gpu.core.kf_transpose_batch(big, arr(C.c_void_p, [src[0].ptr] * n), None, None, None) == -1


# ----------------------------------------------------------------- backward element-wise
@pytest.mark.parametrize("count", COUNTS)
def test_relu_backward_exact(gpu, ab, count):
    """backward_wrappers.cu:41-49: grad = x > 0 ? grad : 0, bit-exact."""
    rng = rng_for("rb", count)
    x = f16(rng.random(count) * 4 - 2)
    g = f16(rng.random(count) * 2 - 1)
    sx, sg = Slot(gpu, x, 1), Slot(gpu, g)
    assert gpu.core.ops_relu_backward(sx.ptr, sg.ptr, count) == 0
    np.testing.assert_array_equal(bits(sg.read()), bits(np.where(x > 0, g, np.float16(0))))


def test_relu_backward_backtest_pin(gpu, ab):
    """cmd/backtest/main.go:67-96: x U[-2,2), n 1024; x > 0.1 passes the gradient
    (|d| < 0.01), x < -0.1 zeroes it (|g| < 1e-3)."""
    rng = np.random.default_rng(67)
    n = 1024
    x, g = rng.random(n) * 4 - 2, rng.random(n) * 2 - 1
    sx, sg = Slot(gpu, f16(x)), Slot(gpu, f16(g))
    assert gpu.core.ops_relu_backward(sx.ptr, sg.ptr, n) == 0
    r = sg.read().astype(np.float64)
    p, z = x > 0.1, x < -0.1
    assert np.all(np.abs(r[p] - g[p]) < 0.01) and np.all(np.abs(r[z]) < 1e-3)


def _h(a):
    return np.asarray(a, np.float32).astype(np.float16).astype(np.float32)


@pytest.mark.parametrize("count", COUNTS)
def test_sigmoid_tanh_backward_fp16_chain(gpu, ab, count):
    """backward_wrappers.cu:51-73 compute in fp16 (__hmul / __hsub):
    sigmoid: g' = (g*out) * (1-out); tanh: g' = g * (1 - out*out), each op rounded."""
    rng = rng_for("stb", count)
    out_s = f16(1 / (1 + np.exp(-(rng.random(count) * 6 - 3))))
    out_t = f16(np.tanh(rng.random(count) * 4 - 2))
    g = f16(rng.random(count) * 2 - 1)
    so, sg = Slot(gpu, out_s), Slot(gpu, g, 1)
    assert gpu.core.ops_sigmoid_backward(so.ptr, sg.ptr, count) == 0
    o, gf = out_s.astype(np.float32), g.astype(np.float32)
    ref = f16(_h(gf * o) * _h(np.float32(1) - o))
    np.testing.assert_array_equal(bits(sg.read()), bits(ref))
    so, sg = Slot(gpu, out_t, 1), Slot(gpu, g)
    assert gpu.core.ops_tanh_backward(so.ptr, sg.ptr, count) == 0
    o = out_t.astype(np.float32)
    ref = f16(gf * _h(np.float32(1) - _h(o * o)))
    np.testing.assert_array_equal(bits(sg.read()), bits(ref))


def test_sigmoid_tanh_backward_backtest_pin(gpu, ab):
    """cmd/backtest/main.go:98-146 (it only prints the error): against the fp32
    formula the fp16 chain (three roundings, cancellation in 1 - out^2 near |out| = 1)
    stays within 2 % relative, backtest's own op threshold (main.go:207)."""
    rng = np.random.default_rng(98)
    n = 1024
    g = (rng.random(n) * 2 - 1).astype(np.float32)
    sig = (1 / (1 + np.exp(-(rng.random(n) * 6 - 3)))).astype(np.float32)
    th = np.tanh(rng.random(n) * 4 - 2).astype(np.float32)
    for fn, out, ref in ((gpu.core.ops_sigmoid_backward, sig, _h(g) * _h(sig) * (1 - _h(sig))),
                         (gpu.core.ops_tanh_backward, th, _h(g) * (1 - _h(th) ** 2))):
        so, sg = Slot(gpu, f16(out)), Slot(gpu, f16(g))
        assert fn(so.ptr, sg.ptr, n) == 0
        assert _max_rel(sg.read(), ref) <= 0.02


# ----------------------------------------------------------------- optimiser
def _register(gpu, w):
    """gpu.NewSGDOptimizer.RegisterParam: fp32 master from the fp16 weights
    (ops_fp16_to_fp32), velocity zero (internal/gpu optimizer)."""
    w16 = Slot(gpu, f16(w))
    n = w16.n
    master = gpu.DeviceBuffer(4 * n)
    assert gpu.core.ops_fp16_to_fp32(w16.ptr, master.ptr, n) == 0
    vel = gpu.upload_f32(np.zeros(n, np.float32))
    return w16, master, vel


def _update(gpu, st, grad, lr, mom):
    w16, master, vel = st
    g = Slot(gpu, f16(grad))
    assert gpu.core.ops_sgd_update(master.ptr, w16.ptr, g.ptr, vel.ptr, lr, mom, w16.n) == 0


def _max_rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.max(np.abs(a - b) / np.maximum(np.abs(b), 1e-6)))


def test_sgd_update_restated(gpu, ab):
    """backward_wrappers.cu:129-142: v = mom*v + g; w32 -= lr*v; w16 = rne(w32)."""
    rng = np.random.default_rng(129)
    n = 4099
    w = rng.standard_normal(n)
    st = _register(gpu, w)
    v = np.zeros(n, np.float32)
    w32 = f16(w).astype(np.float32)
    lr, mom = np.float32(0.05), np.float32(0.9)
    for k in range(3):
        g = f16(rng.standard_normal(n))
        _update(gpu, st, g, lr, mom)
        v = (mom * v.astype(np.float64) + g.astype(np.float64)).astype(np.float32)
        w32 = (w32.astype(np.float64) - lr * v.astype(np.float64)).astype(np.float32)
    gpu.sync()
    np.testing.assert_allclose(gpu.read_f32(st[2].ptr, (n,)), v, rtol=3e-7, atol=1e-6)
    np.testing.assert_allclose(gpu.read_f32(st[1].ptr, (n,)), w32, rtol=3e-7, atol=1e-6)
    assert ulp_dist(st[0].read(), gpu.read_f32(st[1].ptr, (n,))).max() <= 0.5


def test_sgdtest_basic_momentum_master(gpu, ab):
    """cmd/sgdtest/main.go:38-193, thresholds as written there:
    basic (lr 0.01, no momentum): max rel err <= 0.01 vs w16 - lr*g16;
    momentum 0.9, two steps: max rel err <= 0.02 vs the fp16-rounded CPU result;
    fp32 master: w = 1, lr 1e-4, grad 1, 100 steps -> 0.99 within 0.002."""
    rng = np.random.default_rng(38)
    n = 256
    rnd = lambda: (rng.random(n) * 2 - 1).astype(np.float32)  # noqa: E731  (randFloats)
    w, g = rnd(), rnd()
    st = _register(gpu, w)
    _update(gpu, st, g, 0.01, 0.0)
    exp = _h(w) - np.float32(0.01) * _h(g)
    assert _max_rel(st[0].read(), exp) <= 0.01

    w, g1, g2 = rnd(), rnd(), rnd()
    st = _register(gpu, w)
    _update(gpu, st, g1, 0.01, 0.9)
    _update(gpu, st, g2, 0.01, 0.9)
    vel = _h(g1)
    wc = _h(w) - np.float32(0.01) * vel
    vel = np.float32(0.9) * vel + _h(g2)
    wc = wc - np.float32(0.01) * vel
    assert _max_rel(st[0].read(), _h(wc)) <= 0.02

    st = _register(gpu, np.ones(n, np.float32))
    for _ in range(100):
        _update(gpu, st, np.ones(n, np.float32), 1e-4, 0.0)
    got = st[0].read().astype(np.float64)
    assert np.max(np.abs(got - 0.99)) <= 0.002
    # and the failure mode it guards against: fp16-only updates would not move w at all
    assert np.all(got < 1.0)


# ----------------------------------------------------------------- GEMM (strided)
@pytest.mark.parametrize("shareB", [False, True])
def test_gemm_strided(gpu, ab, shareB):
    """ops.cu:402-430: batched C_b = alpha A_b B_b + beta C_b, strideB = 0 shares B.
    Elements within 2 ulp_fp16 + K 2^-23 sum|ab|."""
    rng = rng_for("gs", shareB)
    bc, M, N, K = 3, 37, 72, 40
    A = f16(rng.standard_normal((bc, M, K)))
    B = f16(rng.standard_normal((1 if shareB else bc, K, N)))
    C0 = f16(rng.standard_normal((bc, M, N)))
    dA, dB, dC = gpu.upload_fp16(A), gpu.upload_fp16(B), gpu.upload_fp16(C0)
    h = gpu.core.ops_cublas_create()
    rc = gpu.core.ops_gemm_strided(h, M, N, K, 0.5, dA.ptr, K, M * K, dB.ptr, N, 0 if shareB else K * N,
                                   0.25, dC.ptr, N, M * N, bc)
    gpu.core.ops_cublas_destroy(h)
    assert rc == 0, gpu.core.ops_last_error()
    got = gpu.read_fp16(dC.ptr, (bc, M, N)).astype(np.float64)
    for b in range(bc):
        a, bb = A[b].astype(np.float64), B[0 if shareB else b].astype(np.float64)
        ref = 0.5 * a @ bb + 0.25 * C0[b].astype(np.float64)
        sp = np.spacing(np.abs(ref).astype(np.float16)).astype(np.float64)
        bound = 2 * sp + K * 2.0 ** -23 * 0.5 * (np.abs(a) @ np.abs(bb)) + 1e-7
        assert np.all(np.abs(got[b] - ref) <= bound)


# ----------------------------------------------------------------- bridge batch buffer
def _a256(n):
    return (n + 255) & ~255


@pytest.mark.parametrize("dims", [(1500 * 3, 40, 3, 100, 251, 777), (7, 13, 1, 0, 2, 1)])
def test_bridge_batch_sections(gpu, ab, dims):
    """bridge.cu:177-267: six sections, each 256-byte aligned, in the reference order;
    one host->device copy of the packed buffer; free zeroes the struct."""
    frames, fd, bs, iv, S, A = dims
    p = ab.GPUBatchPtrs()
    assert gpu.core.bridge_batch_alloc(frames, fd, bs, iv, S, A, C.byref(p)) == 0
    sizes = [_a256(frames * fd * 2), _a256(bs * iv * 2), _a256((S + 1) * 4), _a256(A * 4),
             _a256(A * 4), _a256(A * 4)]
    assert [p.features_bytes, p.ivectors_bytes, p.csr_rowptr_bytes, p.csr_colidx_bytes,
            p.csr_labels_bytes, p.csr_weights_bytes] == sizes
    assert p.total_bytes == sum(sizes)
    offs = np.concatenate([[0], np.cumsum(sizes)[:-1]])
    ptrs = [p.d_features, p.d_ivectors, p.d_csr_row_ptr, p.d_csr_col_idx, p.d_csr_labels,
            p.d_csr_weights]
    assert [q - p.d_buffer for q in ptrs] == [int(o) for o in offs]
    assert p.d_buffer % 256 == 0
    host = np.random.default_rng(5).integers(0, 65535, p.total_bytes // 2, dtype=np.uint16)
    pinned = gpu.core.bridge_host_alloc(p.total_bytes)
    assert pinned
    C.memmove(pinned, host.ctypes.data, p.total_bytes)
    assert gpu.core.bridge_batch_transfer(C.byref(p), pinned, p.total_bytes) == 0
    back = np.empty_like(host)
    gpu.check(gpu.core.bridge_read_fp16(back.ctypes.data, p.d_buffer, back.size))
    np.testing.assert_array_equal(back, host)
    feats = np.empty(frames * fd, np.uint16)
    gpu.check(gpu.core.bridge_read_fp16(feats.ctypes.data, p.d_features, feats.size))
    np.testing.assert_array_equal(feats, host[:feats.size])
    gpu.core.bridge_host_free(pinned)
    gpu.core.bridge_batch_free(C.byref(p))
    assert p.d_buffer is None and p.total_bytes == 0 and p.d_features is None
    gpu.core.bridge_batch_free(C.byref(p))  # second free: no-op


# ----------------------------------------------------------------- chain (deterministic)
def _rand_fst(seed, S, P):
    """Branching FST: 1-4 arcs per state, labels in [0, P+1] (0 = epsilon and P+1
    out-of-range are skipped by the reference), two final states."""
    rng = np.random.default_rng(seed)
    row_ptr, dst, lab, w = [0], [], [], []
    for s in range(S):
        for _ in range(int(rng.integers(1, 5))):
            dst.append(int(rng.integers(0, S)))
            lab.append(int(rng.integers(0, P + 2)) if rng.random() < 0.15 else int(rng.integers(1, P + 1)))
            w.append(-float(rng.random()))
        row_ptr.append(len(dst))
    return dict(S=S, A=len(dst), row_ptr=np.array(row_ptr, np.int32), dst=np.array(dst, np.int32),
                pdf1=np.array(lab, np.int32), logw=np.array(w, np.float32),
                final_state=np.array([S - 1, S // 2], np.int32),
                final_w=np.array([0.0, -0.5], np.float32), start=0)


LZ = np.float32(-1e30)


def _logadd(a, b):
    if a <= LZ:
        return b
    if b <= LZ:
        return a
    mx, mn = max(a, b), min(a, b)
    return np.float32(mx + np.float32(np.log1p(np.float32(np.exp(np.float32(mn - mx))))))


def _det_ref(f, x16, P):
    """chain_det.cu:55-237 in float32, the same loop order (forward by destination over
    the reverse CSR in arc order, backward by source, posteriors by source then arc)."""
    S, T = f["S"], x16.shape[0]
    x = x16.astype(np.float32)
    rp, dst, lab, w = f["row_ptr"], f["dst"], f["pdf1"], f["logw"]
    rev = [[] for _ in range(S)]
    for s in range(S):
        for a in range(rp[s], rp[s + 1]):
            rev[dst[a]].append((a, s))
    al = np.full((T + 1, S), LZ, np.float32)
    al[0, f["start"]] = 0
    for t in range(T):
        for d in range(S):
            v = LZ
            for a, s in rev[d]:
                p = lab[a]
                if p <= 0 or p > P or al[t, s] <= LZ:
                    continue
                v = _logadd(v, np.float32(al[t, s] + x[t, p - 1] + w[a]))
            al[t + 1, d] = v
    tot = LZ
    for fs, fw in zip(f["final_state"], f["final_w"]):
        tot = _logadd(tot, np.float32(al[T, fs] + fw))
    be = np.full((T + 1, S), LZ, np.float32)
    be[T, f["final_state"]] = f["final_w"]
    for t in range(T - 1, -1, -1):
        for s in range(S):
            v = LZ
            for a in range(rp[s], rp[s + 1]):
                p = lab[a]
                if p <= 0 or p > P or be[t + 1, dst[a]] <= LZ:
                    continue
                v = _logadd(v, np.float32(be[t + 1, dst[a]] + x[t, p - 1] + w[a]))
            be[t, s] = v
    post = np.zeros((T, P), np.float64)
    for t in range(T):
        for s in range(S):
            if al[t, s] <= LZ:
                continue
            for a in range(rp[s], rp[s + 1]):
                p = lab[a]
                if p <= 0 or p > P or be[t + 1, dst[a]] <= LZ:
                    continue
                lp = min(0.0, float(al[t, s]) + x[t, p - 1] + w[a] + be[t + 1, dst[a]] - tot)
                post[t, p - 1] += np.exp(lp)
    return al, be, float(tot), post


def _upload_fst(gpu, f):
    from kfp16 import chain
    keep = []

    def up(a, dt):
        a = np.ascontiguousarray(a, dt)
        b = gpu.DeviceBuffer(a.nbytes)
        gpu.check(gpu.core.bridge_transfer_int32(b.ptr, a.view(np.int32).ctypes.data, a.size))
        keep.append(b)
        return b.ptr
    fst = chain.ChainFstGPU(up(f["row_ptr"], np.int32), up(f["dst"], np.int32), up(f["pdf1"], np.int32),
                            up(f["logw"], np.float32), up(f["final_state"], np.int32),
                            up(f["final_w"], np.float32), f["S"], f["A"], len(f["final_state"]),
                            f["start"])
    return fst, keep


@pytest.mark.parametrize("S,T,P", [(12, 15, 20), (40, 30, 64)])
def test_chain_det_matches_restatement(gpu, ab, S, T, P):
    f = _rand_fst(S * 100 + T, S, P)
    x = f16(np.random.default_rng(S + T).standard_normal((T, P)))
    al_r, be_r, tot_r, post_r = _det_ref(f, x, P)
    fst, keep = _upload_fst(gpu, f)
    dx = gpu.upload_fp16(x)
    assert gpu.core.chain_workspace_bytes(T, S) == 2 * (T + 1) * S * 4
    al, be = gpu.DeviceBuffer((T + 1) * S * 4), gpu.DeviceBuffer((T + 1) * S * 4)
    tot = C.c_float()
    assert gpu.core.chain_forward_backward_det(dx.ptr, C.byref(fst), T, P, al.ptr, be.ptr,
                                               C.byref(tot)) == 0
    gpu.sync()
    ga, gb = gpu.read_f32(al.ptr, (T + 1, S)), gpu.read_f32(be.ptr, (T + 1, S))
    fin = al_r > LZ
    assert np.array_equal(ga > LZ, fin) and np.array_equal(gb > LZ, be_r > LZ)
    np.testing.assert_allclose(ga[fin], al_r[fin], rtol=1e-5, atol=1e-4)
    np.testing.assert_allclose(gb[be_r > LZ], be_r[be_r > LZ], rtol=1e-5, atol=1e-4)
    assert abs(tot.value - tot_r) <= 1e-4 * max(1.0, abs(tot_r))
    post = gpu.DeviceBuffer(T * P * 4)
    assert gpu.core.chain_compute_posteriors_det(dx.ptr, C.byref(fst), T, P, al.ptr, be.ptr,
                                                 tot.value, post.ptr) == 0
    gpu.sync()
    gp = gpu.read_f32(post.ptr, (T, P))
    np.testing.assert_allclose(gp, post_r, atol=1e-5)
    # the plain entry points return the same deterministic numbers (include/chain.h)
    al2, be2 = gpu.DeviceBuffer((T + 1) * S * 4), gpu.DeviceBuffer((T + 1) * S * 4)
    tot2 = C.c_float()
    assert gpu.core.chain_forward_backward(dx.ptr, C.byref(fst), T, P, al2.ptr, be2.ptr,
                                           C.byref(tot2)) == 0
    gpu.sync()
    assert tot2.value == tot.value
    np.testing.assert_array_equal(gpu.read_f32(al2.ptr, (T + 1, S)), ga)
    # FP32 input, converted to fp16 first (chain_det.cu:412-477)
    x32 = (x.astype(np.float32) + np.float32(1e-4)).astype(np.float32)
    dx32 = gpu.upload_f32(x32)
    np_post = gpu.DeviceBuffer(T * P * 4)
    lp = gpu.core.chain_num_forward_backward_det(fst.row_ptr, fst.col_idx, fst.weights, fst.labels,
                                                 fst.final_states, fst.final_weights, S, f["A"],
                                                 len(f["final_state"]), dx32.ptr, np_post.ptr, T, P,
                                                 None)
    _, _, tot3, post3 = _det_ref(f, f16(x32), P)
    assert abs(lp - tot3) <= 1e-4 * max(1.0, abs(tot3))
    gpu.sync()
    np.testing.assert_allclose(gpu.read_f32(np_post.ptr, (T, P)), post3, atol=1e-5)
    del keep
