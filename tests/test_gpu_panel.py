"""Panel GEMM (csrc/panel.hip) against the tiled MFMA GEMM and an fp64 product.

The panel kernel runs the same v_mfma_f32_16x16x32_f16 sequence in the same K order
and the same 8-column epilogue as gemm_kernel, so for every operand / epilogue mode
it must be BIT-IDENTICAL to the tiled path (kf_gemm_debug_panel toggles them); the
tiled path itself is pinned to the oracle elsewhere (test_gpu_kernels, test_gpu_nnet).
Shapes cover the TDNN-F affine forward (spliced A, clamp policy, k-contiguous
transposed weights, bias / ReLU mask / BN / bypass), the linear input gradient
(spliced A with zero policy and an edge row, op_wrows B, out + out2 with scale2 and
input mask + residual), ragged M, and every instantiated K.
"""
import ctypes as C

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _h(a):
    return np.ascontiguousarray(a, np.float16)


def _run(kf, M, N, K, a, b, e, panel):
    kf.core.kf_gemm_debug_panel(1 if panel else 0)
    try:
        kf.check(kf.core.kf_gemm_fused(M, N, K, C.byref(a), C.byref(b), C.byref(e)), "kf_gemm_fused")
        kf.sync()
    finally:
        kf.core.kf_gemm_debug_panel(-1)


@pytest.fixture(scope="module", autouse=True)
def _sig(gpu):
    gpu.core.kf_gemm_debug_panel.argtypes = [C.c_int]
    gpu.core.kf_gemm_debug_panel.restype = None
    gpu.core.kf_panel_enabled.restype = C.c_int


@pytest.mark.parametrize("M,bn,N,s", [(96000 // 50, 160, 1536, 3), (1000, 160, 1536, 1), (333, 128, 256, 2),
                                      (257, 64, 96, 3), (640, 160, 512, 0)])
def test_affine_forward_bit_identical(gpu, M, bn, N, s):
    """TDNN-F affine: y = relu(splice+(bott) . W + b) -> mask, BN, + 0.66 x."""
    kf = gpu
    rng = np.random.default_rng(M + N)
    K = 2 * bn if s else bn
    bott = _h(rng.standard_normal((M + 2, bn)))
    W = _h(rng.standard_normal((K, N)) / np.sqrt(K))
    x = _h(rng.standard_normal((M, N)))
    bias = _h(rng.uniform(-0.1, 0.1, N))
    sc = rng.uniform(0.5, 1.5, N).astype(np.float32)
    sh = rng.uniform(-0.2, 0.2, N).astype(np.float32)
    d = {k: kf.upload_fp16(v) for k, v in dict(bott=bott, Wt=W.T.copy(), x=x, bias=bias).items()}
    dsc, dsh = kf.upload_f32(sc), kf.upload_f32(sh)
    if s:
        a = kf.operand(d["bott"].ptr, bn, M, K, 1, nparts=2, part_width=bn, tpolicy=1, dt=(0, s))
    else:
        a = kf.operand(d["bott"].ptr, bn, M, K, 1)
    b = kf.operand(d["Wt"].ptr, K, N, K, 1)
    outs = []
    for panel in (True, False):
        out = kf.DeviceBuffer(M * N * 2)
        mask = kf.DeviceBuffer(M * N // 8 + 64)
        e = kf.KfEpilogue(out=out.ptr, ldo=N, alpha=1.0, bias=d["bias"].ptr, relu=1, mask_out=mask.ptr,
                          scale=dsc.ptr, shift=dsh.ptr, resid=d["x"].ptr, ldr=N, resid_alpha=0.66)
        _run(kf, M, N, K, a, b, e, panel)
        outs.append((kf.read_fp16(out.ptr, (M, N)), kf.read_fp16(mask.ptr, (M * N // 16,))))
    np.testing.assert_array_equal(outs[0][0].view(np.uint16), outs[1][0].view(np.uint16))
    np.testing.assert_array_equal(outs[0][1].view(np.uint16), outs[1][1].view(np.uint16))
    # and against fp64: the pre-activation product
    bf = bott.astype(np.float64)[:M]
    rows = np.arange(M)
    A = np.concatenate([bf[rows], bott.astype(np.float64)[np.clip(rows + s, 0, M - 1)]], 1) if s else bf
    v = A @ W.astype(np.float64) + bias.astype(np.float64)
    ref = np.maximum(v, 0) * sc + sh + 0.66 * x.astype(np.float64)
    got = outs[0][0].astype(np.float64)
    assert np.linalg.norm(got - ref) / np.linalg.norm(ref) < 2e-3


@pytest.mark.parametrize("M,din,bn,s", [(2000, 1536, 160, 3), (517, 256, 64, 1), (300, 512, 128, 2)])
def test_linear_dgrad_bit_identical(gpu, M, din, bn, s):
    """TDNN-F linear input gradient: dX = spliceT(dbott) . Wlin^T with the edge row,
    out = g (bypass), out2 = dz = g * bnscale * mask_in, resid = 0.66 gcur."""
    kf = gpu
    rng = np.random.default_rng(M + din)
    K = 2 * bn
    dbott = _h(rng.standard_normal((M + 2, bn)))
    Wlin = _h(rng.standard_normal((2 * din, bn)) / np.sqrt(bn))
    gcur = _h(rng.standard_normal((M, din)))
    sc2 = rng.uniform(0.5, 1.5, din).astype(np.float32)
    mask = rng.integers(0, 256, M * din // 8 + 64).astype(np.uint8)
    d = {k: kf.upload_fp16(v) for k, v in dict(dbott=dbott, W=Wlin, g=gcur).items()}
    dsc2 = kf.upload_f32(sc2)
    dm = kf.upload_fp16(mask.view(np.float16))
    a = kf.operand(d["dbott"].ptr, bn, M, K, 1, nparts=2, part_width=bn, tpolicy=0, dt=(s, 0),
                   edges=[(0, 0, M)])
    b = kf.operand(d["W"].ptr, bn, din, K, 1, nparts=2, part_width=bn, T=2 * din, dt=(0, din))
    outs = []
    for panel in (True, False):
        o1, o2 = kf.DeviceBuffer(M * din * 2), kf.DeviceBuffer(M * din * 2)
        e = kf.KfEpilogue(out=o1.ptr, ldo=din, alpha=1.0, resid=d["g"].ptr, ldr=din, resid_alpha=0.66,
                          out2=o2.ptr, ldo2=din, scale2=dsc2.ptr, mask_in=dm.ptr)
        _run(kf, M, din, K, a, b, e, panel)
        outs.append((kf.read_fp16(o1.ptr, (M, din)), kf.read_fp16(o2.ptr, (M, din))))
    for i in range(2):
        np.testing.assert_array_equal(outs[0][i].view(np.uint16), outs[1][i].view(np.uint16))


def test_panel_enabled_and_fallbacks(gpu):
    """K outside the instantiated set, N % 32 != 0 and beta != 0 fall back to the
    tiled kernel (same result as with the panel forced off)."""
    kf = gpu
    assert kf.core.kf_panel_enabled() in (0, 1)
    rng = np.random.default_rng(3)
    for M, N, K in ((300, 200, 320), (300, 160, 96), (129, 64, 512)):
        A = _h(rng.standard_normal((M, K)))
        Wt = _h(rng.standard_normal((N, K)) / np.sqrt(K))
        dA, dW = kf.upload_fp16(A), kf.upload_fp16(Wt)
        a = kf.operand(dA.ptr, K, M, K, 1)
        b = kf.operand(dW.ptr, K, N, K, 1)
        res = []
        for panel in (True, False):
            out = kf.DeviceBuffer(M * N * 2)
            e = kf.KfEpilogue(out=out.ptr, ldo=N, alpha=1.0)
            _run(kf, M, N, K, a, b, e, panel)
            res.append(kf.read_fp16(out.ptr, (M, N)))
        np.testing.assert_array_equal(res[0].view(np.uint16), res[1].view(np.uint16))


def test_network_bit_identical_with_and_without_panel(gpu):
    """A CNN-TDNN whose TDNN-F (bottleneck 160, stride 3 and 0), prefinal and linear
    input gradients take the panel path: forward activations and every gradient are
    bit-identical to the tiled path, including after an SGD step (the transposed
    weight copies follow the update)."""
    from kfp16 import synth
    xc = synth.load_xconfig("tiny_panel.xconfig")
    T = 300
    feats = gpu.upload_fp16(synth.make_features(T, 40))
    res = []
    for panel in (True, False):
        gpu.core.kf_gemm_debug_panel(1 if panel else 0)
        try:
            net = gpu.Network(xc, max_frames=T)
            synth.init_network(net)
            net.forward(feats.ptr, T)
            out = net.read_activation("output")
            og = gpu.upload_fp16((np.random.default_rng(4).standard_normal(out.shape) * 0.05).astype(np.float16))
            net.backward(og.ptr)
            g = gpu.read_f32(net.grad_ptr, (net.num_params,)).copy()
            net.sgd(1e-3, 0.9)
            net.forward(feats.ptr, T)
            acts = {n: net.read_activation(n) for n, *_ in net.layers}
            res.append((g, acts))
            net.close()
        finally:
            gpu.core.kf_gemm_debug_panel(-1)
    np.testing.assert_array_equal(res[0][0], res[1][0])
    for n in res[0][1]:
        np.testing.assert_array_equal(res[0][1][n].view(np.uint16), res[1][1][n].view(np.uint16), err_msg=n)
