"""HIP path vs the CPU oracle, through the C-ABI (SURVEY §8d tolerances).

Activations: rel-Frobenius <= 2e-3 and max-abs <= 1e-2 * max|ref| against the
oracle's fused-rounding mode (F); rel-Frobenius <= 1e-2 against the reference's
round-after-every-op mode (R). Weight gradients: rel-Frobenius <= 5e-3.
"""
import numpy as np
import pytest

import oracle
from conftest import max_abs_rel, rel_fro

pytestmark = pytest.mark.gpu


def _run_product(kfp16, xcfg, T, seed=42, out_grad=None):
    from kfp16 import synth
    net = kfp16.Network(xcfg, max_frames=T)
    params, bns = synth.init_network(net, seed=seed)
    feats = synth.make_features(T, 40)
    fbuf = kfp16.upload_fp16(feats)
    net.forward(fbuf.ptr, T)
    return net, params, bns, feats, fbuf


def _oracle(xcfg, params, bns, feats, mode=oracle.ROUND_FUSED):
    from kfp16 import synth
    tp = {k: synth.trunc_fp16(v) for k, v in params.items()}   # weights enter by truncation
    on = oracle.OracleNet(xcfg, tp, bns, round_mode=mode, threads=16)
    on.forward(feats.astype(np.float32))
    return on


def test_ops_gemm_matches_fp32(gpu):
    kfp16 = gpu
    rng = np.random.default_rng(3)
    h = kfp16.core.ops_cublas_create()
    for (M, N, K, alpha, beta) in [(256, 128, 64, 1.0, 0.0), (300, 3080, 256, 1.0, 0.0),
                                   (1, 64, 96000, 1.0, 0.0), (130, 160, 3072, 0.5, 1.0),
                                   (37, 24, 9, 1.0, 0.0), (64, 40, 40, 2.0, -1.0),
                                   # short K on the 8-column vector kernel: AddBias's K = 1 form
                                   # (ops.go:335-351, beta = 1), K = 3, K = 8
                                   (1000, 1536, 1, 1.0, 1.0), (77, 40, 3, 0.5, -1.0), (50, 64, 8, 1.0, 0.0)]:
        A = rng.standard_normal((M, K)).astype(np.float16)
        B = (rng.standard_normal((K, N)) / np.sqrt(K)).astype(np.float16)
        C0 = rng.standard_normal((M, N)).astype(np.float16)
        dA, dB, dC = kfp16.upload_fp16(A), kfp16.upload_fp16(B), kfp16.upload_fp16(C0)
        kfp16.check(kfp16.core.ops_gemm(h, M, N, K, alpha, dA.ptr, K, dB.ptr, N, beta, dC.ptr, N), "gemm")
        got = kfp16.read_fp16(dC.ptr, (M, N)).astype(np.float64)
        ref = alpha * (A.astype(np.float64) @ B.astype(np.float64)) + beta * C0.astype(np.float64)
        # fp32 accumulation K * 2^-23 * sum|ab| (scaled by alpha), beta * C in fp32,
        # one fp16 rounding of the result (<= |ref| * 2^-11, doubled for the shifted value)
        mag = np.abs(A).astype(np.float64) @ np.abs(B).astype(np.float64)
        tol = (abs(alpha) * K * 2 ** -23 * mag + 2 ** -23 * abs(beta) * np.abs(C0.astype(np.float64))
               + np.abs(ref) * 2 ** -10 + 2 ** -24)
        assert np.all(np.abs(got - ref) <= tol), (M, N, K, float(np.max(np.abs(got - ref) - tol)))
    kfp16.core.ops_cublas_destroy(h)


def _forward_parity(net, on, onr):
    """Activations within SURVEY §8d tolerances; ReLU decisions agree except for
    a small fraction of near-zero pre-activations."""
    masks = net.relu_masks()
    for name, ty, din, dout in net.layers:
        got = net.read_activation(name).astype(np.float32)
        ref = on.act(name)
        assert rel_fro(got, ref) <= 2e-3, (name, rel_fro(got, ref))
        assert max_abs_rel(got, ref) <= 1e-2, (name, max_abs_rel(got, ref))
        if onr is not None:
            assert rel_fro(got, onr.act(name)) <= 1e-2, (name, "vs R mode")
        if name in masks:
            agree = float(np.mean(masks[name] == on.mask(name)))
            assert agree >= 0.999, (name, agree)
    return masks


@pytest.mark.parametrize("T", [150, 517])
def test_tiny_network_forward_backward(gpu, T):
    kfp16 = gpu
    from kfp16 import synth
    xcfg = synth.load_xconfig("tiny.xconfig")
    net, params, bns, feats, fbuf = _run_product(kfp16, xcfg, T)
    on = _oracle(xcfg, params, bns, feats)
    onr = _oracle(xcfg, params, bns, feats, oracle.ROUND_REF)
    masks = _forward_parity(net, on, onr)
    # backward from a fixed fp16 output gradient; the oracle replays the
    # product's ReLU decisions so gradients compare without flip noise
    on.close()
    on = _oracle(xcfg, params, bns, feats)
    on.forward(feats.astype(np.float32), force_masks=masks)
    P = net.layers[-1][3]
    og = (np.random.default_rng(7).standard_normal((T, P)) * 0.05).astype(np.float16)
    gbuf = kfp16.upload_fp16(og)
    net.backward(gbuf.ptr)
    got = net.read_grads()
    on.backward(og.astype(np.float32))
    ref = on.grads()
    errs = {k: rel_fro(got[k], ref[k]) for k in ref}
    bad = {k: v for k, v in errs.items() if v > 5e-3}
    assert not bad, "grad errors: " + ", ".join(f"{k}={v:.2e}" for k, v in errs.items())


@pytest.mark.parametrize("implicit", [False, True])
def test_tiny_backward_dz_modes(gpu, implicit):
    """nnet_set_implicit_dz off (dz stored by the producing epilogue) and on (g read
    through the ReLU mask, the BN scale folded into W2 / the wgrad reduce), each against the
    oracle at the matching rounding points (kf_oracle.h implicit_dz); the two GPU modes
    agree with each other to a few fp16 roundings."""
    kfp16 = gpu
    from kfp16 import synth
    xcfg = synth.load_xconfig("tiny.xconfig")
    T = 517
    net, params, bns, feats, fbuf = _run_product(kfp16, xcfg, T)
    masks = net.relu_masks()
    tp = {k: synth.trunc_fp16(v) for k, v in params.items()}
    on = oracle.OracleNet(xcfg, tp, bns, round_mode=oracle.ROUND_FUSED, threads=16, implicit_dz=implicit)
    on.forward(feats.astype(np.float32), force_masks=masks)
    P = net.layers[-1][3]
    og = (np.random.default_rng(11).standard_normal((T, P)) * 0.05).astype(np.float16)
    gbuf = kfp16.upload_fp16(og)
    grads = {}
    for mode in (not implicit, implicit):  # the mode under test last
        net.set_implicit_dz(mode)
        net.backward(gbuf.ptr)
        grads[mode] = net.read_grads()
    net.set_implicit_dz(False)
    on.backward(og.astype(np.float32))
    ref = on.grads()
    got = grads[implicit]
    errs = {k: rel_fro(got[k], ref[k]) for k in ref}
    bad = {k: v for k, v in errs.items() if v > 5e-3}
    assert not bad, "grad errors: " + ", ".join(f"{k}={v:.2e}" for k, v in errs.items())
    cross = {k: rel_fro(grads[True][k], grads[False][k]) for k in ref}
    assert max(cross.values()) <= 2e-3, cross
    # the implicit mode reaches the TDNN-F layers with a bypass (tdnnf6-8)
    if implicit:
        assert any(cross[k] > 0 for k in cross if k.startswith("tdnnf7")), cross


def test_sgd_step_matches_oracle(gpu):
    kfp16 = gpu
    from kfp16 import synth
    xcfg = synth.load_xconfig("tiny.xconfig")
    T = 96
    net, params, bns, feats, fbuf = _run_product(kfp16, xcfg, T)
    og = (np.random.default_rng(9).standard_normal((T, 200)) * 0.05).astype(np.float16)
    gbuf = kfp16.upload_fp16(og)
    w0 = net.get_params()
    lr, mom = 1e-3, 0.9
    net.backward(gbuf.ptr)
    g1 = net.read_grads()
    net.sgd(lr, mom)
    net.forward(fbuf.ptr, T)
    net.backward(gbuf.ptr)
    g2 = net.read_grads()
    net.sgd(lr, mom)
    w2 = net.get_params()
    import ctypes
    L = oracle.lib()
    for k in w0:
        w = w0[k].astype(np.float32).ravel().copy()
        v = np.zeros_like(w)
        for g in (g1[k], g2[k]):
            gg = np.ascontiguousarray(g.ravel(), np.float32)
            L.orc_sgd(w.ctypes.data, gg.ctypes.data, v.ctypes.data, lr, mom, w.size)
        np.testing.assert_allclose(w2[k].ravel(), w, rtol=1e-6, atol=1e-7)


@pytest.mark.slow
@pytest.mark.parametrize("implicit", [False, True])
def test_full_model_one_eg(gpu, implicit):
    """The benchmark model (cnn_tdnn_17f) on one 1500-frame eg; the backward with the
    stored dz (default) and with the implicit dz (the 384x160 masked affine input
    gradients and 320x256 masked weight gradients of the 1536-wide layers)."""
    kfp16 = gpu
    from kfp16 import synth
    xcfg = synth.load_xconfig("cnn_tdnn_17f.xconfig")
    T = 1500
    net, params, bns, feats, fbuf = _run_product(kfp16, xcfg, T)
    net.set_implicit_dz(implicit)
    on = _oracle(xcfg, params, bns, feats)
    masks = _forward_parity(net, on, None)
    on.close()
    on = _oracle(xcfg, params, bns, feats)
    on.implicit_dz = int(implicit)
    on.forward(feats.astype(np.float32), force_masks=masks)
    og = (np.random.default_rng(7).standard_normal((T, 3080)) * 0.02).astype(np.float16)
    gbuf = kfp16.upload_fp16(og)
    net.backward(gbuf.ptr)
    got = net.read_grads()
    on.backward(og.astype(np.float32))
    ref = on.grads()
    errs = {k: rel_fro(got[k], ref[k]) for k in ref}
    assert all(v <= 5e-3 for v in errs.values()), errs


@pytest.mark.parametrize("xname,T", [("tiny.xconfig", 300), ("cnn_tdnn_17f.xconfig", 3000)])
def test_wgrad_stream_bit_identical(gpu, xname, T):
    """nnet_backward with the weight gradients on their own stream (the default) against
    the one-stream order: every gradient, and the next step's activations after SGD,
    bit-identical (the same kernels on the same inputs; only the launch streams and the
    alternating dbott buffer differ). Twice in a row with the stream on, so a race on the
    ping-pong buffers between consecutive backward calls would show as well."""
    kfp16 = gpu
    from kfp16 import synth
    xcfg = synth.load_xconfig(xname)
    P = None
    res = []
    for on in (False, True, True):
        net, params, bns, feats, fbuf = _run_product(kfp16, xcfg, T)
        net.set_wgrad_stream(on)
        P = net.layers[-1][3]
        og = (np.random.default_rng(11).standard_normal((T, P)) * 0.05).astype(np.float16)
        gb = kfp16.upload_fp16(og)
        net.backward(gb.ptr)
        net.sgd(1e-3, 0.9)
        net.forward(fbuf.ptr, T)
        net.backward(gb.ptr)
        res.append((net.read_grads(), net.read_activation("output").astype(np.float32)))
        net.close()
    g0, a0 = res[0]
    for g1, a1 in res[1:]:
        for k in g0:
            assert np.array_equal(g0[k], g1[k]), k
        assert np.array_equal(a0, a1)
