"""Kaldi nnet3 import into the MI355X network (nnet_load_kaldi) on the GPU.

A network loaded from Kaldi text must be the network built from the same values
directly: identical fp16 weights (both enter by truncation), identical BatchNorm
scale/shift, and bit-identical forward activations. REPLACE mode must reproduce the
reference's double normalisation (replaceBN, weight_loader.go:1035-1085)."""
import numpy as np
import pytest

import nnet3_text as T
import nnet3_writer as NW

pytestmark = pytest.mark.gpu


def _net(kf, T_=150):
    from kfp16 import synth
    xcfg = synth.load_xconfig("tiny.xconfig")
    return kf.Network(xcfg, max_frames=T_)


def test_loaded_network_equals_direct(gpu):
    kf = gpu
    from kfp16 import model, synth
    T_ = 150
    a = _net(kf, T_)
    params, bns = synth.init_network(a)
    b = _net(kf, T_)
    st = model.Nnet3Model.from_text(NW.network_text(b.layers, params, bns)).load_into(b, model.LOAD_NEW)
    assert st.layers_loaded == sum(1 for l in b.layers if l[1] in (1, 2, 3, 6, 7, 9, 10))
    pa, pb = a.get_params(), b.get_params()
    for k in pa:
        assert np.array_equal(pa[k].view(np.uint32), pb[k].view(np.uint32)), k
    feats = synth.make_features(T_, 40)
    fbuf = kf.upload_fp16(feats)
    a.forward(fbuf.ptr, T_)
    b.forward(fbuf.ptr, T_)
    for name, ty, din, dout in a.layers:
        ga, gb = a.read_activation(name), b.read_activation(name)
        assert np.array_equal(ga.view(np.uint16), gb.view(np.uint16)), name


def test_replace_mode_double_normalises(gpu):
    kf = gpu
    from kfp16 import model, synth
    import ctypes as C
    net = _net(kf)
    params, bns = synth.init_network(net)
    txt = NW.network_text(net.layers, params, bns, rms=0.5)
    st = model.Nnet3Model.from_text(txt).load_into(net, model.LOAD_REPLACE)
    assert st.params > 0
    kf.nnet.nnet_debug_tensor.restype = C.c_void_p
    kf.nnet.nnet_debug_tensor.argtypes = [C.c_void_p, C.c_char_p, C.c_int]
    for li, (name, ty, din, dout) in enumerate(net.layers):
        if ty != 7:
            continue
        m, v, _, _ = bns[(name, 0)]
        g, bt = T.replace_bn(m, v, 1e-3, 0.5)
        inv = (np.float32(1) / np.sqrt(np.asarray(v, np.float32) + np.float32(1e-3))).astype(np.float32)
        want = (g * inv).astype(np.float32)            # gamma' / sqrt(var + eps): normalised twice
        ptr = kf.nnet.nnet_debug_tensor(net.h, b"bn_scale", li)
        got = kf.read_f32(ptr, (dout,))
        np.testing.assert_allclose(got, want, rtol=1e-6)


def test_idct_and_shape_errors(gpu):
    kf = gpu
    from kfp16 import model, synth
    net = _net(kf)
    params, bns = synth.init_network(net)
    M = (np.random.default_rng(1).standard_normal((40, 40)) * 0.2).astype(np.float32)
    model.Nnet3Model.from_text(NW.network_text(net.layers, params, bns, idct=M)).load_into(net)
    feats = synth.make_features(150, 40)
    fbuf = kf.upload_fp16(feats)
    net.forward(fbuf.ptr, 150)
    got = net.read_activation("idct").astype(np.float64)
    ref = feats.astype(np.float64) @ synth.trunc_fp16(M).astype(np.float64)
    assert np.max(np.abs(got - ref)) <= 2e-3 * np.max(np.abs(ref)) + 1e-3
    # a wrongly shaped component leaves the network untouched
    before = net.get_params()
    bad = dict(params)
    bad["output.W"] = np.zeros((64, 100), np.float32)
    with pytest.raises(model.ModelError, match="does not match"):
        model.Nnet3Model.from_text(NW.network_text(net.layers, bad, bns)).load_into(net)
    after = net.get_params()
    assert all(np.array_equal(before[k], after[k]) for k in before)
    with pytest.raises(model.ModelError, match="not found"):
        model.Nnet3Model.from_text("<ComponentName> x <NoOpComponent>\n").load_into(net)
