"""cmd/backtest/main.go:217-427 restated on the MI355X path.

testNetworkBackward (:217-295): the reference's Append network
  linear-component input=Append(idct, ivector) -> batchnorm -> 2 x tdnnf (stride 0)
  -> prefinal -> output, T = 32, features and ivectors [T x 32] uniform(-1, 1),
a random output gradient; every trainable layer must get a non-zero weight gradient.
Here the same network runs through nnet_forward_ivector with one ivector per frame
(B = T sequences of one frame, which is the reference's [T x 32] Append) and is held to
the oracle (activations rel-Frobenius <= 2e-3, gradients <= 5e-3) as well as
to the reference's own criterion (mean |grad| > 1e-10 for each layer).

testNumericalGradient (:299-427): output-layer weight gradient of loss = sum(output)
against central differences with eps = 0.1 on 20 evenly spaced weights, T = 4. The
reference fails only when max rel error > 0.2 AND max abs error > 0.1 (:423).
"""
import numpy as np
import pytest

import oracle
from conftest import rel_fro

pytestmark = pytest.mark.gpu

APPEND_NET = """input name=input dim=40
input name=ivector dim=32
idct-layer name=idct input=input dim=40
linear-component name=linear1 input=Append(idct, ivector) dim=128
batchnorm-component name=bn1
tdnnf-layer name=tdnnf1 dim=128 bottleneck-dim=64 time-stride=0 bypass-scale=0.66
tdnnf-layer name=tdnnf2 dim=128 bottleneck-dim=64 time-stride=0 bypass-scale=0.66
prefinal-layer name=prefinal input=tdnnf2 small-dim=64 big-dim=128
output-layer name=output dim=40 include-log-softmax=false"""

NUMGRAD_NET = """input name=input dim=40
idct-layer name=idct input=input dim=40
linear-component name=linear1 dim=128
batchnorm-component name=bn1
tdnnf-layer name=tdnnf1 dim=128 bottleneck-dim=64 time-stride=0 bypass-scale=0.66
tdnnf-layer name=tdnnf2 dim=128 bottleneck-dim=64 time-stride=0 bypass-scale=0.66
prefinal-layer name=prefinal input=tdnnf2 small-dim=64 big-dim=128
output-layer name=output dim=40 include-log-softmax=false"""


def test_append_network_backward(gpu):
    kf = gpu
    from kfp16 import synth
    T = 32
    rng = np.random.default_rng(217)
    feats = (rng.random((T, 40)) * 2 - 1).astype(np.float16)
    ivec = (rng.random((T, 32)) * 2 - 1).astype(np.float16)
    net = kf.Network(APPEND_NET, max_frames=T)
    params, bns = synth.init_network(net, seed=5)
    fb, ib = kf.upload_fp16(feats), kf.upload_fp16(ivec)
    seq = np.arange(T + 1, dtype=np.int32)
    net.forward_ivector(fb.ptr, T, ib.ptr, seq)
    masks = net.relu_masks()
    tp = {k: synth.trunc_fp16(v) for k, v in params.items()}
    on = oracle.OracleNet(APPEND_NET, tp, bns, round_mode=oracle.ROUND_FUSED, threads=8)
    on.forward(feats.astype(np.float32), force_masks=masks, ivectors=ivec.astype(np.float32), seq_off=seq)
    # the Append node is the column concat [idct | ivector] (forward.go:264-310)
    app = net.read_activation("linear1.append").astype(np.float32)
    np.testing.assert_array_equal(app[:, 40:], ivec.astype(np.float32))
    np.testing.assert_array_equal(app[:, :40], net.read_activation("idct").astype(np.float32))
    for name, ty, din, dout in net.layers:
        got = net.read_activation(name).astype(np.float32)
        assert rel_fro(got, on.act(name)) <= 2e-3, (name, rel_fro(got, on.act(name)))
    og = (rng.random((T, 40)) * 2 - 1).astype(np.float16)
    gb = kf.upload_fp16(og)
    net.backward(gb.ptr)
    got = net.read_grads()
    on.backward(og.astype(np.float32))
    ref = on.grads()
    errs = {k: rel_fro(got[k], ref[k]) for k in ref}
    assert all(v <= 5e-3 for v in errs.values()), errs
    for layer in ("linear1", "tdnnf1", "tdnnf2", "prefinal", "output"):   # main.go:258-291
        ks = [k for k in got if k.startswith(layer + ".")]
        assert ks, layer
        assert max(float(np.mean(np.abs(got[k]))) for k in ks) > 1e-10, layer
    on.close()
    net.close()


def test_append_of_two_frame_level_layers_forward(gpu):
    """Append of two layer outputs (three parts, two hidden concat nodes)."""
    kf = gpu
    from kfp16 import synth
    xcfg = """input name=input dim=40
idct-layer name=idct input=input dim=40
linear-component name=lin dim=64
batchnorm-component name=bn
linear-component name=mix input=Append(bn, idct, lin) dim=96
output-layer name=output dim=40 include-log-softmax=false"""
    T = 50
    net = kf.Network(xcfg, max_frames=T)
    params, bns = synth.init_network(net, seed=9)
    feats = synth.make_features(T, 40)
    fb = kf.upload_fp16(feats)
    net.forward(fb.ptr, T)
    names = [l[0] for l in net.layers]
    assert "mix.append1" in names and "mix.append2" in names
    cat = net.read_activation("mix.append2").astype(np.float32)
    ref = np.concatenate([net.read_activation(n).astype(np.float32) for n in ("bn", "idct", "lin")], 1)
    np.testing.assert_array_equal(cat, ref)
    tp = {k: synth.trunc_fp16(v) for k, v in params.items()}
    on = oracle.OracleNet(xcfg, tp, bns, round_mode=oracle.ROUND_FUSED, threads=8)
    on.forward(feats.astype(np.float32))
    for name in names:
        got = net.read_activation(name).astype(np.float32)
        assert rel_fro(got, on.act(name)) <= 2e-3, (name, rel_fro(got, on.act(name)))
    on.close()
    net.close()


def test_numerical_gradient_output_layer(gpu):
    kf = gpu
    from kfp16 import synth
    T = 4
    rng = np.random.default_rng(299)
    feats = (rng.random((T, 40)) * 2 - 1).astype(np.float16)
    net = kf.Network(NUMGRAD_NET, max_frames=T)
    params, _ = synth.init_network(net, seed=13)
    fb = kf.upload_fp16(feats)

    def loss(p):
        net.set_params(p)
        net.forward(fb.ptr, T)
        return float(net.read_activation("output").astype(np.float64).sum())

    net.forward(fb.ptr, T)
    ones = kf.upload_fp16(np.ones((T, 40), np.float16))
    net.backward(ones.ptr)
    ana = net.read_grads()["output.W"].ravel()
    W = params["output.W"].copy()
    flat = W.ravel()
    eps, n = 0.1, 20
    step = max(1, flat.size // n)
    max_rel = max_abs = 0.0
    for idx in list(range(0, flat.size, step))[:n]:
        orig = flat[idx]
        p = dict(params)
        flat[idx] = orig + eps
        p["output.W"] = flat.reshape(W.shape).copy()
        lp = loss(p)
        flat[idx] = orig - eps
        p["output.W"] = flat.reshape(W.shape).copy()
        lm = loss(p)
        flat[idx] = orig
        num = (lp - lm) / (2 * eps)
        a = float(ana[idx])
        ae = abs(num - a)
        max_abs = max(max_abs, ae)
        max_rel = max(max_rel, ae / max(abs(num), abs(a), 1e-6))
    assert not (max_rel > 0.2 and max_abs > 0.1), (max_rel, max_abs)
    # the output layer is affine in its weights: the difference quotient is exact up to
    # fp16 rounding of the perturbed weights and of the output (|d| <= 2e-2 here)
    assert max_abs <= 2e-2, max_abs
    net.close()
