"""attention-relu-batchnorm layer on the MI355X against the oracle.

Forward: the affine on the fused GEMM, then k_att_fwd (restricted attention + ReLU +
BatchNorm) — the reference's CPU loop (forward.go:795-909), which the oracle restates
(tests/test_oracle_attention.py pins it). Backward: the exact gradient (k_att_bwd_q /
k_att_bwd_kv), compared with the oracle's exact backward (pinned there by finite
differences). Tolerances: SURVEY §8d (activations 2e-3 rel-Frobenius, gradients 5e-3)."""
import numpy as np
import pytest

from conftest import rel_fro
import oracle
from test_gpu_nnet import _forward_parity, _oracle

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("cfg,T", [("tiny_att.xconfig", 96), ("tiny_att.xconfig", 301),
                                   ("cnn_tdnn_17f_att.xconfig", 240)])
def test_attention_network_forward_backward(gpu, cfg, T):
    kf = gpu
    from kfp16 import synth
    xcfg = synth.load_xconfig(cfg)
    net = kf.Network(xcfg, max_frames=T)
    params, bns = synth.init_network(net)
    feats = synth.make_features(T, 40)
    fbuf = kf.upload_fp16(feats)
    net.forward(fbuf.ptr, T)
    on = _oracle(xcfg, params, bns, feats)
    masks = _forward_parity(net, on, None)
    on.close()
    on = _oracle(xcfg, params, bns, feats)
    on.forward(feats.astype(np.float32), force_masks=masks)
    P = [dout for name, ty, din, dout in net.layers if name == "output"][0]
    if cfg == "tiny_att.xconfig":
        og = (np.random.default_rng(7).standard_normal((T, P)) * 0.05).astype(np.float16)
        gbuf = kf.upload_fp16(og)
        net.backward(gbuf.ptr)
        got = net.read_grads()
        on.backward(og.astype(np.float32))
        ref = on.grads()
        errs = {k: rel_fro(got[k], ref[k]) for k in ref}
        bad = {k: v for k, v in errs.items() if v > 5e-3}
        assert not bad, "grad errors: " + ", ".join(f"{k}={v:.2e}" for k, v in errs.items())
        return
    # At full width (8 heads, key 64, value 128) the softmax backward w (dw - <w, dw>)
    # cancels, and fp16 rounding of its inputs moves the gradients at and below the layer
    # by ~1e-2 in the oracle's own F mode against fp32 (scripts/att_precision.py): the GPU
    # and the F restatement are then two independent fp16 draws around the fp32 gradient,
    # and their ratio of errors for one output gradient is noise (scripts/att_diag.py over
    # seeds 7-12: geometric means 1.19, 0.87, 1.10, 0.84, 0.91, 0.68, per-parameter
    # maxima up to 1.48). The bar is statistical: over three seeds the geometric mean of
    # |gpu - fp32| / |F - fp32| over all parameters <= 1.15 (the GPU is on average no
    # noisier than the fp16 restatement), each parameter <= max(5e-3, 1.6 F) and 3e-2.
    on.close()
    logs, bad = [], {}
    for seed in (7, 8, 9):
        og = (np.random.default_rng(seed).standard_normal((T, P)) * 0.05).astype(np.float16)
        gbuf = kf.upload_fp16(og)
        net.forward(fbuf.ptr, T)
        net.backward(gbuf.ptr)
        got = net.read_grads()
        grads = {}
        for mode in (oracle.ROUND_FUSED, oracle.ROUND_NONE):
            on = _oracle(xcfg, params, bns, feats, mode=mode)
            on.forward(feats.astype(np.float32), force_masks=masks)
            on.backward(og.astype(np.float32))
            grads[mode] = on.grads()
            on.close()
        ref, f32 = grads[oracle.ROUND_FUSED], grads[oracle.ROUND_NONE]
        for k in ref:
            g_err, f_err = rel_fro(got[k], f32[k]), rel_fro(ref[k], f32[k])
            if f_err > 0 and g_err > 0:
                logs.append(np.log(g_err / f_err))
            if g_err > max(5e-3, 1.6 * f_err) or g_err > 3e-2:
                bad[(seed, k)] = (g_err, f_err)
    gm = float(np.exp(np.mean(logs)))
    assert not bad, "grad errors vs fp32 (gpu, F): " + ", ".join(f"{k}={a:.2e}/{b:.2e}" for k, (a, b) in bad.items())
    assert gm <= 1.15, f"GPU gradients noisier than the fp16 restatement: geometric-mean error ratio {gm:.3f}"


def test_attention_import_key_scale(gpu):
    """NewNetworkFromKaldi for attention (weight_loader.go:221-275): affine, batchnorm and
    the <KeyScale> of <name>.attention; a different key scale changes the output."""
    kf = gpu
    from kfp16 import model, synth
    import nnet3_writer as NW
    import nnet3_text as TT
    xcfg = synth.load_xconfig("tiny_att.xconfig")
    T = 96
    a = kf.Network(xcfg, max_frames=T)
    params, bns = synth.init_network(a)
    txt = NW.network_text(a.layers, params, bns)
    m, v, _, _ = bns[("attention3", 0)]
    txt += TT.write_component("attention3.affine", "NaturalGradientAffineComponent",
                              params["attention3.W"].T, params["attention3.Bias"].reshape(-1))
    txt += TT.write_component("attention3.batchnorm", "BatchNormComponent", mean=m, var=v, bn_dim=len(m))
    b = kf.Network(xcfg, max_frames=T)
    model.Nnet3Model.from_text(txt).load_into(b)
    feats = synth.make_features(T, 40)
    fbuf = kf.upload_fp16(feats)
    a.forward(fbuf.ptr, T)
    b.forward(fbuf.ptr, T)
    assert np.array_equal(a.read_activation("attention3").view(np.uint16),
                          b.read_activation("attention3").view(np.uint16))
    c = kf.Network(xcfg, max_frames=T)
    model.Nnet3Model.from_text(txt + "<ComponentName> attention3.attention <RestrictedAttentionComponent> "
                               "<NumHeads> 4 <KeyDim> 16 <ValueDim> 32 <KeyScale> 0.9\n").load_into(c)
    c.forward(fbuf.ptr, T)
    assert not np.array_equal(a.read_activation("attention3"), c.read_activation("attention3"))
