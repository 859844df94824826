"""Kaldi's ivector input path on the MI355X against the oracle:
ReplaceIndex(ivector, t, 0) -> ivector-linear -> ivector-batchnorm on one row per
sequence, combine-feature-maps of Append(idct-batchnorm, ivector-batchnorm) with the
per-sequence rows broadcast to their frames, and cnn1 with 6 input filters (im2col +
GEMM). Backward reaches ivector-linear through the per-sequence column sums.
The reference appends tensors of different row counts here (forward.go:263-296), so the
oracle restates Kaldi's semantics (tests: SURVEY §8d tolerances)."""
import numpy as np
import pytest

from conftest import max_abs_rel, rel_fro

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("cfg,T,B", [("tiny_ivec.xconfig", 150, 3), ("tiny_ivec.xconfig", 301, 5),
                                      ("cnn_tdnn_17f_ivec.xconfig", 240, 2),
                                      ("cnn_tdnn_17f_kaldi.xconfig", 240, 2)])
def test_ivector_network_forward_backward(gpu, cfg, T, B):
    kf = gpu
    from kfp16 import synth
    xcfg = synth.load_xconfig(cfg)
    net = kf.Network(xcfg, max_frames=T)
    params, bns = synth.init_network(net)
    feats = synth.make_features(T, 40)
    rng = np.random.default_rng(T)
    ivec = (rng.standard_normal((B, 100)) * 2).astype(np.float16)
    cuts = np.sort(rng.choice(np.arange(10, T - 10), B - 1, replace=False))
    seq = np.concatenate([[0], cuts, [T]]).astype(np.int32)
    fbuf, ibuf = kf.upload_fp16(feats), kf.upload_fp16(ivec)
    net.forward_ivector(fbuf.ptr, T, ibuf.ptr, seq)

    from kfp16 import synth as _s
    import oracle as O
    tp = {k: _s.trunc_fp16(v) for k, v in params.items()}
    on = O.OracleNet(xcfg, tp, bns, round_mode=O.ROUND_FUSED, threads=16)
    on.forward(feats.astype(np.float32), ivectors=ivec.astype(np.float32), seq_off=seq)
    masks = net.relu_masks()
    per_seq = {"ivector-linear", "ivector-batchnorm"}
    for name, ty, din, dout in net.layers:
        got = net.read_activation(name).astype(np.float32)
        ref = on.act(name)
        if name in per_seq:
            got = got[:B]
        assert rel_fro(got, ref) <= 2e-3, (name, rel_fro(got, ref))
        assert max_abs_rel(got, ref) <= 1e-2, (name, max_abs_rel(got, ref))
        if name in masks:
            assert float(np.mean(masks[name] == on.mask(name))) >= 0.999, name
    on.close()
    on = O.OracleNet(xcfg, tp, bns, round_mode=O.ROUND_FUSED, threads=16)
    on.forward(feats.astype(np.float32), force_masks=masks, ivectors=ivec.astype(np.float32), seq_off=seq)
    P = [dout for name, ty, din, dout in net.layers if name == "output"][0]
    og = (np.random.default_rng(7).standard_normal((T, P)) * 0.05).astype(np.float16)
    gbuf = kf.upload_fp16(og)
    net.backward(gbuf.ptr)
    got = net.read_grads()
    on.backward(og.astype(np.float32))
    ref = on.grads()
    errs = {k: rel_fro(got[k], ref[k]) for k in ref}
    bad = {k: v for k, v in errs.items() if v > 5e-3}
    assert not bad, "grad errors: " + ", ".join(f"{k}={v:.2e}" for k, v in errs.items())
    assert np.abs(got["ivector-linear.W"]).sum() > 0
    for k in got:  # the xent branch (Kaldi recipe config) gets no gradient
        if k.startswith(("prefinal-xent.", "output-xent.")):
            assert not np.any(got[k]), k


def test_ivector_input_required(gpu):
    kf = gpu
    from kfp16 import synth
    net = kf.Network(synth.load_xconfig("tiny_ivec.xconfig"), max_frames=64)
    fbuf = kf.upload_fp16(np.zeros((64, 40), np.float16))
    with pytest.raises(kf.KfError, match="ivector"):
        net.forward(fbuf.ptr, 64)
