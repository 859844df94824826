"""The gotorch-style float64 CPU network (oracle/gotorch_net.c, SURVEY §8 row P2: the
reference's Go CPU path as the CPU baseline's template) against the oracle's unrounded
fp32 restatement of the same network: activations and gradients agree to fp32 precision,
so the baseline times the same computation in the reference's CPU style."""
import numpy as np
import pytest

import oracle
from conftest import rel_fro


@pytest.mark.parametrize("T", [23, 64])
def test_gotorch_net_matches_oracle(T):
    import kfp16
    from kfp16 import synth
    xcfg = synth.load_xconfig("tiny.xconfig")
    net = kfp16.Network(xcfg, max_frames=T, layout_only=True)  # shapes only, no device
    params = synth.make_params(net.params)
    bns = synth.make_bn_all(synth.bn_specs(net.layers, *synth.layer_dims(net)))
    net.close()
    tp = {k: synth.trunc_fp16(v) for k, v in params.items()}
    feats = synth.make_features(T, 40).astype(np.float32)
    on = oracle.OracleNet(xcfg, tp, bns, round_mode=oracle.ROUND_NONE, threads=4)
    gt = oracle.GotorchNet(on, workers=4)
    on.forward(feats)
    gt.forward(feats)
    for L in on.L:
        assert rel_fro(gt.act(L["name"]), on.act(L["name"])) < 1e-5, L["name"]
    og = (np.random.default_rng(3).standard_normal((T, on.L[-1]["out_dim"])) * 0.05).astype(np.float32)
    on.backward(og)
    gt.backward(og)
    ref, got = on.grads(), gt.grads()
    assert set(ref) == set(got)
    for k in ref:
        assert rel_fro(got[k], ref[k].ravel()) < 1e-5, k
    # SGD (model.go:236-268): w -= lr * (0.9 v + g) with v = 0 on the first step
    w0 = gt._t("output", 5)
    gt.sgd(1e-2)
    assert np.allclose(gt._t("output", 5), w0 - 1e-2 * got["output.W"])
    gt.close()
    on.close()
