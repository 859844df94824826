"""The drop-in path end to end: the reference's Network.Forward host sequence
(internal/nnet/forward.go:148-1001, one ABI call per step: ops_gemm, the K = 1 GEMM
AddBias of ops.go:335-351, ops_relu, ops_batchnorm_forward, ops_copy / ops_concat_cols
splices, ops_add_scaled bypass; host im2col for the convolutions) replayed over this
build's C-ABI by kfp16.refpath, on cnn_tdnn_17f at T = 1500, against the oracle's
R mode (one fp16 rounding after every reference op). Bar: every layer's
activation within rel-Frobenius 1e-2 of R mode; the replay and the product's fused
path agree within the same bar (they differ only in where they round)."""
import numpy as np
import pytest

import oracle
from conftest import rel_fro

pytestmark = [pytest.mark.gpu, pytest.mark.slow]


@pytest.mark.parametrize("xname,T", [("tiny.xconfig", 300), ("cnn_tdnn_17f.xconfig", 1500)])
def test_refpath_forward_matches_r_mode(gpu, xname, T):
    kf = gpu
    from kfp16 import refpath, synth
    xcfg = synth.load_xconfig(xname)
    net = kf.Network(xcfg, max_frames=T)
    params, bns = synth.init_network(net, seed=21)
    feats = synth.make_features(T, 40, seed=9)
    fb = kf.upload_fp16(feats)
    rp = refpath.RefPathForward(xcfg, params, bns, T)
    rp.forward(fb.ptr, T)
    net.forward(fb.ptr, T)
    tp = {k: synth.trunc_fp16(v) for k, v in params.items()}
    onr = oracle.OracleNet(xcfg, tp, bns, round_mode=oracle.ROUND_REF, threads=16)
    onr.forward(feats.astype(np.float32))
    worst = {}
    for L in rp.layers:
        name = L["name"]
        got = rp.read(name).astype(np.float32)
        e = rel_fro(got, onr.act(name))
        worst[name] = e
        assert e <= 1e-2, (name, e)
        assert rel_fro(net.read_activation(name).astype(np.float32), got) <= 1e-2, name
    print("refpath vs R mode, worst layers:", sorted(worst.items(), key=lambda kv: -kv[1])[:3])
    rp.close()
    net.close()

