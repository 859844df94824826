"""The build's conv layers against the reference's own conv formulation
(oracle/ref_emulation.py, internal/nnet/forward.go:418-524), on the GPU.

With cross-product weights that carry only the reference's zipped taps (t_i, h_i),
every conv layer of tiny.xconfig computed by the MI355X kernels (cnn1: k_conv_c1,
cnn2-4: the implicit-im2col MFMA GEMM) must equal the reference's formulation of that
layer — zipped patches, GEMM, bias, ReLU, filter-major reorder, BN, each stored fp16 —
read through the filter-major permutation. Each layer is fed the GPU's own input to it.
Tolerance: rel-Frobenius <= 1e-2 (the R-mode bar of SURVEY §8d: the reference rounds
after every op, the build once per tensor) and max-abs <= 2e-2 * max|ref|.
"""
import numpy as np
import pytest

import ref_emulation as RE
from conftest import max_abs_rel, rel_fro

pytestmark = pytest.mark.gpu


def test_conv_layers_match_reference_formulation(gpu):
    kf = gpu
    import oracle
    from kfp16 import synth
    xcfg = synth.load_xconfig("tiny.xconfig")
    L = {l["name"]: l for l in oracle.parse_xconfig(xcfg)}
    T = 150
    net = kf.Network(xcfg, max_frames=T)
    params, bns = synth.init_network(net, seed=3)
    rng = np.random.default_rng(17)
    wzip = {}
    for name in ("cnn1", "cnn2", "cnn3", "cnn4"):
        l = L[name]
        wz = (rng.standard_normal((3 * l["fin"], l["fout"])) * np.sqrt(2.0 / (3 * l["fin"]))).astype(np.float32)
        wzip[name] = wz
        params[name + ".W"] = RE.cross_weights_from_zipped(wz, l["fin"], l["toffs"], l["hoffs"])
    net.set_params(params)
    feats = synth.make_features(T, 40)
    fb = kf.upload_fp16(feats)
    net.forward(fb.ptr, T)
    for name in ("cnn1", "cnn2", "cnn3", "cnn4"):
        l = L[name]
        x = net.read_activation(l["input"]).astype(np.float32)
        m, v, g, b = bns[(name, 0)]
        bn = (np.repeat(m, l["hout"]), np.repeat(v, l["hout"]), np.repeat(g, l["hout"]),
              np.repeat(b, l["hout"]), 1e-3)
        ref = RE.conv_relu_bn_ref(x, T, l["hin"], l["fin"], l["hout"], l["sub"], l["toffs"], l["hoffs"],
                                  synth.trunc_fp16(wzip[name]), synth.trunc_fp16(params[name + ".Bias"])[0], bn)
        got = RE.height_major_to_filter_major(net.read_activation(name).astype(np.float32), T,
                                              l["hout"], l["fout"])
        assert rel_fro(got, ref) <= 1e-2, (name, rel_fro(got, ref))
        assert max_abs_rel(got, ref) <= 2e-2, (name, max_abs_rel(got, ref))
    net.close()
