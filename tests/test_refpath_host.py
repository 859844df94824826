"""Host-side pieces of kfp16.refpath that restate reference code (no GPU):
makeIDCTMatrix (forward.go:1190-1210) and float32ToFP16Bits (tensor.go:158-173)."""
import numpy as np

import oracle


def test_refpath_pieces_match_restatements():
    from kfp16 import refpath, synth
    np.testing.assert_array_equal(refpath.idct_matrix(40, 22.0), oracle.idct_matrix(40, 22.0))
    a = np.random.default_rng(0).standard_normal(4096).astype(np.float32) * 3
    a[:4] = [1e-6, -1e-7, 7e5, -7e5]   # subnormal flush and overflow to inf
    np.testing.assert_array_equal(refpath.fp16_trunc(a).astype(np.float32), synth.trunc_fp16(a))


def test_refpath_parses_the_benchmark_model():
    from kfp16 import refpath, synth
    layers = refpath.parse_layers(synth.load_xconfig("cnn_tdnn_17f.xconfig"))
    kinds = [L["kind"] for L in layers]
    assert kinds.count("tdnnf-layer") == 17 and kinds.count("conv-relu-batchnorm-layer") == 6
    cnn3 = next(L for L in layers if L["name"] == "cnn3")
    assert (cnn3["fin"], cnn3["hout"], cnn3["sub"], len(cnn3["offs"])) == (64, 20, 2, 9)
    t8 = next(L for L in layers if L["name"] == "tdnnf8")
    assert (t8["stride"], t8["bn_dim"], t8["bypass"]) == (3, 160, 0.66)
