"""Host-layer xconfig parsing / layer resolution (internal/nnet/xconfig.go,
layers.go restated in C++), checked without a device."""
import pytest

import kfp16
from kfp16 import synth


def test_synthetic_model_dims():
    layers, nparams = kfp16.parse_summary(synth.load_xconfig("cnn_tdnn_17f.xconfig"))
    d = {n: (t, i, o) for n, t, i, o in layers}
    assert d["cnn1"] == (6, 40, 2560) and d["cnn3"][2] == 20 * 128 and d["cnn6"][2] == 2560
    assert d["tdnnf7"] == (7, 2560, 1536) and d["tdnnf23"] == (7, 1536, 1536)
    assert d["prefinal-chain"] == (9, 256, 256) and d["output"] == (10, 256, 3080)
    assert nparams == 19_527_112          # 19.53 M
    _, n3072 = kfp16.parse_summary(synth.load_xconfig("cnn_tdnn_17f_3072.xconfig"))
    assert n3072 == 69_067_208            # 69.07 M


def test_tokenizer_keeps_parenthesised_values_and_skips_vars():  # xconfig.go:215-271
    text = """input name=input dim=40
input name=ivector dim=100
linear-component name=lin input=Append(input, ivector) dim=32 $opts
output-layer name=output dim=8
"""
    layers, _ = kfp16.parse_summary(text)
    assert layers[2] == ("lin", 2, 140, 32)
    assert layers[3] == ("output", 10, 32, 8)


def test_resolve_prefix_names():  # layers.go:357-374
    text = """input name=input dim=40
linear-component name=tdnn1.affine dim=16
linear-component name=x input=tdnn1 dim=8
"""
    layers, _ = kfp16.parse_summary(text)
    assert layers[-1] == ("x", 2, 16, 8)


@pytest.mark.parametrize("text,msg", [
    ("foo-layer name=x dim=3\n", "unknown layer type"),
    ("input name=input dim=40\nlinear-component dim=3\n", "missing name"),
    ("input name=input dim=40\ntdnnf-layer name=t dim=10\n", "bottleneck-dim"),
    ("input name=input dim=40\nlinear-component name=l input=nope dim=4\n", "not found"),
])
def test_errors(text, msg):
    with pytest.raises(kfp16.KfError, match=msg):
        kfp16.parse_summary(text)
