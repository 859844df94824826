"""Kaldi nnet3 text import (include/kf_model.h, host/nnet3_import.cpp) on the CPU.

The expectations of the reference's internal/nnet/weight_loader_test.go are restated
case for case on its own fixtures (tests/golden/nnet3_*.txt, extracted by
tests/golden/make_nnet3_fixtures.py), and the C++ parser is compared field by field
with the pure-Python restatement in oracle/nnet3_text.py.
"""
import os

import numpy as np
import pytest

import nnet3_text as T
from kfp16 import model

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _fixture(n):
    return open(os.path.join(GOLD, f"nnet3_{n}.txt")).read()


def _close(a, b, tol):
    assert abs(float(a) - float(b)) <= tol, (a, b)


def test_parse_nnet3_text():                       # TestParseNnet3Text / TestComponentCount
    m = model.Nnet3Model.from_text(_fixture("components"))
    assert sorted(m.names()) == sorted([
        "idct", "ivector-linear", "ivector-batchnorm", "cnn1.conv", "cnn1.relu", "cnn1.batchnorm",
        "tdnnf7.linear", "tdnnf7.affine", "tdnnf7.batchnorm", "prefinal-chain.affine", "output.affine",
        "noop1", "output-xent.log-softmax"])
    c = m["idct"]
    assert c.type == "FixedAffineComponent" and c.linear.shape == (2, 4) and len(c.bias) == 4
    _close(c.linear[0, 0], 0.1581139, 1e-5)
    _close(c.linear[1, 0], 0.1581139, 1e-5)
    c = m["ivector-linear"]
    assert c.type == "LinearComponent" and c.linear.shape == (2, 3)
    assert c.learning_rate == np.float32(0.0001) and c.l2_regularize == np.float32(0.03)
    assert c.max_change == np.float32(0.75)
    c = m["ivector-batchnorm"]
    assert c.type == "BatchNormComponent" and c.epsilon == np.float32(0.001)
    assert c.target_rms == np.float32(0.025) and c.count == 176000
    assert len(c.stats_mean) == 4 and len(c.stats_var) == 4
    _close(c.stats_mean[0], -0.005183299, 1e-6)
    _close(c.stats_var[0], 0.1, 1e-6)
    c = m["cnn1.conv"]
    assert c.type == "TimeHeightConvolutionComponent"
    assert (c.num_filters_in, c.num_filters_out, c.height_in, c.height_out) == (6, 48, 40, 40)
    assert c.linear.shape == (2, 3) and len(c.bias) == 3
    _close(c.bias[0], 0.05598261, 1e-6)
    c = m["tdnnf7.linear"]
    assert c.type == "TdnnComponent" and c.linear.shape == (2, 2) and len(c.bias) == 0
    _close(c.linear[0, 0], 3.699428e-43, 1e-45)     # float32 denormal kept
    c = m["tdnnf7.affine"]
    assert c.linear.shape == (2, 3) and len(c.bias) == 3
    _close(c.bias[0], -1.943402e-05, 1e-8)
    c = m["prefinal-chain.affine"]
    assert c.type == "NaturalGradientAffineComponent" and c.linear.shape == (2, 2) and len(c.bias) == 2
    c = m["output.affine"]
    assert c.linear.shape == (3, 3)
    _close(c.linear[2, 2], 0.9, 1e-6)
    c = m["noop1"]
    assert c.type == "NoOpComponent" and c.linear.size == 0
    assert m["output-xent.log-softmax"].type == "LogSoftmaxComponent"


def test_real_batchnorm_line():                    # TestParseRealBatchNormLine
    c = model.Nnet3Model.from_text(_fixture("bn_line"))["prefinal-chain.batchnorm2"]
    assert c.epsilon == np.float32(0.001) and c.target_rms == 1.0 and c.count == 41344
    assert len(c.stats_mean) == 3
    _close(c.stats_mean[0], 4.844032e-10, 1e-15)


def test_inline_vector_and_prefinal_line():        # TestParseInlineVector / TestParseRealPrefinalLine
    c = model.Nnet3Model.from_text(_fixture("inline_vector"))["test"]
    assert len(c.stats_mean) == 3 and len(c.stats_var) == 3
    _close(c.stats_mean[0], 0.1, 1e-6)
    _close(c.stats_var[2], 0.6, 1e-6)
    c = model.Nnet3Model.from_text(_fixture("prefinal_line"))["prefinal-chain.affine"]
    assert c.linear.shape == (2, 2) and len(c.bias) == 2


def test_batchnorm_computation():                  # TestBatchNormComputation (replaceBN arithmetic)
    g, b = T.replace_bn([-0.005183299], [0.1], 0.001, 0.025)
    _close(g[0], 0.025 / np.sqrt(0.1 + 0.001), 1e-5)
    _close(b[0], 0.005183299 * g[0], 1e-8)


def _same(cpp, py):
    for name, pc in py.items():
        c = cpp[name]
        assert c.type == pc["type"]
        assert c.linear.shape == ((pc["rows"], pc["cols"]) if pc["linear"] else (0, 0))
        for arr, key in ((c.linear.reshape(-1), "linear"), (c.bias, "bias"), (c.stats_mean, "mean"),
                         (c.stats_var, "var")):
            assert np.array_equal(arr.view(np.uint32), np.asarray(pc[key], np.float32).view(np.uint32)), (name, key)
        assert (c.count, c.num_filters_in, c.num_filters_out, c.height_in, c.height_out) == \
            (pc["count"], pc["nfi"], pc["nfo"], pc["hin"], pc["hout"])
        for a, k in ((c.epsilon, "eps"), (c.target_rms, "rms"), (c.learning_rate, "lr"), (c.max_change, "maxc"),
                     (c.l2_regularize, "l2")):
            assert np.float32(a) == np.float32(pc[k]), (name, k)
    assert sorted(cpp.names()) == sorted(py)


@pytest.mark.parametrize("fx", ["components", "bn_line", "inline_vector", "prefinal_line"])
def test_cpp_matches_oracle_on_fixtures(fx):
    txt = _fixture(fx)
    _same(model.Nnet3Model.from_text(txt), T.parse(txt))


def test_edge_cases_match_oracle():
    txt = "\r\n".join([
        "junk before any component <LinearParams> [ 1 2 3 ]",
        "<ComponentName> a <AffineComponent> <LearningRate> 1e500 <MaxChange> abc <LinearParams>  [ 7 8",
        "  1 2 x 3",                      # unparsable token skipped
        "  4 5 1e99 6 ]",                 # float32 overflow skipped
        "<BiasParams>  [ ]",              # empty vector: no bias
        "<ComponentName> b <BatchNormComponent> <Epsilon> 0 <TargetRms> 2 <Count> 5 <StatsMean> [ 1 2 ]",
        "<StatsVar> [ 3 4 ]",
        "<Epsilon> 0.5 <TargetRms> 9 <Count> 6",   # continuation tags: eps set (was 0), rms kept, count overwritten
        "<ComponentName> a <LinearComponent> <Params>  [",
        "  0.5 0.25",
        "",
        "  0.125 0.0625 ]",
        "<ComponentName> c <X> <StatsMean> [",
        "  1 2 3",                        # never closed: finished at end of input
    ])
    cpp, py = model.Nnet3Model.from_text(txt), T.parse(txt)
    _same(cpp, py)
    assert cpp["a"].type == "LinearComponent" and cpp["a"].linear.tolist() == [[0.5, 0.25], [0.125, 0.0625]]
    b = cpp["b"]
    assert b.epsilon == 0.5 and b.target_rms == 2 and b.count == 6
    assert cpp["c"].stats_mean.tolist() == [1, 2, 3]
    assert cpp.names() == ["a", "b", "c"]


def test_generated_model_text_matches_oracle():
    rng = np.random.default_rng(0)
    parts = []
    for i in range(5):
        parts.append(T.write_component(f"tdnnf{i}.affine", "TdnnComponent", rng.standard_normal((48, 96)) * 1e-3,
                                       rng.standard_normal(48)))
        parts.append(T.write_component(f"tdnnf{i}.batchnorm", "BatchNormComponent", mean=rng.standard_normal(48),
                                       var=rng.uniform(0.5, 2, 48), bn_dim=48))
    txt = "".join(parts)
    cpp, py = model.Nnet3Model.from_text(txt), T.parse(txt)
    _same(cpp, py)
    assert cpp["tdnnf3.affine"].linear.shape == (48, 96)


def test_errors():
    with pytest.raises(model.ModelError, match="cannot open"):
        model.Nnet3Model.from_file("/nonexistent/final.txt")
    with pytest.raises(model.ModelError, match="nnet3-copy"):
        model.Nnet3Model.export("/nonexistent/final.mdl")   # Kaldi is not in this image
