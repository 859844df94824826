"""The oracle's ivector front end (oracle/kf_oracle.c: per-sequence layers, ORC_COMBINE).

Kaldi semantics: ReplaceIndex(ivector, t, 0) gives every frame of a
sequence that sequence's ivector, so ivector-linear and ivector-batchnorm run on one row
per sequence, and combine-feature-maps interleaves per height the nf1 feature filters
with the nf2 ivector filters of the frame's sequence. The reference appends tensors of
different row counts here (internal/nnet/forward.go:263-296), so there is no reference
output to pin against. Forward is pinned by a float64 numpy restatement of those
semantics. Backward, including the per-sequence column sums into ivector-linear, is
pinned by central finite differences of the oracle's own forward."""
import numpy as np

import oracle

XCFG = """input name=ivector dim=7
input name=input dim=4
linear-component name=ivector-linear input=ReplaceIndex(ivector, t, 0) dim=12
batchnorm-component name=ivector-batchnorm target-rms=0.5
batchnorm-component name=feat-batchnorm input=input
combine-feature-maps-layer name=combine input=Append(feat-batchnorm, ivector-batchnorm) num-filters1=1 num-filters2=3 height=4
output-layer name=output dim=5 include-log-softmax=false
"""
SEQ = np.array([0, 4, 5, 11], np.int32)   # ragged: 4, 1 and 6 frames
EPS = 1e-3


def _setup(seed=0):
    rng = np.random.default_rng(seed)
    params = {"ivector-linear.W": rng.standard_normal((7, 12)).astype(np.float32) * 0.5,
              "output.W": rng.standard_normal((16, 5)).astype(np.float32) * 0.4,
              "output.Bias": rng.standard_normal((1, 5)).astype(np.float32) * 0.1}
    bns = {("ivector-batchnorm", 0): (rng.standard_normal(12).astype(np.float32) * 0.1,
                                      (rng.random(12) + 0.5).astype(np.float32),
                                      np.ones(12, np.float32), np.zeros(12, np.float32))}
    x = rng.standard_normal((int(SEQ[-1]), 4)).astype(np.float32)
    iv = rng.standard_normal((len(SEQ) - 1, 7)).astype(np.float32)
    return params, bns, x, iv


def _ref_forward(params, bns, x, iv):
    """Kaldi's front end in float64: per-sequence linear + target-rms BN, broadcast, combine."""
    m, v, _, _ = bns[("ivector-batchnorm", 0)]
    lin = iv.astype(np.float64) @ params["ivector-linear.W"]
    ibn = (lin - m) * (0.5 / np.sqrt(v.astype(np.float64) + EPS))
    fbn = x.astype(np.float64) / np.sqrt(1 + EPS)
    T, H, n1, n2 = x.shape[0], 4, 1, 3
    comb = np.zeros((T, H * (n1 + n2)))
    for s in range(len(SEQ) - 1):
        for t in range(SEQ[s], SEQ[s + 1]):
            for h in range(H):
                comb[t, h * 4] = fbn[t, h]
                comb[t, h * 4 + 1:h * 4 + 4] = ibn[s, h * 3:h * 3 + 3]
    out = comb @ params["output.W"] + params["output.Bias"]
    return lin, ibn, comb, out


def test_forward_matches_kaldi_semantics():
    params, bns, x, iv = _setup()
    on = oracle.OracleNet(XCFG, params, bns, round_mode=oracle.ROUND_NONE)
    on.forward(x, ivectors=iv, seq_off=SEQ)
    lin, ibn, comb, out = _ref_forward(params, bns, x, iv)
    assert on.act("ivector-linear").shape == (3, 12)
    np.testing.assert_allclose(on.act("ivector-linear"), lin, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(on.act("ivector-batchnorm"), ibn, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(on.act("combine"), comb, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(on.act("output"), out, rtol=1e-5, atol=1e-5)


def test_backward_matches_finite_differences():
    params, bns, x, iv = _setup(1)
    og = np.random.default_rng(3).standard_normal((x.shape[0], 5)).astype(np.float32)
    on = oracle.OracleNet(XCFG, params, bns, round_mode=oracle.ROUND_NONE)
    on.forward(x, ivectors=iv, seq_off=SEQ)
    on.backward(og)
    grads = on.grads()

    def loss(p):
        o2 = oracle.OracleNet(XCFG, p, bns, round_mode=oracle.ROUND_NONE)
        o2.forward(x, ivectors=iv, seq_off=SEQ)
        return float(np.sum(o2.act("output").astype(np.float64) * og))

    for key in ("ivector-linear.W", "output.W"):
        g = grads[key].reshape(params[key].shape)
        assert np.abs(g).sum() > 0, key
        for i in range(params[key].shape[0]):
            for j in range(0, params[key].shape[1], 2):
                eps = 1e-2
                pp, pm = dict(params), dict(params)
                pp[key], pm[key] = params[key].copy(), params[key].copy()
                pp[key][i, j] += eps
                pm[key][i, j] -= eps
                num = (loss(pp) - loss(pm)) / (2 * eps)
                assert abs(num - g[i, j]) <= 1e-3 * max(1.0, abs(g[i, j])), (key, (i, j), num, g[i, j])


def test_sequence_without_ivector_rows_is_independent():
    """Changing one sequence's ivector changes only that sequence's frames."""
    params, bns, x, iv = _setup(2)
    on = oracle.OracleNet(XCFG, params, bns, round_mode=oracle.ROUND_NONE)
    on.forward(x, ivectors=iv, seq_off=SEQ)
    a = on.act("output")
    iv2 = iv.copy()
    iv2[1] += 1.0
    on.forward(x, ivectors=iv2, seq_off=SEQ)
    b = on.act("output")
    changed = np.any(a != b, axis=1)
    assert changed.tolist() == [False] * 4 + [True] + [False] * 6
