"""The oracle's restricted attention (oracle/kf_oracle.c att_forward / att_backward).

Forward: against a direct numpy restatement of the reference's per-head loop
(internal/nnet/forward.go:850-893), including the zero-padded context rows.
Backward: the reference has no gradient for this layer (network_backward.go:539-544
reuses its conv backward), so the oracle's exact backward is pinned by central finite
differences of the oracle's own forward (no rounding, ReLU decisions replayed)."""
import numpy as np

import oracle

XCFG = """input name=input dim=24
attention-relu-batchnorm-layer name=att num-heads=2 value-dim=6 key-dim=5 num-left-inputs=3 num-right-inputs=1 time-stride=2
output-layer name=output dim=8 include-log-softmax=false
"""


def _setup(seed=0, T=23):
    rng = np.random.default_rng(seed)
    L = oracle.parse_xconfig(XCFG)
    A = 2 * (2 * 5 + 6 + 5)
    params = {"att.W": rng.standard_normal((24, A)).astype(np.float32) * 0.4,
              "att.Bias": rng.standard_normal((1, A)).astype(np.float32) * 0.1,
              "output.W": rng.standard_normal((L[0]["out_dim"], 8)).astype(np.float32) * 0.3,
              "output.Bias": np.zeros((1, 8), np.float32)}
    x = rng.standard_normal((T, 24)).astype(np.float32)
    return params, x


def _ref_forward(params, x):
    """forward.go:813-893 in float64 (no rounding): affine, padded per-head attention."""
    H, kd, vd, ctx, nl, st = 2, 5, 6, 5, 3, 2
    A = 2 * kd + vd + ctx
    proj = x.astype(np.float64) @ params["att.W"] + params["att.Bias"]
    T = x.shape[0]
    out = np.zeros((T, H * (vd + ctx)))
    for h in range(H):
        for t in range(T):
            q = proj[t, h * A:(h + 1) * A]
            b = np.zeros(ctx)
            rows = [t + (o - nl) * st for o in range(ctx)]
            for o, r in enumerate(rows):
                k = proj[r, h * A:h * A + kd] if 0 <= r < T else np.zeros(kd)
                b[o] = q[kd + vd + kd + o] + (1 / np.sqrt(kd)) * q[kd + vd:kd + vd + kd] @ k
            w = np.exp(b - b.max())
            w /= w.sum()
            for o, r in enumerate(rows):
                if 0 <= r < T:
                    out[t, h * (vd + ctx):h * (vd + ctx) + vd] += w[o] * proj[r, h * A + kd:h * A + kd + vd]
                out[t, h * (vd + ctx) + vd + o] = w[o]
    return out


def test_forward_matches_reference_loop():
    params, x = _setup()
    on = oracle.OracleNet(XCFG, params, {}, round_mode=oracle.ROUND_NONE)
    on.forward(x)
    ref = np.maximum(_ref_forward(params, x), 0.0) / np.sqrt(1 + 1e-3)  # ReLU; identity-stats BatchNorm (eps 1e-3)
    np.testing.assert_allclose(on.act("att"), ref, rtol=2e-5, atol=2e-6)


def test_backward_matches_finite_differences():
    params, x = _setup(1)
    on = oracle.OracleNet(XCFG, params, {}, round_mode=oracle.ROUND_NONE)
    on.forward(x)
    masks = {"att": on.mask("att")}
    og = np.random.default_rng(5).standard_normal((x.shape[0], 8)).astype(np.float32)
    on.backward(og)
    g = on.grads()["att.W"]

    def loss(W):
        p = dict(params)
        p["att.W"] = W
        o2 = oracle.OracleNet(XCFG, p, {}, round_mode=oracle.ROUND_NONE)
        o2.forward(x, force_masks=masks)
        return float(np.sum(o2.act("output").astype(np.float64) * og))

    rng = np.random.default_rng(2)
    picks = [tuple(int(v) for v in np.unravel_index(i, g.shape)) for i in np.argsort(-np.abs(g).ravel())[:12]]
    picks += [(int(rng.integers(24)), int(rng.integers(g.shape[1]))) for _ in range(6)]
    for (i, j) in picks:
        eps = 2e-3
        Wp, Wm = params["att.W"].copy(), params["att.W"].copy()
        Wp[i, j] += eps
        Wm[i, j] -= eps
        num = (loss(Wp) - loss(Wm)) / (2 * eps)
        assert abs(num - g[i, j]) <= 2e-2 * max(1.0, abs(g[i, j])), ((i, j), num, g[i, j])
