"""The chain-objective oracle (oracle/kf_oracle_chain.c) pinned before it is
trusted as the checker of the HIP kernels.

Pins, in order of strength:
  * the reference's own fixture of internal/nnet/backward_test.go:28-140 (linear
    numerator FST, T=10, 20 pdfs, nnet = 0.5*sin(0.1*i)): the numerator log-prob
    is the sum of the path's outputs, its posteriors are one-hot, and the
    finite-difference gradient equals the posteriors (tolerance 1e-3, as there);
  * an independent float64 dense-matrix restatement of the leaky-HMM
    denominator recursion of chain_den.cu:496-706 (numpy, no shared code);
  * finite differences of the denominator log-prob (its gradient is the
    denominator posterior — Kaldi's identity the reference relies on);
  * the assembly rules of backward.go:224-371 (penalty on even frames only, L2
    term, NaN rule).
The reference's real-data constants (chainverify/main.go:83-96) need den.fst and
cegs archives that are not in its repository: parity on real data is unpinned.
"""
import numpy as np
import pytest

import oracle


def linear_fst(T, P):
    """backward_test.go:47-63: state t -> t+1 with pdf t % P, weight 0; every
    state final (computeChainLossCPU :196-199). Labels here are 1-indexed."""
    S = T + 1
    return dict(S=S, A=T, row_ptr=np.array(list(range(T)) + [T, T], np.int32)[: S + 1],
                dst=np.arange(1, T + 1, dtype=np.int32),
                pdf1=(np.arange(T) % P + 1).astype(np.int32),
                logw=np.zeros(T, np.float32), final_state=np.arange(S, dtype=np.int32),
                final_w=np.zeros(S, np.float32), start=0)


def fixture_nnet(T, P):
    return (np.sin(np.arange(T * P) * 0.1) * 0.5).astype(np.float32).reshape(T, P)


def test_backward_test_go_fixture():
    T, P = 10, 20
    f = linear_fst(T, P)
    x = fixture_nnet(T, P)
    lp, post = oracle.num_forward_backward(f, x)
    path = x[np.arange(T), np.arange(T) % P]
    assert abs(lp - float(np.sum(path.astype(np.float64)))) < 1e-5
    onehot = np.zeros((T, P), np.float32)
    onehot[np.arange(T), np.arange(T) % P] = 1
    np.testing.assert_allclose(post, onehot, atol=1e-6)
    # finite differences (backward_test.go:84-133, epsilon 1e-4 there; the
    # objective is linear in x on this FST, so any step is exact)
    eps = 1e-2
    for idx in range(0, T * P, 4):
        t, p = divmod(idx, P)
        xp, xm = x.copy(), x.copy()
        xp[t, p] += eps
        xm[t, p] -= eps
        fd = (oracle.num_forward_backward(f, xp, False)[0]
              - oracle.num_forward_backward(f, xm, False)[0]) / (2 * eps)
        assert abs(fd - post[t, p]) <= 1e-3 * max(1.0, abs(fd)), (t, p, fd, post[t, p])


def small_den(S=24, A=90, P=12, seed=5):
    rng = np.random.default_rng(seed)
    src = np.concatenate([np.arange(S), rng.integers(0, S, A - S)]).astype(np.int32)
    dst = np.concatenate([(np.arange(S) + 1) % S, rng.integers(0, S, A - S)]).astype(np.int32)
    order = np.argsort(src, kind="stable")
    src, dst = src[order], dst[order]
    pdf0 = rng.integers(0, P, A).astype(np.int32)
    tp = np.exp(-rng.uniform(0.5, 5, A)).astype(np.float32)
    return dict(S=S, P=P, A=A, src=src, dst=dst, pdf0=pdf0, tp=tp, start=0)


def dense_den_f64(g, init, x, leaky):
    """Independent float64 restatement: per frame a dense S x S transition
    matrix M_t[i, j] = sum_{arcs i->j} tp * exp(clamp(x_t[pdf])); alpha' recursion
    with per-frame normalisation, then the backward/posterior pass."""
    S, P = g["S"], g["P"]
    T = x.shape[0]
    ex = np.exp(np.clip(x.astype(np.float64), -30, 30))
    init = init.astype(np.float64)
    alphas, sums = [], []
    a = init.copy()
    s = a.sum()
    ad = a + s * leaky * init
    alphas.append(ad)
    sums.append(s)
    logc = 0.0
    for t in range(T):
        M = np.zeros((S, S))
        np.add.at(M, (g["src"], g["dst"]), g["tp"].astype(np.float64) * ex[t, g["pdf0"]])
        a = (ad @ M) / s
        logc += np.log(s)
        s = a.sum()
        ad = a + s * leaky * init
        alphas.append(ad)
        sums.append(s)
    total = ad.sum()
    lp = np.log(total) + logc
    post = np.zeros((T, P))
    bd = np.full(S, 1.0 / total)
    b = bd + leaky * (init @ bd)
    for t in range(T - 1, -1, -1):
        w = g["tp"].astype(np.float64) * ex[t, g["pdf0"]]
        occ = alphas[t][g["src"]] * w * b[g["dst"]] / sums[t]
        np.add.at(post[t], g["pdf0"], occ)
        bd = np.zeros(S)
        np.add.at(bd, g["src"], w * b[g["dst"]])
        bd /= sums[t]
        b = bd + leaky * (init @ bd)
    return lp, post


def test_initial_probs_match_f64_restatement():
    g = small_den()
    init = oracle.den_initial_probs(g)
    cur = np.zeros(g["S"])
    cur[0] = 1.0
    avg = np.zeros(g["S"])
    for _ in range(100):
        avg += cur / 100.0
        nxt = np.zeros(g["S"])
        np.add.at(nxt, g["dst"], cur[g["src"]] * g["tp"].astype(np.float64))
        cur = nxt / nxt.sum()
    np.testing.assert_allclose(init, avg.astype(np.float32), rtol=1e-6, atol=1e-12)
    assert abs(float(init.sum()) - 1.0) < 1e-5 and np.all(init >= 0)


@pytest.mark.parametrize("leaky", [1e-5, 0.1])
def test_den_matches_dense_f64(leaky):
    g = small_den()
    init = oracle.den_initial_probs(g)
    x = np.random.default_rng(1).standard_normal((9, g["P"])).astype(np.float32) * 2
    x[3, 2] = 40.0  # exercises the +-30 clamp of kernel_apply_exp
    lp, post = oracle.den_forward_backward(g, init, x, leaky)
    lp64, post64 = dense_den_f64(g, init, x, leaky)
    assert abs(lp - lp64) <= 1e-5 * max(1.0, abs(lp64))
    np.testing.assert_allclose(post, post64, atol=2e-6)
    # per-frame occupation sums to 1
    np.testing.assert_allclose(post.sum(1), 1.0, atol=1e-5)


def test_den_finite_difference():
    g = small_den()
    init = oracle.den_initial_probs(g)
    x = np.random.default_rng(2).standard_normal((6, g["P"])).astype(np.float32)
    lp, post = oracle.den_forward_backward(g, init, x)
    eps = 1e-2
    for t in range(6):
        for p in range(0, g["P"], 3):
            xp, xm = x.copy(), x.copy()
            xp[t, p] += eps
            xm[t, p] -= eps
            fd = (oracle.den_forward_backward(g, init, xp, posteriors=False)[0]
                  - oracle.den_forward_backward(g, init, xm, posteriors=False)[0]) / (2 * eps)
            assert abs(fd - post[t, p]) <= 3e-3, (t, p, fd, post[t, p])


def test_full_size_den_and_num_properties():
    from kfp16 import synth
    g = synth.make_den_graph()
    init = oracle.den_initial_probs(g)
    f = synth.make_num_fst(0)
    x = (np.random.default_rng(0).standard_normal((490, 3080)) * 2).astype(np.float16).astype(np.float32)
    lp, post = oracle.den_forward_backward(g, init, x)
    assert np.isfinite(lp)
    np.testing.assert_allclose(post.sum(1), 1.0, atol=1e-4)
    nl, npost = oracle.num_forward_backward(f, x)
    assert np.isfinite(nl) and nl < lp + 1e4
    # float32 log-domain sums lose ~|total| * 2^-24 per frame (the reference's own precision)
    np.testing.assert_allclose(npost.sum(1), 1.0, atol=3e-3)


def test_objective_assembly_rules():
    g = small_den()
    init = oracle.den_initial_probs(g)
    T, P = 8, g["P"]
    f = linear_fst(T, P)
    x = np.random.default_rng(3).standard_normal((T, P)).astype(np.float32)
    x[0, 1], x[1, 1], x[2, 3] = 35.0, -40.0, -31.0   # frame 1 is odd: not penalised
    d, r = oracle.chain_objf(g, init, f, x, l2=0.0, oor=0.01)
    assert r["out_of_range"] == 2 and r["ok"] == 1
    xr = x.astype(np.float16).astype(np.float32)
    nl, npost = oracle.num_forward_backward(f, xr)
    dl, dpost = oracle.den_forward_backward(g, init, x)
    ref = npost - dpost
    ref[0, 1] += (30.0 - 35.0) * 0.02
    ref[2, 3] += (-30.0 + 31.0) * 0.02
    np.testing.assert_allclose(d, ref, atol=1e-6)
    assert abs(r["objf"] - (nl - dl)) < 1e-3
    d2, r2 = oracle.chain_objf(g, init, f, x, l2=0.5, oor=0.0)
    np.testing.assert_allclose(d2, npost - dpost - 0.5 * x, atol=1e-5)
    assert abs(r2["l2_term"] + 0.25 * float(np.sum(x.astype(np.float64) ** 2))) < 1e-3
    xn = x.copy()
    xn[4, 4] = np.nan  # on the numerator path (pdf 4 at frame 4)
    d3, r3 = oracle.chain_objf(g, init, f, xn)
    assert r3["ok"] == 0 and r3["objf"] == -10.0 * T and not np.any(d3)
