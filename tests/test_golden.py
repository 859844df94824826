"""The oracle against the committed fixtures of tests/golden/ (see make_golden.py
for their provenance)."""
import os

import numpy as np

import oracle

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _bt_fst(z, x):
    T, P = x.shape
    S = T + 1
    # the GPU / oracle ABI takes 1-based labels (0 = epsilon): pdf0 + 1 (chain.h)
    return dict(S=S, A=T, row_ptr=z["row_ptr"][:S + 1], dst=z["col_idx"], pdf1=z["pdf0"] + 1,
                logw=z["weights"], final_state=np.arange(S, dtype=np.int32),
                final_w=np.zeros(S, np.float32), start=0)


def test_backward_test_fd_fixture():
    """internal/nnet/backward_test.go:28-140, restated exactly (make_golden.py).

    The oracle's numerator (kf_oracle_chain.c, chain_det.cu) must reproduce the
    restated computeChainLossCPU: its log-prob, its posteriors, and — through finite
    differences of the oracle's own log-prob with the reference's eps = 1e-4 float32
    perturbation — the numerical gradient at the reference's 50 positions, within the
    reference's tolerance (relative 1e-3, or absolute 1e-6).

    The reference's check compares that numerical gradient with num_post - den_post,
    where den_post is the uniform stand-in 1/numPdfs whose log-prob -T log numPdfs does
    not depend on the output. Its criterion therefore flags every checked position by
    exactly den_post (0.05): recorded here, not hidden."""
    z = np.load(os.path.join(GOLD, "backward_test_fd.npz"))
    x = z["nnet"]
    T, P = x.shape
    f = _bt_fst(z, x)
    lp, post = oracle.num_forward_backward(f, x)
    assert abs(lp - float(z["num_logprob"])) <= 1e-5
    assert abs((lp - float(z["den_logprob"])) - float(z["base_loss"])) <= 1e-5
    np.testing.assert_allclose(post, z["num_post"], atol=1e-6)
    np.testing.assert_allclose(post - z["den_post"], z["analytical"], atol=1e-6)
    xw = x.copy().ravel()
    e32 = np.float32(float(z["eps"]))
    for k, idx in enumerate(z["fd_idx"]):
        xw[idx] = np.float32(xw[idx] + e32)
        lpp, _ = oracle.num_forward_backward(f, xw.reshape(T, P), posteriors=False)
        xw[idx] = np.float32(xw[idx] - np.float32(2) * e32)
        lpm, _ = oracle.num_forward_backward(f, xw.reshape(T, P), posteriors=False)
        xw[idx] = np.float32(xw[idx] + e32)
        # float32 log-probs: the difference quotient is good to ~1e-3 at eps = 1e-4
        num = (lpp - lpm) / (2 * float(z["eps"]))
        ref = float(z["numerical"][k])
        assert abs(num - ref) <= max(1e-3 * abs(ref), 2e-3), (idx, num, ref)
        gnum = float(post.ravel()[idx])
        assert abs(gnum - ref) <= max(1e-3 * abs(ref), 1e-6), (idx, gnum, ref)
        # the reference's own criterion against num_post - den_post
        ana = float(z["analytical"].ravel()[idx])
        assert abs(abs(ref - ana) - 1.0 / P) <= 1e-3 * max(1.0, abs(ref))
    np.testing.assert_array_equal(xw.reshape(T, P), z["nnet_after"])


def test_den_small_fixture():
    z = np.load(os.path.join(GOLD, "den_small.npz"))
    g = dict(S=len(z["init"]), P=int(z["nnet"].shape[1]), A=len(z["src"]), src=z["src"],
             dst=z["dst"], pdf0=z["pdf0"], tp=z["tp"], start=0)
    np.testing.assert_allclose(oracle.den_initial_probs(g), z["init"], rtol=1e-6, atol=1e-12)
    for tag, leaky in (("l5", 1e-5), ("l1", 0.1)):
        lp, post = oracle.den_forward_backward(g, z["init"], z["nnet"], leaky)
        ref = float(z["logprob_" + tag])
        assert abs(lp - ref) <= 1e-5 * max(1.0, abs(ref))
        np.testing.assert_allclose(post, z["post_" + tag], atol=2e-6)
