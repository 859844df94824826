"""The oracle against the committed fixtures of tests/golden/ (see make_golden.py
for their provenance)."""
import os

import numpy as np

import oracle

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_chain_linear_fst_fixture():
    """internal/nnet/backward_test.go:28-140's fixture with its analytic answers."""
    z = np.load(os.path.join(GOLD, "chain_linear_fst.npz"))
    x = z["nnet"]
    T, P = x.shape
    S = T + 1
    f = dict(S=S, A=T, row_ptr=np.array(list(range(T)) + [T, T], np.int32)[: S + 1],
             dst=np.arange(1, T + 1, dtype=np.int32), pdf1=z["pdf1"], logw=np.zeros(T, np.float32),
             final_state=np.arange(S, dtype=np.int32), final_w=np.zeros(S, np.float32), start=0)
    lp, post = oracle.num_forward_backward(f, x)
    assert abs(lp - float(z["num_logprob"])) < 1e-5
    np.testing.assert_allclose(post, z["num_post"], atol=1e-6)


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
