#!/usr/bin/env python3
"""Generates the committed golden fixtures under tests/golden/ (run from the repo root:
python tests/golden/make_golden.py). Each fixture is data only — inputs and the
expected outputs — and names where its expected values come from.

  chain_linear_fst.npz  internal/nnet/backward_test.go:28-140's own fixture: a linear
                        numerator FST (T=10, 20 pdfs, weight 0, every state final) on
                        nnet[i] = 0.5*sin(0.1*i). Expected values are analytic: the
                        single path's log-prob is the sum of its outputs and its
                        posteriors are one-hot.
  den_small.npz         a 24-state / 90-arc leaky-HMM denominator graph; expected
                        log-probs and posteriors from a float64 dense-matrix
                        restatement of chain_den.cu:496-706 (independent of the C oracle;
                        the reference's CUDA den cannot run in this container).
"""
import os
import sys

import numpy as np

ROOT = os.path.normpath(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle"),
                os.path.join(ROOT, "kaldi-fp16_amd", "python")]
OUT = os.path.dirname(os.path.abspath(__file__))


def chain_linear():
    T, P = 10, 20
    x = (np.sin(np.arange(T * P) * 0.1) * 0.5).astype(np.float32).reshape(T, P)
    path = x[np.arange(T), np.arange(T) % P].astype(np.float64)
    post = np.zeros((T, P), np.float32)
    post[np.arange(T), np.arange(T) % P] = 1.0
    np.savez_compressed(os.path.join(OUT, "chain_linear_fst.npz"), nnet=x,
                        pdf1=(np.arange(T) % P + 1).astype(np.int32), num_logprob=path.sum(),
                        num_post=post)


def den_small():
    from test_oracle_chain import dense_den_f64, small_den
    g = small_den()
    # initial probs by the float64 100-iteration rule (denominator.go:131-171)
    cur = np.zeros(g["S"])
    cur[0] = 1.0
    avg = np.zeros(g["S"])
    for _ in range(100):
        avg += cur / 100.0
        nxt = np.zeros(g["S"])
        np.add.at(nxt, g["dst"], cur[g["src"]] * g["tp"].astype(np.float64))
        cur = nxt / nxt.sum()
    init = avg.astype(np.float32)
    x = np.random.default_rng(1).standard_normal((9, g["P"])).astype(np.float32) * 2
    x[3, 2] = 40.0
    out = dict(src=g["src"], dst=g["dst"], pdf0=g["pdf0"], tp=g["tp"], init=init, nnet=x)
    for tag, leaky in (("l5", 1e-5), ("l1", 0.1)):
        lp, post = dense_den_f64(g, init, x, leaky)
        out["logprob_" + tag] = np.float64(lp)
        out["post_" + tag] = post
    np.savez_compressed(os.path.join(OUT, "den_small.npz"), **out)


if __name__ == "__main__":
    chain_linear()
    den_small()
    print("wrote", sorted(f for f in os.listdir(OUT) if f.endswith(".npz")))
