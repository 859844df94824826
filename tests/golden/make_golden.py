#!/usr/bin/env python3
"""Generates the committed golden fixtures under tests/golden/ (run from the repo root:
python tests/golden/make_golden.py). Each fixture is data only — inputs and the
expected outputs — and names where its expected values come from.

  backward_test_fd.npz  internal/nnet/backward_test.go:28-140 restated exactly: the linear
                        numerator FST (T=10, 20 pdfs, 0-based pdfIds = i % numPdfs,
                        weight 0, every state final) on nnet[i] = float32(0.5*sin(0.1*i)),
                        computeChainLossCPU (:152-257, float64, log-domain numerator
                        plus the uniform-denominator stand-in) and the finite-difference
                        loop (:84-131: eps 1e-4 applied in float32, 50 positions with
                        step T*numPdfs/50, the +eps / -2eps / +eps sequence kept in
                        place). Expected values are that restatement's outputs.
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


def _log_add(a, b):
    """backward_test.go:261-272"""
    if a == -np.inf:
        return b
    if b == -np.inf:
        return a
    if a > b:
        return a + np.log1p(np.exp(b - a))
    return b + np.log1p(np.exp(a - b))


def compute_chain_loss_cpu(x, row_ptr, col_idx, weights, pdf_ids, T, P, S, want_post):
    """backward_test.go:152-257, float64, same loop order."""
    alpha = np.full((T + 1) * S, -np.inf)
    beta = np.full((T + 1) * S, -np.inf)
    alpha[0] = 0.0
    for t in range(T):
        for s in range(S):
            if alpha[t * S + s] == -np.inf:
                continue
            for a in range(row_ptr[s], row_ptr[s + 1]):
                d, p = int(col_idx[a]), int(pdf_ids[a])
                lp = float(x[t * P + p]) + float(weights[a])
                alpha[(t + 1) * S + d] = _log_add(alpha[(t + 1) * S + d], alpha[t * S + s] + lp)
    num_total = -np.inf
    for s in range(S):
        num_total = _log_add(num_total, alpha[T * S + s])
    beta[T * S:(T + 1) * S] = 0.0
    for t in range(T - 1, -1, -1):
        for s in range(S):
            for a in range(row_ptr[s], row_ptr[s + 1]):
                d, p = int(col_idx[a]), int(pdf_ids[a])
                lp = float(x[t * P + p]) + float(weights[a])
                beta[t * S + s] = _log_add(beta[t * S + s], beta[(t + 1) * S + d] + lp)
    num_post = den_post = None
    if want_post:
        num_post = np.zeros(T * P, np.float32)
        for t in range(T):
            for s in range(S):
                if alpha[t * S + s] == -np.inf:
                    continue
                for a in range(row_ptr[s], row_ptr[s + 1]):
                    d, p = int(col_idx[a]), int(pdf_ids[a])
                    lp = float(x[t * P + p]) + float(weights[a])
                    lpost = alpha[t * S + s] + lp + beta[(t + 1) * S + d] - num_total
                    num_post[t * P + p] += np.float32(np.exp(lpost))
        den_post = np.full(T * P, np.float32(1.0 / P), np.float32)
    den_total = -float(T) * np.log(float(P))
    return num_total - den_total, num_post, den_post, num_total, den_total


def backward_test_fd():
    T, P, eps, n_samples = 10, 20, 1e-4, 50
    S = T + 1
    row_ptr = np.zeros(S + 1, np.int32)
    col_idx = np.zeros(T, np.int32)
    weights = np.zeros(T, np.float32)
    pdf_ids = np.zeros(T, np.int32)
    for i in range(T):
        row_ptr[i], col_idx[i], pdf_ids[i] = i, i + 1, i % P
    row_ptr[T] = T
    row_ptr[T + 1] = T  # Go's zero value of the last entry (rowPtr has numStates+1 slots)
    x = (np.sin(np.arange(T * P, dtype=np.float64) * 0.1) * 0.5).astype(np.float32)
    x0 = x.copy()
    base, num_post, den_post, num_total, den_total = compute_chain_loss_cpu(
        x, row_ptr, col_idx, weights, pdf_ids, T, P, S, True)
    ana = (np.float32(1.0) * (num_post - den_post)).astype(np.float32)
    step = max(1, T * P // n_samples)
    idxs, plus, minus, num_grad = [], [], [], []
    e32 = np.float32(eps)
    idx = 0
    while idx < T * P and len(idxs) < n_samples:
        x[idx] = np.float32(x[idx] + e32)
        lp = compute_chain_loss_cpu(x, row_ptr, col_idx, weights, pdf_ids, T, P, S, False)[0]
        x[idx] = np.float32(x[idx] - np.float32(2) * e32)
        lm = compute_chain_loss_cpu(x, row_ptr, col_idx, weights, pdf_ids, T, P, S, False)[0]
        x[idx] = np.float32(x[idx] + e32)
        idxs.append(idx)
        plus.append(lp)
        minus.append(lm)
        num_grad.append((lp - lm) / (2 * eps))
        idx += step
    np.savez_compressed(os.path.join(OUT, "backward_test_fd.npz"), nnet=x0.reshape(T, P),
                        nnet_after=x.reshape(T, P), row_ptr=row_ptr, col_idx=col_idx,
                        weights=weights, pdf0=pdf_ids, base_loss=np.float64(base),
                        num_logprob=np.float64(num_total), den_logprob=np.float64(den_total),
                        num_post=num_post.reshape(T, P), den_post=den_post.reshape(T, P),
                        analytical=ana.reshape(T, P), fd_idx=np.array(idxs, np.int32),
                        loss_plus=np.array(plus), loss_minus=np.array(minus),
                        numerical=np.array(num_grad), eps=np.float64(eps))


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
    backward_test_fd()
    den_small()
    print("wrote", sorted(f for f in os.listdir(OUT) if f.endswith(".npz")))
