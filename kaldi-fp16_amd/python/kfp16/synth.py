"""Synthetic model / egs generator pinned by SURVEY.md §8d and BASELINE.md §2.

The reference's real model, egs and den.fst live outside its repository, so the
benchmark and the parity tests run on this fixed synthetic setup:
  * weights: Xavier-normal sqrt(2/(fan_in+fan_out)) from default_rng(42) in
    parameter order (the reference's randTensor, forward.go:1161-1168), stored
    fp16 by truncation on upload (internal/gpu/tensor.go:158-173);
  * biases U(-0.05, 0.05) from default_rng(43) (the reference zero-initialises;
    non-zero biases exercise the bias path);
  * frozen BatchNorm: mean ~ N(0, 0.1^2), var ~ U(0.5, 2), gamma 1, beta 0,
    eps 1e-3 (identityBN's eps, forward.go:1185) from default_rng(44);
  * features x ~ N(0, 1) from default_rng(1234), fp16 round-to-nearest-even
    (internal/fp16/fp16.go:12-70, applied by TransferBatch).
Pure numpy; no device work.
"""
from __future__ import annotations

import os

import numpy as np

CONFIG_DIR = os.path.normpath(os.path.join(os.path.dirname(__file__), "..", "..", "..", "configs"))


def load_xconfig(name: str) -> str:
    with open(os.path.join(CONFIG_DIR, name)) as f:
        return f.read()


def make_params(param_shapes: dict, seed: int = 42, bias_seed: int = 43) -> dict:
    """param_shapes: name -> (rows, cols) in the network's parameter order."""
    rw = np.random.default_rng(seed)
    rb = np.random.default_rng(bias_seed)
    out = {}
    for name, (r, c, *_rest) in param_shapes.items():
        if name.endswith("Bias"):
            out[name] = rb.uniform(-0.05, 0.05, size=(r, c)).astype(np.float32)
        else:
            scale = np.sqrt(2.0 / (r + c))
            out[name] = (rw.standard_normal((r, c)) * scale).astype(np.float32)
    return out


def bn_layers(layers):
    """(layer name, which, dim) for every frozen BatchNorm of the network."""
    res = []
    for name, ty, din, dout in layers:
        if ty in (3,):  # batchnorm-component
            res.append((name, 0, dout))
    return res


def make_bn(dim: int, rng) -> tuple:
    mean = rng.normal(0.0, 0.1, size=dim).astype(np.float32)
    var = rng.uniform(0.5, 2.0, size=dim).astype(np.float32)
    return mean, var, np.ones(dim, np.float32), np.zeros(dim, np.float32)


def bn_specs(net_layers, conv_fout: dict, prefinal_dims: dict):
    """Every BatchNorm (layer, which, dim) in the order the generator draws them."""
    specs = []
    for name, ty, din, dout in net_layers:
        if ty == 3:            # batchnorm-component
            specs.append((name, 0, dout))
        elif ty == 6:          # conv-relu-batchnorm: per filter
            specs.append((name, 0, conv_fout[name]))
        elif ty in (7, 8):     # tdnnf, attention-relu-batchnorm
            specs.append((name, 0, dout))
        elif ty == 9:          # prefinal: big then small
            big, small = prefinal_dims[name]
            specs.append((name, 0, big))
            specs.append((name, 1, small))
    return specs


def make_bn_all(specs, seed: int = 44) -> dict:
    rng = np.random.default_rng(seed)
    return {(name, which): make_bn(dim, rng) for name, which, dim in specs}


def make_features(T: int, dim: int, seed: int = 1234) -> np.ndarray:
    rng = np.random.default_rng(seed)
    return rng.standard_normal((T, dim)).astype(np.float32).astype(np.float16)


def layer_dims(net):
    """Recover per-layer structural dims from the network's parameter shapes."""
    conv_fout, prefinal = {}, {}
    for name, ty, din, dout in net.layers:
        if ty == 6:
            conv_fout[name] = net.params[name + ".W"][1]
        if ty == 9:
            prefinal[name] = (net.params[name + ".BigW"][1], dout)
    return conv_fout, prefinal


def init_network(net, seed: int = 42):
    """Draw synthetic weights + BN statistics and load them into `net`.
    Returns (params dict fp32 pre-truncation, bn dict)."""
    params = make_params(net.params, seed=seed)
    net.set_params(params)
    conv_fout, prefinal = layer_dims(net)
    bns = make_bn_all(bn_specs(net.layers, conv_fout, prefinal))
    for (name, which), (m, v, g, b) in bns.items():
        net.set_bn(name, which, m, v, g, b, eps=1e-3)
    return params, bns


def trunc_fp16(a: np.ndarray) -> np.ndarray:
    """internal/gpu/tensor.go:158-173 truncating fp32->fp16, returned as fp32 values."""
    a = np.ascontiguousarray(a, dtype=np.float32)
    bits = a.view(np.uint32)
    sign = ((bits >> 16) & 0x8000).astype(np.uint16)
    exp = ((bits >> 23) & 0xFF).astype(np.int32) - 127
    frac = bits & 0x7FFFFF
    h = np.where(exp > 15, sign | 0x7C00,
                 np.where(exp < -14, sign,
                          sign | ((np.clip(exp, -14, 15) + 15).astype(np.uint16) << 10)
                          | (frac >> 13).astype(np.uint16))).astype(np.uint16)
    return h.view(np.float16).astype(np.float32)


# ---------------------------------------------------------------- chain supervision
# the reference's den.fst / cegs archives are not in its repository,
# so the objective runs on a fixed synthetic supervision of the same shape.

def make_den_graph(num_states: int = 7052, num_arcs: int = 113380, num_pdfs: int = 3080,
                   seed: int = 99) -> dict:
    """Denominator graph: a ring s -> s+1 plus uniformly random arcs, labels
    U[1, num_pdfs], tropical weights U[0.5, 5]; arcs listed state by state as an
    FST stores them. Returned in the NativeDenominator form (denominator.go:78-95):
    pdf0 = label - 1, tp = float32(exp(-weight)); start state 0."""
    rng = np.random.default_rng(seed)
    S, A = num_states, num_arcs
    nr = A - S
    src = np.concatenate([np.arange(S), rng.integers(0, S, size=nr)]).astype(np.int32)
    dst = np.concatenate([(np.arange(S) + 1) % S, rng.integers(0, S, size=nr)]).astype(np.int32)
    label = rng.integers(1, num_pdfs + 1, size=A).astype(np.int32)
    weight = rng.uniform(0.5, 5.0, size=A).astype(np.float32)
    order = np.argsort(src, kind="stable")
    src, dst, label, weight = src[order], dst[order], label[order], weight[order]
    tp = np.exp(-weight.astype(np.float64)).astype(np.float32)
    return dict(S=S, P=num_pdfs, A=A, src=src, dst=dst, pdf0=(label - 1).astype(np.int32),
                tp=tp, start=0)


def make_num_fst(eg: int, num_states: int = 250, num_pdfs: int = 3080) -> dict:
    """Numerator FST of eg `eg` (seed 7+eg): a self-loop and a forward arc per
    state (the last state has only its self-loop), tropical weight 0.6931 on every
    arc, labels U[1, num_pdfs], final state num_states-1 with weight 0. CSR with
    negated (log) weights, as sparse.FstToCSR does (sparse.go:54-91)."""
    rng = np.random.default_rng(7 + eg)
    S = num_states
    row_ptr, dst = [0], []
    for s in range(S):
        dst.append(s)
        if s + 1 < S:
            dst.append(s + 1)
        row_ptr.append(len(dst))
    A = len(dst)
    pdf1 = rng.integers(1, num_pdfs + 1, size=A).astype(np.int32)
    logw = np.full(A, -np.float32(0.6931), dtype=np.float32)
    return dict(S=S, A=A, row_ptr=np.array(row_ptr, np.int32), dst=np.array(dst, np.int32),
                pdf1=pdf1, logw=logw, final_state=np.array([S - 1], np.int32),
                final_w=np.zeros(1, np.float32), start=0)


def chain_layout(num_egs: int, frames_per_eg: int = 1500, left_context: int = 30,
                 subsample: int = 3):
    """Rows of the concatenated output that carry supervision: eg i frame k sits
    at row i*frames_per_eg + left_context + k*subsample (chain_loss.go:243-259);
    (frames_per_eg - left_context) // subsample = 490 frames per eg."""
    fps = (frames_per_eg - left_context) // subsample
    row0 = (np.arange(num_egs) * frames_per_eg + left_context).astype(np.int32)
    return row0, np.full(num_egs, fps, np.int32), subsample
