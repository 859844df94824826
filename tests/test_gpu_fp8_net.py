"""MXFP8 forward (BASELINE configs[4], nnet_set_fp8).

Parity: against the oracle's MXFP8 emulation (same quantisation points and OCP MX
rule, oracle/kf_oracle.c mx8), rel-Frobenius <= 5e-3 up to and including the first
layer whose GEMMs run in fp8 — the fp16 path's bar plus the rare e4m3 rounding
flips that accumulation-order noise causes. Past that layer the two quantised
computations diverge chaotically (an fp16-ulp input difference crosses an e4m3
rounding boundary with probability ~2^-7 and then moves the element by 2^-4), so
deeper layers are held to the precision bound and must stay closer to the MX
emulation than to the fp16 oracle. Precision: against the fp16 oracle the activations drift by the e4m3
rounding of both GEMM operands, ~4.3% per GEMM (measured by tests/mx_ref.py on
Gaussian data); the per-layer bound is 0.15 and the SURVEY §8d objective bound
|d objf/frame| <= 1e-2 applies to the chain objective. SURVEY §8d proposed 5e-2 for
the activations; with two chained e4m3 GEMMs per TDNN-F layer that bound sits
below the format's floor.

Per-layer parity without the chaos (test_*_fp8_layers_isolated): every fp8-GEMM layer
alone in the MX emulation on the GPU's own inputs (fp16 activation and the MXFP8 copy
its GEMM read) is held to the fp16 bar, 5e-3."""
import numpy as np
import pytest

import oracle
from conftest import rel_fro

pytestmark = pytest.mark.gpu

MX_PARITY_TOL = 5e-3   # vs the oracle's MXFP8 emulation
FP8_ACT_TOL = 0.15     # vs the fp16 oracle (precision, not parity)
FP8_OBJF_TOL = 1e-2


def _net(kfp16, xcfg, T):
    from kfp16 import synth
    net = kfp16.Network(xcfg, max_frames=T)
    params, bns = synth.init_network(net, seed=42)
    feats = synth.make_features(T, 40)
    return net, params, bns, feats, kfp16.upload_fp16(feats)


def _oracle(xcfg, params, bns, feats, mx8=False):
    from kfp16 import synth
    tp = {k: synth.trunc_fp16(v) for k, v in params.items()}
    on = oracle.OracleNet(xcfg, tp, bns, round_mode=oracle.ROUND_FUSED, threads=16, mx8=mx8)
    on.forward(feats.astype(np.float32))
    return on


FP8_TYPES = (7, 2, 9, 10)  # TDNNF, Linear, Prefinal, Output (kf_nnet.h layer codes)


def _check_mx(net, errs, perr, first_tol=MX_PARITY_TOL):
    msg = "; ".join(f"{k} {perr[k]:.3g}/{errs[k]:.3g}" for k in errs)
    first = next(i for i, L in enumerate(net.layers) if L[1] in FP8_TYPES)
    for i, (name, ty, din, dout) in enumerate(net.layers):
        assert errs[name] <= FP8_ACT_TOL, msg
        if i <= first:
            assert perr[name] <= first_tol, msg
        elif ty in FP8_TYPES:
            assert perr[name] < errs[name], msg


def test_tiny_fp8_forward(gpu):
    kfp16 = gpu
    from kfp16 import synth
    xcfg = synth.load_xconfig("tiny.xconfig")
    T = 300
    net, params, bns, feats, fbuf = _net(kfp16, xcfg, T)
    on = _oracle(xcfg, params, bns, feats)
    om = _oracle(xcfg, params, bns, feats, mx8=True)
    net.set_fp8(True)
    net.forward(fbuf.ptr, T)
    errs, perr = {}, {}
    for name, ty, din, dout in net.layers:
        got = net.read_activation(name).astype(np.float32)
        errs[name] = rel_fro(got, on.act(name))
        perr[name] = rel_fro(got, om.act(name))
    _check_mx(net, errs, perr)
    om.close()
    # the GEMM layers really ran at fp8 precision (not silently fp16)
    assert errs["output"] > 2e-3, errs
    # switching back restores the fp16 path (oracle tolerance 2e-3)
    net.set_fp8(False)
    net.forward(fbuf.ptr, T)
    assert rel_fro(net.read_activation("output").astype(np.float32), on.act("output")) <= 2e-3
    on.close()
    net.close()


@pytest.mark.slow
def test_config5_fp8_forward_and_objective(gpu):
    """cnn_tdnn_17f_3072 (configs[4] model) on one 1500-frame eg; objective on the
    synthetic den graph and eg 0's numerator FST, computed by the oracle from the
    fp8 GPU output and from the oracle's own output."""
    kfp16 = gpu
    from kfp16 import synth
    xcfg = synth.load_xconfig("cnn_tdnn_17f_3072.xconfig")
    T = 1500
    net, params, bns, feats, fbuf = _net(kfp16, xcfg, T)
    on = _oracle(xcfg, params, bns, feats)
    net.set_fp8(True)
    net.forward(fbuf.ptr, T)
    errs = {name: rel_fro(net.read_activation(name).astype(np.float32), on.act(name))
            for name, ty, din, dout in net.layers}
    assert all(e <= FP8_ACT_TOL for e in errs.values()), "; ".join(f"{k} {v:.3g}" for k, v in errs.items())
    om = _oracle(xcfg, params, bns, feats, mx8=True)
    perr = {name: rel_fro(net.read_activation(name).astype(np.float32), om.act(name))
            for name, ty, din, dout in net.layers}
    om.close()
    # cnn6 (the first fp8 layer's input) already differs from the oracle by ~3.5e-4
    # (fp32 accumulation order over K = 2304); that input noise flips ~4x more e4m3
    # roundings than in the tiny model, hence the first-layer bound of 2e-2 here
    _check_mx(net, errs, perr, first_tol=2e-2)
    P = net.layers[-1][3]
    g = synth.make_den_graph(num_pdfs=P)
    init = oracle.den_initial_probs(g)
    f = synth.make_num_fst(0, num_pdfs=P)
    row0, nfr, stride = synth.chain_layout(1, T)
    rows = row0[0] + np.arange(nfr[0]) * stride
    _, r8 = oracle.chain_objf(g, init, f, net.read_activation("output").astype(np.float32)[rows])
    _, r16 = oracle.chain_objf(g, init, f, on.act("output")[rows])
    d = abs(r8["objf"] - r16["objf"]) / nfr[0]
    assert r8["ok"] == 1 and d <= FP8_OBJF_TOL, (r8["objf"] / nfr[0], r16["objf"] / nfr[0])
    on.close()
    net.close()


def _e4m3_values():
    """OCP e4m3 (bias 7, no infinities, S.1111.111 = NaN) as float64 per byte"""
    v = np.arange(256)
    sign, e, m = (v >> 7) & 1, (v >> 3) & 15, v & 7
    val = np.where(e == 0, m / 8.0 * 2.0 ** -6, (1 + m / 8.0) * 2.0 ** (e - 7.0))
    val = np.where((e == 15) & (m == 7), np.nan, val)
    return np.where(sign == 1, -val, val)


def _read_mx_input(kfp16, net, li, T, din):
    """the dequantised MXFP8 copy layer li's GEMM read (nnet_debug_tensor x8q / x8s)"""
    import ctypes as C
    q = kfp16.nnet.nnet_debug_tensor(net.h, b"x8q", li)
    sc = kfp16.nnet.nnet_debug_tensor(net.h, b"x8s", li)
    if not q:
        return None
    ld = (din + 127) // 128 * 128
    qb = np.frombuffer(kfp16.read_fp16(q, (T * ld // 2,)).tobytes(), np.uint8).reshape(T, ld)
    sb = np.frombuffer(kfp16.read_fp16(sc, ((T * ld // 32 + 1) // 2,)).tobytes(), np.uint8)[: T * ld // 32]
    scale = np.ldexp(1.0, sb.astype(np.int64) - 127).reshape(T, ld // 32)
    x = _e4m3_values()[qb] * np.repeat(scale, 32, axis=1)
    assert np.isfinite(x).all()
    return x[:, :din].astype(np.float32)


def _layer_line(xcfg, name):
    """the layer's xconfig line without its input= (the one-layer net reads `input`)"""
    import re
    for line in xcfg.splitlines():
        if re.search(rf"\bname={re.escape(name)}(\s|$)", line):
            return re.sub(r"\binput=\S+\s*", "", line).strip()
    raise KeyError(name)


def _isolated_fp8_errors(kfp16, xcfg, T):
    """MXFP8 forward on the GPU; then every fp8-GEMM layer alone in the oracle's MX
    emulation on the GPU's own inputs (its fp16 input activation and the MXFP8 copy the
    GPU GEMM read), so that no upstream e4m3 flip reaches the comparison"""
    net, params, bns, feats, fbuf = _net(kfp16, xcfg, T)
    net.set_fp8(True)
    net.forward(fbuf.ptr, T)
    index = {L[0]: i for i, L in enumerate(net.layers)}
    inputs = {}
    for L in oracle.parse_xconfig(xcfg):
        inputs[L["name"]] = L["input"]
    from kfp16 import synth
    tp = {k: synth.trunc_fp16(v) for k, v in params.items()}
    errs = {}
    for li, (name, ty, din, dout) in enumerate(net.layers):
        if ty not in FP8_TYPES:
            continue
        src = inputs[name]
        x = net.read_activation(src).astype(np.float32) if src in index else feats.astype(np.float32)
        x8 = _read_mx_input(kfp16, net, li, T, din)
        one = f"input name=input dim={din}\n{_layer_line(xcfg, name)}\n"
        on = oracle.OracleNet(one, tp, bns, round_mode=oracle.ROUND_FUSED, threads=16, mx8=True)
        on.forward(x, features8=x8)
        errs[name] = (rel_fro(net.read_activation(name).astype(np.float32), on.act(name)), x8 is not None)
        on.close()
    net.close()
    return errs


MX_LAYER_TOL = 5e-3   # one layer on identical fp8 inputs: the fp16 bar


def _check_isolated(errs):
    msg = "; ".join(f"{k} {e:.3g}{'' if f8 else ' (fp16 input)'}" for k, (e, f8) in errs.items())
    print("isolated MXFP8 layer errors vs the MX emulation:", msg)
    assert sum(f8 for e, f8 in errs.values()) >= 2, msg
    assert all(e <= MX_LAYER_TOL for e, f8 in errs.values()), msg


def test_tiny_fp8_layers_isolated(gpu):
    from kfp16 import synth
    _check_isolated(_isolated_fp8_errors(gpu, synth.load_xconfig("tiny.xconfig"), 300))


@pytest.mark.slow
def test_config5_fp8_layers_isolated(gpu):
    """every fp8 layer of the configs[4] model (cnn_tdnn_17f_3072) on one 1500-frame eg"""
    from kfp16 import synth
    _check_isolated(_isolated_fp8_errors(gpu, synth.load_xconfig("cnn_tdnn_17f_3072.xconfig"), 1500))


# weight gradients vs the oracle's MXFP8 emulation (chaotic e4m3 flips, as above); measured
# at most 6.3 % (tiny) and 7.2 % (3072 model) with the MXFP8 affine input gradients on (r4)
FP8_GRAD_TOL = 0.10


def _fp8_backward_errors(kfp16, xcfg, T, seed=7, mode=1):
    """MXFP8 train step on the GPU (nnet_set_fp8 `mode`: 1 = MXFP8 forward and strided
    TDNN-F affine input gradients, 2 = MXFP8 forward, all-fp16 backward) back-propagating a
    fixed output gradient; the oracle replays the GPU's ReLU decisions in its fp16 and its
    MX-emulating step (the same mode) and back-propagates the same gradient. Returns
    ({param: err vs MX emulation}, {param: err vs fp16}, the params of layers up to the
    first fp8 layer that no e4m3 backward product reaches)."""
    from kfp16 import synth
    net, params, bns, feats, fbuf = _net(kfp16, xcfg, T)
    net.set_fp8(mode)
    net.forward(fbuf.ptr, T)
    masks = net.relu_masks()
    P = net.layers[-1][3]
    og = (np.random.default_rng(seed).standard_normal((T, P)) * 0.05).astype(np.float16)
    gbuf = kfp16.upload_fp16(og)
    net.backward(gbuf.ptr)
    got = net.read_grads()
    first = next(i for i, L in enumerate(net.layers) if L[1] in FP8_TYPES)
    # layers up to the first fp8 layer see no e4m3 flip in the forward, and none in the
    # backward unless an MXFP8 affine input gradient (strided TDNN-F) sits above them: then
    # the chaotic divergence starts there and they get the deep layers' bars
    mx_dgrad = [i for i, L in enumerate(net.layers)
                if mode == 1 and kfp16.nnet.nnet_debug_tensor(net.h, b"w8dq", i)]
    early = {L[0] for i, L in enumerate(net.layers[:first + 1]) if not any(j > i for j in mx_dgrad)}
    net.close()
    tp = {k: synth.trunc_fp16(v) for k, v in params.items()}
    refs = []
    for mx8 in (mode, 0):
        on = oracle.OracleNet(xcfg, tp, bns, round_mode=oracle.ROUND_FUSED, threads=16, mx8=mx8)
        on.forward(feats.astype(np.float32), force_masks=masks)
        on.backward(og.astype(np.float32))
        refs.append(on.grads())
        on.close()
    emx = {k: rel_fro(got[k], refs[0][k]) for k in refs[0]}
    e16 = {k: rel_fro(got[k], refs[1][k]) for k in refs[1]}
    early_params = {k for k in emx if k.split(".")[0] in early}
    return emx, e16, early_params


def _check_fp8_grads(emx, e16, early_params, early_tol):
    """every gradient within FP8_GRAD_TOL of the MX emulation; those of layers no e4m3 flip
    reaches within early_tol; the rest no further from the emulation than from fp16"""
    msg = "; ".join(f"{k} {emx[k]:.3g}/{e16[k]:.3g}" for k in emx)
    print("\nfp8 backward weight-gradient rel-Frobenius errors (bar: %.2f; early layers %.3g)" %
          (FP8_GRAD_TOL, early_tol))
    print("%-28s %12s %12s %s" % ("parameter", "vs MX emul", "vs fp16", "early"))
    for k in emx:
        print("%-28s %12.4g %12.4g %s" % (k, emx[k], e16[k], "yes" if k in early_params else ""))
    for k in emx:
        assert emx[k] <= FP8_GRAD_TOL, msg
        if k in early_params:
            assert emx[k] <= early_tol, msg
        else:  # the backward differentiates the fp8 forward it ran after
            assert emx[k] <= max(e16[k], 5e-3), msg
    # the gradients really carry the fp8 forward (not a silently fp16 one)
    assert max(e16.values()) > 1e-2, msg


def test_tiny_fp8_backward(gpu):
    """configs[4]'s train step (MXFP8 forward, MXFP8 strided TDNN-F affine input
    gradients, the rest of the backward fp16): its weight gradients follow the oracle's
    MX emulation (replayed ReLU decisions)"""
    from kfp16 import synth
    emx, e16, early = _fp8_backward_errors(gpu, synth.load_xconfig("tiny.xconfig"), 300)
    _check_fp8_grads(emx, e16, early, early_tol=2e-2)


def test_tiny_fp8_backward_fp16_dgrad(gpu):
    """the MXFP8 forward with an all-fp16 backward (nnet_set_fp8 mode 2): no e4m3 rounding
    reaches the layers up to the first fp8 layer, which then hold the fp16 weight-gradient
    bar, 5e-3 (the conv and first TDNN-F gradients, measured <= 1.5e-3; with the MXFP8 input
    gradients on they sit below one and get only the deep layers' bars)"""
    from kfp16 import synth
    emx, e16, early = _fp8_backward_errors(gpu, synth.load_xconfig("tiny.xconfig"), 300, mode=2)
    assert early, "no early layers"
    _check_fp8_grads(emx, e16, early, early_tol=5e-3)


@pytest.mark.slow
def test_config5_fp8_backward(gpu):
    """the same on the configs[4] model (cnn_tdnn_17f_3072), 150 frames"""
    from kfp16 import synth
    emx, e16, early = _fp8_backward_errors(gpu, synth.load_xconfig("cnn_tdnn_17f_3072.xconfig"), 150)
    _check_fp8_grads(emx, e16, early, early_tol=2e-2)


@pytest.mark.slow
def test_config5_fp8_backward_fp16_dgrad(gpu):
    """mode 2 on the configs[4] model: the early layers (convs, tdnnf7) within 5e-3
    (measured <= 3e-3)"""
    from kfp16 import synth
    emx, e16, early = _fp8_backward_errors(gpu, synth.load_xconfig("cnn_tdnn_17f_3072.xconfig"), 150, mode=2)
    assert early, "no early layers"
    _check_fp8_grads(emx, e16, early, early_tol=5e-3)


def _mx_rows(kfp16, q, sc, rows, ld):
    """dequantised [rows x ld] MXFP8 buffer (e4m3 bytes q, E8M0 scales sc [rows x ld/32])"""
    qb = np.frombuffer(kfp16.read_fp16(q, (rows * ld // 2,)).tobytes(), np.uint8).reshape(rows, ld)
    n = rows * ld // 32
    sb = np.frombuffer(kfp16.read_fp16(sc, ((n + 1) // 2,)).tobytes(), np.uint8)[:n].reshape(rows, ld // 32)
    return qb, sb, _e4m3_values()[qb] * np.repeat(np.ldexp(1.0, sb.astype(np.int64) - 127), 32, axis=1)


def _isolated_dgrad_errors(kfp16, xcfg, T, seed=3):
    """The MXFP8 affine input gradient of every strided TDNN-F layer, on the GPU's own
    operands: the backward is stopped right after the layer (nnet_backward_n), and its
    bottleneck gradient is held to the GEMM element bound of the float64 product of the
    e4m3 copies it read (dz's, written by the layer above's epilogue, and W2's rows), with
    row T-1 in fp16 through the clamped-edge sum. The copies themselves: W2's bit-exact
    against tests/mx_ref.py, dz's against the quantisation of the stored fp16 dz (the
    epilogue quantises the unrounded value, so a code may differ where the fp16 rounding
    crosses an e4m3 boundary)."""
    import re
    from mx_ref import mx_quantize
    from kfp16 import synth
    net, params, bns, feats, fbuf = _net(kfp16, xcfg, T)
    net.set_fp8(True)
    net.forward(fbuf.ptr, T)
    P = net.layers[-1][3]
    og = kfp16.upload_fp16((np.random.default_rng(seed).standard_normal((T, P)) * 0.05).astype(np.float16))
    lines = {m.group(1): l for l in xcfg.splitlines() if (m := re.search(r"\bname=(\S+)", l))}
    order, li = [], len(net.layers) - 1   # the backward's layer order (chain output down)
    inputs = {L["name"]: L["input"] for L in oracle.parse_xconfig(xcfg)}
    index = {L[0]: i for i, L in enumerate(net.layers)}
    while li >= 0:
        order.append(li)
        src = inputs[net.layers[li][0]]
        li = index.get(src, -1)
    out = {}
    for n, li in enumerate(order, 1):
        name, ty, din, dout = net.layers[li]
        if not kfp16.nnet.nnet_debug_tensor(net.h, b"w8dq", li):
            continue
        s = int(re.search(r"time-stride=(\d+)", lines[name]).group(1))
        bn = int(re.search(r"bottleneck-dim=(\d+)", lines[name]).group(1))
        kfp16.check(kfp16.nnet.nnet_backward_n(net.h, og.ptr, n), "backward_n")
        kfp16.sync()
        buf = [i for i in (0, 1, 2) if (kfp16.nnet.nnet_debug_tensor(net.h, b"dz8layer", i) or 0) == li + 1]
        assert len(buf) == 1, (name, "no e4m3 dz copy was written for this layer")
        i = buf[0]
        pw = (dout + 127) // 128 * 128
        dz = kfp16.read_fp16(kfp16.nnet.nnet_debug_tensor(net.h, f"dz{i}".encode(), 0), (T + 1, dout))
        dzq, dzs, dz8 = _mx_rows(kfp16, kfp16.nnet.nnet_debug_tensor(net.h, b"dz8q", i),
                                 kfp16.nnet.nnet_debug_tensor(net.h, b"dz8s", i), T, pw)
        wq, ws, w8 = _mx_rows(kfp16, kfp16.nnet.nnet_debug_tensor(net.h, b"w8dq", li),
                              kfp16.nnet.nnet_debug_tensor(net.h, b"w8ds", li), bn, 2 * pw)
        W2 = synth.trunc_fp16(params[name + ".AffineW"]).astype(np.float32)   # [2 bn x dout]
        for p in (0, 1):   # the weight copy: bit-exact
            rq, rs = mx_quantize(np.pad(W2[p * bn:(p + 1) * bn], ((0, 0), (0, pw - dout))))
            np.testing.assert_array_equal(wq[:, p * pw:(p + 1) * pw], rq)
            np.testing.assert_array_equal(ws[:, p * pw // 32:(p + 1) * pw // 32], rs)
        rq, rs = mx_quantize(np.pad(dz[:T].astype(np.float32), ((0, 0), (0, pw - dout))))
        code_agree = float((dzq == rq).mean())
        dbott = kfp16.read_fp16(kfp16.nnet.nnet_debug_tensor(net.h, b"dbott", 0), (T, bn)).astype(np.float64)
        a0 = a1 = dz8[:, :dout]   # both parts read dz's copy: rows t and t - s
        b0, b1 = w8[:, :dout], w8[:, pw:pw + dout]
        ref = a0 @ b0.T
        mag = np.abs(a0) @ np.abs(b0).T
        ref[s:] += a1[:T - s] @ b1.T
        mag[s:] += np.abs(a1[:T - s]) @ np.abs(b1).T
        # row T-1: fp16 operands, the second part being the rounded clamped-edge sum
        edge = dz[max(T - 1 - s, 0):T].astype(np.float32).sum(0).astype(np.float16).astype(np.float64)
        W2d = W2.astype(np.float64)
        ref[T - 1] = dz[T - 1].astype(np.float64) @ W2d[:bn].T + edge @ W2d[bn:].T
        mag[T - 1] = np.abs(dz[T - 1].astype(np.float64)) @ np.abs(W2d[:bn]).T + np.abs(edge) @ np.abs(W2d[bn:]).T
        ulp = np.spacing(np.abs(ref).astype(np.float16)).astype(np.float64)
        bound = 2 * ulp + 2 * dout * 2.0 ** -23 * mag + 1e-7
        excess = float(np.max(np.abs(dbott - ref) - bound))
        out[name] = (excess, code_agree, rel_fro(dbott, ref))
    net.close()
    return out


def _check_dgrad_isolated(res):
    msg = "; ".join(f"{k} excess {e:.3g} dz-codes {c:.5f} rel {r:.3g}" for k, (e, c, r) in res.items())
    print("isolated MXFP8 affine input gradients:", msg)
    assert len(res) >= 2, msg
    for e, c, r in res.values():
        assert e <= 0, msg          # every element within the GEMM bound of its own operands
        assert c >= 0.99, msg       # dz's copy is dz's quantisation up to boundary flips


def test_tiny_fp8_dgrad_isolated(gpu):
    from kfp16 import synth
    _check_dgrad_isolated(_isolated_dgrad_errors(gpu, synth.load_xconfig("tiny.xconfig"), 300))


@pytest.mark.slow
def test_config5_fp8_dgrad_isolated(gpu):
    from kfp16 import synth
    _check_dgrad_isolated(_isolated_dgrad_errors(gpu, synth.load_xconfig("cnn_tdnn_17f_3072.xconfig"), 300))
