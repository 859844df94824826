"""T1: the composed TrainStep (internal/nnet/train_step.go:142-283) on the GPU against the
oracle's composition of the same four stages on CPU:

  forward (forward.go:148-202) -> chain objective and derivative on the supervised rows
  (backward.go:224-371, one numerator FST per eg, leaky-HMM den) -> backward
  (network_backward.go:94-700) -> SGD with momentum (optimize.go:95-142).

Two egs of 150 frames through tiny.xconfig (every layer kind of the benchmark model).
The oracle replays the GPU's ReLU decisions (as in test_gpu_nnet.py) and takes its
objective derivative from its own forward output. Tolerances: objective
per frame |d| <= 1e-3; weight gradients and the SGD update (w_new - w_old) rel-Frobenius
<= 5e-3 per tensor.
"""
import numpy as np
import pytest

import oracle
from conftest import rel_fro

pytestmark = pytest.mark.gpu

NEGS, FPE, P = 2, 150, 200


def test_train_step_matches_oracle_composition(gpu):
    kf = gpu
    from kfp16 import chain, synth
    xcfg = synth.load_xconfig("tiny.xconfig")
    T = NEGS * FPE
    net = kf.Network(xcfg, max_frames=T)
    params, bns = synth.init_network(net, seed=11)
    feats = synth.make_features(T, 40, seed=5)
    fbuf = kf.upload_fp16(feats)
    den = synth.make_den_graph(num_states=300, num_arcs=3000, num_pdfs=P)
    init = oracle.den_initial_probs(den)
    fsts = [synth.make_num_fst(i, num_states=20, num_pdfs=P) for i in range(NEGS)]
    row0, frames, stride = synth.chain_layout(NEGS, FPE)

    # ---- GPU step
    w0 = net.get_params()
    net.forward(fbuf.ptr, T)
    masks = net.relu_masks()
    obj = chain.Chain(chain.DenGraph(den), max_seqs=4, max_frames=int(frames.max()))
    g = kf.DeviceBuffer(T * P * 2)
    kf.core.bridge_gpu_memset(g.ptr, 0, T * P * 2)
    obj.compute(chain.NumBatch(fsts), net.activation("output")[0], P, T, row0, frames, stride, g.ptr, P)
    res = obj.result()
    assert res.num_ok == NEGS
    net.backward(g.ptr)
    grads = net.read_grads()
    lr, mom = 1e-4, 0.9
    net.sgd(lr, mom)
    w1 = net.get_params()

    # ---- oracle composition
    tp = {k: synth.trunc_fp16(v) for k, v in params.items()}
    on = oracle.OracleNet(xcfg, tp, bns, round_mode=oracle.ROUND_FUSED, threads=16)
    on.forward(feats.astype(np.float32), force_masks=masks)
    out = on.act("output")
    og = np.zeros_like(out)
    objf = 0.0
    for i in range(NEGS):
        rows = row0[i] + np.arange(frames[i]) * stride
        deriv, r = oracle.chain_objf(den, init, fsts[i], out[rows])
        og[rows] = -deriv
        objf += r["objf"]
    assert abs(res.objf - objf) / res.frames <= 1e-3, (res.objf, objf)
    on.backward(og)
    ref = on.grads()
    errs = {k: rel_fro(grads[k], ref[k]) for k in ref}
    bad = {k: v for k, v in errs.items() if v > 5e-3}
    assert not bad, "grad errors: " + ", ".join(f"{k}={v:.2e}" for k, v in sorted(errs.items()))
    L = oracle.lib()
    for k in ref:
        w = w0[k].astype(np.float32).ravel().copy()
        v = np.zeros_like(w)
        gg = np.ascontiguousarray(ref[k].ravel(), np.float32)
        L.orc_sgd(w.ctypes.data, gg.ctypes.data, v.ctypes.data, lr, mom, w.size)
        d_gpu = w1[k].ravel().astype(np.float64) - w0[k].ravel()
        d_ref = w.astype(np.float64) - w0[k].ravel()
        assert rel_fro(d_gpu, d_ref) <= 5e-3, (k, rel_fro(d_gpu, d_ref))
    on.close()
    net.close()
