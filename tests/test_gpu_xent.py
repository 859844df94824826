"""Xent output branch: a network with prefinal-xent + output-xent
(log-softmax) beside the chain output. Forward: both outputs match the oracle (output-xent
rows are log-probabilities). Backward: seeded at the chain output only
(network_backward.go:102-115), so the xent branch's parameters get zero gradient and
the chain path's gradients match the oracle seeded the same way."""
import numpy as np
import pytest

import oracle
from conftest import rel_fro
from test_gpu_nnet import _forward_parity, _oracle

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("T", [150, 333])
def test_xent_branch_forward_backward(gpu, T):
    kf = gpu
    from kfp16 import synth
    xcfg = synth.load_xconfig("tiny_xent.xconfig")
    net = kf.Network(xcfg, max_frames=T)
    params, bns = synth.init_network(net)
    feats = synth.make_features(T, 40)
    fbuf = kf.upload_fp16(feats)
    net.forward(fbuf.ptr, T)
    on = _oracle(xcfg, params, bns, feats)
    masks = _forward_parity(net, on, None)
    lx = net.read_activation("output-xent").astype(np.float64)
    np.testing.assert_allclose(np.exp(lx).sum(1), 1.0, atol=2e-2)   # rows are log-probabilities
    on.close()
    on = _oracle(xcfg, params, bns, feats)
    on.forward(feats.astype(np.float32), force_masks=masks)
    og = (np.random.default_rng(7).standard_normal((T, 200)) * 0.05).astype(np.float16)
    gbuf = kf.upload_fp16(og)
    net.backward(gbuf.ptr)
    got = net.read_grads()
    on.backward(og.astype(np.float32))
    ref = on.grads()
    for k in ref:
        if k.startswith(("prefinal-xent.", "output-xent.")):
            assert not np.any(got[k]), k          # no gradient reaches the xent branch
        else:
            assert rel_fro(got[k], ref[k]) <= 5e-3, (k, rel_fro(got[k], ref[k]))


def test_log_softmax_kernel_negative_rows(gpu):
    """ops_log_softmax on all-negative rows (where the reference's integer atomicMax row
    max fails) and on widths off the fast path."""
    kf = gpu
    rng = np.random.default_rng(2)
    for rows, cols in [(37, 3080), (5, 4096), (9, 200), (3, 4104), (4, 13)]:
        x = (rng.standard_normal((rows, cols)) * 3 - 20).astype(np.float16)
        d = kf.upload_fp16(x)
        kf.check(kf.core.ops_log_softmax(d.ptr, rows, cols), "log_softmax")
        kf.sync()
        got = kf.read_fp16(d.ptr, (rows, cols)).astype(np.float64)
        xd = x.astype(np.float64)
        ref = xd - (xd.max(1, keepdims=True) + np.log(np.exp(xd - xd.max(1, keepdims=True)).sum(1, keepdims=True)))
        assert np.max(np.abs(got - ref)) <= 2 ** -10 * np.max(np.abs(ref)) + 1e-3, (rows, cols)
