"""Deterministic check of the two-stream backward's ordering.

The weight gradients run on a stream of their own beside the input-gradient chain
(DESIGN §8a); events order every shared buffer (the three-deep dz / g / dbott ring, the
per-stream split-K slabs of kf_workspace_stream). test_gpu_nnet's
test_wgrad_stream_bit_identical can only catch a missing order when the timing happens
to expose it. Here nnet_debug_backward stalls the weight-gradient stream with a spin
kernel before each of its batches of work, so it runs far behind the chain, for each
placement of the TDNN-F affine weight gradients (KF_BWD_MAIN_AFF 0 / 1 / 2), and every
gradient and the next step's output must still be bit-identical to the one-stream order.
"""
import numpy as np
import pytest

from test_gpu_nnet import _run_product

STALL = 400_000   # GPU clock cycles per batch of side work (~0.2 ms)


def _two_steps(kfp16, xcfg, T, on, main_aff=-1, stall=0, implicit=False, rsub=False):
    net, params, bns, feats, fbuf = _run_product(kfp16, xcfg, T)
    net.set_wgrad_stream(on)
    net.set_implicit_dz(implicit)
    net.debug_backward(main_aff, stall)
    if rsub:
        net.set_row_subsampling(3)
    P = net.layers[-1][3]
    net.forward(fbuf.ptr, T)
    rows = net.row_set()[0] or T
    assert not rsub or rows < T
    og = (np.random.default_rng(11).standard_normal((rows, P)) * 0.05).astype(np.float16)
    gb = kfp16.upload_fp16(og)
    net.forward(fbuf.ptr, T)
    net.backward(gb.ptr)
    net.sgd(1e-3, 0.9)
    net.forward(fbuf.ptr, T)
    net.backward(gb.ptr)
    out = (net.read_grads(), net.read_activation("output").astype(np.float32))
    net.close()
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["plain", "implicit", "rsub"])
def test_stalled_wgrad_stream_bit_identical(gpu, mode):
    """rsub: the row-subsampled step (compact TDNN-F stack, cnn6 on the row set with its
    tail window on the weight-gradient stream)"""
    kfp16 = gpu
    from kfp16 import synth
    kfp16.core.kf_pending_clear()
    xcfg = synth.load_xconfig("cnn_tdnn_17f.xconfig")
    T = 3000
    implicit, rsub = mode == "implicit", mode == "rsub"
    g0, a0 = _two_steps(kfp16, xcfg, T, False, implicit=implicit, rsub=rsub)
    for main_aff in (0, 1, 2):
        for stall in (0, STALL):
            g1, a1 = _two_steps(kfp16, xcfg, T, True, main_aff, stall, implicit, rsub)
            for k in g0:
                assert np.array_equal(g0[k], g1[k]), (main_aff, stall, k)
            assert np.array_equal(a0, a1), (main_aff, stall)
    assert kfp16.pending_log() is None, kfp16.pending_log()
