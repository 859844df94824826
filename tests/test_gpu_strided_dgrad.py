"""The conv input gradients. The strided conv's input gradient (height-subsample-out 2: cnn3, cnn5 of the benchmark
model) as one GEMM over both residues (network.cpp hsub_merge, KF_HSUB_MERGE) against one
GEMM per residue: the merged weight rows keep each residue's taps in their order and the
zero blocks add exact zeros, so every gradient must be bit-identical. The gradient of a
strided conv's input reaches every weight gradient below it (cnn2, cnn1).
"""
import os

import numpy as np
import pytest

from test_gpu_wgrad_order import _two_steps


@pytest.mark.gpu
@pytest.mark.parametrize("rsub", [False, True])
def test_strided_dgrad_merged_bit_identical(gpu, rsub):
    kfp16 = gpu
    from kfp16 import synth
    kfp16.core.kf_pending_clear()
    xcfg = synth.load_xconfig("cnn_tdnn_17f.xconfig")
    T = 1500
    old = os.environ.get("KF_HSUB_MERGE")
    try:
        os.environ["KF_HSUB_MERGE"] = "0"
        g0, a0 = _two_steps(kfp16, xcfg, T, True, rsub=rsub)
        for lim in ("128", "256"):
            os.environ["KF_HSUB_MERGE"] = lim
            g1, a1 = _two_steps(kfp16, xcfg, T, True, rsub=rsub)
            for k in g0:
                assert np.array_equal(g0[k], g1[k]), (lim, k)
            assert np.array_equal(a0, a1), lim
    finally:
        if old is None:
            os.environ.pop("KF_HSUB_MERGE", None)
        else:
            os.environ["KF_HSUB_MERGE"] = old
    assert kfp16.pending_log() is None, kfp16.pending_log()


@pytest.mark.gpu
@pytest.mark.parametrize("rsub", [False, True])
def test_conv_dgrad_transposed_weights_bit_identical(gpu, rsub):
    """The conv input gradients with the weights as per-tap transposed blocks (network.cpp
    dgrad_wt, the default) against the shifted k-contiguous weight rows (KF_DGRAD_WT=0):
    the same K order, so every gradient must be bit-identical."""
    kfp16 = gpu
    from kfp16 import synth
    kfp16.core.kf_pending_clear()
    xcfg = synth.load_xconfig("cnn_tdnn_17f.xconfig")
    T = 1500
    old = os.environ.get("KF_DGRAD_WT")
    try:
        os.environ["KF_DGRAD_WT"] = "0"
        g0, a0 = _two_steps(kfp16, xcfg, T, True, rsub=rsub)
        os.environ["KF_DGRAD_WT"] = "1"
        g1, a1 = _two_steps(kfp16, xcfg, T, True, rsub=rsub)
    finally:
        if old is None:
            os.environ.pop("KF_DGRAD_WT", None)
        else:
            os.environ["KF_DGRAD_WT"] = old
    for k in g0:
        assert np.array_equal(g0[k], g1[k]), k
    assert np.array_equal(a0, a1)
    assert kfp16.pending_log() is None, kfp16.pending_log()
