"""The drop-in boundary: every function include/*.h declares is exported by the
built C-ABI library that implements it (no device calls)."""
import ctypes
import os

import pytest

import kfp16

HEADERS = {
    "bridge.h": "libkaldi_fp16.so",
    "ops.h": "libkaldi_fp16.so",
    "kf_ops.h": "libkaldi_fp16.so",
    "chain.h": "libkaldi_fp16.so",
    "chain_den.h": "libkaldi_fp16.so",
    "chain_backward_api.h": "libkaldi_fp16.so",
    "kf_chain.h": "libkaldi_fp16.so",
    "cnn_fp16.h": "libkaldi_fp16.so",
    "kaldi_bridge.h": "libkaldi_fp16_cgo.so",
    "kf_nnet.h": "libkaldi_fp16_nnet.so",
    "kf_egs.h": "libkaldi_fp16_egs.so",
    "kf_model.h": "libkaldi_fp16_nnet.so",
}


@pytest.mark.parametrize("header", sorted(HEADERS))
def test_header_symbols_exported(header):
    path = os.path.join(kfp16.INCDIR, header)
    if not os.path.exists(path):
        pytest.skip(f"{header} not part of this build yet")
    lib = ctypes.CDLL(os.path.join(kfp16.LIBDIR, HEADERS[header]))
    names = kfp16.read_header_symbols(header)
    assert names, header
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, f"{header}: not exported: {missing}"


def test_errors_start_clear():
    assert kfp16.core.ops_last_error() is None
    assert kfp16.core.bridge_last_error() is None


def test_loss_scaler_rules():
    """kaldi_loss_scaler_* (cgo_interface.cu:379-445) is host state only: backoff
    0.5 on overflow, growth 2 after 2000 clean steps, clamp to [1, 65536]."""
    from kfp16 import bridge_abi as kb
    ls = kb.cgo.kaldi_loss_scaler_create(1024.0)
    assert kb.cgo.kaldi_loss_scaler_get_scale(ls) == 1024.0
    kb.cgo.kaldi_loss_scaler_update(ls, 1)
    assert kb.cgo.kaldi_loss_scaler_get_scale(ls) == 512.0
    for _ in range(1999):
        kb.cgo.kaldi_loss_scaler_update(ls, 0)
    assert kb.cgo.kaldi_loss_scaler_get_scale(ls) == 512.0
    kb.cgo.kaldi_loss_scaler_update(ls, 0)
    assert kb.cgo.kaldi_loss_scaler_get_scale(ls) == 1024.0
    kb.cgo.kaldi_loss_scaler_update(ls, 1)  # an overflow resets the clean-step count
    for _ in range(1999):
        kb.cgo.kaldi_loss_scaler_update(ls, 0)
    assert kb.cgo.kaldi_loss_scaler_get_scale(ls) == 512.0
    for _ in range(20):
        kb.cgo.kaldi_loss_scaler_update(ls, 1)
    assert kb.cgo.kaldi_loss_scaler_get_scale(ls) == 1.0
    kb.cgo.kaldi_loss_scaler_free(ls)
    big = kb.cgo.kaldi_loss_scaler_create(1e9)
    kb.cgo.kaldi_loss_scaler_update(big, 0)
    assert kb.cgo.kaldi_loss_scaler_get_scale(big) == 65536.0
    kb.cgo.kaldi_loss_scaler_free(big)
    assert kb.cgo.kaldi_loss_scaler_get_scale(None) == 1.0


def test_kaldi_handles_without_device():
    """Opaque handles and NULL tolerance that need no device memory."""
    from kfp16 import bridge_abi as kb
    ctx = kb.cgo.kaldi_cublas_create()
    assert ctx
    kb.cgo.kaldi_cublas_enable_tensor_cores(ctx)
    kb.cgo.kaldi_cublas_destroy(ctx)
    assert kb.cgo.kaldi_tensor_rows(None) == 0 and kb.cgo.kaldi_tensor_size(None) == 0
    kb.cgo.kaldi_tensor_free(None)
    kb.cgo.kaldi_relu(None)
    assert kb.cgo.kaldi_get_last_error() is None
