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
    "cnn_fp16.h": "libkaldi_fp16.so",
    "kaldi_bridge.h": "libkaldi_fp16_cgo.so",
    "kf_nnet.h": "libkaldi_fp16_nnet.so",
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
