"""kfp16.model — ctypes binding of the Kaldi nnet3 model import (include/kf_model.h):
ParseNnet3Text / ExportModelText / LoadWeights / NewNetworkFromKaldi of
internal/nnet/weight_loader.go. Parsing and loading run in libkaldi_fp16_nnet.so."""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import KfError, nnet

_vp, _i = C.c_void_p, C.c_int
_fp = C.POINTER(C.c_float)

LOAD_NEW, LOAD_REPLACE = 0, 1


class KfNnet3Component(C.Structure):
    _fields_ = [("name", C.c_char_p), ("type", C.c_char_p), ("linear", _fp), ("linear_rows", _i),
                ("linear_cols", _i), ("bias", _fp), ("bias_dim", _i), ("stats_mean", _fp),
                ("mean_dim", _i), ("stats_var", _fp), ("var_dim", _i), ("count", C.c_double),
                ("epsilon", C.c_float), ("target_rms", C.c_float), ("num_filters_in", _i),
                ("num_filters_out", _i), ("height_in", _i), ("height_out", _i), ("num_heads", _i),
                ("key_dim", _i), ("value_dim", _i), ("key_scale", C.c_float),
                ("learning_rate", C.c_float), ("max_change", C.c_float), ("l2_regularize", C.c_float)]


class KfLoadStats(C.Structure):
    _fields_ = [("layers_loaded", _i), ("layers_skipped", _i), ("params", C.c_longlong)]


def _sig(name, res, *args):
    fn = getattr(nnet, name)
    fn.restype = res
    fn.argtypes = list(args)


_sig("kf_nnet3_last_error", C.c_char_p)
_sig("kf_nnet3_parse_text", _vp, C.c_char_p, C.c_size_t)
_sig("kf_nnet3_read_text_file", _vp, C.c_char_p)
_sig("kf_nnet3_export", _vp, C.c_char_p)
_sig("kf_nnet3_free", None, _vp)
_sig("kf_nnet3_num_components", _i, _vp)
_sig("kf_nnet3_component", _i, _vp, _i, C.POINTER(KfNnet3Component))
_sig("kf_nnet3_find", _i, _vp, C.c_char_p)
_sig("nnet_load_kaldi", _i, _vp, _vp, _i, C.POINTER(KfLoadStats))
_sig("nnet_set_idct", _i, _vp, C.c_char_p, _vp, _i, _i)


class ModelError(KfError):
    pass


def last_error() -> str:
    e = nnet.kf_nnet3_last_error()
    return e.decode() if e else ""


def _arr(ptr, n):
    return np.ctypeslib.as_array(ptr, shape=(n,)).copy() if n > 0 and ptr else np.zeros(0, np.float32)


@dataclass
class Component:
    """KaldiComponent (weight_loader.go:28-61)."""
    name: str
    type: str
    linear: np.ndarray      # [rows, cols] (Kaldi [out x in])
    bias: np.ndarray
    stats_mean: np.ndarray
    stats_var: np.ndarray
    count: float
    epsilon: float
    target_rms: float
    num_filters_in: int
    num_filters_out: int
    height_in: int
    height_out: int
    learning_rate: float
    max_change: float
    l2_regularize: float

    @property
    def linear_rows(self):
        return self.linear.shape[0]

    @property
    def linear_cols(self):
        return self.linear.shape[1]


class Nnet3Model:
    """Parsed components of an nnet3 text model (ParseNnet3Text)."""

    def __init__(self, handle):
        self._h = None
        if not handle:
            raise ModelError(last_error())
        self._h = handle

    @classmethod
    def from_text(cls, text: str) -> "Nnet3Model":
        b = text.encode()
        return cls(nnet.kf_nnet3_parse_text(b, len(b)))

    @classmethod
    def from_file(cls, path: str) -> "Nnet3Model":
        return cls(nnet.kf_nnet3_read_text_file(path.encode()))

    @classmethod
    def export(cls, mdl_path: str) -> "Nnet3Model":
        """ExportModelText: needs Kaldi's nnet3-copy on PATH."""
        return cls(nnet.kf_nnet3_export(mdl_path.encode()))

    def __len__(self):
        return nnet.kf_nnet3_num_components(self._h)

    def component(self, idx: int) -> Component:
        c = KfNnet3Component()
        if nnet.kf_nnet3_component(self._h, idx, C.byref(c)) != 0:
            raise ModelError(last_error())
        lin = _arr(c.linear, c.linear_rows * c.linear_cols).reshape(c.linear_rows, c.linear_cols)
        return Component(c.name.decode(), c.type.decode(), lin, _arr(c.bias, c.bias_dim),
                         _arr(c.stats_mean, c.mean_dim), _arr(c.stats_var, c.var_dim), c.count, c.epsilon,
                         c.target_rms, c.num_filters_in, c.num_filters_out, c.height_in, c.height_out,
                         c.learning_rate, c.max_change, c.l2_regularize)

    def __getitem__(self, name: str) -> Component:
        i = nnet.kf_nnet3_find(self._h, name.encode())
        if i < 0:
            raise KeyError(name)
        return self.component(i)

    def __contains__(self, name: str) -> bool:
        return nnet.kf_nnet3_find(self._h, name.encode()) >= 0

    def names(self):
        return [self.component(i).name for i in range(len(self))]

    def load_into(self, net, mode: int = LOAD_NEW) -> KfLoadStats:
        """LoadWeights (LOAD_REPLACE) / NewNetworkFromKaldi (LOAD_NEW) into a kfp16.Network."""
        st = KfLoadStats()
        if nnet.nnet_load_kaldi(net.h, self._h, mode, C.byref(st)) != 0:
            raise ModelError(last_error())
        return st

    def close(self):
        if self._h:
            nnet.kf_nnet3_free(self._h)
            self._h = None

    def __del__(self):
        if getattr(self, "_h", None):
            self.close()
