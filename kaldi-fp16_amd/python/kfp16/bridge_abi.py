"""ctypes bindings of the go/kaldibridge ABI (include/kaldi_bridge.h,
libkaldi_fp16_cgo.so) and the CNN launch wrappers (include/cnn_fp16.h,
libkaldi_fp16.so): the calls go/kaldibridge/bridge.go:14-53 and
cnn_bridge.go:14-72 make, bound the way the tests use them."""
import ctypes as C

from . import _load, core

cgo = _load("libkaldi_fp16_cgo.so")

_vp, _i, _f, _sz = C.c_void_p, C.c_int, C.c_float, C.c_size_t
_fp = C.POINTER(C.c_float)


def _sig(lib, name, res, *args):
    fn = getattr(lib, name)
    fn.restype = res
    fn.argtypes = list(args)
    return fn


for name, res, args in [
    ("kaldi_cublas_create", _vp, ()),
    ("kaldi_cublas_destroy", None, (_vp,)),
    ("kaldi_cublas_enable_tensor_cores", None, (_vp,)),
    ("kaldi_tensor_create", _vp, (_i, _i)),
    ("kaldi_tensor_zeros", _vp, (_i, _i)),
    ("kaldi_tensor_ones", _vp, (_i, _i)),
    ("kaldi_tensor_free", None, (_vp,)),
    ("kaldi_tensor_rows", _i, (_vp,)),
    ("kaldi_tensor_cols", _i, (_vp,)),
    ("kaldi_tensor_size", _sz, (_vp,)),
    ("kaldi_tensor_data", _vp, (_vp,)),
    ("kaldi_tensor_copy_from_host_fp32", None, (_vp, _fp, _sz)),
    ("kaldi_tensor_copy_to_host_fp32", None, (_vp, _fp, _sz)),
    ("kaldi_gemm", None, (_vp, _vp, _vp, _vp, _f, _f, _i, _i)),
    ("kaldi_relu", None, (_vp,)),
    ("kaldi_sigmoid", None, (_vp,)),
    ("kaldi_tanh", None, (_vp,)),
    ("kaldi_softmax", None, (_vp,)),
    ("kaldi_add", None, (_vp, _vp)),
    ("kaldi_scale", None, (_vp, _f)),
    ("kaldi_loss_scaler_create", _vp, (_f,)),
    ("kaldi_loss_scaler_free", None, (_vp,)),
    ("kaldi_loss_scaler_get_scale", _f, (_vp,)),
    ("kaldi_loss_scaler_update", None, (_vp, _i)),
    ("kaldi_get_last_error", C.c_char_p, ()),
    ("kaldi_clear_error", None, ()),
]:
    _sig(cgo, name, res, *args)

for name, args in [
    ("launch_conv1d_forward_fp16", (_vp, _vp, _vp, _vp) + (_i,) * 8 + (_vp,)),
    ("launch_conv1d_backward_fp16", (_vp,) * 6 + (_i,) * 8 + (_vp,)),
    ("launch_maxpool1d_forward_fp16", (_vp, _vp, _vp) + (_i,) * 5 + (_vp,)),
    ("launch_maxpool1d_backward_fp16", (_vp, _vp, _vp) + (_i,) * 4 + (_vp,)),
    ("launch_stats_pooling_fp16", (_vp, _vp, _i, _i, _i, _vp)),
    ("launch_batchnorm1d_forward_fp16", (_vp,) * 8 + (_i, _i, _i, _f, _f, C.c_bool, _vp)),
    ("launch_layernorm_forward_fp16", (_vp,) * 4 + (_i, _i, _i, _f, _vp)),
    ("launch_depthwise_conv1d_fp16", (_vp,) * 4 + (_i,) * 6 + (_vp,)),
    ("launch_pointwise_conv1d_fp16", (_vp,) * 4 + (_i,) * 4 + (_vp,)),
]:
    _sig(core, name, None, *args)


def last_error():
    e = cgo.kaldi_get_last_error()
    return e.decode() if e else None


class Tensor:
    """An opaque kaldibridge tensor (fp16 rows x cols on the device)."""

    def __init__(self, rows, cols, kind="create"):
        fn = {"create": cgo.kaldi_tensor_create, "zeros": cgo.kaldi_tensor_zeros,
              "ones": cgo.kaldi_tensor_ones}[kind]
        self.h = fn(rows, cols)
        if not self.h:
            raise RuntimeError(f"kaldi_tensor_{kind}: {last_error()}")

    @classmethod
    def from_numpy(cls, a):
        import numpy as np
        a = np.ascontiguousarray(a, dtype=np.float32)
        t = cls(a.shape[0], a.shape[1])
        cgo.kaldi_tensor_copy_from_host_fp32(t.h, a.ctypes.data_as(_fp), a.size)
        return t

    def numpy(self):
        import numpy as np
        out = np.zeros((self.rows, self.cols), np.float32)
        cgo.kaldi_tensor_copy_to_host_fp32(self.h, out.ctypes.data_as(_fp), out.size)
        return out

    @property
    def rows(self):
        return cgo.kaldi_tensor_rows(self.h)

    @property
    def cols(self):
        return cgo.kaldi_tensor_cols(self.h)

    @property
    def ptr(self):
        return cgo.kaldi_tensor_data(self.h)

    def free(self):
        if self.h:
            cgo.kaldi_tensor_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass
